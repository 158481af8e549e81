// buf_probe.hip -- semantics probe for gfx950 raw buffer ops (not product code):
// does the range check include soffset?  do unaligned b32 stores write all 4 bytes?
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void probe(uint8_t *buf, uint32_t *out) {
    if (threadIdx.x != 0) return;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(buf, 0, 16, 0x00020000);
    out[0] = __builtin_amdgcn_raw_buffer_load_b32(rs, 0, 20, 0);   // voff 0, soff 20 (beyond 16)
    out[1] = __builtin_amdgcn_raw_buffer_load_b32(rs, 20, 0, 0);   // voff 20
    out[2] = __builtin_amdgcn_raw_buffer_load_b32(rs, 4, 8, 0);    // voff 4 + soff 8 = 12 (in range)
    out[3] = __builtin_amdgcn_raw_buffer_load_b32(rs, 14, 0, 0);   // straddles 16
    out[4] = __builtin_amdgcn_raw_buffer_load_b32(rs, 6, 0, 0);    // unaligned in range
    __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(buf + 64, 0, 64, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b32(0xddccbbaau, rw, 2, 0, 0);       // unaligned store
    __builtin_amdgcn_raw_buffer_store_b32(0x44332211u, rw, 0, 60, 0);      // soff 60 + 4 = 64 (edge)
    __builtin_amdgcn_raw_buffer_store_b32(0x88776655u, rw, 0, 64, 0);      // soff 64: out of range?
}
int main() {
    uint8_t *b; uint32_t *o;
    (void)hipMalloc(&b, 256); (void)hipMalloc(&o, 64);
    uint8_t h[256]; for (int i = 0; i < 256; i++) h[i] = (uint8_t)i;
    (void)hipMemcpy(b, h, 256, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, b, o);
    uint32_t r[5]; (void)hipMemcpy(r, o, 20, hipMemcpyDeviceToHost);
    (void)hipMemcpy(h, b, 256, hipMemcpyDeviceToHost);
    printf("soff20 %08x voff20 %08x v4s8 %08x straddle %08x unal6 %08x\n", r[0], r[1], r[2], r[3], r[4]);
    printf("bytes 64..71: "); for (int i = 64; i < 72; i++) printf("%02x ", h[i]);
    printf("\nbytes 124..135: "); for (int i = 124; i < 136; i++) printf("%02x ", h[i]);
    printf("\n");
    return 0;
}
