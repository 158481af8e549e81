// ldsdma_probe.hip -- semantics probe (not product code): LDS-DMA dwordx4 from 2-aligned global
// addresses (global_load_lds and raw buffer form) and the range check's zero fill.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((address_space(3))) void lds_void;
__global__ void probe(const uint8_t *buf, uint8_t *out) {
    __shared__ __attribute__((aligned(16))) uint8_t L[4 * 1024];
    const int t = threadIdx.x;
    for (int i = t; i < 4096; i += 64) L[i] = 0xee;
    __syncthreads();
    // A: global_load_lds x4 from buf + 2 + 16*lane  -> L[0..1024)
    __builtin_amdgcn_global_load_lds((const void *)(buf + 2 + 16 * t), (lds_void *)&L[0], 16, 0, 0);
    // B: raw buffer LDS-DMA x4, voffset 2 + 16*lane, resource of 1000 bytes -> L[1024..2048)
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(buf), 0, 1000, 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void *)&L[1024], 16, 2 + 16 * t, 0, 0, 0);
    // C: raw buffer LDS-DMA x4 with soffset 6, voffset 16*lane  -> L[2048..3072)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void *)&L[2048], 16, 16 * t, 6, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = t; i < 3072; i += 64) out[i] = L[i];
}
int main() {
    uint8_t *b, *o;
    (void)hipMalloc(&b, 4096); (void)hipMalloc(&o, 4096);
    uint8_t h[4096];
    for (int i = 0; i < 4096; i++) h[i] = (uint8_t)(i * 7 + 3);
    (void)hipMemcpy(b, h, 4096, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, b, o);
    uint8_t r[3072];
    if (hipMemcpy(r, o, 3072, hipMemcpyDeviceToHost) != hipSuccess) { printf("fault\n"); return 1; }
    int badA = 0, badB = 0, badC = 0;
    for (int i = 0; i < 1024; i++) if (r[i] != h[2 + i]) badA++;
    for (int i = 0; i < 1024; i++) { uint8_t e = (2 + i < 1000) ? h[2 + i] : 0; if (r[1024 + i] != e) badB++; }
    for (int i = 0; i < 1024; i++) { uint8_t e = (6 + i < 1000) ? h[6 + i] : 0; if (r[2048 + i] != e) badC++; }
    printf("A global_load_lds x4 @+2: %d bad bytes\n", badA);
    printf("B buffer lds x4 voff+2 range 1000: %d bad bytes (first 1000-2.. vs zero fill)\n", badB);
    printf("C buffer lds x4 soff 6: %d bad bytes\n", badC);
    printf("A[0..8]:"); for (int i = 0; i < 8; i++) printf(" %02x", r[i]); printf("  want"); for (int i = 0; i < 8; i++) printf(" %02x", h[2+i]); printf("\n");
    printf("B[990..1010]:"); for (int i = 990; i < 1010; i++) printf(" %02x", r[1024+i]); printf("\n");
    printf("C[990..1010]:"); for (int i = 990; i < 1010; i++) printf(" %02x", r[2048+i]); printf("\n");
    return 0;
}
