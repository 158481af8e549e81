"""The encode's byte mix (4.29 GB in, 14.64 GB out) streamed by tape_amd/libtecprobe.so in three
output shapes, interleaved: 0 blocks, 1 rows from 2-aligned starts (the kernel's stores, nt), 2 rows
with 16-B-aligned interior pieces and 2-byte head / tail stores, 3 rows with write-back stores, 4
rows with nt interior and write-back junction pieces, 5 whole-line rows (1,408 B from 128-B-aligned
starts, the same two store instructions per row).  Measurement only."""
import ctypes as C
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = C.CDLL(os.path.join(ROOT, "tape_amd", "libtecprobe.so"))
f = lib.tec_probe_encode_mix
f.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_int, C.c_int, C.c_int, C.c_void_p, C.POINTER(C.c_float)]
dev = torch.device("cuda", 0)
nin, nout = 1024 * 4194304, 1024 * 14300960
d_in = torch.empty(nin, dtype=torch.uint8, device=dev)
d_out = torch.empty(nout, dtype=torch.uint8, device=dev)
d_in.random_(0, 255)
s = torch.cuda.current_stream()
for rnd in range(3):
    for shape, wgs in ((0, 1024), (1, 1024), (4, 1024), (5, 1024)):
        ms = C.c_float()
        r = f(d_in.data_ptr(), nin, d_out.data_ptr(), nout, shape, wgs, 5, C.c_void_p(s.cuda_stream), C.byref(ms))
        assert r == 0, r
        print(f"round {rnd} shape {shape} wgs {wgs}: {ms.value:.4f} ms", flush=True)
