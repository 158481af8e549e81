"""Probe (not a test): H2D alone, D2H alone, and both at once on two streams, pinned buffers,
1 GiB each -- is the PCIe link used full duplex by concurrent hipMemcpyAsync?"""
import time
import torch

n = 1 << 30
h_a = torch.empty(n, dtype=torch.uint8).pin_memory()
h_b = torch.empty(n, dtype=torch.uint8).pin_memory()
d_a = torch.empty(n, dtype=torch.uint8, device="cuda")
d_b = torch.empty(n, dtype=torch.uint8, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def run(h2d, d2h, reps=4):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        if h2d:
            with torch.cuda.stream(s1):
                d_a.copy_(h_a, non_blocking=True)
        if d2h:
            with torch.cuda.stream(s2):
                h_b.copy_(d_b, non_blocking=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    return reps * n * (int(h2d) + int(d2h)) / dt / 1e9


run(True, True, 1)
print(f"H2D alone {run(True, False):.1f} GB/s, D2H alone {run(False, True):.1f} GB/s, "
      f"both at once {run(True, True):.1f} GB/s aggregate")
