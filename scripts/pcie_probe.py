"""Diagnostic: pinned host <-> HBM copy bandwidth (1 GiB), each direction alone
and both at once on two streams."""
import time
import torch
n = 1 << 30
h1 = torch.empty(n, dtype=torch.uint8).pin_memory()
h2 = torch.empty(n, dtype=torch.uint8).pin_memory()
d1 = torch.empty(n, dtype=torch.uint8, device="cuda")
d2 = torch.empty(n, dtype=torch.uint8, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
def run(f, reps=3):
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize(); t0 = time.perf_counter(); f(); torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best
t = run(lambda: d1.copy_(h1, non_blocking=True)); print(f"H2D {n/t/1e9:.1f} GB/s")
t = run(lambda: h1.copy_(d1, non_blocking=True)); print(f"D2H {n/t/1e9:.1f} GB/s")
def both():
    with torch.cuda.stream(s1): d1.copy_(h1, non_blocking=True)
    with torch.cuda.stream(s2): h2.copy_(d2, non_blocking=True)
t = run(both); print(f"H2D+D2H concurrent {2*n/t/1e9:.1f} GB/s total")
