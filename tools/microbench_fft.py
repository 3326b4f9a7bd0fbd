"""Microbenchmark of the native Hartley passes vs torch.fft (rocFFT) on one GPU.
Prints per-transform time and effective GB/s (2 passes x (read+write) x N x 8 B
for a 2-D fp64 Hartley)."""
import sys
import time

import torch

sys.path.insert(0, ".")
from nifty_amd import _native as nat  # noqa: E402


def bench(fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e-3


for shp, dt in [((1024, 1024), torch.float64), ((2048, 2048), torch.float64), ((4096, 4096), torch.float64),
                ((2048, 2048), torch.float32), ((4096, 4096), torch.float32), ((256, 256, 256), torch.float64)]:
    x = torch.randn(shp, dtype=dt, device="cuda")
    out = torch.empty_like(x)
    axes = tuple(range(len(shp)))
    t = bench(lambda: nat.hartley(x, axes, out=out))
    N = x.numel()
    es = x.element_size()
    byts = len(shp) * 2 * N * es
    tr = bench(lambda: torch.fft.rfftn(x))
    print(f"{shp} {dt}: native hartley {t*1e6:8.1f} us  {byts/t/1e9:7.1f} GB/s(model) | torch rfftn {tr*1e6:8.1f} us", flush=True)
