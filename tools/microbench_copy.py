"""Reference bandwidths on the box: device copy / read-reduce of the array
sizes the 2-D fp64 passes move (to judge the FFT passes against)."""
import sys

import torch

sys.path.insert(0, ".")


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


for n in (1024, 2048, 4096):
    a = torch.randn(n * (n // 2 + 1) * 2, dtype=torch.float64, device="cuda")
    b = torch.empty_like(a)
    t = bench(lambda: b.copy_(a))
    by = 2 * a.numel() * 8
    t2 = bench(lambda: torch.add(a, a, out=b))
    c = torch.randn(8 * a.numel(), dtype=torch.float64, device="cuda")
    d = torch.empty_like(c)
    t3 = bench(lambda: d.copy_(c))
    print(f"n={n}: copy {by/1e6:.1f} MB {t*1e6:.1f} us {by/t/1e9:.0f} GB/s | add {t2*1e6:.1f} us | "
          f"8x larger copy {t3*1e6:.1f} us {8*by/t3/1e9:.0f} GB/s", flush=True)
