"""Per-pass times of the batched 2-D fp64 Hartley (the CG matvec's shape:
4 x 2048^2, axes (1, 2)) and its error against torch.fft, for comparing
column-pass variants selected by environment switches (NFT_COL1P ...).
Usage: python tools/mb_col.py [label]"""
import sys
from collections import defaultdict

import torch

sys.path.insert(0, ".")
from nifty_amd import _native as nat  # noqa: E402

label = sys.argv[1] if len(sys.argv) > 1 else ""
for shp, axes in [((4, 2048, 2048), (1, 2)), ((2048, 2048), (0, 1)), ((4, 1024, 1024), (1, 2))]:
    torch.manual_seed(0)
    x = torch.randn(shp, dtype=torch.float64, device="cuda")
    out = torch.empty_like(x)
    for _ in range(3):
        nat.hartley(x, axes, out=out)
    F = torch.fft.fftn(x, dim=axes)
    ref = F.real + F.imag
    err = ((out - ref).abs().max() / ref.abs().max()).item()
    torch.cuda.synchronize()
    torch.cuda._sleep(100_000_000)
    reps = 20
    with nat.LaunchProfile() as p:
        for _ in range(reps):
            nat.hartley(x, axes, out=out)
    acc = defaultdict(float)
    cnt = defaultdict(int)
    for lab, ms in p.records:
        acc[lab] += ms
        cnt[lab] += 1
    tot = sum(acc.values()) / reps * 1e3
    nbytes = x.numel() * 8 * 2
    parts = ", ".join(f"{k} {acc[k] / cnt[k] * 1e3:.1f}us x{cnt[k] // reps}" for k in acc)
    print(f"[{label}] {shp}: total {tot:.1f} us ({nbytes / tot / 1e3:.0f} GB/s of 2 passes) err {err:.1e} | {parts}",
          flush=True)
