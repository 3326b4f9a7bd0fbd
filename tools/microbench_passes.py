"""Per-pass times (nft_prof_*) of the 2-D fp64 Hartley at a few sizes, for
FFT engine tuning (e.g. NFT_FFT_WG_PER_CU)."""
import sys
from collections import defaultdict

import torch

sys.path.insert(0, ".")
from nifty_amd import _native as nat  # noqa: E402

for shp in [(1024, 1024), (2048, 2048), (4096, 4096), (256, 256, 256)]:
    x = torch.randn(shp, dtype=torch.float64, device="cuda")
    out = torch.empty_like(x)
    axes = tuple(range(len(shp)))
    for _ in range(5):
        nat.hartley(x, axes, out=out)
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
    parts = ", ".join(f"{k} {acc[k] / cnt[k] * 1e3:.1f}us x{cnt[k] // reps}" for k in acc)
    print(f"{shp}: total {tot:.1f} us | {parts}", flush=True)
