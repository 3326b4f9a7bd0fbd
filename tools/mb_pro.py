"""Per-pass times of the CF Jacobian's batched forward transform (prologue
A x_b + xi0 dA_b[pindex], 4 x 2048^2 fp64) for the R2C+prologue variants
selected by NFT_PRO_PAIRS=1 / NFT_PRO_PAIRS_L.  Usage: python tools/mb_pro.py LABEL"""
import sys
from collections import defaultdict

import torch

sys.path.insert(0, ".")
from nifty_amd import _native as nat  # noqa: E402

label = sys.argv[1]
n, k = 2048, 4
dev = "cuda"
g = torch.Generator(device="cpu").manual_seed(2)
P = n * n
a = torch.randn((n, n), generator=g, dtype=torch.float64).to(dev)
b = torch.randn((n, n), generator=g, dtype=torch.float64).to(dev)
# bin index of |k| on the harmonic grid (the real access pattern)
kx = torch.fft.fftfreq(n, device=dev, dtype=torch.float64) * n
kk = torch.sqrt(kx[:, None] ** 2 + kx[None, :] ** 2)
uq, idx = torch.unique(kk, return_inverse=True)
idx = idx.to(torch.int32).contiguous()
nbins = uq.numel()
if len(sys.argv) > 2 and sys.argv[2] == "seq":   # coalesced stand-in: the gather cost alone
    idx = (torch.arange(n * n, device=dev, dtype=torch.int64) * nbins // (n * n)).to(torch.int32).view(n, n)
if len(sys.argv) > 2 and sys.argv[2] == "zero":
    idx = torch.zeros((n, n), device=dev, dtype=torch.int32)
c = torch.randn((nbins, k), generator=g, dtype=torch.float64).to(dev)
size = P + 2 * nbins + 64
X = torch.randn((k, size), generator=g, dtype=torch.float64).to(dev)
out = torch.empty((k, n, n), dtype=torch.float64, device=dev)
args = dict(pro=dict(a=a, x=X[0, :], b=b, c=c, index=idx), shape=out.shape,
            batch=dict(period=P, x=size, c=1, c_elem=k))
for _ in range(3):
    nat.hartley_fused(out, (1, 2), 0.7, **args)
torch.cuda.synchronize()
ck = float(out.double().abs().sum())
torch.cuda._sleep(50_000_000)
reps = 20
with nat.LaunchProfile() as p:
    for _ in range(reps):
        nat.hartley_fused(out, (1, 2), 0.7, **args)
acc = defaultdict(float)
cnt = defaultdict(int)
for lab, ms in p.records:
    acc[lab] += ms
    cnt[lab] += 1
tot = sum(acc.values()) / reps * 1e3
parts = ", ".join(f"{kk} {acc[kk] / cnt[kk] * 1e3:.1f}us x{cnt[kk] // reps}" for kk in acc)
print(f"[{label}] total {tot:.1f} us | {parts} | checksum {ck:.12e}", flush=True)
