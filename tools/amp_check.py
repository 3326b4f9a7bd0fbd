"""Batched amplitude JVP/VJP at the C3 size (2048^2, B = 313,847, 4 RHS):
per-launch times (nft_prof_*) and outputs saved for a bitwise comparison of
the fused one-launch kernels against the multi-kernel path
(NFT_AMP_FUSED=0).  Usage: python tools/amp_check.py LABEL [n]"""
import sys
from collections import defaultdict

import numpy as np
import torch

sys.path.insert(0, ".")
import nifty_amd as ift  # noqa: E402
from nifty_amd import _native as nat  # noqa: E402

label = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
ift.config.set_device("cuda:0")
args = dict(offset_mean=0, offset_std=(1e-3, 1e-6), fluctuations=(1., 0.8),
            loglogavgslope=(-3., 1), flexibility=(2, 1.), asperity=(0.5, 0.4))
cf = ift.SimpleCorrelatedField(ift.RGSpace((n, n)), **args)
amp = cf.amp
keys = list(amp.domain_dict)
with ift.random.Context(3):
    x = ift.from_random(cf.domain, "normal")
    lat = ift.from_random(cf.domain, "normal")
_, c = amp.forward({k: x[k].val for k in keys})
const, keep = amp.native_const(c)
from nifty_amd.packing import PackedLayout  # noqa: E402

lay = PackedLayout(cf.domain)
k = 4
torch.manual_seed(0)
D = torch.randn(k, lay.size, dtype=torch.float64, device="cuda")
off = dict(zip(lay.keys, lay.offsets))
da = torch.empty(k, amp.B, dtype=torch.float64, device="cuda")
g = torch.randn(k, amp.B, dtype=torch.float64, device="cuda")
Q = torch.zeros(k, lay.size, dtype=torch.float64, device="cuda")
for _ in range(3):
    amp.native_jvp_batched(const, D, off, da)
    amp.native_vjp_batched(const, g, Q, off, D, 0.5)
torch.cuda.synchronize()
# amplitude keys only (the xi segment of Q is untouched): a few MB
ak = [kk for kk in lay.keys if kk != "xi"]
res = {"da": da.cpu().numpy().copy()}
for kk in ak:
    o, nn = off[kk], lay.sizes[lay.keys.index(kk)]
    res["Q_" + kk] = Q[:, o:o + nn].cpu().numpy().copy()
# single-RHS calls must equal the batched rows bitwise
da1 = torch.empty(1, amp.B, dtype=torch.float64, device="cuda")
Q1 = torch.zeros(1, lay.size, dtype=torch.float64, device="cuda")
eq = True
for r in range(k):
    amp.native_jvp_batched(const, D[r:r + 1].contiguous(), off, da1)
    amp.native_vjp_batched(const, g[r:r + 1].contiguous(), Q1, off, D[r:r + 1].contiguous(), 0.5)
    eq &= bool(torch.equal(da1[0], da[r])) and bool(torch.equal(Q1[0], Q[r]))
torch.cuda.synchronize()
torch.cuda._sleep(50_000_000)
reps = 20
with nat.LaunchProfile() as p:
    for _ in range(reps):
        amp.native_jvp_batched(const, D, off, da)
        amp.native_vjp_batched(const, g, Q, off, D, 0.5)
acc = defaultdict(float)
cnt = defaultdict(int)
for lab, ms in p.records:
    acc[lab] += ms
    cnt[lab] += 1
tot = sum(acc.values()) / reps * 1e3
parts = ", ".join(f"{kk} {acc[kk] / cnt[kk] * 1e3:.1f}us" for kk in acc)
print(f"[{label}] B={amp.B} k={k}: jvp+vjp {tot:.1f} us | {parts} | single==batched {eq}", flush=True)
if label.startswith("cmp"):
    np.savez(f"gpurun_out/amp_{label}.npz", **res)
# grid-barrier cost
import ctypes  # noqa: E402
lib = nat.load()
for G in (256, 512, 1280):
    for nb in (1, 11):
        lib.nft_amp_barrier_probe(nb, G, nat.stream_ptr())
    torch.cuda.synchronize()
    with nat.LaunchProfile() as p:
        for nb in (1, 11):
            lib.nft_amp_barrier_probe(nb, G, nat.stream_ptr())
    t = [ms * 1e3 for _, ms in p.records]
    print(f"[{label}] barrier G={G}: 1 -> {t[0]:.1f} us, 11 -> {t[1]:.1f} us: {(t[1] - t[0]) / 10:.2f} us per barrier",
          flush=True)
