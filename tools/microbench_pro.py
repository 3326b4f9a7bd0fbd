"""Batched fused Hartley first pass (prologue A*x + xi0*dA[pindex]) at 2048^2,
k=4 items: which operand costs what.  Per-pass times from nft_prof events."""
import sys
from collections import defaultdict

import torch

sys.path.insert(0, ".")
import nifty_amd as ift  # noqa: E402
from nifty_amd import _native as nat  # noqa: E402


def run(label, fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    torch.cuda._sleep(100_000_000)
    with nat.LaunchProfile() as p:
        for _ in range(reps):
            fn()
    acc, cnt = defaultdict(float), defaultdict(int)
    for lab, ms in p.records:
        acc[lab] += ms
        cnt[lab] += 1
    print(label, " ".join(f"{k}={acc[k] / cnt[k] * 1e3:.1f}us" for k in acc), flush=True)


def main(n=2048, k=4):
    ift.config.set_device("cuda:0")
    sp = ift.RGSpace((n, n))
    ps = ift.PowerSpace(sp.get_default_codomain())
    pidx = torch.as_tensor(ps.pindex.astype("int32"), device="cuda").reshape(n, n).contiguous()
    B = ps.shape[0]
    dev = "cuda"
    N = n * n
    a = torch.randn(n, n, dtype=torch.float64, device=dev)
    xi0 = torch.randn(n, n, dtype=torch.float64, device=dev)
    X = torch.randn(k, N, dtype=torch.float64, device=dev)
    da = torch.randn(k, B, dtype=torch.float64, device=dev)
    out = torch.empty(k, n, n, dtype=torch.float64, device=dev)
    pn = ps.pindex.ravel()
    import numpy as np
    _, first = np.unique(pn, return_index=True)
    order = np.argsort(first, kind="stable")
    rank = np.empty_like(order)
    rank[order] = np.arange(order.size)
    fa_idx = torch.as_tensor(rank[pn].astype("int32"), device=dev).reshape(n, n).contiguous()
    sorted_idx = (torch.arange(N, device=dev, dtype=torch.int32) // (N // B + 1)).reshape(n, n).contiguous()
    zero_idx = torch.zeros(n, n, dtype=torch.int32, device=dev)
    bt = dict(period=N, x=N, c=B)
    for lab, pro in [("full", dict(a=a, x=X[0], b=xi0, c=da, index=pidx)),
                     ("first-app", dict(a=a, x=X[0], b=xi0, c=da, index=fa_idx)),
                     ("sorted-idx", dict(a=a, x=X[0], b=xi0, c=da, index=sorted_idx)),
                     ("zero-idx", dict(a=a, x=X[0], b=xi0, c=da, index=zero_idx)),
                     ("a*x only", dict(a=a, x=X[0])),
                     ("x only", dict(x=X[0]))]:
        run(f"k={k} {lab:10s}", lambda: nat.hartley_fused(out, (1, 2), 1.0, pro=pro, shape=out.shape, batch=bt))
    da_il = torch.randn(B, k, dtype=torch.float64, device=dev)
    pro = dict(a=a, x=X[0], b=xi0, c=da_il, index=pidx)
    run(f"k={k} interleaved", lambda: nat.hartley_fused(out, (1, 2), 1.0, pro=pro, shape=out.shape,
                                                        batch=dict(period=N, x=N, c=1, c_elem=k)))
    # bin scatter: |k| order vs first-appearance order of the bins
    w = torch.randn(k, N, dtype=torch.float64, device=dev)
    ga = torch.empty(k, B, dtype=torch.float64, device=dev)
    for lab, key in (("|k| order", pn), ("first-app", rank[pn])):
        perm = np.argsort(key, kind="stable")
        cnt = np.bincount(key, minlength=B)
        offs = np.zeros(B + 1, dtype=np.int64)
        np.cumsum(cnt, out=offs[1:])
        tp = torch.as_tensor(perm.astype("int32"), device=dev)
        to = torch.as_tensor(offs.astype("int32"), device=dev)
        run(f"scatter k={k} {lab}", lambda: nat.bin_scatter(w, tp, to, ga, k, N, B, 1))
        run(f"scatter k=1 {lab}", lambda: nat.bin_scatter(w[0], tp, to, ga[0], 1, N, B, 1))
    one = torch.empty(n, n, dtype=torch.float64, device=dev)
    run("k=1 full      ", lambda: nat.hartley_fused(one, (0, 1), 1.0, pro=dict(a=a, x=X[0].reshape(n, n), b=xi0,
                                                                                  c=da[0], index=pidx)))
    run("k=1 plain     ", lambda: nat.hartley_fused(one, (0, 1), 1.0, x=X[0].reshape(n, n)))


if __name__ == "__main__":
    main()
