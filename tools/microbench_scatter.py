"""bin_scatter at 2048^2 (k=1 and k=4): real power-spectrum binning vs the
same bin sizes with a sorted (identity) permutation -- separates the gather
cost from the per-bin phase."""
import sys
from collections import defaultdict

import numpy as np
import torch

sys.path.insert(0, ".")
import nifty_amd as ift  # noqa: E402
from nifty_amd import _native as nat  # noqa: E402
from nifty_amd.operators.distributors import BinIndex  # noqa: E402


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


def main(n=2048):
    ift.config.set_device("cuda:0")
    h = ift.RGSpace((n, n), harmonic=True)
    pidx = np.asarray(ift.PowerSpace(h).pindex).ravel()
    B = int(pidx.max()) + 1
    N = pidx.size
    for lab, pi in (("power", pidx),):
        for po in (False,):
            b = BinIndex(pi, B, "cuda")
            b.PIXEL_ORDER = po
            for k in (1, 4):
                w = torch.randn(k, N, dtype=torch.float64, device="cuda")
                ga = torch.empty(k, B, dtype=torch.float64, device="cuda")
                run(f"{lab:6s} pixel_order={po} k={k}",
                    lambda: nat.bin_scatter(w, b.perm, b.offsets, ga, k, N, B, 1, order=b.gather_order))
                run(f"{lab:6s} no-order         k={k}",
                    lambda: nat.bin_scatter(w, b.perm, b.offsets, ga, k, N, B, 1))
                bf = BinIndex(pi.reshape(n, n), B, "cuda", fold=True)
                run(f"{lab:6s} mirror-folded    k={k}", lambda: bf.scatter(w, ga, k))


if __name__ == "__main__":
    main()
