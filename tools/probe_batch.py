"""Per-kernel times of the batched sampling matvec (k right-hand sides) at the
bench problem, vs k single matvecs (nft_prof_* HIP events)."""
import sys
from collections import defaultdict

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402


def prof(fn, reps=5):
    from nifty_amd import _native
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    torch.cuda._sleep(300_000_000)
    with _native.LaunchProfile() as p:
        for _ in range(reps):
            fn()
    acc = defaultdict(float)
    for lab, ms in p.records:
        acc[lab] += ms * 1e3 / reps
    return acc


def main():
    import nifty_amd as ift
    from nifty_amd.minimization.fused_cg import fusable_metric
    ift.config.set_device("cuda:0")
    cf, R, lh, pos, _ = bench.build_problem(ift, 2048, 16384)
    dtype, f_lh = lh.get_transformation()
    fl = f_lh(ift.Linearization.make_var(pos))
    met = (ift.SandwichOperator.make(fl.jac, ift.ScalingOperator(f_lh.target, 1., dtype))
           + ift.ScalingOperator(fl.domain, 1., float))
    core, W, shift = fusable_metric(met)
    lay = core.layout
    for k in (1, 2, 4, 8):
        D = torch.stack([lay.pack(ift.from_random(cf.domain, "normal")) for _ in range(k)])
        Q = torch.zeros_like(D)
        a = prof(lambda: core.metric_flat_batch(D, Q, W, 0.0))
        tot = sum(a.values())
        print(f"k={k}: total {tot:.1f} us = {tot / k:.1f} us per RHS")
        for lab, us in sorted(a.items(), key=lambda kv: -kv[1]):
            print(f"   {lab:22s} {us:8.1f} us  ({us / k:6.1f} per RHS)")


if __name__ == "__main__":
    main()
