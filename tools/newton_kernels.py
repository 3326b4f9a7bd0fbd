"""Per-kernel table of one application of the batched geoVI Newton metric
(geovi_batch.metric_batch: M_i v = u + J_i^T J0 u, u = v + J0^T J_i v) on
the bench's C3 problem, k right-hand sides, with HIP events on the launch
stream (nft_prof_*), and the graph-free wall time of the application.
Usage: python tools/newton_kernels.py [k]"""
import os
import sys
import time
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    import nifty_amd as ift
    from nifty_amd import _native
    from nifty_amd.minimization import geovi_batch
    ift.config.set_device("cuda:0")
    cf, R, lh, pos, _ = bench.build_problem(ift, 2048, 16384)
    _, f_lh = lh.get_transformation()
    mini = ift.NewtonCG(ift.GradientNormController(iteration_limit=2))
    gb = geovi_batch.plan(mini, f_lh, None, pos)
    lay = gb.layout
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    X0 = gb.x0.repeat(k, 1) + 0.01 * torch.randn((k, lay.size), dtype=torch.float64, device="cuda", generator=g)
    M = gb.tmean.unsqueeze(0).repeat(k, 1)
    _, _, _, states = gb.evaluate(X0, M)
    mv = gb.metric_batch(states)
    D = torch.randn((k, lay.size), dtype=torch.float64, device="cuda", generator=g)
    Q = torch.empty_like(D)
    for _ in range(3):
        mv(D, Q)
    torch.cuda.synchronize()
    reps = 10
    t = time.perf_counter()
    for _ in range(reps):
        mv(D, Q)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t) / reps * 1e6
    torch.cuda._sleep(200_000_000)
    with _native.LaunchProfile() as p:
        for _ in range(reps):
            mv(D, Q)
    acc = defaultdict(lambda: [0, 0.0])
    for lab, ms in p.records:
        acc[lab][0] += 1
        acc[lab][1] += ms * 1e3
    tot = sum(v[1] for v in acc.values()) / reps
    print(f"Newton metric, k={k}: {wall:.0f} us per application (eager wall), sum of launches {tot:.0f} us")
    for lab, (n, us) in sorted(acc.items(), key=lambda x: -x[1][1]):
        print(f"   {lab:24s} launches {n // reps:3d}  {us / reps:8.1f} us")


if __name__ == "__main__":
    main()
