"""Per-kernel time of one batched geoVI Newton-metric matvec (the matvec of
the NewtonCG direction solves, geovi_batch.GeoVIBatch.metric_batch) at the
bench's C3 problem, k samples with their own expansion states, and the
graph-replayed wall time of the matvec and of a whole CG iteration around
it.  Usage: python tools/newton_probe.py [k]"""
import os
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    import nifty_amd as ift
    from nifty_amd import _native
    from nifty_amd.minimization import fused_cg, geovi_batch
    ift.config.set_device("cuda:0")
    cf, R, lh, pos, _ = bench.build_problem(ift, 2048, 16384)
    _, f_lh = lh.get_transformation()
    mini = ift.NewtonCG(ift.GradientNormController(iteration_limit=2))
    gb = geovi_batch.plan(mini, f_lh, None, pos)
    assert gb is not None
    lay = gb.layout
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    X = gb.x0.repeat(k, 1) + 0.01 * torch.randn((k, lay.size), dtype=torch.float64, device="cuda", generator=g)
    M = gb.tmean.unsqueeze(0).repeat(k, 1)
    _, _, _, states = gb.evaluate(X, M)
    mv = gb.metric_batch(states)
    D = torch.randn((k, lay.size), dtype=torch.float64, device="cuda", generator=g)
    Q = torch.zeros_like(D)
    for _ in range(3):
        mv(D, Q)
    torch.cuda.synchronize()
    torch.cuda._sleep(200_000_000)
    reps = 5
    with _native.LaunchProfile() as prof:
        for _ in range(reps):
            mv(D, Q)
    acc = defaultdict(lambda: [0, 0.0])
    for lab, ms in prof.records:
        acc[lab][0] += 1
        acc[lab][1] += ms
    tot = 0.0
    for lab, (c, ms) in sorted(acc.items(), key=lambda kv: -kv[1][1]):
        tot += ms / reps
        print(f"  {lab:24s} launches/mv {c // reps:3d}  {ms / reps * 1e3:8.1f} us per mv", flush=True)
    print(f"sum of marked launches {tot * 1e3:.1f} us per mv (k={k})", flush=True)
    # wall: eager and graph-replayed
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        mv(D, Q)
    ev[1].record()
    torch.cuda.synchronize()
    print(f"eager mv wall {ev[0].elapsed_time(ev[1]) * 1e3 / reps:.1f} us", flush=True)
    gr = fused_cg._capture(lambda: mv(D, Q))
    gr.replay()
    torch.cuda.synchronize()
    ev[0].record()
    for _ in range(reps * 4):
        gr.replay()
    ev[1].record()
    torch.cuda.synchronize()
    print(f"graph mv wall {ev[0].elapsed_time(ev[1]) * 1e3 / (4 * reps):.1f} us", flush=True)
    # torch kernels inside one mv
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CUDA]) as p:
        mv(D, Q)
        torch.cuda.synchronize()
    by = defaultdict(lambda: [0, 0.0])
    for e in p.events():
        if e.device_type == torch.autograd.DeviceType.CUDA:
            by[e.name][0] += 1
            by[e.name][1] += e.time_range.elapsed_us()
    for nm, (c, us) in sorted(by.items(), key=lambda kv: -kv[1][1])[:30]:
        print(f"    {us:9.1f} us {c:4d}  {nm[:100]}", flush=True)


if __name__ == "__main__":
    main()
