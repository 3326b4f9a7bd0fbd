"""Host overhead of the value-driven Newton-direction CG: one batched solve of
k right-hand sides on the geoVI Newton metric (geovi_batch._MetricCore, the
bench's C3 problem) with AbsDeltaEnergyController(iteration_limit=10) as
NewtonCG's direction requests use it -- wall time per iteration from the
host -- against the graph-replayed GPU time of the same iteration body
(direction, matvec, curvature, update).  Usage: python tools/newton_cg_probe.py [k] [--solves-only]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    solves_only = "--solves-only" in sys.argv   # (for a kernel trace of the eager solves)
    import nifty_amd as ift
    from nifty_amd import _native
    from nifty_amd.minimization import fused_cg, geovi_batch
    ift.config.set_device("cuda:0")
    lib = _native.load()
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
    core = geovi_batch._MetricCore(gb.metric_batch(states), lay)
    G = torch.randn((k, lay.size), dtype=torch.float64, device="cuda", generator=g)
    for rep in range(3):
        ctls = [ift.AbsDeltaEnergyController(1e-300, iteration_limit=10) for _ in range(k)]
        cg = fused_cg.FusedCGBatch(core, None, 0.0, ctls, 20)
        starts = [fused_cg._State(0.0, 1.0, lambda: None) for _ in range(k)]
        torch.cuda.synchronize()
        t = time.perf_counter()
        cg.run_packed(torch.zeros_like(G), -G, G, starts)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t
        print(f"solve {rep}: {cg.niter} iterations, {wall * 1e3:.1f} ms, {wall / cg.niter * 1e6:.0f} us per "
              f"iteration (k={k}, path {cg.path})", flush=True)
    if solves_only:
        return
    # where the solve loop's host time goes beyond the body and the read
    import cProfile
    import pstats
    ctls = [ift.AbsDeltaEnergyController(1e-300, iteration_limit=10) for _ in range(k)]
    cg = fused_cg.FusedCGBatch(core, None, 0.0, ctls, 20)
    starts = [fused_cg._State(0.0, 1.0, lambda: None) for _ in range(k)]
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    cg.run_packed(torch.zeros_like(G), -G, G, starts)
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(30)
    n = lay.size
    X, Rr, D = torch.zeros_like(G), -G.clone(), G.clone()
    Q = torch.zeros_like(X)
    SC = torch.zeros((k, _native.CG_NSCALARS), dtype=torch.float64, device=X.device)
    SC[:, _native.CG_GAMMA] = 1.0
    SC[:, _native.CG_GPREV] = 1.0
    ws = _native.workspace(k * lib.nft_reduce_workspace(n), X.device, "cgb")
    bufs = (X, Rr, D, Q, SC, ws)
    for _ in range(2):
        bench.cg_iteration(lib, core, None, 0.0, bufs, k)
    torch.cuda.synchronize()
    gr = fused_cg._capture(lambda: bench.cg_iteration(lib, core, None, 0.0, bufs, k))
    gr.replay()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(10):
        gr.replay()
    ev[1].record()
    torch.cuda.synchronize()
    print(f"graph-replayed iteration body: {ev[0].elapsed_time(ev[1]) * 1e3 / 10:.0f} us (k={k})", flush=True)
    # the same body queued eagerly back to back (no host read between):
    # the device time of eager launches without the host's decision loop
    torch.cuda._sleep(200_000_000)
    ev[0].record()
    for _ in range(10):
        bench.cg_iteration(lib, core, None, 0.0, bufs, k)
    ev[1].record()
    torch.cuda.synchronize()
    print(f"eager iteration body queued back to back: {ev[0].elapsed_time(ev[1]) * 1e3 / 10:.0f} us (k={k})",
          flush=True)
    # the eager loop's host round trip without the controllers: body, async
    # copy of the scalars, wait (stream synchronize / spinning event query)
    host = torch.zeros((k, _native.CG_NSCALARS), dtype=torch.float64).pin_memory()
    for mode in ("stream-sync", "event-spin", "stream-sync"):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(10):
            bench.cg_iteration(lib, core, None, 0.0, bufs, k)
            host.copy_(SC, non_blocking=True)
            if mode == "stream-sync":
                torch.cuda.current_stream().synchronize()
            else:
                e = torch.cuda.Event()
                e.record()
                while not e.query():
                    pass
            h = host.numpy()
            float(h[0, 0])
        wall = (time.perf_counter() - t) / 10
        print(f"eager body + scalar read ({mode}): {wall * 1e6:.0f} us per iteration", flush=True)
    # host enqueue time of one eager iteration body while the GPU is busy
    torch.cuda._sleep(2_000_000_000)
    ts = []
    for _ in range(5):
        t = time.perf_counter()
        bench.cg_iteration(lib, core, None, 0.0, bufs, k)
        ts.append(time.perf_counter() - t)
    torch.cuda.synchronize()
    print(f"host enqueue of one iteration body: {min(ts) * 1e6:.0f} us min, {sorted(ts)[2] * 1e6:.0f} us median",
          flush=True)
    # where the host time goes: the profile of one enqueue
    import cProfile
    import pstats
    torch.cuda._sleep(2_000_000_000)
    pr = cProfile.Profile()
    pr.enable()
    bench.cg_iteration(lib, core, None, 0.0, bufs, k)
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("cumulative").print_stats(25)


if __name__ == "__main__":
    main()
