"""The bench's batched CG iteration (C3, 4 RHS) captured as the HIP graph the
timed loop replays, replayed REPLAYS times (default 20) -- the command to
run under rocprofv3 --kernel-trace so that tools/trace_labels.py can
summarise the replayed kernels per label (profiles/*_trace_labels.json).
Prints the HIP-event wall time per replay."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import nifty_amd as ift
    from nifty_amd import _native
    from nifty_amd.minimization import fused_cg
    ift.config.set_device("cuda:0")
    cf, R, lh, pos, _ = bench.build_problem(ift, 2048, 16384)
    k = 4
    lib = _native.load()
    core, W, shift, XS = bench.probe_setup(ift, lh, pos, k)
    X, Rr, D = XS[:k].clone(), XS[k:2 * k].clone(), XS[2 * k:].clone()
    Q = torch.zeros_like(X)
    SC = torch.zeros((k, _native.CG_NSCALARS), dtype=torch.float64, device=X.device)
    SC[:, _native.CG_GAMMA] = 1.0
    SC[:, _native.CG_GPREV] = 1.0
    ws = _native.workspace(k * lib.nft_reduce_workspace(X.shape[1]), X.device, "cgb")
    bufs = (X, Rr, D, Q, SC, ws)

    def body():
        # as bench.cg_iteration_wall: every replay continues the CG (the
        # scalars never freeze a right-hand side), no restore inside the graph
        bench.cg_iteration(lib, core, W, shift, bufs, k)
    for _ in range(3):
        body()
    torch.cuda.synchronize()
    lz = bench.lazy_spec(core, k, X.shape[1], X.dtype) if os.environ.get("LAZY_CHUNK") == "1" else None
    if lz is not None:
        # the timed loop's count-only chunk: REPLAYS (19) steps with the
        # deferred iterate from slot 0, then the flush (the trace's trailing
        # dispatch, outside the periodic tail tools/trace_labels.py reads)
        wall = bench.cg_iteration_lazy_wall(lib, core, W, shift, bufs, k, lz, int(os.environ.get("REPLAYS", "19")))
        print(f"lazy chunk: {wall:.1f} us per iteration, flush included", flush=True)
        return
    g = fused_cg._capture(body)
    g.replay()
    torch.cuda.synchronize()
    reps = int(os.environ.get("REPLAYS", "20"))
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(reps):
        g.replay()
    t1.record()
    torch.cuda.synchronize()
    if float(SC[:, _native.CG_DONE].abs().sum()) != 0.0:
        raise RuntimeError("replay_probe: a right-hand side froze during the replays")
    print(f"graph replay: {t0.elapsed_time(t1) * 1e3 / reps:.1f} us per iteration ({reps} replays)", flush=True)


if __name__ == "__main__":
    main()
