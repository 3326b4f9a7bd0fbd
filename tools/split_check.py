"""Does the two-stream CG iteration (fused_cg._SplitIteration) overlap?
Times R iterations eagerly and as HIP-graph replays, split and one-stream, at
the bench size (2048^2, 4 RHS).  Usage: python tools/split_check.py"""
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(reps):
        fn()
    t1.record()
    torch.cuda.synchronize()
    return t0.elapsed_time(t1) * 1e3 / reps


def main():
    import nifty_amd as ift
    from nifty_amd import _native
    from nifty_amd.minimization import fused_cg
    ift.config.set_device("cuda:0")
    cf, R, lh, pos, _ = bench.build_problem(ift, 2048, 16384)
    k = 4
    core, W, shift, XS = bench.probe_setup(ift, lh, pos, k)
    lib = _native.load()
    n = XS.shape[1]
    X, Rr, D = XS[:k].clone(), XS[k:2 * k].clone(), XS[2 * k:].clone()
    Q = torch.zeros_like(X)
    SC = torch.zeros((k, _native.CG_NSCALARS), dtype=torch.float64, device=X.device)
    SC[:, _native.CG_GAMMA] = 1.0
    SC[:, _native.CG_GPREV] = 1.0
    SC0 = SC.clone()
    ws = _native.workspace(k * lib.nft_reduce_workspace(n), X.device, "cgb")
    bufs = (X, Rr, D, Q, SC, ws)
    nq = fused_cg._quad_blocks(core, W, X.dtype)
    split = fused_cg._SplitIteration(lib, core, W, n, k, nq, shift, False)

    def one():
        SC.copy_(SC0)
        bench.cg_iteration(lib, core, W, shift, bufs, k)

    def two():
        SC.copy_(SC0)
        split(X, Rr, D, Q, None, SC)

    def amp_only():
        da = core.mv_amp_jvp(D)
        core.mv_amp_vjp(D, core._mv_bufs(k)["w"], Q, 0.0)
        return da

    res = {}
    if "--trace" in sys.argv:     # a few eager split iterations for a kernel trace
        for _ in range(5):
            two()
        torch.cuda.synchronize()
        return
    if "--trace-graph" in sys.argv:   # graph replays of the one-stream iteration
        for _ in range(3):
            one()
        g = fused_cg._capture(one)
        for _ in range(5):
            g.replay()
        torch.cuda.synchronize()
        return
    for name, fn in (("one-stream", one), ("split", two), ("amp chains only", amp_only)):
        res[name + " eager"] = timeit(fn)
        g = fused_cg._capture(fn)
        res[name + " graph"] = timeit(g.replay)
    for kk, v in res.items():
        print(f"{kk:28s} {v:8.1f} us per iteration", flush=True)


if __name__ == "__main__":
    main()
