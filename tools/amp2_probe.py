"""Kernel-level probe of the bench's batched CG iteration (4 RHS, 2048^2 LOS
problem): runs the iteration body (bench.cg_iteration, the timed loop's
kernels and arguments) `PROBE_REPS` times -- for rocprofv3 --kernel-trace
--stats -- and prints the HIP-event duration of the graph-replayed
iteration.  NFT_CG_AMP2=0 gives the separate amplitude launches; PROBE_N sets
the grid (default 2048), NFT_LIB another build of the library."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import nifty_amd as ift
    from nifty_amd import _native
    ift.config.set_device("cuda:0")
    n = int(os.environ.get("PROBE_N", "2048"))
    cf, R, lh, pos, _ = bench.build_problem(ift, n, 16384)
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
    reps = int(os.environ.get("PROBE_REPS", "30"))
    for _ in range(reps):
        bench.cg_iteration(lib, core, W, shift, bufs, k)
    torch.cuda.synchronize()
    if os.environ.get("PROBE_NOWALL"):  # the kernel trace only (ablation builds)
        return
    us = bench.cg_iteration_wall(lib, core, W, shift, bufs, k)
    print("NFT_CG_AMP2=%s N=%d iteration %.1f us" % (os.environ.get("NFT_CG_AMP2", "1"), n, us), flush=True)


if __name__ == "__main__":
    main()
