"""LOS forward / adjoint timing on the bench's plan (2048^2, 16384 lines,
K = 4 vectors, one shared column scale as in the sampling metric): one
workgroup per work item vs one per box, segments in (box, line) order vs
longest first, bitwise checked against each other (tuning probe only)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def timed(fn, reps=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    import nifty_amd as ift
    from nifty_amd import _native as nat
    ift.config.set_device("cuda:0")
    cf, R, lh, pos, _ = bench.build_problem(ift, 2048, 16384)
    k = 4
    N = 2048 * 2048
    X = torch.randn((k, N), dtype=torch.float64, device="cuda")
    cs = torch.rand((k, N), dtype=torch.float64, device="cuda")
    y = torch.empty((k, R.target.shape[0]), dtype=torch.float64, device="cuda")
    out = torch.empty_like(X)
    from nifty_amd.library import los_response
    ref = None
    sp = R.domain[0]
    for name, boxwg, tile, srt in (("items", False, 1, False), ("boxes", True, 1, False)):
        los_response.BOX_WG = boxwg
        los_response.TILE = tile
        los_response.SORT_SEGMENTS = srt
        R._plan_np = los_response.box_plan(*R._coo, sp.shape, R.target.shape[0])
        R._plan = None
        plan = R._box_plan()
        y.zero_()
        nat.los_forward_ex(plan, X, y, colscale=cs[0])
        if ref is None:
            ref = y.clone()
        else:
            d = float(((y - ref).abs().max() / ref.abs().max()).item())
            print(f"{name} bitwise equal: {bool(torch.equal(ref, y))}, max rel diff {d:.3g}", flush=True)
        for rep in range(2):
            us = timed(lambda: nat.los_forward_ex(plan, X, y, colscale=cs[0]))
            print(f"fwd {name} {us:.1f} us", flush=True)
        with nat.LaunchProfile() as prof:
            for _ in range(10):
                nat.los_forward_ex(plan, X, y, colscale=cs[0])
        acc = {}
        for lab, ms in prof.records:
            acc.setdefault(lab, []).append(ms * 1e3)
        print("   " + ", ".join(f"{k} {sum(v) / len(v):.1f} us" for k, v in acc.items()), flush=True)
    aref = None
    for pad in (False, True, False, True):
        los_response.ADJ_VEC = pad
        los_response.ADJ_PAD = False
        R._plan_np = los_response.box_plan(*R._coo, sp.shape, R.target.shape[0])
        R._plan = None
        plan = R._box_plan()
        out.zero_()
        nat.los_adjoint_batched(plan, y, out, rowscale=cs[0])
        if aref is None:
            aref = out.clone()
        eq = bool(torch.equal(aref, out))
        print(f"adj vec={int(pad)} {timed(lambda: nat.los_adjoint_batched(plan, y, out, rowscale=cs[0])):.1f} us "
              f"(bitwise equal: {eq})", flush=True)


if __name__ == "__main__":
    main()
