"""demo64 linear-CG trace vs the reference (debugging aid)."""
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "tests"))
import test_geovi_trace_gpu as T  # noqa: E402
from conftest import golden  # noqa: E402
from trace_compare import our_events  # noqa: E402


def main():
    import nifty_amd as ift
    from nifty_amd.minimization import fused_cg, trace
    ift.config.set_device("cuda:0")
    if len(sys.argv) > 1:
        fused_cg.CURV_DATA_VALUE = sys.argv[1] != "0"
    G = golden("geovi_trace.npz")
    name = "demo64"
    c = T.CASES[name]
    cf, lh, pos = T._problem(ift, G, name)
    H = ift.StandardHamiltonian(lh, T._ctl(ift, c["lin"]))
    mini = ift.NewtonCG(T._ctl(ift, c["newton"]), max_cg_iterations=c["max_cg"])
    trace.TRACE = []
    ift.random.push_sseq_from_seed(c["seed"])
    ift.draw_samples(pos, H, mini, c["nsamp"], True)
    ift.random.pop_sseq()
    ev = trace.TRACE
    trace.TRACE = None
    for s in range(int(G[name + "_nsamples"])):
        ours = our_events(ev, s)[0][1]
        base = T._ref_events(G, name, "", s)[0][1]
        print(f"sample {s}: ours {len(ours)} checks, ref {len(base)}")
        for i in range(max(len(ours), len(base))):
            o = ours[i] if i < len(ours) else np.nan
            b = base[i] if i < len(base) else np.nan
            do = o - ours[i - 1] if 0 < i < len(ours) else np.nan
            db = b - base[i - 1] if 0 < i < len(base) else np.nan
            print(f"  {i:3d} ours {o:.12g} ref {b:.12g}  dE ours {do:.6g} ref {db:.6g}")


if __name__ == "__main__":
    main()
