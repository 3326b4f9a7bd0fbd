"""Print the build's and the reference's decision trace of one geoVI trace
case (tests/golden/geovi_trace.npz) side by side (debugging aid)."""
import sys
import numpy as np
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import torch  # noqa
from conftest import golden
import test_geovi_trace_gpu as T
from trace_compare import our_events
import nifty_amd as ift
from nifty_amd.minimization import geovi_batch, trace

name = sys.argv[1]
batched = sys.argv[2] == "1"
G = golden("geovi_trace.npz")
c = T.CASES[name]
cf, lh, pos = T._problem(ift, G, name)
H = ift.StandardHamiltonian(lh, T._ctl(ift, c["lin"]))
mini = ift.NewtonCG(T._ctl(ift, c["newton"]), max_cg_iterations=c["max_cg"])
geovi_batch.ENABLED = batched
trace.TRACE = []
ift.random.push_sseq_from_seed(c["seed"])
sl = ift.draw_samples(pos, H, mini, c["nsamp"], True, napprox=c.get("napprox", 0))
ift.random.pop_sseq()
ev = trace.TRACE
trace.TRACE = None
np.set_printoptions(precision=10, linewidth=200)
from nifty_amd.minimization import trace as _tr
for t, v in _tr.by_tag(ev).items():
    if t[0] == "trialD":
        print(t, v)
for s in range(int(G[name + "_nsamples"])):
    ours = our_events(ev, s)
    base = T._ref_events(G, name, "", s)
    perts = [T._ref_events(G, name, f"p{j + 1}_", s) for j in range(int(G[name + "_nperturbed"]))]
    for i, (k, vb) in enumerate(base):
        vo = ours[i][1] if i < len(ours) else []
        print(f"s{s} ev{i} {k}: ours {len(vo)} ref {len(vb)} perts {[len(p[i][1]) for p in perts if i < len(p)]}")
        if k in ("dir", "newton", "trial", "trialE"):
            print("   ours", np.array(vo))
            print("   ref ", np.array(vb))
            for p in perts:
                if i < len(p):
                    print("   pert", np.array(p[i][1]))
