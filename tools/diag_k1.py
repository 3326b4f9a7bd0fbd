"""diagnostic: a geoVI / MGVI sample drawn alone (k = 1) vs the same sample
drawn in its mirrored pair (k = 2); prints the max relative difference"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import nifty_amd as ift  # noqa: E402
from conftest import golden  # noqa: E402
from test_optimize_kl_gpu import _problem  # noqa: E402

lh, pos = _problem(ift, golden("optkl32.npz"))
H = ift.StandardHamiltonian(lh, ift.GradientNormController(iteration_limit=8))
for geo in (False, True):
    mini = ift.NewtonCG(ift.GradientNormController(iteration_limit=1)) if geo else None
    out = {}
    for mirror in (False, True):
        ift.random.push_sseq_from_seed(61)
        sl = ift.draw_samples(pos, H, mini, 1, mirror)
        ift.random.pop_sseq()
        out[mirror] = sl.local_item(0)
    for k in pos.keys():
        a, b = out[False][k].val.cpu().numpy(), out[True][k].val.cpu().numpy()
        print("geo" if geo else "mgvi", k, float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300)), flush=True)
