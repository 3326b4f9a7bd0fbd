"""Per-sample Hamiltonian values: kl_batch vs the operator path."""
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import nifty_amd as ift  # noqa: E402
from nifty_amd.minimization import geovi_batch  # noqa: E402
from test_geovi_batch_gpu import _problem  # noqa: E402

ift.config.set_device("cuda:0")
for kind in ("los", "gauss", "poisson"):
    cf, lh, pos = _problem(ift, kind)
    H = ift.StandardHamiltonian(lh, ift.GradientNormController(iteration_limit=5))
    ift.random.push_sseq_from_seed(7)
    sl = ift.draw_samples(pos, H, None, 2, True)
    ift.random.pop_sseq()
    P = list(sl.local_iterator())
    vals, grads = geovi_batch.kl_batch(H, P)
    for i, p in enumerate(P):
        t = H(ift.Linearization.make_var(p))
        print(kind, i, vals[i], t.val.val.item(), "lh", lh(p).val.item(), "prior", 0.5 * p.s_vdot(p))
