"""Component check of the batched geoVI energy (minimization/geovi_batch.py)
against the operator path: transformation mean, value, gradient, f_lh,
per-sample Jacobian and its adjoint, Newton metric."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import nifty_amd as ift  # noqa: E402
from nifty_amd.minimization import geovi_batch  # noqa: E402
from test_geovi_batch_gpu import _problem  # noqa: E402


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


def main(kind):
    ift.config.set_device("cuda:0")
    cf, lh, pos = _problem(ift, kind)
    dtype, f_lh = lh.get_transformation()
    fl = f_lh(ift.Linearization.make_var(pos))
    transformation = ift.ScalingOperator(f_lh.domain, 1.) + fl.jac.adjoint @ f_lh
    tmean = pos + fl.jac.adjoint(fl.val)
    mini = ift.NewtonCG(ift.GradientNormController(iteration_limit=1))
    gb = geovi_batch.plan(mini, f_lh, None, pos)
    lay = gb.layout
    keys = list(cf.domain.keys())
    t_b = lay.unpack(gb.tmean)
    print("tmean", {k: rel(t_b[k].val.cpu().numpy(), tmean[k].val.cpu().numpy()) for k in keys})
    ift.random.push_sseq_from_seed(3)
    y = ift.from_random(cf.domain, "normal")
    p2 = pos + 0.3 * ift.from_random(cf.domain, "normal")
    v = ift.from_random(cf.domain, "normal")
    m = tmean + y
    en = ift.EnergyAdapter(p2, ift.GaussianEnergy(m) @ transformation, nanisinf=True, want_metric=True)
    X = torch.stack([lay.pack(p2), lay.pack(pos)])
    M = torch.stack([gb.tmean + lay.pack(y), gb.tmean + lay.pack(y)])
    vals, gn, G, states = gb.evaluate(X, M)
    print("value", vals[0], en.value, "rel", abs(vals[0] - en.value) / abs(en.value))
    print("gnorm", gn[0], en.gradient_norm)
    g_b = lay.unpack(G[0])
    print("grad", {k: rel(g_b[k].val.cpu().numpy(), en.gradient[k].val.cpu().numpy()) for k in keys})
    F, st = gb.pipe.fwd(X[:1])
    fref = f_lh(p2).val.cpu().numpy()
    print("f_lh", rel(F[0].cpu().numpy().reshape(fref.shape), fref))
    fl2 = f_lh(ift.Linearization.make_var(p2))
    jv = gb.pipe.jvp(st, lay.pack(v).reshape(1, -1))
    jref = fl2.jac(v).val.cpu().numpy()
    print("J v", rel(jv[0].cpu().numpy().reshape(jref.shape), jref))
    jv2 = gb.pipe.jvp(states, torch.stack([lay.pack(v), lay.pack(v)]))
    print("J v (batch of 2, per item)", rel(jv2[0].cpu().numpy().reshape(jref.shape), jref))
    u = ift.from_random(fl2.target, "normal")
    Q = torch.zeros((1, lay.size), dtype=torch.float64, device="cuda")
    jtu = lay.unpack(gb.pipe.vjp(st, u.val.reshape((1,) + tuple(u.val.shape)).contiguous(), Q)[0])
    jtref = fl2.jac.adjoint(u)
    print("J^T u", {k: rel(jtu[k].val.cpu().numpy(), jtref[k].val.cpu().numpy()) for k in keys})
    U2 = torch.stack([u.val, u.val]).contiguous()
    Q2 = torch.zeros((2, lay.size), dtype=torch.float64, device="cuda")
    jtu2 = lay.unpack(gb.pipe.vjp(states, U2, Q2)[0])
    print("J^T u (batch of 2)", {k: rel(jtu2[k].val.cpu().numpy(), jtref[k].val.cpu().numpy()) for k in keys})
    mv = gb.metric_batch(gb.pipe.stack([(states, 0)]))
    Qm = torch.zeros((1, lay.size), dtype=torch.float64, device="cuda")
    mv(lay.pack(v).reshape(1, -1), Qm)
    mref = en.metric(v)
    mb = lay.unpack(Qm[0])
    print("metric", {k: rel(mb[k].val.cpu().numpy(), mref[k].val.cpu().numpy()) for k in keys})
    ift.random.pop_sseq()


if __name__ == "__main__":
    for kind in sys.argv[1:] or ["los", "gauss", "poisson"]:
        print("==", kind, flush=True)
        main(kind)
