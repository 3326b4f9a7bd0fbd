"""The RCCL ("nccl") branch of the KL-mean exchange, run on the one GPU of
the box as a world-size-1 process group.

The multi-GPU path is one process per GPU with the KL value +
gradient summed by ONE all-reduce of a packed buffer (utilities.allreduce_sum;
reference src/minimization/sample_list.py:327-341, src/utilities.py:331-390).
The 2-rank tests (test_dist_gpu.py) share one GPU and so run over gloo; here
the same code takes its device-tensor branches (`TorchComm._staged` is false,
`_comm_device` keeps the buffers on the GPU) through RCCL:

* allreduce_sum in fast and deterministic mode on fp64, fp32 and complex
  payloads (a complex run after an odd count of real elements) -- bitwise the
  serial pairwise sum (one rank: the collective adds nothing);
* draw_samples + SampledKLEnergyClass (MGVI and geoVI, mirrored pairs) and the
  KL metric through TorchComm(nccl) -- bitwise the comm=None run.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

CF_ARGS = dict(offset_mean=0, offset_std=(1e-3, 1e-6), fluctuations=(1., 0.8),
               loglogavgslope=(-3., 1), flexibility=(2, 1.), asperity=(0.5, 0.4))


@pytest.fixture(scope="module")
def nccl_comm(dev):
    import torch.distributed as dist
    import nifty_amd as ift
    if dist.is_initialized():
        pytest.skip("a process group is already initialised in this process")
    # HSA_ENABLE_IPC_MODE_LEGACY=0 must be in the environment before the GPU
    # initialises (it is exported on the box and in the image); a world-size-1
    # group exchanges no IPC handles either way
    prev = ift.config.device() if callable(getattr(ift.config, "device", None)) else None
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1)
    ift.config.set_device("cuda:0")
    comm = ift.TorchComm()
    assert comm.backend == "nccl" and comm.Get_size() == 1
    try:
        yield comm
    finally:
        try:
            dist.barrier()
        finally:
            dist.destroy_process_group()
            if prev is not None:
                ift.config.set_device(prev)


def _payloads(seed):
    """three per-sample items: (fp64 Field, fp32 tensor, odd-length fp64
    tensor, complex128 tensor) on the GPU"""
    import nifty_amd as ift
    g = torch.Generator(device="cuda:0")
    g.manual_seed(seed)
    sp = ift.RGSpace((17, 9))
    out = []
    for _ in range(3):
        f = ift.Field(ift.DomainTuple.make(sp), torch.randn(sp.shape, dtype=torch.float64, device="cuda:0",
                                                             generator=g))
        a32 = torch.randn(33, dtype=torch.float32, device="cuda:0", generator=g)
        odd = torch.randn(7, dtype=torch.float64, device="cuda:0", generator=g)
        z = torch.randn(5, dtype=torch.complex128, device="cuda:0", generator=g)
        out.append((f, a32, odd, z))
    return out


def _eq(a, b):
    import nifty_amd as ift
    if isinstance(a, tuple):
        assert len(a) == len(b)
        for x, y in zip(a, b):
            _eq(x, y)
        return
    if isinstance(a, ift.Field):
        assert a.domain == b.domain
        a, b = a.val, b.val
    assert a.dtype == b.dtype and a.device == b.device, (a.dtype, b.dtype, a.device, b.device)
    assert torch.equal(a, b)


@pytest.mark.parametrize("det", [False, True])
def test_allreduce_sum_rccl_bitwise(nccl_comm, det):
    from nifty_amd import utilities
    vals = _payloads(11)
    ref = utilities.pairwise_sum(list(vals))
    got = utilities.allreduce_sum(list(vals), nccl_comm, deterministic=det)
    _eq(got, ref)
    # the buffers stay on the GPU: RCCL takes device tensors in place
    pk = utilities._Packed(ref, nccl_comm)
    assert all(b.is_cuda for b in pk.bufs)
    assert not nccl_comm._staged(pk.bufs[0])


def test_allreduce_tensor_rccl_inplace(nccl_comm):
    t = torch.arange(1000, dtype=torch.float64, device="cuda:0") * 0.1
    ref = t.clone()
    out = nccl_comm.allreduce_tensor_(t)
    assert out.data_ptr() == t.data_ptr() and torch.equal(t, ref)
    c = torch.randn(16, dtype=torch.complex64, device="cuda:0")
    cr = torch.view_as_real(c)
    nccl_comm.allreduce_tensor_(cr)
    assert torch.equal(torch.view_as_complex(cr), c)


def _kl_run(comm):
    import nifty_amd as ift
    from nifty_amd import utilities
    from conftest import golden
    G = golden("losmetric64.npz")
    sp = ift.RGSpace((64, 64))
    cf = ift.SimpleCorrelatedField(sp, **CF_ARGS)
    R = ift.LOSResponse(sp, starts=list(G["starts"]), ends=list(G["ends"]))
    N = ift.ScalingOperator(R.target, 1e-3, np.float64)
    lh = ift.GaussianEnergy(ift.makeField(R.target, G["data"]), inverse_covariance=N.inverse) @ R(ift.sigmoid(cf))
    pos = ift.MultiField.from_dict({k: ift.makeField(cf.domain[k], G["pos_" + k]) for k in cf.domain.keys()},
                                   cf.domain)
    H = ift.StandardHamiltonian(lh, ift.GradientNormController(iteration_limit=10))
    out = {}
    for geo in (False, True):
        for det in (True, False):
            utilities.DETERMINISTIC_ALLREDUCE = det
            try:
                mini = ift.NewtonCG(ift.GradientNormController(iteration_limit=1)) if geo else None
                ift.random.push_sseq_from_seed(51)
                sl = ift.draw_samples(pos, H, mini, 2, True, comm=comm)
                ift.random.pop_sseq()
                kl = ift.SampledKLEnergyClass(sl, H, [], None, True)
                with ift.random.Context(7):
                    v = ift.from_random(cf.domain, "normal")
                mvf = kl.apply_metric(v)
            finally:
                utilities.DETERMINISTIC_ALLREDUCE = False
            out[(geo, det)] = (
                kl.value, {k: kl.gradient[k].val.cpu().numpy() for k in kl.gradient.keys()},
                [{k: sl._r[i][k].val.cpu().numpy() for k in cf.domain.keys()} for i in range(len(sl._r))],
                {k: mvf[k].val.cpu().numpy() for k in mvf.keys()})
    return out


@pytest.fixture(scope="module")
def kl_pair(nccl_comm):
    return _kl_run(None), _kl_run(nccl_comm)


@pytest.mark.parametrize("geo", [False, True])
@pytest.mark.parametrize("det", [True, False])
def test_draw_samples_kl_rccl_bitwise(kl_pair, geo, det):
    """draw_samples + SampledKLEnergyClass + apply_metric through
    TorchComm(nccl) at world size 1: bitwise the comm=None run"""
    single, rccl = kl_pair
    v1, g1, s1, m1 = single[(geo, det)]
    v, g, s, m = rccl[(geo, det)]
    assert v == v1
    for k in g1:
        np.testing.assert_array_equal(g[k], g1[k], err_msg=k)
    assert len(s) == len(s1) > 0
    for a, b in zip(s, s1):
        for k in b:
            np.testing.assert_array_equal(a[k], b[k])
    for k in m1:
        np.testing.assert_array_equal(m[k], m1[k], err_msg=k)
