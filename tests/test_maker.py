"""CPU: CorrelatedFieldMaker host logic (src/library/correlated_fields.py:
388-1115) -- latent keys against the reference's (cfm.npz), which case lowers
to the fused operator, and the reference's error behaviour.  No compute."""
import numpy as np
import pytest

from conftest import golden


def _keys(G, tag):
    return sorted(k[len(tag) + 2:] for k in G.files if k.startswith(tag + "x_"))


def test_maker_keys_and_lowering():
    import nifty_amd as ift
    from nifty_amd.library.correlated_fields_simple import _CorrelatedFieldModel
    from test_maker_gpu import _maker
    G = golden("cfm.npz")
    for tag in ("prod_", "one_", "unit_", "mat_"):
        cfm = _maker(ift, tag)
        op = cfm.finalize(prior_info=0)
        assert sorted(op.domain.keys()) == _keys(G, tag), tag
        assert isinstance(op, _CorrelatedFieldModel) == (tag == "one_"), tag
        assert op.target.shape == G[tag + "val"].shape


def test_maker_errors():
    import nifty_amd as ift
    sp = ift.RGSpace(16)
    with pytest.raises(NotImplementedError):
        ift.CorrelatedFieldMaker("", total_N=2)
    cfm = ift.CorrelatedFieldMaker("")
    with pytest.raises(ValueError):
        cfm.add_fluctuations(sp, (1., 1.), None, (1., 1.), (-2., 1.))
    with pytest.raises(ValueError):
        cfm.add_fluctuations(sp, (1., 1.), (-1., 1.), None, (-2., 1.))
    with pytest.raises(TypeError):
        cfm.add_fluctuations(sp, (1., 1., 1.), None, None, (-2., 1.))
    with pytest.raises(NotImplementedError):
        cfm.azm
    cfm.add_fluctuations(sp, (1., 1.), None, None, (-2., 1.))
    cfm.add_fluctuations(ift.RGSpace(8), (1., 1.), None, None, (-2., 1.), prefix="b")
    with pytest.raises(TypeError):
        cfm.set_amplitude_total_offset(0., (1., 2., 3.))
    cfm.set_amplitude_total_offset(0., None)
    with pytest.raises(RuntimeError):
        cfm.get_normalized_amplitudes()
    with pytest.raises(NotImplementedError):
        cfm.amplitude
    with pytest.raises(ValueError):
        cfm.slice_fluctuation(2)
    with pytest.raises(ValueError):
        cfm.moment_slice_to_average(-1.)
    assert np.isscalar(cfm.azm) and cfm.azm == 0.
