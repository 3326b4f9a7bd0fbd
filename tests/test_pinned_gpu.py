"""GPU (page-locked host memory needs the device): the pinned registry behind
prefetched draws (random.py _pin / take_pinned) -- a served array hands over
its pinned tensor once and only as itself (not a view sharing its address),
and the registry stays within its byte and count caps."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_take_pinned_identity(dev):
    from nifty_amd import random as nr
    a = nr._pin(np.random.default_rng(0).standard_normal((512, 512)))
    assert nr.take_pinned(a.T) is None          # same address, other layout
    assert nr.take_pinned(a[:, ::2]) is None
    assert nr.take_pinned(a.reshape(-1)) is None
    t = nr.take_pinned(a)
    assert t is not None and t.is_pinned() and tuple(t.shape) == a.shape
    assert np.shares_memory(t.numpy(), a)
    assert nr.take_pinned(a) is None            # handed over once


def test_pinned_caps(dev, monkeypatch):
    from nifty_amd import random as nr
    monkeypatch.setattr(nr, "_PIN_CAP", 5 << 20)
    kept = [nr._pin(np.ones((1 << 17,))) for _ in range(8)]   # 1 MiB each
    assert nr._pinned_bytes <= 5 << 20 and len(nr._pinned) <= 5
    # the newest survive, the oldest were dropped (their arrays stay valid)
    assert nr.take_pinned(kept[-1]) is not None
    assert nr.take_pinned(kept[0]) is None
    assert all(float(k.sum()) == 1 << 17 for k in kept)
    while nr._pinned:
        nr._unpin(next(iter(nr._pinned)))
    assert nr._pinned_bytes == 0
