"""Random-number state: a stack of numpy SeedSequences / PCG64 Generators.

Same semantics as src/random.py:84-291 (push/pop, spawn_sseq, Context), so a
given seed produces the identical stream of normals as the reference.  Draws
are made on the host with numpy (bit-compatibility, SURVEY.md §7 "hard parts")
and uploaded to the device by Field.from_random.

Host draws are the one part of sampling that does not run on the GPU (4M
normals take ~45 ms on one core), so they are taken off the critical path:
every Context records the draws made in it (a "script"); draw_samples asks
``prefetch`` to replay that script on background threads (one seed each) for the seed
sequences it will use next (the remaining local samples, and the children the
next spawn_sseq call will produce).  A Context entered with a prefetched seed
serves the pre-drawn arrays while the requests match the script, and
otherwise rebuilds the exact generator state (re-drawing what it served) and
continues from the generator: results are bit-identical either way; a wrong
prediction only costs background CPU time.
"""
import os
import threading
import weakref
from concurrent.futures import ThreadPoolExecutor

import numpy as np

_sseq = [np.random.SeedSequence(42)]
_rng = [np.random.default_rng(_sseq[-1])]


def getState():
    import pickle
    return pickle.dumps((_sseq, _rng))


def setState(state):
    import pickle
    global _sseq, _rng
    _sseq, _rng = pickle.loads(state)


def spawn_sseq(n, parent=None):
    if parent is None:
        parent = _sseq[-1]
    return parent.spawn(n)


def current_rng():
    return _rng[-1]


def push_sseq(sseq):
    _sseq.append(sseq)
    _rng.append(np.random.default_rng(_sseq[-1]))


def push_sseq_from_seed(seed):
    _sseq.append(np.random.SeedSequence(seed))
    _rng.append(np.random.default_rng(_sseq[-1]))


def pop_sseq():
    _sseq.pop()
    _rng.pop()


class Random:
    @staticmethod
    def pm1(dtype, shape):
        if np.issubdtype(dtype, np.complexfloating):
            x = np.array([1 + 0j, 0 + 1j, -1 + 0j, 0 - 1j], dtype=dtype)
            x = x[_rng[-1].integers(0, 4, size=shape)]
        else:
            x = 2 * _rng[-1].integers(0, 2, size=shape) - 1
        return x.astype(dtype, copy=False)

    @staticmethod
    def normal(dtype, shape, mean=0., std=1.):
        if not (np.issubdtype(dtype, np.floating) or np.issubdtype(dtype, np.complexfloating)):
            raise TypeError("dtype must be float or complex")
        if not np.isscalar(mean) or not np.isscalar(std):
            raise TypeError("mean and std must be scalars")
        if np.issubdtype(type(std), np.complexfloating):
            raise TypeError("std must not be complex")
        if ((not np.issubdtype(dtype, np.complexfloating)) and
                np.issubdtype(type(mean), np.complexfloating)):
            raise TypeError("mean must not be complex for a real result field")
        if np.issubdtype(dtype, np.complexfloating):
            x = np.empty(shape, dtype=dtype)
            x.real = _rng[-1].normal(np.real(mean), std, shape)
            x.imag = _rng[-1].normal(np.imag(mean), std, shape)
        else:
            x = _rng[-1].normal(mean, std, shape).astype(dtype, copy=False)
        return x

    @staticmethod
    def uniform(dtype, shape, low=0., high=1.):
        if not np.isscalar(low) or not np.isscalar(high):
            raise TypeError("low and high must be scalars")
        if np.issubdtype(dtype, np.complexfloating):
            x = np.empty(shape, dtype=dtype)
            x.real = _rng[-1].uniform(low, high, shape)
            x.imag = _rng[-1].uniform(low, high, shape)
        elif np.issubdtype(dtype, np.integer):
            x = _rng[-1].integers(low, high + 1, shape)
        else:
            x = _rng[-1].uniform(low, high, shape)
        return x.astype(dtype, copy=False)


# ------------------------------------------------------------- prefetching
_RECORDED = ("normal", "uniform", "integers")


def _req(method, args, kwargs):
    def norm(v):
        if isinstance(v, (list, tuple)):
            return tuple(int(a) for a in v)
        if isinstance(v, (np.integer, int)):
            return int(v)
        if isinstance(v, (np.floating, float)):
            return float(v)
        if isinstance(v, type):
            return v.__name__
        return v
    return (method, tuple(norm(a) for a in args), tuple(sorted((k, norm(v)) for k, v in kwargs.items())))


def _sseq_key(ss):
    return (repr(ss.entropy), tuple(ss.spawn_key), ss.pool_size)


class _Recorder:
    """Generator proxy that logs the recorded draw requests of a Context."""

    def __init__(self, gen):
        self._gen = gen
        self.script = []

    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        attr = getattr(self._gen, name)
        if name in _RECORDED:
            def rec(*args, **kwargs):
                if self.script is not None:
                    self.script.append(_req(name, args, kwargs))
                return attr(*args, **kwargs)
            return rec
        self.script = None  # an unrecorded draw: the script cannot be replayed
        return attr


class _Serving:
    """Generator proxy that serves prefetched draws while requests match."""

    def __init__(self, sseq, script, arrays):
        self._sseq = sseq
        self._script, self._arrays = script, arrays
        self._pos = 0
        self._gen = None
        self.script = []

    def _materialize(self):
        if self._gen is None:
            g = np.random.default_rng(self._sseq)
            for (name, args, kw) in self._script[:self._pos]:
                getattr(g, name)(*args, **dict(kw))
            self._gen = g
        return self._gen

    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        if self._gen is None and name in _RECORDED:
            def serve(*args, **kwargs):
                r = _req(name, args, kwargs)
                if self.script is not None:
                    self.script.append(r)
                if self._gen is None and self._pos < len(self._script) and self._script[self._pos] == r:
                    self._pos += 1
                    return self._arrays[self._pos - 1]
                return getattr(self._materialize(), name)(*args, **kwargs)
            return serve
        if name not in _RECORDED:
            self.script = None
        return getattr(self._materialize(), name)


_pool = None
# background generator threads: each prefetched seed sequence replays its
# script on its own generator (numpy fills release the GIL), so the samples'
# draws are made side by side; the values do not depend on the thread count.
# (One thread: the 4 x 2 x 16.7M normals of a 4096^2 step took 813 of its
# 1242 ms waiting for the host.)
_WORKERS = max(1, int(os.environ.get("NFT_RNG_WORKERS", "4")))
_cache = {}
_lock = threading.Lock()
last_script = None


# Large prefetched draws are written into page-locked host memory on the
# background thread, so the Field upload of a served array is an asynchronous
# DMA instead of a pageable copy the host waits for (field._to_tensor looks the
# pinned tensor up by address).  The served array is a view of that memory:
# the same values, only where they live differs.
_PIN_BYTES = 1 << 20
_PIN_CAP = 1 << 31          # page-locked bytes held for served draws at most
_pinned = {}                # address -> (pinned tensor, weakref of the served array)
_pinned_bytes = 0


def _unpin(key):
    global _pinned_bytes
    ent = _pinned.pop(key, None)
    if ent is not None:
        _pinned_bytes -= ent[0].numel() * ent[0].element_size()
    return ent


def _pin(a):
    global _pinned_bytes
    if not isinstance(a, np.ndarray) or a.nbytes < _PIN_BYTES or a.dtype.kind not in "fc":
        return a
    try:
        import torch
        if not torch.cuda.is_available():
            return a
        t = torch.from_numpy(np.ascontiguousarray(a)).pin_memory()
    except Exception:     # no page-locked memory available: serve the plain array
        return a
    v = t.numpy()
    with _lock:
        _unpin(v.ctypes.data)
        _pinned[v.ctypes.data] = (t, weakref.ref(v))
        _pinned_bytes += t.numel() * t.element_size()
        # draws converted before their upload (fp32 casts, complex assembly,
        # arithmetic) never come back: the oldest go first, by count and bytes
        while _pinned and (len(_pinned) > 64 or _pinned_bytes > _PIN_CAP):
            _unpin(next(iter(_pinned)))
    return v


def take_pinned(arr):
    """the page-locked tensor behind a served prefetched draw, or None: only
    for the served array object itself (a view of it -- transposed, sliced --
    shares its address but not its layout)"""
    if not _pinned or not isinstance(arr, np.ndarray):
        return None
    with _lock:
        ent = _pinned.get(arr.ctypes.data)
        if ent is None or ent[1]() is not arr:
            return None
        _unpin(arr.ctypes.data)
    t = ent[0]
    if tuple(t.shape) != arr.shape or t.numpy().dtype != arr.dtype or not arr.flags.c_contiguous:
        return None
    return t


def _run_script(sseq, script):
    g = np.random.default_rng(sseq)
    return [_pin(getattr(g, name)(*args, **dict(kw))) for (name, args, kw) in script]


def predict_spawn(n, parent=None):
    """The SeedSequences the next spawn_sseq(n, parent) call will return,
    without spawning."""
    if parent is None:
        parent = _sseq[-1]
    k0 = parent.n_children_spawned
    return [np.random.SeedSequence(parent.entropy, spawn_key=tuple(parent.spawn_key) + (k0 + i,),
                                   pool_size=parent.pool_size) for i in range(n)]


def prefetch(sseqs, script):
    """Replay `script` for each SeedSequence in the background."""
    global _pool
    if not script:
        return
    if _pool is None:
        _pool = ThreadPoolExecutor(max_workers=_WORKERS, thread_name_prefix="nft-rng")
    with _lock:
        for ss in sseqs:
            key = _sseq_key(ss)
            if key not in _cache:
                _cache[key] = (list(script), _pool.submit(_run_script, ss, list(script)))
        while len(_cache) > 16:
            _cache.pop(next(iter(_cache)))


def _take(sseq):
    with _lock:
        ent = _cache.pop(_sseq_key(sseq), None)
    if ent is None:
        return None
    script, fut = ent
    return script, fut.result()


class Context:
    """``with Context(seed_or_sseq): ...`` scoped RNG state (random.py:261-291)."""

    def __init__(self, inp):
        if not isinstance(inp, np.random.SeedSequence):
            inp = np.random.SeedSequence(inp)
        self._sseq = inp

    def __enter__(self):
        self._depth = len(_sseq)
        pre = _take(self._sseq)
        _sseq.append(self._sseq)
        if pre is None:
            self._proxy = _Recorder(np.random.default_rng(self._sseq))
        else:
            self._proxy = _Serving(self._sseq, *pre)
        _rng.append(self._proxy)

    def __exit__(self, exc_type, exc_value, tb):
        global last_script
        pop_sseq()
        if self._depth != len(_sseq):
            raise RuntimeError("inconsistent RNG usage detected")
        if self._proxy.script:
            last_script = self._proxy.script
        return exc_type is None

    @property
    def script(self):
        """draw requests made so far in this context (None if not replayable)"""
        return self._proxy.script
