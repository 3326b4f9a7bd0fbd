"""ctypes binding of ``libnifty_amd.so`` (the C ABI declared in
``include/nifty_amd.h``).

PyTorch is plumbing only: it owns the device buffers (caching allocator) and
the stream; every hot-path computation is a call into the HIP library.  There
is no CPU fallback: calling a hot-path function on a CPU tensor, or on a
machine where the library cannot be loaded, raises.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NFT_LIB") or os.path.join(_HERE, "libnifty_amd.so")

# names and argument signatures of every exported symbol (kept in sync with
# include/nifty_amd.h; tests/test_abi.py checks both directions)
_i, _i64, _sz, _d, _p = ctypes.c_int, ctypes.c_int64, ctypes.c_size_t, ctypes.c_double, ctypes.c_void_p
SIGNATURES = {
    "nft_last_error": (ctypes.c_char_p, []),
    "nft_release_caches": (None, []),
    "nft_fft_prepare": (_i, [_i, _i]),
    "nft_hartley_workspace": (_i, [_i, _p, _i, _p, _i, ctypes.POINTER(_sz)]),
    "nft_hartley": (_i, [_p, _p, _i, _p, _i, _p, _i, _i, _d, _p, _sz, _p]),
    "nft_fft_c2c": (_i, [_p, _p, _i, _p, _i, _p, _i, _i, _d, _p]),
    "nft_reduce_workspace": (_sz, [_i64]),
    "nft_dot": (_i, [_p, _p, _i64, _i, _p, _p, _p]),
    "nft_scale": (_i, [_p, _i64, _i, _d, _p]),
    "nft_sigmoid_pair": (_i, [_p, _p, _p, _i64, _i, _p]),
    "nft_cg_curv": (_i, [_p, _p, _i64, _i, _d, _p, _p, _p]),
    "nft_dot_batched": (_i, [_p, _p, _i64, _i64, _i, _i, _p, _i64, _p, _p]),
    "nft_cg_curv_batched": (_i, [_p, _p, _i64, _i64, _i, _i, _d, _p, _p, _p]),
    "nft_cg_update_batched": (_i, [_p, _p, _p, _p, _p, _i64, _i64, _i, _i, _d, _p, _p, _p]),
    "nft_cg_direction_batched": (_i, [_p, _p, _i64, _i64, _i, _i, _p, _p]),
    "nft_cg_residual_batched": (_i, [_p, _p, _p, _p, _i64, _i64, _i, _i, _d, _p, _p, _p]),
    "nft_cg_update": (_i, [_p, _p, _p, _p, _p, _i64, _i, _d, _p, _p, _p]),
    "nft_cg_direction": (_i, [_p, _p, _i64, _i, _p, _p]),
    "nft_cg_residual": (_i, [_p, _p, _p, _p, _i64, _i, _d, _p, _p, _p]),
    "nft_bin_gather": (_i, [_p, _p, _p, _i64, _i64, _i64, _i64, _i, _p]),
    "nft_bin_scatter": (_i, [_p, _p, _p, _p, _i64, _i64, _i64, _i64, _i, _p]),
    "nft_bin_chunk": (_i, []),
    "nft_bin_fold": (_i, [_p, _p, _i64, _i, _p, _i, _p]),
    "nft_bin_fold_half": (_i, [_p, _p, _i64, _i, _p, _i, _p]),
    "nft_bin_fold_half_sorted": (_i, [_p, _p, _p, _i64, _i, _p, _i, _p]),
    "nft_bin_scatter_il_chunk": (_i, [_i64]),
    "nft_bin_scatter_il": (_i, [_p, _p, _p, _p, _p, _i64, _i64, _i64, _i, _p]),
    "nft_bin_scatter_folded": (_i, [_p, _p, _p, _p, _p, _i64, _i64, _i64, _i, _p]),
    "nft_bin_scatter_ordered": (_i, [_p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _i, _p]),
    "nft_spmv_csr": (_i, [_p, _p, _p, _p, _p, _i64, _i, _d, _i64, _p]),
    "nft_csr_rowblocks": (_i, [_p, _i64, _p, _i64, ctypes.POINTER(_i64)]),
    "nft_spmv_scaled": (_i, [_p, _p, _p, _p, _i64, _p, _p, _p, _p, _i64, _i, _d, _p]),
    "nft_hartley_fused_workspace": (_i, [_i, _p, _i, _p, _i, ctypes.POINTER(_sz)]),
    "nft_hartley_fused": (_i, [_p, _p, _p, _i, _p, _i, _p, _i, _i, _d, _p, _sz, _p]),
    "nft_los_workspace": (_sz, [_p]),
    "nft_los_forward": (_i, [_p, _p, _p, _p, _p, _p, _i, _d, _p]),
    "nft_los_adjoint": (_i, [_p, _p, _p, _p, _p, _i, _d, _p]),
    "nft_los_forward_batched": (_i, [_p, _p, _p, _p, _p, _p, _i, _d, _i, _i64, _i64, _p]),
    "nft_los_adjoint_batched": (_i, [_p, _p, _p, _p, _p, _i, _d, _i, _i64, _i64, _p]),
    "nft_los_adjoint_fold": (_i, [_p, _p, _p, _p, _p, _i, _d, _i, _i64, _i64, _p, _i, _i, _p, _i64, _p]),
    "nft_los_quad_blocks": (_i, [_p]),
    "nft_los_forward_quad_batched": (_i, [_p, _p, _p, _p, _p, _p, _i, _d, _i, _i64, _i64, _p, _i64, _p]),
    "nft_los_forward_ex": (_i, [_p, _p, _p, _i64, _p, _p, _p, _i, _d, _i, _i64, _i64, _p, _i64, _p]),
    "nft_los_adjoint_ex": (_i, [_p, _p, _p, _p, _i64, _p, _i, _d, _i, _i64, _i64, _p]),
    "nft_cg_dd_blocks": (_i, [_i64]),
    "nft_cg_direction_dd_batched": (_i, [_p, _p, _i64, _i64, _i, _i, _p, _d, _p, _i64, _p]),
    "nft_fold_partials": (_i, [_p, _i, _i, _p, _i64, _p]),
    "nft_cg_lazy_flush": (_i, [_p, _p, _p, _i64, _p, _i64, _i, _i64, _i64, _i, _i, _p]),
    "nft_prof_begin": (_i, [_i]),
    "nft_prof_end": (_i, [_p, _p, _i, ctypes.POINTER(_i)]),
    "nft_prof_label": (ctypes.c_char_p, [_i]),
    "nft_amp_workspace": (_sz, [_i64]),
    "nft_amp_jvp": (_i, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p]),
    "nft_amp_vjp": (_i, [_p, _p, _p, _p, _p]),
    "nft_amp_jvp_batched": (_i, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i, _i64, _i64, _i64, _p]),
    "nft_amp_vjp_batched": (_i, [_p, _p, _p, _p, _p, _i, _i64, _i64, _p]),
    "nft_hartley_cg_blocks": (_i, [_i, _p, _i, _p, _i]),
    "nft_hartley_dir_blocks": (_i, [_i, _p]),
    "nft_cg_update_seg_batched": (_i, [_p, _p, _p, _p, _p, _i64, _i64, _i, _i, _d, _p, _p, _i, _i, _p]),
    "nft_cg_update_seg2_batched": (_i, [_p, _p, _p, _p, _i64, _i, _i64, _i64, _i, _i64, _i, _i, _d, _p, _p, _i, _p]),
    "nft_cg_direction_dd2_batched": (_i, [_p, _p, _i64, _i64, _i64, _i64, _i, _i, _p, _d, _p, _i64, _i64, _p]),
    "nft_cg_finalize_batched": (_i, [_p, _i, _i, _p, _p]),
    "nft_amp2_enabled": (_i, []),
    "nft_amp2_set_enabled": (None, [_i]),
    "nft_amp2_tiles": (_i, [_i64, _i, _i]),
    "nft_amp2_tab_size": (_i64, [_i64]),
    "nft_amp2_prepare": (_i, [_p, _p, _i, _p, _p]),
    # two-phase amplitude kernels: one device-global counter set, so eager
    # calls from several streams / threads are serialised by the library, but
    # HIP graphs holding these kernels must never be replayed concurrently
    # with each other or with eager calls on another stream (nifty_amd.h)
    "nft_amp2_jvp": (_i, [_p, _p, _i, _p, _p, _i64, _p, _i64, _i64, _p, _i, _p, _p, _i64, _d, _i, _p, _p]),
    "nft_amp2_vjp": (_i, [_p, _p, _i, _p, _i64, _p, _p, _p, _i64, _d, _p, _i, _p, _p, _i64, _p, _i64, _i64, _i, _i,
                          _p, _p]),
    "nft_amp_forward_buf": (_i64, [_i64]),
    "nft_amp_forward_batched": (_i, [_p, _p, _p, _p, _p, _p, _p, _i64, _i, _p, _i64, _p, _i64, _p, _p, _p]),
}


class HartleyFuse(ctypes.Structure):
    """nft_hartley_fuse (include/nifty_amd.h)."""
    _fields_ = [(n, _p) for n in ("pro_a", "pro_x", "pro_b", "pro_c", "pro_index", "epi_a", "epi_d", "epi_b",
                                  "epi_out2")] + [("epi_shift", _d)] + \
               [(n, _i64) for n in ("batch_period", "x_bstride", "c_bstride", "out_bstride", "d_bstride",
                                    "out2_bstride", "c_estride", "a_bstride", "b_bstride", "ea_bstride",
                                    "eb_bstride", "pro_folded")] + \
               [(n, _p) for n in ("cg_x", "cg_r", "cg_d", "cg_sc", "cg_part")] + \
               [("cg_stride", _i64), ("cg_shift", _d), ("cg_nbtot", ctypes.c_int32), ("cg_blk0", ctypes.c_int32)] + \
               [(n, _p) for n in ("dir_r", "dir_sc", "dir_part")] + \
               [("dir_pstride", _i64), ("dir_shift", _d), ("dir_blk0", ctypes.c_int32), ("dir_pad", ctypes.c_int32)] + \
               [("epi_out2_pairs", _i64)] + \
               [("quad_part", _p), ("quad_pstride", _i64), ("quad_blk0", ctypes.c_int32), ("quad_pad", ctypes.c_int32)] + \
               [("lazy_ring", _p), ("lazy_sstride", _i64), ("lazy_alpha", _p), ("lazy_nslot", _i64)] + \
               [("fold_part", _p), ("fold_nb", _i64), ("fold_out", _p), ("fold_ostride", _i64), ("fold_nrhs", _i64)]


class LosPlan(ctypes.Structure):
    """nft_los_plan (include/nifty_amd.h)."""
    _fields_ = [("H", _i64), ("W", _i64), ("bh", _i), ("bw", _i), ("nby", _i), ("nbx", _i),
                ("nbox", _i64), ("nlos", _i64), ("nitems", _i64), ("nseg", _i64)] + \
               [(n, _p) for n in ("item_box", "item_seg", "item_ent", "seg_ent", "seg_slot", "ent_loc", "ent_wf",
                                  "los_ptr", "box_ent", "pix_off", "box_lptr", "box_lines", "ent_lidx")] + \
               [("lidx8", _i), ("ent_wa", _p), ("box_item", _p), ("box_ent_adj", _p)]


class AmpConst(ctypes.Structure):
    """nft_amp_const (include/nifty_amd.h)."""
    _fields_ = [(n, _p) for n in ("c0", "sf", "p0", "p1", "p2", "lv", "vslope", "sc", "Qf", "Qa",
                                  "mspec", "An")] + \
               [(n, _d) for n in ("fl", "S", "ls_f", "sig_s", "zm", "ls_o", "total_volume")] + \
               [("B", _i64), ("has_flex", _i), ("has_asp", _i), ("has_zm", _i)]


class AmpModel(ctypes.Structure):
    """nft_amp_model (include/nifty_amd.h)."""
    _fields_ = [(n, _p) for n in ("vslope", "sc", "mult", "lv", "sqrt_lv", "shift0")] + \
               [(n, _d) for n in ("lm_f", "ls_f", "mu_s", "sig_s", "lm_x", "ls_x", "lm_a", "ls_a", "lm_o", "ls_o",
                                  "total_volume")] + \
               [("B", _i64), ("has_flex", _i), ("has_asp", _i), ("has_zm", _i)]


class AmpOut(ctypes.Structure):
    """nft_amp_out (include/nifty_amd.h)."""
    _fields_ = [(n, _p) for n in ("fl", "sl", "flex", "asp", "zm", "spec",
                                  "dfl", "dsl", "dflex", "dasp", "dzm", "dspec")] + [("shift", _d)]

CG_GAMMA, CG_GPREV, CG_CURV, CG_ALPHA, CG_XR, CG_XB, CG_FLAG, CG_DD, CG_DONE, CG_ITER, CG_AUTO, CG_LAZY = range(12)
CG_NSCALARS = 16
AMP2_FALLBACK = 1  # NFT_AMP2_FALLBACK

_lib = None
_load_error = None


class NativeError(RuntimeError):
    pass


def load(required=True):
    """Load the shared library once.  Raises NativeError if it is missing."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if _load_error is None:
        try:
            lib = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
        except OSError as e:
            _load_error = f"cannot load {LIB_PATH}: {e} (run __graft_entry__.build())"
        except AttributeError as e:
            _load_error = f"{LIB_PATH} lacks a symbol: {e} (stale build?)"
    if _lib is None and required:
        raise NativeError(_load_error)
    return _lib


def _check(status):
    if status != 0:
        msg = _lib.nft_last_error().decode(errors="replace")
        raise NativeError(f"nifty_amd native call failed ({status}): {msg}")


def dtype_code(t):
    if t in (torch.float64, torch.complex128):
        return 0
    if t in (torch.float32, torch.complex64):
        return 1
    raise TypeError(f"unsupported dtype {t}")


def require_device(*tensors):
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise NativeError("nifty_amd hot-path ops run on the GPU only "
                              f"(got a {t.device} tensor); no CPU fallback exists")
        if not t.is_contiguous():
            raise NativeError("nifty_amd hot-path ops need contiguous tensors")


_stream_ok = False


def stream_ptr():
    """hipStream_t of torch's current stream on the current device (raw query:
    torch.cuda.current_stream() re-runs lazy-init checks on every call)."""
    global _stream_ok
    if not _stream_ok:
        torch.cuda.init()
        _stream_ok = True
    return ctypes.c_void_p(torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice()))


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _shape_args(shape, axes):
    nd = len(shape)
    sh = (ctypes.c_int64 * max(nd, 1))(*shape)
    ax = (ctypes.c_int * max(len(axes), 1))(*axes)
    return nd, sh, len(axes), ax


_ws_cache = {}


def workspace(nbytes, device, tag="ws"):
    """Grow-only per-(device, tag) scratch buffer owned by the torch allocator."""
    key = (str(device), tag)
    buf = _ws_cache.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)
        _ws_cache[key] = buf
    return buf


def hartley(x, axes, convention=0, scale=1.0, out=None):
    """out = scale * genuine Hartley transform of real x over `axes`."""
    lib = load()
    require_device(x)
    if x.is_complex():
        raise TypeError("hartley expects a real tensor")
    if out is None:
        out = torch.empty_like(x)
    nd, sh, na, ax = _shape_args(tuple(x.shape), tuple(axes))
    dt = dtype_code(x.dtype)
    nbytes = ctypes.c_size_t(0)
    _check(lib.nft_hartley_workspace(nd, sh, na, ax, dt, ctypes.byref(nbytes)))
    ws = workspace(nbytes.value, x.device, "hartley")
    _check(lib.nft_hartley(ptr(x), ptr(out), nd, sh, na, ax, dt, int(convention), float(scale),
                           ptr(ws), ctypes.c_size_t(ws.numel()), stream_ptr()))
    return out


def fft_c2c(z, axes, forward=True, scale=1.0, out=None):
    lib = load()
    require_device(z)
    if not z.is_complex():
        raise TypeError("fft_c2c expects a complex tensor")
    if out is None:
        out = torch.empty_like(z)
    nd, sh, na, ax = _shape_args(tuple(z.shape), tuple(axes))
    _check(lib.nft_fft_c2c(ptr(z), ptr(out), nd, sh, na, ax, dtype_code(z.dtype), int(bool(forward)),
                           float(scale), stream_ptr()))
    return out


def dot(a, b, out=None):
    """Device fp64 scalar sum(a*b) (real tensors, deterministic)."""
    lib = load()
    require_device(a, b)
    if a.numel() != b.numel():
        raise ValueError("dot: size mismatch")
    if out is None:
        out = torch.empty((), dtype=torch.float64, device=a.device)
    n = a.numel()
    ws = workspace(lib.nft_reduce_workspace(n), a.device, "reduce")
    _check(lib.nft_dot(ptr(a), ptr(b), n, dtype_code(a.dtype), ptr(out), ptr(ws), stream_ptr()))
    return out


def sigmoid_pair(x, v, d):
    """v = 0.5 + 0.5 tanh(x), d = 0.5 (1 - tanh(x)^2) in one pass
    (nft_sigmoid_pair: bitwise the torch elementwise passes of
    pointwise._sigmoid); contiguous device tensors of one dtype."""
    require_device(x, v, d)
    if not (x.is_contiguous() and v.is_contiguous() and d.is_contiguous()
            and x.dtype == v.dtype == d.dtype and x.numel() == v.numel() == d.numel()):
        raise NativeError("sigmoid_pair: contiguous x, v, d of one dtype and size required")
    _check(load().nft_sigmoid_pair(ptr(x), ptr(v), ptr(d), x.numel(), dtype_code(x.dtype), stream_ptr()))
    return v, d


def bin_gather(src, pindex, out, pre, npix, nbins, post):
    lib = load()
    require_device(src, pindex, out)
    _check(lib.nft_bin_gather(ptr(src), ptr(pindex), ptr(out), pre, npix, nbins, post,
                              dtype_code(src.dtype), stream_ptr()))
    return out


def bin_scatter(src, perm, offsets, out, pre, npix, nbins, post, order=None):
    """order: BinIndex.gather_order = (gpix, gslot, chunk_bins) (pixel-ordered
    chunk gathers, precomputed chunk bounds; gpix/gslot may be None; same
    result bitwise) or None."""
    lib = load()
    require_device(src, perm, offsets, out)
    if order is not None:
        gpix, gslot, cb = order
        _check(lib.nft_bin_scatter_ordered(ptr(src), ptr(perm), ptr(offsets), ptr(gpix), ptr(gslot), ptr(cb),
                                           ptr(out), pre, npix, nbins, post, dtype_code(src.dtype), stream_ptr()))
        return out
    _check(lib.nft_bin_scatter(ptr(src), ptr(perm), ptr(offsets), ptr(out), pre, npix, nbins, post,
                               dtype_code(src.dtype), stream_ptr()))
    return out


def bin_fold(src, out, pre, shape):
    """Mirror fold of (pre, *shape) onto (pre, *[n//2+1]) (nft_bin_fold)."""
    lib = load()
    require_device(src, out)
    sh = (ctypes.c_int64 * len(shape))(*shape)
    _check(lib.nft_bin_fold(ptr(src), ptr(out), pre, len(shape), sh, dtype_code(src.dtype), stream_ptr()))
    return out


def bin_fold_half(src, out, pre, shape):
    """Mirror fold onto (pre, *[n//2+1]) from point-mirror pair sums on the
    half grid (pre, *shape[:-1], shape[-1]//2+1) (nft_bin_fold_half)."""
    lib = load()
    require_device(src, out)
    sh = (ctypes.c_int64 * len(shape))(*shape)
    _check(lib.nft_bin_fold_half(ptr(src), ptr(out), pre, len(shape), sh, dtype_code(src.dtype), stream_ptr()))
    return out


def bin_fold_half_sorted(src, out, cpos, pre, shape):
    """the half-grid fold in bin-sorted order, items of a cell adjacent:
    out[cpos[cell] * pre + p] (nft_bin_fold_half_sorted)"""
    lib = load()
    require_device(src, out) if cpos is None else require_device(src, out, cpos)
    sh = (ctypes.c_int64 * len(shape))(*shape)
    _check(lib.nft_bin_fold_half_sorted(ptr(src), ptr(out), ptr(cpos), pre, len(shape), sh, dtype_code(src.dtype),
                                        stream_ptr()))
    return out


def bin_scatter_il(src, perm, offsets, out, pre, npix, nbins, chunk_bins=None):
    """out[p, b] = sum over bin b's cells of src[cell * pre + p] (the
    interleaved fold of bin_fold_half_sorted with cpos None;
    nft_bin_scatter_il; chunk_bins: the plan's chunk -> first bin table for
    nft_bin_scatter_il_chunk(pre) positions per chunk, or None)"""
    lib = load()
    require_device(src, perm, offsets, out)
    _check(lib.nft_bin_scatter_il(ptr(src), ptr(perm), ptr(offsets), ptr(chunk_bins), ptr(out), pre, npix, nbins,
                                  dtype_code(src.dtype), stream_ptr()))
    return out


def bin_scatter_folded(src, perm, offsets, out, pre, npix, nbins, chunk_bins=None):
    """out[p, b] = sum over bin b's cells of src[p, cell] (a planar mirror
    fold) in nft_bin_scatter_il's arithmetic: bitwise the interleaved sums
    for any item count (nft_bin_scatter_folded; chunk_bins: the
    nft_bin_chunk() table or None)"""
    lib = load()
    require_device(src, perm, offsets, out)
    _check(lib.nft_bin_scatter_folded(ptr(src), ptr(perm), ptr(offsets), ptr(chunk_bins), ptr(out), pre, npix,
                                      nbins, dtype_code(src.dtype), stream_ptr()))
    return out


def spmv_csr(indptr, indices, weights, x, y, scale=1.0):
    lib = load()
    require_device(indptr, indices, weights, x, y)
    nrows = indptr.numel() - 1
    _check(lib.nft_spmv_csr(ptr(indptr), ptr(indices), ptr(weights), ptr(x), ptr(y), nrows,
                            dtype_code(x.dtype), float(scale), indices.numel(), stream_ptr()))
    return y


def csr_rowblocks(indptr):
    """CSR-stream row blocks for a host int64 indptr array (numpy)."""
    import numpy as np
    lib = load()
    indptr = np.ascontiguousarray(indptr, dtype=np.int64)
    nrows = indptr.size - 1
    cap = nrows + 2
    blocks = np.empty(cap, dtype=np.int32)
    nb = ctypes.c_int64(0)
    _check(lib.nft_csr_rowblocks(indptr.ctypes.data, nrows, blocks.ctypes.data, cap, ctypes.byref(nb)))
    return blocks[:nb.value + 1].copy()


def spmv_scaled(indptr, indices, weights, rowblocks, x, y, colscale=None, rowscale=None, scale=1.0):
    lib = load()
    require_device(indptr, indices, weights, rowblocks, x, y, colscale, rowscale)
    nrows = indptr.numel() - 1
    nb = rowblocks.numel() - 1 if rowblocks is not None else 0
    _check(lib.nft_spmv_scaled(ptr(indptr), ptr(indices), ptr(weights), ptr(rowblocks), nb, ptr(x),
                               ptr(colscale), ptr(rowscale), ptr(y), nrows, dtype_code(x.dtype),
                               float(scale), stream_ptr()))
    return y


def hartley_cg_blocks(shape, axes, dtype):
    """partial blocks per item of the CG-carrying epilogue for a batched
    transform of `shape` (leading batch axis) over `axes`, 0 if unsupported"""
    nd, sh, na, ax = _shape_args(tuple(shape), tuple(axes))
    return int(load().nft_hartley_cg_blocks(nd, sh, na, ax, dtype_code(dtype)))


def hartley_dir_blocks(grid):
    """blocks (d.d partials per item) of the folded prologue over `grid`"""
    sh = (ctypes.c_int64 * len(grid))(*[int(n) for n in grid])
    return int(load().nft_hartley_dir_blocks(len(grid), sh))


def _set_lazy(f, lz):
    """nft_hartley_fuse.lazy_*: lz = dict(ring=base of slot 1 (a tensor view
    laid out like the direction), sstride=elements between slots,
    alpha=(k, nslot) fp64 rows, nslot=)"""
    ring, al = lz["ring"], lz["alpha"]
    if not (ring.is_cuda and al.is_cuda and al.dtype == torch.float64):
        raise NativeError("lazy iterate: device ring and fp64 device alphas")
    f.lazy_ring = ring.data_ptr()
    f.lazy_sstride = int(lz["sstride"])
    f.lazy_alpha = al.data_ptr()
    f.lazy_nslot = int(lz["nslot"])


def cg_lazy_flush(x, d, ring, sstride, alpha, nslot, nsteps, n, vstride, k):
    """nft_cg_lazy_flush on the grid segment views x / d / ring (rows vstride
    apart, ring slot 1 at `ring`)"""
    _check(load().nft_cg_lazy_flush(ptr(x), ptr(d), ptr(ring), int(sstride), ptr(alpha), int(nslot), int(nsteps),
                                    int(n), int(vstride), int(k), dtype_code(x.dtype), stream_ptr()))


def hartley_fused(out, axes, scale=1.0, x=None, pro=None, epi=None, convention=0, shape=None, batch=None, cg=None,
                  quad=None, fold=None):
    """out = epilogue(scale * Hartley(prologue)) with
    pro = dict(a=, x=, b=, c=, index=) (or fold=True and c per fundamental
    cell instead of index, nft_hartley_fuse.pro_folded) and
    epi = dict(a=, d=, shift=, b=, out2=)
    (nft_hartley_fused); `x` is the plain input when no prologue is given.
    Batched transforms: `shape` = (k, *grid), axes over the grid, and
    batch = dict(period=, x=, c=, out=, d=, out2=) with the per-item strides
    of the operands (elements); `out` may then be a strided base pointer.
    fold: (part, nb, nrhs, out_address, out_stride) of an nft_fold_partials
    call carried by the transform's R2C row pass (nft_hartley_fuse.fold_*)."""
    lib = load()
    f = HartleyFuse()
    if batch:
        f.batch_period = int(batch["period"])
        for k, fld in (("x", "x_bstride"), ("c", "c_bstride"), ("out", "out_bstride"), ("d", "d_bstride"),
                       ("out2", "out2_bstride"), ("c_elem", "c_estride"), ("a", "a_bstride"),
                       ("b", "b_bstride"), ("ea", "ea_bstride"), ("eb", "eb_bstride")):
            setattr(f, fld, int(batch.get(k, 0)))
    tens = [out, x]
    if pro:
        for k, fld in (("a", "pro_a"), ("x", "pro_x"), ("b", "pro_b"), ("c", "pro_c"), ("index", "pro_index")):
            v = pro.get(k)
            tens.append(v)
            setattr(f, fld, v.data_ptr() if v is not None else None)
        f.pro_folded = 1 if pro.get("fold") else 0
        dr = pro.get("dir")
        if dr:
            # the CG direction carried by the folded prologue (nft_hartley_fuse.dir_*)
            for k, fld in (("r", "dir_r"), ("sc", "dir_sc"), ("part", "dir_part")):
                v = dr[k]
                if not v.is_cuda:
                    raise NativeError("nifty_amd hot-path ops run on the GPU only; no CPU fallback exists")
                setattr(f, fld, v.data_ptr())
            f.dir_pstride = int(dr["pstride"])
            f.dir_shift = float(dr["shift"])
            f.dir_blk0 = int(dr["blk0"])
            if dr.get("lazy"):
                _set_lazy(f, dr["lazy"])
    if epi:
        for k, fld in (("a", "epi_a"), ("d", "epi_d"), ("b", "epi_b"), ("out2", "epi_out2")):
            v = epi.get(k)
            tens.append(v)
            setattr(f, fld, v.data_ptr() if v is not None else None)
        f.epi_shift = float(epi.get("shift", 0.0))
        f.epi_out2_pairs = 1 if epi.get("pairs") else 0
    if cg:
        # the CG update carried by the epilogue (nft_hartley_fuse.cg_*):
        # x / r / d are strided base pointers of the grid segment
        for k, fld in (("x", "cg_x"), ("r", "cg_r"), ("d", "cg_d"), ("sc", "cg_sc"), ("part", "cg_part")):
            v = cg[k]
            if not v.is_cuda:
                raise NativeError("nifty_amd hot-path ops run on the GPU only; no CPU fallback exists")
            setattr(f, fld, v.data_ptr())
        f.cg_stride = int(cg["stride"])
        f.cg_shift = float(cg["shift"])
        f.cg_nbtot = int(cg["nbtot"])
        f.cg_blk0 = int(cg["blk0"])
        if cg.get("lazy"):
            _set_lazy(f, cg["lazy"])
    if quad:
        # per-tile partials of h * (epi_a * h) (nft_hartley_fuse.quad_*)
        qp = quad["part"]
        if not (qp.is_cuda and qp.dtype == torch.float64 and qp.stride(-1) == 1):
            raise NativeError("quad part: fp64 device rows with unit element stride")
        f.quad_part = qp.data_ptr()
        f.quad_pstride = int(quad["pstride"])
        f.quad_blk0 = int(quad.get("blk0", 0))
    if fold is not None:
        part, nb, nrhs, faddr, fstride = fold
        if not (part.is_cuda and part.dtype == torch.float64):
            raise NativeError("carried fold: fp64 device partials")
        f.fold_part = part.data_ptr()
        f.fold_nb = int(nb)
        f.fold_out = int(faddr)
        f.fold_ostride = int(fstride)
        f.fold_nrhs = int(nrhs)
    if batch:
        for t in tens:
            if t is not None and not t.is_cuda:
                raise NativeError("nifty_amd hot-path ops run on the GPU only; no CPU fallback exists")
    else:
        require_device(*tens)
    for t in tens:
        if t is not None and t.dtype != out.dtype and t.dtype != torch.int32:
            raise TypeError("hartley_fused: operand dtype mismatch")
    nd, sh, na, ax = _shape_args(tuple(out.shape) if shape is None else tuple(shape), tuple(axes))
    dt = dtype_code(out.dtype)
    nbytes = ctypes.c_size_t(0)
    _check(lib.nft_hartley_fused_workspace(nd, sh, na, ax, dt, ctypes.byref(nbytes)))
    ws = workspace(nbytes.value, out.device, "hartley")
    _check(lib.nft_hartley_fused(ctypes.byref(f), ptr(x), ptr(out), nd, sh, na, ax, dt, int(convention),
                                 float(scale), ptr(ws), ctypes.c_size_t(ws.numel()), stream_ptr()))
    return out


def los_forward(plan, x, y, colscale=None, rowscale=None, scale=1.0):
    """y = scale * rowscale * R (colscale * x) on a box plan (LosPlan)."""
    lib = load()
    require_device(x, y, colscale, rowscale)
    ws = workspace(lib.nft_los_workspace(ctypes.byref(plan)), x.device, "los")
    _check(lib.nft_los_forward(ctypes.byref(plan), ptr(x), ptr(colscale), ptr(rowscale), ptr(y), ptr(ws),
                               dtype_code(x.dtype), float(scale), stream_ptr()))
    return y


def los_adjoint(plan, y, out, colscale=None, rowscale=None, scale=1.0):
    """out = scale * rowscale * R^T (colscale * y)."""
    lib = load()
    require_device(y, out, colscale, rowscale)
    _check(lib.nft_los_adjoint(ctypes.byref(plan), ptr(y), ptr(colscale), ptr(rowscale), ptr(out),
                               dtype_code(y.dtype), float(scale), stream_ptr()))
    return out


def los_forward_batched(plan, x, y, colscale=None, rowscale=None, scale=1.0):
    """y[b] = scale * rowscale * R (colscale * x[b]) for b < k (x: (k, ...) contiguous)."""
    lib = load()
    require_device(x, y, colscale, rowscale)
    k = x.shape[0]
    ws = workspace(k * lib.nft_los_workspace(ctypes.byref(plan)), x.device, "los")
    _check(lib.nft_los_forward_batched(ctypes.byref(plan), ptr(x), ptr(colscale), ptr(rowscale), ptr(y), ptr(ws),
                                       dtype_code(x.dtype), float(scale), k, x[0].numel(), y[0].numel(),
                                       stream_ptr()))
    return y


def los_forward_quad_batched(plan, x, y, qpart, colscale=None, rowscale=None, scale=1.0):
    """los_forward_batched plus the per-block partials of sum_l t_l y_l
    (qpart: (k, >= nft_los_quad_blocks) fp64 rows, see nifty_amd.h)."""
    lib = load()
    require_device(x, y, colscale, rowscale)
    if not (qpart.is_cuda and qpart.dtype == torch.float64 and qpart.stride(1) == 1 and qpart.shape[0] >= x.shape[0]):
        raise NativeError("qpart: (k, >= nft_los_quad_blocks) fp64 device rows with unit element stride")
    k = x.shape[0]
    ws = workspace(k * lib.nft_los_workspace(ctypes.byref(plan)), x.device, "los")
    _check(lib.nft_los_forward_quad_batched(ctypes.byref(plan), ptr(x), ptr(colscale), ptr(rowscale), ptr(y),
                                            ptr(ws), dtype_code(x.dtype), float(scale), k, x[0].numel(),
                                            y[0].numel(), ptr(qpart), qpart.stride(0), stream_ptr()))
    return y


def los_adjoint_batched(plan, y, out, colscale=None, rowscale=None, scale=1.0, fold=None):
    """out[b] = scale * rowscale * R^T (colscale * y[b]).  fold: (part, nb,
    nrhs, out_address, out_stride) of an nft_fold_partials call carried by the
    same launch (nft_los_adjoint_fold)."""
    lib = load()
    require_device(y, out, colscale, rowscale)
    k = y.shape[0]
    if fold is not None:
        part, nb, nrhs, faddr, fstride = fold
        require_device(part)
        _check(lib.nft_los_adjoint_fold(ctypes.byref(plan), ptr(y), ptr(colscale), ptr(rowscale), ptr(out),
                                        dtype_code(y.dtype), float(scale), k, y[0].numel(), out[0].numel(),
                                        ptr(part), int(nb), int(nrhs), ctypes.c_void_p(faddr), int(fstride),
                                        stream_ptr()))
        return out
    _check(lib.nft_los_adjoint_batched(ctypes.byref(plan), ptr(y), ptr(colscale), ptr(rowscale), ptr(out),
                                       dtype_code(y.dtype), float(scale), k, y[0].numel(), out[0].numel(),
                                       stream_ptr()))
    return out


def _pixel_scale_stride(sc, k, npix):
    """Per-vector pixel-side scale: (k, npix) rows -> stride npix, one shared
    (npix,) / (1, npix) vector -> 0."""
    if sc is None:
        return 0
    if not sc.is_contiguous():
        raise NativeError("pixel scale: contiguous tensor required")
    if sc.numel() == npix:
        return 0
    if sc.numel() == k * npix:
        return npix
    raise NativeError(f"pixel scale: {sc.numel()} elements for {k} vectors of {npix} pixels")


def los_forward_ex(plan, x, y, colscale=None, rowscale=None, scale=1.0, qpart=None):
    """y[b] = scale * rowscale * R (colscale[b] * x[b]): colscale one shared
    pixel vector or one per vector (nft_los_forward_ex); qpart as in
    los_forward_quad_batched or None."""
    lib = load()
    require_device(x, y, colscale, rowscale)
    k = x.shape[0]
    if not (x.is_contiguous() and y.is_contiguous()):
        raise NativeError("los_forward_ex: contiguous x and y required")
    css = _pixel_scale_stride(colscale, k, x[0].numel())
    qs = 0
    if qpart is not None:
        if not (qpart.is_cuda and qpart.dtype == torch.float64 and qpart.stride(1) == 1
                and qpart.shape[0] >= k):
            raise NativeError("qpart: (k, >= nft_los_quad_blocks) fp64 device rows with unit element stride")
        qs = qpart.stride(0)
    ws = workspace(k * lib.nft_los_workspace(ctypes.byref(plan)), x.device, "los")
    _check(lib.nft_los_forward_ex(ctypes.byref(plan), ptr(x), ptr(colscale), css, ptr(rowscale), ptr(y), ptr(ws),
                                  dtype_code(x.dtype), float(scale), k, x[0].numel(), y[0].numel(), ptr(qpart), qs,
                                  stream_ptr()))
    return y


def los_adjoint_ex(plan, y, out, colscale=None, rowscale=None, scale=1.0):
    """out[b] = scale * rowscale[b] * R^T (colscale * y[b]): the pixel-side
    rowscale one shared vector or one per vector (nft_los_adjoint_ex)."""
    lib = load()
    require_device(y, out, colscale, rowscale)
    k = y.shape[0]
    if not (y.is_contiguous() and out.is_contiguous()):
        raise NativeError("los_adjoint_ex: contiguous y and out required")
    rss = _pixel_scale_stride(rowscale, k, out[0].numel())
    _check(lib.nft_los_adjoint_ex(ctypes.byref(plan), ptr(y), ptr(colscale), ptr(rowscale), rss, ptr(out),
                                  dtype_code(y.dtype), float(scale), k, y[0].numel(), out[0].numel(), stream_ptr()))
    return out


def amp_jvp(const, t_fl, t_sl, t_flex, t_asp, t_zm, t_spec, da):
    """da = J_amp t (constants `const`: AmpConst holding device pointers)."""
    lib = load()
    require_device(t_fl, t_sl, t_flex, t_asp, t_zm, t_spec, da)
    ws = workspace(lib.nft_amp_workspace(const.B), da.device, "amp")
    _check(lib.nft_amp_jvp(ctypes.byref(const), ptr(t_fl), ptr(t_sl), ptr(t_flex), ptr(t_asp),
                           ptr(t_zm), ptr(t_spec), ptr(da), ptr(ws), stream_ptr()))
    return da


def amp_vjp(const, g, out):
    """out (AmpOut of device pointers) = shift * d + J_amp^T g."""
    lib = load()
    require_device(g)
    ws = workspace(lib.nft_amp_workspace(const.B), g.device, "amp")
    _check(lib.nft_amp_vjp(ctypes.byref(const), ptr(g), ctypes.byref(out), ptr(ws), stream_ptr()))


class LaunchProfile:
    """``with LaunchProfile() as p: ...`` -> p.records = [(label, ms), ...] for
    every hot-path kernel launched inside (HIP events on the launch stream)."""

    def __init__(self, capacity=4096):
        self.capacity = capacity
        self.records = []

    def __enter__(self):
        _check(load().nft_prof_begin(self.capacity))
        return self

    def __exit__(self, *exc):
        lib = load()
        ms = (ctypes.c_float * self.capacity)()
        n = ctypes.c_int(0)
        _check(lib.nft_prof_end(stream_ptr(), ms, self.capacity, ctypes.byref(n)))
        self.records = [(lib.nft_prof_label(i).decode(), float(ms[i])) for i in range(n.value)]
        return False
