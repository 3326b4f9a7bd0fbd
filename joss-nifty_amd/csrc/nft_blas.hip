// Deterministic reductions and fused conjugate-gradient vector primitives.
//
// Replaces, for the CG hot loop:
//   ducc_dispatch.vdot / Field.s_vdot   src/ducc_dispatch.py:53-58,81-86,
//                                       src/field.py:296-347
//   the vector algebra of ConjugateGradient.__call__
//                                       src/minimization/conjugate_gradient.py:78-126
//   QuadraticEnergy value bookkeeping   src/minimization/quadratic_energy.py:31-39
//
// All sums accumulate in fp64 (also for fp32 storage) with a fixed two-level
// tree: per-workgroup partials (wave64 shuffles + LDS) written to a partials
// buffer, then one workgroup folds the partials in index order.  Results are
// bitwise reproducible run to run (no float atomics).
//
// CG scalars live on the device (so a whole iteration can be captured in a
// hipGraph) in a small double array, see the CG_* indices in nifty_amd.h.
#include "nft_api_internal.hpp"
#include "../../include/nifty_amd.h"

namespace nft {

constexpr int RED_NT = 256;
constexpr int RED_MAXBLOCKS = 1024;

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  return v;
}

// block reduction of NV values per thread; result valid in thread 0
template <int NV>
__device__ __forceinline__ void block_sum(double (&v)[NV], double* sh) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    double s = wave_sum(v[k]);
    if (lane == 0) sh[k * (RED_NT / 64) + wid] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      double s = 0;
      for (int w = 0; w < RED_NT / 64; ++w) s += sh[k * (RED_NT / 64) + w];
      v[k] = s;
    }
  }
}

static int red_blocks(long long n) {
  long long b = (n + (RED_NT * 8) - 1) / (RED_NT * 8);
  if (b < 1) b = 1;
  if (b > RED_MAXBLOCKS) b = RED_MAXBLOCKS;
  return (int)b;
}

// ------------------------------------------------------------------ dot
template <typename T>
__global__ __launch_bounds__(RED_NT) void dot_partial(const T* __restrict__ a, const T* __restrict__ b,
                                                      long long n, long long vs, double* __restrict__ part) {
  __shared__ double sh[RED_NT / 64];
  a += (long long)blockIdx.y * vs;
  b += (long long)blockIdx.y * vs;
  part += (long long)blockIdx.y * gridDim.x;
  double v[1] = {0.0};
  const long long stride = (long long)gridDim.x * RED_NT;
  for (long long i = (long long)blockIdx.x * RED_NT + threadIdx.x; i < n; i += stride)
    v[0] += (double)a[i] * (double)b[i];
  block_sum<1>(v, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = v[0];
}

// partial sums of d.(q + shift*d): the curvature of a CG step for the metric
// shift*1 + M' when only q = M' d was formed (the shift never touches HBM)
template <typename T>
__global__ __launch_bounds__(RED_NT) void curv_partial(const T* __restrict__ d, const T* __restrict__ q,
                                                       long long n, long long vs, T shift,
                                                       double* __restrict__ part) {
  __shared__ double sh[RED_NT / 64];
  d += (long long)blockIdx.y * vs;
  q += (long long)blockIdx.y * vs;
  part += (long long)blockIdx.y * gridDim.x;
  double v[1] = {0.0};
  const long long stride = (long long)gridDim.x * RED_NT;
  for (long long i = (long long)blockIdx.x * RED_NT + threadIdx.x; i < n; i += stride) {
    const T di = d[i];
    const T qi = q[i] + shift * di;
    v[0] += (double)di * (double)qi;
  }
  block_sum<1>(v, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = v[0];
}

// fold `nb` partial vectors of width W (layout part[k*nb + b]) into out[k]
// fold `nb` partial vectors of width W (layout part[k*nb + b]) into out[k];
// one workgroup per RHS (partials advance by W*nb, out by ostride)
template <int W>
__global__ __launch_bounds__(RED_NT) void fold_partials(const double* __restrict__ part, int nb,
                                                        double* __restrict__ out, long long ostride) {
  __shared__ double sh[W * (RED_NT / 64)];
  part += (long long)blockIdx.x * W * nb;
  out += (long long)blockIdx.x * ostride;
  double v[W];
#pragma unroll
  for (int k = 0; k < W; ++k) v[k] = 0.0;
  // the rows interleaved and 8 strides unrolled: the loads issue together,
  // each row's sum keeps its order (bitwise the plain loops)
#pragma unroll 8
  for (int b = threadIdx.x; b < nb; b += RED_NT) {
#pragma unroll
    for (int k = 0; k < W; ++k) v[k] += part[k * nb + b];
  }
  block_sum<W>(v, sh);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < W; ++k) out[k] = v[k];
  }
}

int scale_real_impl(void* x, long long n, int dtype, double scale, hipStream_t s);

// ------------------------------------------------------------------ scale
// Value and derivative of NIFTy's sigmoid (src/pointwise.py: 0.5 + 0.5
// tanh(x) and 0.5 (1 - tanh(x)^2), pointwise.py:31-33 here) in one pass over
// x, every operation rounded as the separate elementwise passes round it (no
// contraction; the same tanh): bitwise those passes
template <typename T>
__global__ void sigmoid_pair_kernel(const T* __restrict__ x, T* __restrict__ v, T* __restrict__ d, long long n) {
#pragma clang fp contract(off)
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const T t = tanh(x[i]);
    const T h = (T)0.5 * t;
    v[i] = (T)0.5 + h;
    const T q = t * t;
    d[i] = (T)0.5 * ((T)1 - q);
  }
}

template <typename T>
__global__ void scale_kernel(T* __restrict__ x, long long n, T s) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) x[i] *= s;
}

int scale_real(void* x, long long n, int dtype, double scale, hipStream_t s) {
  if (n <= 0) return NFT_OK;
  int nb = (int)std::min<long long>((n + 255) / 256, 4096);
  if (dtype == 0) hipLaunchKernelGGL(scale_kernel<double>, dim3(nb), dim3(256), 0, s, (double*)x, n, scale);
  else hipLaunchKernelGGL(scale_kernel<float>, dim3(nb), dim3(256), 0, s, (float*)x, n, (float)scale);
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

// ------------------------------------------------------------------ CG
// Every CG kernel handles a batch of independent right-hand sides: blockIdx.y
// selects the RHS (vectors advance by `vs` elements, scalars by
// NFT_CG_NSCALARS, partials by 3*nb).  Each RHS runs exactly the arithmetic
// and reduction tree of a single solve, so a batched solve is bitwise equal
// to solving the RHS one after another.  sc[NFT_CG_DONE] != 0 freezes a RHS
// (the host sets it once that RHS's controller has stopped).
//
// x -= alpha d ; r -= alpha (q + shift d)  with alpha = sc[GAMMA] / sc[CURV]
// partial dots: r.r, x.r, x.b
// A non-finite or non-positive curvature, or alpha < 0, leaves x and r
// untouched (the host maps the flag to IterationController.ERROR, exactly
// like conjugate_gradient.py:85-95 returns the previous energy).
template <typename T>
__global__ __launch_bounds__(RED_NT) void cg_update_kernel(T* __restrict__ x, T* __restrict__ r,
                                                           const T* __restrict__ d,
                                                           const T* __restrict__ q,
                                                           const T* __restrict__ b, long long n, long long vs,
                                                           T shift, const double* __restrict__ sc,
                                                           double* __restrict__ part, int nbtot, int blk0,
                                                           int nb1 = 0, long long o2 = 0, long long n2 = 0,
                                                           int blk2 = 0) {
  // two ranges in one launch (nb1 > 0): blocks [0, nb1) serve [0, n) with
  // partial slots blk0 + block, the rest serve [o2, o2 + n2) with slots
  // blk2 + (block - nb1) -- per block exactly the work of separate launches
  __shared__ double sh[3 * (RED_NT / 64)];
  int bx = blockIdx.x, gx = gridDim.x;
  long long o = (long long)blockIdx.y * vs;
  if (nb1 > 0) {
    if (bx < nb1) {
      gx = nb1;
    } else {
      bx -= nb1;
      gx -= nb1;
      o += o2;
      n = n2;
      blk0 = blk2;
    }
  }
  sc += blockIdx.y * NFT_CG_NSCALARS;
  part += (long long)blockIdx.y * 3 * nbtot + blk0;
  x += o;
  r += o;
  d += o;
  q += o;
  if (b) b += o;
  const double curv = sc[NFT_CG_CURV], gprev = sc[NFT_CG_GAMMA];
  const double alpha = gprev / curv;
  const bool ok = (curv == curv) && curv != 0.0 && (alpha >= 0.0) && (alpha == alpha) &&
                  sc[NFT_CG_DONE] == 0.0;
  const T al = (T)alpha;
  double v[3] = {0.0, 0.0, 0.0};
  const long long stride = (long long)gx * RED_NT;
  for (long long i = (long long)bx * RED_NT + threadIdx.x; i < n; i += stride) {
    // d and q are read whether or not the step applies, so that their loads
    // need not wait for the scalars that decide it (same arithmetic)
    T xi = x[i], ri = r[i];
    const T di = d[i], qi = q[i];
    if (ok) {
      xi = xi - al * di;
      ri = ri - al * (qi + shift * di);
      x[i] = xi;
      r[i] = ri;
    }
    const double bi = b ? (double)b[i] : 0.0;
    v[0] += (double)ri * (double)ri;
    v[1] += (double)xi * (double)ri;
    v[2] += (double)xi * bi;
  }
  block_sum<3>(v, sh);
  if (threadIdx.x == 0) {
    part[0 * nbtot + bx] = v[0];
    part[1 * nbtot + bx] = v[1];
    part[2 * nbtot + bx] = v[2];
  }
}

// one workgroup per RHS: fold the 3 partial vectors, shift gamma, record alpha/flags
__global__ __launch_bounds__(RED_NT) void cg_finalize_kernel(const double* __restrict__ part, int nb,
                                                             double* __restrict__ sc) {
  __shared__ double sh[3 * (RED_NT / 64)];
  sc += blockIdx.x * NFT_CG_NSCALARS;
  part += (long long)blockIdx.x * 3 * nb;
  double v[3] = {0.0, 0.0, 0.0};
  // rows interleaved, 8 strides unrolled (each row's order unchanged)
#pragma unroll 8
  for (int b = threadIdx.x; b < nb; b += RED_NT) {
#pragma unroll
    for (int k = 0; k < 3; ++k) v[k] += part[k * nb + b];
  }
  block_sum<3>(v, sh);
  if (threadIdx.x == 0 && sc[NFT_CG_DONE] == 0.0) {
    const double curv = sc[NFT_CG_CURV], gprev = sc[NFT_CG_GAMMA];
    const double alpha = gprev / curv;
    const bool ok = (curv == curv) && curv != 0.0 && (alpha >= 0.0) && (alpha == alpha);
    sc[NFT_CG_ALPHA] = alpha;
    sc[NFT_CG_FLAG] = ok ? 0.0 : 1.0;
    sc[NFT_CG_ITER] += 1.0;
    if (ok) {
      sc[NFT_CG_GPREV] = gprev;
      sc[NFT_CG_GAMMA] = v[0];
      sc[NFT_CG_XR] = v[1];
      sc[NFT_CG_XB] = v[2];
    }
    // terminal whatever the controller decides (conjugate_gradient.py:84-118:
    // ERROR on the guard, CONVERGED on gamma == 0, ERROR on gamma < 0 / NaN):
    // freeze now, so steps the host queued behind this one leave it alone
    // (the gamma test only while the host queues several steps: a residual
    // refresh step recomputes gamma after this finalize)
    if (!ok || (sc[NFT_CG_AUTO] != 0.0 && !(v[0] > 0.0))) sc[NFT_CG_DONE] = 2.0;
  }
}

// d = max(0, gamma/gprev) d + r
template <typename T>
__global__ void cg_dir_kernel(T* __restrict__ d, const T* __restrict__ r, long long n, long long vs,
                              const double* __restrict__ sc) {
  sc += blockIdx.y * NFT_CG_NSCALARS;
  if (sc[NFT_CG_DONE] != 0.0) return;
  d += (long long)blockIdx.y * vs;
  r += (long long)blockIdx.y * vs;
  double beta = sc[NFT_CG_GAMMA] / sc[NFT_CG_GPREV];
  if (!(beta > 0.0)) beta = 0.0;
  const T bt = (T)beta;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    d[i] = bt * d[i] + r[i];
}

// d = max(0, gamma/gprev) d + r, and per-block partials of shift * d.d: the
// identity part of the curvature d.(shift d + J^T W J d) when the J side
// comes from the data space (nft_los_forward_quad_batched), so no pass over
// q and d is needed for the curvature (nft_fold_partials sums both)
template <typename T>
__global__ __launch_bounds__(RED_NT) void cg_dir_dd_kernel(T* __restrict__ d, const T* __restrict__ r, long long n,
                                                           long long vs, const double* __restrict__ sc,
                                                           double shift, double* __restrict__ part,
                                                           long long pstride, int nb1 = 0, long long o2 = 0,
                                                           long long n2 = 0, long long poff2 = 0) {
  // two ranges in one launch (nb1 > 0, as cg_update_kernel): the second
  // range's partials start poff2 slots after the first's
  __shared__ double sh[RED_NT / 64];
  int bx = blockIdx.x, gx = gridDim.x;
  long long o = 0;
  sc += blockIdx.y * NFT_CG_NSCALARS;
  part += (long long)blockIdx.y * pstride;
  if (nb1 > 0) {
    if (bx < nb1) {
      gx = nb1;
    } else {
      bx -= nb1;
      gx -= nb1;
      o = o2;
      n = n2;
      part += poff2;
    }
  }
  d += (long long)blockIdx.y * vs + o;
  r += (long long)blockIdx.y * vs + o;
  // the first element's operands in flight before the scalars are read
  const long long i0 = (long long)bx * RED_NT + threadIdx.x;
  T d0 = (T)0, r0 = (T)0;
  if (i0 < n) {
    d0 = d[i0];
    r0 = r[i0];
  }
  if (sc[NFT_CG_DONE] != 0.0) {
    if (threadIdx.x == 0) part[bx] = 0.0;
    return;
  }
  double beta = sc[NFT_CG_GAMMA] / sc[NFT_CG_GPREV];
  if (!(beta > 0.0)) beta = 0.0;
  const T bt = (T)beta;
  double v[1] = {0.0};
  const long long stride = (long long)gx * RED_NT;
  if (i0 < n) {
    const T di = bt * d0 + r0;
    d[i0] = di;
    v[0] += (double)di * (double)di;
  }
#pragma unroll 4
  for (long long i = i0 + stride; i < n; i += stride) {
    const T di = bt * d[i] + r[i];
    d[i] = di;
    v[0] += (double)di * (double)di;
  }
  block_sum<1>(v, sh);
  if (threadIdx.x == 0) part[bx] = shift * v[0];
}

// r = (ax + shift x) - b (exact residual refresh, conjugate_gradient.py:103-105
// via QuadraticEnergy.__init__) and partial dots r.r, x.r, x.b
template <typename T>
__global__ __launch_bounds__(RED_NT) void cg_residual_kernel(T* __restrict__ r, const T* __restrict__ ax,
                                                             const T* __restrict__ x,
                                                             const T* __restrict__ b, long long n, long long vs,
                                                             T shift, const double* __restrict__ sc,
                                                             double* __restrict__ part) {
  __shared__ double sh[3 * (RED_NT / 64)];
  const long long o = (long long)blockIdx.y * vs;
  sc += blockIdx.y * NFT_CG_NSCALARS;
  part += (long long)blockIdx.y * 3 * gridDim.x;
  const bool live = sc[NFT_CG_DONE] == 0.0;
  r += o;
  ax += o;
  x += o;
  if (b) b += o;
  double v[3] = {0.0, 0.0, 0.0};
  const long long stride = (long long)gridDim.x * RED_NT;
  for (long long i = (long long)blockIdx.x * RED_NT + threadIdx.x; i < n; i += stride) {
    const T bi = b ? b[i] : (T)0;
    const T xt = x[i];
    T ri;
    if (live) {
      ri = (ax[i] + shift * xt) - bi;
      r[i] = ri;
    } else {
      ri = r[i];
    }
    const double xi = (double)xt;
    v[0] += (double)ri * (double)ri;
    v[1] += xi * (double)ri;
    v[2] += xi * (double)bi;
  }
  block_sum<3>(v, sh);
  if (threadIdx.x == 0) {
    const int nb = gridDim.x;
    part[0 * nb + blockIdx.x] = v[0];
    part[1 * nb + blockIdx.x] = v[1];
    part[2 * nb + blockIdx.x] = v[2];
  }
}

__global__ void cg_residual_finalize(const double* __restrict__ part, int nb, double* __restrict__ sc) {
  __shared__ double sh[3 * (RED_NT / 64)];
  sc += blockIdx.x * NFT_CG_NSCALARS;
  part += (long long)blockIdx.x * 3 * nb;
  double v[3] = {0.0, 0.0, 0.0};
  // rows interleaved, 8 strides unrolled (each row's order unchanged)
#pragma unroll 8
  for (int b = threadIdx.x; b < nb; b += RED_NT) {
#pragma unroll
    for (int k = 0; k < 3; ++k) v[k] += part[k * nb + b];
  }
  block_sum<3>(v, sh);
  if (threadIdx.x == 0 && sc[NFT_CG_DONE] == 0.0) {
    sc[NFT_CG_GPREV] = sc[NFT_CG_GAMMA];
    sc[NFT_CG_GAMMA] = v[0];
    sc[NFT_CG_XR] = v[1];
    sc[NFT_CG_XB] = v[2];
  }
}

// fixed-order sum of nb partials per RHS with one 1024-thread workgroup per
// RHS (thread-strided sums, then the wave / LDS tree)
__global__ __launch_bounds__(1024) void fold_wide(const double* __restrict__ part, int nb, double* __restrict__ out,
                                                  long long ostride) {
  __shared__ double sh[16];
  part += (long long)blockIdx.x * nb;
  double v = 0.0;
  for (int b = threadIdx.x; b < nb; b += 1024) v += part[b];
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < 16; ++w) t += sh[w];
    out[(long long)blockIdx.x * ostride] = t;
  }
}

// the deferred iterate's flush (nft_cg_lazy_flush): per element the recorded
// steps in order, each the CG epilogue's x - alpha d
template <typename T>
__global__ __launch_bounds__(256) void lazy_flush_kernel(T* __restrict__ x, T* __restrict__ d,
                                                         const T* __restrict__ ring, long long ss,
                                                         const double* __restrict__ alpha, long long nslot, int m,
                                                         long long n, long long vs) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const int b = (int)blockIdx.y;
  if (i >= n) return;
  const long long e = (long long)b * vs + i;
  const double* al = alpha + (long long)b * nslot;
  T xi = x[e];
  T dl = d[e];
  for (int t = 0; t < m; ++t) {
    const double a = al[t];
    const T di = ring[(long long)t * ss + e];
    if (a == a) {
      const T at = (T)a;
      xi = xi - at * di;
    }
    dl = di;
  }
  x[e] = xi;
  d[e] = dl;
}

}  // namespace nft

using namespace nft;

extern "C" {

size_t nft_reduce_workspace(int64_t n) { return (size_t)3 * red_blocks(n) * sizeof(double); }

int nft_dot_batched(const void* a, const void* b, int64_t n, int64_t vstride, int nrhs, int dtype, double* out,
                    int64_t out_stride, void* ws, hipStream_t stream) {
  if (n < 0 || !out || !ws || nrhs < 1) {
    set_last_error("nft_dot: bad arguments");
    return NFT_ERR_ARG;
  }
  int nb = red_blocks(n);
  double* part = (double*)ws;
  const dim3 grid(nb, nrhs);
  prof_mark(stream, "dot_partial");
  if (dtype == 0)
    hipLaunchKernelGGL(dot_partial<double>, grid, dim3(RED_NT), 0, stream, (const double*)a, (const double*)b,
                       (long long)n, (long long)vstride, part);
  else if (dtype == 1)
    hipLaunchKernelGGL(dot_partial<float>, grid, dim3(RED_NT), 0, stream, (const float*)a, (const float*)b,
                       (long long)n, (long long)vstride, part);
  else {
    set_last_error("nft_dot: bad dtype %d", dtype);
    return NFT_ERR_ARG;
  }
  prof_mark(stream, "fold_partials");
  hipLaunchKernelGGL(fold_partials<1>, dim3(nrhs), dim3(RED_NT), 0, stream, part, nb, out, (long long)out_stride);
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

int nft_dot(const void* a, const void* b, int64_t n, int dtype, double* out, void* ws, hipStream_t stream) {
  return nft_dot_batched(a, b, n, 0, 1, dtype, out, 0, ws, stream);
}

int nft_scale(void* x, int64_t n, int dtype, double scale, hipStream_t stream) {
  return scale_real(x, n, dtype, scale, stream);
}

int nft_sigmoid_pair(const void* x, void* v, void* d, int64_t n, int dtype, hipStream_t stream) {
  if (n < 0 || (n > 0 && (!x || !v || !d))) {
    set_last_error("nft_sigmoid_pair: bad arguments");
    return NFT_ERR_ARG;
  }
  if (n == 0) return NFT_OK;
  const unsigned nb = (unsigned)std::min<long long>((n + 255) / 256, 65536);
  if (dtype == 0)
    hipLaunchKernelGGL(sigmoid_pair_kernel<double>, dim3(nb), dim3(256), 0, stream, (const double*)x, (double*)v,
                       (double*)d, (long long)n);
  else if (dtype == 1)
    hipLaunchKernelGGL(sigmoid_pair_kernel<float>, dim3(nb), dim3(256), 0, stream, (const float*)x, (float*)v,
                       (float*)d, (long long)n);
  else {
    set_last_error("nft_sigmoid_pair: bad dtype %d", dtype);
    return NFT_ERR_ARG;
  }
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

int nft_cg_curv_batched(const void* d, const void* q, int64_t n, int64_t vstride, int nrhs, int dtype, double shift,
                        double* sc, void* ws, hipStream_t stream) {
  int nb = red_blocks(n);
  double* part = (double*)ws;
  const dim3 grid(nb, nrhs);
  prof_mark(stream, "curv_partial");
  if (dtype == 0)
    hipLaunchKernelGGL(curv_partial<double>, grid, dim3(RED_NT), 0, stream, (const double*)d, (const double*)q,
                       (long long)n, (long long)vstride, shift, part);
  else if (dtype == 1)
    hipLaunchKernelGGL(curv_partial<float>, grid, dim3(RED_NT), 0, stream, (const float*)d, (const float*)q,
                       (long long)n, (long long)vstride, (float)shift, part);
  else {
    set_last_error("nft_cg_curv: bad dtype %d", dtype);
    return NFT_ERR_ARG;
  }
  prof_mark(stream, "fold_partials");
  hipLaunchKernelGGL(fold_partials<1>, dim3(nrhs), dim3(RED_NT), 0, stream, part, nb, sc + NFT_CG_CURV,
                     (long long)NFT_CG_NSCALARS);
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

int nft_cg_curv(const void* d, const void* q, int64_t n, int dtype, double shift, double* sc, void* ws,
                hipStream_t stream) {
  return nft_cg_curv_batched(d, q, n, 0, 1, dtype, shift, sc, ws, stream);
}

int nft_cg_update_batched(void* x, void* r, const void* d, const void* q, const void* b, int64_t n, int64_t vstride,
                          int nrhs, int dtype, double shift, double* sc, void* ws, hipStream_t stream) {
  int nb = red_blocks(n);
  double* part = (double*)ws;
  const dim3 grid(nb, nrhs);
  prof_mark(stream, "cg_update_kernel");
  if (dtype == 0)
    hipLaunchKernelGGL(cg_update_kernel<double>, grid, dim3(RED_NT), 0, stream, (double*)x, (double*)r,
                       (const double*)d, (const double*)q, (const double*)b, (long long)n, (long long)vstride,
                       shift, sc, part, nb, 0);
  else if (dtype == 1)
    hipLaunchKernelGGL(cg_update_kernel<float>, grid, dim3(RED_NT), 0, stream, (float*)x, (float*)r,
                       (const float*)d, (const float*)q, (const float*)b, (long long)n, (long long)vstride,
                       (float)shift, sc, part, nb, 0);
  else {
    set_last_error("nft_cg_update: bad dtype %d", dtype);
    return NFT_ERR_ARG;
  }
  prof_mark(stream, "cg_finalize_kernel");
  hipLaunchKernelGGL(cg_finalize_kernel, dim3(nrhs), dim3(RED_NT), 0, stream, part, nb, sc);
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

int nft_cg_update_seg_batched(void* x, void* r, const void* d, const void* q, const void* b, int64_t n,
                              int64_t vstride, int nrhs, int dtype, double shift, const double* sc, double* part,
                              int nbtot, int blk0, hipStream_t stream) {
  const int nb = red_blocks(n);
  if (blk0 < 0 || blk0 + nb > nbtot || !part) {
    set_last_error("nft_cg_update_seg: partial blocks [%d, %d) outside [0, %d)", blk0, blk0 + nb, nbtot);
    return NFT_ERR_ARG;
  }
  const dim3 grid(nb, nrhs);
  prof_mark(stream, "cg_update_seg");
  if (dtype == 0)
    hipLaunchKernelGGL(cg_update_kernel<double>, grid, dim3(RED_NT), 0, stream, (double*)x, (double*)r,
                       (const double*)d, (const double*)q, (const double*)b, (long long)n, (long long)vstride,
                       shift, sc, part, nbtot, blk0);
  else if (dtype == 1)
    hipLaunchKernelGGL(cg_update_kernel<float>, grid, dim3(RED_NT), 0, stream, (float*)x, (float*)r,
                       (const float*)d, (const float*)q, (const float*)b, (long long)n, (long long)vstride,
                       (float)shift, sc, part, nbtot, blk0);
  else {
    set_last_error("nft_cg_update_seg: bad dtype %d", dtype);
    return NFT_ERR_ARG;
  }
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

int nft_cg_update_seg2_batched(void* x, void* r, const void* d, const void* q, int64_t n1, int blk1, int64_t o2,
                               int64_t n2, int blk2, int64_t vstride, int nrhs, int dtype, double shift,
                               const double* sc, double* part, int nbtot, hipStream_t stream) {
  const int nb1 = red_blocks(n1), nb2 = red_blocks(n2);
  if (n1 < 1 || n2 < 1 || o2 < n1 || blk1 < 0 || blk2 < 0 || blk1 + nb1 > nbtot || blk2 + nb2 > nbtot || !part ||
      (blk1 < blk2 + nb2 && blk2 < blk1 + nb1)) {
    set_last_error("nft_cg_update_seg2: bad ranges or partial blocks");
    return NFT_ERR_ARG;
  }
  const dim3 grid(nb1 + nb2, nrhs);
  prof_mark(stream, "cg_update_seg2");
  if (dtype == 0)
    hipLaunchKernelGGL(cg_update_kernel<double>, grid, dim3(RED_NT), 0, stream, (double*)x, (double*)r,
                       (const double*)d, (const double*)q, (const double*)nullptr, (long long)n1,
                       (long long)vstride, shift, sc, part, nbtot, blk1, nb1, (long long)o2, (long long)n2, blk2);
  else if (dtype == 1)
    hipLaunchKernelGGL(cg_update_kernel<float>, grid, dim3(RED_NT), 0, stream, (float*)x, (float*)r,
                       (const float*)d, (const float*)q, (const float*)nullptr, (long long)n1, (long long)vstride,
                       (float)shift, sc, part, nbtot, blk1, nb1, (long long)o2, (long long)n2, blk2);
  else {
    set_last_error("nft_cg_update_seg2: bad dtype %d", dtype);
    return NFT_ERR_ARG;
  }
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

int nft_cg_finalize_batched(const double* part, int nbtot, int nrhs, double* sc, hipStream_t stream) {
  prof_mark(stream, "cg_finalize_kernel");
  hipLaunchKernelGGL(cg_finalize_kernel, dim3(nrhs), dim3(RED_NT), 0, stream, part, nbtot, sc);
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

int nft_cg_update(void* x, void* r, const void* d, const void* q, const void* b, int64_t n, int dtype,
                  double shift, double* sc, void* ws, hipStream_t stream) {
  return nft_cg_update_batched(x, r, d, q, b, n, 0, 1, dtype, shift, sc, ws, stream);
}

int nft_cg_direction_batched(void* d, const void* r, int64_t n, int64_t vstride, int nrhs, int dtype,
                             const double* sc, hipStream_t stream) {
  int nb = (int)std::min<long long>((n + 255) / 256, 8192);
  if (nb < 1) nb = 1;
  const dim3 grid(nb, nrhs);
  prof_mark(stream, "cg_dir_kernel");
  if (dtype == 0)
    hipLaunchKernelGGL(cg_dir_kernel<double>, grid, dim3(256), 0, stream, (double*)d, (const double*)r,
                       (long long)n, (long long)vstride, sc);
  else if (dtype == 1)
    hipLaunchKernelGGL(cg_dir_kernel<float>, grid, dim3(256), 0, stream, (float*)d, (const float*)r, (long long)n,
                       (long long)vstride, sc);
  else {
    set_last_error("nft_cg_direction: bad dtype %d", dtype);
    return NFT_ERR_ARG;
  }
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

int nft_cg_dd_blocks(int64_t n) { return red_blocks(n); }

int nft_cg_direction_dd_batched(void* d, const void* r, int64_t n, int64_t vstride, int nrhs, int dtype,
                                const double* sc, double shift, double* part, int64_t pstride, hipStream_t stream) {
  const int nb = red_blocks(n);
  if (!part || pstride < nb || nrhs < 1) {
    set_last_error("nft_cg_direction_dd: partials need pstride >= nft_cg_dd_blocks(n)");
    return NFT_ERR_ARG;
  }
  const dim3 grid(nb, nrhs);
  prof_mark(stream, "cg_dir_dd");
  if (dtype == 0)
    hipLaunchKernelGGL(cg_dir_dd_kernel<double>, grid, dim3(RED_NT), 0, stream, (double*)d, (const double*)r,
                       (long long)n, (long long)vstride, sc, shift, part, (long long)pstride);
  else if (dtype == 1)
    hipLaunchKernelGGL(cg_dir_dd_kernel<float>, grid, dim3(RED_NT), 0, stream, (float*)d, (const float*)r,
                       (long long)n, (long long)vstride, sc, shift, part, (long long)pstride);
  else {
    set_last_error("nft_cg_direction_dd: bad dtype %d", dtype);
    return NFT_ERR_ARG;
  }
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

int nft_cg_direction_dd2_batched(void* d, const void* r, int64_t n1, int64_t o2, int64_t n2, int64_t vstride,
                                 int nrhs, int dtype, const double* sc, double shift, double* part, int64_t poff2,
                                 int64_t pstride, hipStream_t stream) {
  const int nb1 = red_blocks(n1), nb2 = red_blocks(n2);
  if (!part || n1 < 1 || n2 < 1 || o2 < n1 || nrhs < 1 || poff2 < nb1 || pstride < poff2 + nb2) {
    set_last_error("nft_cg_direction_dd2: bad ranges or partial slots");
    return NFT_ERR_ARG;
  }
  const dim3 grid(nb1 + nb2, nrhs);
  prof_mark(stream, "cg_dir_dd2");
  if (dtype == 0)
    hipLaunchKernelGGL(cg_dir_dd_kernel<double>, grid, dim3(RED_NT), 0, stream, (double*)d, (const double*)r,
                       (long long)n1, (long long)vstride, sc, shift, part, (long long)pstride, nb1, (long long)o2,
                       (long long)n2, (long long)poff2);
  else if (dtype == 1)
    hipLaunchKernelGGL(cg_dir_dd_kernel<float>, grid, dim3(RED_NT), 0, stream, (float*)d, (const float*)r,
                       (long long)n1, (long long)vstride, sc, shift, part, (long long)pstride, nb1, (long long)o2,
                       (long long)n2, (long long)poff2);
  else {
    set_last_error("nft_cg_direction_dd2: bad dtype %d", dtype);
    return NFT_ERR_ARG;
  }
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

int nft_cg_lazy_flush(void* x, void* d, const void* ring, int64_t sstride, const double* alpha, int64_t nslot,
                      int nsteps, int64_t n, int64_t vstride, int nrhs, int dtype, hipStream_t stream) {
  if (!x || !d || !ring || !alpha || nsteps < 0 || nsteps > nslot || n < 0 || vstride < n || nrhs < 1 ||
      nrhs > 65535 || sstride < (int64_t)nrhs * vstride || (dtype != 0 && dtype != 1)) {
    set_last_error("nft_cg_lazy_flush: bad arguments");
    return NFT_ERR_ARG;
  }
  if (n == 0 || nsteps == 0) return NFT_OK;
  const dim3 grid((unsigned)((n + 255) / 256), (unsigned)nrhs);
  prof_mark(stream, "cg_lazy_flush");
  if (dtype == 0)
    hipLaunchKernelGGL(lazy_flush_kernel<double>, grid, dim3(256), 0, stream, (double*)x, (double*)d,
                       (const double*)ring, (long long)sstride, alpha, (long long)nslot, nsteps, (long long)n,
                       (long long)vstride);
  else
    hipLaunchKernelGGL(lazy_flush_kernel<float>, grid, dim3(256), 0, stream, (float*)x, (float*)d,
                       (const float*)ring, (long long)sstride, alpha, (long long)nslot, nsteps, (long long)n,
                       (long long)vstride);
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

int nft_fold_partials(const double* part, int nb, int nrhs, double* out, int64_t out_stride, hipStream_t stream) {
  if (!part || !out || nb < 1 || nrhs < 1) {
    set_last_error("nft_fold_partials: bad arguments");
    return NFT_ERR_ARG;
  }
  prof_mark(stream, "fold_partials");
  hipLaunchKernelGGL(fold_wide, dim3(nrhs), dim3(1024), 0, stream, part, nb, out, (long long)out_stride);
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

int nft_cg_direction(void* d, const void* r, int64_t n, int dtype, const double* sc, hipStream_t stream) {
  return nft_cg_direction_batched(d, r, n, 0, 1, dtype, sc, stream);
}

int nft_cg_residual_batched(void* r, const void* ax, const void* x, const void* b, int64_t n, int64_t vstride,
                            int nrhs, int dtype, double shift, double* sc, void* ws, hipStream_t stream) {
  int nb = red_blocks(n);
  double* part = (double*)ws;
  const dim3 grid(nb, nrhs);
  prof_mark(stream, "cg_residual_kernel");
  if (dtype == 0)
    hipLaunchKernelGGL(cg_residual_kernel<double>, grid, dim3(RED_NT), 0, stream, (double*)r, (const double*)ax,
                       (const double*)x, (const double*)b, (long long)n, (long long)vstride, shift, sc, part);
  else if (dtype == 1)
    hipLaunchKernelGGL(cg_residual_kernel<float>, grid, dim3(RED_NT), 0, stream, (float*)r, (const float*)ax,
                       (const float*)x, (const float*)b, (long long)n, (long long)vstride, (float)shift, sc,
                       part);
  else {
    set_last_error("nft_cg_residual: bad dtype %d", dtype);
    return NFT_ERR_ARG;
  }
  prof_mark(stream, "cg_residual_finalize");
  hipLaunchKernelGGL(cg_residual_finalize, dim3(nrhs), dim3(RED_NT), 0, stream, part, nb, sc);
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

int nft_cg_residual(void* r, const void* ax, const void* x, const void* b, int64_t n, int dtype, double shift,
                    double* sc, void* ws, hipStream_t stream) {
  return nft_cg_residual_batched(r, ax, x, b, n, 0, 1, dtype, shift, sc, ws, stream);
}

}  // extern "C"
