// Sparse line-of-sight response: y = scale * W x with W in CSR form, fp32
// weights upcast to the field precision (src/library/los_response.py:197,
// 220-233: scipy COO matvec / rmatvec with float32 data).  The adjoint uses
// the same kernels on the CSC (= transposed CSR) arrays.
//
// Two row regimes:
//  * long rows (R x: one row per line of sight, ~1.5 n nonzeros in 2-D):
//    one wave64 per row, four independent gathers in flight per lane, fixed
//    shuffle-tree reduction;
//  * short rows (R^T y: one row per pixel, a handful of nonzeros): CSR-stream.
//    Host-built row blocks (<= 256 rows, <= 2048 nonzeros each) let a
//    workgroup read its whole nonzero range coalesced, stage the products in
//    LDS and let thread t sum row t's segment in storage order.  A single row
//    longer than the LDS tile gets a block of its own (block-wide reduction).
// Optional per-column and per-row scale vectors fuse the diagonal factors
// that surround the response in a sampling metric (sigmoid', noise weights)
// into the gather and the store.  No atomics: results are deterministic.
#include "nft_api_internal.hpp"

namespace nft {

constexpr int SP_ROWS = 256;   // max rows per stream block (one thread per row)
constexpr int SP_NNZ = 2048;   // max nonzeros per stream block (LDS tile)

template <typename T>
__global__ __launch_bounds__(256) void spmv_vector_kernel(const int64_t* __restrict__ ptr, const int* __restrict__ idx,
                                                          const float* __restrict__ w, const T* __restrict__ x,
                                                          const T* __restrict__ cs, const T* __restrict__ rs,
                                                          T* __restrict__ y, long long nrows, double scale) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= nrows) return;
  const long long lo = ptr[row], hi = ptr[row + 1];
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  long long j = lo + lane;
  for (; j + 192 < hi; j += 256) {
    const int c0 = idx[j], c1 = idx[j + 64], c2 = idx[j + 128], c3 = idx[j + 192];
    const float w0 = w[j], w1 = w[j + 64], w2 = w[j + 128], w3 = w[j + 192];
    double x0 = x[c0], x1 = x[c1], x2 = x[c2], x3 = x[c3];
    if (cs) {
      x0 *= (double)cs[c0];
      x1 *= (double)cs[c1];
      x2 *= (double)cs[c2];
      x3 *= (double)cs[c3];
    }
    a0 += (double)w0 * x0;
    a1 += (double)w1 * x1;
    a2 += (double)w2 * x2;
    a3 += (double)w3 * x3;
  }
  for (; j < hi; j += 64) {
    const int c = idx[j];
    double xv = x[c];
    if (cs) xv *= (double)cs[c];
    a0 += (double)w[j] * xv;
  }
  double acc = (a0 + a1) + (a2 + a3);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
  if (lane == 0) {
    acc *= scale;
    if (rs) acc *= (double)rs[row];
    y[row] = (T)acc;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void spmv_stream_kernel(const int64_t* __restrict__ ptr, const int* __restrict__ idx,
                                                          const float* __restrict__ w, const int* __restrict__ rb,
                                                          const T* __restrict__ x, const T* __restrict__ cs,
                                                          const T* __restrict__ rs, T* __restrict__ y,
                                                          double scale) {
  __shared__ double prod[SP_NNZ];
  __shared__ double red[4];
  const int r0 = rb[blockIdx.x], r1 = rb[blockIdx.x + 1];
  const long long j0 = ptr[r0], j1 = ptr[r1];
  const int tid = threadIdx.x;
  if (j1 - j0 > SP_NNZ) {
    // one long row (r1 == r0 + 1): strided partial sums + fixed tree
    double acc = 0.0;
    for (long long j = j0 + tid; j < j1; j += 256) {
      const int c = idx[j];
      double xv = x[c];
      if (cs) xv *= (double)cs[c];
      acc += (double)w[j] * xv;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
    if ((tid & 63) == 0) red[tid >> 6] = acc;
    __syncthreads();
    if (tid == 0) {
      double v = ((red[0] + red[1]) + (red[2] + red[3])) * scale;
      if (rs) v *= (double)rs[r0];
      y[r0] = (T)v;
    }
    return;
  }
  const int n = (int)(j1 - j0);
  for (int k = tid; k < n; k += 256) {
    const long long j = j0 + k;
    const int c = idx[j];
    double xv = x[c];
    if (cs) xv *= (double)cs[c];
    prod[k] = (double)w[j] * xv;
  }
  __syncthreads();
  const int r = r0 + tid;
  if (r < r1) {
    const int a = (int)(ptr[r] - j0), b = (int)(ptr[r + 1] - j0);
    double acc = 0.0;
    for (int k = a; k < b; ++k) acc += prod[k];
    acc *= scale;
    if (rs) acc *= (double)rs[r];
    y[r] = (T)acc;
  }
}

template <typename T>
__global__ void spmv_thread_kernel(const int64_t* __restrict__ ptr, const int* __restrict__ idx,
                                   const float* __restrict__ w, const T* __restrict__ x, T* __restrict__ y,
                                   long long nrows, double scale) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long row = (long long)blockIdx.x * blockDim.x + threadIdx.x; row < nrows; row += stride) {
    double acc = 0.0;
    for (long long j = ptr[row]; j < ptr[row + 1]; ++j) acc += (double)w[j] * (double)x[idx[j]];
    y[row] = (T)(acc * scale);
  }
}

template <typename T>
static void launch_scaled(const int64_t* indptr, const int* indices, const float* weights, const int* rb,
                          int64_t nblocks, const void* x, const void* cs, const void* rs, void* y, int64_t nrows,
                          double scale, hipStream_t s) {
  if (rb) {
    hipLaunchKernelGGL(spmv_stream_kernel<T>, dim3((unsigned)nblocks), dim3(256), 0, s, indptr, indices, weights,
                       rb, (const T*)x, (const T*)cs, (const T*)rs, (T*)y, scale);
  } else {
    hipLaunchKernelGGL(spmv_vector_kernel<T>, dim3((unsigned)((nrows + 3) / 4)), dim3(256), 0, s, indptr,
                       indices, weights, (const T*)x, (const T*)cs, (const T*)rs, (T*)y, (long long)nrows,
                       scale);
  }
}

}  // namespace nft

using namespace nft;

extern "C" {

int nft_spmv_csr(const int64_t* indptr, const int* indices, const float* weights, const void* x, void* y,
                 int64_t nrows, int dtype, double scale, int64_t nnz, hipStream_t stream) {
  if (nrows <= 0) return NFT_OK;
  if (dtype != 0 && dtype != 1) {
    set_last_error("nft_spmv_csr: bad dtype %d", dtype);
    return NFT_ERR_ARG;
  }
  if (nnz / nrows >= 32) {
    if (dtype == 0)
      launch_scaled<double>(indptr, indices, weights, nullptr, 0, x, nullptr, nullptr, y, nrows, scale, stream);
    else
      launch_scaled<float>(indptr, indices, weights, nullptr, 0, x, nullptr, nullptr, y, nrows, scale, stream);
  } else {
    long long nb = (nrows + 255) / 256;
    if (nb > 65536) nb = 65536;
    if (dtype == 0)
      hipLaunchKernelGGL(spmv_thread_kernel<double>, dim3((unsigned)nb), dim3(256), 0, stream, indptr, indices,
                         weights, (const double*)x, (double*)y, (long long)nrows, scale);
    else
      hipLaunchKernelGGL(spmv_thread_kernel<float>, dim3((unsigned)nb), dim3(256), 0, stream, indptr, indices,
                         weights, (const float*)x, (float*)y, (long long)nrows, scale);
  }
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

int nft_csr_rowblocks(const int64_t* indptr, int64_t nrows, int* blocks, int64_t cap, int64_t* nblocks) {
  int64_t nb = 0, r = 0;
  if (cap < 1) return NFT_ERR_ARG;
  blocks[0] = 0;
  while (r < nrows) {
    int64_t e = r + 1;
    while (e < nrows && e - r < SP_ROWS && indptr[e + 1] - indptr[r] <= SP_NNZ) ++e;
    if (++nb >= cap) {
      set_last_error("nft_csr_rowblocks: capacity %lld too small", (long long)cap);
      return NFT_ERR_ARG;
    }
    blocks[nb] = (int)e;
    r = e;
  }
  *nblocks = nb;
  return NFT_OK;
}

int nft_spmv_scaled(const int64_t* indptr, const int* indices, const float* weights, const int* rowblocks,
                    int64_t nblocks, const void* x, const void* colscale, const void* rowscale, void* y,
                    int64_t nrows, int dtype, double scale, hipStream_t stream) {
  if (nrows <= 0) return NFT_OK;
  if (dtype == 0)
    launch_scaled<double>(indptr, indices, weights, rowblocks, nblocks, x, colscale, rowscale, y, nrows, scale,
                          stream);
  else if (dtype == 1)
    launch_scaled<float>(indptr, indices, weights, rowblocks, nblocks, x, colscale, rowscale, y, nrows, scale,
                         stream);
  else {
    set_last_error("nft_spmv_scaled: bad dtype %d", dtype);
    return NFT_ERR_ARG;
  }
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

}  // extern "C"
