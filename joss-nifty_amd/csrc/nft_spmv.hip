// Sparse line-of-sight response: y = scale * W x with W in CSR form, fp32
// weights upcast to the field precision (src/library/los_response.py:197,
// 220-233: scipy COO matvec / rmatvec with float32 data).  The adjoint uses
// the same kernel on the CSC (= transposed CSR) arrays.
//
// Rows with many nonzeros (LOS rows: ~2 n per 2-D line) are reduced by one
// wave64 each (lanes stride the row, fixed-order shuffle tree); rows with few
// nonzeros (pixel columns of the adjoint) by one thread each.  No atomics:
// results are deterministic.
#include "nft_api_internal.hpp"

namespace nft {

template <typename T>
__global__ __launch_bounds__(256) void spmv_wave_kernel(const int64_t* __restrict__ ptr, const int* __restrict__ idx,
                                                        const float* __restrict__ w, const T* __restrict__ x,
                                                        T* __restrict__ y, long long nrows, T scale) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= nrows) return;
  const long long lo = ptr[row], hi = ptr[row + 1];
  double acc = 0.0;
  for (long long j = lo + lane; j < hi; j += 64) acc += (double)w[j] * (double)x[idx[j]];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
  if (lane == 0) y[row] = (T)(acc * (double)scale);
}

template <typename T>
__global__ void spmv_thread_kernel(const int64_t* __restrict__ ptr, const int* __restrict__ idx,
                                   const float* __restrict__ w, const T* __restrict__ x, T* __restrict__ y,
                                   long long nrows, T scale) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long row = (long long)blockIdx.x * blockDim.x + threadIdx.x; row < nrows; row += stride) {
    double acc = 0.0;
    for (long long j = ptr[row]; j < ptr[row + 1]; ++j) acc += (double)w[j] * (double)x[idx[j]];
    y[row] = (T)(acc * (double)scale);
  }
}

}  // namespace nft

using namespace nft;

extern "C" {

int nft_spmv_csr(const int64_t* indptr, const int* indices, const float* weights, const void* x, void* y,
                 int64_t nrows, int dtype, double scale, int64_t nnz, hipStream_t stream) {
  if (nrows <= 0) return NFT_OK;
  const bool wave = nnz / nrows >= 32;
  if (wave) {
    dim3 grid((unsigned)((nrows + 3) / 4)), block(256);
    if (dtype == 0)
      hipLaunchKernelGGL(spmv_wave_kernel<double>, grid, block, 0, stream, indptr, indices, weights,
                         (const double*)x, (double*)y, (long long)nrows, scale);
    else
      hipLaunchKernelGGL(spmv_wave_kernel<float>, grid, block, 0, stream, indptr, indices, weights,
                         (const float*)x, (float*)y, (long long)nrows, (float)scale);
  } else {
    long long nb = (nrows + 255) / 256;
    if (nb > 65536) nb = 65536;
    if (dtype == 0)
      hipLaunchKernelGGL(spmv_thread_kernel<double>, dim3((unsigned)nb), dim3(256), 0, stream, indptr, indices,
                         weights, (const double*)x, (double*)y, (long long)nrows, scale);
    else
      hipLaunchKernelGGL(spmv_thread_kernel<float>, dim3((unsigned)nb), dim3(256), 0, stream, indptr, indices,
                         weights, (const float*)x, (float*)y, (long long)nrows, (float)scale);
  }
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

}  // extern "C"
