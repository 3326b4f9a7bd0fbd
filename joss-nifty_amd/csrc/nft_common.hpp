// Shared device/host helpers for the nifty_amd C-ABI library (gfx950 only).
//
// Complex values are HIP's native double2/float2 so that one complex fp64
// element is a single 16-byte (dwordx4) load/store.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nft {

template <typename T> struct VecOf;
template <> struct VecOf<double> { using type = double2; };
template <> struct VecOf<float> { using type = float2; };
template <typename T> using cplx_t = typename VecOf<T>::type;

template <typename C> __device__ __forceinline__ C cadd(C a, C b) { return {a.x + b.x, a.y + b.y}; }
template <typename C> __device__ __forceinline__ C csub(C a, C b) { return {a.x - b.x, a.y - b.y}; }
template <typename C> __device__ __forceinline__ C cmul(C a, C b) {
  return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x};
}
template <typename C> __device__ __forceinline__ C cconj(C a) { return {a.x, -a.y}; }
// multiply by -i : (x + iy)(-i) = y - ix
template <typename C> __device__ __forceinline__ C cmul_mi(C a) { return {a.y, -a.x}; }
// multiply by +i
template <typename C> __device__ __forceinline__ C cmul_pi(C a) { return {-a.y, a.x}; }
template <typename C, typename T> __device__ __forceinline__ C cscale(C a, T s) { return {a.x * s, a.y * s}; }

void set_last_error(const char* fmt, ...);

// Launch profiler (nft_prof_begin / nft_prof_end): while active, prof_mark
// records a HIP event on the launch stream before every hot-path kernel, so
// consecutive events bracket exactly one kernel.  Inactive: one branch.
extern bool g_prof_on;
void prof_mark_impl(hipStream_t s, const char* label);
inline void prof_mark(hipStream_t s, const char* label) {
  if (g_prof_on) prof_mark_impl(s, label);
}

}  // namespace nft

// error codes of the C ABI (NFT_OK / NFT_ERR_*) live in the public header
#include "../../include/nifty_amd.h"

#define NFT_HIP_CHECK(expr)                                                        \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess) {                                                        \
      nft::set_last_error("%s:%d %s -> %s", __FILE__, __LINE__, #expr,             \
                          hipGetErrorString(_e));                                  \
      return NFT_ERR_HIP;                                                     \
    }                                                                              \
  } while (0)
