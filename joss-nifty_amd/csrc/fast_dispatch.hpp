// Host-side dispatch of the engine-v2 kernels: thread-count choice per
// length and tiling, launch, and the four-step split of long strided axes.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "fast_passes.hpp"
#include "nft_api_internal.hpp"

namespace nft {
namespace fast {

// threads per workgroup for a pass of length N
constexpr int nt_rows(int N) { return N <= 2048 ? 256 : (N == 4096 ? 512 : 1024); }
// strided: aim for >= 16 adjacent columns per tile
// (N = 512 with 512 threads -- 8-line tiles, two workgroups per CU -- measured
// slower at 512^3: C4 iteration 14.2 -> 15.1 ms)
constexpr int nt_strided(int N) { return N <= 128 ? 256 : (N == 256 ? 512 : 1024); }
// fp64 strided passes up to length 128 run their L = nt_strided(N) * VPT / N
// line tile with twice the threads at VP = 4 values each: the same tile, LDS
// and tile count (every tile partial in the same slot), twice the resident
// waves (their ~38 KB tile held them at 4 per SIMD): at 4 x 2048^2 fft_c2c
// 54 -> 50 us, fft_unpack 65 -> 57 us, iteration -7..-9 us.  fp32 tiles take
// half the LDS and already run 8 waves per SIMD: VP = 4 only costs there
// (4096^2: c2c 120 -> 130 us, unpack+quad 196 -> 211 us)
#ifndef NFT_STRIDED_VP4
#define NFT_STRIDED_VP4 1
#endif
template <typename T>
constexpr int vp_strided(int N) { return (NFT_STRIDED_VP4 && sizeof(T) == 8 && N <= 128) ? 4 : VPT; }
template <typename T>
constexpr int nt_strided_launch(int N) { return nt_strided(N) * VPT / vp_strided<T>(N); }
// (the fp64 row passes of length 512..2048 the same way, the persistent R2C at
// 512 threads: fft_r2c 63 -> 68 us at 4 x 2048^2, not kept)

inline bool is_pow2(long long n) { return n > 0 && (n & (n - 1)) == 0; }

inline bool rows_supported(int N) { return is_pow2(N) && N >= 8 && N <= 8192; }
inline bool strided_supported(int N) { return is_pow2(N) && N >= 8 && N <= 512; }
// lengths handled as a four-step pair of strided passes
inline bool fourstep_supported(int N) { return is_pow2(N) && N >= 1024 && N <= 16384; }
// N = N1 * N2 with N1 >= N2: the second (unpack) pass, which carries the
// epilogues, gets the shorter length and hence more adjacent lines per tile
// (2048 = 64 x 32: the CG-carrying unpack 211 -> 201 us per 4-RHS launch,
// iteration -9 us against 32 x 64)
inline void fourstep_split(int N, int& N1, int& N2) {
  int p = 0;
  while ((1 << p) < N) ++p;
  N2 = 1 << (p / 2);
  N1 = N / N2;
}

template <typename T, int N, int NT, int KIND, bool ROWS, int VP = VPT>
static int launch_one(const FastArgs<T>& a, hipStream_t s) {
  constexpr int L = NT * VP / N;
  const size_t lds = pass_lds_bytes<T, N, NT, KIND, ROWS, VP>();
  long long ntiles;
  if (ROWS) {
    long long nl = (KIND == K_R2C || KIND == K_H1D) ? (a.Ireal + 1) / 2 : a.g.O;
    ntiles = (nl + L - 1) / L;
  } else {
    const long long LC = L >> a.los;
    if (LC < 1 || (a.g.O & ((1LL << a.los) - 1)) != 0) {
      set_last_error("strided pass: %d items per tile do not divide O = %lld", 1 << a.los, a.g.O);
      return NFT_ERR_ARG;
    }
    ntiles = (a.g.O >> a.los) * a.g.M * ((a.g.I + LC - 1) / LC);
  }
  if (ntiles <= 0) return NFT_OK;
  if (ntiles > 0x7fffffffLL) {
    set_last_error("too many tiles");
    return NFT_ERR_UNSUPPORTED;
  }
  if (lds > 65536) {
    static bool attr_set = false;
    if (!attr_set) {
      (void)hipFuncSetAttribute((const void*)fast_kernel<T, N, NT, KIND, ROWS, false, 0, VP>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if constexpr (persist_ok<N, NT, KIND, VP>())
        (void)hipFuncSetAttribute((const void*)fast_kernel<T, N, NT, KIND, ROWS, true, 0, VP>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if constexpr (KIND == K_UNPACK && !ROWS) {
        (void)hipFuncSetAttribute((const void*)fast_kernel<T, N, NT, KIND, ROWS, false, 1, VP>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        (void)hipFuncSetAttribute((const void*)fast_kernel<T, N, NT, KIND, ROWS, false, 2, VP>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      }
      attr_set = true;
    }
  }
  FastArgs<T> b = a;
  b.ntiles = ntiles;
  b.bgroup = 0;
  b.bmode = 0;
  if (a.f.o2h && (KIND != K_UNPACK || ROWS) && a.f.epi) {
    set_last_error("out2 pair sums: only the strided unpack pass stores them");
    return NFT_ERR_UNSUPPORTED;
  }
  // the carried curvature fold: extra leading workgroups of the R2C row pass
  const int nfold = KIND == K_R2C ? a.f.fnrhs : 0;
  if (a.f.fnrhs > 0 && (KIND != K_R2C || !a.f.fpart || !a.f.fout || a.f.fnb < 1 || a.f.fnrhs > 65535)) {
    set_last_error("carried curvature fold: only the R2C row pass carries it (partials, output, nb >= 1)");
    return NFT_ERR_UNSUPPORTED;
  }
  if (a.f.cg || a.f.quad) {
    // the CG update / the quadratic-form partials ride only in the strided
    // unpack pass, one item per tile
    if (KIND != K_UNPACK || ROWS || a.los != 0 || a.f.nb < 1 || a.g.O != a.f.nb || ntiles % a.g.O != 0 ||
        (a.f.quad && (a.f.cg || !a.f.ea || a.f.ed || a.f.out2))) {
      set_last_error("CG-carrying / quadratic-form epilogue: needs the strided unpack pass with one item per "
                     "tile (quad: epi_a only)");
      return NFT_ERR_UNSUPPORTED;
    }
    b.f.ctr = ntiles / a.g.O;
  }
  {
    // batch items sharing prologue / epilogue operands: keep one tile's items on one XCD
    const FuseArgs& f = a.f;
    const bool shared = (f.pro && ((f.pa && !f.sa) || (f.pb && !f.sb))) || (f.epi && ((f.ea && !f.sea) || (f.eb && !f.seb)));
    // measured slower at 2048^2 with 4 items for the r2c prologue and the
    // plain epilogue (r2c+pro 200 -> 211 us, unpack+epi 148 -> 177 us), faster
    // for the CG-carrying epilogue, which is bound by its HBM traffic (the
    // contiguous flavour, 231 -> 221 us), and for the quadratic-form one (its
    // shared weight read once per tile group: 1938 -> 1666 us at 512^3, 2
    // items; unchanged at 4096^2): those passes only
    const int mode = (f.cg || f.quad) ? 2 : 0;
    if (mode > 0 && shared && f.P > 0 && f.nb > 1 && ntiles % (8LL * f.nb) == 0) {
      b.bgroup = f.nb;
      b.bmode = mode;
    }
  }
  // persistent grid (plain R2C rows): per_cu workgroups per CU
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
      ncu = v;
    else
      ncu = 256;
  }
  constexpr int per_cu = 8 * 256 / NT;  // 2048 threads per CU
  static const char* const kind_name[4] = {"fft_c2c", "fft_r2c", "fft_h1d", "fft_unpack"};
  static const char* const kind_fused[4] = {"fft_c2c", "fft_r2c+pro", "fft_h1d+fused", "fft_unpack+epi"};
  prof_mark(s, a.f.cg ? "fft_unpack+cg" : a.f.quad ? "fft_unpack+quad" : (a.f.pro || a.f.epi) ? kind_fused[KIND] : kind_name[KIND]);
  bool launched = false;
  if constexpr (persist_ok<N, NT, KIND, VP>()) {
    if (!launched && !a.f.pro) {
      const long long grid = std::min<long long>(ntiles, (long long)ncu * std::max(1, per_cu)) + nfold;
      hipLaunchKernelGGL((fast_kernel<T, N, NT, KIND, ROWS, true, 0, VP>), dim3((unsigned)grid), dim3(NT), lds, s, b);
      launched = true;
    }
  }
  if constexpr (KIND == K_UNPACK && !ROWS) {
    if (!launched && a.f.cg) {
      hipLaunchKernelGGL((fast_kernel<T, N, NT, KIND, ROWS, false, 1, VP>), dim3((unsigned)ntiles), dim3(NT), lds, s, b);
      launched = true;
    }
    if (!launched && a.f.quad) {
      hipLaunchKernelGGL((fast_kernel<T, N, NT, KIND, ROWS, false, 2, VP>), dim3((unsigned)ntiles), dim3(NT), lds, s, b);
      launched = true;
    }
  }
  if (!launched)
    hipLaunchKernelGGL((fast_kernel<T, N, NT, KIND, ROWS, false, 0, VP>), dim3((unsigned)(ntiles + nfold)), dim3(NT),
                       lds, s, b);
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

template <typename T, int KIND, bool ROWS>
static int launch_n(int N, const FastArgs<T>& a, hipStream_t s) {
#define NFT_CASE(n)                                                                \
  case n:                                                                          \
    if constexpr (ROWS)                                                            \
      return launch_one<T, n, nt_rows(n), KIND, ROWS>(a, s);                       \
    else                                                                           \
      return launch_one<T, n, nt_strided_launch<T>(n), KIND, ROWS, vp_strided<T>(n)>(a, s);
  if (ROWS) {
    switch (N) {
      NFT_CASE(8) NFT_CASE(16) NFT_CASE(32) NFT_CASE(64) NFT_CASE(128) NFT_CASE(256) NFT_CASE(512)
      NFT_CASE(1024) NFT_CASE(2048) NFT_CASE(4096) NFT_CASE(8192)
    }
  } else {
    switch (N) {
      NFT_CASE(8) NFT_CASE(16) NFT_CASE(32) NFT_CASE(64) NFT_CASE(128) NFT_CASE(256) NFT_CASE(512)
    }
  }
#undef NFT_CASE
  set_last_error("engine v2: unsupported length %d", N);
  return NFT_ERR_UNSUPPORTED;
}

template <typename T>
static int launch(int kind, bool rows, int N, FastArgs<T>& a, hipStream_t s) {
  const void* tw = nullptr;
  int st = get_twiddles(N, sizeof(T) == 8 ? 0 : 1, &tw);
  if (st != NFT_OK) return st;
  a.tw = tw;
  if (rows) {
    switch (kind) {
      case K_C2C: return launch_n<T, K_C2C, true>(N, a, s);
      case K_R2C: return launch_n<T, K_R2C, true>(N, a, s);
      case K_H1D: return launch_n<T, K_H1D, true>(N, a, s);
      case K_UNPACK: return launch_n<T, K_UNPACK, true>(N, a, s);
    }
  } else {
    switch (kind) {
      case K_C2C: return launch_n<T, K_C2C, false>(N, a, s);
      case K_UNPACK: return launch_n<T, K_UNPACK, false>(N, a, s);
    }
  }
  set_last_error("engine v2: unsupported kind");
  return NFT_ERR_UNSUPPORTED;
}

}  // namespace fast
}  // namespace nft
