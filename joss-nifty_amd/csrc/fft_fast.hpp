// Compile-time power-of-two FFT passes for gfx950 (engine v2).
//
// For N = 2^p the radix plan is fixed at compile time (one radix-2 or -4
// stage first if p % 3 != 0, then radix-8 stages), every thread owns exactly
// VPT = 8 complex values per stage (L = NT*8/N lines per workgroup), and all
// index arithmetic is shifts and masks.  This keeps the register budget low
// (two or more waves per SIMD for fp64) and removes the runtime radix switch
// of the generic engine (fft_core.hpp), which stays in use for other lengths.
//
// Lines are addressed (o, m, i) -> o*so + m*sm + i*si + x*sn, with separate
// input and output strides.  The m dimension expresses the two sub-passes of
// a four-step decomposition N = N1*N2 of a strided axis:
//   A: lines (n2, c), elements rows n2 + N2*j (j < N1), FFT_N1, then the
//      twiddle W_N^(n2*k1), written back in place;
//   B: lines (k1, c), elements rows N2*k1 + n2 (n2 < N2), FFT_N2, output
//      element k2 lands on row k1 + N1*k2.
// Both sub-passes tile L adjacent columns (i) with L*16 B >= 512 B row
// segments, so a 2048-point fp64 column transform streams at full width
// instead of holding one 32 KB column per workgroup.
#pragma once
#include "fft_core.hpp"

namespace nft {
namespace fast {

constexpr int VPT = 8;

constexpr int ilog2(int n) { return n <= 1 ? 0 : 1 + ilog2(n / 2); }
// radix of the stage that starts at span NS (product of previous radices)
constexpr int radix_at(int N, int NS) {
  return (NS == 1 && ilog2(N) % 3 == 1) ? 2 : ((NS == 1 && ilog2(N) % 3 == 2) ? 4 : 8);
}

struct Lines {
  long long O, M, I;                   // line grid
  long long in_so, in_sm, in_si, in_sn;
  long long out_so, out_sm, out_si, out_sn;
};

// W_N^m from the quarter table twq[r] = W_N^r (r < N/4) held in LDS:
// W_N^(m) = (-i)^q W_N^(m mod N/4), q = m div N/4 -- swaps and negations
// only, so the value is the full table's entry bit for bit (nft_fft.hip:
// twiddle_host builds the table by the same rotations).
template <typename T, int N>
__device__ __forceinline__ cplx_t<T> tw_at(const cplx_t<T>* twq, int m) {
  constexpr int SHQ = ilog2(N) - 2;
  const int q = m >> SHQ;
  cplx_t<T> w = twq[m & ((N >> 2) - 1)];
  if (q & 1) w = cplx_t<T>{w.y, -w.x};
  if (q & 2) w = cplx_t<T>{-w.x, -w.y};
  return w;
}

// LDS position of element x of a line: PS >= 0 inserts one pad slot every
// 2^PS elements, so the stride-R butterfly writes of the first stages (and
// the strided passes' column-interleaved fills) spread over all banks
// (MI355X_MICROARCH.md LDS table: ds_write_b128 serves 8 lanes per cycle,
// 16-byte lanes at a 128-byte stride all hit one bank group).
template <int PS>
__device__ __forceinline__ constexpr int padx(int x) {
  if constexpr (PS >= 0) return x + (x >> PS);
  else return x;
}
template <int N, int PS>
constexpr int padded_len() {
  return PS >= 0 ? N + (N >> PS) : N;
}

// -------------------------------------------------------------- one stage
template <typename T, int N, int NT, int L, int PITCH, int R, int NS, int PS>
__device__ __forceinline__ void stage(cplx_t<T>* lds, const cplx_t<T>* __restrict__ tw, int tid) {
  using C = cplx_t<T>;
  constexpr int NBL = N / R;
  constexpr int NBF = L * NBL;
  constexpr int BPT = (NBF + NT - 1) / NT;
  constexpr int SH_NBL = ilog2(NBL);
  constexpr int TSTRIDE = N / (NS * R);
  C v[BPT][R];
#pragma unroll
  for (int i = 0; i < BPT; ++i) {
    const int b = tid + i * NT;
    if (NBF % NT == 0 || b < NBF) {
      const int line = b >> SH_NBL;
      const int j = b & (NBL - 1);
      const C* src = lds + line * PITCH;
#pragma unroll
      for (int t = 0; t < R; ++t) v[i][t] = src[padx<PS>(j + t * NBL)];
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < BPT; ++i) {
    const int b = tid + i * NT;
    if (NBF % NT == 0 || b < NBF) {
      const int line = b >> SH_NBL;
      const int j = b & (NBL - 1);
      const int k = j & (NS - 1);
      if constexpr (NS > 1) {
        const int step = k * TSTRIDE;
#pragma unroll
        for (int t = 1; t < R; ++t) v[i][t] = cmul(v[i][t], tw_at<T, N>(tw, t * step));
      }
      dftR<T, R>(v[i]);
      C* dst = lds + line * PITCH;
      const int d0 = (j - k) * R + k;
#pragma unroll
      for (int t = 0; t < R; ++t) dst[padx<PS>(d0 + t * NS)] = v[i][t];
    }
  }
  __syncthreads();
}

template <typename T, int N, int NT, int L, int PITCH, int NS, int PS>
__device__ __forceinline__ void stages(cplx_t<T>* lds, const cplx_t<T>* __restrict__ tw, int tid) {
  if constexpr (NS < N) {
    constexpr int R = radix_at(N, NS);
    stage<T, N, NT, L, PITCH, R, NS, PS>(lds, tw, tid);
    stages<T, N, NT, L, PITCH, NS * R, PS>(lds, tw, tid);
  }
}

// forward FFT of the L lines in LDS (caller synced after filling); tw is the
// LDS quarter twiddle table (tw_at)
template <typename T, int N, int NT, int L, int PITCH, int PS = -1>
__device__ __forceinline__ void fft(cplx_t<T>* lds, const cplx_t<T>* __restrict__ tw, int tid) {
  stages<T, N, NT, L, PITCH, 1, PS>(lds, tw, tid);
}

// -------------------------------------------------------------- tiles
// rows tiling: line l of tile -> flat line index tile*L + l over (o) (M == I == 1)
// strided tiling: tile -> (o, m, i0); line l -> i = i0 + l
struct Tile {
  long long o, m, i0;
};

template <int L>
__device__ __forceinline__ Tile strided_tile(const Lines& g, long long t, int los = 0) {
  // los = log2 of the items (o) per tile: lines l -> (o + (l >> (log2 L - los)),
  // i0 + (l mod (L >> los))); los = 0: all L lines in one o
  const long long LC = L >> los;
  const long long tilesI = (g.I + LC - 1) / LC;
  Tile r;
  long long om = t / tilesI;
  r.i0 = (t - om * tilesI) * LC;
  const long long og = om / g.M;
  r.m = om - og * g.M;
  r.o = og << los;
  return r;
}

}  // namespace fast
}  // namespace nft
