// LDS-resident batched line FFT engine for gfx950 (CDNA4, wave64).
//
// A workgroup owns L complex lines of length n staged in LDS (one line every
// `pitch` complex elements).  The transform is a self-sorting (Stockham)
// mixed-radix FFT, radices {8,4,2,3,5,7}, run IN PLACE in LDS: every thread
// first pulls the R inputs of each of its butterflies into registers, the
// workgroup barriers, then every thread writes its R outputs back.  A thread
// owns at most VPT values per stage (static register indexing; no scratch).
// Lengths with a prime factor > 7 fall back to a direct O(n^2) DFT per line
// (only used for the small odd test geometries of the reference suite).
//
// Forward transform convention: X[k] = sum_x x[x] exp(-2 pi i k x / n),
// unnormalised, i.e. what scipy.fft.fftn / ducc0.fft.c2c(forward=True) compute
// and what src/ducc_dispatch.py:38-50 builds the Hartley transform from.
// Twiddles come from a per-length table tw[i] = exp(-2 pi i * i / n) (fp64
// accurate, built on the host, see nft_fft.hip).
#pragma once
#include "nft_common.hpp"

namespace nft {

constexpr int FFT_MAXSTAGES = 24;

struct FftPlanDev {
  int n;
  int nstages;  // 0 => direct DFT
  int radix[FFT_MAXSTAGES];
};

// division helper: power-of-two lengths use shifts
struct FastDiv {
  uint32_t d;
  int shift;  // >= 0 if d is a power of two
  __host__ __device__ FastDiv() : d(1), shift(0) {}
  __host__ __device__ explicit FastDiv(uint32_t dd) : d(dd), shift(-1) {
    if (dd && (dd & (dd - 1)) == 0) {
      int s = 0;
      while ((1u << s) < dd) ++s;
      shift = s;
    }
  }
  __device__ __forceinline__ uint32_t div(uint32_t a) const { return shift >= 0 ? (a >> shift) : a / d; }
  __device__ __forceinline__ uint32_t mod(uint32_t a) const {
    return shift >= 0 ? (a & (d - 1)) : a - (a / d) * d;
  }
};

// ------------------------------------------------------------------ small DFTs
// All forward (W_R = exp(-2 pi i / R)).
template <typename C> __device__ __forceinline__ void dft2(C* v) {
  C a = v[0], b = v[1];
  v[0] = cadd(a, b);
  v[1] = csub(a, b);
}

template <typename C> __device__ __forceinline__ void dft4(C* v) {
  C t0 = cadd(v[0], v[2]), t1 = csub(v[0], v[2]);
  C t2 = cadd(v[1], v[3]), t3 = cmul_mi(csub(v[1], v[3]));
  v[0] = cadd(t0, t2);
  v[2] = csub(t0, t2);
  v[1] = cadd(t1, t3);
  v[3] = csub(t1, t3);
}

template <typename T> __device__ __forceinline__ void dft8(cplx_t<T>* v) {
  using C = cplx_t<T>;
  const T r = (T)0.70710678118654752440084436210484903928483593768847;
  // radix-2 first layer on (j, j+4)
  C a0 = cadd(v[0], v[4]), a4 = csub(v[0], v[4]);
  C a1 = cadd(v[1], v[5]), a5 = csub(v[1], v[5]);
  C a2 = cadd(v[2], v[6]), a6 = csub(v[2], v[6]);
  C a3 = cadd(v[3], v[7]), a7 = csub(v[3], v[7]);
  // twiddles W8^j on the odd half: a5*W8, a6*W8^2=-i, a7*W8^3
  a5 = C{(a5.x + a5.y) * r, (a5.y - a5.x) * r};
  a6 = cmul_mi(a6);
  a7 = C{(a7.y - a7.x) * r, -(a7.x + a7.y) * r};
  C e[4] = {a0, a1, a2, a3};
  C o[4] = {a4, a5, a6, a7};
  dft4(e);
  dft4(o);
  v[0] = e[0]; v[2] = e[1]; v[4] = e[2]; v[6] = e[3];
  v[1] = o[0]; v[3] = o[1]; v[5] = o[2]; v[7] = o[3];
}

template <typename T> __device__ __forceinline__ void dft3(cplx_t<T>* v) {
  using C = cplx_t<T>;
  const T s = (T)0.86602540378443864676372317075293618347140262690519;
  C a = v[0], b = v[1], c = v[2];
  C sum = cadd(b, c), dif = csub(b, c);
  C m = C{a.x - (T)0.5 * sum.x, a.y - (T)0.5 * sum.y};
  C rot = C{dif.y * s, -dif.x * s};  // -i * s * (b - c)
  v[0] = cadd(a, sum);
  v[1] = cadd(m, rot);
  v[2] = csub(m, rot);
}

template <typename T> __device__ __forceinline__ void dft5(cplx_t<T>* v) {
  using C = cplx_t<T>;
  const T c1 = (T)0.30901699437494742410229341718281905886436448684263;   // cos(2pi/5)
  const T c2 = (T)-0.80901699437494742410229341718281905886436448684263;  // cos(4pi/5)
  const T s1 = (T)0.95105651629515357211643933337938214340569863412575;   // sin(2pi/5)
  const T s2 = (T)0.58778525229247312916870595463907276859765243764314;   // sin(4pi/5)
  C a0 = v[0];
  C b1 = cadd(v[1], v[4]), d1 = csub(v[1], v[4]);
  C b2 = cadd(v[2], v[3]), d2 = csub(v[2], v[3]);
  C r1 = C{a0.x + c1 * b1.x + c2 * b2.x, a0.y + c1 * b1.y + c2 * b2.y};
  C r2 = C{a0.x + c2 * b1.x + c1 * b2.x, a0.y + c2 * b1.y + c1 * b2.y};
  // -i*(s1 d1 + s2 d2), -i*(s2 d1 - s1 d2)
  C i1 = C{s1 * d1.x + s2 * d2.x, s1 * d1.y + s2 * d2.y};
  C i2 = C{s2 * d1.x - s1 * d2.x, s2 * d1.y - s1 * d2.y};
  i1 = cmul_mi(i1);
  i2 = cmul_mi(i2);
  v[0] = C{a0.x + b1.x + b2.x, a0.y + b1.y + b2.y};
  v[1] = cadd(r1, i1);
  v[4] = csub(r1, i1);
  v[2] = cadd(r2, i2);
  v[3] = csub(r2, i2);
}

template <typename T> __device__ __forceinline__ void dft7(cplx_t<T>* v) {
  using C = cplx_t<T>;
  const T c1 = (T)0.62348980185873353052500488400423981063227473089640;
  const T c2 = (T)-0.22252093395631440428890256449679475946635556876452;
  const T c3 = (T)-0.90096886790241912623610231950744505116591916213184;
  const T s1 = (T)0.78183148246802980870844452667405775023233451870868;
  const T s2 = (T)0.97492791218182360701813168299393121723278580062000;
  const T s3 = (T)0.43388373911755812047576833284835875460999072778746;
  C a0 = v[0];
  C b1 = cadd(v[1], v[6]), d1 = csub(v[1], v[6]);
  C b2 = cadd(v[2], v[5]), d2 = csub(v[2], v[5]);
  C b3 = cadd(v[3], v[4]), d3 = csub(v[3], v[4]);
  C r1 = C{a0.x + c1 * b1.x + c2 * b2.x + c3 * b3.x, a0.y + c1 * b1.y + c2 * b2.y + c3 * b3.y};
  C r2 = C{a0.x + c2 * b1.x + c3 * b2.x + c1 * b3.x, a0.y + c2 * b1.y + c3 * b2.y + c1 * b3.y};
  C r3 = C{a0.x + c3 * b1.x + c1 * b2.x + c2 * b3.x, a0.y + c3 * b1.y + c1 * b2.y + c2 * b3.y};
  C i1 = C{s1 * d1.x + s2 * d2.x + s3 * d3.x, s1 * d1.y + s2 * d2.y + s3 * d3.y};
  C i2 = C{s2 * d1.x - s3 * d2.x - s1 * d3.x, s2 * d1.y - s3 * d2.y - s1 * d3.y};
  C i3 = C{s3 * d1.x - s1 * d2.x + s2 * d3.x, s3 * d1.y - s1 * d2.y + s2 * d3.y};
  i1 = cmul_mi(i1);
  i2 = cmul_mi(i2);
  i3 = cmul_mi(i3);
  v[0] = C{a0.x + b1.x + b2.x + b3.x, a0.y + b1.y + b2.y + b3.y};
  v[1] = cadd(r1, i1);
  v[6] = csub(r1, i1);
  v[2] = cadd(r2, i2);
  v[5] = csub(r2, i2);
  v[3] = cadd(r3, i3);
  v[4] = csub(r3, i3);
}

template <typename T, int R> __device__ __forceinline__ void dftR(cplx_t<T>* v) {
  if constexpr (R == 2) dft2(v);
  else if constexpr (R == 3) dft3<T>(v);
  else if constexpr (R == 4) dft4(v);
  else if constexpr (R == 5) dft5<T>(v);
  else if constexpr (R == 7) dft7<T>(v);
  else if constexpr (R == 8) dft8<T>(v);
}

// ------------------------------------------------------------- Stockham stage
// Govindaraju et al. (SC'08) self-sorting formulation: butterfly j of a stage
// with current span Ns reads x[j + t*n/R], twiddles by W_{Ns*R}^{t*(j%Ns)},
// and writes y[(j/Ns)*Ns*R + j%Ns + t*Ns].
template <typename T, int R, int VPT, int NT>
__device__ __forceinline__ void stockham_stage(cplx_t<T>* lds, int pitch, int n, int L, int Ns,
                                               const cplx_t<T>* __restrict__ tw, int tid,
                                               cplx_t<T> (&v)[VPT]) {
  using C = cplx_t<T>;
  constexpr int BPT = VPT / R;
  const int nbl = n / R;  // butterflies per line
  const int nbf = L * nbl;
  const FastDiv dnbl((uint32_t)nbl), dNs((uint32_t)Ns);
#pragma unroll
  for (int i = 0; i < BPT; ++i) {
    int b = tid + i * NT;
    if (b < nbf) {
      int line = dnbl.div(b);
      int j = b - line * nbl;
      const C* src = lds + line * pitch + j;
#pragma unroll
      for (int t = 0; t < R; ++t) v[i * R + t] = src[t * nbl];
    }
  }
  __syncthreads();
  const int tstride = n / (Ns * R);
#pragma unroll
  for (int i = 0; i < BPT; ++i) {
    int b = tid + i * NT;
    if (b < nbf) {
      int line = dnbl.div(b);
      int j = b - line * nbl;
      int k = dNs.mod(j);
      if (Ns > 1) {
        const int step = k * tstride;
#pragma unroll
        for (int t = 1; t < R; ++t) v[i * R + t] = cmul(v[i * R + t], tw[t * step]);
      }
      dftR<T, R>(&v[i * R]);
      C* dst = lds + line * pitch + (j - k) * R + k;
#pragma unroll
      for (int t = 0; t < R; ++t) dst[t * Ns] = v[i * R + t];
    }
  }
  __syncthreads();
}

// Direct DFT of every line (n with a prime factor > 7).
template <typename T, int VPT, int NT>
__device__ __forceinline__ void direct_dft(cplx_t<T>* lds, int pitch, int n, int L,
                                           const cplx_t<T>* __restrict__ tw, int tid,
                                           cplx_t<T> (&v)[VPT]) {
  using C = cplx_t<T>;
  const int tot = L * n;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    int b = tid + i * NT;
    if (b < tot) {
      int line = b / n;
      int k = b - line * n;
      const C* src = lds + line * pitch;
      C acc = C{(T)0, (T)0};
      int idx = 0;
      for (int j = 0; j < n; ++j) {
        C w = tw[idx];
        C x = src[j];
        acc.x += x.x * w.x - x.y * w.y;
        acc.y += x.x * w.y + x.y * w.x;
        idx += k;
        if (idx >= n) idx -= n;
      }
      v[i] = acc;
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    int b = tid + i * NT;
    if (b < tot) {
      int line = b / n;
      int k = b - line * n;
      lds[line * pitch + k] = v[i];
    }
  }
  __syncthreads();
}

// Full forward FFT of L lines resident in LDS.  Caller has synchronised after
// filling LDS; on return LDS holds the spectra and the workgroup is synced.
template <typename T, int VPT, int NT>
__device__ __forceinline__ void lds_fft(cplx_t<T>* lds, int pitch, int L, const FftPlanDev& p,
                                        const cplx_t<T>* __restrict__ tw, int tid) {
  cplx_t<T> v[VPT];
  if (p.nstages == 0) {
    direct_dft<T, VPT, NT>(lds, pitch, p.n, L, tw, tid, v);
    return;
  }
  int Ns = 1;
  for (int s = 0; s < p.nstages; ++s) {
    const int R = p.radix[s];
    switch (R) {
      case 8: stockham_stage<T, 8, VPT, NT>(lds, pitch, p.n, L, Ns, tw, tid, v); break;
      case 4: stockham_stage<T, 4, VPT, NT>(lds, pitch, p.n, L, Ns, tw, tid, v); break;
      case 2: stockham_stage<T, 2, VPT, NT>(lds, pitch, p.n, L, Ns, tw, tid, v); break;
      case 3: stockham_stage<T, 3, VPT, NT>(lds, pitch, p.n, L, Ns, tw, tid, v); break;
      case 5: stockham_stage<T, 5, VPT, NT>(lds, pitch, p.n, L, Ns, tw, tid, v); break;
      case 7: stockham_stage<T, 7, VPT, NT>(lds, pitch, p.n, L, Ns, tw, tid, v); break;
      default: break;
    }
    Ns *= R;
  }
}

}  // namespace nft
