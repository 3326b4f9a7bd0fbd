// Engine-v2 pass kernels (power-of-two lengths, compile-time plans).
//
// KIND: C2C (complex in/out, optional conj, scale, four-step post-twiddle),
//       R2C (rows only: two real rows -> two half spectra),
//       H1D (rows only: two real rows -> two real 1-D Hartley transforms),
//       UNPACK (complex in -> real Hartley out at k and at -k / mirror line).
// ROWS: contiguous lines (axis innermost) vs strided (L adjacent columns).
#pragma once
#include "fft_fast.hpp"
#include "fft_passes.hpp"

namespace nft {
namespace fast {

enum Kind { K_C2C = 0, K_R2C = 1, K_H1D = 2, K_UNPACK = 3 };

// Optional elementwise work fused into the first / last pass of a transform
// (flat real indices of the input / output array):
//   prologue  u[i] = (pa ? pa[i] : 1) * px[i] + (pb ? pb[i] * pc[pidx[i]] : 0)
//   epilogue  out[j] = (ea ? ea[j] : 1) * h + (ed ? eshift * ed[j] : 0);
//             out2[j] = eb[j] * h   (if out2)
struct FuseArgs {
  const void *pa, *px, *pb, *pc;
  const int* pidx;
  const void *ea, *ed, *eb;
  void* out2;
  double eshift;
  int pro, epi;
};

template <typename T>
__device__ __forceinline__ T fuse_pro(const FuseArgs& f, long long i) {
  T v = ((const T*)f.px)[i];
  if (f.pa) v *= ((const T*)f.pa)[i];
  if (f.pb) v += ((const T*)f.pb)[i] * ((const T*)f.pc)[f.pidx[i]];
  return v;
}

template <typename T>
__device__ __forceinline__ void fuse_store(const FuseArgs& f, T* out, long long j, T h) {
  if (!f.epi) {
    out[j] = h;
    return;
  }
  T r = f.ea ? ((const T*)f.ea)[j] * h : h;
  if (f.ed) r += (T)f.eshift * ((const T*)f.ed)[j];
  out[j] = r;
  if (f.out2) ((T*)f.out2)[j] = ((const T*)f.eb)[j] * h;
}

template <typename T> struct FastArgs {
  Lines g;
  const void* in;
  void* out;
  const void* tw;     // length-N table exp(-2 pi i k/N)
  const void* tw2;    // four-step post-twiddle table of length Nfull (or null)
  long long Ireal;    // pair modes: number of real rows
  int conj_in, conj_out, sigma;
  int km, kx, Nfull;  // UNPACK: full-axis index k = m*km + x*kx, transform length Nfull
  long long rs;       // UNPACK: real-output stride along the axis
  T scale;
  LineDesc desc;      // UNPACK: (o, i) -> real output line / mirror line
  FuseArgs f;         // R2C/H1D: prologue; UNPACK/H1D: epilogue
};

template <typename T, int N, int NT, int KIND, bool ROWS>
__global__ __launch_bounds__(NT) void fast_kernel(FastArgs<T> a) {
  using C = cplx_t<T>;
  constexpr int L = NT * VPT / N;
  static_assert(L >= 1, "NT*VPT must cover one line");
  constexpr int PITCH = ROWS ? N : N + 1;
  constexpr int SHN = ilog2(N), SHL = ilog2(L);
  extern __shared__ __align__(16) unsigned char smem[];
  C* lds = (C*)smem;
  const int tid = threadIdx.x;
  const long long t = blockIdx.x;
  const Lines& g = a.g;

  // ------------------------------------------------------------ load
  long long o = 0, m = 0, i0 = 0;
  if constexpr (ROWS) {
    o = t * L;  // first line of the tile
  } else {
    Tile tl = strided_tile<L>(g, t);
    o = tl.o;
    m = tl.m;
    i0 = tl.i0;
  }
#pragma unroll
  for (int r = 0; r < VPT; ++r) {
    const int e = tid + r * NT;
    int l, x;
    if constexpr (ROWS) {
      l = e >> SHN;
      x = e & (N - 1);
    } else {
      x = e >> SHL;
      l = e & (L - 1);
    }
    C v = C{(T)0, (T)0};
    if constexpr (KIND == K_R2C || KIND == K_H1D) {
      const T* in = (const T*)a.in;
      const long long row0 = 2 * (o + l);
      if (row0 < a.Ireal) {
        const long long i0 = row0 * g.in_so + (long long)x * g.in_sn;
        if (a.f.pro) {
          v.x = fuse_pro<T>(a.f, i0);
          if (row0 + 1 < a.Ireal) v.y = fuse_pro<T>(a.f, i0 + g.in_so);
        } else {
          v.x = in[i0];
          if (row0 + 1 < a.Ireal) v.y = in[i0 + g.in_so];
        }
      }
    } else {
      const C* in = (const C*)a.in;
      bool valid;
      long long off;
      if constexpr (ROWS) {
        valid = (o + l) < g.O;
        off = (o + l) * g.in_so + (long long)x * g.in_sn;
      } else {
        valid = (i0 + l) < g.I;
        off = o * g.in_so + m * g.in_sm + (i0 + l) * g.in_si + (long long)x * g.in_sn;
      }
      if (valid) v = in[off];
      if (a.conj_in) v.y = -v.y;
    }
    lds[l * PITCH + x] = v;
  }
  __syncthreads();
  fft<T, N, NT, L, PITCH>(lds, (const C*)a.tw, tid);

  // ------------------------------------------------------------ store
  if constexpr (KIND == K_C2C) {
    C* out = (C*)a.out;
    const C* tw2 = (const C*)a.tw2;
#pragma unroll
    for (int r = 0; r < VPT; ++r) {
      const int e = tid + r * NT;
      int l, x;
      if constexpr (ROWS) {
        l = e >> SHN;
        x = e & (N - 1);
      } else {
        x = e >> SHL;
        l = e & (L - 1);
      }
      C v = lds[l * PITCH + x];
      if (tw2) v = cmul(v, tw2[(m * x) & (a.Nfull - 1)]);
      if (a.conj_out) v.y = -v.y;
      v.x *= a.scale;
      v.y *= a.scale;
      if constexpr (ROWS) {
        if ((o + l) < g.O) out[(o + l) * g.out_so + (long long)x * g.out_sn] = v;
      } else {
        if ((i0 + l) < g.I)
          out[o * g.out_so + m * g.out_sm + (i0 + l) * g.out_si + (long long)x * g.out_sn] = v;
      }
    }
  } else if constexpr (KIND == K_R2C || KIND == K_H1D) {
    static_assert(ROWS, "pair modes are rows-only in engine v2");
    if constexpr (KIND == K_R2C) {
      C* out = (C*)a.out;
      constexpr int NH = N / 2 + 1;
      const T h = (T)0.5 * a.scale;
      for (int e = tid; e < L * NH; e += NT) {
        const int l = e / NH;
        const int k = e - l * NH;
        const long long row0 = 2 * (o + l);
        if (row0 >= a.Ireal) continue;
        const C zk = lds[l * PITCH + k];
        const C zm = lds[l * PITCH + ((N - k) & (N - 1))];
        const C xa = C{h * (zk.x + zm.x), h * (zk.y - zm.y)};
        const C xb = C{h * (zk.y + zm.y), -h * (zk.x - zm.x)};
        const long long ko = (long long)k * g.out_sn;
        out[row0 * g.out_so + ko] = xa;
        if (row0 + 1 < a.Ireal) out[(row0 + 1) * g.out_so + ko] = xb;
      }
    } else {
      T* out = (T*)a.out;
      const T hs = (T)0.5 * a.scale, sg = (T)a.sigma;
#pragma unroll
      for (int r = 0; r < VPT; ++r) {
        const int e = tid + r * NT;
        const int l = e >> SHN;
        const int k = e & (N - 1);
        const long long row0 = 2 * (o + l);
        if (row0 >= a.Ireal) continue;
        const C zk = lds[l * PITCH + k];
        const C zm = lds[l * PITCH + ((N - k) & (N - 1))];
        const long long ko = (long long)k * g.out_sn;
        fuse_store<T>(a.f, out, row0 * g.out_so + ko, hs * ((zk.x + zm.x) + sg * (zk.y - zm.y)));
        if (row0 + 1 < a.Ireal)
          fuse_store<T>(a.f, out, (row0 + 1) * g.out_so + ko, hs * ((zk.y + zm.y) - sg * (zk.x - zm.x)));
      }
    }
  } else {  // UNPACK
    T* out = (T*)a.out;
    UnpackLine* lines = (UnpackLine*)(smem + (size_t)L * PITCH * sizeof(C));
    for (int l = tid; l < L; l += NT) {
      UnpackLine u;
      bool valid;
      if constexpr (ROWS) {
        valid = (o + l) < g.O;
        if (valid) u = unpack_line(a.desc, o + l, 0);
      } else {
        valid = (i0 + l) < g.I;
        if (valid) u = unpack_line(a.desc, o, i0 + l);
      }
      if (!valid) {
        u.valid = 0;
        u.mirror = 0;
        u.base = u.mbase = 0;
      }
      lines[l] = u;
    }
    __syncthreads();
    const T sg = (T)a.sigma, sc = a.scale;
    const int Nf = a.Nfull;
#pragma unroll
    for (int r = 0; r < VPT; ++r) {
      const int e = tid + r * NT;
      int l, x;
      if constexpr (ROWS) {
        l = e >> SHN;
        x = e & (N - 1);
      } else {
        x = e >> SHL;
        l = e & (L - 1);
      }
      const UnpackLine u = lines[l];
      if (!u.valid) continue;
      const C f = lds[l * PITCH + x];
      const int k = (int)m * a.km + x * a.kx;
      fuse_store<T>(a.f, out, u.base + (long long)k * a.rs, sc * (f.x + sg * f.y));
      if (u.mirror) {
        const int km = (k == 0) ? 0 : Nf - k;
        fuse_store<T>(a.f, out, u.mbase + (long long)km * a.rs, sc * (f.x - sg * f.y));
      }
    }
  }
}

}  // namespace fast
}  // namespace nft
