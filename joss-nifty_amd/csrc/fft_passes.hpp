// Batched axis passes built on the LDS line-FFT engine (fft_core.hpp).
//
// A "pass" transforms every line of a d-dimensional array along one axis.
// Lines are addressed as (o, i): o runs over the flattened dims before the
// axis, i over the flattened dims after it; element x of line (o, i) sits at
// o*so + i*si + x*sn.  Two tilings:
//   rows    (axis is the innermost dim, I == 1): a workgroup takes L
//           consecutive lines, each a contiguous run in memory;
//   strided (axis is not innermost): a workgroup takes L consecutive i of
//           one o, so every row of the tile is an L-element contiguous segment.
//
// Pass kinds (each is one kernel launch, one read + one write of the data):
//   C2C     complex -> complex (optionally conjugating in/out = inverse)
//   R2C     two real lines packed as re/im of one complex line, split into
//           the two half spectra (k = 0..n/2) after the FFT
//   H1D     two real lines packed, written back as their real 1-D Hartley
//           transforms (single-axis hartley)
//   UNPACK  final pass of a multi-axis Hartley transform: the line holds the
//           half-spectrum F over all transformed axes; it is written as real
//           H = Re F + s Im F to line l and as Re F(-k) - s Im F(-k) to the
//           mirror line l' (all transformed coordinates negated).
#pragma once
#include "fft_core.hpp"

namespace nft {

constexpr int MAXD = 8;

// Describes how a line position (o, i) of the complex half-spectrum buffer maps
// to the real output array, for the UNPACK pass.
struct LineDesc {
  int nout, nin;             // number of dims before / after the pass axis
  int ext[MAXD];             // extents in the complex buffer (outer dims first, then inner)
  long long rstride[MAXD];   // strides in the real output
  int nreal[MAXD];           // real extents (for mirroring)
  int neg[MAXD];             // 1 if the coordinate is negated in the mirror line
  int half;                  // index (into the arrays above) of the half-spectrum dim, -1 if none
};

template <typename T> struct PassArgs {
  FftPlanDev plan;
  const void* in;
  void* out;
  long long in_so, in_si, in_sn;     // input strides (in elements of the input type)
  long long out_so, out_si, out_sn;  // output strides (elements of output type)
  long long O, I;                    // line-space extents (complex lines)
  long long Ireal;                   // pair modes: real extent along the pairing dim
  int rows;                          // 1 = rows tiling, 0 = strided tiling
  int L;                             // lines per workgroup
  int pitch;                         // LDS pitch (complex elements)
  int conj_in, conj_out;
  int sigma;                         // +1 non-canonical Hartley (Re+Im), -1 canonical (Re-Im)
  T scale;
  const void* tw;                    // twiddle table exp(-2 pi i k / n), k < n
  LineDesc desc;
};

// Line position -> (o, i) for line l of tile `tile`.
struct TileMap {
  long long o, i;
  bool valid;
};

template <typename T>
__device__ __forceinline__ TileMap tile_line(const PassArgs<T>& a, long long tile, int l) {
  TileMap m;
  if (a.rows) {
    m.o = tile * a.L + l;
    m.i = 0;
    m.valid = m.o < a.O;
  } else {
    long long tilesI = (a.I + a.L - 1) / a.L;
    m.o = tile / tilesI;
    m.i = (tile - m.o * tilesI) * a.L + l;
    m.valid = m.i < a.I;
  }
  return m;
}

// element e of the tile -> (line l, position x).  rows: x fastest; strided: l fastest
template <typename T>
__device__ __forceinline__ void tile_elem(const PassArgs<T>& a, int e, const FastDiv& dn,
                                          const FastDiv& dL, int& l, int& x) {
  if (a.rows) {
    l = dn.div(e);
    x = e - l * a.plan.n;
  } else {
    x = dL.div(e);
    l = e - x * a.L;
  }
}

// ------------------------------------------------------------------ loaders
// complex lines
template <typename T, int NT>
__device__ __forceinline__ void load_c(const PassArgs<T>& a, long long tile, cplx_t<T>* lds) {
  using C = cplx_t<T>;
  const C* __restrict__ in = (const C*)a.in;
  const int n = a.plan.n, tot = a.L * n;
  const FastDiv dn(n), dL(a.L);
  for (int e = threadIdx.x; e < tot; e += NT) {
    int l, x;
    tile_elem(a, e, dn, dL, l, x);
    TileMap m = tile_line(a, tile, l);
    C v = C{(T)0, (T)0};
    if (m.valid) v = in[m.o * a.in_so + m.i * a.in_si + (long long)x * a.in_sn];
    if (a.conj_in) v.y = -v.y;
    lds[l * a.pitch + x] = v;
  }
}

// pairs of real lines (along the pairing dim) as re/im
template <typename T, int NT>
__device__ __forceinline__ void load_rp(const PassArgs<T>& a, long long tile, cplx_t<T>* lds) {
  using C = cplx_t<T>;
  const T* __restrict__ in = (const T*)a.in;
  const int n = a.plan.n, tot = a.L * n;
  const FastDiv dn(n), dL(a.L);
  for (int e = threadIdx.x; e < tot; e += NT) {
    int l, x;
    tile_elem(a, e, dn, dL, l, x);
    TileMap m = tile_line(a, tile, l);
    C v = C{(T)0, (T)0};
    if (m.valid) {
      long long xo = (long long)x * a.in_sn;
      if (a.rows) {
        long long r0 = 2 * m.o;
        v.x = in[r0 * a.in_so + xo];
        if (r0 + 1 < a.Ireal) v.y = in[(r0 + 1) * a.in_so + xo];
      } else {
        long long c0 = 2 * m.i;
        v.x = in[m.o * a.in_so + c0 * a.in_si + xo];
        if (c0 + 1 < a.Ireal) v.y = in[m.o * a.in_so + (c0 + 1) * a.in_si + xo];
      }
    }
    lds[l * a.pitch + x] = v;
  }
}

// ------------------------------------------------------------------ storers
template <typename T, int NT>
__device__ __forceinline__ void store_c(const PassArgs<T>& a, long long tile, const cplx_t<T>* lds) {
  using C = cplx_t<T>;
  C* __restrict__ out = (C*)a.out;
  const int n = a.plan.n, tot = a.L * n;
  const FastDiv dn(n), dL(a.L);
  for (int e = threadIdx.x; e < tot; e += NT) {
    int l, x;
    tile_elem(a, e, dn, dL, l, x);
    TileMap m = tile_line(a, tile, l);
    if (!m.valid) continue;
    C v = lds[l * a.pitch + x];
    if (a.conj_out) v.y = -v.y;
    v.x *= a.scale;
    v.y *= a.scale;
    out[m.o * a.out_so + m.i * a.out_si + (long long)x * a.out_sn] = v;
  }
}

// split packed pair spectra into the two half spectra k = 0..n/2
template <typename T, int NT>
__device__ __forceinline__ void store_r2c(const PassArgs<T>& a, long long tile, const cplx_t<T>* lds) {
  using C = cplx_t<T>;
  C* __restrict__ out = (C*)a.out;
  const int n = a.plan.n, nh = n / 2 + 1, tot = a.L * nh;
  const FastDiv dn(nh), dL(a.L);
  for (int e = threadIdx.x; e < tot; e += NT) {
    int l, k;
    if (a.rows) { l = dn.div(e); k = e - l * nh; }
    else { k = dL.div(e); l = e - k * a.L; }
    TileMap m = tile_line(a, tile, l);
    if (!m.valid) continue;
    C zk = lds[l * a.pitch + k];
    C zm = lds[l * a.pitch + (k == 0 ? 0 : n - k)];
    const T h = (T)0.5;
    C xa = C{h * (zk.x + zm.x), h * (zk.y - zm.y)};
    C xb = C{h * (zk.y + zm.y), -h * (zk.x - zm.x)};
    xa.x *= a.scale; xa.y *= a.scale;
    xb.x *= a.scale; xb.y *= a.scale;
    long long ko = (long long)k * a.out_sn;
    if (a.rows) {
      long long r0 = 2 * m.o;
      out[r0 * a.out_so + ko] = xa;
      if (r0 + 1 < a.Ireal) out[(r0 + 1) * a.out_so + ko] = xb;
    } else {
      long long c0 = 2 * m.i;
      out[m.o * a.out_so + c0 * a.out_si + ko] = xa;
      if (c0 + 1 < a.Ireal) out[m.o * a.out_so + (c0 + 1) * a.out_si + ko] = xb;
    }
  }
}

// real 1-D Hartley transforms of the packed pair
template <typename T, int NT>
__device__ __forceinline__ void store_h1d(const PassArgs<T>& a, long long tile, const cplx_t<T>* lds) {
  using C = cplx_t<T>;
  T* __restrict__ out = (T*)a.out;
  const int n = a.plan.n, tot = a.L * n;
  const FastDiv dn(n), dL(a.L);
  const T hs = (T)0.5 * a.scale, sg = (T)a.sigma;
  for (int e = threadIdx.x; e < tot; e += NT) {
    int l, k;
    tile_elem(a, e, dn, dL, l, k);
    TileMap m = tile_line(a, tile, l);
    if (!m.valid) continue;
    C zk = lds[l * a.pitch + k];
    C zm = lds[l * a.pitch + (k == 0 ? 0 : n - k)];
    T ha = hs * ((zk.x + zm.x) + sg * (zk.y - zm.y));
    T hb = hs * ((zk.y + zm.y) - sg * (zk.x - zm.x));
    long long ko = (long long)k * a.out_sn;
    if (a.rows) {
      long long r0 = 2 * m.o;
      out[r0 * a.out_so + ko] = ha;
      if (r0 + 1 < a.Ireal) out[(r0 + 1) * a.out_so + ko] = hb;
    } else {
      long long c0 = 2 * m.i;
      out[m.o * a.out_so + c0 * a.out_si + ko] = ha;
      if (c0 + 1 < a.Ireal) out[m.o * a.out_so + (c0 + 1) * a.out_si + ko] = hb;
    }
  }
}

// per-line output bases for UNPACK: decode (o, i) into coordinates
struct UnpackLine {
  long long base, mbase;
  int valid, mirror;
};

__device__ __forceinline__ UnpackLine unpack_line(const LineDesc& d, long long o, long long i) {
  UnpackLine u;
  u.base = 0;
  u.mbase = 0;
  u.valid = 1;
  u.mirror = 0;
  int c[MAXD];
  // outer dims: o row-major over dims [0, nout)
  for (int k = d.nout - 1; k >= 0; --k) {
    long long q = o / d.ext[k];
    c[k] = (int)(o - q * d.ext[k]);
    o = q;
  }
  for (int k = d.nout + d.nin - 1; k >= d.nout; --k) {
    long long q = i / d.ext[k];
    c[k] = (int)(i - q * d.ext[k]);
    i = q;
  }
  for (int k = 0; k < d.nout + d.nin; ++k) {
    int m = c[k];
    if (d.neg[k]) m = (c[k] == 0) ? 0 : d.nreal[k] - c[k];
    u.base += (long long)c[k] * d.rstride[k];
    u.mbase += (long long)m * d.rstride[k];
  }
  if (d.half >= 0) {
    int ch = c[d.half], nr = d.nreal[d.half];
    if (ch > nr / 2) u.valid = 0;
    u.mirror = (ch != 0) && (2 * ch != nr);
  }
  return u;
}

template <typename T, int NT>
__device__ __forceinline__ void store_unpack(const PassArgs<T>& a, long long tile, const cplx_t<T>* lds,
                                             UnpackLine* lines) {
  using C = cplx_t<T>;
  T* __restrict__ out = (T*)a.out;
  for (int l = threadIdx.x; l < a.L; l += NT) {
    TileMap m = tile_line(a, tile, l);
    UnpackLine u;
    if (m.valid) u = unpack_line(a.desc, m.o, m.i);
    else { u.valid = 0; u.mirror = 0; u.base = u.mbase = 0; }
    lines[l] = u;
  }
  __syncthreads();
  const int n = a.plan.n, tot = a.L * n;
  const FastDiv dn(n), dL(a.L);
  const T sg = (T)a.sigma, sc = a.scale;
  for (int e = threadIdx.x; e < tot; e += NT) {
    int l, x;
    tile_elem(a, e, dn, dL, l, x);
    UnpackLine u = lines[l];
    if (!u.valid) continue;
    long long xo = (long long)x * a.out_sn;
    C f = lds[l * a.pitch + x];
    out[u.base + xo] = sc * (f.x + sg * f.y);
    if (u.mirror) {
      C g = lds[l * a.pitch + (x == 0 ? 0 : n - x)];
      out[u.mbase + xo] = sc * (g.x - sg * g.y);
    }
  }
}

}  // namespace nft
