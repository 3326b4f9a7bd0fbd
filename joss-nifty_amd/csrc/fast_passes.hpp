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
//   prologue  u[i] = (pa ? pa[j] : 1) * px[b*sx + j] + (pb ? pb[j] * pc[b*sc + pidx[j]*ce] : 0)
//   epilogue  out[b*so + j] = (ea ? ea[j] : 1) * h + (ed ? eshift * ed[b*sd + j] : 0);
//             out2[b*s2 + j] = eb[j] * h   (if out2)
// For a batch of transforms (leading batch axis, P elements per item) b = i / P
// and j = i mod P: pidx is shared by the batch, pa, pb, ea, eb too unless
// given a per-item stride, the other operands advance by their own batch
// stride.  P = 0: one item (b = 0, j = i).
struct FuseArgs {
  const void *pa, *px, *pb, *pc;
  const int* pidx;
  const void *ea, *ed, *eb;
  void* out2;
  double eshift;
  int pro, epi;
  long long P;
  int pshift;  // log2(P) if P is a power of two, else -1
  int nb;      // number of batch items (P > 0)
  long long sx, sc, so, sd, s2;
  long long ce;  // element stride of pc (>= 1)
  long long sa, sb, sea, seb;  // per-item strides of pa, pb, ea, eb (0: shared)
  // folded bin gather (nft_hartley_fuse.pro_folded): item grid n[0..fnd)
  // (all transform axes), fundamental-cell strides fs[] (C order over n/2+1)
  int fnd;
  long long fn[3], fs[3];
  // CG update carried by the unpack epilogue (nft_hartley_fuse.cg_*)
  int cg;
  void *cx, *cr;
  const void* cd;
  const double* csc;
  double* cpart;
  long long cst;   // row stride of x / r / d
  double cshift;
  int cnbtot, cblk0;
  long long ctr;   // tiles per item of the carrying pass (set by the launcher)
  // out2 as point-mirror pair sums on the half grid (nft_hartley_fuse.epi_out2_pairs):
  // out2[b * s2 + row * nh + col] = eb*h at (row, col) + eb*h at the point mirror
  int o2h;
  long long nlast, nh;
  // CG direction carried by the folded prologue (nft_hartley_fuse.dir_*)
  const void* dr;
  const double* dsc;
  double* dpart;
  long long dps;
  double dshift;
  int dblk0;
  // quadratic form of a pointwise weight carried by the unpack epilogue
  // (nft_hartley_fuse.quad_*): per tile the sum of h * (ea * h) over its
  // elements at qpart[item * qps + qblk0 + tile] (one item per tile)
  int quad;
  double* qpart;
  long long qps;
  int qblk0;
  // deferred iterate (nft_hartley_fuse.lazy_*): direction ring slots 1.. at
  // lring + (s - 1) * lss, alphas at lalpha[item * lnslot + s]
  int lazy;
  void* lring;
  long long lss;
  double* lalpha;
  long long lnslot;
  // CG curvature fold carried by the R2C row pass (nft_hartley_fuse.fold_*):
  // its first fnrhs workgroups write fout[r * fos] = the sum of
  // fpart[r * fnb + b] over b < fnb, before the pass's own tiles
  const double* fpart;
  double* fout;
  long long fos;
  int fnb, fnrhs;
};

// One RHS of the carried fold in nft_fold_partials' order (fold_wide: 1024
// thread-strided sums, the 16 waves' shuffle trees, the wave totals in order)
// by an NT-thread workgroup: virtual thread q * NT + t (q < 1024 / NT) keeps
// its own sum, so the result is bitwise the separate launch's.
template <int NT>
__device__ __forceinline__ void cg_fold_rhs(const FuseArgs& f, int r, double* sh) {
  static_assert(NT >= 64 && NT <= 1024 && 1024 % NT == 0, "cg_fold_rhs: NT divides 1024");
  constexpr int V = 1024 / NT, WPB = NT / 64;
  const double* part = f.fpart + (long long)r * f.fnb;
  const int t = threadIdx.x;
  double v[V];
#pragma unroll
  for (int q = 0; q < V; ++q) {
    v[q] = 0.0;
    for (int b = q * NT + t; b < f.fnb; b += 1024) v[q] += part[b];
  }
#pragma unroll
  for (int q = 0; q < V; ++q)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v[q] += __shfl_down(v[q], off, 64);
  if ((t & 63) == 0) {
#pragma unroll
    for (int q = 0; q < V; ++q) sh[q * WPB + (t >> 6)] = v[q];
  }
  __syncthreads();
  if (t == 0) {
    double s = 0.0;
    for (int w = 0; w < 16; ++w) s += sh[w];
    f.fout[(long long)r * f.fos] = s;
  }
}

// element index into pc of item-element j: its bin (pidx[j]) or, folded, the
// bin of its fundamental cell (pidx[cell(j)]), times the element stride
// (an item has < 2^31 elements: 32-bit index arithmetic)
__device__ __forceinline__ long long pro_cidx(const FuseArgs& f, long long j) {
  if (f.fnd == 0) return (long long)f.pidx[j] * f.ce;
  unsigned c = 0, r = (unsigned)j;
  for (int a = f.fnd - 1; a >= 0; --a) {
    const unsigned n = (unsigned)f.fn[a];
    const unsigned q = r / n;
    const unsigned k = r - q * n;
    r = q;
    c += (k <= n - k ? k : n - k) * (unsigned)f.fs[a];
  }
  return (long long)f.pidx[c] * f.ce;
}

__device__ __forceinline__ void fuse_split(const FuseArgs& f, long long i, long long& b, long long& j) {
  if (f.P == 0) {
    b = 0;
    j = i;
  } else if (f.pshift >= 0) {
    b = i >> f.pshift;
    j = i & (f.P - 1);
  } else {
    b = i / f.P;
    j = i - b * f.P;
  }
}

template <typename T>
__device__ __forceinline__ T fuse_pro(const FuseArgs& f, long long i) {
  long long b, j;
  fuse_split(f, i, b, j);
  T v = ((const T*)f.px)[b * f.sx + j];
  if (f.pa) v *= ((const T*)f.pa)[b * f.sa + j];
  if (f.pb) v += ((const T*)f.pb)[b * f.sb + j] * ((const T*)f.pc)[b * f.sc + pro_cidx(f, j)];
  return v;
}

template <typename T>
__device__ __forceinline__ void fuse_store(const FuseArgs& f, T* out, long long i, T h) {
  if (!f.epi) {
    out[i] = h;
    return;
  }
  long long b, j;
  fuse_split(f, i, b, j);
  T r = f.ea ? ((const T*)f.ea)[b * f.sea + j] * h : h;
  if (f.ed) r += (T)f.eshift * ((const T*)f.ed)[b * f.sd + j];
  out[b * f.so + j] = r;
  if (f.out2 && !f.o2h) ((T*)f.out2)[b * f.s2 + j] = ((const T*)f.eb)[b * f.seb + j] * h;
}

// point-mirror pair sum of the second epilogue output on the half grid: the
// element at flat index ib (column <= n_last / 2) and, when the line has one,
// its point mirror im (the same thread stores both in the unpack pass)
template <typename T>
__device__ __forceinline__ void fuse_store_pair(const FuseArgs& f, long long ib, T hb, bool mir, long long im, T hm) {
  long long b, j;
  fuse_split(f, ib, b, j);
  T w = ((const T*)f.eb)[b * f.seb + j] * hb;
  if (mir) {
    long long b2, j2;
    fuse_split(f, im, b2, j2);
    w += ((const T*)f.eb)[b2 * f.seb + j2] * hm;
  }
  const long long row = j / f.nlast, col = j - row * f.nlast;
  ((T*)f.out2)[b * f.s2 + row * f.nh + col] = w;
}

// epilogue store that carries the CG update instead of storing q = ea * h:
// the per-element arithmetic of cg_update_kernel (nft_blas.hip) on the value
// q that pass would have read back
template <typename T>
__device__ __forceinline__ void fuse_store_cg(const FuseArgs& f, long long i, T h, T al, bool ok, T shift,
                                              double& rr, double& xr) {
  long long b, j;
  fuse_split(f, i, b, j);
  const T q = f.ea ? ((const T*)f.ea)[b * f.sea + j] * h : h;
  if (f.out2 && !f.o2h) ((T*)f.out2)[b * f.s2 + j] = ((const T*)f.eb)[b * f.seb + j] * h;
  const long long e = b * f.cst + j;
  T xi = ((T*)f.cx)[e], ri = ((T*)f.cr)[e];
  if (ok) {
    const T di = ((const T*)f.cd)[e];
    xi = xi - al * di;
    ri = ri - al * (q + shift * di);
    ((T*)f.cx)[e] = xi;
    ((T*)f.cr)[e] = ri;
  }
  rr += (double)ri * (double)ri;
  xr += (double)xi * (double)ri;
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
  long long ntiles;   // tiles of the pass (set by the launcher)
  int bgroup;         // > 1: batch-aware XCD tile remap over this many items (set by the launcher)
  int bmode;          // remap flavour: 1 batch_tile, 2 batch_tile_contig
  int los;            // strided: log2 of the items (o) sharing one tile (their lines side by side)
};

// Batch-aware XCD remap.  Tiles are numbered batch-major (t = b * TR + r) and
// the operands shared by the batch (amplitude, xi0, pindex) are indexed by r
// only.  Workgroups are observed to be dealt round-robin over the 8 XCDs
// (MI355X_MICROARCH.md §Workgroup dispatch), so workgroup w runs on XCD group
// w % 8 at slot w / 8: giving the K items of one tile r consecutive slots of
// one XCD group makes the K reads of r's shared operands hit that XCD's L2
// instead of all going to HBM.  A bijection on [0, ntiles) when TR % 8 == 0
// (the launcher checks); placement is a speed choice only.
__device__ __forceinline__ long long batch_tile(long long w, long long ntiles, int K) {
  const long long TR = ntiles / K;
  const long long xg = w & 7, slot = w >> 3;
  const long long rl = slot / K, b = slot - rl * K;
  return b * TR + rl * 8 + xg;
}
// Contiguous variant: XCD group xg owns the tile range [xg TR/8, (xg+1) TR/8)
// and walks it in order, the K items of a tile back to back, so adjacent
// tiles (whose unaligned mirror-line runs share boundary cache lines) are
// also on one XCD at about the same time.  A bijection when TR % 8 == 0.
__device__ __forceinline__ long long batch_tile_contig(long long w, long long ntiles, int K) {
  const long long TR = ntiles / K;
  const long long xg = w & 7, slot = w >> 3;
  const long long rl = slot / K, b = slot - rl * K;
  return b * TR + xg * (TR >> 3) + rl;
}

// Persistent, prefetching tile loop: measured faster only for the plain
// real-to-complex row pass (256-thread workgroups, N <= 2048).  Everywhere
// else -- strided passes, and the R2C pass with a prologue, whose gathers
// cannot be prefetched -- one tile per workgroup at the lower register count
// (more resident waves) wins.
// (the persistent variant for N = 4096 with 512 threads measured slower:
// fp32 4096^2 R2C 141 -> 190 us per 4-RHS launch)
template <int N, int NT, int KIND, int VP = VPT>
constexpr bool persist_ok() {
  return N <= 2048 && NT * VP <= 256 * VPT && KIND == K_R2C;
}

// in-line LDS padding of a pass (fft_fast.hpp padx): every 8 elements for
// the strided passes, none for the row passes
template <int N, bool ROWS>
constexpr int pass_pad() {
  return ROWS ? -1 : 3;
}
// values per load group of the CG-carrying unpack epilogue (2 measured
// 209 -> 219 us at 4 x 2048^2)
constexpr int CG_CH_VALUES = 1;
// values per load group of the quadratic-form epilogue (EM 2)
constexpr int QUAD_CH_VALUES = 8;
// line pitch in LDS: the (padded) length, +1 for strided passes so the L
// lines' element x fall in different banks
template <int N, bool ROWS>
constexpr int pass_pitch() {
  return padded_len<N, pass_pad<N, ROWS>()>() + (ROWS ? 0 : 1);
}

// dynamic LDS of a pass: L lines (+ the unpack line table), then the
// quarter twiddle table (N/4 entries) at a 16-byte aligned offset
template <typename T, int N, int NT, int KIND, bool ROWS, int VP = VPT>
constexpr size_t tw_lds_offset() {
  constexpr int L = NT * VP / N;
  constexpr int PITCH = pass_pitch<N, ROWS>();
  return ((size_t)L * PITCH * sizeof(cplx_t<T>) + (KIND == K_UNPACK ? (size_t)L * sizeof(UnpackLine) : 0) + 15) &
         ~(size_t)15;
}
template <typename T, int N, int NT, int KIND, bool ROWS, int VP = VPT>
constexpr size_t pass_lds_bytes() {
  return tw_lds_offset<T, N, NT, KIND, ROWS, VP>() + (size_t)(N / 4) * sizeof(cplx_t<T>);
}

// EM (unpack passes): epilogue mode -- 0 plain, 1 the CG-carrying epilogue
// (a.f.cg), 2 the plain epilogue plus the per-tile quadratic-form partials
// (a.f.quad).  Each compiled alone: the plain unpack instance carries none of
// their registers (occupancy)
// VP: values per thread in the load / store phases (L = NT * VP / N lines per
// tile): the strided passes run VP = 4 at twice the threads of VPT = 8 -- the
// same tile and LDS, twice the resident waves
template <typename T, int N, int NT, int KIND, bool ROWS, bool PF, int EM = 0, int VP = VPT>
__global__ __launch_bounds__(NT) void fast_kernel(FastArgs<T> a) {
  // Persistent: workgroup b processes tiles b, b + G, b + 2G, ...  The input
  // of tile t + G is loaded into registers while tile t is transformed and
  // stored, so each workgroup keeps loads, LDS work and stores in flight at
  // once (at 2048^2 fp64 a pass has ~4 tiles per CU: without the overlap it
  // is one latency-bound wave of load, compute, store).  The prologue variant
  // (gathers feeding arithmetic) loads at the top of the loop instead.
  using C = cplx_t<T>;
  constexpr int L = NT * VP / N;
  static_assert(L >= 1, "NT*VP must cover one line");
  constexpr int PITCH = pass_pitch<N, ROWS>();
  constexpr int PS = pass_pad<N, ROWS>();
  constexpr int SHN = ilog2(N), SHL = ilog2(L);
  extern __shared__ __align__(16) unsigned char smem[];
  C* lds = (C*)smem;
  // the carried curvature fold: the first workgroups of the R2C row pass
  int nfold = 0;
  if constexpr (KIND == K_R2C) {
    nfold = a.f.fnrhs;
    if ((int)blockIdx.x < nfold) {
      cg_fold_rhs<NT>(a.f, (int)blockIdx.x, (double*)smem);
      return;
    }
  }
  C* twq = (C*)(smem + tw_lds_offset<T, N, NT, KIND, ROWS, VP>());
  for (int r = threadIdx.x; r < N / 4; r += NT) twq[r] = ((const C*)a.tw)[r];  // synced before the first stage
  const int tid = threadIdx.x;
  const Lines& g = a.g;
  const long long ntiles = a.ntiles;

  auto tile_of = [&](long long t, long long& o, long long& m, long long& i0) {
    if constexpr (ROWS) {
      o = t * L;  // first line of the tile
      m = 0;
      i0 = 0;
    } else {
      Tile tl = strided_tile<L>(g, t, a.los);
      o = tl.o;
      m = tl.m;
      i0 = tl.i0;
    }
  };
  // strided line l of the tile at (o, i0): its o and i (several items per tile: los > 0)
  const int lcs = SHL - a.los;
  auto line_oi = [&](long long o, long long i0, int l, long long& lo_, long long& li) {
    lo_ = o + (l >> lcs);
    li = i0 + (l & ((1 << lcs) - 1));
  };
  auto lx_of = [&](int r, int& l, int& x) {
    const int e = tid + r * NT;
    if constexpr (ROWS) {
      l = e >> SHN;
      x = e & (N - 1);
    } else {
      x = e >> SHL;
      l = e & (L - 1);
    }
  };
  // global -> registers (input values of tile t in load order)
  auto load = [&](long long t, C (&rv)[VP]) {
    long long o, m, i0;
    tile_of(t, o, m, i0);
#pragma unroll
    for (int r = 0; r < VP; ++r) {
      int l, x;
      lx_of(r, l, x);
      C v = C{(T)0, (T)0};
      if constexpr (KIND == K_R2C || KIND == K_H1D) {
        const T* in = (const T*)a.in;
        const long long row0 = 2 * (o + l);
        if (row0 < a.Ireal) {
          const long long e0 = row0 * g.in_so + (long long)x * g.in_sn;
          // the persistent variant never runs a prologue (launch_one)
          if (!PF && a.f.pro) {
            v.x = fuse_pro<T>(a.f, e0);
            if (row0 + 1 < a.Ireal) v.y = fuse_pro<T>(a.f, e0 + g.in_so);
          } else {
            v.x = in[e0];
            if (row0 + 1 < a.Ireal) v.y = in[e0 + g.in_so];
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
          long long lo_, li;
          line_oi(o, i0, l, lo_, li);
          valid = li < g.I && lo_ < g.O;
          off = lo_ * g.in_so + m * g.in_sm + li * g.in_si + (long long)x * g.in_sn;
        }
        if (valid) v = in[off];
        if (a.conj_in) v.y = -v.y;
      }
      rv[r] = v;
    }
  };

  constexpr bool PERSIST = PF;
  constexpr bool prefetch = PF;  // launched persistent only without a prologue
  C rv[VP];
  long long t = (long long)blockIdx.x - nfold;
  const long long gstride = (long long)gridDim.x - nfold;
  if constexpr (!PERSIST) {
    if (a.bgroup > 1) t = a.bmode == 2 ? batch_tile_contig(t, ntiles, a.bgroup) : batch_tile(t, ntiles, a.bgroup);
  }
  if (prefetch && t < ntiles) load(t, rv);
  while (t < ntiles) {
    if (!prefetch) load(t, rv);
#pragma unroll
    for (int r = 0; r < VP; ++r) {
      int l, x;
      lx_of(r, l, x);
      lds[l * PITCH + padx<PS>(x)] = rv[r];
    }
    __syncthreads();
    const long long tn = PERSIST ? t + gstride : ntiles;
    if (prefetch && tn < ntiles) load(tn, rv);  // in flight during the FFT and the stores
    fft<T, N, NT, L, PITCH, PS>(lds, twq, tid);
    long long o, m, i0;
    tile_of(t, o, m, i0);

    // ---------------------------------------------------------- store
    if constexpr (KIND == K_C2C) {
      C* out = (C*)a.out;
      const C* tw2 = (const C*)a.tw2;
#pragma unroll
      for (int r = 0; r < VP; ++r) {
        int l, x;
        lx_of(r, l, x);
        C v = lds[l * PITCH + padx<PS>(x)];
        if (tw2) v = cmul(v, tw2[(m * x) & (a.Nfull - 1)]);
        if (a.conj_out) v.y = -v.y;
        v.x *= a.scale;
        v.y *= a.scale;
        if constexpr (ROWS) {
          if ((o + l) < g.O) out[(o + l) * g.out_so + (long long)x * g.out_sn] = v;
        } else {
          long long lo_, li;
          line_oi(o, i0, l, lo_, li);
          if (li < g.I && lo_ < g.O)
            out[lo_ * g.out_so + m * g.out_sm + li * g.out_si + (long long)x * g.out_sn] = v;
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
          const C zk = lds[l * PITCH + padx<PS>(k)];
          const C zm = lds[l * PITCH + padx<PS>((N - k) & (N - 1))];
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
        for (int r = 0; r < VP; ++r) {
          const int e = tid + r * NT;
          const int l = e >> SHN;
          const int k = e & (N - 1);
          const long long row0 = 2 * (o + l);
          if (row0 >= a.Ireal) continue;
          const C zk = lds[l * PITCH + padx<PS>(k)];
          const C zm = lds[l * PITCH + padx<PS>((N - k) & (N - 1))];
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
          long long lo_, li;
          line_oi(o, i0, l, lo_, li);
          valid = li < g.I && lo_ < g.O;
          if (valid) u = unpack_line(a.desc, lo_, li);
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
      if constexpr (EM == 0) {
#pragma unroll
        for (int r = 0; r < VP; ++r) {
          int l, x;
          lx_of(r, l, x);
          const UnpackLine u = lines[l];
          if (!u.valid) continue;
          const C f = lds[l * PITCH + padx<PS>(x)];
          const int k = (int)m * a.km + x * a.kx;
          const long long ib = u.base + (long long)k * a.rs;
          const T hb = sc * (f.x + sg * f.y);
          fuse_store<T>(a.f, out, ib, hb);
          long long im = 0;
          T hm = (T)0;
          if (u.mirror) {
            const int km = (k == 0) ? 0 : Nf - k;
            im = u.mbase + (long long)km * a.rs;
            hm = sc * (f.x - sg * f.y);
            fuse_store<T>(a.f, out, im, hm);
          }
          if (a.f.o2h) fuse_store_pair<T>(a.f, ib, hb, u.mirror != 0, im, hm);
        }
      } else if constexpr (EM == 2) {
        // out = ea * h (shared weight, no shift / second output) and the
        // tile's sum of h * out: the metric's data-space quadratic form
        // (J d).W(J d) of a pointwise W, one item per tile (los = 0)
        // every weight load of a group of QCH values first, then the products,
        // stores and sums in the element order (each load waited on before
        // the next value's store otherwise: one round trip per value); the
        // second phase re-derives the indices and values from LDS (registers)
        const long long item = o;
        const T* __restrict__ ea = (const T*)a.f.ea;
        double qs = 0.0;
        constexpr int QCH = QUAD_CH_VALUES < VP ? QUAD_CH_VALUES : VP;
        auto elem = [&](int r, int h, bool& use, T& hv, long long& b, long long& j) {
          int l, x;
          lx_of(r, l, x);
          const UnpackLine u = lines[l];
          const C f = lds[l * PITCH + padx<PS>(x)];
          const int k = (int)m * a.km + x * a.kx;
          use = u.valid != 0 && (h == 0 || u.mirror != 0);
          hv = h == 0 ? sc * (f.x + sg * f.y) : sc * (f.x - sg * f.y);
          const long long idx = h == 0 ? u.base + (long long)k * a.rs : u.mbase + (long long)((k == 0) ? 0 : Nf - k) * a.rs;
          fuse_split(a.f, idx, b, j);
        };
#pragma unroll
        for (int r0 = 0; r0 < VP; r0 += QCH) {
          T wv[QCH][2];
#pragma unroll
          for (int c = 0; c < QCH; ++c) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              bool use;
              T hv;
              long long b, j;
              elem(r0 + c, h, use, hv, b, j);
              wv[c][h] = use ? ea[b * a.f.sea + j] : (T)0;
            }
          }
#pragma unroll
          for (int c = 0; c < QCH; ++c) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              bool use;
              T hv;
              long long b, j;
              elem(r0 + c, h, use, hv, b, j);
              if (!use) continue;
              const T q = wv[c][h] * hv;
              out[b * a.f.so + j] = q;
              qs += (double)hv * (double)q;
            }
          }
        }
        __shared__ double qsh[NT / 64];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) qs += __shfl_down(qs, off, 64);
        if ((tid & 63) == 0) qsh[tid >> 6] = qs;
        __syncthreads();
        if (tid == 0) {
          double s0 = 0.0;
          for (int w = 0; w < NT / 64; ++w) s0 += qsh[w];
          a.f.qpart[item * a.f.qps + a.f.qblk0 + (t - item * a.f.ctr)] = s0;
        }
      } else {
        // one item per tile (los = 0): its step length from its CG scalars
        const long long item = o;
        const double* scb = a.f.csc + item * NFT_CG_NSCALARS;
        const double curv = scb[NFT_CG_CURV], gprev = scb[NFT_CG_GAMMA];
        const double alpha = gprev / curv;
        const bool ok = (curv == curv) && curv != 0.0 && (alpha >= 0.0) && (alpha == alpha) &&
                        scb[NFT_CG_DONE] == 0.0;
        const T al = (T)alpha, shift = (T)a.f.cshift;
        double rr = 0.0, xr = 0.0;
        // two phases per group of CG_CH values: every operand load of the
        // group first, then the arithmetic and the stores -- the loads of
        // x and r cannot pass the previous stores to x and r otherwise
        // (same arrays, runtime offsets), which serialised one memory
        // round trip per element
        constexpr int CG_CH = CG_CH_VALUES;
        // deferred iterate (nft_hartley_fuse.lazy_*): d from the ring slot this
        // step's prologue wrote, x untouched, the step's alpha recorded
        const bool lazy = a.f.lazy != 0;
        // (clamped: a counter out of range never addresses outside the ring)
        const long long sl = lazy ? min(max((long long)scb[NFT_CG_LAZY], 0LL), a.f.lnslot - 1) : 0;
        if (lazy && tid == 0 && t - item * a.f.ctr == 0)
          a.f.lalpha[item * a.f.lnslot + sl] = ok ? alpha : __builtin_nan("");
        const T* __restrict__ ea = (const T*)a.f.ea;
        const T* __restrict__ eb = (const T*)a.f.eb;
        const T* __restrict__ cd = lazy ? (const T*)a.f.lring + sl * a.f.lss : (const T*)a.f.cd;
        T* __restrict__ cx = (T*)a.f.cx;
        T* __restrict__ cr = (T*)a.f.cr;
#pragma unroll
        for (int r0 = 0; r0 < VP; r0 += CG_CH) {
          long long ev[CG_CH][2], jv[CG_CH][2], bv[CG_CH][2];
          bool use[CG_CH][2];
          T hv[CG_CH][2], xv[CG_CH][2], rv_[CG_CH][2], dv[CG_CH][2], qv[CG_CH][2], wv[CG_CH][2];
#pragma unroll
          for (int c = 0; c < CG_CH; ++c) {
            int l, x;
            lx_of(r0 + c, l, x);
            const UnpackLine u = lines[l];
            const C fv = lds[l * PITCH + padx<PS>(x)];
            const int k = (int)m * a.km + x * a.kx;
            const int km = (k == 0) ? 0 : Nf - k;
            use[c][0] = u.valid != 0;
            use[c][1] = u.valid != 0 && u.mirror != 0;
            hv[c][0] = sc * (fv.x + sg * fv.y);
            hv[c][1] = sc * (fv.x - sg * fv.y);
            const long long idx[2] = {u.base + (long long)k * a.rs, u.mbase + (long long)km * a.rs};
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              long long b, j;
              fuse_split(a.f, idx[h], b, j);
              bv[c][h] = b;
              jv[c][h] = j;
              ev[c][h] = b * a.f.cst + j;
              xv[c][h] = rv_[c][h] = dv[c][h] = qv[c][h] = wv[c][h] = (T)0;
              if (use[c][h]) {
                if (!lazy) xv[c][h] = cx[ev[c][h]];
                rv_[c][h] = cr[ev[c][h]];
                if (ok) dv[c][h] = cd[ev[c][h]];
                qv[c][h] = ea ? ea[b * a.f.sea + j] : (T)1;
                if (a.f.out2) wv[c][h] = eb[b * a.f.seb + j];
              }
            }
          }
#pragma unroll
          for (int c = 0; c < CG_CH; ++c) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              if (!use[c][h]) continue;
              // the per-element arithmetic of fuse_store_cg
              const T q = ea ? qv[c][h] * hv[c][h] : hv[c][h];
              T xi = xv[c][h], ri = rv_[c][h];
              if (ok) {
                const T di = dv[c][h];
                xi = xi - al * di;
                ri = ri - al * (q + shift * di);
                if (!lazy) cx[ev[c][h]] = xi;
                cr[ev[c][h]] = ri;
              }
              rr += (double)ri * (double)ri;
              if (!lazy) xr += (double)xi * (double)ri;
              if (a.f.out2 && !a.f.o2h) ((T*)a.f.out2)[bv[c][h] * a.f.s2 + jv[c][h]] = wv[c][h] * hv[c][h];
            }
            if (a.f.o2h && use[c][0]) {
              T w = wv[c][0] * hv[c][0];
              if (use[c][1]) w += wv[c][1] * hv[c][1];
              const long long j = jv[c][0];
              const long long row = j / a.f.nlast, col = j - row * a.f.nlast;
              ((T*)a.f.out2)[bv[c][0] * a.f.s2 + row * a.f.nh + col] = w;
            }
          }
        }
        // fixed-order block sums (wave shuffles, then the waves in order)
        __shared__ double cgsh[2 * (NT / 64)];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
          rr += __shfl_down(rr, off, 64);
          xr += __shfl_down(xr, off, 64);
        }
        if ((tid & 63) == 0) {
          cgsh[2 * (tid >> 6)] = rr;
          cgsh[2 * (tid >> 6) + 1] = xr;
        }
        __syncthreads();
        if (tid == 0) {
          double s0 = 0.0, s1 = 0.0;
          for (int w = 0; w < NT / 64; ++w) {
            s0 += cgsh[2 * w];
            s1 += cgsh[2 * w + 1];
          }
          const long long nbt = a.f.cnbtot;
          double* pp = a.f.cpart + item * 3 * nbt + a.f.cblk0 + (t - item * a.f.ctr);
          pp[0] = s0;
          pp[nbt] = s1;
          pp[2 * nbt] = 0.0;
        }
      }
    }
    if constexpr (!PERSIST) break;
    __syncthreads();  // LDS free for the next tile
    t = tn;
  }
}

}  // namespace fast
}  // namespace nft
