// Box-blocked line-of-sight response (LOSResponse.apply, src/library/
// los_response.py:226-233; the reference applies a scipy COO matrix whose
// entries it stores grouped by 16x16 pixel boxes, :180-224).
//
// The grid is cut into 256-pixel boxes (16x16 over the last two axes; 1x256
// for 1-D grids).  Both directions work box by box, so every pixel-side
// access is a coalesced tile access instead of a random gather:
//
//  forward  y = rs * R (cs * x):
//    K1 (one workgroup per work item = box + range of its (box, los)
//        segments): stage cs*x of the box in LDS (16 rows of 128 B), form
//        w * u[loc] for the item's entries (8-bit local pixel index + fp32
//        weight per nonzero), and sum each segment in storage order; the
//        partial goes to its slot in LOS-major order, the K vectors of a
//        slot adjacent (one 8K-byte store per segment).
//    K2 (one wave per line of sight): fixed-order sum of its slots, read
//        contiguously for all K vectors.
//  adjoint  out = rs * R^T (cs * y):
//    K3 (one workgroup per box): the values cs*y of the ~100 lines crossing
//        the box are cached in LDS once; w * y[line] for the box's entries
//        (sorted by local pixel, storage order within a pixel; 8-bit line
//        index + fp32 weight) is staged in LDS chunk by chunk and thread t
//        sums pixel t's run; the box tile is written coalesced.
//
// All reductions run in a fixed order: deterministic, no atomics.
#include <algorithm>
#include <cstdlib>

#include "nft_api_internal.hpp"

namespace nft {

constexpr int LOS_CAP_F = 2048;  // entries per forward work item (host-guaranteed)
constexpr int LOS_CH_A = 2048;   // adjoint: entries staged in LDS per chunk
constexpr int LOS_YL = 2048;     // adjoint: LDS slots for the line values of a box (all batch vectors)
constexpr int LOS_KMAX = 8;      // vectors per batched launch
// forward: one lane per segment (<= 256 segments per work item,
// host-guaranteed: one round of the 256 lanes), summing the segment's
// entries in the order the earlier four-lane groups did -- four strided
// partial sums (entries a + q, a + q + 4, ... into acc[q]), then
// (acc0 + acc1) + (acc2 + acc3), the quad's xor-shuffle tree -- so the
// results are bitwise those of four lanes per segment (the sampling CG with
// value-driven controllers follows the reference's decisions only with this
// rounding: a plain serial sum moved demo64's AbsDelta solve from 28 to 24
// checks).  Four lanes with shuffles: 131 us; one lane: 120 us (4 x 2048^2,
// per-box kernel): the segments are short (16 entries on average at 2048^2 /
// 16384 lines) and the shuffles and idle lanes of a partly filled second
// round cost more than the longer chain per lane.
// sum of the products w_k * u[l_k][b] over entries [a, e) of a segment for
// the K vectors, in the four-lane order (see above)
template <int K, typename F>
__device__ __forceinline__ void seg_sum4(int a, int e, F&& prod, double (&out)[K]) {
#pragma clang fp contract(off)
  double acc[4][K];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int b = 0; b < K; ++b) acc[q][b] = 0.0;
  for (int k = a; k < e; k += 4) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (k + q < e) prod(k + q, acc[q]);
  }
#pragma unroll
  for (int b = 0; b < K; ++b) out[b] = (acc[0][b] + acc[1][b]) + (acc[2][b] + acc[3][b]);
}

struct BoxGeom {
  long long H, W;
  int bh, bw, nby, nbx;
  __device__ __forceinline__ long long pixel(int box, int t, bool& ok) const {
    const int bpl = nby * nbx;
    const long long l = box / bpl;
    const int r = box - (int)(l * bpl);
    const int by = r / nbx, bx = r - by * nbx;
    const int ly = t / bw, lx = t - ly * bw;
    const long long y = (long long)by * bh + ly, x = (long long)bx * bw + lx;
    ok = (y < H) && (x < W);
    return (l * H + y) * W + x;
  }
};

// Batched over K vectors (template, 1 <= K <= LOS_KMAX): the entries of a
// work item (fp32 weight + 8-bit local pixel) are staged in LDS ONCE and
// applied to every vector's tile; each segment's lane accumulates all K
// vectors in registers.  Per vector the products and their summation order
// are those of K = 1 (bitwise).
//
// Segment s's partial of vector b goes to part[seg_slot[s] * pk + b] (pk =
// vectors of the call): one contiguous store per segment for all vectors, and
// the reduce reads each line's slots contiguously.  The bounds and slot of a
// thread's segment are loaded before the barrier, off the critical path of
// the segment loop.

template <typename T, int K>
__global__ __launch_bounds__(256) void los_fwd_items(nft_los_plan p, const T* __restrict__ x,
                                                     const T* __restrict__ cs, double* __restrict__ part,
                                                     long long xs, int pk, long long css, int kv) {
  // every product is rounded before it is summed, in all K variants alike
  // (no FMA contraction): batched results are bitwise the K = 1 results
#pragma clang fp contract(off)
  constexpr int PER = LOS_CAP_F / 256;
  // pixel-major tile: the K values of one pixel are adjacent (one or two
  // 16-byte LDS reads per entry instead of K 8-byte ones)
  __shared__ __align__(16) double u[256][K];
  __shared__ float ew[K == 1 ? 1 : LOS_CAP_F];
  __shared__ unsigned char el[K == 1 ? 1 : LOS_CAP_F];
  __shared__ double prodbuf[K == 1 ? LOS_CAP_F : 1];
  const BoxGeom g{p.H, p.W, p.bh, p.bw, p.nby, p.nbx};
  const int it = (int)blockIdx.x, t = threadIdx.x;
  if (it >= p.nitems) return;
  const int box = p.item_box[it];
  bool ok;
  const long long px = g.pixel(box, t, ok);
  const int s0 = p.item_seg[it], s1 = p.item_seg[it + 1];
  const int e0 = p.item_ent[it], e1 = p.item_ent[it + 1];
  const int n = e1 - e0;
  const bool staged = n <= LOS_CAP_F;  // host plans always fit; others take the direct path
  float wv[PER];
  unsigned char lv[PER];
  if (staged) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int k = t + i * 256;
      wv[i] = k < n ? p.ent_wf[e0 + k] : 0.f;
      lv[i] = k < n ? p.ent_loc[e0 + k] : 0;
    }
  }
  // column (pixel-side) scale: shared by the vectors (css = 0) or one per vector
#pragma unroll
  for (int b = 0; b < K; ++b) {
    double v = 0.0;
    if (ok && b < kv) {
      v = (double)x[b * xs + px];
      if (cs) v *= (double)cs[b * css + px];
    }
    u[t][b] = v;
  }
  // one lane per segment: thread t serves segment s0 + t (+ 256 r beyond
  // the host guarantee)
  const int sq = s0 + t;
  const int sa = sq < s1 ? p.seg_ent[sq] - e0 : 0;
  const int sb = sq < s1 ? p.seg_ent[sq + 1] - e0 : 0;
  const int so = sq < s1 ? p.seg_slot[sq] : 0;
  if (K > 1 && staged) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int k = t + i * 256;
      if (k < n) {
        ew[k] = wv[i];
        el[k] = lv[i];
      }
    }
  }
  __syncthreads();
  if constexpr (K == 1) {
    // single vector: stage the products once (fewer LDS reads per entry)
    double* prod = prodbuf;
    if (staged) {
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int k = t + i * 256;
        if (k < n) prod[k] = (double)wv[i] * u[lv[i]][0];
      }
    }
    __syncthreads();
    auto seg1 = [&](int slot, int a, int e) {
      double a0[1];
      if (staged) {
        seg_sum4<1>(a, e, [&](int k, double(&acc)[1]) { acc[0] += prod[k]; }, a0);
      } else {
        seg_sum4<1>(a, e, [&](int k, double(&acc)[1]) {
          acc[0] = acc[0] + (double)p.ent_wf[e0 + k] * u[p.ent_loc[e0 + k]][0];
        }, a0);
      }
      part[(long long)slot * pk] = a0[0];
    };
    if (sq < s1) seg1(so, sa, sb);
    for (int s = sq + 256; s < s1; s += 256) seg1(p.seg_slot[s], p.seg_ent[s] - e0, p.seg_ent[s + 1] - e0);
    return;
  }
  auto segk = [&](int slot, int a, int e) {
    double acc[K];
    seg_sum4<K>(a, e, [&](int k, double(&c)[K]) {
      const double w = staged ? (double)ew[k] : (double)p.ent_wf[e0 + k];
      const int l = staged ? el[k] : p.ent_loc[e0 + k];
#pragma unroll
      for (int b = 0; b < K; ++b) c[b] = c[b] + w * u[l][b];
    }, acc);
#pragma unroll
    for (int b = 0; b < K; ++b)
      if (b < kv) part[(long long)slot * pk + b] = acc[b];
  };
  if (sq < s1) segk(so, sa, sb);
  for (int s = sq + 256; s < s1; s += 256) segk(p.seg_slot[s], p.seg_ent[s] - e0, p.seg_ent[s + 1] - e0);
}

// One workgroup per box (nft_los_plan.box_item, K > 1): the pixel tile's
// loads depend on the box index only, so they issue at once, beside the box's
// segment / entry bounds; a box of several work items (> LOS_CAP_F entries
// or > 256 segments) loops over them with the tile staged once.  The entries
// of an item are staged from the aligned 16-entry chunks covering it (one
// uint4 of pixel indices and four float4 of weights per thread; entry k of
// the item at LDS slot (e0 & 15) + k).  LDS holds the tile, the entries and
// the segment ends (19.5 KB at K = 4: 8 workgroups per CU; with the partial
// slots staged too, 20.5 KB and 7 workgroups, 126-129 instead of 111-113 us at
// 4 x 2048^2 -- the slot is loaded from global memory ahead of each segment's
// sum instead; staging 3072 / 4096 entries instead of 2048, fewer boxes of
// several items but 6 / 5 workgroups: 134 / 150 us).  The sums take K lanes per segment
// (lane b: vector b; ~90 segments per box leave one lane per segment mostly
// idle), each in seg_sum4's four-lane order: per segment and vector the
// products and their order are los_fwd_items' (bitwise).  (Measured against
// one lane per segment: 125-130 vs 130-132 us at 4 x 2048^2, Newton-metric
// CG 4080-4092 vs 4113-4119 us per 7-RHS iteration; an XCD-contiguous box
// order measured slower, 156 us -- the dense middle boxes then load a few
// XCDs --, and a persistent grid that loads item i + G while summing item i
// slower still, 162-186 us, at 4-5 instead of 7 waves per SIMD.)
template <typename T, int K>
__global__ __launch_bounds__(256) void los_fwd_boxes(nft_los_plan p, const T* __restrict__ x,
                                                     const T* __restrict__ cs, double* __restrict__ part,
                                                     long long xs, int pk, long long css, int kv) {
#pragma clang fp contract(off)
  static_assert(K > 1, "one vector takes los_fwd_items");
  __shared__ __align__(16) double u[256][K];
  __shared__ __align__(16) float ew[LOS_CAP_F + 16];
  __shared__ __align__(16) unsigned char el[LOS_CAP_F + 16];
  // the item's segment ends and partial slots
  __shared__ int send[256];
  const BoxGeom g{p.H, p.W, p.bh, p.bw, p.nby, p.nbx};
  const int box = (int)blockIdx.x;
  if (box >= p.nbox) return;
  const int t = threadIdx.x;
  bool ok;
  const long long px = g.pixel(box, t, ok);
  double xv[K];
#pragma unroll
  for (int b = 0; b < K; ++b) {
    double v = 0.0;
    if (ok && b < kv) {
      v = (double)x[b * xs + px];
      if (cs) v *= (double)cs[b * css + px];
    }
    xv[b] = v;
  }
  const int bs0 = p.box_lptr[box], bs1 = p.box_lptr[box + 1];
  const int be0 = p.box_ent[box], be1 = p.box_ent[box + 1];
  const bool multi = (be1 - be0 > LOS_CAP_F) || (bs1 - bs0 > 256);
  int ci = 0, ci1 = 0;
  int s0 = bs0, s1 = bs1, e0 = be0, e1 = be1;
  if (multi) {
    ci = p.box_item[box];
    ci1 = p.box_item[box + 1];
    s1 = p.item_seg[ci + 1];
    e1 = p.item_ent[ci + 1];
  }
  for (bool first = true;; first = false) {
    const int n = e1 - e0;
    const int eo = e0 & 15;
    uint4 vl = make_uint4(0, 0, 0, 0);
    float4 vw[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) vw[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (16 * t < eo + n) {
      const long long c = (long long)(e0 - eo) + 16 * t;
      vl = *(const uint4*)(p.ent_loc + c);
#pragma unroll
      for (int j = 0; j < 4; ++j) vw[j] = *(const float4*)(p.ent_wf + c + 4 * j);
    }
    const int sq = s0 + t;  // segment t's end and slot (<= 256 per work item)
    const int sb = sq < s1 ? p.seg_ent[sq + 1] - e0 : 0;
    if (first) {
#pragma unroll
      for (int b = 0; b < K; ++b) u[t][b] = xv[b];
    } else {
      __syncthreads();  // the previous item's entries are read
    }
    if (16 * t < eo + n) {
      *(uint4*)(el + 16 * t) = vl;
#pragma unroll
      for (int j = 0; j < 4; ++j) *(float4*)(ew + 16 * t + 4 * j) = vw[j];
    }
    if (sq < s1) {
      send[t] = sb;
    }
    __syncthreads();
    // K lanes per segment, lane b summing vector b in the four-lane order of
    // seg_sum4 (bitwise its value)
    constexpr int SPR = 256 / K;
    const int b = t % K, ns = s1 - s0;
    for (int j = t / K; j < ns; j += SPR) {
      const int so_j = p.seg_slot[s0 + j];  // issued ahead of the sum, used by its store
      const int a = (j ? send[j - 1] : 0) + eo, e = send[j] + eo;
      double acc[4] = {0.0, 0.0, 0.0, 0.0};
      for (int k = a; k < e; k += 4) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (k + q < e) acc[q] = acc[q] + (double)ew[k + q] * u[el[k + q]][b];
      }
      if (b < kv) part[(long long)so_j * pk + b] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    }
    if (!multi || ++ci >= ci1) break;
    s0 = s1;
    e0 = e1;
    s1 = p.item_seg[ci + 1];
    e1 = p.item_ent[ci + 1];
  }
}

// one wave per line of sight, all K vectors: the line's slots (boxes
// ascending) hold K adjacent partials each; per vector a fixed-order sum
// (lane strides, then a shuffle tree).  qpart (optional): per workgroup and
// vector the sum over its 4 lines of t_l * y_l, t_l = (R (cs x))_l before
// the row scale -- the data-space quadratic form x . (cs R^T (rs' R cs x))
// of the sampling-metric middle (nft_los_forward_quad_batched)
template <typename T, int K>
__global__ __launch_bounds__(256) void los_fwd_reduce(nft_los_plan p, const double* __restrict__ part,
                                                      const T* __restrict__ rs, T* __restrict__ y, double scale,
                                                      long long ys, double* __restrict__ qpart,
                                                      long long qstride) {
  __shared__ double qs[4][LOS_KMAX];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long long l = (long long)blockIdx.x * 4 + w;
  const bool valid = l < p.nlos;
  double acc[LOS_KMAX];
#pragma unroll
  for (int v = 0; v < LOS_KMAX; ++v) acc[v] = 0.0;
  if (valid) {
    const int a = p.los_ptr[l], b = p.los_ptr[l + 1];
    for (int k = a + lane; k < b; k += 64) {
      const double* q = part + (long long)k * K;
#pragma unroll
      for (int v = 0; v < LOS_KMAX; ++v)
        if (v < K) acc[v] += q[v];
    }
  }
#pragma unroll
  for (int v = 0; v < LOS_KMAX; ++v) {
    if (v < K) {
      double s = acc[v];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
      if (lane == 0) {
        double yy = 0.0;
        if (valid) {
          yy = s * scale;
          if (rs) yy *= (double)rs[l];
          y[v * ys + l] = (T)yy;
        }
        if (qpart) qs[w][v] = valid ? s * (double)(T)yy : 0.0;
      }
    }
  }
  if (qpart) {
    __syncthreads();
    if (threadIdx.x < K) {
      const int v = threadIdx.x;
      qpart[v * qstride + blockIdx.x] = ((qs[0][v] + qs[1][v]) + qs[2][v]) + qs[3][v];
    }
  }
}

// The CG curvature fold (nft_fold_partials) carried by an adjoint launch as
// its first nrhs workgroups (nft_los_adjoint_fold): out[r * ostride] = the sum
// of part[r * nb + b] over b < nb in fold_wide's order -- 1024 thread-strided
// sums (here virtual thread q * 256 + t, q < 4), the 16 waves' shuffle trees,
// the wave totals in order -- so bitwise the separate launch.
struct LosFold {
  const double* part;
  double* out;
  long long ostride;
  int nb, nrhs;
};
__device__ __forceinline__ void los_fold_rhs(const LosFold& f, int r, double* sh) {
  const double* part = f.part + (long long)r * f.nb;
  const int t = threadIdx.x;
  double v[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    v[q] = 0.0;
    for (int b = q * 256 + t; b < f.nb; b += 1024) v[q] += part[b];
  }
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v[q] += __shfl_down(v[q], off, 64);
  if ((t & 63) == 0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) sh[q * 4 + (t >> 6)] = v[q];
  }
  __syncthreads();
  if (t == 0) {
    double s = 0.0;
    for (int w = 0; w < 16; ++w) s += sh[w];
    f.out[(long long)r * f.ostride] = s;
  }
}

// Batched over K vectors (template): the chunk's entries (line index +
// fp32 weight) are staged in LDS once; every pixel thread sums its run for
// all K vectors in registers from the per-vector line tables.  Per vector the
// products and their order are those of K = 1 (bitwise).
template <typename T, typename IDX, int K, bool VEC = false>
__global__ __launch_bounds__(256) void los_adj_boxes(nft_los_plan p, const IDX* __restrict__ lidx,
                                                     const T* __restrict__ yv, const T* __restrict__ cs,
                                                     const T* __restrict__ rs, T* __restrict__ out, double scale,
                                                     long long ys, long long os, long long rss, int kv,
                                                     LosFold fold) {
#pragma clang fp contract(off)
  constexpr int PER = LOS_CH_A / 256;
  // line table: 256 lines per vector cover every box of an 8-bit-index plan
  // (boxes with more lines read y from global memory); sized per K so that
  // K = 4 fits 8 workgroups per CU (18 KB of LDS instead of 28 KB)
  constexpr int YL = 256 * K < LOS_YL ? 256 * K : LOS_YL;
  __shared__ __align__(16) double yl[YL];
  // K == 1 uses ew as a double product buffer (LOS_CH_A doubles)
  __shared__ __align__(16) float ew[K == 1 ? 2 * LOS_CH_A : LOS_CH_A];
  __shared__ __align__(16) IDX el[K == 1 ? 1 : LOS_CH_A];
  const BoxGeom g{p.H, p.W, p.bh, p.bw, p.nby, p.nbx};
  if ((int)blockIdx.x < fold.nrhs) {  // the carried curvature fold (first workgroups)
    los_fold_rhs(fold, (int)blockIdx.x, yl);
    return;
  }
  const int box = (int)blockIdx.x - fold.nrhs, t = threadIdx.x;
  if (box >= p.nbox) return;
  const int l0 = p.box_lptr[box], nl = p.box_lptr[box + 1] - l0;
  // 16-entry chunks with 16-byte loads (box runs padded, box_ent_adj)
  constexpr bool vec = VEC && sizeof(IDX) == 1 && K > 1;
  const int* __restrict__ bent = p.box_ent_adj ? p.box_ent_adj : p.box_ent;
  const int e0 = bent[box], n = bent[box + 1] - e0;
  const unsigned short* off = p.pix_off + (size_t)box * 257;
  const int a = off[t], b = off[t + 1];
  // the pixel's row scales are loaded up front (off the tail of the block)
  bool ok;
  const long long px = g.pixel(box, t, ok);
  double rsv[K];
#pragma unroll
  for (int v = 0; v < K; ++v) rsv[v] = (rs && ok && v < kv) ? (double)rs[v * rss + px] : 1.0;
  // line table, line-major: yl[li * K + v]
  // the first chunk's entry loads go out before the line-table staging so the
  // two dependent load chains overlap
  int lv[PER];
  float wv[PER];
  uint4 vl = make_uint4(0, 0, 0, 0);
  float4 vw[4];
  auto vload = [&](int c0, int cn) {
    const int k = 16 * t;
#pragma unroll
    for (int j = 0; j < 4; ++j) vw[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    vl = make_uint4(0, 0, 0, 0);
    if (k < cn && k < LOS_CH_A) {
      vl = *(const uint4*)((const unsigned char*)lidx + e0 + c0 + k);
#pragma unroll
      for (int j = 0; j < 4; ++j) vw[j] = *(const float4*)(p.ent_wa + e0 + c0 + k + 4 * j);
    }
  };
  if constexpr (vec) {
    vload(0, min(LOS_CH_A, n));
  } else {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int k = t + i * 256;
      lv[i] = k < n ? (int)lidx[e0 + k] : 0;
      wv[i] = k < n ? p.ent_wa[e0 + k] : 0.f;
    }
  }
  const bool tab = nl * K <= YL;  // line values of this box (all vectors) cached in LDS
  if (tab) {
    for (int i = t; i < nl; i += 256) {
      const int li = p.box_lines[l0 + i];
      const double c = cs ? (double)cs[li] : 1.0;
#pragma unroll
      for (int v = 0; v < K; ++v) {
        double yy = v < kv ? (double)yv[v * ys + li] : 0.0;
        if (cs) yy *= c;
        yl[i * K + v] = yy;
      }
    }
  }
  double acc[K];
#pragma unroll
  for (int v = 0; v < K; ++v) acc[v] = 0.0;
  for (int c0 = 0; c0 < n; c0 += LOS_CH_A) {  // uniform over the block
    const int cn = min(LOS_CH_A, n - c0);
    if (c0 > 0 && vec) {
      if constexpr (vec) vload(c0, cn);
    } else if (c0 > 0) {
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int k = t + i * 256;
        lv[i] = k < cn ? (int)lidx[e0 + c0 + k] : 0;
        wv[i] = k < cn ? p.ent_wa[e0 + c0 + k] : 0.f;
      }
    }
    __syncthreads();  // previous chunk consumed (and line table written)
    const int lo = max(a, c0), hi = min(b, c0 + cn);
    if constexpr (K == 1) {
      // single vector: stage the products once (the float/index buffers
      // double as the product buffer)
      double* prod = (double*)ew;
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int k = t + i * 256;
        if (k < cn) {
          double yy;
          if (tab) {
            yy = yl[lv[i]];
          } else {
            const int gl = p.box_lines[l0 + lv[i]];
            yy = (double)yv[gl];
            if (cs) yy *= (double)cs[gl];
          }
          prod[k] = (double)wv[i] * yy;
        }
      }
      __syncthreads();
      for (int k = lo; k < hi; ++k) acc[0] += prod[k - c0];
      continue;
    }
    if constexpr (vec) {
      const int k = 16 * t;
      if (k < cn && k < LOS_CH_A) {
        *(uint4*)((unsigned char*)el + k) = vl;
#pragma unroll
        for (int j = 0; j < 4; ++j) *(float4*)(ew + k + 4 * j) = vw[j];
      }
    } else {
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int k = t + i * 256;
        if (k < cn) {
          ew[k] = wv[i];
          el[k] = (IDX)lv[i];
        }
      }
    }
    __syncthreads();
    for (int k = lo; k < hi; ++k) {
      const double w = (double)ew[k - c0];
      const int li = el[k - c0];
      if (tab) {
#pragma unroll
        for (int v = 0; v < K; ++v) acc[v] = acc[v] + w * yl[li * K + v];
      } else {
        const int gl = p.box_lines[l0 + li];
        const double cc = cs ? (double)cs[gl] : 1.0;
#pragma unroll
        for (int v = 0; v < K; ++v) {
          double yy = v < kv ? (double)yv[v * ys + gl] : 0.0;
          if (cs) yy *= cc;
          acc[v] = acc[v] + w * yy;
        }
      }
    }
  }
  if (ok) {
    // pixel-side scale: shared by the vectors (rss = 0) or one per vector
#pragma unroll
    for (int v = 0; v < K; ++v) {
      double o = acc[v] * scale;
      if (rs) o *= rsv[v];
      if (v < kv) out[v * os + px] = (T)o;
    }
  }
}

template <typename T, int K>
static void fwd_items_k(const nft_los_plan* p, const T* x, const T* cs, double* part, long long xs, int pk,
                        long long css, int kv, hipStream_t s) {
  if constexpr (K > 1) {
    if (p->box_item) {
      hipLaunchKernelGGL((los_fwd_boxes<T, K>), dim3((unsigned)p->nbox), dim3(256), 0, s, *p, x, cs, part, xs, pk,
                         css, kv);
      return;
    }
  }
  hipLaunchKernelGGL((los_fwd_items<T, K>), dim3((unsigned)p->nitems), dim3(256), 0, s, *p, x, cs, part, xs, pk, css,
                     kv);
}

template <typename T, typename IDX, int K>
static void adj_boxes_k(const nft_los_plan* p, const IDX* li, const T* y, const T* cs, const T* rs, T* out,
                        double scale, long long ys, long long os, long long rss, int kv, hipStream_t s,
                        const LosFold& fold) {
  const dim3 grid((unsigned)(p->nbox + fold.nrhs));
  if constexpr (K > 1 && sizeof(IDX) == 1) {
    if (p->box_ent_adj) {
      hipLaunchKernelGGL((los_adj_boxes<T, IDX, K, true>), grid, dim3(256), 0, s, *p, li, y, cs, rs, out, scale, ys, os,
                         rss, kv, fold);
      return;
    }
  }
  hipLaunchKernelGGL((los_adj_boxes<T, IDX, K>), grid, dim3(256), 0, s, *p, li, y, cs, rs, out, scale, ys, os, rss,
                     kv, fold);
}

// vectors are processed in groups of 8 / 4 / 2 / 1 (template sizes); a
// remainder of 5-7 (3) vectors takes ONE launch of the 8 (4) instance with
// the missing vectors masked (kv valid), not 4 + 2 + 1 launches that each
// stream the whole matrix (the geoVI Newton metrics' batches shrink through
// every count as samples finish).  Per vector the arithmetic does not depend
// on the instance (bitwise).
// (Two launches of the 4 instance for 5-8 vectors, whose 19.5 KB of LDS
// allow 8 workgroups per CU against 5 for the 8 instance: Newton-metric CG
// 4175 vs 4101 us per 7-RHS iteration, 4692 vs 4572 at 8 -- one launch kept.)
static int kgroup(int k) { return k >= 5 ? 8 : (k >= 3 ? 4 : (k == 2 ? 2 : 1)); }

template <typename T>
static int los_forward_t(const nft_los_plan* p, const void* x, const void* cs, const void* rs, void* y, double* part,
                         double scale, int K, long long xs, long long ys, hipStream_t s, double* qpart = nullptr,
                         long long qstride = 0, long long css = 0) {
  prof_mark(s, "los_fwd_items");
  if (p->nitems > 0) {
    for (int v = 0; v < K;) {
      const int g = kgroup(K - v), kv = std::min(g, K - v);
      const T* xv = (const T*)x + v * xs;
      const T* cv = cs ? (const T*)cs + v * css : nullptr;
      double* pv = part + v;  // slot-major partials, K per slot
      switch (g) {
        case 8: fwd_items_k<T, 8>(p, xv, cv, pv, xs, K, css, kv, s); break;
        case 4: fwd_items_k<T, 4>(p, xv, cv, pv, xs, K, css, kv, s); break;
        case 2: fwd_items_k<T, 2>(p, xv, cv, pv, xs, K, css, kv, s); break;
        default: fwd_items_k<T, 1>(p, xv, cv, pv, xs, K, css, 1, s); break;
      }
      v += kv;
    }
  }
  prof_mark(s, "los_fwd_reduce");
  if (p->nlos > 0) {
    const dim3 grid((unsigned)((p->nlos + 3) / 4));
#define NFT_RED(KK)                                                                                          \
  case KK:                                                                                                   \
    hipLaunchKernelGGL((los_fwd_reduce<T, KK>), grid, dim3(256), 0, s, *p, part, (const T*)rs, (T*)y, scale, \
                       ys, qpart, qstride);                                                                  \
    break;
    switch (K) {
      NFT_RED(1) NFT_RED(2) NFT_RED(3) NFT_RED(4) NFT_RED(5) NFT_RED(6) NFT_RED(7) NFT_RED(8)
      default: break;
    }
#undef NFT_RED
  }
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

template <typename T, typename IDX>
static void los_adjoint_idx(const nft_los_plan* p, const IDX* li, const void* y, const void* cs, const void* rs,
                            void* out, double scale, int K, long long ys, long long os, hipStream_t s,
                            long long rss = 0, const LosFold* fold = nullptr) {
  const LosFold none{nullptr, nullptr, 0, 0, 0};
  for (int v = 0; v < K;) {
    const int g = kgroup(K - v), kv = std::min(g, K - v);
    const T* yv = (const T*)y + v * ys;
    const T* rv = rs ? (const T*)rs + v * rss : nullptr;
    T* ov = (T*)out + v * os;
    const LosFold& fv = (v == 0 && fold) ? *fold : none;  // the first launch carries it
    switch (g) {
      case 8: adj_boxes_k<T, IDX, 8>(p, li, yv, (const T*)cs, rv, ov, scale, ys, os, rss, kv, s, fv); break;
      case 4: adj_boxes_k<T, IDX, 4>(p, li, yv, (const T*)cs, rv, ov, scale, ys, os, rss, kv, s, fv); break;
      case 2: adj_boxes_k<T, IDX, 2>(p, li, yv, (const T*)cs, rv, ov, scale, ys, os, rss, kv, s, fv); break;
      default: adj_boxes_k<T, IDX, 1>(p, li, yv, (const T*)cs, rv, ov, scale, ys, os, rss, 1, s, fv); break;
    }
    v += kv;
  }
}

template <typename T>
static int los_adjoint_t(const nft_los_plan* p, const void* y, const void* cs, const void* rs, void* out, double scale,
                         int K, long long ys, long long os, hipStream_t s, long long rss = 0,
                         const LosFold* fold = nullptr) {
  if (p->nbox <= 0) return NFT_OK;
  prof_mark(s, "los_adj_boxes");
  if (p->lidx8)
    los_adjoint_idx<T, unsigned char>(p, (const unsigned char*)p->ent_lidx, y, cs, rs, out, scale, K, ys, os, s, rss,
                                      fold);
  else
    los_adjoint_idx<T, unsigned short>(p, (const unsigned short*)p->ent_lidx, y, cs, rs, out, scale, K, ys, os, s,
                                       rss, fold);
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

static int check_plan(const nft_los_plan* p) {
  if (!p || p->bh * p->bw != 256 || p->nbx <= 0 || p->nby <= 0) {
    set_last_error("nft_los: invalid plan (boxes must hold 256 pixels)");
    return NFT_ERR_ARG;
  }
  return NFT_OK;
}

}  // namespace nft

using namespace nft;

extern "C" {

size_t nft_los_workspace(const nft_los_plan* p) { return (size_t)(p ? p->nseg : 0) * sizeof(double) + 256; }

int nft_los_forward_batched(const nft_los_plan* p, const void* x, const void* colscale, const void* rowscale,
                            void* y, void* ws, int dtype, double scale, int nvec, int64_t x_stride,
                            int64_t y_stride, hipStream_t stream) {
  int st = check_plan(p);
  if (st != NFT_OK) return st;
  if (nvec < 1 || nvec > LOS_KMAX) {
    set_last_error("nft_los_forward: 1 <= nvec <= %d", LOS_KMAX);
    return NFT_ERR_ARG;
  }
  if (dtype == 0)
    return los_forward_t<double>(p, x, colscale, rowscale, y, (double*)ws, scale, nvec, x_stride, y_stride, stream);
  if (dtype == 1)
    return los_forward_t<float>(p, x, colscale, rowscale, y, (double*)ws, scale, nvec, x_stride, y_stride, stream);
  set_last_error("nft_los_forward: bad dtype %d", dtype);
  return NFT_ERR_ARG;
}

int nft_los_quad_blocks(const nft_los_plan* p) { return p ? (int)((p->nlos + 3) / 4) : 0; }

int nft_los_forward_quad_batched(const nft_los_plan* p, const void* x, const void* colscale, const void* rowscale,
                                 void* y, void* ws, int dtype, double scale, int nvec, int64_t x_stride,
                                 int64_t y_stride, double* qpart, int64_t qstride, hipStream_t stream) {
  int st = check_plan(p);
  if (st != NFT_OK) return st;
  if (nvec < 1 || nvec > LOS_KMAX || !qpart || qstride < nft_los_quad_blocks(p)) {
    set_last_error("nft_los_forward_quad: 1 <= nvec <= %d, qpart with qstride >= nft_los_quad_blocks", LOS_KMAX);
    return NFT_ERR_ARG;
  }
  if (dtype == 0)
    return los_forward_t<double>(p, x, colscale, rowscale, y, (double*)ws, scale, nvec, x_stride, y_stride, stream,
                                 qpart, qstride);
  if (dtype == 1)
    return los_forward_t<float>(p, x, colscale, rowscale, y, (double*)ws, scale, nvec, x_stride, y_stride, stream,
                                qpart, qstride);
  set_last_error("nft_los_forward_quad: bad dtype %d", dtype);
  return NFT_ERR_ARG;
}

int nft_los_forward(const nft_los_plan* p, const void* x, const void* colscale, const void* rowscale, void* y,
                    void* ws, int dtype, double scale, hipStream_t stream) {
  return nft_los_forward_batched(p, x, colscale, rowscale, y, ws, dtype, scale, 1, 0, 0, stream);
}

int nft_los_adjoint_batched(const nft_los_plan* p, const void* y, const void* colscale, const void* rowscale,
                            void* out, int dtype, double scale, int nvec, int64_t y_stride, int64_t out_stride,
                            hipStream_t stream) {
  int st = check_plan(p);
  if (st != NFT_OK) return st;
  if (nvec < 1 || nvec > LOS_KMAX) {
    set_last_error("nft_los_adjoint: 1 <= nvec <= %d", LOS_KMAX);
    return NFT_ERR_ARG;
  }
  if (dtype == 0)
    return los_adjoint_t<double>(p, y, colscale, rowscale, out, scale, nvec, y_stride, out_stride, stream);
  if (dtype == 1)
    return los_adjoint_t<float>(p, y, colscale, rowscale, out, scale, nvec, y_stride, out_stride, stream);
  set_last_error("nft_los_adjoint: bad dtype %d", dtype);
  return NFT_ERR_ARG;
}

int nft_los_adjoint_fold(const nft_los_plan* p, const void* y, const void* colscale, const void* rowscale, void* out,
                         int dtype, double scale, int nvec, int64_t y_stride, int64_t out_stride,
                         const double* fold_part, int fold_nb, int fold_nrhs, double* fold_out, int64_t fold_ostride,
                         hipStream_t stream) {
  int st = check_plan(p);
  if (st != NFT_OK) return st;
  if (nvec < 1 || nvec > LOS_KMAX || p->nbox <= 0 || !fold_part || !fold_out || fold_nb < 1 || fold_nrhs < 1 ||
      fold_ostride < 1) {
    set_last_error("nft_los_adjoint_fold: 1 <= nvec <= %d, a non-empty plan and fold partials / output", LOS_KMAX);
    return NFT_ERR_ARG;
  }
  const LosFold f{fold_part, fold_out, (long long)fold_ostride, fold_nb, fold_nrhs};
  if (dtype == 0)
    return los_adjoint_t<double>(p, y, colscale, rowscale, out, scale, nvec, y_stride, out_stride, stream, 0, &f);
  if (dtype == 1)
    return los_adjoint_t<float>(p, y, colscale, rowscale, out, scale, nvec, y_stride, out_stride, stream, 0, &f);
  set_last_error("nft_los_adjoint_fold: bad dtype %d", dtype);
  return NFT_ERR_ARG;
}

int nft_los_adjoint(const nft_los_plan* p, const void* y, const void* colscale, const void* rowscale, void* out,
                    int dtype, double scale, hipStream_t stream) {
  return nft_los_adjoint_batched(p, y, colscale, rowscale, out, dtype, scale, 1, 0, 0, stream);
}

int nft_los_forward_ex(const nft_los_plan* p, const void* x, const void* colscale, int64_t colscale_stride,
                       const void* rowscale, void* y, void* ws, int dtype, double scale, int nvec, int64_t x_stride,
                       int64_t y_stride, double* qpart, int64_t qstride, hipStream_t stream) {
  int st = check_plan(p);
  if (st != NFT_OK) return st;
  if (nvec < 1 || nvec > LOS_KMAX || colscale_stride < 0 || (qpart && qstride < nft_los_quad_blocks(p))) {
    set_last_error("nft_los_forward_ex: 1 <= nvec <= %d, colscale_stride >= 0, qstride >= nft_los_quad_blocks",
                   LOS_KMAX);
    return NFT_ERR_ARG;
  }
  if (dtype == 0)
    return los_forward_t<double>(p, x, colscale, rowscale, y, (double*)ws, scale, nvec, x_stride, y_stride, stream,
                                 qpart, qstride, colscale_stride);
  if (dtype == 1)
    return los_forward_t<float>(p, x, colscale, rowscale, y, (double*)ws, scale, nvec, x_stride, y_stride, stream,
                                qpart, qstride, colscale_stride);
  set_last_error("nft_los_forward_ex: bad dtype %d", dtype);
  return NFT_ERR_ARG;
}

int nft_los_adjoint_ex(const nft_los_plan* p, const void* y, const void* colscale, const void* rowscale,
                       int64_t rowscale_stride, void* out, int dtype, double scale, int nvec, int64_t y_stride,
                       int64_t out_stride, hipStream_t stream) {
  int st = check_plan(p);
  if (st != NFT_OK) return st;
  if (nvec < 1 || nvec > LOS_KMAX || rowscale_stride < 0) {
    set_last_error("nft_los_adjoint_ex: 1 <= nvec <= %d, rowscale_stride >= 0", LOS_KMAX);
    return NFT_ERR_ARG;
  }
  if (dtype == 0)
    return los_adjoint_t<double>(p, y, colscale, rowscale, out, scale, nvec, y_stride, out_stride, stream,
                                 rowscale_stride);
  if (dtype == 1)
    return los_adjoint_t<float>(p, y, colscale, rowscale, out, scale, nvec, y_stride, out_stride, stream,
                                rowscale_stride);
  set_last_error("nft_los_adjoint_ex: bad dtype %d", dtype);
  return NFT_ERR_ARG;
}

}  // extern "C"
