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
//        partial goes to its slot in LOS-major order.
//    K2 (one wave per line of sight): fixed-order sum of its partials.
//  adjoint  out = rs * R^T (cs * y):
//    K3 (one workgroup per box): the values cs*y of the ~100 lines crossing
//        the box are cached in LDS once; w * y[line] for the box's entries
//        (sorted by local pixel, storage order within a pixel; 8-bit line
//        index + fp32 weight) is staged in LDS chunk by chunk and thread t
//        sums pixel t's run; the box tile is written coalesced.
//
// All reductions run in a fixed order: deterministic, no atomics.
#include "nft_api_internal.hpp"

namespace nft {

constexpr int LOS_CAP_F = 2048;  // entries per forward work item (host-guaranteed)
constexpr int LOS_CH_A = 2048;   // adjoint: entries staged in LDS per chunk
constexpr int LOS_LMAX = 1024;   // adjoint: lines per box cached in LDS

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

template <typename T>
__global__ __launch_bounds__(256) void los_fwd_items(nft_los_plan p, const T* __restrict__ x,
                                                     const T* __restrict__ cs, double* __restrict__ part) {
  constexpr int PER = LOS_CAP_F / 256;
  __shared__ double u[256];
  __shared__ double prod[LOS_CAP_F];
  const BoxGeom g{p.H, p.W, p.bh, p.bw, p.nby, p.nbx};
  const int it = blockIdx.x, t = threadIdx.x;
  const int box = p.item_box[it];
  bool ok;
  const long long px = g.pixel(box, t, ok);
  double v = 0.0;
  if (ok) {
    v = (double)x[px];
    if (cs) v *= (double)cs[px];
  }
  u[t] = v;
  const int s0 = p.item_seg[it], s1 = p.item_seg[it + 1];
  const int e0 = p.item_ent[it], e1 = p.item_ent[it + 1];
  const int n = e1 - e0;
  const bool staged = n <= LOS_CAP_F;  // host plans always fit; others take the direct path
  float wv[PER];
  int lv[PER];
  if (staged) {
    // issue every entry load of this thread before the tile is needed
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int k = t + i * 256;
      wv[i] = k < n ? p.ent_wf[e0 + k] : 0.f;
      lv[i] = k < n ? p.ent_loc[e0 + k] : 0;
    }
  }
  // four lanes per segment; the first segment's bounds are loaded early too
  const int sub = t & 3;
  int s = s0 + (t >> 2);
  int sa = 0, sb = 0, slot = 0;
  if (s < s1) {
    sa = p.seg_ent[s] - e0;
    sb = p.seg_ent[s + 1] - e0;
    slot = p.seg_slot[s];
  }
  __syncthreads();
  if (staged) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int k = t + i * 256;
      if (k < n) prod[k] = (double)wv[i] * u[lv[i]];
    }
  }
  __syncthreads();
  // strided partial sums + fixed xor-tree per segment
  while (s < s1) {
    double acc = 0.0;
    if (staged) {
      for (int k = sa + sub; k < sb; k += 4) acc += prod[k];
    } else {
      for (int k = sa + sub; k < sb; k += 4) acc += (double)p.ent_wf[e0 + k] * u[p.ent_loc[e0 + k]];
    }
    acc += __shfl_xor(acc, 1, 64);
    acc += __shfl_xor(acc, 2, 64);
    if (sub == 0) part[slot] = acc;
    s += 64;
    if (s < s1) {
      sa = p.seg_ent[s] - e0;
      sb = p.seg_ent[s + 1] - e0;
      slot = p.seg_slot[s];
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void los_fwd_reduce(nft_los_plan p, const double* __restrict__ part,
                                                      const T* __restrict__ rs, T* __restrict__ y, double scale) {
  const int lane = threadIdx.x & 63;
  const long long l = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (l >= p.nlos) return;
  const int a = p.los_ptr[l], b = p.los_ptr[l + 1];
  double acc = 0.0;
  for (int k = a + lane; k < b; k += 64) acc += part[k];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
  if (lane == 0) {
    acc *= scale;
    if (rs) acc *= (double)rs[l];
    y[l] = (T)acc;
  }
}

template <typename T, typename IDX>
__global__ __launch_bounds__(256) void los_adj_boxes(nft_los_plan p, const IDX* __restrict__ lidx,
                                                     const T* __restrict__ yv, const T* __restrict__ cs,
                                                     const T* __restrict__ rs, T* __restrict__ out, double scale) {
  constexpr int PER = LOS_CH_A / 256;
  __shared__ double yl[LOS_LMAX];
  __shared__ double prod[LOS_CH_A];
  const BoxGeom g{p.H, p.W, p.bh, p.bw, p.nby, p.nbx};
  const int box = blockIdx.x, t = threadIdx.x;
  const int l0 = p.box_lptr[box], nl = p.box_lptr[box + 1] - l0;
  const int e0 = p.box_ent[box], n = p.box_ent[box + 1] - e0;
  const unsigned short* off = p.pix_off + (size_t)box * 257;
  const int a = off[t], b = off[t + 1];
  // the first chunk's entry loads go out before the line-table staging so the
  // two dependent load chains overlap
  int lv[PER];
  float wv[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int k = t + i * 256;
    lv[i] = k < n ? (int)lidx[e0 + k] : 0;
    wv[i] = k < n ? p.ent_wa[e0 + k] : 0.f;
  }
  const bool tab = nl <= LOS_LMAX;  // line values of this box cached in LDS
  if (tab) {
    for (int i = t; i < nl; i += 256) {
      const int li = p.box_lines[l0 + i];
      double v = (double)yv[li];
      if (cs) v *= (double)cs[li];
      yl[i] = v;
    }
  }
  double acc = 0.0;
  for (int c0 = 0; c0 < n; c0 += LOS_CH_A) {  // uniform over the block
    const int cn = min(LOS_CH_A, n - c0);
    if (c0 > 0) {
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int k = t + i * 256;
        lv[i] = k < cn ? (int)lidx[e0 + c0 + k] : 0;
        wv[i] = k < cn ? p.ent_wa[e0 + c0 + k] : 0.f;
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int k = t + i * 256;
      if (k < cn) {
        double yy;
        if (tab) {
          yy = yl[lv[i]];
        } else {
          const int li = p.box_lines[l0 + lv[i]];
          yy = (double)yv[li];
          if (cs) yy *= (double)cs[li];
        }
        prod[k] = (double)wv[i] * yy;
      }
    }
    __syncthreads();
    const int lo = max(a, c0), hi = min(b, c0 + cn);
    for (int k = lo; k < hi; ++k) acc += prod[k - c0];
  }
  bool ok;
  const long long px = g.pixel(box, t, ok);
  if (ok) {
    acc *= scale;
    if (rs) acc *= (double)rs[px];
    out[px] = (T)acc;
  }
}

template <typename T>
static int los_forward_t(const nft_los_plan* p, const void* x, const void* cs, const void* rs, void* y, double* part,
                         double scale, hipStream_t s) {
  prof_mark(s, "los_fwd_items");
  if (p->nitems > 0)
    hipLaunchKernelGGL(los_fwd_items<T>, dim3((unsigned)p->nitems), dim3(256), 0, s, *p, (const T*)x, (const T*)cs,
                       part);
  prof_mark(s, "los_fwd_reduce");
  if (p->nlos > 0)
    hipLaunchKernelGGL(los_fwd_reduce<T>, dim3((unsigned)((p->nlos + 3) / 4)), dim3(256), 0, s, *p, part,
                       (const T*)rs, (T*)y, scale);
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

template <typename T>
static int los_adjoint_t(const nft_los_plan* p, const void* y, const void* cs, const void* rs, void* out, double scale,
                         hipStream_t s) {
  if (p->nbox <= 0) return NFT_OK;
  prof_mark(s, "los_adj_boxes");
  if (p->lidx8)
    hipLaunchKernelGGL((los_adj_boxes<T, unsigned char>), dim3((unsigned)p->nbox), dim3(256), 0, s, *p,
                       (const unsigned char*)p->ent_lidx, (const T*)y, (const T*)cs, (const T*)rs, (T*)out, scale);
  else
    hipLaunchKernelGGL((los_adj_boxes<T, unsigned short>), dim3((unsigned)p->nbox), dim3(256), 0, s, *p,
                       (const unsigned short*)p->ent_lidx, (const T*)y, (const T*)cs, (const T*)rs, (T*)out, scale);
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

int nft_los_forward(const nft_los_plan* p, const void* x, const void* colscale, const void* rowscale, void* y,
                    void* ws, int dtype, double scale, hipStream_t stream) {
  int st = check_plan(p);
  if (st != NFT_OK) return st;
  if (dtype == 0) return los_forward_t<double>(p, x, colscale, rowscale, y, (double*)ws, scale, stream);
  if (dtype == 1) return los_forward_t<float>(p, x, colscale, rowscale, y, (double*)ws, scale, stream);
  set_last_error("nft_los_forward: bad dtype %d", dtype);
  return NFT_ERR_ARG;
}

int nft_los_adjoint(const nft_los_plan* p, const void* y, const void* colscale, const void* rowscale, void* out,
                    int dtype, double scale, hipStream_t stream) {
  int st = check_plan(p);
  if (st != NFT_OK) return st;
  if (dtype == 0) return los_adjoint_t<double>(p, y, colscale, rowscale, out, scale, stream);
  if (dtype == 1) return los_adjoint_t<float>(p, y, colscale, rowscale, out, scale, stream);
  set_last_error("nft_los_adjoint: bad dtype %d", dtype);
  return NFT_ERR_ARG;
}

}  // extern "C"
