#include <algorithm>
// Power-bin gather / scatter (PowerDistributor) for gfx950.
//
//   nft_bin_gather   out[p, i, q] = in[p, pindex[i], q]
//                    == DOFDistributor._times, src/operators/distributors.py:114-119
//   nft_bin_scatter  out[p, b, q] = sum_{i: pindex[i]==b} in[p, i, q]
//                    == DOFDistributor._adjoint_times + utilities.special_add_at
//                    (np.bincount), distributors.py:105-112, utilities.py:223-242
//
// The scatter is a segmented reduction over a precomputed stable bin->pixel
// permutation (CSR: perm, offsets).  Each (p, b, q) is summed by one thread in
// ascending pixel order, i.e. in exactly the order np.bincount accumulates, so
// the result is bitwise identical to the reference and run-to-run
// deterministic (no float atomics).
#include <cstdlib>

#include "nft_api_internal.hpp"

namespace nft {

template <typename T>
__global__ void bin_gather_kernel(const T* __restrict__ in, const int* __restrict__ pindex,
                                  T* __restrict__ out, long long pre, long long npix, long long nbins,
                                  long long post) {
  const long long tot = pre * npix * post;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += stride) {
    long long q = e % post;
    long long t = e / post;
    long long i = t % npix;
    long long p = t / npix;
    out[e] = in[(p * nbins + pindex[i]) * post + q];
  }
}

template <typename T>
__global__ void bin_scatter_kernel(const T* __restrict__ in, const int* __restrict__ perm,
                                   const int* __restrict__ offs, T* __restrict__ out, long long pre,
                                   long long npix, long long nbins, long long post) {
  const long long tot = pre * nbins * post;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += stride) {
    long long q = e % post;
    long long t = e / post;
    long long b = t % nbins;
    long long p = t / nbins;
    const T* src = in + p * npix * post + q;
    T acc = (T)0;
    for (int j = offs[b]; j < offs[b + 1]; ++j) acc += src[(long long)perm[j] * post];
    out[e] = acc;
  }
}

// pre == post == 1: element-parallel gather + per-bin sums.  Block c owns the
// sorted positions [c*BS_CH, (c+1)*BS_CH) and every bin that starts there; it
// gathers in[perm[j]] for its range with all loads in flight (the per-bin
// thread loop above is a chain of dependent random loads), stages them in LDS
// and sums each bin sequentially in ascending j (np.bincount order, bit-exact);
// a bin running past the chunk end reads its tail from global memory.
//
// XCD-aware chunk order: workgroups are dealt to the 8 XCDs round-robin, so
// workgroup w processes chunk (w % 8) * per + w / 8 -- each XCD walks one
// contiguous range of sorted positions, i.e. one annulus of the k-plane, and
// its random reads stay inside a working set that fits its own 4 MB L2
// instead of every XCD touching every cache line of the input.
constexpr int BS_CH = 2048;
constexpr int NXCD = 8;

//
// Pixel-ordered chunk gathers (gpix / gslot non-null): the entries of a chunk
// are loaded in ascending pixel order -- a chunk holds one thin annulus of the
// k-plane, crossed by each grid row in a few short runs, so consecutive lanes
// read nearby addresses instead of one cache line each -- and stored to their
// bin-sorted LDS slot; the per-bin sums are unchanged (bitwise).
//
// LW (the mirror-folded bins of the CF Jacobian adjoint, nft_bin_scatter_folded):
// bins of more than 64 positions are summed one wave each exactly as
// bin_scatter_il sums them (lane-strided partials, then the shuffle tree), so
// the planar and the interleaved folded sums agree bitwise for every item
// count; without LW every bin is one thread's ascending chain (np.bincount's
// order, the PowerDistributor's bit-exact adjoint).
template <typename T, int K, bool LW = false>
__global__ __launch_bounds__(256) void bin_scatter_chunk(const T* __restrict__ in, const int* __restrict__ perm,
                                                         const int* __restrict__ offs,
                                                         const int* __restrict__ gpix,
                                                         const unsigned short* __restrict__ gslot,
                                                         const int* __restrict__ cbins,
                                                         T* __restrict__ out, long long npix, long long nbins,
                                                         int nchunks) {
  // K inputs (items of the batch) per workgroup: perm, the chunk bounds and
  // the bin offsets are loaded once for all of them, and every lane keeps
  // K * PER gathers in flight.  With precomputed chunk bounds the bin
  // offsets are loaded before the barrier too (off the critical path).
  constexpr int PER = BS_CH / 256;
  constexpr int BPT = 2;  // bins per thread handled with prefetched offsets
  constexpr int LONGB = 64;
  __shared__ T vals[K][BS_CH];
  __shared__ int bnd[2];
  __shared__ int nlong;
  __shared__ int longb[LW ? BS_CH / LONGB + 1 : 1];
  const int per = (nchunks + NXCD - 1) / NXCD;
  const int c = (int)(blockIdx.x % NXCD) * per + (int)(blockIdx.x / NXCD);
  if (c >= nchunks) return;
  in += (long long)blockIdx.y * K * npix;  // batch of inputs sharing the binning (pre axis)
  out += (long long)blockIdx.y * K * nbins;
  const long long j0 = (long long)c * BS_CH;
  const int t = threadIdx.x;
  const int n = (int)(npix - j0 < BS_CH ? npix - j0 : BS_CH);
  int b0 = 0, b1 = 0;
  long long oa[BPT], oe[BPT];
  if (cbins) {
    b0 = cbins[c];
    b1 = cbins[c + 1];
#pragma unroll
    for (int q = 0; q < BPT; ++q) {
      const int bq = b0 + t + q * 256;
      oa[q] = bq < b1 ? offs[bq] : 0;
      oe[q] = bq < b1 ? offs[bq + 1] : 0;
    }
  }
  int pv[PER], sl[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int e = t + i * 256;
    pv[i] = e < n ? (gpix ? gpix[j0 + e] : perm[j0 + e]) : 0;
    sl[i] = gpix ? (e < n ? (int)gslot[j0 + e] : 0) : e;
  }
  T v[K][PER];
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int i = 0; i < PER; ++i) v[k][i] = t + i * 256 < n ? in[k * npix + pv[i]] : (T)0;
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int i = 0; i < PER; ++i)
      if (t + i * 256 < n) vals[k][sl[i]] = v[k][i];
  if (LW && t == 0) nlong = 0;
  if (!cbins && t < 2) {
    // first bin whose start offset is >= j0 (+ BS_CH)
    const long long target = j0 + (t ? BS_CH : 0);
    long long lo = 0, hi = nbins;  // search in offs[0..nbins)
    while (lo < hi) {
      const long long mid = (lo + hi) >> 1;
      if ((long long)offs[mid] < target) lo = mid + 1;
      else hi = mid;
    }
    // the last chunk also owns trailing empty bins (start offset == npix)
    bnd[t] = (t && j0 + BS_CH >= npix) ? (int)nbins : (int)lo;
  }
  __syncthreads();
  if (!cbins) {
    b0 = bnd[0];
    b1 = bnd[1];
  }
  for (int q = 0, b = b0 + t; b < b1; ++q, b += 256) {
    long long a, e;
    if (cbins && q < BPT) {  // prefetched above (same b, b < b1)
      a = oa[q];
      e = oe[q];
    } else {
      a = offs[b];
      e = offs[b + 1];
    }
    if (LW && e - a > LONGB) {
      longb[atomicAdd(&nlong, 1)] = b;  // list order is irrelevant: one bin per entry
      continue;
    }
    T acc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = (T)0;
    for (long long j = a; j < e; ++j) {
      if (j - j0 < BS_CH) {
#pragma unroll
        for (int k = 0; k < K; ++k) acc[k] += vals[k][j - j0];
      } else {
        const int p = perm[j];
#pragma unroll
        for (int k = 0; k < K; ++k) acc[k] += in[k * npix + p];
      }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) out[k * nbins + b] = acc[k];
  }
  if constexpr (LW) {
    __syncthreads();
    const int w = t >> 6, lane = t & 63;
    for (int i = w; i < nlong; i += 4) {
      const int b = longb[i];
      const long long a = offs[b], e = offs[b + 1];
      T acc[K];
#pragma unroll
      for (int k = 0; k < K; ++k) acc[k] = (T)0;
      for (long long j = a + lane; j < e; j += 64) {
        if (j - j0 < BS_CH) {
#pragma unroll
          for (int k = 0; k < K; ++k) acc[k] += vals[k][j - j0];
        } else {
          const int p = perm[j];
#pragma unroll
          for (int k = 0; k < K; ++k) acc[k] += in[k * npix + p];
        }
      }
#pragma unroll
      for (int k = 0; k < K; ++k) {
        T v = acc[k];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
        if (lane == 0) out[k * nbins + b] = v;
      }
    }
  }
}


// Mirror fold of a harmonic-grid array (pre, n_0, ..., n_{d-1}) onto its
// fundamental cell (pre, h_0, ..., h_{d-1}), h_a = n_a/2 + 1:
//   out[p, q] = sum over the distinct mirror images i of q (i_a = q_a or
//               n_a - q_a) of in[p, i]
// |k| -- hence the power bin -- is invariant under k_a -> -k_a on every axis
// (RGSpace.get_k_length_array, rg_space.py:101-121), so the bin sums of the
// grid equal the bin sums of the folded cell (2^d fewer scattered gathers).
// Each output sums its <= 2^d images in a fixed order (deterministic); the
// last axis is the fastest thread index: the reads of q and n - q are two
// coalesced runs (one ascending, one descending).
constexpr int FOLD_MAXD = 3;
struct FoldShape {
  int d;
  long long n[FOLD_MAXD], h[FOLD_MAXD];
  long long nin, nout;  // elements per pre item
};

// fold from point-mirror pair sums on the half grid (last axis h = n/2+1):
// the sign flips of the first d-1 axes only, in the order of bin_fold_kernel
template <typename T>
__global__ __launch_bounds__(256) void bin_fold_half_kernel(const T* __restrict__ in, T* __restrict__ out,
                                                            FoldShape fs, long long pre, long long nhalf) {
  const long long tot = pre * fs.nout;
  const int D = fs.d;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < tot;
       e += (long long)gridDim.x * blockDim.x) {
    long long r = e % fs.nout;
    const long long p = e / fs.nout;
    long long q[FOLD_MAXD], m[FOLD_MAXD];
    bool two[FOLD_MAXD];
#pragma unroll
    for (int a = FOLD_MAXD - 1; a >= 0; --a) {
      if (a < D) {
        q[a] = r % fs.h[a];
        r /= fs.h[a];
        m[a] = fs.n[a] - q[a];
        two[a] = q[a] != 0 && m[a] != q[a];
      } else {
        q[a] = m[a] = 0;
        two[a] = false;
      }
    }
    const T* src = in + p * nhalf;
    T acc = (T)0;
#pragma unroll
    for (int s = 0; s < (1 << (FOLD_MAXD - 1)); ++s) {
      bool ok = true;
      long long idx = 0;
#pragma unroll
      for (int a = 0; a < FOLD_MAXD; ++a) {
        if (a >= D) continue;
        if (a == D - 1) {           // the half axis: no flip
          idx = idx * fs.h[a] + q[a];
          continue;
        }
        const bool hi = (s >> (FOLD_MAXD - 2 - a)) & 1;
        ok = ok && (!hi || two[a]);
        idx = idx * fs.n[a] + (hi ? m[a] : q[a]);
      }
      // patterns that flip axes beyond d-1 do not exist
      for (int a = D - 1; a < FOLD_MAXD - 1; ++a) ok = ok && !((s >> (FOLD_MAXD - 2 - a)) & 1);
      if (ok) acc += src[idx];
    }
    out[e] = acc;
  }
}

// The same fold, one workgroup per output row (the last, unflipped axis):
// the row's <= 2^(d-1) image rows are resolved once per workgroup and the
// threads stream along them -- no per-element 64-bit div / mod (which bound
// the element-per-thread kernel above at ~2.5 TB/s).  Summation order and
// start value as in bin_fold_half_kernel (bitwise).
template <typename T>
__global__ __launch_bounds__(256) void bin_fold_half_rows(const T* __restrict__ in, T* __restrict__ out,
                                                          FoldShape fs, long long nouter, long long nhalf) {
  const int D = fs.d;
  const long long hl = fs.h[D - 1];
  for (long long o = blockIdx.x; o < nouter; o += gridDim.x) {
    long long r = o;
    long long q[FOLD_MAXD], m[FOLD_MAXD];
    bool two[FOLD_MAXD];
#pragma unroll
    for (int a = FOLD_MAXD - 1; a >= 0; --a) {
      q[a] = m[a] = 0;
      two[a] = false;
      if (a < D - 1) {
        q[a] = r % fs.h[a];
        r /= fs.h[a];
        m[a] = fs.n[a] - q[a];
        two[a] = q[a] != 0 && m[a] != q[a];
      }
    }
    const long long p = r;
    long long roff[1 << (FOLD_MAXD - 1)];
    bool rok[1 << (FOLD_MAXD - 1)];
#pragma unroll
    for (int s = 0; s < (1 << (FOLD_MAXD - 1)); ++s) {
      bool ok = true;
      long long idx = 0;
#pragma unroll
      for (int a = 0; a < FOLD_MAXD - 1; ++a) {
        if (a >= D - 1) continue;
        const bool hi = (s >> (FOLD_MAXD - 2 - a)) & 1;
        ok = ok && (!hi || two[a]);
        idx = idx * fs.n[a] + (hi ? m[a] : q[a]);
      }
      for (int a = D - 1; a < FOLD_MAXD - 1; ++a) ok = ok && !((s >> (FOLD_MAXD - 2 - a)) & 1);
      rok[s] = ok;
      roff[s] = idx * hl;
    }
    const T* src = in + p * nhalf;
    T* dst = out + o * hl;
    // FU values per thread in flight: every load of a group before its stores
    constexpr int FU = 4;
    for (long long x0 = threadIdx.x; x0 < hl; x0 += FU * (long long)blockDim.x) {
      T v[FU][1 << (FOLD_MAXD - 1)];
#pragma unroll
      for (int u = 0; u < FU; ++u) {
        const long long x = x0 + u * (long long)blockDim.x;
#pragma unroll
        for (int s = 0; s < (1 << (FOLD_MAXD - 1)); ++s) v[u][s] = (rok[s] && x < hl) ? src[roff[s] + x] : (T)0;
      }
#pragma unroll
      for (int u = 0; u < FU; ++u) {
        const long long x = x0 + u * (long long)blockDim.x;
        if (x >= hl) break;
        T acc = (T)0;
#pragma unroll
        for (int s = 0; s < (1 << (FOLD_MAXD - 1)); ++s)
          if (rok[s]) acc += v[u][s];
        dst[x] = acc;
      }
    }
  }
}

// bin_fold_half_rows over the flat output index (one output per thread, its
// row decoded with 32-bit divisions): the row launch spends a second round
// of loads on each row's last element (h = n/2 + 1 = 4 x 256 + 1 at 2048^2).
// Same sums in the same order (bitwise).
template <typename T>
__global__ __launch_bounds__(256) void bin_fold_half_flat_planar(const T* __restrict__ in, T* __restrict__ out,
                                                                 FoldShape fs, unsigned tot, long long nhalf) {
  const unsigned e = blockIdx.x * 256u + threadIdx.x;
  if (e >= tot) return;
  const int D = fs.d;
  const unsigned hl = (unsigned)fs.h[D - 1];
  const unsigned o = e / hl, x = e - o * hl;
  unsigned r = o;
  long long q[FOLD_MAXD], m[FOLD_MAXD];
  bool two[FOLD_MAXD];
#pragma unroll
  for (int a = FOLD_MAXD - 1; a >= 0; --a) {
    q[a] = m[a] = 0;
    two[a] = false;
    if (a < D - 1) {
      const unsigned h = (unsigned)fs.h[a];
      const unsigned qq = r % h;
      r /= h;
      q[a] = qq;
      m[a] = fs.n[a] - q[a];
      two[a] = q[a] != 0 && m[a] != q[a];
    }
  }
  const T* src = in + (long long)r * nhalf + x;  // r: the item
  constexpr int NS = 1 << (FOLD_MAXD - 1);
  T v[NS];
  bool rok[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    bool ok = true;
    long long idx = 0;
#pragma unroll
    for (int a = 0; a < FOLD_MAXD - 1; ++a) {
      if (a >= D - 1) continue;
      const bool hi = (s >> (FOLD_MAXD - 2 - a)) & 1;
      ok = ok && (!hi || two[a]);
      idx = idx * fs.n[a] + (hi ? m[a] : q[a]);
    }
    for (int a = D - 1; a < FOLD_MAXD - 1; ++a) ok = ok && !((s >> (FOLD_MAXD - 2 - a)) & 1);
    rok[s] = ok;
    v[s] = ok ? src[idx * (long long)hl] : (T)0;
  }
  T acc = (T)0;
#pragma unroll
  for (int s = 0; s < NS; ++s)
    if (rok[s]) acc += v[s];
  out[e] = acc;
}

// The half-grid fold written in bin-sorted order, the items of a cell
// adjacent: out[cpos[cell] * pre + p] (cpos = inverse of the folded index's
// stable bin -> cell permutation).  One workgroup per cell row, all pre items
// per thread (<= 8: one 8 pre-byte store per cell).  Summation order and
// start value as in bin_fold_half_kernel (bitwise); bin_sum_sorted then sums
// each bin over a contiguous run, in the order of bin_scatter_chunk.
template <typename T, int PRE>
__global__ __launch_bounds__(256) void bin_fold_half_sorted(const T* __restrict__ in, T* __restrict__ out,
                                                            const int* __restrict__ cpos, FoldShape fs,
                                                            long long nrows, long long nhalf, int pre) {
  const int D = fs.d;
  const long long hl = fs.h[D - 1];
  for (long long o = blockIdx.x; o < nrows; o += gridDim.x) {
    long long r = o;
    long long q[FOLD_MAXD], m[FOLD_MAXD];
    bool two[FOLD_MAXD];
#pragma unroll
    for (int a = FOLD_MAXD - 1; a >= 0; --a) {
      q[a] = m[a] = 0;
      two[a] = false;
      if (a < D - 1) {
        q[a] = r % fs.h[a];
        r /= fs.h[a];
        m[a] = fs.n[a] - q[a];
        two[a] = q[a] != 0 && m[a] != q[a];
      }
    }
    long long roff[1 << (FOLD_MAXD - 1)];
    bool rok[1 << (FOLD_MAXD - 1)];
#pragma unroll
    for (int s = 0; s < (1 << (FOLD_MAXD - 1)); ++s) {
      bool ok = true;
      long long idx = 0;
#pragma unroll
      for (int a = 0; a < FOLD_MAXD - 1; ++a) {
        if (a >= D - 1) continue;
        const bool hi = (s >> (FOLD_MAXD - 2 - a)) & 1;
        ok = ok && (!hi || two[a]);
        idx = idx * fs.n[a] + (hi ? m[a] : q[a]);
      }
      for (int a = D - 1; a < FOLD_MAXD - 1; ++a) ok = ok && !((s >> (FOLD_MAXD - 2 - a)) & 1);
      rok[s] = ok;
      roff[s] = idx * hl;
    }
    // FU values per thread in flight (all their loads before the stores)
    constexpr int FU = PRE <= 4 ? 2 : 1;
    for (long long x0 = threadIdx.x; x0 < hl; x0 += FU * (long long)blockDim.x) {
      T v[FU][PRE][1 << (FOLD_MAXD - 1)];
#pragma unroll
      for (int u = 0; u < FU; ++u) {
        const long long x = x0 + u * (long long)blockDim.x;
#pragma unroll
        for (int p = 0; p < PRE; ++p)
#pragma unroll
          for (int s = 0; s < (1 << (FOLD_MAXD - 1)); ++s)
            v[u][p][s] = (x < hl && p < pre && rok[s]) ? in[p * nhalf + roff[s] + x] : (T)0;
      }
#pragma unroll
      for (int u = 0; u < FU; ++u) {
        const long long x = x0 + u * (long long)blockDim.x;
        if (x >= hl) break;
        const long long dpos = (cpos ? (long long)cpos[o * hl + x] : o * hl + x) * pre;
        T accs[PRE];
#pragma unroll
        for (int p = 0; p < PRE; ++p) {
          T acc = (T)0;
#pragma unroll
          for (int s = 0; s < (1 << (FOLD_MAXD - 1)); ++s)
            if (rok[s]) acc += v[u][p][s];
          accs[p] = acc;
        }
        if (PRE % 2 == 0 && pre == PRE) {
          // the cell's items as 2-wide vector stores (8 PRE-byte aligned run)
          typedef T V2 __attribute__((ext_vector_type(2)));
#pragma unroll
          for (int p = 0; p < PRE; p += 2) {
            V2 w;
            w.x = accs[p];
            w.y = accs[p + 1];
            *(V2*)(out + dpos + p) = w;
          }
        } else {
#pragma unroll
          for (int p = 0; p < PRE; ++p) {
            if (p >= pre) break;
            out[dpos + p] = accs[p];
          }
        }
      }
    }
  }
}

// bin_fold_half_sorted over the flat cell index: one cell per thread, the
// cell row decoded per thread.  A row-per-workgroup launch runs ~2 rounds of
// its loads per row (h = n/2 + 1 cells: the last round for one cell) at 2
// workgroups per CU for 1024^2; here every thread issues its loads once and
// the grid holds n/2 + 1 times more threads.  Same sums in the same order,
// same stores (bitwise).
template <typename T, int PRE>
__global__ __launch_bounds__(256) void bin_fold_half_flat(const T* __restrict__ in, T* __restrict__ out,
                                                          const int* __restrict__ cpos, FoldShape fs,
                                                          unsigned ncell, long long nhalf, int pre) {
  const unsigned e = blockIdx.x * 256u + threadIdx.x;
  if (e >= ncell) return;
  const int D = fs.d;
  const unsigned hl = (unsigned)fs.h[D - 1];
  const unsigned o = e / hl, x = e - o * hl;
  unsigned r = o;
  long long q[FOLD_MAXD], m[FOLD_MAXD];
  bool two[FOLD_MAXD];
#pragma unroll
  for (int a = FOLD_MAXD - 1; a >= 0; --a) {
    q[a] = m[a] = 0;
    two[a] = false;
    if (a < D - 1) {
      const unsigned h = (unsigned)fs.h[a];
      const unsigned qq = r % h;
      r /= h;
      q[a] = qq;
      m[a] = fs.n[a] - q[a];
      two[a] = q[a] != 0 && m[a] != q[a];
    }
  }
  constexpr int NS = 1 << (FOLD_MAXD - 1);
  long long roff[NS];
  bool rok[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    bool ok = true;
    long long idx = 0;
#pragma unroll
    for (int a = 0; a < FOLD_MAXD - 1; ++a) {
      if (a >= D - 1) continue;
      const bool hi = (s >> (FOLD_MAXD - 2 - a)) & 1;
      ok = ok && (!hi || two[a]);
      idx = idx * fs.n[a] + (hi ? m[a] : q[a]);
    }
    for (int a = D - 1; a < FOLD_MAXD - 1; ++a) ok = ok && !((s >> (FOLD_MAXD - 2 - a)) & 1);
    rok[s] = ok;
    roff[s] = idx * (long long)hl;
  }
  T v[PRE][NS];
#pragma unroll
  for (int p = 0; p < PRE; ++p)
#pragma unroll
    for (int s = 0; s < NS; ++s) v[p][s] = (p < pre && rok[s]) ? in[p * nhalf + roff[s] + x] : (T)0;
  const long long dpos = (cpos ? (long long)cpos[e] : (long long)e) * pre;
  T accs[PRE];
#pragma unroll
  for (int p = 0; p < PRE; ++p) {
    T acc = (T)0;
#pragma unroll
    for (int s = 0; s < NS; ++s)
      if (rok[s]) acc += v[p][s];
    accs[p] = acc;
  }
  if (PRE % 2 == 0 && pre == PRE) {
    typedef T V2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int p = 0; p < PRE; p += 2) {
      V2 w;
      w.x = accs[p];
      w.y = accs[p + 1];
      *(V2*)(out + dpos + p) = w;
    }
  } else {
#pragma unroll
    for (int p = 0; p < PRE; ++p) {
      if (p >= pre) break;
      out[dpos + p] = accs[p];
    }
  }
}

// The bin sums of the fold in cell order with the items interleaved
// (bin_fold_half_sorted with cpos = NULL: in[cell * PRE + p]): chunks of CH
// bin-sorted positions as in bin_scatter_chunk, one 8 PRE-byte gather per
// position for all items (the planar layout gathers PRE cache lines), bins
// summed in ascending position from 0 (bitwise bin_scatter_chunk).
template <typename T, int PRE, int CH>
__global__ __launch_bounds__(256) void bin_scatter_il(const T* __restrict__ in, const int* __restrict__ perm,
                                                      const int* __restrict__ offs, const int* __restrict__ cb,
                                                      T* __restrict__ out, long long npix, long long nbins,
                                                      int nchunks) {
  static_assert(CH % 256 == 0, "bin_scatter_il loads CH / 256 positions per thread");
  constexpr int PER = CH / 256;
  // bins of more than LONGB positions (3-D grids: 512^3 has 87 k of its
  // 141 k folded bins above 64 cells, up to 747) are summed by one wave each
  // -- lane-strided partials, then a fixed shuffle tree -- instead of one
  // thread's serial chain; shorter bins keep the sequential sum (2-D grids:
  // at most 40 cells per folded bin up to 4096^2, so their sums are unchanged)
  constexpr int LONGB = 64;
  __shared__ T vals[PRE][CH];
  __shared__ int bnd[2];
  __shared__ int nlong;
  __shared__ int longb[CH / LONGB + 1];
  const int per = (nchunks + NXCD - 1) / NXCD;
  const int c = (int)(blockIdx.x % NXCD) * per + (int)(blockIdx.x / NXCD);
  if (c >= nchunks) return;
  const long long j0 = (long long)c * CH;
  const int t = threadIdx.x;
  const int n = (int)(npix - j0 < CH ? npix - j0 : CH);
  int pv[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int e = t + i * 256;
    pv[i] = e < n ? perm[j0 + e] : 0;
  }
  T v[PER][PRE];
#pragma unroll
  for (int i = 0; i < PER; ++i)
#pragma unroll
    for (int p = 0; p < PRE; ++p) v[i][p] = t + i * 256 < n ? in[(long long)pv[i] * PRE + p] : (T)0;
  if (t == 0) nlong = 0;
  if (t < 2 && cb) {
    bnd[t] = cb[c + t];  // the plan's chunk -> first bin table
  } else if (t < 2) {
    // first bin whose start offset is >= j0 (+ CH): a chain of ~20 dependent
    // loads per workgroup, the table's reason
    const long long target = j0 + (t ? CH : 0);
    long long lo = 0, hi = nbins;
    while (lo < hi) {
      const long long mid = (lo + hi) >> 1;
      if ((long long)offs[mid] < target) lo = mid + 1;
      else hi = mid;
    }
    bnd[t] = (t && j0 + CH >= npix) ? (int)nbins : (int)lo;
  }
#pragma unroll
  for (int i = 0; i < PER; ++i)
#pragma unroll
    for (int p = 0; p < PRE; ++p)
      if (t + i * 256 < n) vals[p][t + i * 256] = v[i][p];
  __syncthreads();
  const int b0 = bnd[0], b1 = bnd[1];
  for (int b = b0 + t; b < b1; b += 256) {
    const long long a = offs[b], e = offs[b + 1];
    if (e - a > LONGB) {
      longb[atomicAdd(&nlong, 1)] = b;  // list order is irrelevant: one bin per entry
      continue;
    }
    T acc[PRE];
#pragma unroll
    for (int p = 0; p < PRE; ++p) acc[p] = (T)0;
    for (long long j = a; j < e; ++j) {
      if (j - j0 < CH) {
#pragma unroll
        for (int p = 0; p < PRE; ++p) acc[p] += vals[p][j - j0];
      } else {
        const long long q = (long long)perm[j] * PRE;
#pragma unroll
        for (int p = 0; p < PRE; ++p) acc[p] += in[q + p];
      }
    }
#pragma unroll
    for (int p = 0; p < PRE; ++p) out[p * nbins + b] = acc[p];
  }
  __syncthreads();
  const int w = t >> 6, lane = t & 63;
  for (int i = w; i < nlong; i += 4) {
    const int b = longb[i];
    const long long a = offs[b], e = offs[b + 1];
    T acc[PRE];
#pragma unroll
    for (int p = 0; p < PRE; ++p) acc[p] = (T)0;
    for (long long j = a + lane; j < e; j += 64) {
      if (j - j0 < CH) {
#pragma unroll
        for (int p = 0; p < PRE; ++p) acc[p] += vals[p][j - j0];
      } else {
        const long long q = (long long)perm[j] * PRE;
#pragma unroll
        for (int p = 0; p < PRE; ++p) acc[p] += in[q + p];
      }
    }
#pragma unroll
    for (int p = 0; p < PRE; ++p) {
      T v = acc[p];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
      if (lane == 0) out[p * nbins + b] = v;
    }
  }
}


// I: index type -- 32-bit when pre * nin < 2^31 (the usual case: cheaper
// div/mod per element), 64-bit otherwise
template <typename T, typename I>
__global__ __launch_bounds__(256) void bin_fold_kernel(const T* __restrict__ in, T* __restrict__ out, FoldShape fs,
                                                       long long pre) {
  const I tot = (I)(pre * fs.nout), nout = (I)fs.nout, nin = (I)fs.nin;
  I n[FOLD_MAXD], h[FOLD_MAXD];
#pragma unroll
  for (int a = 0; a < FOLD_MAXD; ++a) {
    n[a] = (I)fs.n[a];
    h[a] = (I)fs.h[a];
  }
  const I stride = (I)gridDim.x * blockDim.x;
  for (I e = (I)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += stride) {
    I r = e % nout;
    const I p = e / nout;
    I q[FOLD_MAXD], m[FOLD_MAXD];
    bool two[FOLD_MAXD];
#pragma unroll
    for (int a = FOLD_MAXD - 1; a >= 0; --a) {
      if (a < fs.d) {
        q[a] = r % h[a];
        r /= h[a];
        m[a] = n[a] - q[a];
        two[a] = q[a] != 0 && m[a] != q[a];
      } else {
        q[a] = m[a] = 0;
        two[a] = false;
      }
    }
    const T* src = in + p * nin;
    T acc = (T)0;
#pragma unroll
    for (int s = 0; s < (1 << FOLD_MAXD); ++s) {
      bool ok = true;
      I idx = 0;
#pragma unroll
      for (int a = 0; a < FOLD_MAXD; ++a) {
        if (a >= fs.d) {
          ok = ok && !((s >> (FOLD_MAXD - 1 - a)) & 1);
          continue;
        }
        const bool hi = (s >> (FOLD_MAXD - 1 - a)) & 1;
        ok = ok && (!hi || two[a]);
        idx = idx * n[a] + (hi ? m[a] : q[a]);
      }
      if (ok) acc += src[idx];
    }
    out[e] = acc;
  }
}


static int nblocks(long long tot) {
  long long b = (tot + 255) / 256;
  if (b < 1) b = 1;
  if (b > 65536) b = 65536;
  return (int)b;
}

}  // namespace nft

using namespace nft;

extern "C" {

int nft_bin_gather(const void* in, const int* pindex, void* out, int64_t pre, int64_t npix,
                   int64_t nbins, int64_t post, int dtype, hipStream_t stream) {
  long long tot = pre * npix * post;
  if (tot <= 0) return NFT_OK;
  if (dtype == 0)
    hipLaunchKernelGGL(bin_gather_kernel<double>, dim3(nblocks(tot)), dim3(256), 0, stream,
                       (const double*)in, pindex, (double*)out, (long long)pre, (long long)npix, (long long)nbins, (long long)post);
  else if (dtype == 1)
    hipLaunchKernelGGL(bin_gather_kernel<float>, dim3(nblocks(tot)), dim3(256), 0, stream,
                       (const float*)in, pindex, (float*)out, (long long)pre, (long long)npix, (long long)nbins, (long long)post);
  else {
    set_last_error("nft_bin_gather: bad dtype");
    return NFT_ERR_ARG;
  }
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

int nft_bin_chunk(void) { return BS_CH; }

int nft_bin_scatter(const void* in, const int* perm, const int* offsets, void* out, int64_t pre,
                    int64_t npix, int64_t nbins, int64_t post, int dtype, hipStream_t stream) {
  return nft_bin_scatter_ordered(in, perm, offsets, nullptr, nullptr, nullptr, out, pre, npix, nbins, post, dtype,
                                 stream);
}

int nft_bin_scatter_ordered(const void* in, const int* perm, const int* offsets, const int* gpix,
                            const uint16_t* gslot, const int* cbins, void* out, int64_t pre, int64_t npix,
                            int64_t nbins, int64_t post, int dtype, hipStream_t stream) {
  if ((gpix == nullptr) != (gslot == nullptr)) {
    set_last_error("nft_bin_scatter_ordered: gpix and gslot must both be given or both be NULL");
    return NFT_ERR_ARG;
  }
  long long tot = pre * nbins * post;
  if (tot <= 0) return NFT_OK;
  if (post == 1 && pre <= 65535 && (dtype == 0 || dtype == 1)) {
    const int nchunks = (int)((npix + BS_CH - 1) / BS_CH);
    const unsigned nb = (unsigned)(((nchunks + NXCD - 1) / NXCD) * NXCD);
    if (npix <= 0) {
      NFT_HIP_CHECK(hipMemsetAsync(out, 0, (size_t)pre * nbins * (dtype == 0 ? 8 : 4), stream));
      return NFT_OK;
    }
    prof_mark(stream, "bin_scatter");
    // one item per workgroup row (several items per workgroup measured slower
    // at 2048^2, 4 items: 109 us for one, 118 for two, 133 for four)
    const dim3 grid(nb, (unsigned)pre);
#define NFT_SCAT(TT, KK)                                                                                 \
  hipLaunchKernelGGL((bin_scatter_chunk<TT, KK>), grid, dim3(256), 0, stream, (const TT*)in, perm, offsets, gpix, \
                     (const unsigned short*)gslot, cbins, (TT*)out, (long long)npix, (long long)nbins, nchunks)
    if (dtype == 0) NFT_SCAT(double, 1);
    else NFT_SCAT(float, 1);
#undef NFT_SCAT
    NFT_HIP_CHECK(hipGetLastError());
    return NFT_OK;
  }
  if (dtype == 0)
    hipLaunchKernelGGL(bin_scatter_kernel<double>, dim3(nblocks(tot)), dim3(256), 0, stream,
                       (const double*)in, perm, offsets, (double*)out, (long long)pre, (long long)npix,
                       (long long)nbins, (long long)post);
  else if (dtype == 1)
    hipLaunchKernelGGL(bin_scatter_kernel<float>, dim3(nblocks(tot)), dim3(256), 0, stream,
                       (const float*)in, perm, offsets, (float*)out, (long long)pre, (long long)npix,
                       (long long)nbins, (long long)post);
  else {
    set_last_error("nft_bin_scatter: bad dtype");
    return NFT_ERR_ARG;
  }
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

int nft_bin_scatter_folded(const void* in, const int* perm, const int* offsets, const int* chunk_bins, void* out,
                           int64_t pre, int64_t npix, int64_t nbins, int dtype, hipStream_t stream) {
  if (pre < 1 || pre > 65535 || npix < 0 || nbins < 0 || !perm || !offsets || !(dtype == 0 || dtype == 1)) {
    set_last_error("nft_bin_scatter_folded: need 1 <= pre <= 65535, perm, offsets and dtype 0 / 1");
    return NFT_ERR_ARG;
  }
  if (nbins == 0) return NFT_OK;
  if (npix == 0) {
    NFT_HIP_CHECK(hipMemsetAsync(out, 0, (size_t)pre * nbins * (dtype == 0 ? 8 : 4), stream));
    return NFT_OK;
  }
  const int nchunks = (int)((npix + BS_CH - 1) / BS_CH);
  const unsigned nb = (unsigned)(((nchunks + NXCD - 1) / NXCD) * NXCD);
  prof_mark(stream, "bin_scatter");
  const dim3 grid(nb, (unsigned)pre);
  if (dtype == 0)
    hipLaunchKernelGGL((bin_scatter_chunk<double, 1, true>), grid, dim3(256), 0, stream, (const double*)in, perm,
                       offsets, nullptr, nullptr, chunk_bins, (double*)out, (long long)npix, (long long)nbins,
                       nchunks);
  else
    hipLaunchKernelGGL((bin_scatter_chunk<float, 1, true>), grid, dim3(256), 0, stream, (const float*)in, perm,
                       offsets, nullptr, nullptr, chunk_bins, (float*)out, (long long)npix, (long long)nbins,
                       nchunks);
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

int nft_bin_fold_half(const void* in, void* out, int64_t pre, int ndim, const int64_t* shape, int dtype,
                      hipStream_t stream) {
  if (ndim < 1 || ndim > FOLD_MAXD || pre < 0) {
    set_last_error("nft_bin_fold_half: need 1 <= ndim <= 3 and pre >= 0");
    return NFT_ERR_ARG;
  }
  FoldShape fs;
  fs.d = ndim;
  fs.nin = 1;
  fs.nout = 1;
  for (int a = 0; a < FOLD_MAXD; ++a) fs.n[a] = fs.h[a] = 1;
  long long nhalf = 1;
  for (int a = 0; a < ndim; ++a) {
    if (shape[a] < 1) {
      set_last_error("nft_bin_fold_half: bad shape");
      return NFT_ERR_ARG;
    }
    fs.n[a] = shape[a];
    fs.h[a] = shape[a] / 2 + 1;
    fs.nin *= shape[a];
    fs.nout *= fs.h[a];
    nhalf *= (a == ndim - 1) ? fs.h[a] : shape[a];
  }
  const long long tot = pre * fs.nout;
  if (tot <= 0) return NFT_OK;
  prof_mark(stream, "bin_fold");
  // one output per thread (NFT_FOLD_FLAT=0: one workgroup per output row)
  const char* fenv = getenv("NFT_FOLD_FLAT");
  const bool flat = !(fenv && fenv[0] == '0') && tot < (1LL << 31) - 256;
  constexpr bool rows = true;
  const long long nouter = tot / fs.h[ndim - 1];
  const unsigned rgrid = (unsigned)std::min<long long>(nouter, 1LL << 20);
  if (flat && dtype == 0)
    hipLaunchKernelGGL(bin_fold_half_flat_planar<double>, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream,
                       (const double*)in, (double*)out, fs, (unsigned)tot, nhalf);
  else if (flat && dtype == 1)
    hipLaunchKernelGGL(bin_fold_half_flat_planar<float>, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream,
                       (const float*)in, (float*)out, fs, (unsigned)tot, nhalf);
  else if (rows && dtype == 0)
    hipLaunchKernelGGL(bin_fold_half_rows<double>, dim3(rgrid), dim3(256), 0, stream, (const double*)in,
                       (double*)out, fs, nouter, nhalf);
  else if (rows && dtype == 1)
    hipLaunchKernelGGL(bin_fold_half_rows<float>, dim3(rgrid), dim3(256), 0, stream, (const float*)in,
                       (float*)out, fs, nouter, nhalf);
  else if (dtype == 0)
    hipLaunchKernelGGL(bin_fold_half_kernel<double>, dim3(nblocks(tot)), dim3(256), 0, stream, (const double*)in,
                       (double*)out, fs, (long long)pre, nhalf);
  else if (dtype == 1)
    hipLaunchKernelGGL(bin_fold_half_kernel<float>, dim3(nblocks(tot)), dim3(256), 0, stream, (const float*)in,
                       (float*)out, fs, (long long)pre, nhalf);
  else {
    set_last_error("nft_bin_fold_half: bad dtype");
    return NFT_ERR_ARG;
  }
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

int nft_bin_fold_half_sorted(const void* in, void* out, const int* cpos, int64_t pre, int ndim,
                             const int64_t* shape, int dtype, hipStream_t stream) {
  if (ndim < 1 || ndim > FOLD_MAXD || pre < 1 || pre > 8) {
    set_last_error("nft_bin_fold_half_sorted: need 1 <= ndim <= 3 and 1 <= pre <= 8");
    return NFT_ERR_ARG;
  }
  FoldShape fs{};
  fs.d = ndim;
  fs.nin = 1;
  fs.nout = 1;
  for (int a = 0; a < FOLD_MAXD; ++a) fs.n[a] = fs.h[a] = 1;
  long long nhalf = 1;
  for (int a = 0; a < ndim; ++a) {
    if (shape[a] < 1) {
      set_last_error("nft_bin_fold_half_sorted: bad shape");
      return NFT_ERR_ARG;
    }
    fs.n[a] = shape[a];
    fs.h[a] = shape[a] / 2 + 1;
    fs.nin *= shape[a];
    fs.nout *= fs.h[a];
    nhalf *= (a == ndim - 1) ? fs.h[a] : shape[a];
  }
  const long long nrows = fs.nout / fs.h[ndim - 1];
  const unsigned grid = (unsigned)std::min<long long>(nrows, 1LL << 20);
  // the flat launch (NFT_FOLD_FLAT=0: one workgroup per cell row)
  const char* fenv = getenv("NFT_FOLD_FLAT");
  const bool flat_knob = !(fenv && fenv[0] == '0');
  const bool flat = flat_knob && fs.nout < (1LL << 31) - 256;
  const unsigned fgrid = (unsigned)((fs.nout + 255) / 256);
  prof_mark(stream, "bin_fold");
#define NFT_FS(TT, PP)                                                                                          \
  do {                                                                                                          \
    if (flat)                                                                                                   \
      hipLaunchKernelGGL((bin_fold_half_flat<TT, PP>), dim3(fgrid), dim3(256), 0, stream, (const TT*)in,        \
                         (TT*)out, cpos, fs, (unsigned)fs.nout, nhalf, (int)pre);                               \
    else                                                                                                        \
      hipLaunchKernelGGL((bin_fold_half_sorted<TT, PP>), dim3(grid), dim3(256), 0, stream, (const TT*)in,      \
                         (TT*)out, cpos, fs, nrows, nhalf, (int)pre);                                           \
  } while (0)
  if (dtype == 0) {
    if (pre <= 1) NFT_FS(double, 1);
    else if (pre <= 2) NFT_FS(double, 2);
    else if (pre <= 4) NFT_FS(double, 4);
    else NFT_FS(double, 8);
  } else if (dtype == 1) {
    if (pre <= 1) NFT_FS(float, 1);
    else if (pre <= 2) NFT_FS(float, 2);
    else if (pre <= 4) NFT_FS(float, 4);
    else NFT_FS(float, 8);
  } else {
    set_last_error("nft_bin_fold_half_sorted: bad dtype");
    return NFT_ERR_ARG;
  }
#undef NFT_FS
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

// bin-sorted positions x items per nft_bin_scatter_il workgroup (4096 measured 31 -> 36 us)
constexpr int SIL_CH = 2048;
static int sil_chunk(int64_t pre) { return SIL_CH / pre >= 256 ? (int)(SIL_CH / pre) / 256 * 256 : 256; }
int nft_bin_scatter_il_chunk(int64_t pre) { return (pre == 2 || pre == 4 || pre == 8) ? sil_chunk(pre) : 0; }
int nft_bin_scatter_il(const void* in, const int* perm, const int* offsets, const int* chunk_bins, void* out,
                       int64_t pre, int64_t npix, int64_t nbins, int dtype, hipStream_t stream) {
  if (!(pre == 2 || pre == 4 || pre == 8) || npix < 0 || nbins < 0 || !perm || !offsets) {
    set_last_error("nft_bin_scatter_il: need pre in {2, 4, 8}, perm and offsets");
    return NFT_ERR_ARG;
  }
  if (nbins == 0) return NFT_OK;
  if (npix == 0) {
    NFT_HIP_CHECK(hipMemsetAsync(out, 0, (size_t)pre * nbins * (dtype == 0 ? 8 : 4), stream));
    return NFT_OK;
  }
  prof_mark(stream, "bin_scatter");
#define NFT_SIL(TT, PP)                                                                                       \
  {                                                                                                           \
    constexpr int CH = SIL_CH / PP >= 256 ? (SIL_CH / PP) / 256 * 256 : 256;                                 \
    const int nch = (int)((npix + CH - 1) / CH);                                                              \
    const unsigned nb = (unsigned)(((nch + NXCD - 1) / NXCD) * NXCD);                                         \
    hipLaunchKernelGGL((bin_scatter_il<TT, PP, CH>), dim3(nb), dim3(256), 0, stream, (const TT*)in, perm, offsets, \
                       chunk_bins, (TT*)out, (long long)npix, (long long)nbins, nch);                         \
  }
  if (dtype == 0) {
    if (pre == 2) NFT_SIL(double, 2) else if (pre == 4) NFT_SIL(double, 4) else NFT_SIL(double, 8)
  } else if (dtype == 1) {
    if (pre == 2) NFT_SIL(float, 2) else if (pre == 4) NFT_SIL(float, 4) else NFT_SIL(float, 8)
  } else {
    set_last_error("nft_bin_scatter_il: bad dtype");
    return NFT_ERR_ARG;
  }
#undef NFT_SIL
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

int nft_bin_fold(const void* in, void* out, int64_t pre, int ndim, const int64_t* shape, int dtype,
                 hipStream_t stream) {
  if (ndim < 1 || ndim > FOLD_MAXD || pre < 0) {
    set_last_error("nft_bin_fold: need 1 <= ndim <= 3 and pre >= 0");
    return NFT_ERR_ARG;
  }
  FoldShape fs{};
  fs.d = ndim;
  fs.nin = fs.nout = 1;
  for (int a = 0; a < ndim; ++a) {
    if (shape[a] < 1) {
      set_last_error("nft_bin_fold: bad shape");
      return NFT_ERR_ARG;
    }
    fs.n[a] = shape[a];
    fs.h[a] = shape[a] / 2 + 1;
    fs.nin *= fs.n[a];
    fs.nout *= fs.h[a];
  }
  const long long tot = pre * fs.nout;
  if (tot <= 0) return NFT_OK;
  prof_mark(stream, "bin_fold");
  const bool i32 = pre * fs.nin < (1LL << 31) - 65536LL * 256;  // grid-stride increments stay in range
#define NFT_FOLD(TT, II)                                                                                     \
  hipLaunchKernelGGL((bin_fold_kernel<TT, II>), dim3(nblocks(tot)), dim3(256), 0, stream, (const TT*)in, \
                     (TT*)out, fs, (long long)pre)
  if (dtype == 0) {
    if (i32) NFT_FOLD(double, unsigned);
    else NFT_FOLD(double, long long);
  } else if (dtype == 1) {
    if (i32) NFT_FOLD(float, unsigned);
    else NFT_FOLD(float, long long);
  } else {
    set_last_error("nft_bin_fold: bad dtype");
    return NFT_ERR_ARG;
  }
#undef NFT_FOLD
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

}  // extern "C"

