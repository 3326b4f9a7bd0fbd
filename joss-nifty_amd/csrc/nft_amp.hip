// Correlated-field amplitude Jacobian (JVP / VJP) on the power-spectrum bins.
//
// Replaces, for the sampling metric, the B-sized operator subtree of the
// reference's CF model (src/library/correlated_fields.py:91-201,
// correlated_fields_simple.py:86-127): NormalTransform/LognormalTransform
// scalings, _TwoLogIntegrations (two cumulative sums), _SlopeRemover,
// _Normalization (exp, sum over modes, sqrt), zero-mode insertion and volume
// scaling.  The nonlinear parts are linearised at the expansion point; all
// per-bin constants of that linearisation are precomputed there (see
// AmpConst), so a JVP or VJP is four to six bandwidth-light kernels instead of
// ~25 small tensor ops:
//
//   JVP:  scan(t1*sf) -> t = (c+c_prev)/2*lv + t0*c0 -> scan(t) -> dapre -> da
//   VJP:  gapre -> reverse scan -> reverse scan -> spectrum / scalar cotangents
//
// Scans are block-local (1024 elements per workgroup) with the carry of each
// block obtained by summing the totals of all preceding blocks in index order:
// O(nblocks) per block, deterministic, no inter-workgroup hand-off.
#include "nft_api_internal.hpp"

namespace nft {

using AmpConst = nft_amp_const;
using AmpOut = nft_amp_out;

// right-hand side blockIdx.y of a batched launch: latent tangents / cotangents
// advance by ls elements, B-sized vectors by vs, the workspace by wsd
__device__ __forceinline__ void amp_out_offset(nft_amp_out& o, long long off) {
  if (o.fl) o.fl += off;
  if (o.sl) o.sl += off;
  if (o.flex) o.flex += off;
  if (o.asp) o.asp += off;
  if (o.zm) o.zm += off;
  if (o.spec) o.spec += off;
  if (o.dfl) o.dfl += off;
  if (o.dsl) o.dsl += off;
  if (o.dflex) o.dflex += off;
  if (o.dasp) o.dasp += off;
  if (o.dzm) o.dzm += off;
  if (o.dspec) o.dspec += off;
}

constexpr int AT = 256;          // threads per block
constexpr int AE = 4;            // elements per thread
constexpr int ABLK = AT * AE;    // elements per block

__device__ __forceinline__ double wsum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  return v;
}

// block-wide sum, result broadcast to all threads
__device__ __forceinline__ double block_total(double v, double* sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wsum(v);
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  double t = 0;
#pragma unroll
  for (int i = 0; i < AT / 64; ++i) t += sh[i];
  __syncthreads();
  return t;
}

// inclusive block scan of AE values per thread in STRIPED layout: v[k] is
// element k*AT + threadIdx.x of the block (so every global access of a block
// is a coalesced 2 KB run per k).  REV scans from the end.  Wave scans by
// shuffles, then one fixed-order pass over the AE*AT/64 wave totals.
// Returns the block total.
template <bool REV>
__device__ __forceinline__ double block_scan(double (&v)[AE], double* sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int NW = AT / 64;
#pragma unroll
  for (int k = 0; k < AE; ++k) {
    double x = v[k];
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const double y = REV ? __shfl_down(x, off, 64) : __shfl_up(x, off, 64);
      if (REV ? (lane + off < 64) : (lane >= off)) x += y;
    }
    v[k] = x;
    if (lane == (REV ? 0 : 63)) sh[k * NW + w] = x;
  }
  __syncthreads();
  double total = 0.0;
#pragma unroll
  for (int k = 0; k < AE; ++k) {
    const int me = k * NW + w;
    double off = 0.0;
    if (!REV) {
      for (int i = 0; i < me; ++i) off += sh[i];
    } else {
      for (int i = AE * NW - 1; i > me; --i) off += sh[i];
    }
    v[k] += off;
  }
  if (!REV) {
    for (int i = 0; i < AE * NW; ++i) total += sh[i];
  } else {
    for (int i = AE * NW - 1; i >= 0; --i) total += sh[i];
  }
  __syncthreads();
  return total;
}

// sum of block totals [0, blk) (or (blk, nb) for REV) in index order
template <bool REV>
__device__ __forceinline__ double carry_in(const double* tot, int blk, int nb, double* sh) {
  double s = 0;
  if (!REV) {
    for (int i = threadIdx.x; i < blk; i += AT) s += tot[i];
  } else {
    for (int i = blk + 1 + threadIdx.x; i < nb; i += AT) s += tot[i];
  }
  return block_total(s, sh);
}

// ------------------------------------------------------------------ JVP
// J1: cs1 = local scan of t1*sf over j < B-2
__global__ __launch_bounds__(AT) void amp_jvp_1(AmpConst c_, const AmpConst* __restrict__ dcs, const double* __restrict__ tspec,
                                                double* __restrict__ loc, double* __restrict__ tot1, long long ls, long long vs, long long wsd) {
  const AmpConst c = dcs ? dcs[blockIdx.y] : c_;
  if (tspec) tspec += blockIdx.y * ls;
  loc += blockIdx.y * wsd;
  tot1 += blockIdx.y * wsd;
  __shared__ double sh[2 * AT];
  const long long M = c.B - 2;
  const long long j0 = (long long)blockIdx.x * ABLK + threadIdx.x;
  double v[AE];
#pragma unroll
  for (int k = 0; k < AE; ++k) {
    long long j = j0 + (long long)k * AT;
    v[k] = j < M ? tspec[M + j] * c.sf[j] : 0.0;
  }
  double t = block_scan<false>(v, sh);
#pragma unroll
  for (int k = 0; k < AE; ++k)
    if (j0 + (long long)k * AT < M) loc[j0 + (long long)k * AT] = v[k];
  if (threadIdx.x == 0) tot1[blockIdx.x] = t;
}

// J3: c = loc + carry; t = (c + c_prev)/2*lv + t0*c0; local scan of t
__global__ __launch_bounds__(AT) void amp_jvp_3(AmpConst c_, const AmpConst* __restrict__ dcs, const double* __restrict__ tspec,
                                                const double* __restrict__ tot1, double* __restrict__ loc,
                                                double* __restrict__ tot2, long long ls, long long vs, long long wsd) {
  const AmpConst c = dcs ? dcs[blockIdx.y] : c_;
  if (tspec) tspec += blockIdx.y * ls;
  tot1 += blockIdx.y * wsd;
  loc += blockIdx.y * wsd;
  tot2 += blockIdx.y * wsd;
  __shared__ double sh[2 * AT];
  const long long M = c.B - 2;
  const int nb = (int)((M + ABLK - 1) / ABLK);
  const double carry = carry_in<false>(tot1, blockIdx.x, nb, sh);
  const long long j0 = (long long)blockIdx.x * ABLK + threadIdx.x;
  double v[AE];
#pragma unroll
  for (int k = 0; k < AE; ++k) {
    long long j = j0 + (long long)k * AT;
    if (j < M) {
      const double cj = loc[j] + carry;
      const double u1 = tspec[M + j] * c.sf[j];
      const double cp = cj - u1;
      v[k] = (cj + cp) / 2 * c.lv[j] + tspec[j] * c.c0[j];
    } else {
      v[k] = 0.0;
    }
  }
  double t = block_scan<false>(v, sh);
#pragma unroll
  for (int k = 0; k < AE; ++k)
    if (j0 + (long long)k * AT < M) loc[j0 + (long long)k * AT] = v[k];
  if (threadIdx.x == 0) tot2[blockIdx.x] = t;
}

// J5: tl = [0,0, loc + carry]; dapre; partial sums of mspec*dapre
__global__ __launch_bounds__(AT) void amp_jvp_5(AmpConst c_, const AmpConst* __restrict__ dcs, const double* tfl, const double* tsl,
                                                const double* tflex, const double* tasp,
                                                const double* __restrict__ loc, const double* __restrict__ tot2,
                                                double* __restrict__ dapre, double* __restrict__ part, long long ls, long long vs, long long wsd) {
  const AmpConst c = dcs ? dcs[blockIdx.y] : c_;
  if (tfl) tfl += blockIdx.y * ls;
  if (tsl) tsl += blockIdx.y * ls;
  if (tflex) tflex += blockIdx.y * ls;
  if (tasp) tasp += blockIdx.y * ls;
  loc += blockIdx.y * wsd;
  tot2 += blockIdx.y * wsd;
  dapre += blockIdx.y * wsd;
  part += blockIdx.y * wsd;
  __shared__ double sh[2 * AT];
  const long long B = c.B, M = B - 2;
  const int nbM = c.has_flex ? (int)((M + ABLK - 1) / ABLK) : 0;
  double T = 0;  // tl[B-1] = total of the second scan
  if (c.has_flex) T = carry_in<false>(tot2, nbM, nbM, sh);
  const double ssl = c.sig_s * tsl[0];
  const double sf_ = c.has_flex ? tflex[0] : 0.0;
  const double sa_ = c.has_asp ? tasp[0] : 0.0;
  const long long b0 = (long long)blockIdx.x * ABLK;
  // tl_b needs scan position j = b-2; this block's j-range spans at most the
  // scan blocks blk0 and blk0+1
  const int blk0 = b0 >= 2 ? (int)((b0 - 2) / ABLK) : 0;
  double cr0 = 0, cr1 = 0;
  if (c.has_flex) {
    cr0 = carry_in<false>(tot2, blk0, nbM, sh);
    cr1 = cr0 + (blk0 < nbM ? tot2[blk0] : 0.0);
  }
  double acc = 0;
  for (int k = 0; k < AE; ++k) {
    const long long b = b0 + threadIdx.x + (long long)k * AT;
    if (b >= B) continue;
    double tl = 0;
    if (c.has_flex && b >= 2) {
      const long long j = b - 2;
      tl = loc[j] + ((int)(j / ABLK) == blk0 ? cr0 : cr1);
    }
    double d = c.vslope[b] * ssl + tl - T * c.sc[b];
    if (c.has_flex) d += sf_ * c.Qf[b];
    if (c.has_asp) d += sa_ * c.Qa[b];
    dapre[b] = d;
    acc += c.mspec[b] * d;
  }
  (void)tfl;
  const double s = block_total(acc, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// J7: da from dapre and dS = sum(part)
__global__ __launch_bounds__(AT) void amp_jvp_7(AmpConst c_, const AmpConst* __restrict__ dcs, const double* tfl, const double* tzm,
                                                const double* __restrict__ dapre, const double* __restrict__ part,
                                                int npart, double* __restrict__ da, long long ls, long long vs, long long wsd,
                                                long long des) {
  const AmpConst c = dcs ? dcs[blockIdx.y] : c_;
  if (tfl) tfl += blockIdx.y * ls;
  if (tzm) tzm += blockIdx.y * ls;
  dapre += blockIdx.y * wsd;
  part += blockIdx.y * wsd;
  da += blockIdx.y * vs;
  __shared__ double sh[2 * AT];
  double s = 0;
  for (int i = threadIdx.x; i < npart; i += AT) s += part[i];
  const double dS = block_total(s, sh);
  const double dfl = c.fl * c.ls_f * tfl[0];
  const long long B = c.B;
  for (long long b = (long long)blockIdx.x * AT + threadIdx.x; b < B; b += (long long)gridDim.x * AT) {
    double v;
    if (b == 0) {
      v = c.has_zm ? c.zm * c.ls_o * tzm[0] : 0.0;
    } else {
      const double An = c.An[b];
      v = dfl * An + c.fl * An * (dapre[b] / 2. - dS / (2. * c.S));
    }
    da[b * des] = v * c.total_volume;
  }
}

// ------------------------------------------------------------------ VJP
// V1: partials of R1 = sum_{b>=1} TV*g_b*An_b
__global__ __launch_bounds__(AT) void amp_vjp_1(AmpConst c_, const AmpConst* __restrict__ dcs, const double* __restrict__ g, double* __restrict__ part, long long ls, long long vs, long long wsd) {
  const AmpConst c = dcs ? dcs[blockIdx.y] : c_;
  g += blockIdx.y * vs;
  part += blockIdx.y * wsd;
  __shared__ double sh[2 * AT];
  double s = 0;
  for (long long b = (long long)blockIdx.x * AT + threadIdx.x; b < c.B; b += (long long)gridDim.x * AT)
    if (b > 0) s += c.total_volume * g[b] * c.An[b];
  s = block_total(s, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// V2: gapre; partials R2 = sum vslope*gapre, R3 = sum gapre*sc
__global__ __launch_bounds__(AT) void amp_vjp_2(AmpConst c_, const AmpConst* __restrict__ dcs, const double* __restrict__ g,
                                                const double* __restrict__ part1, int np1,
                                                double* __restrict__ gapre, double* __restrict__ part23, long long ls, long long vs, long long wsd) {
  const AmpConst c = dcs ? dcs[blockIdx.y] : c_;
  g += blockIdx.y * vs;
  part1 += blockIdx.y * wsd;
  gapre += blockIdx.y * wsd;
  part23 += blockIdx.y * wsd;
  __shared__ double sh[2 * AT];
  double s = 0;
  for (int i = threadIdx.x; i < np1; i += AT) s += part1[i];
  const double R1 = block_total(s, sh);
  const double k = c.fl * R1 / (2. * c.S);
  double r2 = 0, r3 = 0;
  for (long long b = (long long)blockIdx.x * AT + threadIdx.x; b < c.B; b += (long long)gridDim.x * AT) {
    const double gm = b > 0 ? c.total_volume * g[b] : 0.0;
    const double gAn = c.fl * gm;
    const double ga = c.An[b] * gAn / 2. - c.mspec[b] * k;
    gapre[b] = ga;
    r2 += c.vslope[b] * ga;
    r3 += ga * c.sc[b];
  }
  r2 = block_total(r2, sh);
  r3 = block_total(r3, sh);
  if (threadIdx.x == 0) {
    part23[2 * blockIdx.x] = r2;
    part23[2 * blockIdx.x + 1] = r3;
  }
}

// gtl[2+j] = gapre[2+j], minus R3 at the last bin
__device__ __forceinline__ double gtl_at(const AmpConst& c, const double* gapre, long long j, double R3) {
  const long long b = j + 2;
  return gapre[b] - (b == c.B - 1 ? R3 : 0.0);
}

// V3: reverse local scan of gtl[2:] -> y (local) ; totals
__global__ __launch_bounds__(AT) void amp_vjp_3(AmpConst c_, const AmpConst* __restrict__ dcs, const double* __restrict__ gapre,
                                                const double* __restrict__ part23, int np,
                                                double* __restrict__ loc, double* __restrict__ tot, long long ls, long long vs, long long wsd) {
  const AmpConst c = dcs ? dcs[blockIdx.y] : c_;
  gapre += blockIdx.y * wsd;
  part23 += blockIdx.y * wsd;
  loc += blockIdx.y * wsd;
  tot += blockIdx.y * wsd;
  __shared__ double sh[2 * AT];
  double s = 0;
  for (int i = threadIdx.x; i < np; i += AT) s += part23[2 * i + 1];
  const double R3 = block_total(s, sh);
  const long long M = c.B - 2;
  const long long j0 = (long long)blockIdx.x * ABLK + threadIdx.x;
  double v[AE];
#pragma unroll
  for (int k = 0; k < AE; ++k) {
    long long j = j0 + (long long)k * AT;
    v[k] = j < M ? gtl_at(c, gapre, j, R3) : 0.0;
  }
  double t = block_scan<true>(v, sh);
#pragma unroll
  for (int k = 0; k < AE; ++k)
    if (j0 + (long long)k * AT < M) loc[j0 + (long long)k * AT] = v[k];
  if (threadIdx.x == 0) tot[blockIdx.x] = t;
}

// V4: y = loc + suffix carry (g0); z = y*lv/2; w = z_j + z_{j+1}; reverse local scan of w
__global__ __launch_bounds__(AT) void amp_vjp_4(AmpConst c_, const AmpConst* __restrict__ dcs, const double* __restrict__ gapre,
                                                const double* __restrict__ part23, int np,
                                                const double* __restrict__ tot3, double* __restrict__ y,
                                                double* __restrict__ loc, double* __restrict__ tot4, long long ls, long long vs, long long wsd) {
  const AmpConst c = dcs ? dcs[blockIdx.y] : c_;
  gapre += blockIdx.y * wsd;
  part23 += blockIdx.y * wsd;
  tot3 += blockIdx.y * wsd;
  y += blockIdx.y * wsd;
  loc += blockIdx.y * wsd;
  tot4 += blockIdx.y * wsd;
  __shared__ double sh[2 * AT];
  double s = 0;
  for (int i = threadIdx.x; i < np; i += AT) s += part23[2 * i + 1];
  const double R3 = block_total(s, sh);
  const long long M = c.B - 2;
  const int nb = (int)((M + ABLK - 1) / ABLK);
  const double carry = carry_in<true>(tot3, blockIdx.x, nb, sh);
  const long long j0 = (long long)blockIdx.x * ABLK + threadIdx.x;
  double v[AE];
#pragma unroll
  for (int k = 0; k < AE; ++k) {
    long long j = j0 + (long long)k * AT;
    if (j < M) {
      const double yj = y[j] = loc[j] + carry;
      const double zj = yj * c.lv[j] / 2.;
      double zn = 0.0;
      if (j + 1 < M) zn = (yj - gtl_at(c, gapre, j, R3)) * c.lv[j + 1] / 2.;
      v[k] = zj + zn;
    } else {
      v[k] = 0.0;
    }
  }
  double t = block_scan<true>(v, sh);
#pragma unroll
  for (int k = 0; k < AE; ++k)
    if (j0 + (long long)k * AT < M) loc[j0 + (long long)k * AT] = v[k];
  if (threadIdx.x == 0) tot4[blockIdx.x] = t;
}



// V5: g1 = loc + carry; spectrum cotangents; partials R4, R5
__global__ __launch_bounds__(AT) void amp_vjp_5(AmpConst c_, const AmpConst* __restrict__ dcs, AmpOut o, const double* __restrict__ y,
                                                const double* __restrict__ loc, const double* __restrict__ tot4,
                                                double* __restrict__ part45, long long ls, long long vs, long long wsd) {
  const AmpConst c = dcs ? dcs[blockIdx.y] : c_;
  amp_out_offset(o, blockIdx.y * ls);
  y += blockIdx.y * wsd;
  loc += blockIdx.y * wsd;
  tot4 += blockIdx.y * wsd;
  part45 += blockIdx.y * wsd;
  __shared__ double sh[2 * AT];
  const long long M = c.B - 2;
  const int nb = (int)((M + ABLK - 1) / ABLK);
  const double carry = carry_in<true>(tot4, blockIdx.x, nb, sh);
  const long long j0 = (long long)blockIdx.x * ABLK + threadIdx.x;
  double r4 = 0, r5 = 0;
#pragma unroll
  for (int k = 0; k < AE; ++k) {
    long long j = j0 + (long long)k * AT;
    if (j < M) {
      const double g0 = y[j];
      const double g1 = loc[j] + carry;
      double s0 = g0 * c.c0[j], s1 = g1 * c.sf[j];
      if (o.dspec) {
        s0 += o.shift * o.dspec[j];
        s1 += o.shift * o.dspec[M + j];
      }
      o.spec[j] = s0;
      o.spec[M + j] = s1;
      r4 += g0 * c.p0[j] + g1 * c.p2[j];
      if (c.has_asp) r5 += g0 * c.p1[j];
    }
  }
  r4 = block_total(r4, sh);
  r5 = block_total(r5, sh);
  if (threadIdx.x == 0) {
    part45[2 * blockIdx.x] = r4;
    part45[2 * blockIdx.x + 1] = r5;
  }
}

// V6: scalar cotangents (one block)
__global__ __launch_bounds__(AT) void amp_vjp_6(AmpConst c_, const AmpConst* __restrict__ dcs, AmpOut o, const double* __restrict__ g,
                                                const double* __restrict__ part1, int np1,
                                                const double* __restrict__ part23, int np23,
                                                const double* __restrict__ part45, int np45, long long ls, long long vs, long long wsd) {
  const AmpConst c = dcs ? dcs[blockIdx.y] : c_;
  amp_out_offset(o, blockIdx.y * ls);
  g += blockIdx.y * vs;
  part1 += blockIdx.y * wsd;
  part23 += blockIdx.y * wsd;
  part45 += blockIdx.y * wsd;
  __shared__ double sh[2 * AT];
  double a = 0, b2 = 0, b4 = 0, b5 = 0;
  for (int i = threadIdx.x; i < np1; i += AT) a += part1[i];
  for (int i = threadIdx.x; i < np23; i += AT) b2 += part23[2 * i];
  for (int i = threadIdx.x; i < np45; i += AT) {
    b4 += part45[2 * i];
    b5 += part45[2 * i + 1];
  }
  const double R1 = block_total(a, sh);
  const double R2 = block_total(b2, sh);
  const double R4 = block_total(b4, sh);
  const double R5 = block_total(b5, sh);
  if (threadIdx.x == 0) {
    const double sh_ = o.shift;
    o.fl[0] = c.fl * c.ls_f * R1 + (o.dfl ? sh_ * o.dfl[0] : 0.0);
    o.sl[0] = c.sig_s * R2 + (o.dsl ? sh_ * o.dsl[0] : 0.0);
    if (c.has_flex) o.flex[0] = R4 + (o.dflex ? sh_ * o.dflex[0] : 0.0);
    if (c.has_asp) o.asp[0] = R5 + (o.dasp ? sh_ * o.dasp[0] : 0.0);
    if (c.has_zm) o.zm[0] = c.zm * c.ls_o * c.total_volume * g[0] + (o.dzm ? sh_ * o.dzm[0] : 0.0);
  }
}

static int nblk(long long n, int per) { return (int)std::max<long long>(1, (n + per - 1) / per); }

}  // namespace nft

using namespace nft;

extern "C" {

size_t nft_amp_workspace(int64_t B) { return (size_t)(3 * B + 16 * (B / 256 + 16)) * sizeof(double); }

int nft_amp_jvp_batched(const nft_amp_const* cst, const nft_amp_const* dcs, const double* tfl, const double* tsl,
                        const double* tflex, const double* tasp, const double* tzm, const double* tspec, double* da,
                        double* ws, int nrhs, int64_t lat_stride, int64_t da_stride, int64_t da_elem_stride,
                        hipStream_t s) {
  const AmpConst& c = *cst;
  const long long B = c.B, M = B - 2;
  const long long wsd = (long long)(nft_amp_workspace(B) / sizeof(double));
  const long long ls = lat_stride, vs = da_stride;
  double* loc = ws;                 // M
  double* dapre = ws + B;           // B
  double* tot1 = ws + 2 * B;        // nbM
  const int nbM = nblk(M, ABLK);
  double* tot2 = tot1 + nbM + 1;
  const int nbB = nblk(B, ABLK);
  double* part = tot2 + nbM + 1;
  const unsigned ny = (unsigned)nrhs;
  if (c.has_flex) {
    prof_mark(s, "amp_jvp_1");
    hipLaunchKernelGGL(amp_jvp_1, dim3(nbM, ny), dim3(AT), 0, s, c, dcs, tspec, loc, tot1, ls, vs, wsd);
    prof_mark(s, "amp_jvp_3");
    hipLaunchKernelGGL(amp_jvp_3, dim3(nbM, ny), dim3(AT), 0, s, c, dcs, tspec, tot1, loc, tot2, ls, vs, wsd);
  }
  prof_mark(s, "amp_jvp_5");
  hipLaunchKernelGGL(amp_jvp_5, dim3(nbB, ny), dim3(AT), 0, s, c, dcs, tfl, tsl, tflex, tasp, loc, tot2, dapre, part, ls,
                     vs, wsd);
  prof_mark(s, "amp_jvp_7");
  hipLaunchKernelGGL(amp_jvp_7, dim3(nblk(B, AT) < 1024 ? nblk(B, AT) : 1024, ny), dim3(AT), 0, s, c, dcs, tfl, tzm,
                     dapre, part, nbB, da, ls, vs, wsd, (long long)(da_elem_stride > 0 ? da_elem_stride : 1));
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

int nft_amp_jvp(const nft_amp_const* cst, const double* tfl, const double* tsl, const double* tflex,
                const double* tasp, const double* tzm, const double* tspec, double* da, double* ws, hipStream_t s) {
  return nft_amp_jvp_batched(cst, nullptr, tfl, tsl, tflex, tasp, tzm, tspec, da, ws, 1, 0, 0, 1, s);
}

int nft_amp_vjp_batched(const nft_amp_const* cst, const nft_amp_const* dcs, const double* g, const nft_amp_out* out,
                        double* ws, int nrhs, int64_t lat_stride, int64_t g_stride, hipStream_t s) {
  const AmpConst& c = *cst;
  const AmpOut& o = *out;
  const long long B = c.B, M = B - 2;
  const long long wsd = (long long)(nft_amp_workspace(B) / sizeof(double));
  const long long ls = lat_stride, vs = g_stride;
  double* gapre = ws;               // B
  double* loc = ws + B;             // M
  double* y = ws + 2 * B;           // M
  const int nbM = nblk(M, ABLK);
  const int nr = std::min(nblk(B, AT), 1024);
  double* part1 = ws + 3 * B;
  double* part23 = part1 + nr + 1;
  double* tot3 = part23 + 2 * nr + 2;
  double* tot4 = tot3 + nbM + 1;
  double* part45 = tot4 + nbM + 1;
  const unsigned ny = (unsigned)nrhs;
  prof_mark(s, "amp_vjp_1");
  hipLaunchKernelGGL(amp_vjp_1, dim3(nr, ny), dim3(AT), 0, s, c, dcs, g, part1, ls, vs, wsd);
  prof_mark(s, "amp_vjp_2");
  hipLaunchKernelGGL(amp_vjp_2, dim3(nr, ny), dim3(AT), 0, s, c, dcs, g, part1, nr, gapre, part23, ls, vs, wsd);
  if (c.has_flex) {
    prof_mark(s, "amp_vjp_3");
    hipLaunchKernelGGL(amp_vjp_3, dim3(nbM, ny), dim3(AT), 0, s, c, dcs, gapre, part23, nr, loc, tot3, ls, vs, wsd);
    prof_mark(s, "amp_vjp_4");
    hipLaunchKernelGGL(amp_vjp_4, dim3(nbM, ny), dim3(AT), 0, s, c, dcs, gapre, part23, nr, tot3, y, loc, tot4, ls, vs,
                       wsd);
    prof_mark(s, "amp_vjp_5");
    hipLaunchKernelGGL(amp_vjp_5, dim3(nbM, ny), dim3(AT), 0, s, c, dcs, o, y, loc, tot4, part45, ls, vs, wsd);
  }
  prof_mark(s, "amp_vjp_6");
  hipLaunchKernelGGL(amp_vjp_6, dim3(1, ny), dim3(AT), 0, s, c, dcs, o, g, part1, nr, part23, nr, part45,
                     c.has_flex ? nbM : 0, ls, vs, wsd);
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

int nft_amp_vjp(const nft_amp_const* cst, const double* g, const nft_amp_out* out, double* ws, hipStream_t s) {
  return nft_amp_vjp_batched(cst, nullptr, g, out, ws, 1, 0, 0, s);
}

}  // extern "C"
