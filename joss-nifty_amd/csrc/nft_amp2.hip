// Correlated-field amplitude Jacobian, two launches per JVP / VJP, carrying
// the amplitude keys' CG direction (JVP) and the CG update + finalize (VJP).
//
// Same operator as nft_amp.hip (reference: src/library/correlated_fields.py
// :105-212 -- _SlopeRemover, _TwoLogIntegrations, _Normalization --, and the
// scalings of correlated_fields_simple.py:86-127), linearised at one
// expansion point.  The JVP / VJP are linear in the tangent / cotangent; the
// two cumulative sums of the integrated Wiener process and the normalisation
// make every bin depend on global quantities (scan carries of earlier / later
// bins, the slope remover's last value T, the normalisation sums), all of them
// LINEAR in the tangent.  The bins are cut into tiles; then
//
//   JVP   c_j  = loc1_j + C1(i)                       C1(i) = sum_{t<i} a1(t)
//         tl_j = loc2_j + C1(i) LVc_j + C2(i)         C2(i) = sum_{t<i} a2(t) + C1(t) LVt(t)
//         dS   = sum_t m1(t) + C2(t) MS2(t) + C1(t) MS3(t)  + ssl KV + sflex KF + sasp KA - T M4
//   VJP   y_j  = yG_j - k ym_j + beta(i)              beta(i) = SG(i) - k SM(i) - R3
//         g1_j = g1G_j - k g1m_j + beta(i) g1l_j + S1(i)
//
// (loc*, yG, g1G: tile-local scans of the tangent / cotangent).  Everything
// that involves the expansion point alone -- the constant scans ym, g1m, g1l,
// LVc, the constant tile sums MS2, MS3, AWM, ... and the global sums M4, KV,
// KF, KA -- is formed ONCE per linearisation point (nft_amp2_prepare, tables
// at nft_amp_const.tab), and every tile sum the carries need from the
// tangent is a DOT PRODUCT of the tangent with a constant vector ("sum_j y_j
// c_j" with y a tile-local reverse scan of G is "sum_j G_j F(c)_j" with F(c)
// the tile-local forward scan of c, and vice versa):
//
//   a1 = d1.sf      a2 = d0.c0 + d1.ka      m1 = d0.(c0 RM) + d1.kb      (JVP)
//   aggG = G.1   AWG = G.k1   P0G = G.k2   Q2G = G.k3   P1G = G.k4        (VJP)
//
// so the first launch of each (phase A) is a pure streaming pass: no scans,
// one workgroup per tile for a group of right-hand sides that share constants
// (the constants are read once and held once in registers); the last
// workgroup of a group to finish forms the carries of every tile (fixed-order
// scans over the tile sums).  The second launch (phase B) reads its tile's
// carries, redoes the tile-local scans of the tangent / cotangent and writes
// the outputs (the VJP's: the CG update, and in the last workgroup of a group
// the CG finalize).  All sums are fixed-order, so results are deterministic
// and, per right-hand side, independent of how many share the launch.
//
// Concurrency: the finalize's arrival counters are one device-global set, so
// these kernels must not run concurrently on two streams (the library's
// contract: one stream per device, include/nifty_amd.h).
#include <algorithm>
#include <cstdlib>

#include "nft_api_internal.hpp"
#include "../../include/nifty_amd.h"

namespace nft {
namespace amp2 {

using AmpConst = nft_amp_const;
constexpr int NT = 512;   // threads per workgroup, one bin per thread per sub-chunk
constexpr int NW = NT / 64;
constexpr int MAXNB = 640;  // tiles per right-hand side at most: the tile grows with B
constexpr int MAXR = 256;   // right-hand sides per launch
constexpr int NS_ = NFT_CG_NSCALARS;
constexpr int TPT = (MAXNB + NT - 1) / NT;  // tiles per thread in the carry scans

enum { KFL = 0, KSL = 1, KFLEX = 2, KASP = 3, KZM = 4, KSPEC = 5 };

// ---------------------------------------------------------------- tables
// per-bin tables (M each, padded): JVP ka, c0RM, kb, LVc; VJP k1..k4, ym, g1m, g1l
enum { T_KA = 0, T_C0RM, T_KB, T_LVC, T_K1, T_K2, T_K3, T_K4, T_YM, T_G1M, T_G1L, T_N };
// constant tile rows (nb each, padded); P*: per-tile partials of the globals
enum { R_LVT = 0, R_MS2, R_MS3, R_AWM, R_AWL, R_P0M, R_P0S, R_Q2M, R_Q2L, R_P2S, R_P1M, R_P1S, R_SM, R_PM4, R_PKV,
       R_PKF, R_PKA, R_N };
// globals: M4 = sum msv sc, KV = sum msv vslope, KF = sum msv Qf, KA = sum msv Qa (all bins)
enum { G_M4 = 0, G_KV, G_KF, G_KA, G_N = 8 };

struct Geo {
  int M, sub, nb;         // spectrum bins, sub-chunks per tile, tiles
  long long Mp, nbp;      // padded strides
  __host__ __device__ long long tl() const { return (long long)sub * NT; }
};
__host__ __device__ inline Geo geo_of(long long B) {
  Geo g;
  const long long M = B - 2 > 0 ? B - 2 : 1;
  int s = 1;
  while ((M + (long long)s * NT - 1) / ((long long)s * NT) > MAXNB) s *= 2;
  g.M = (int)(B - 2);
  g.sub = s;
  g.nb = (int)((M + (long long)s * NT - 1) / ((long long)s * NT));
  g.Mp = (M + 63) & ~63LL;
  g.nbp = ((long long)g.nb + 63) & ~63LL;
  return g;
}
__host__ __device__ inline long long tab_len(const Geo& g) { return (long long)T_N * g.Mp + (long long)R_N * g.nbp + G_N; }
__device__ __forceinline__ const double* tabv(const double* t, const Geo& g, int q) { return t + (long long)q * g.Mp; }
__device__ __forceinline__ const double* tabr(const double* t, const Geo& g, int q) {
  return t + (long long)T_N * g.Mp + (long long)q * g.nbp;
}
__device__ __forceinline__ const double* tabg(const double* t, const Geo& g) {
  return t + (long long)T_N * g.Mp + (long long)R_N * g.nbp;
}

// the per-bin arrays are read through pointers loaded from a struct: cast
// them to the global address space (else flat loads, waited on with LDS)
typedef __attribute__((address_space(1))) const double gdouble;
__device__ __forceinline__ gdouble* G_(const double* p) { return (gdouble*)p; }

// constant sets: by value (kernel argument) or from device memory through
// the constant address space (pointers land in SGPRs)
typedef __attribute__((address_space(4))) const unsigned long long cword;
static_assert(sizeof(AmpConst) % 8 == 0, "nft_amp_const is read as 64-bit words");
__device__ __forceinline__ AmpConst load_const(const AmpConst* p) {
  AmpConst v;
  unsigned long long* d = (unsigned long long*)&v;
  cword* q = (cword*)p;
#pragma unroll
  for (int k = 0; k < (int)(sizeof(AmpConst) / 8); ++k) d[k] = q[k];
  return v;
}
// MODE 0: the host set (argument); 1: one device set per RHS; 2: one device set for all
template <int MODE>
__device__ __forceinline__ AmpConst const_of(const AmpConst& c, const AmpConst* dcs, const AmpConst* dc1, int r) {
  if constexpr (MODE == 1) return load_const(dcs + r);
  else if constexpr (MODE == 2) return load_const(dc1);
  else return c;
}

// ------------------------------------------------------------ block helpers
// NV block totals at once: per value the wave tree, then the waves in order
// (value by value, so that the tree needs one temporary)
template <int NV>
__device__ __forceinline__ void btot(double (&v)[NV], double* sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v[k] += __shfl_down(v[k], off, 64);
  }
  __syncthreads();
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k) sh[k * NW + w] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    double t = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) t += sh[k * NW + i];
    v[k] = t;
  }
  __syncthreads();
}

// NV block totals into LDS: after the call, total k is at sh[NV * NW + k]
// (thread k sums the wave totals of value k in wave order; nobody holds all
// NV * NW partials in registers).  sh: NV * (NW + 1) doubles.
template <int NV>
__device__ __forceinline__ void btot_sh(double (&v)[NV], double* sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v[k] += __shfl_down(v[k], off, 64);
  }
  __syncthreads();
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k) sh[k * NW + w] = v[k];
  }
  __syncthreads();
  if (threadIdx.x < NV) {
    const int k = threadIdx.x;
    double t = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) t += sh[k * NW + i];
    sh[NV * NW + k] = t;
  }
  __syncthreads();
}

// inclusive block scans of NA arrays (one value per thread, thread order),
// forward or reversed: wave scans by shuffles; then thread (a, w) forms the
// fixed-order sum of the waves before (after) wave w for array a, so every
// thread reads one offset per array.  tot: the block totals.  sh: NA (2 NW
// + 1) doubles.
template <int NA, bool REV>
__device__ __forceinline__ void bscan(double (&v)[NA], double (&tot)[NA], double* sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    double y[NA];
#pragma unroll
    for (int a = 0; a < NA; ++a) y[a] = REV ? __shfl_down(v[a], off, 64) : __shfl_up(v[a], off, 64);
    const bool take = REV ? (lane + off < 64) : (lane >= off);
#pragma unroll
    for (int a = 0; a < NA; ++a)
      if (take) v[a] += y[a];
  }
  if (lane == (REV ? 0 : 63)) {
#pragma unroll
    for (int a = 0; a < NA; ++a) sh[a * NW + w] = v[a];
  }
  __syncthreads();
  if (threadIdx.x < NA * NW) {
    const int a = threadIdx.x / NW, w2 = threadIdx.x - a * NW;
    double off = 0.0, run = 0.0;
    if (!REV) {
#pragma unroll
      for (int q = 0; q < NW; ++q) {
        if (q < w2) off += sh[a * NW + q];
        run += sh[a * NW + q];
      }
    } else {
#pragma unroll
      for (int q = NW - 1; q >= 0; --q) {
        if (q > w2) off += sh[a * NW + q];
        run += sh[a * NW + q];
      }
    }
    sh[NA * NW + a * NW + w2] = off;
    if (w2 == 0) sh[2 * NA * NW + a] = run;
  }
  __syncthreads();
#pragma unroll
  for (int a = 0; a < NA; ++a) {
    v[a] += sh[NA * NW + a * NW + w];
    tot[a] = sh[2 * NA * NW + a];
  }
  __syncthreads();
}

// exclusive scans over the tiles (nb <= MAXNB values, TPT per thread in
// chunks of NT, thread order within a chunk), forward or reversed, of NA rows
// at once; x[a][c] is tile c * NT + tid (0 past nb)
template <int NA, bool REV>
__device__ __forceinline__ void tile_scan(const double (&x)[NA][TPT], double (&ex)[NA][TPT], double (&tot)[NA],
                                          double* sh) {
  double run[NA];
#pragma unroll
  for (int a = 0; a < NA; ++a) run[a] = 0.0;
#pragma unroll
  for (int cc = 0; cc < TPT; ++cc) {
    const int c = REV ? TPT - 1 - cc : cc;
    double v[NA], t[NA];
#pragma unroll
    for (int a = 0; a < NA; ++a) v[a] = x[a][c];
    bscan<NA, REV>(v, t, sh);
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      ex[a][c] = run[a] + (v[a] - x[a][c]);
      run[a] += t[a];
    }
  }
#pragma unroll
  for (int a = 0; a < NA; ++a) tot[a] = run[a];
}

// ------------------------------------------------------------ arrival
// Arrival counters of the VJP's finalize (per group of right-hand sides):
// arrival i of n counts at group counter i % 16, the last arrival of a group
// at the top counter (hundreds of atomics on one address serialise at the
// memory-side atomic unit, sixteen lines do not); each counter is reset by
// the arrival that completes it.  Release / acquire at agent scope: the
// partials a workgroup stored before it arrives are visible to the last one.
constexpr int NGRP = 16;
struct Line {
  unsigned v[16];  // one 64-byte line per counter
};
__device__ Line g_arrive[3][MAXR][NGRP + 1];  // jvp_a, vjp_a, vjp_b

__device__ __forceinline__ bool last_arrival(Line* ctr, int idx, int n, int* lds_flag) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const int ng = n < NGRP ? n : NGRP;
    const int q = idx % ng;
    const unsigned gsz = (unsigned)(n / ng + (q < n % ng ? 1 : 0));
    bool last = false;
    if (__hip_atomic_fetch_add(&ctr[q].v[0], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gsz - 1) {
      __hip_atomic_store(&ctr[q].v[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__hip_atomic_fetch_add(&ctr[NGRP].v[0], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
          (unsigned)ng - 1) {
        __hip_atomic_store(&ctr[NGRP].v[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = true;
      }
    }
    *lds_flag = last ? 1 : 0;
  }
  __syncthreads();
  const bool last = *lds_flag != 0;
  if (last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return last;
}

__device__ __forceinline__ double beta_of(const double* scb) {
  double beta = scb[NFT_CG_GAMMA] / scb[NFT_CG_GPREV];
  if (!(beta > 0.0)) beta = 0.0;
  return beta;
}

// workgroup -> (tile, group of KG right-hand sides); RHS r = g * KG + q
__device__ __forceinline__ void place(int nb, int& tile, int& grp) {
  tile = (int)(blockIdx.x % (unsigned)nb);
  grp = (int)(blockIdx.x / (unsigned)nb);
}

// ================================================================= PREPARE
struct PrepArgs {
  AmpConst c;              // host set (item_consts NULL) or B + flags
  AmpConst* dcs;           // device sets (one per row) or null
  double* tab;             // row r's tables at tab + r * ts
  long long ts;
  int nrow;
};

// one workgroup per (tile, row): the constant tile-local scans -> tables,
// the constant tile sums -> rows
template <bool DEV>
__global__ __launch_bounds__(NT) void prep_tiles(PrepArgs a) {
#pragma clang fp contract(off)
  __shared__ double sh[(R_P1S + 5) * (NW + 1)];
  const Geo g = geo_of(a.c.B);
  const int i = (int)(blockIdx.x % (unsigned)g.nb), r = (int)(blockIdx.x / (unsigned)g.nb);
  const AmpConst c = DEV ? load_const(a.dcs + r) : a.c;
  double* tab = a.tab + (long long)r * a.ts;
  const int tid = threadIdx.x;
  const bool flex = c.has_flex, asp = c.has_asp;
  const long long j0 = (long long)i * g.tl();
  auto T = [&](int q) { return tab + (long long)q * g.Mp; };
  auto R = [&](int q) { return tab + (long long)T_N * g.Mp + (long long)q * g.nbp; };
  // globals' partials over the tile's bins (+ bins 0, 1 in tile 0)
  double pg[4] = {0.0, 0.0, 0.0, 0.0};  // msv sc, msv vsl, msv Qf, msv Qa
  // row sums
  double rs[R_P1S + 1];
#pragma unroll
  for (int q = 0; q <= R_P1S; ++q) rs[q] = 0.0;
  // forward pass over the sub-chunks: LVc, k1 = F(l1) - l2, k2 = F(p0),
  // k3 = F(l1 p2c) - l2 p2c with p2c = F(p2), k4 = F(p1)
  double cf[5] = {0.0, 0.0, 0.0, 0.0, 0.0};  // running carries: lv, l1, p2, l1 p2c, p0 (p1 below)
  double cp1 = 0.0;
  for (int s = 0; s < g.sub; ++s) {
    const long long j = j0 + (long long)s * NT + tid;
    const bool ok = j < g.M;
    const long long b = j + 2;
    const double msv = ok ? G_(c.mspec)[b] : 0.0;
    const double scv = ok ? G_(c.sc)[b] : 0.0;
    const double vsl = ok ? G_(c.vslope)[b] : 0.0;
    pg[0] += msv * scv;
    pg[1] += msv * vsl;
    if (flex) pg[2] += msv * (ok ? G_(c.Qf)[b] : 0.0);
    if (asp) pg[3] += msv * (ok ? G_(c.Qa)[b] : 0.0);
    if (!flex) continue;
    const bool okf = ok;
    const double lv = okf ? G_(c.lv)[j] : 0.0;
    const double lvn = (okf && j + 1 < g.M) ? G_(c.lv)[j + 1] : 0.0;
    const double l1 = lv / 2. + lvn / 2., l2 = lvn / 2.;
    const double p0 = okf ? G_(c.p0)[j] : 0.0;
    const double p1 = (okf && asp) ? G_(c.p1)[j] : 0.0;
    const double p2 = okf ? G_(c.p2)[j] : 0.0;
    double v[6] = {lv, l1, p2, 0.0, p0, p1}, t[6];
    // p2c first (l1 p2c needs it): scan lv, l1, p2, p0, p1 together
    {
      double u[5] = {lv, l1, p2, p0, p1}, tu[5];
      bscan<5, false>(u, tu, sh);
      v[0] = u[0] + cf[0];
      v[1] = u[1] + cf[1];
      v[2] = u[2] + cf[2];
      v[4] = u[3] + cf[4];
      v[5] = u[4] + cp1;
      cf[0] += tu[0];
      cf[1] += tu[1];
      cf[2] += tu[2];
      cf[4] += tu[3];
      cp1 += tu[4];
    }
    const double p2c = v[2];
    double w3[1] = {l1 * p2c}, t3[1];
    bscan<1, false>(w3, t3, sh);
    const double f3 = w3[0] + cf[3];
    cf[3] += t3[0];
    (void)t;
    const double LVc = v[0];
    const double k1 = v[1] - l2, k2 = v[4], k3 = f3 - l2 * p2c, k4 = v[5];
    if (ok) {
      T(T_LVC)[j] = LVc;
      T(T_K1)[j] = k1;
      T(T_K2)[j] = k2;
      T(T_K3)[j] = k3;
      T(T_K4)[j] = asp ? k4 : 0.0;
    }
    rs[R_LVT] += lv;
    rs[R_MS2] += msv;
    rs[R_MS3] += msv * LVc;
    rs[R_AWL] += l1;
    rs[R_P0M] += msv * k2;
    rs[R_P0S] += p0;
    rs[R_Q2M] += msv * k3;
    rs[R_Q2L] += l1 * p2c;
    rs[R_P2S] += p2;
    rs[R_P1M] += msv * (asp ? k4 : 0.0);
    rs[R_P1S] += p1;
  }
  // reverse pass: RL = R(lv), RM = R(msv) = ym, RLM = R(lv RM), g1m = R(RM l1 - msv l2),
  // g1l = R(l1); ka = sf (RL - lv/2), c0RM = c0 RM, kb = sf (RLM - lv RM/2); AWM
  if (flex) {
    double cr[5] = {0.0, 0.0, 0.0, 0.0, 0.0};  // lv, msv, lv RM, w(msv), l1
    for (int s = g.sub - 1; s >= 0; --s) {
      const long long j = j0 + (long long)s * NT + tid;
      const bool ok = j < g.M;
      const long long b = j + 2;
      const double msv = ok ? G_(c.mspec)[b] : 0.0;
      const double lv = ok ? G_(c.lv)[j] : 0.0;
      const double lvn = (ok && j + 1 < g.M) ? G_(c.lv)[j + 1] : 0.0;
      const double l1 = lv / 2. + lvn / 2., l2 = lvn / 2.;
      const double sf = ok ? G_(c.sf)[j] : 0.0, c0 = ok ? G_(c.c0)[j] : 0.0;
      double u[3] = {lv, msv, l1}, tu[3];
      bscan<3, true>(u, tu, sh);
      const double RL = u[0] + cr[0], RM = u[1] + cr[1], G1L = u[2] + cr[4];
      cr[0] += tu[0];
      cr[1] += tu[1];
      cr[4] += tu[2];
      const double wm = RM * l1 - msv * l2;
      double u2[2] = {lv * RM, wm}, tu2[2];
      bscan<2, true>(u2, tu2, sh);
      const double RLM = u2[0] + cr[2], G1M = u2[1] + cr[3];
      cr[2] += tu2[0];
      cr[3] += tu2[1];
      if (ok) {
        T(T_KA)[j] = sf * (RL - lv / 2.);
        T(T_C0RM)[j] = c0 * RM;
        T(T_KB)[j] = sf * (RLM - lv * RM / 2.);
        T(T_YM)[j] = RM;
        T(T_G1M)[j] = G1M;
        T(T_G1L)[j] = G1L;
      }
      rs[R_AWM] += wm;
    }
  }
  if (i == 0 && tid < 2) {  // bins 0 and 1: no integrated part
    const int b = tid;
    const double ms = G_(c.mspec)[b];
    pg[0] += ms * G_(c.sc)[b];
    pg[1] += ms * G_(c.vslope)[b];
    if (flex) pg[2] += ms * G_(c.Qf)[b];
    if (asp) pg[3] += ms * G_(c.Qa)[b];
  }
  double all[R_P1S + 1 + 4];
#pragma unroll
  for (int q = 0; q <= R_P1S; ++q) all[q] = rs[q];
#pragma unroll
  for (int q = 0; q < 4; ++q) all[R_P1S + 1 + q] = pg[q];
  constexpr int NA = R_P1S + 1 + 4;
  btot_sh<NA>(all, sh);
  if (tid == 0) {
    const double* tot = sh + NA * NW;
#pragma unroll
    for (int q = 0; q <= R_P1S; ++q) R(q)[i] = tot[q];
    R(R_PM4)[i] = tot[R_P1S + 1];
    R(R_PKV)[i] = tot[R_P1S + 2];
    R(R_PKF)[i] = tot[R_P1S + 3];
    R(R_PKA)[i] = tot[R_P1S + 4];
  }
}

// one workgroup per row: SM (exclusive suffix of MS2 over the tiles) and the
// globals (fixed-order sums of the tile partials); sets the row's tab pointer
template <bool DEV>
__global__ __launch_bounds__(NT) void prep_globals(PrepArgs a) {
#pragma clang fp contract(off)
  __shared__ double sh[8 * NW];
  const Geo g = geo_of(a.c.B);
  const int r = blockIdx.x;
  double* tab = a.tab + (long long)r * a.ts;
  auto R = [&](int q) { return tab + (long long)T_N * g.Mp + (long long)q * g.nbp; };
  const int tid = threadIdx.x;
  double x[1][TPT], ex[1][TPT], tot[1];
  double p[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int cc = 0; cc < TPT; ++cc) {
    const int t = cc * NT + tid;
    const bool ok = t < g.nb;
    x[0][cc] = ok ? R(R_MS2)[t] : 0.0;
    p[0] += ok ? R(R_PM4)[t] : 0.0;
    p[1] += ok ? R(R_PKV)[t] : 0.0;
    p[2] += ok ? R(R_PKF)[t] : 0.0;
    p[3] += ok ? R(R_PKA)[t] : 0.0;
  }
  tile_scan<1, true>(x, ex, tot, sh);
#pragma unroll
  for (int cc = 0; cc < TPT; ++cc) {
    const int t = cc * NT + tid;
    if (t < g.nb) R(R_SM)[t] = ex[0][cc];
  }
  btot<4>(p, sh);
  if (tid == 0) {
    double* gl = tab + (long long)T_N * g.Mp + (long long)R_N * g.nbp;
    gl[G_M4] = p[0];
    gl[G_KV] = p[1];
    gl[G_KF] = p[2];
    gl[G_KA] = p[3];
    if (DEV) a.dcs[r].tab = tab;
  }
}

// ======================================================================= JVP
struct JvpArgs {
  AmpConst c;              // constants (shared by every RHS), B and flags
  const AmpConst* dcs;     // per-RHS constants (device) or null
  const AmpConst* dc1;     // one device constant set shared by every RHS, or null
  double* t[6];            // tangent keys of RHS 0 (rows ls apart); with dir the CG direction, updated in place
  const double* r[6];      // residual keys of RHS 0 (dir only)
  long long ls;
  double* da;              // da[r * vs + b * des]
  long long vs, des;
  double* ws;              // per-RHS workspace, wsd doubles apart
  long long wsd;
  int nrhs;
  int dir;                 // carry d = max(0, gamma/gprev) d + r on the amplitude keys
  const double* sc;        // CG scalar blocks (dir)
  double* part;            // d.d partials: part[r * pstride + tile] = shift * d.d (dir)
  long long pstride;
  double shift;
};

// workspace rows of one RHS (JVP): a1, a2, m1 (phase A) and the carries C1,
// C2 (phase A's last workgroup) [nbp each], then the scalars: the scalar
// keys' tangents after the direction update [5], T, ds
enum { W_A1 = 0, W_A2, W_M1, W_C1, W_C2, W_JN };
enum { J_T = 5, J_DS = 6 };
__device__ __forceinline__ double* wrow(double* W, const Geo& g, int q) { return W + (long long)q * g.nbp; }

// phase A: direction update and the tile's dot products a1, a2, m1 for each
// RHS of the group (+ tile 0: the scalar keys, stashed in the workspace)
template <int MODE, int KG>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(4))) void jvp_a(JvpArgs a) {
#pragma clang fp contract(off)
  __shared__ double sh[(4 * KG) * (NW + 1)];
  __shared__ int lflag;
  const Geo g = geo_of(a.c.B);
  int i, grp;
  place(g.nb, i, grp);
  const int tid = threadIdx.x;
  const AmpConst c = const_of<MODE>(a.c, a.dcs, a.dc1, grp * KG);
  const bool flex = a.c.has_flex, asp = a.c.has_asp;
  const double* tb = c.tab;
  if (!tb) return;  // constants without tables (nft_amp2_prepare not run): no access
  double bt[KG];
  bool live[KG], upd[KG], has[KG];
#pragma unroll
  for (int q = 0; q < KG; ++q) {
    const int r = grp * KG + q;
    has[q] = r < a.nrhs;
    bt[q] = 0.0;
    live[q] = false;
    if (a.dir && has[q]) {
      const double* scb = a.sc + (long long)r * NS_;
      live[q] = scb[NFT_CG_DONE] == 0.0;
      bt[q] = beta_of(scb);
    }
    upd[q] = a.dir && live[q];
  }
  // a1, a2, m1, dd per RHS
  double s[4 * KG];
#pragma unroll
  for (int k = 0; k < 4 * KG; ++k) s[k] = 0.0;
  if (flex) {
    const long long j0 = (long long)i * g.tl();
    for (int sc_ = 0; sc_ < g.sub; ++sc_) {
      const long long j = j0 + (long long)sc_ * NT + tid;
      const bool ok = j < g.M;
      double sf = 0, c0 = 0, ka = 0, c0rm = 0, kb = 0;
      if (ok) {
        sf = G_(c.sf)[j];
        c0 = G_(c.c0)[j];
        ka = G_(tabv(tb, g, T_KA))[j];
        c0rm = G_(tabv(tb, g, T_C0RM))[j];
        kb = G_(tabv(tb, g, T_KB))[j];
      }
      double d0[KG], d1[KG], r0[KG], r1[KG];
#pragma unroll
      for (int q = 0; q < KG; ++q) {
        const long long ro = (long long)(grp * KG + q) * a.ls;
        const bool okq = ok && has[q];
        d0[q] = okq ? a.t[KSPEC][ro + j] : 0.0;
        d1[q] = okq ? a.t[KSPEC][ro + g.M + j] : 0.0;
        r0[q] = (okq && upd[q]) ? a.r[KSPEC][ro + j] : 0.0;
        r1[q] = (okq && upd[q]) ? a.r[KSPEC][ro + g.M + j] : 0.0;
      }
#pragma unroll
      for (int q = 0; q < KG; ++q) {
        if (ok && upd[q] && has[q]) {
          const long long ro = (long long)(grp * KG + q) * a.ls;
          d0[q] = bt[q] * d0[q] + r0[q];
          d1[q] = bt[q] * d1[q] + r1[q];
          a.t[KSPEC][ro + j] = d0[q];
          a.t[KSPEC][ro + g.M + j] = d1[q];
          s[4 * q + 3] += d0[q] * d0[q] + d1[q] * d1[q];
        }
        s[4 * q + 0] += d1[q] * sf;
        s[4 * q + 1] += d0[q] * c0 + d1[q] * ka;
        s[4 * q + 2] += d0[q] * c0rm + d1[q] * kb;
      }
    }
  }
  btot_sh<4 * KG>(s, sh);
  const double* tot = sh + 4 * KG * NW;
#pragma unroll
  for (int q = 0; q < KG; ++q) if (tid == q) {
    const int r = grp * KG + q;
    if (has[q]) {
      double* W = a.ws + (long long)r * a.wsd;
      wrow(W, g, W_A1)[i] = tot[4 * q + 0];
      wrow(W, g, W_A2)[i] = tot[4 * q + 1];
      wrow(W, g, W_M1)[i] = tot[4 * q + 2];
      double v = tot[4 * q + 3];
      if (i == 0) {
        // the scalar keys: new direction stashed (phase B writes it back: the
        // other workgroups of this launch still read the old one)
        const long long ro = (long long)r * a.ls;
        double* stash = wrow(W, g, W_JN);
#pragma unroll
        for (int k = 0; k < 5; ++k) {
          double sv = 0.0;
          if (a.t[k] && !(k == KFLEX && !flex) && !(k == KASP && !asp) && !(k == KZM && !a.c.has_zm)) {
            sv = a.t[k][ro];
            if (upd[q]) sv = bt[q] * sv + a.r[k][ro];
          }
          stash[k] = sv;
          if (a.dir) v += sv * sv;
        }
      }
      if (a.dir) a.part[(long long)r * a.pstride + i] = live[q] ? a.shift * v : 0.0;
    }
  }
  // the carries of every tile (the group's last workgroup): C1 = exclusive
  // scan of a1, C2 = exclusive scan of a2 + C1 LVt, T = its total, ds = sum
  // m1 + C2 MS2 + C1 MS3; right-hand sides one after the other
  if (!flex) return;
  if (!last_arrival(g_arrive[0][grp], i, g.nb, &lflag)) return;
  double LT[1][TPT], M2[TPT], M3[TPT];
#pragma unroll
  for (int cc = 0; cc < TPT; ++cc) {
    const int t = cc * NT + tid;
    const bool ok = t < g.nb;
    LT[0][cc] = ok ? G_(tabr(tb, g, R_LVT))[t] : 0.0;
    M2[cc] = ok ? G_(tabr(tb, g, R_MS2))[t] : 0.0;
    M3[cc] = ok ? G_(tabr(tb, g, R_MS3))[t] : 0.0;
  }
#pragma unroll 1
  for (int q = 0; q < KG; ++q) {
    if (!has[q]) break;
    double* W = a.ws + (long long)(grp * KG + q) * a.wsd;
    double A1[1][TPT], A2[TPT], M1[TPT], C1[1][TPT], C2[1][TPT], y2[1][TPT], tt[1];
#pragma unroll
    for (int cc = 0; cc < TPT; ++cc) {
      const int t = cc * NT + tid;
      const bool ok = t < g.nb;
      A1[0][cc] = ok ? wrow(W, g, W_A1)[t] : 0.0;
      A2[cc] = ok ? wrow(W, g, W_A2)[t] : 0.0;
      M1[cc] = ok ? wrow(W, g, W_M1)[t] : 0.0;
    }
    tile_scan<1, false>(A1, C1, tt, sh);
#pragma unroll
    for (int cc = 0; cc < TPT; ++cc) y2[0][cc] = A2[cc] + C1[0][cc] * LT[0][cc];
    double T[1];
    tile_scan<1, false>(y2, C2, T, sh);
    double ds[1] = {0.0};
#pragma unroll
    for (int cc = 0; cc < TPT; ++cc) {
      const int t = cc * NT + tid;
      if (t < g.nb) {
        ds[0] += M1[cc] + C2[0][cc] * M2[cc] + C1[0][cc] * M3[cc];
        wrow(W, g, W_C1)[t] = C1[0][cc];
        wrow(W, g, W_C2)[t] = C2[0][cc];
      }
    }
    btot<1>(ds, sh);
    if (tid == 0) {
      wrow(W, g, W_JN)[J_T] = T[0];
      wrow(W, g, W_JN)[J_DS] = ds[0];
    }
  }
}

// phase B: the carries of this tile from every tile's a1, a2, m1, the
// tile-local scans of the (updated) tangent, da; tile 0 also bins 0, 1 and
// the scalar keys' new direction
template <int MODE, int KG>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(4))) void jvp_b(JvpArgs a) {
#pragma clang fp contract(off)
  __shared__ double sh[KG * (2 * NW + 1)];
  const Geo g = geo_of(a.c.B);
  int i, grp;
  place(g.nb, i, grp);
  const int tid = threadIdx.x;
  const AmpConst c = const_of<MODE>(a.c, a.dcs, a.dc1, grp * KG);
  const bool flex = a.c.has_flex, asp = a.c.has_asp;
  const double* tb = c.tab;
  if (!tb) return;  // constants without tables (nft_amp2_prepare not run): no access
  const double* gl = tabg(tb, g);
  bool has[KG];
  const double* sv[KG];
#pragma unroll
  for (int q = 0; q < KG; ++q) {
    const int r = grp * KG + q;
    has[q] = r < a.nrhs;
    sv[q] = wrow(a.ws + (long long)(has[q] ? r : grp * KG) * a.wsd, g, W_JN);
  }
  const long long j0 = (long long)i * g.tl();
  // ---- this tile's carries (phase A's last workgroup formed them)
  double C1v[KG], C2v[KG], Tv[KG], dSv[KG];
#pragma unroll
  for (int q = 0; q < KG; ++q) {
    const double* W = a.ws + (long long)(grp * KG + (has[q] ? q : 0)) * a.wsd;
    C1v[q] = flex ? wrow((double*)W, g, W_C1)[i] : 0.0;
    C2v[q] = flex ? wrow((double*)W, g, W_C2)[i] : 0.0;
    Tv[q] = flex ? sv[q][J_T] : 0.0;
    const double ssl = c.sig_s * sv[q][KSL];
    double d = (flex ? sv[q][J_DS] : 0.0) + ssl * gl[G_KV];
    if (flex) d += sv[q][KFLEX] * gl[G_KF];
    if (asp) d += sv[q][KASP] * gl[G_KA];
    dSv[q] = d - Tv[q] * gl[G_M4];
  }
  // ---- per bin: the tile-local scans and da
  double run1[KG], run2[KG];
#pragma unroll
  for (int q = 0; q < KG; ++q) run1[q] = run2[q] = 0.0;
  for (int s = 0; s < g.sub; ++s) {
    const long long j = j0 + (long long)s * NT + tid;
    const bool ok = j < g.M;
    const long long b = j + 2;
    double sf = 0, c0 = 0, lv = 0, lvc = 0, vsl = 0, qf = 0, qa = 0, scv = 0, an = 0;
    if (ok) {
      vsl = G_(c.vslope)[b];
      scv = G_(c.sc)[b];
      an = G_(c.An)[b];
      if (flex) {
        sf = G_(c.sf)[j];
        c0 = G_(c.c0)[j];
        lv = G_(c.lv)[j];
        lvc = G_(tabv(tb, g, T_LVC))[j];
        qf = G_(c.Qf)[b];
        if (asp) qa = G_(c.Qa)[b];
      }
    }
    double th[KG], u[KG];
    if (flex) {
      double d0[KG], d1[KG];
#pragma unroll
      for (int q = 0; q < KG; ++q) {
        const long long ro = (long long)(grp * KG + q) * a.ls;
        const bool okq = ok && has[q];
        d0[q] = okq ? a.t[KSPEC][ro + j] : 0.0;
        d1[q] = okq ? a.t[KSPEC][ro + g.M + j] : 0.0;
        u[q] = d1[q] * sf;
      }
      double tu[KG];
#pragma unroll
      for (int q = 0; q < KG; ++q) th[q] = u[q];
      bscan<KG, false>(th, tu, sh);  // th = loc1 (within the sub-chunk)
#pragma unroll
      for (int q = 0; q < KG; ++q) {
        const double loc1 = th[q] + run1[q];
        run1[q] += tu[q];
        th[q] = (d0[q] * c0 - u[q] / 2 * lv) + loc1 * lv;
      }
      bscan<KG, false>(th, tu, sh);  // th = loc2
#pragma unroll
      for (int q = 0; q < KG; ++q) {
        th[q] += run2[q];
        run2[q] += tu[q];
      }
    }
    if (!ok) continue;
#pragma unroll
    for (int q = 0; q < KG; ++q) {
      if (!has[q]) continue;
      const int r = grp * KG + q;
      const double ssl = c.sig_s * sv[q][KSL];
      double d = vsl * ssl + (flex ? th[q] : 0.0);
      if (flex) d += sv[q][KFLEX] * qf;
      if (asp) d += sv[q][KASP] * qa;
      const double dp = (d + (C2v[q] + C1v[q] * lvc)) - Tv[q] * scv;
      const double dfl = c.fl * c.ls_f * sv[q][KFL];
      a.da[(long long)r * a.vs + b * a.des] =
          (dfl * an + c.fl * an * (dp / 2. - dSv[q] / (2. * c.S))) * c.total_volume;
    }
  }
  if (i == 0 && tid < 2 * KG) {
    const int q = tid >> 1, b = tid & 1;
    if (has[q]) {
      const int r = grp * KG + q;
      const double* s_ = sv[q];
      const double dfl = c.fl * c.ls_f * s_[KFL];
      double v;
      if (b == 0) {
        v = c.has_zm ? c.zm * c.ls_o * s_[KZM] : 0.0;
      } else {
        double d = G_(c.vslope)[b] * (c.sig_s * s_[KSL]);
        if (flex) d += s_[KFLEX] * G_(c.Qf)[b];
        if (asp) d += s_[KASP] * G_(c.Qa)[b];
        const double dp = d - Tv[q] * G_(c.sc)[b];
        const double An = G_(c.An)[b];
        v = dfl * An + c.fl * An * (dp / 2. - dSv[q] / (2. * c.S));
      }
      a.da[(long long)r * a.vs + b * a.des] = v * c.total_volume;
      if (b == 0 && a.dir && a.sc[(long long)r * NS_ + NFT_CG_DONE] == 0.0) {
        const long long ro = (long long)r * a.ls;
#pragma unroll
        for (int k = 0; k < 5; ++k)
          if (a.t[k] && !(k == KFLEX && !flex) && !(k == KASP && !asp) && !(k == KZM && !c.has_zm)) a.t[k][ro] = s_[k];
      }
    }
  }
}

// ======================================================================= VJP
struct VjpArgs {
  AmpConst c;
  const AmpConst* dcs;
  const AmpConst* dc1;
  const double* g;         // g[r * gs + b]
  long long gs;
  // plain mode: out keys (= shift * d + J^T g) and the d keys for the shift
  // CG mode (cg): x, r, d keys, updated x -= alpha d, r -= alpha (q + shift d)
  double* o[6];
  double* o2[6];           // cg: r keys
  const double* d[6];      // d keys (shift / cg)
  long long ls;
  double shift;
  double* ws;
  long long wsd;
  int nrhs;
  int cg;
  double* sc;              // CG scalar blocks (cg: alpha read, finalized here)
  double* part;            // cg: rr / xr partials per tile, part[r * pstride + {0, nb} + tile]
  long long pstride;
  const double* gpart;     // cg: the grid segment's partials (rows rr, xr at 0 and gpr) per RHS
  long long gps, gpr;
  int ngp;
};

// workspace rows of one RHS (VJP)
enum { V_R1 = 0, V_R2G, V_R3G, V_AGG, V_AWG, V_P0G, V_Q2G, V_P1G, V_CRR, V_CXR, V_N };
// ... then the carries of phase A's last workgroup: beta(t), S1(t) [nbp
// each], and the scalars k, R1, R2, u0 (flexibility), u1 (asperity)
enum { V_BT = V_N, V_S1, V_SC };
enum { S_K = 0, S_R1, S_R2, S_U0, S_U1 };

// phase A: the tile's dot products of G = An fl TV g / 2 with the constant
// vectors (+ its slice of the grid segment's CG partials)
template <int MODE, int KG>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(4))) void vjp_a(VjpArgs a) {
#pragma clang fp contract(off)
  __shared__ double sh[(V_N * KG) * (NW + 1)];
  __shared__ int lflag;
  const Geo g = geo_of(a.c.B);
  int i, grp;
  place(g.nb, i, grp);
  const int tid = threadIdx.x;
  const AmpConst c = const_of<MODE>(a.c, a.dcs, a.dc1, grp * KG);
  const bool flex = a.c.has_flex, asp = a.c.has_asp;
  const double* tb = c.tab;
  if (!tb) return;  // constants without tables (nft_amp2_prepare not run): no access
  const double TV = c.total_volume;
  bool has[KG];
#pragma unroll
  for (int q = 0; q < KG; ++q) has[q] = grp * KG + q < a.nrhs;
  double s[V_N * KG];
#pragma unroll
  for (int k = 0; k < V_N * KG; ++k) s[k] = 0.0;
  const long long j0 = (long long)i * g.tl();
  for (int sc_ = 0; sc_ < g.sub; ++sc_) {
    const long long j = j0 + (long long)sc_ * NT + tid;
    const bool ok = j < g.M;
    const long long b = j + 2;
    double an = 0, vsl = 0, scv = 0, k1 = 0, k2 = 0, k3 = 0, k4 = 0;
    if (ok) {
      an = G_(c.An)[b];
      vsl = G_(c.vslope)[b];
      scv = G_(c.sc)[b];
      if (flex) {
        k1 = G_(tabv(tb, g, T_K1))[j];
        k2 = G_(tabv(tb, g, T_K2))[j];
        k3 = G_(tabv(tb, g, T_K3))[j];
        if (asp) k4 = G_(tabv(tb, g, T_K4))[j];
      }
    }
    double gb[KG];
#pragma unroll
    for (int q = 0; q < KG; ++q) gb[q] = (ok && has[q]) ? a.g[(long long)(grp * KG + q) * a.gs + b] : 0.0;
#pragma unroll
    for (int q = 0; q < KG; ++q) {
      const double G = an * (c.fl * (TV * gb[q])) / 2.;
      double* S = s + V_N * q;
      S[V_R1] += TV * gb[q] * an;
      S[V_R2G] += vsl * G;
      S[V_R3G] += G * scv;
      S[V_AGG] += G;
      S[V_AWG] += G * k1;
      S[V_P0G] += G * k2;
      S[V_Q2G] += G * k3;
      S[V_P1G] += G * k4;
    }
  }
  if (i == 0 && tid < 2) {  // bins 0 and 1
    const int b = tid;
    const double an = G_(c.An)[b], vs = G_(c.vslope)[b], scb = G_(c.sc)[b];
#pragma unroll
    for (int q = 0; q < KG; ++q) {
      if (!has[q]) continue;
      const double g_ = a.g[(long long)(grp * KG + q) * a.gs + b];
      const double ga = an * (c.fl * (b > 0 ? TV * g_ : 0.0)) / 2.;
      double* S = s + V_N * q;
      if (b > 0) S[V_R1] += TV * g_ * an;
      S[V_R2G] += vs * ga;
      S[V_R3G] += ga * scb;
    }
  }
  if (a.cg) {
    const int per = (a.ngp + g.nb - 1) / g.nb;
    const int lo = i * per, hi = min(a.ngp, lo + per);
#pragma unroll
    for (int q = 0; q < KG; ++q) {
      if (!has[q]) continue;
      const double* gp = a.gpart + (long long)(grp * KG + q) * a.gps;
      for (int t = lo + tid; t < hi; t += NT) {
        s[V_N * q + V_CRR] += gp[t];
        s[V_N * q + V_CXR] += gp[a.gpr + t];
      }
    }
  }
  btot_sh<V_N * KG>(s, sh);
  const double* tot = sh + V_N * KG * NW;
#pragma unroll
  for (int q = 0; q < KG; ++q) if (tid == q && has[q]) {
    double* W = a.ws + (long long)(grp * KG + q) * a.wsd;
#pragma unroll
    for (int k = 0; k < V_N; ++k) wrow(W, g, k)[i] = tot[V_N * q + k];
  }
  // the carries of every tile (the group's last workgroup), right-hand sides
  // one after the other: k = fl R1 / (2 S), R3 = R3G - k R3M; beta(t) =
  // SG(t) - k SM(t) - R3 (SG: sum of aggG over the tiles after t); S1 =
  // exclusive reverse scan of (AWG - k AWM) + beta AWL; R2 = R2G - k R2M;
  // u0, u1 = the flexibility / asperity cotangents
  if (!last_arrival(g_arrive[1][grp], i, g.nb, &lflag)) return;
  double SM[TPT], AWM[TPT], AWL[TPT];
#pragma unroll
  for (int cc = 0; cc < TPT; ++cc) {
    const int t = cc * NT + tid;
    const bool ok = flex && t < g.nb;
    SM[cc] = ok ? G_(tabr(tb, g, R_SM))[t] : 0.0;
    AWM[cc] = ok ? G_(tabr(tb, g, R_AWM))[t] : 0.0;
    AWL[cc] = ok ? G_(tabr(tb, g, R_AWL))[t] : 0.0;
  }
#pragma unroll 1
  for (int q = 0; q < KG; ++q) {
    if (!has[q]) break;
    double* W = a.ws + (long long)(grp * KG + q) * a.wsd;
    double gs[3] = {0.0, 0.0, 0.0};
    double AG[1][TPT], AW[TPT];
#pragma unroll
    for (int cc = 0; cc < TPT; ++cc) {
      const int t = cc * NT + tid;
      const bool ok = t < g.nb;
      gs[0] += ok ? wrow(W, g, V_R1)[t] : 0.0;
      gs[1] += ok ? wrow(W, g, V_R3G)[t] : 0.0;
      gs[2] += ok ? wrow(W, g, V_R2G)[t] : 0.0;
      AG[0][cc] = (ok && flex) ? wrow(W, g, V_AGG)[t] : 0.0;
      AW[cc] = (ok && flex) ? wrow(W, g, V_AWG)[t] : 0.0;
    }
    btot<3>(gs, sh);
    const double k_ = c.fl * gs[0] / (2. * c.S);
    const double R3s = gs[1] - k_ * tabg(tb, g)[G_M4];
    double u[2] = {0.0, 0.0};
    if (flex) {
      double SG[1][TPT], z[1][TPT], S1[1][TPT], tt[1], BT[TPT];
      tile_scan<1, true>(AG, SG, tt, sh);
#pragma unroll
      for (int cc = 0; cc < TPT; ++cc) {
        const int t = cc * NT + tid;
        BT[cc] = (SG[0][cc] - k_ * SM[cc]) - R3s;
        z[0][cc] = t < g.nb ? ((AW[cc] - k_ * AWM[cc]) + BT[cc] * AWL[cc]) : 0.0;
      }
      tile_scan<1, true>(z, S1, tt, sh);
#pragma unroll
      for (int cc = 0; cc < TPT; ++cc) {
        const int t = cc * NT + tid;
        if (t >= g.nb) continue;
        wrow(W, g, V_BT)[t] = BT[cc];
        wrow(W, g, V_S1)[t] = S1[0][cc];
        u[0] += ((wrow(W, g, V_P0G)[t] - k_ * G_(tabr(tb, g, R_P0M))[t]) + BT[cc] * G_(tabr(tb, g, R_P0S))[t]) +
                ((wrow(W, g, V_Q2G)[t] - k_ * G_(tabr(tb, g, R_Q2M))[t]) + BT[cc] * G_(tabr(tb, g, R_Q2L))[t]) +
                S1[0][cc] * G_(tabr(tb, g, R_P2S))[t];
        if (asp) u[1] += (wrow(W, g, V_P1G)[t] - k_ * G_(tabr(tb, g, R_P1M))[t]) + BT[cc] * G_(tabr(tb, g, R_P1S))[t];
      }
    }
    btot<2>(u, sh);
    if (tid == 0) {
      double* sc_ = wrow(W, g, V_SC);
      sc_[S_K] = k_;
      sc_[S_R1] = gs[0];
      sc_[S_R2] = gs[2] - k_ * tabg(tb, g)[G_KV];
      sc_[S_U0] = u[0];
      sc_[S_U1] = u[1];
    }
  }
}

// phase B: this tile's carries (k, beta, S1) from every tile's sums, the
// tile-local reverse scans of G and w, the spectrum cotangents (plain: the
// outputs; cg: the update); tile 0 the scalar cotangents; cg: the r.r / x.r
// partials and, in the last workgroup of the group, the finalize
template <int MODE, int KG>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(4))) void vjp_b(VjpArgs a) {
#pragma clang fp contract(off)
  __shared__ double sh[(2 * KG) * (NW + 1)];
  __shared__ int lflag;
  const Geo g = geo_of(a.c.B);
  int i, grp;
  place(g.nb, i, grp);
  const int tid = threadIdx.x;
  const AmpConst c = const_of<MODE>(a.c, a.dcs, a.dc1, grp * KG);
  const bool flex = a.c.has_flex, asp = a.c.has_asp;
  const double* tb = c.tab;
  if (!tb) return;  // constants without tables (nft_amp2_prepare not run): no access
  const double TV = c.total_volume;
  bool has[KG];
#pragma unroll
  for (int q = 0; q < KG; ++q) has[q] = grp * KG + q < a.nrhs;
  // ---- this tile's carries (phase A's last workgroup formed them)
  double kv[KG], bet[KG], S1v[KG];
#pragma unroll
  for (int q = 0; q < KG; ++q) {
    const double* W = a.ws + (long long)(grp * KG + (has[q] ? q : 0)) * a.wsd;
    kv[q] = wrow((double*)W, g, V_SC)[S_K];
    bet[q] = flex ? wrow((double*)W, g, V_BT)[i] : 0.0;
    S1v[q] = flex ? wrow((double*)W, g, V_S1)[i] : 0.0;
  }
  double al[KG];
  bool okc[KG];
#pragma unroll
  for (int q = 0; q < KG; ++q) {
    al[q] = 0.0;
    okc[q] = false;
    if (a.cg && has[q]) {
      const double* scb = a.sc + (long long)(grp * KG + q) * NS_;
      const double curv = scb[NFT_CG_CURV], gprev = scb[NFT_CG_GAMMA];
      al[q] = gprev / curv;
      okc[q] = (curv == curv) && curv != 0.0 && (al[q] >= 0.0) && (al[q] == al[q]) && scb[NFT_CG_DONE] == 0.0;
    }
  }
  double rr[KG], xr[KG];
#pragma unroll
  for (int q = 0; q < KG; ++q) rr[q] = xr[q] = 0.0;
  // ---- per bin, sub-chunks from the last (reverse scans)
  if (flex) {
    double ry[KG], rw[KG];
#pragma unroll
    for (int q = 0; q < KG; ++q) ry[q] = rw[q] = 0.0;
    const long long j0 = (long long)i * g.tl();
    for (int s = g.sub - 1; s >= 0; --s) {
      const long long j = j0 + (long long)s * NT + tid;
      const bool ok = j < g.M;
      const long long b = j + 2;
      // the scans' operands first; the output operands after the scans (a
      // second load round, fewer live registers through the scans)
      double an = 0, lv = 0, lvn = 0;
      if (ok) {
        an = G_(c.An)[b];
        lv = G_(c.lv)[j];
        lvn = j + 1 < g.M ? G_(c.lv)[j + 1] : 0.0;
      }
      double G[KG], y[KG], w[KG], ty[KG];
#pragma unroll
      for (int q = 0; q < KG; ++q) {
        const double gb = (ok && has[q]) ? a.g[(long long)(grp * KG + q) * a.gs + b] : 0.0;
        G[q] = an * (c.fl * (TV * gb)) / 2.;
        y[q] = G[q];
      }
      bscan<KG, true>(y, ty, sh);
#pragma unroll
      for (int q = 0; q < KG; ++q) {
        y[q] += ry[q];
        ry[q] += ty[q];
        w[q] = y[q] * lv / 2. + (y[q] - G[q]) * lvn / 2.;
      }
      bscan<KG, true>(w, ty, sh);
#pragma unroll
      for (int q = 0; q < KG; ++q) {
        w[q] += rw[q];
        rw[q] += ty[q];
      }
      if (!ok) continue;
      const double ym = G_(tabv(tb, g, T_YM))[j], g1m = G_(tabv(tb, g, T_G1M))[j];
      const double g1l = G_(tabv(tb, g, T_G1L))[j], c0 = G_(c.c0)[j], sf = G_(c.sf)[j];
      // every operand of the group first (the stores to x / r cannot be
      // passed by later loads of the same arrays), then the arithmetic
      double X0[KG], X1[KG], R0[KG], R1[KG], D0[KG], D1[KG];
#pragma unroll
      for (int q = 0; q < KG; ++q) {
        const long long ro = (long long)(grp * KG + q) * a.ls;
        const double* ds = a.d[KSPEC] ? a.d[KSPEC] + ro : nullptr;
        X0[q] = X1[q] = R0[q] = R1[q] = D0[q] = D1[q] = 0.0;
        if (!has[q]) continue;
        if (ds) {
          D0[q] = ds[j];
          D1[q] = ds[g.M + j];
        }
        if (a.cg) {
          X0[q] = a.o[KSPEC][ro + j];
          X1[q] = a.o[KSPEC][ro + g.M + j];
          R0[q] = a.o2[KSPEC][ro + j];
          R1[q] = a.o2[KSPEC][ro + g.M + j];
        }
      }
#pragma unroll
      for (int q = 0; q < KG; ++q) {
        if (!has[q]) continue;
        const long long ro = (long long)(grp * KG + q) * a.ls;
        const double yv = (y[q] - kv[q] * ym) + bet[q];
        const double g1 = ((w[q] - kv[q] * g1m) + bet[q] * g1l) + S1v[q];
        const double q0 = yv * c0, q1 = g1 * sf;
        double* os = a.o[KSPEC] + ro;
        if (!a.cg) {
          double v0 = q0, v1 = q1;
          if (a.d[KSPEC]) {
            v0 += a.shift * D0[q];
            v1 += a.shift * D1[q];
          }
          os[j] = v0;
          os[g.M + j] = v1;
        } else {
          double* rsp = a.o2[KSPEC] + ro;
          double xa = X0[q], xb = X1[q], ra = R0[q], rb = R1[q];
          const double d0 = D0[q], d1 = D1[q];
          if (okc[q]) {
            xa = xa - al[q] * d0;
            ra = ra - al[q] * (q0 + a.shift * d0);
            xb = xb - al[q] * d1;
            rb = rb - al[q] * (q1 + a.shift * d1);
            os[j] = xa;
            rsp[j] = ra;
            os[g.M + j] = xb;
            rsp[g.M + j] = rb;
          }
          rr[q] += ra * ra + rb * rb;
          xr[q] += xa * ra + xb * rb;
        }
      }
    }
  }
  // scalar cotangents (tile 0, thread q for RHS q): fl, sl, flex, asp, zm
#pragma unroll
  for (int q = 0; q < KG; ++q) if (i == 0 && tid == q && has[q]) {
    const int r = grp * KG + q;
    const long long ro = (long long)r * a.ls;
    double qv[5];
    bool hs[5];
    const double* scq = wrow(a.ws + (long long)r * a.wsd, g, V_SC);
    qv[KFL] = c.fl * c.ls_f * scq[S_R1];
    hs[KFL] = true;
    qv[KSL] = c.sig_s * scq[S_R2];
    hs[KSL] = true;
    qv[KFLEX] = scq[S_U0];
    hs[KFLEX] = flex;
    qv[KASP] = scq[S_U1];
    hs[KASP] = asp;
    qv[KZM] = c.has_zm ? c.zm * c.ls_o * TV * a.g[(long long)r * a.gs] : 0.0;
    hs[KZM] = c.has_zm;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      if (!hs[k] || !a.o[k]) continue;
      if (!a.cg) {
        a.o[k][ro] = qv[k] + (a.d[k] ? a.shift * a.d[k][ro] : 0.0);
      } else {
        double x = a.o[k][ro], rv = a.o2[k][ro];
        const double d = a.d[k][ro];
        if (okc[q]) {
          x = x - al[q] * d;
          rv = rv - al[q] * (qv[k] + a.shift * d);
          a.o[k][ro] = x;
          a.o2[k][ro] = rv;
        }
        rr[q] += rv * rv;
        xr[q] += x * rv;
      }
    }
  }
  if (!a.cg) return;
  double v[2 * KG];
#pragma unroll
  for (int q = 0; q < KG; ++q) {
    v[2 * q] = rr[q];
    v[2 * q + 1] = xr[q];
  }
  btot_sh<2 * KG>(v, sh);
  const double* tot = sh + 2 * KG * NW;
#pragma unroll
  for (int q = 0; q < KG; ++q) if (tid == q && has[q]) {
    const int r = grp * KG + q;
    const double* W = a.ws + (long long)r * a.wsd;
    double* pp = a.part + (long long)r * a.pstride;
    // this tile's amplitude sums, then its slice of the grid partials
    pp[i] = tot[2 * q] + wrow((double*)W, g, V_CRR)[i];
    pp[g.nb + i] = tot[2 * q + 1] + wrow((double*)W, g, V_CXR)[i];
  }
  // finalize (the last workgroup of the group): each RHS's tile partials
  // folded in index order, then cg_finalize_kernel's bookkeeping; one wave
  // per right-hand side
  if (!last_arrival(g_arrive[2][grp], i, g.nb, &lflag)) return;
  const int lane = tid & 63, wv = tid >> 6;
  if (wv < KG && has[wv]) {
    const int r = grp * KG + wv;
    const double* pp = a.part + (long long)r * a.pstride;
    double f0 = 0.0, f1 = 0.0;
    for (int t = lane; t < g.nb; t += 64) {
      f0 += pp[t];
      f1 += pp[g.nb + t];
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      f0 += __shfl_down(f0, off, 64);
      f1 += __shfl_down(f1, off, 64);
    }
    if (lane == 0) {
      double* scb = a.sc + (long long)r * NS_;
      if (scb[NFT_CG_DONE] == 0.0) {
        const double curv = scb[NFT_CG_CURV], gprev = scb[NFT_CG_GAMMA];
        const double alpha = gprev / curv;
        const bool ok = (curv == curv) && curv != 0.0 && (alpha >= 0.0) && (alpha == alpha);
        scb[NFT_CG_ALPHA] = alpha;
        scb[NFT_CG_FLAG] = ok ? 0.0 : 1.0;
        scb[NFT_CG_ITER] += 1.0;
        if (ok) {
          scb[NFT_CG_GPREV] = gprev;
          scb[NFT_CG_GAMMA] = f0;
          scb[NFT_CG_XR] = f1;
          scb[NFT_CG_XB] = 0.0;
        }
        if (!ok || (scb[NFT_CG_AUTO] != 0.0 && !(f0 > 0.0))) scb[NFT_CG_DONE] = 2.0;
      }
    }
  }
}

// ------------------------------------------------------------------ launch
static int g_override = -1;
static bool enabled() {
  static const int on = getenv("NFT_AMP2") ? atoi(getenv("NFT_AMP2")) : 1;
  return g_override >= 0 ? g_override != 0 : on != 0;
}

}  // namespace amp2
}  // namespace nft

using namespace nft;
using namespace nft::amp2;

namespace {
// right-hand sides per workgroup (at most kmax: the register budget of the
// kernel): the constant sets of MODE 1 differ per RHS
int kg_of(int nrhs, int mode, int kmax) {
  if (mode == 1 || nrhs <= 1 || kmax <= 1) return 1;
  return (nrhs == 2 || kmax == 2) ? 2 : 4;
}
// tuning probe (NFT_AMP2_KA / _KB / _KV = 1, 2 or 4): RHS per workgroup of
// the JVP's first / second launch and of the VJP's
int kg_env(const char* name, int def) {
  const char* e = getenv(name);
  const int v = e ? atoi(e) : 0;
  return (v == 1 || v == 2 || v == 4) ? v : def;
}

#define NFT_AMP2_LAUNCH(KERN, ARGS, MODE, KG, GRID, S)                                              \
  do {                                                                                              \
    if ((MODE) == 1) hipLaunchKernelGGL((KERN<1, 1>), GRID, dim3(NT), 0, S, ARGS);                  \
    else if ((MODE) == 2) {                                                                         \
      if ((KG) == 1) hipLaunchKernelGGL((KERN<2, 1>), GRID, dim3(NT), 0, S, ARGS);                  \
      else if ((KG) == 2) hipLaunchKernelGGL((KERN<2, 2>), GRID, dim3(NT), 0, S, ARGS);             \
      else hipLaunchKernelGGL((KERN<2, 4>), GRID, dim3(NT), 0, S, ARGS);                            \
    } else {                                                                                        \
      if ((KG) == 1) hipLaunchKernelGGL((KERN<0, 1>), GRID, dim3(NT), 0, S, ARGS);                  \
      else if ((KG) == 2) hipLaunchKernelGGL((KERN<0, 2>), GRID, dim3(NT), 0, S, ARGS);             \
      else hipLaunchKernelGGL((KERN<0, 4>), GRID, dim3(NT), 0, S, ARGS);                            \
    }                                                                                               \
  } while (0)

// tiles per RHS (0: not applicable -- NFT_AMP2=0, B < 3, too many RHS)
int tiles_of(long long B, int nrhs) {
  if (!enabled() || B < 3 || nrhs < 1 || nrhs > MAXR) return 0;
  const Geo g = geo_of(B);
  const long long wsd = (long long)(nft_amp_workspace(B) / sizeof(double));
  if ((long long)V_SC * g.nbp + 8 > wsd || (long long)W_JN * g.nbp + 8 > wsd) return 0;
  return g.nb;
}
}  // namespace

extern "C" {

int nft_amp2_enabled(void) { return enabled() ? 1 : 0; }

void nft_amp2_set_enabled(int on) { g_override = on < 0 ? -1 : (on != 0); }

int nft_amp2_tiles(int64_t B, int nrhs, int item_mode) {
  (void)item_mode;
  return tiles_of(B, nrhs);
}

int64_t nft_amp2_tab_len(int64_t B) { return B < 3 ? 0 : tab_len(geo_of(B)); }

int nft_amp2_prepare(const nft_amp_const* c, nft_amp_const* item_consts, int nrow, double* tab, int64_t tab_stride,
                     hipStream_t stream) {
  if (!c || c->B < 3 || !tab || nrow < 1 || (nrow > 1 && !item_consts) ||
      (item_consts && tab_stride < nft_amp2_tab_len(c->B)) || (c->has_asp && !c->has_flex)) {
    set_last_error("nft_amp2_prepare: invalid arguments");
    return NFT_ERR_ARG;
  }
  if (!item_consts && (!c->mspec || !c->sc || !c->vslope || !c->An ||
                       (c->has_flex && (!c->lv || !c->sf || !c->c0 || !c->p0 || !c->p2 || !c->Qf)) ||
                       (c->has_asp && (!c->p1 || !c->Qa)))) {
    set_last_error("nft_amp2_prepare: a constant array the flags need is NULL");
    return NFT_ERR_ARG;
  }
  PrepArgs a{};
  a.c = *c;
  a.dcs = item_consts;
  a.tab = tab;
  a.ts = tab_stride;
  a.nrow = nrow;
  const Geo g = geo_of(c->B);
  prof_mark(stream, "amp2_prepare");
  if (item_consts) {
    hipLaunchKernelGGL((prep_tiles<true>), dim3((unsigned)(g.nb * nrow)), dim3(NT), 0, stream, a);
    hipLaunchKernelGGL((prep_globals<true>), dim3((unsigned)nrow), dim3(NT), 0, stream, a);
  } else {
    hipLaunchKernelGGL((prep_tiles<false>), dim3((unsigned)g.nb), dim3(NT), 0, stream, a);
    hipLaunchKernelGGL((prep_globals<false>), dim3(1), dim3(NT), 0, stream, a);
  }
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

int nft_amp2_jvp(const nft_amp_const* cst_, const nft_amp_const* item_consts, int item_mode, double* const* t,
                 const double* const* r, int64_t lat_stride, double* da, int64_t da_stride, int64_t da_elem_stride,
                 double* ws, int nrhs, const double* sc, double* part, int64_t pstride, double shift,
                 hipStream_t stream) {
  if (!cst_ || !t || !da || !ws || nrhs < 1 || cst_->B < 3 || (cst_->has_flex && !t[KSPEC]) ||
      (r && (!sc || !part))) {
    set_last_error("nft_amp2_jvp: invalid arguments");
    return NFT_ERR_ARG;
  }
  if (item_mode < 0 || item_mode > 2 || (item_mode != 0 && !item_consts) || (item_mode == 0 && !cst_->tab)) {
    set_last_error("nft_amp2_jvp: invalid item_mode / item_consts, or constants without tables (nft_amp2_prepare)");
    return NFT_ERR_ARG;
  }
  const int nb = tiles_of(cst_->B, nrhs);
  if (!nb) return NFT_AMP2_FALLBACK;
  JvpArgs a{};
  a.c = *cst_;
  a.dcs = item_mode == 1 ? item_consts : nullptr;
  a.dc1 = item_mode == 2 ? item_consts : nullptr;
  for (int q = 0; q < 6; ++q) {
    a.t[q] = t[q];
    a.r[q] = r ? r[q] : nullptr;
    if (r && t[q] && !r[q]) {
      set_last_error("nft_amp2_jvp: a direction key without its residual");
      return NFT_ERR_ARG;
    }
  }
  a.ls = lat_stride;
  a.da = da;
  a.vs = da_stride;
  a.des = da_elem_stride > 0 ? da_elem_stride : 1;
  a.ws = ws;
  a.wsd = (long long)(nft_amp_workspace(cst_->B) / sizeof(double));
  a.nrhs = nrhs;
  a.dir = r != nullptr;
  a.sc = sc;
  a.part = part;
  a.pstride = pstride;
  a.shift = shift;
  const int ka = kg_of(nrhs, item_mode, kg_env("NFT_AMP2_KA", 4)), kb = kg_of(nrhs, item_mode, kg_env("NFT_AMP2_KB", 2));
  prof_mark(stream, a.dir ? "amp_jvp_a+dir" : "amp_jvp_a");
  NFT_AMP2_LAUNCH(jvp_a, a, item_mode, ka, dim3((unsigned)(nb * ((nrhs + ka - 1) / ka))), stream);
  prof_mark(stream, "amp_jvp_b");
  NFT_AMP2_LAUNCH(jvp_b, a, item_mode, kb, dim3((unsigned)(nb * ((nrhs + kb - 1) / kb))), stream);
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

int nft_amp2_vjp(const nft_amp_const* cst_, const nft_amp_const* item_consts, int item_mode, const double* g,
                 int64_t g_stride, double* const* out, double* const* out2, const double* const* d,
                 int64_t lat_stride, double shift, double* ws, int nrhs, double* sc, double* part, int64_t pstride,
                 const double* gpart, int64_t gp_stride, int64_t gp_row, int ngp, hipStream_t stream) {
  if (!cst_ || !g || !out || !ws || nrhs < 1 || cst_->B < 3 || (cst_->has_flex && !out[KSPEC]) ||
      (out2 && (!d || !sc || !part || (ngp > 0 && !gpart)))) {
    set_last_error("nft_amp2_vjp: invalid arguments");
    return NFT_ERR_ARG;
  }
  if (item_mode < 0 || item_mode > 2 || (item_mode != 0 && !item_consts) || (item_mode == 0 && !cst_->tab)) {
    set_last_error("nft_amp2_vjp: invalid item_mode / item_consts, or constants without tables (nft_amp2_prepare)");
    return NFT_ERR_ARG;
  }
  const int nb = tiles_of(cst_->B, nrhs);
  if (!nb) return NFT_AMP2_FALLBACK;
  VjpArgs a{};
  a.c = *cst_;
  a.dcs = item_mode == 1 ? item_consts : nullptr;
  a.dc1 = item_mode == 2 ? item_consts : nullptr;
  a.g = g;
  a.gs = g_stride;
  for (int q = 0; q < 6; ++q) {
    a.o[q] = out[q];
    a.o2[q] = out2 ? out2[q] : nullptr;
    a.d[q] = d ? d[q] : nullptr;
    if (out2 && out[q] && (!out2[q] || !d[q])) {
      set_last_error("nft_amp2_vjp: a CG key without its residual / direction");
      return NFT_ERR_ARG;
    }
  }
  a.ls = lat_stride;
  a.shift = shift;
  a.ws = ws;
  a.wsd = (long long)(nft_amp_workspace(cst_->B) / sizeof(double));
  a.nrhs = nrhs;
  a.cg = out2 != nullptr;
  a.sc = sc;
  a.part = part;
  a.pstride = pstride;
  a.gpart = gpart;
  a.gps = gp_stride;
  a.gpr = gp_row;
  a.ngp = a.cg ? ngp : 0;
  const int kg = kg_of(nrhs, item_mode, kg_env("NFT_AMP2_KV", 1));
  const dim3 grid((unsigned)(nb * ((nrhs + kg - 1) / kg)));
  prof_mark(stream, a.cg ? "amp_vjp_a+cg" : "amp_vjp_a");
  NFT_AMP2_LAUNCH(vjp_a, a, item_mode, kg, grid, stream);
  prof_mark(stream, a.cg ? "amp_vjp_b+cg" : "amp_vjp_b");
  NFT_AMP2_LAUNCH(vjp_b, a, item_mode, kg, grid, stream);
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

}  // extern "C"
