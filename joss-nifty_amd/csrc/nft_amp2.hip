// Correlated-field amplitude Jacobian in two launches per JVP / VJP ("two-phase
// tiles"), optionally carrying the amplitude keys' CG direction (JVP) and the
// CG update + finalize of the iteration (VJP).
//
// Same operator as nft_amp.hip (reference: src/library/correlated_fields.py
// :105-212 -- _SlopeRemover, _TwoLogIntegrations, _Normalization --, and the
// scalings of correlated_fields_simple.py:86-127), linearised at one
// expansion point.  The JVP / VJP are linear in the tangent / cotangent, and
// every global quantity they need -- the two scan carries of each tile, the
// slope-remover's last value T, the normalisation sums dS / R1 / R3 -- enters
// LINEARLY.  So each workgroup (one scan tile of E*256 bins, all K right-hand
// sides of its group) first computes everything tile-local: local scans
// without carries, and the handful of per-tile sums the carries and globals
// are made of (phase A, first launch); the second launch combines them in a
// fixed order over the tiles and redoes the tile-local scans to form the
// outputs (phase B):
//
//   JVP   c_j  = loc1_j + C1(i)                       C1(i) = sum_{t<i} agg1(t)
//         tl_j = loc2_j + C1(i) LVc_j + C2(i)         C2(i) = sum_{t<i} agg2(t) + C1(t) LVt(t)
//         dS   = sum_t MS1(t) + C2(t) MS2(t) + C1(t) MS3(t) - T MS4
//   VJP   gapre_b = G_b - k mspec_b,  k = fl R1 / (2 S),  R3 = R3G - k R3m
//         y_j  = yG_j - k ym_j + beta(i)              beta(i) = SG(i) - k SM(i) - R3
//         g1_j = g1G_j - k g1m_j + beta(i) g1l_j + S1(i)
//
// (loc*, yG, ym, g1*: tile-local scans; SG, SM, S1: sums over the tiles after
// i).  Against the ten stream-ordered kernels of nft_amp.hip (four for the
// JVP, six for the VJP, each a full pass per RHS over B-sized intermediates)
// this reads the per-bin constants once for the K right-hand sides of a
// workgroup, writes one B-sized intermediate (the JVP's pre-slope values) and
// takes one kernel boundary per JVP / VJP.  A grid barrier in place of that
// boundary would need the whole problem resident in registers at once
// (measured: ~40 VGPRs per bin and RHS, beyond the 256 CUs at C3's 4 x 313k
// bins), so phase B re-derives the tile-local scans from its inputs instead
// (bitwise the values of phase A).  All sums are fixed-order (tile-local
// striped scans, then scans / totals over the tiles in index order), so
// results are deterministic and, per right-hand side, independent of how many
// share the launch.
#include <algorithm>
#include <cstdlib>
#include <mutex>

#include "nft_api_internal.hpp"
#include "../../include/nifty_amd.h"

namespace nft {
namespace amp2 {

using AmpConst = nft_amp_const;
constexpr int NT = 256;
constexpr int NW = NT / 64;
constexpr int E = 4;  // bins per thread: tile = E * NT bins, whatever the batch size
constexpr int TL = E * NT;
constexpr int MAXR = 256;     // right-hand sides per launch (per-RHS arrival counters)
constexpr int NS_ = NFT_CG_NSCALARS;
// minimum waves per SIMD asked of the compiler for the four tile kernels
// (__launch_bounds__ second argument; 0: none)
#ifndef NFT_AMP2_WAVES
#define NFT_AMP2_WAVES 0
#endif
#if NFT_AMP2_WAVES > 0
#define NFT_AMP2_LB __launch_bounds__(NT, NFT_AMP2_WAVES)
#else
#define NFT_AMP2_LB __launch_bounds__(NT)
#endif

enum { KFL = 0, KSL = 1, KFLEX = 2, KASP = 3, KZM = 4, KSPEC = 5 };

// the per-bin constants are read through pointers loaded from a struct (the
// device constant sets): cast them to the global address space, or every
// read is a flat load waited on with the LDS traffic
typedef __attribute__((address_space(1))) const double gdouble;
__device__ __forceinline__ gdouble* G_(const double* p) { return (gdouble*)p; }

// device-coherent scalar access for the values exchanged between workgroups
__device__ __forceinline__ double cld(const double* p) {
  return __hip_atomic_load(const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void cst(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------ block helpers
__device__ __forceinline__ double wsum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  return v;
}

// NV block totals at once; per value the wave tree and the waves in order
template <int NV>
__device__ __forceinline__ void btot(double (&v)[NV], double* sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // the wave trees of the NV values step by step (one LDS round trip per step)
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    double y[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) y[k] = __shfl_down(v[k], off, 64);
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] += y[k];
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

// inclusive scans of NA independent arrays of EE values per thread in
// STRIPED layout (v[a][e] is element e*NT + tid: every global access of a
// tile is one coalesced run per e), forward or reversed: wave scans by
// shuffles -- all NA*EE of a step issued together, one LDS round trip per
// step --, then per element the fixed-order sum of the preceding (following)
// wave segments, segment (e, w) in the order e*NW + w.  One barrier pair.
// tot[a]: totals.
template <int NA, int EE, bool REV>
__device__ __forceinline__ void scan_arr(double (&v)[NA][EE], double (&tot)[NA], double* sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int NSEG = EE * NW;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    double y[NA][EE];
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int e = 0; e < EE; ++e) y[a][e] = REV ? __shfl_down(v[a][e], off, 64) : __shfl_up(v[a][e], off, 64);
    const bool take = REV ? (lane + off < 64) : (lane >= off);
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int e = 0; e < EE; ++e)
        if (take) v[a][e] += y[a][e];
  }
  if (lane == (REV ? 0 : 63)) {
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int e = 0; e < EE; ++e) sh[a * NSEG + e * NW + w] = v[a][e];
  }
  __syncthreads();
#pragma unroll
  for (int a = 0; a < NA; ++a) {
    const double* s = sh + a * NSEG;
    double run = 0.0;  // the segments of the elements before (after) e
    if (!REV) {
#pragma unroll
      for (int e = 0; e < EE; ++e) {
        double off = run;
#pragma unroll
        for (int q = 0; q < NW; ++q) {
          if (q < w) off += s[e * NW + q];
          run += s[e * NW + q];
        }
        v[a][e] += off;
      }
    } else {
#pragma unroll
      for (int e = EE - 1; e >= 0; --e) {
        double off = run;
#pragma unroll
        for (int q = NW - 1; q >= 0; --q) {
          if (q > w) off += s[e * NW + q];
          run += s[e * NW + q];
        }
        v[a][e] += off;
      }
    }
    tot[a] = run;
  }
  __syncthreads();
}

// ------------------------------------------------------------ arrival
// Per-RHS arrival counters of the first launches (the last workgroup of a
// RHS forms that RHS's tile carries).  Hierarchical: arrival i
// of n counts at group counter i % 16, the last arrival of a group at the top
// counter -- a few hundred atomics on ONE address serialise at the memory-side
// atomic unit (tens of microseconds), sixteen lines do not.  Each counter is
// reset by the arrival that completes it.
//
// Hand-over between the workgroups of ONE launch: the values the last
// arrival reads are written with device-coherent stores (cst: agent-scope
// atomic stores, written through the XCD's L2) and read with device-coherent
// loads (cld: they bypass the reader's L2, which may hold lines of the
// previous launch), and every thread waits for its stores (s_waitcnt) before
// its workgroup's counter increment.  Agent-scope release / acquire fences
// would formally order plain stores instead, but on gfx950 an agent-scope
// release writes back the whole XCD L2 (the eight L2s are not coherent with
// each other): one write-back per workgroup measured 2-3x slower here
// (round 4: a VJP first launch 36 -> 131 us, second 116 -> 210 us at C3).
// Values handed to a LATER launch need neither (kernel boundaries write back
// and invalidate the L2s).  The counters are one device-global set (and the
// callers share one workspace): two calls must never run concurrently.  The
// launcher enforces it (guard_enter below): a call on another stream than
// the previous call's waits for that stream's work first.
constexpr int NGRP = 16;
struct Line {
  unsigned v[16];  // one 64-byte line per counter
};
__device__ Line g_arrive[2][MAXR][NGRP + 1];

// true in exactly one of the n workgroups (arrival index idx) that call it
// with the same counter set, after every caller's device-coherent stores
// before the call are complete
__device__ __forceinline__ bool last_arrival(Line* ctr, int idx, int n, int* lds_flag) {
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) {
    const int ng = n < NGRP ? n : NGRP;
    const int q = idx % ng;
    const unsigned gsz = (unsigned)(n / ng + (q < n % ng ? 1 : 0));
    bool last = false;
    if (__hip_atomic_fetch_add(&ctr[q].v[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gsz - 1) {
      __hip_atomic_store(&ctr[q].v[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__hip_atomic_fetch_add(&ctr[NGRP].v[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
          (unsigned)ng - 1) {
        __hip_atomic_store(&ctr[NGRP].v[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = true;
      }
    }
    *lds_flag = last ? 1 : 0;
  }
  __syncthreads();
  return *lds_flag != 0;
}

// Workgroup -> (tile, RHS): a 1-D grid of roundup(nb, 8) * k workgroups in
// which the k right-hand sides of one tile are consecutive slots of one XCD
// group (workgroups are dealt round-robin over the 8 XCDs: w and w + 8 share
// one), so the per-bin constants the RHS share are read from HBM once and
// from that XCD's L2 after; padding workgroups return at once.
__device__ __forceinline__ bool place(int nb, int k, int& tile, int& r) {
  const int w = blockIdx.x, xg = w & 7, slot = w >> 3;
  const int bl = slot / k;
  r = slot - bl * k;
  tile = bl * 8 + xg;
  return tile < nb;
}
static unsigned grid_of(int nb, int k) { return (unsigned)(((nb + 7) & ~7) * k); }

__device__ __forceinline__ double beta_of(const double* scb) {
  double beta = scb[NFT_CG_GAMMA] / scb[NFT_CG_GPREV];
  if (!(beta > 0.0)) beta = 0.0;
  return beta;
}

// exclusive block scan of Q values per thread (striped: tile t0 + q*NT +
// tid), forward or reversed, with a running carry across chunks: ex = the
// exclusive values, run advanced by the chunk total
template <bool REV, int Q>
__device__ __forceinline__ void chunk_scan(const double (&x)[Q], double (&ex)[Q], double& run, double* sh) {
  double v[1][Q], t[1];
#pragma unroll
  for (int q = 0; q < Q; ++q) v[0][q] = x[q];
  scan_arr<1, Q, REV>(v, t, sh);
#pragma unroll
  for (int q = 0; q < Q; ++q) ex[q] = run + (v[0][q] - x[q]);
  run += t[0];
}
constexpr int CQ = 2;  // tiles per thread in the carry scans (chunks of 512 tiles)


// ======================================================================= JVP
// VT: storage of the latent vectors, da and g (double, or float for the
// fp32-storage CG); constants, workspace, sums and CG scalars stay double
template <typename VT>
struct Jvp2Args {
  AmpConst c;              // constants (shared by every RHS), B and flags
  const AmpConst* dcs;     // per-RHS constants (device) or null
  const AmpConst* dc1;     // one device constant set shared by every RHS, or null
  VT* t[6];                // tangent keys of RHS 0 (rows ls apart); with dir the CG direction, updated in place
  const VT* r[6];          // residual keys of RHS 0 (dir only)
  long long ls;
  VT* da;                  // da[r * vs + b * des]
  long long vs, des;
  double* ws;              // per-RHS workspace, wsd doubles apart
  long long wsd;
  int nrhs, nb;
  int dir;                 // carry d = max(0, gamma/gprev) d + r on the amplitude keys
  const double* sc;        // CG scalar blocks (dir)
  double* part;            // d.d partials: part[r * pstride + tile] = shift * d.d (dir)
  long long pstride;
  double shift;
  const double* tab;       // constant-scan table (nft_amp2_prepare) or null
};

// workspace of one RHS: Eh [M, padded], the tile sums (7 rows of nb: agg1,
// agg2, MS1, LVt, MS2, MS3, MS4), 8 scalars (the 5 tangents after the
// direction update), the carries C1 [nb], C2 [nb], then T, dS
struct JWs {
  long long rows, scal, c1, c2, glb;
};
__device__ __host__ __forceinline__ JWs jws(int M, int nb) {
  JWs w;
  w.rows = ((long long)M + 63) & ~63LL;
  w.scal = w.rows + 7LL * nb;
  w.c1 = w.scal + 8;
  w.c2 = w.c1 + nb;
  w.glb = w.c2 + nb;
  return w;
}

// Constant-scan table of one constant set (nft_amp2_prepare, modes 0 / 2):
// the tile-local scans and tile sums that involve the constants only -- the
// forward scan of lv (LVc), the reverse scans of mspec (ym) and of the two
// constant VJP weights (g1m, g1l), the forward scan of p2 (p2c), and the
// constant tile-sum rows of the JVP (LVt, MS2..MS4) and the VJP -- formed
// once per linearisation by the kernels' own scan and sum code on the same
// operands, so the TB kernels read bitwise the values they would otherwise
// form, with a third to a half of the scans.
enum { TJ_LVT = 0, TJ_MS2, TJ_MS3, TJ_MS4, TV_R2M, TV_R3M, TV_AM, TV_AWM, TV_AWL, TV_P0M, TV_P0S, TV_Q2M, TV_Q2L,
       TV_P2S, TV_P1M, TV_P1S, T_NROWS };
struct Tab {
  long long lvc, ym, g1m, g1l, p2c, rows;
};
__device__ __host__ __forceinline__ Tab tab_of(int M, int nb) {
  const long long Mp = ((long long)M + 63) & ~63LL;
  Tab t;
  t.lvc = 0;
  t.ym = Mp;
  t.g1m = 2 * Mp;
  t.g1l = 3 * Mp;
  t.p2c = 4 * Mp;
  t.rows = 5 * Mp;
  (void)nb;
  return t;
}
__host__ __forceinline__ long long tab_size(long long B, int nb) {
  return tab_of((int)(B - 2), nb).rows + (long long)T_NROWS * nb;
}
// the constant set of RHS r by item mode (a template parameter, so that a
// device set is read with scalar loads from the constant address space: its
// pointers land in SGPRs and the per-bin loads wait on nothing)
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
template <int MODE>
__device__ __forceinline__ AmpConst const_of(const AmpConst& c, const AmpConst* dcs, const AmpConst* dc1, int r) {
  if constexpr (MODE == 1) return load_const(dcs + r);
  else if constexpr (MODE == 2) return load_const(dc1);
  else return c;
}

// first launch: direction update, tile-local scans, Eh, the tile sums; the
// last workgroup of each RHS then forms that RHS's tile carries.  TB: the
// constant scan (LVc) and sums (LVt, MS2..MS4) from the table
template <typename VT, int MODE, bool TB>
__global__ NFT_AMP2_LB void jvp2a_kernel(Jvp2Args<VT> a) {
  __shared__ double sh[2 * E * NW + 8 * NW];
  __shared__ int lflag;
  int i, r;
  if (!place(a.nb, a.nrhs, i, r)) return;
  const int tid = threadIdx.x;
  const AmpConst c = const_of<MODE>(a.c, a.dcs, a.dc1, r);  // by value: loaded once, no aliasing with the stores
  const int M = (int)(a.c.B - 2);
  const bool flex = a.c.has_flex, asp = a.c.has_asp;
  const int nb = a.nb;
  const int j0 = i * TL + tid;  // striped: bin j0 + e * NT
  const long long ro = (long long)r * a.ls;
  double* __restrict__ W = a.ws + (long long)r * a.wsd;
  const JWs L = jws(M, nb);
  bool live = false;
  double bt = 0.0;
  if (a.dir) {
    const double* scb = a.sc + (long long)r * NS_;
    live = scb[NFT_CG_DONE] == 0.0;
    bt = beta_of(scb);
  }
  const bool upd = a.dir && live;
  // every load of the phase first (the direction's stores cannot be passed)
  double sv[5];
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    sv[q] = 0.0;
    if (!a.t[q] || (q == KFLEX && !flex) || (q == KASP && !asp) || (q == KZM && !c.has_zm)) continue;
    sv[q] = a.t[q][ro];
    if (upd) sv[q] = bt * sv[q] + a.r[q][ro];
  }
  double d0[E], d1[E], r0[E], r1[E], lvv[E], c0v[E], sfv[E], vsl[E], qf[E], qa[E], msv[E], scv[E];
  VT* __restrict__ ts = a.t[KSPEC] ? a.t[KSPEC] + ro : nullptr;
  const VT* __restrict__ rs = (upd && a.r[KSPEC]) ? a.r[KSPEC] + ro : nullptr;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int j = j0 + e * NT;
    const bool ok = j < M;
    const int b = j + 2;
    const bool okf = ok && flex;
    d0[e] = okf ? ts[j] : 0.0;
    d1[e] = okf ? ts[M + j] : 0.0;
    r0[e] = (okf && rs) ? rs[j] : 0.0;
    r1[e] = (okf && rs) ? rs[M + j] : 0.0;
    lvv[e] = okf ? G_(c.lv)[j] : 0.0;
    c0v[e] = okf ? G_(c.c0)[j] : 0.0;
    sfv[e] = okf ? G_(c.sf)[j] : 0.0;
    vsl[e] = ok ? G_(c.vslope)[b] : 0.0;
    qf[e] = okf ? G_(c.Qf)[b] : 0.0;
    qa[e] = (ok && asp) ? G_(c.Qa)[b] : 0.0;
    msv[e] = ok ? G_(c.mspec)[b] : 0.0;
    scv[e] = (ok && !TB) ? G_(c.sc)[b] : 0.0;
  }
  double dd = 0.0;
  constexpr int NTH = TB ? 1 : 2;
  double u[1][E], th[NTH][E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int j = j0 + e * NT;
    if (rs && j < M) {
      d0[e] = bt * d0[e] + r0[e];
      d1[e] = bt * d1[e] + r1[e];
      ts[j] = d0[e];
      ts[M + j] = d1[e];
      dd += d0[e] * d0[e] + d1[e] * d1[e];
    }
    // t = (c + c_prev)/2 lv + t0 c0 with c_prev = c - u (amp_jvp_3) is
    // loc1 lv + pre on the carry-free local scan loc1
    u[0][e] = d1[e] * sfv[e];
    th[0][e] = d0[e] * c0v[e] - u[0][e] / 2 * lvv[e];
    if constexpr (!TB) th[NTH - 1][e] = lvv[e];
  }
  double agg1 = 0.0, agg2 = 0.0, LVt = 0.0;
  if (flex) {
    double t1[1], t2[NTH];
    scan_arr<1, E, false>(u, t1, sh);  // u -> loc1
    agg1 = t1[0];
#pragma unroll
    for (int e = 0; e < E; ++e) th[0][e] += u[0][e] * lvv[e];
    scan_arr<NTH, E, false>(th, t2, sh);  // -> loc2 (, LVc)
    agg2 = t2[0];
    LVt = t2[NTH - 1];
  }
  // Eh = vslope ssl + loc2 + sf Qf + sa Qa (stored); tile sums MS1..MS4, d.d
  const double ssl = c.sig_s * sv[KSL];
  constexpr int KD = TB ? 1 : 4;  // the d.d slot
  double s[KD + 1];
#pragma unroll
  for (int q = 0; q < KD; ++q) s[q] = 0.0;
  s[KD] = dd;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int j = j0 + e * NT;
    if (j >= M) continue;
    double d = vsl[e] * ssl + (flex ? th[0][e] : 0.0);
    if (flex) d += sv[KFLEX] * qf[e];
    if (asp) d += sv[KASP] * qa[e];
    W[j] = d;
    s[0] += msv[e] * d;
    if constexpr (!TB) {
      s[1] += msv[e];
      s[2] += msv[e] * (flex ? th[NTH - 1][e] : 0.0);
      s[3] += msv[e] * scv[e];
    }
  }
  if (i == 0 && tid < 2) {  // bins 0 and 1: no integrated part
    const int b = tid;
    const double ms = G_(c.mspec)[b];
    double d = G_(c.vslope)[b] * ssl;
    if (flex) d += sv[KFLEX] * G_(c.Qf)[b];
    if (asp) d += sv[KASP] * G_(c.Qa)[b];
    s[0] += ms * d;
    if constexpr (!TB) s[3] += ms * G_(c.sc)[b];
  }
  btot<KD + 1>(s, sh);
  if (tid == 0) {
    double* R = W + L.rows;
    cst(R + 0 * nb + i, agg1);
    cst(R + 1 * nb + i, agg2);
    cst(R + 2 * nb + i, s[0]);
    if constexpr (!TB) {
      cst(R + 3 * nb + i, LVt);
      cst(R + 4 * nb + i, s[1]);
      cst(R + 5 * nb + i, s[2]);
      cst(R + 6 * nb + i, s[3]);
    }
    if (i == 0) {
#pragma unroll
      for (int q = 0; q < 5; ++q) W[L.scal + q] = sv[q];
    }
    if (a.dir) {
      double v = s[KD];
      if (i == 0) {
#pragma unroll
        for (int q = 0; q < 5; ++q) v += sv[q] * sv[q];
      }
      a.part[(long long)r * a.pstride + i] = live ? a.shift * v : 0.0;
    }
  }
  // the tile carries of this RHS (its last workgroup): chunks of 256 tiles
  // in order, C1 = exclusive scan of agg1, C2 = exclusive scan of
  // agg2 + C1 LVt, T = their total, dS = sum MS1 + C2 MS2 + C1 MS3 - T MS4
  if (!last_arrival(g_arrive[0][r], i, nb, &lflag)) return;
  const double* R = W + L.rows;
  const double* TR = TB ? a.tab + tab_of(M, nb).rows : nullptr;
  double run1 = 0.0, run2 = 0.0, ds = 0.0, m4 = 0.0;
  for (int t0 = 0; t0 < nb; t0 += CQ * NT) {
    // every row of the chunk loaded first
    double A1[CQ], A2[CQ], M1[CQ], LT[CQ], M2[CQ], M3[CQ], M4[CQ];
#pragma unroll
    for (int q = 0; q < CQ; ++q) {
      const int t = t0 + q * NT + tid;
      const bool ok = t < nb;
      A1[q] = ok ? cld(R + 0 * nb + t) : 0.0;
      A2[q] = ok ? cld(R + 1 * nb + t) : 0.0;
      M1[q] = ok ? cld(R + 2 * nb + t) : 0.0;
      if constexpr (TB) {
        LT[q] = ok ? TR[TJ_LVT * nb + t] : 0.0;
        M2[q] = ok ? TR[TJ_MS2 * nb + t] : 0.0;
        M3[q] = ok ? TR[TJ_MS3 * nb + t] : 0.0;
        M4[q] = ok ? TR[TJ_MS4 * nb + t] : 0.0;
      } else {
        LT[q] = ok ? cld(R + 3 * nb + t) : 0.0;
        M2[q] = ok ? cld(R + 4 * nb + t) : 0.0;
        M3[q] = ok ? cld(R + 5 * nb + t) : 0.0;
        M4[q] = ok ? cld(R + 6 * nb + t) : 0.0;
      }
    }
    double C1[CQ], C2[CQ], y2[CQ];
#pragma unroll
    for (int q = 0; q < CQ; ++q) C1[q] = C2[q] = 0.0;
    if (flex) {
      chunk_scan<false, CQ>(A1, C1, run1, sh);
#pragma unroll
      for (int q = 0; q < CQ; ++q) y2[q] = A2[q] + C1[q] * LT[q];
      chunk_scan<false, CQ>(y2, C2, run2, sh);
    }
#pragma unroll
    for (int q = 0; q < CQ; ++q) {
      const int t = t0 + q * NT + tid;
      if (t >= nb) continue;
      W[L.c1 + t] = C1[q];
      W[L.c2 + t] = C2[q];
      ds += M1[q] + C2[q] * M2[q] + C1[q] * M3[q];
      m4 += M4[q];
    }
  }
  double v[2] = {ds, m4};
  btot<2>(v, sh);
  if (tid == 0) {
    const double T = flex ? run2 : 0.0;
    W[L.glb] = T;
    W[L.glb + 1] = v[0] - T * v[1];
  }
}

// second launch: da from Eh and the carries; tile 0 writes the scalar keys'
// new direction.  TB: LVc from the table
template <typename VT, int MODE, bool TB>
__global__ NFT_AMP2_LB void jvp2b_kernel(Jvp2Args<VT> a) {
  __shared__ double sh[E * NW + 8];
  int i, r;
  if (!place(a.nb, a.nrhs, i, r)) return;
  const int tid = threadIdx.x;
  const AmpConst c = const_of<MODE>(a.c, a.dcs, a.dc1, r);  // by value: loaded once, no aliasing with the stores
  const int M = (int)(a.c.B - 2);
  const bool flex = a.c.has_flex, asp = a.c.has_asp;
  const int nb = a.nb;
  const int j0 = i * TL + tid;  // striped: bin j0 + e * NT
  const double* __restrict__ W = a.ws + (long long)r * a.wsd;
  const JWs L = jws(M, nb);
  double eh[E], anv[E], scv[E], lvc[1][E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int j = j0 + e * NT;
    const bool ok = j < M;
    eh[e] = ok ? W[j] : 0.0;
    anv[e] = ok ? G_(c.An)[j + 2] : 0.0;
    scv[e] = ok ? G_(c.sc)[j + 2] : 0.0;
    lvc[0][e] = (ok && flex) ? (TB ? a.tab[j] : G_(c.lv)[j]) : 0.0;  // table: lvc at offset 0
  }
  const double C1 = W[L.c1 + i], C2 = W[L.c2 + i], T = W[L.glb], dS = W[L.glb + 1];
  const double* sv = W + L.scal;
  const double sfl = sv[KFL];
  if (flex && !TB) {
    double t[1];
    scan_arr<1, E, false>(lvc, t, sh);
  }
  const double dfl = c.fl * c.ls_f * sfl;
  VT* __restrict__ dr = a.da + (long long)r * a.vs;
  const int des = (int)a.des;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int j = j0 + e * NT;
    if (j >= M) continue;
    const double dp = (eh[e] + (C2 + C1 * lvc[0][e])) - T * scv[e];
    const double An = anv[e];
    dr[(j + 2) * des] = (dfl * An + c.fl * An * (dp / 2. - dS / (2. * c.S))) * c.total_volume;
  }
  if (i == 0 && tid < 2) {
    const int b = tid;
    double v;
    if (b == 0) {
      v = c.has_zm ? c.zm * c.ls_o * sv[KZM] : 0.0;
    } else {
      double d = G_(c.vslope)[b] * (c.sig_s * sv[KSL]);
      if (flex) d += sv[KFLEX] * G_(c.Qf)[b];
      if (asp) d += sv[KASP] * G_(c.Qa)[b];
      const double dp = d - T * G_(c.sc)[b];
      const double An = G_(c.An)[b];
      v = dfl * An + c.fl * An * (dp / 2. - dS / (2. * c.S));
    }
    dr[b * des] = v * c.total_volume;
  }
  if (a.dir && i == 0 && tid == 0 && a.sc[(long long)r * NS_ + NFT_CG_DONE] == 0.0) {
    const long long ro = (long long)r * a.ls;
#pragma unroll
    for (int q = 0; q < 5; ++q)
      if (a.t[q] && !(q == KFLEX && !flex) && !(q == KASP && !asp) && !(q == KZM && !c.has_zm)) a.t[q][ro] = sv[q];
  }
}

// ======================================================================= VJP
template <typename VT>
struct Vjp2Args {
  AmpConst c;
  const AmpConst* dcs;
  const AmpConst* dc1;
  const VT* g;             // g[r * gs + b]
  long long gs;
  // plain mode: out keys (= shift * d + J^T g) and the d keys for the shift
  // CG mode (cg): x, r, d keys, updated x -= alpha d, r -= alpha (q + shift d)
  VT* o[6];
  VT* o2[6];               // cg: r keys
  const VT* d[6];          // d keys (shift / cg)
  long long ls;
  double shift;
  double* ws;
  long long wsd;
  int nrhs, nb;
  int cg;
  double* sc;              // CG scalar blocks (cg: alpha read, finalized here)
  double* part;            // cg: rr / xr partials per tile, part[r * pstride + {0, nb} + tile]
  long long pstride;
  const double* gpart;     // cg: the grid segment's partials (rows rr, xr at 0 and gpr) per RHS
  long long gps, gpr;
  int ngp;
  const double* tab;       // constant-scan table (nft_amp2_prepare) or null
};

// workspace of one RHS: the tile sums (V_NROWS rows of nb), then the carries
// beta [nb], S1 [nb], then k, R1, R2, R4, R5
enum { V_R1 = 0, V_R2G, V_R3G, V_R2M, V_R3M, V_AG, V_AM, V_AWG, V_AWM, V_AWL, V_P0G, V_P0M, V_P0S, V_Q2G, V_Q2M,
       V_Q2L, V_P2S, V_P1G, V_P1M, V_P1S, V_CRR, V_CXR, V_NROWS };
struct VWs {
  long long bet, s1, glb;
};
__device__ __host__ __forceinline__ VWs vws(int nb) {
  VWs w;
  w.bet = (long long)V_NROWS * nb;
  w.s1 = w.bet + nb;
  w.glb = w.s1 + nb;
  return w;
}

// the table row of a VJP workspace row that is constant (-1: not constant)
__device__ __forceinline__ int vtab_row(int q) {
  switch (q) {
    case V_R2M: return TV_R2M;
    case V_R3M: return TV_R3M;
    case V_AM: return TV_AM;
    case V_AWM: return TV_AWM;
    case V_AWL: return TV_AWL;
    case V_P0M: return TV_P0M;
    case V_P0S: return TV_P0S;
    case V_Q2M: return TV_Q2M;
    case V_Q2L: return TV_Q2L;
    case V_P2S: return TV_P2S;
    case V_P1M: return TV_P1M;
    case V_P1S: return TV_P1S;
    default: return -1;
  }
}

// tile-local reverse scans of the VJP: y = [G, mspec] (yG, ym), then
// w = y lv/2 + y_{j+1} lv_{j+1}/2 with y_{j+1} = y_j - (its own term) for
// both and wl = lv/2 + lv_{j+1}/2; second: the reverse scans of w (g1G, g1m,
// g1l).  Both launches run it on the same inputs (bitwise the same values).
__device__ __forceinline__ void vjp_scans(const double (&G)[E], const double (&msv)[E], const double (&lvv)[E],
                                          const double (&lvn)[E], double (&y)[2][E], double (&w)[3][E],
                                          double (&ty)[2], double (&tw)[3], double* sh, bool second) {
#pragma unroll
  for (int e = 0; e < E; ++e) {
    y[0][e] = G[e];
    y[1][e] = msv[e];
  }
  scan_arr<2, E, true>(y, ty, sh);
#pragma unroll
  for (int e = 0; e < E; ++e) {
    w[0][e] = y[0][e] * lvv[e] / 2. + (y[0][e] - G[e]) * lvn[e] / 2.;
    w[1][e] = y[1][e] * lvv[e] / 2. + (y[1][e] - msv[e]) * lvn[e] / 2.;
    w[2][e] = lvv[e] / 2. + lvn[e] / 2.;
  }
  if (second) scan_arr<3, E, true>(w, tw, sh);
}

// the same for the cotangent terms only (the constant-scan table holds the
// mspec / weight scans): y = reverse scan of G, w = its weight term and,
// second, the reverse scan of w -- per array the operations of vjp_scans
__device__ __forceinline__ void vjp_scans_g(const double (&G)[E], const double (&lvv)[E], const double (&lvn)[E],
                                            double (&y)[1][E], double (&w)[1][E], double& ty, double* sh,
                                            bool second) {
#pragma unroll
  for (int e = 0; e < E; ++e) y[0][e] = G[e];
  double t[1];
  scan_arr<1, E, true>(y, t, sh);
  ty = t[0];
#pragma unroll
  for (int e = 0; e < E; ++e) w[0][e] = y[0][e] * lvv[e] / 2. + (y[0][e] - G[e]) * lvn[e] / 2.;
  if (second) {
    double t2[1];
    scan_arr<1, E, true>(w, t2, sh);
  }
}

// first launch: the tile sums (and, cg, this tile's slice of the grid
// segment's r.r / x.r partials); the last workgroup of each RHS then forms
// that RHS's k, R1, R2, R4, R5 and the carries beta, S1 of every tile.  TB:
// the constant rows and scans from the table
template <typename VT, int MODE, bool TB>
__global__ NFT_AMP2_LB void vjp2a_kernel(Vjp2Args<VT> a) {
  __shared__ double sh[3 * E * NW + 24 * NW];
  __shared__ int lflag;
  int i, r;
  if (!place(a.nb, a.nrhs, i, r)) return;
  const int tid = threadIdx.x;
  const AmpConst c = const_of<MODE>(a.c, a.dcs, a.dc1, r);  // by value: loaded once, no aliasing with the stores
  const int M = (int)(a.c.B - 2);
  const bool flex = a.c.has_flex, asp = a.c.has_asp;
  const int nb = a.nb;
  const int j0 = i * TL + tid;  // striped: bin j0 + e * NT
  const double TV = c.total_volume;
  double* __restrict__ W = a.ws + (long long)r * a.wsd;
  const VT* __restrict__ gr = a.g + (long long)r * a.gs;
  double gb[E], anv[E], msv[E], vsl[E], scv[E], lvv[E], lvn[E], p0v[E], p1v[E], pc[1][E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int j = j0 + e * NT;
    const bool ok = j < M, okf = ok && flex;
    const int b = j + 2;
    gb[e] = ok ? gr[b] : 0.0;
    anv[e] = ok ? G_(c.An)[b] : 0.0;
    msv[e] = (ok && !TB) ? G_(c.mspec)[b] : 0.0;
    vsl[e] = ok ? G_(c.vslope)[b] : 0.0;
    scv[e] = ok ? G_(c.sc)[b] : 0.0;
    lvv[e] = okf ? G_(c.lv)[j] : 0.0;
    lvn[e] = (okf && j + 1 < M) ? G_(c.lv)[j + 1] : 0.0;
    p0v[e] = okf ? G_(c.p0)[j] : 0.0;
    p1v[e] = (okf && asp) ? G_(c.p1)[j] : 0.0;
    pc[0][e] = okf ? (TB ? a.tab[tab_of(M, nb).p2c + j] : G_(c.p2)[j]) : 0.0;  // TB: already scanned
  }
  // grid partial slice (cg)
  double crr = 0.0, cxr = 0.0;
  if (a.cg) {
    const int per = (a.ngp + nb - 1) / nb;
    const int lo = i * per, hi = min(a.ngp, lo + per);
    const double* gp = a.gpart + (long long)r * a.gps;
    for (int t = lo + tid; t < hi; t += NT) {
      crr += gp[t];
      cxr += gp[a.gpr + t];
    }
  }
  // G_b = An_b (fl TV g_b) / 2 (gapre without its normalisation term)
  double G[E];
  // every row but aggG / aggm (scan totals) and P2S; TB: the cotangent rows
  // R1, R2G, R3G, AWG, P0G, Q2G, P1G, CRR, CXR only
  constexpr int NV = TB ? 8 : V_NROWS - 3;
  double s[NV + 1];
#pragma unroll
  for (int q = 0; q <= NV; ++q) s[q] = 0.0;
  // s index of row q: q < V_AG -> q; V_AWG.. -> q - 2 (aggG, aggm skipped), P2S skipped
  auto S = [&](int row) -> double& {
    if constexpr (TB) {
      switch (row) {
        case V_R1: return s[0];
        case V_R2G: return s[1];
        case V_R3G: return s[2];
        case V_AWG: return s[3];
        case V_P0G: return s[4];
        case V_Q2G: return s[5];
        case V_P1G: return s[6];
        case V_CRR: return s[7];
        default: return s[8];  // V_CXR
      }
    } else {
      return s[row < V_AG ? row : (row < V_P2S ? row - 2 : row - 3)];
    }
  };
#pragma unroll
  for (int e = 0; e < E; ++e) {
    G[e] = anv[e] * (c.fl * (TV * gb[e])) / 2.;
    S(V_R1) += TV * gb[e] * anv[e];
    S(V_R2G) += vsl[e] * G[e];
    S(V_R3G) += G[e] * scv[e];
    if constexpr (!TB) {
      S(V_R2M) += vsl[e] * msv[e];
      S(V_R3M) += msv[e] * scv[e];
    }
  }
  if (i == 0 && tid < 2) {  // bins 0 and 1
    const int b = tid;
    const double an = G_(c.An)[b], ms = G_(c.mspec)[b], vs = G_(c.vslope)[b], scb = G_(c.sc)[b];
    const double g_ = gr[b];
    const double ga = an * (c.fl * (b > 0 ? TV * g_ : 0.0)) / 2.;
    if (b > 0) S(V_R1) += TV * g_ * an;
    S(V_R2G) += vs * ga;
    S(V_R3G) += ga * scb;
    if constexpr (!TB) {
      S(V_R2M) += vs * ms;
      S(V_R3M) += ms * scb;
    }
  }
  double ty[2] = {0.0, 0.0}, tpc[1] = {0.0};
  if constexpr (TB) {
    if (flex) {
      double y[1][E], w[1][E];
      vjp_scans_g(G, lvv, lvn, y, w, ty[0], sh, false);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        S(V_AWG) += w[0][e];
        S(V_P0G) += y[0][e] * p0v[e];
        S(V_Q2G) += w[0][e] * pc[0][e];
        S(V_P1G) += y[0][e] * p1v[e];
      }
    }
  } else if (flex) {
    double y[2][E], w[3][E], tw[3];
    vjp_scans(G, msv, lvv, lvn, y, w, ty, tw, sh, false);
    // p2c: tile-local forward scan of p2, so that sum_j g1_j p2_j (g1 the
    // reverse scan of w) is sum_j w_j p2c_j without that second scan
    scan_arr<1, E, false>(pc, tpc, sh);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      S(V_AWG) += w[0][e];
      S(V_AWM) += w[1][e];
      S(V_AWL) += w[2][e];
      S(V_P0G) += y[0][e] * p0v[e];
      S(V_P0M) += y[1][e] * p0v[e];
      S(V_P0S) += p0v[e];
      S(V_Q2G) += w[0][e] * pc[0][e];
      S(V_Q2M) += w[1][e] * pc[0][e];
      S(V_Q2L) += w[2][e] * pc[0][e];
      S(V_P1G) += y[0][e] * p1v[e];
      S(V_P1M) += y[1][e] * p1v[e];
      S(V_P1S) += p1v[e];
    }
  }
  S(V_CRR) += crr;
  S(V_CXR) += cxr;
  btot<NV + 1>(s, sh);
  if (tid == 0) {
#pragma unroll
    for (int q = 0; q < V_NROWS; ++q) {
      if (TB && vtab_row(q) >= 0) continue;
      double v;
      if (q == V_AG) v = ty[0];
      else if (q == V_AM) v = ty[1];
      else if (q == V_P2S) v = tpc[0];
      else v = S(q);
      cst(W + (long long)q * nb + i, v);
    }
  }
  if (!last_arrival(g_arrive[1][r], i, nb, &lflag)) return;
  // this RHS's globals (fixed-order sums over the tiles) ...
  const double* TR = TB ? a.tab + tab_of(M, nb).rows : nullptr;
  auto row = [&](int q, int t) {
    if constexpr (TB) {
      const int tq = vtab_row(q);
      if (tq >= 0) return TR[(long long)tq * nb + t];
    }
    return cld(W + (long long)q * nb + t);
  };
  double gsum[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  for (int t = tid; t < nb; t += NT) {
    gsum[0] += row(V_R1, t);
    gsum[1] += row(V_R3G, t);
    gsum[2] += row(V_R3M, t);
    gsum[3] += row(V_R2G, t);
    gsum[4] += row(V_R2M, t);
  }
  btot<5>(gsum, sh);
  const double kv = c.fl * gsum[0] / (2. * c.S);
  const double R3 = gsum[1] - kv * gsum[2];
  const VWs L = vws(nb);
  // ... and, from the last tile down in chunks of 512, the carries
  // beta(t) = SG - k SM - R3 and S1(t) (exclusive reverse sums), R4, R5
  double u[2] = {0.0, 0.0};
  if (flex) {
    double rg = 0.0, rm = 0.0, rz = 0.0;
    const int nch = (nb + CQ * NT - 1) / (CQ * NT);
    for (int ch = nch - 1; ch >= 0; --ch) {
      // every row of the chunk loaded first
      constexpr int NRW = 14;
      const int rows_[NRW] = {V_AG, V_AM, V_AWG, V_AWM, V_AWL, V_P0G, V_P0M, V_P0S, V_Q2G, V_Q2M, V_Q2L, V_P2S,
                              V_P1G, V_P1M};
      double x[NRW][CQ], p1s[CQ];
#pragma unroll
      for (int q = 0; q < CQ; ++q) {
        const int t = ch * CQ * NT + q * NT + tid;
        const bool ok = t < nb;
#pragma unroll
        for (int k = 0; k < NRW; ++k) x[k][q] = ok ? row(rows_[k], t) : 0.0;
        p1s[q] = ok ? row(V_P1S, t) : 0.0;
      }
      double sg[CQ], sm[CQ], z[CQ], S1[CQ], bet[CQ];
      chunk_scan<true, CQ>(x[0], sg, rg, sh);
      chunk_scan<true, CQ>(x[1], sm, rm, sh);
#pragma unroll
      for (int q = 0; q < CQ; ++q) {
        const int t = ch * CQ * NT + q * NT + tid;
        bet[q] = (sg[q] - kv * sm[q]) - R3;
        z[q] = t < nb ? ((x[2][q] - kv * x[3][q]) + bet[q] * x[4][q]) : 0.0;
      }
      chunk_scan<true, CQ>(z, S1, rz, sh);
#pragma unroll
      for (int q = 0; q < CQ; ++q) {
        const int t = ch * CQ * NT + q * NT + tid;
        if (t >= nb) continue;
        W[L.bet + t] = bet[q];
        W[L.s1 + t] = S1[q];
        u[0] += ((x[5][q] - kv * x[6][q]) + bet[q] * x[7][q]) + ((x[8][q] - kv * x[9][q]) + bet[q] * x[10][q]) +
                S1[q] * x[11][q];
        u[1] += (x[12][q] - kv * x[13][q]) + bet[q] * p1s[q];
      }
    }
  }
  btot<2>(u, sh);
  if (tid == 0) {
    W[L.glb + 0] = kv;
    W[L.glb + 1] = gsum[0];
    W[L.glb + 2] = gsum[3] - kv * gsum[4];
    W[L.glb + 3] = u[0];
    W[L.glb + 4] = u[1];
  }
}

// second launch: the tile-local scans again and the spectrum cotangents
// (plain: outputs; cg: the update), tile 0 the scalar cotangents; cg: the
// r.r / x.r partials and the finalize by the last workgroup of the grid.
// TB: the constant scans from the table
template <typename VT, int MODE, bool TB>
__global__ NFT_AMP2_LB void vjp2b_kernel(Vjp2Args<VT> a) {
  __shared__ double sh[3 * E * NW + 8];
  int i, r;
  const bool valid = place(a.nb, a.nrhs, i, r);
  if (!valid) return;
  const int tid = threadIdx.x;
  const AmpConst c = const_of<MODE>(a.c, a.dcs, a.dc1, r);  // by value: loaded once, no aliasing with the stores
  const int M = (int)(a.c.B - 2);
  const bool flex = a.c.has_flex, asp = a.c.has_asp;
  const int nb = a.nb;
  const int j0 = i * TL + tid;  // striped: bin j0 + e * NT
  const double TV = c.total_volume;
  const double* __restrict__ W = a.ws + (long long)r * a.wsd;
  const VT* __restrict__ gr = a.g + (long long)r * a.gs;
  const VWs L = vws(nb);
  const long long ro = (long long)r * a.ls;
  // every load first (the output operands loaded after the scans measured
  // slower: 54 -> 61 us at C3)
  double gb[E], anv[E], msv[E], lvv[E], lvn[E], c0v[E], sfv[E], x0[E], x1[E], r0[E], r1[E], d0[E], d1[E];
  VT* __restrict__ os = a.o[KSPEC] ? a.o[KSPEC] + ro : nullptr;
  VT* __restrict__ rsp = (a.cg && a.o2[KSPEC]) ? a.o2[KSPEC] + ro : nullptr;
  const VT* __restrict__ ds = a.d[KSPEC] ? a.d[KSPEC] + ro : nullptr;
  auto out_loads = [&]() {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int j = j0 + e * NT;
      const bool okf = j < M && flex;
      c0v[e] = okf ? G_(c.c0)[j] : 0.0;
      sfv[e] = okf ? G_(c.sf)[j] : 0.0;
      x0[e] = (okf && rsp) ? os[j] : 0.0;
      x1[e] = (okf && rsp) ? os[M + j] : 0.0;
      r0[e] = (okf && rsp) ? rsp[j] : 0.0;
      r1[e] = (okf && rsp) ? rsp[M + j] : 0.0;
      d0[e] = (okf && ds) ? ds[j] : 0.0;
      d1[e] = (okf && ds) ? ds[M + j] : 0.0;
    }
  };
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int j = j0 + e * NT;
    const bool ok = j < M, okf = ok && flex;
    gb[e] = okf ? gr[j + 2] : 0.0;
    anv[e] = okf ? G_(c.An)[j + 2] : 0.0;
    msv[e] = (okf && !TB) ? G_(c.mspec)[j + 2] : 0.0;
    lvv[e] = okf ? G_(c.lv)[j] : 0.0;
    lvn[e] = (okf && j + 1 < M) ? G_(c.lv)[j + 1] : 0.0;
  }
  // TB: ym, g1m, g1l (the mspec scan and the two constant weight scans)
  double tym[E], tgm[E], tgl[E];
  if constexpr (TB) {
    const Tab T = tab_of(M, nb);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int j = j0 + e * NT;
      const bool okf = j < M && flex;
      tym[e] = okf ? a.tab[T.ym + j] : 0.0;
      tgm[e] = okf ? a.tab[T.g1m + j] : 0.0;
      tgl[e] = okf ? a.tab[T.g1l + j] : 0.0;
    }
  }
  out_loads();
  const double kv = W[L.glb + 0];
  const double bet = W[L.bet + i], S1 = W[L.s1 + i];
  double al = 0.0;
  bool okc = false;
  if (a.cg) {
    const double* scb = a.sc + (long long)r * NS_;
    const double curv = scb[NFT_CG_CURV], gprev = scb[NFT_CG_GAMMA];
    al = gprev / curv;
    okc = (curv == curv) && curv != 0.0 && (al >= 0.0) && (al == al) && scb[NFT_CG_DONE] == 0.0;
  }
  double rr = 0.0, xr = 0.0;
  if (flex) {
    double G[E];
#pragma unroll
    for (int e = 0; e < E; ++e) G[e] = anv[e] * (c.fl * (TV * gb[e])) / 2.;
    double y[TB ? 1 : 2][E], w[TB ? 1 : 3][E], ty[2], tw[3];
    if constexpr (TB) vjp_scans_g(G, lvv, lvn, y, w, ty[0], sh, true);
    else vjp_scans(G, msv, lvv, lvn, y, w, ty, tw, sh, true);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int j = j0 + e * NT;
      if (j >= M) continue;
      const double ym = TB ? tym[e] : y[TB ? 0 : 1][e];
      const double wm = TB ? tgm[e] : w[TB ? 0 : 1][e], wl = TB ? tgl[e] : w[TB ? 0 : 2][e];
      const double yv = (y[0][e] - kv * ym) + bet;
      const double g1 = ((w[0][e] - kv * wm) + bet * wl) + S1;
      const double q0 = yv * c0v[e], q1 = g1 * sfv[e];
      if (!a.cg) {
        double v0 = q0, v1 = q1;
        if (ds) {
          v0 += a.shift * d0[e];
          v1 += a.shift * d1[e];
        }
        os[j] = v0;
        os[M + j] = v1;
      } else {
        double xa = x0[e], xb = x1[e], ra = r0[e], rb = r1[e];
        if (okc) {
          xa = xa - al * d0[e];
          ra = ra - al * (q0 + a.shift * d0[e]);
          xb = xb - al * d1[e];
          rb = rb - al * (q1 + a.shift * d1[e]);
          os[j] = xa;
          rsp[j] = ra;
          os[M + j] = xb;
          rsp[M + j] = rb;
        }
        rr += ra * ra + rb * rb;
        xr += xa * ra + xb * rb;
      }
    }
  }
  // scalar cotangents (tile 0, thread 0): fl, sl, flex, asp, zm
  if (i == 0 && tid == 0) {
    double qv[5];
    bool has[5];
    qv[KFL] = c.fl * c.ls_f * W[L.glb + 1];
    has[KFL] = true;
    qv[KSL] = c.sig_s * W[L.glb + 2];
    has[KSL] = true;
    qv[KFLEX] = W[L.glb + 3];
    has[KFLEX] = flex;
    qv[KASP] = W[L.glb + 4];
    has[KASP] = asp;
    qv[KZM] = c.has_zm ? c.zm * c.ls_o * TV * gr[0] : 0.0;
    has[KZM] = c.has_zm;
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      if (!has[q] || !a.o[q]) continue;
      if (!a.cg) {
        a.o[q][ro] = qv[q] + (a.d[q] ? a.shift * a.d[q][ro] : 0.0);
      } else {
        double x = a.o[q][ro], rv = a.o2[q][ro];
        const double d = a.d[q][ro];
        if (okc) {
          x = x - al * d;
          rv = rv - al * (qv[q] + a.shift * d);
          a.o[q][ro] = x;
          a.o2[q][ro] = rv;
        }
        rr += rv * rv;
        xr += x * rv;
      }
    }
  }
  if (!a.cg) return;
  double v[2] = {rr, xr};
  btot<2>(v, sh);
  if (tid == 0) {
    double* pp = a.part + (long long)r * a.pstride;
    // this tile's amplitude sums, then its slice of the grid partials (read
    // by fin_kernel)
    pp[i] = v[0] + W[(long long)V_CRR * nb + i];
    pp[nb + i] = v[1] + W[(long long)V_CXR * nb + i];
  }
  // the finalize runs as a launch of its own (fin_kernel): a last-arrival
  // finalize in this kernel made every workgroup wait for its stores and an
  // atomic before it could retire (4-RHS VJP at 2048^2 45 -> 37 + 6 us, 4096^2
  // fp32 153 -> 140 + 6 us; iteration -9 us at both)
}

// the finalize of RHS r: the tile partials folded in index order, then
// cg_finalize_kernel's bookkeeping
template <typename VT>
__device__ __forceinline__ void fin_rhs(const Vjp2Args<VT>& a, int r, double* sh) {
  const int tid = threadIdx.x, nb = a.nb;
  {
    const double* pp = a.part + (long long)r * a.pstride;
    double f[2] = {0.0, 0.0};
    for (int t = tid; t < nb; t += NT) {
      f[0] += pp[t];
      f[1] += pp[nb + t];
    }
    btot<2>(f, sh);
    if (tid == 0) {
      double* scb = a.sc + (long long)r * NS_;
      scb[NFT_CG_LAZY] += 1.0;  // the deferred iterate's ring slot (every step, stopped or not)
      if (scb[NFT_CG_DONE] == 0.0) {
        const double curv = scb[NFT_CG_CURV], gprev = scb[NFT_CG_GAMMA];
        const double alpha = gprev / curv;
        const bool ok = (curv == curv) && curv != 0.0 && (alpha >= 0.0) && (alpha == alpha);
        scb[NFT_CG_ALPHA] = alpha;
        scb[NFT_CG_FLAG] = ok ? 0.0 : 1.0;
        scb[NFT_CG_ITER] += 1.0;
        if (ok) {
          scb[NFT_CG_GPREV] = gprev;
          scb[NFT_CG_GAMMA] = f[0];
          scb[NFT_CG_XR] = f[1];
          scb[NFT_CG_XB] = 0.0;
        }
        if (!ok || (scb[NFT_CG_AUTO] != 0.0 && !(f[0] > 0.0))) scb[NFT_CG_DONE] = 2.0;
      }
    }
  }
}

// the finalize: one workgroup per RHS, after every tile of vjp2b_kernel
template <typename VT>
__global__ __launch_bounds__(NT) void fin_kernel(Vjp2Args<VT> a) {
  __shared__ double sh[8 * NW];
  fin_rhs(a, (int)blockIdx.x, sh);
}

// ======================================================== constant-scan table
// one workgroup per tile: the constant scans and tile sums of the four
// kernels, each by the code (scan_arr / btot, the same operands and order of
// the per-thread sums) the non-table kernels run on them
template <int MODE>
__global__ __launch_bounds__(NT) void prep_kernel(AmpConst c0_, const AmpConst* dc1, int nb, double* __restrict__ tab) {
  __shared__ double sh[3 * E * NW + 24 * NW];
  const int i = blockIdx.x;
  if (i >= nb) return;
  const int tid = threadIdx.x;
  const AmpConst c = const_of<MODE>(c0_, nullptr, dc1, 0);
  const int M = (int)(c0_.B - 2);
  const bool flex = c0_.has_flex, asp = c0_.has_asp;
  const int j0 = i * TL + tid;
  const Tab T = tab_of(M, nb);
  double* TR = tab + T.rows;
  double lvv[E], lvn[E], msv[E], scv[E], vsl[E], p0v[E], p1v[E], pc[1][E], lvc[1][E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int j = j0 + e * NT;
    const bool ok = j < M, okf = ok && flex;
    const int b = j + 2;
    lvv[e] = okf ? G_(c.lv)[j] : 0.0;
    lvn[e] = (okf && j + 1 < M) ? G_(c.lv)[j + 1] : 0.0;
    msv[e] = ok ? G_(c.mspec)[b] : 0.0;
    scv[e] = ok ? G_(c.sc)[b] : 0.0;
    vsl[e] = ok ? G_(c.vslope)[b] : 0.0;
    p0v[e] = okf ? G_(c.p0)[j] : 0.0;
    p1v[e] = (okf && asp) ? G_(c.p1)[j] : 0.0;
    pc[0][e] = okf ? G_(c.p2)[j] : 0.0;
    lvc[0][e] = lvv[e];
  }
  // JVP (jvp2a): LVc and LVt; MS2 = sum mspec, MS3 = sum mspec LVc, MS4 =
  // sum mspec sc (+ bins 0 and 1 on tile 0)
  double LVt = 0.0;
  if (flex) {
    double t[1];
    scan_arr<1, E, false>(lvc, t, sh);
    LVt = t[0];
  }
  double sj[3] = {0.0, 0.0, 0.0};
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int j = j0 + e * NT;
    if (j >= M) continue;
    sj[0] += msv[e];
    sj[1] += msv[e] * (flex ? lvc[0][e] : 0.0);
    sj[2] += msv[e] * scv[e];
  }
  if (i == 0 && tid < 2) sj[2] += G_(c.mspec)[tid] * G_(c.sc)[tid];
  btot<3>(sj, sh);
  // VJP (vjp2a / vjp2b): ym, the weight scans g1m / g1l, p2c and the rows
  double y[2][E], w[3][E], ty[2] = {0.0, 0.0}, tw[3], tpc[1] = {0.0};
  double G0[E];
#pragma unroll
  for (int e = 0; e < E; ++e) G0[e] = 0.0;
  constexpr int NR = 12;
  double sv[NR];  // R2M R3M AWM AWL P0M P0S Q2M Q2L P1M P1S (+2 unused)
#pragma unroll
  for (int q = 0; q < NR; ++q) sv[q] = 0.0;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    sv[0] += vsl[e] * msv[e];
    sv[1] += msv[e] * scv[e];
  }
  if (i == 0 && tid < 2) {
    const int b = tid;
    const double ms = G_(c.mspec)[b], vs = G_(c.vslope)[b], scb = G_(c.sc)[b];
    sv[0] += vs * ms;
    sv[1] += ms * scb;
  }
  if (flex) {
    vjp_scans(G0, msv, lvv, lvn, y, w, ty, tw, sh, false);
    scan_arr<1, E, false>(pc, tpc, sh);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      sv[2] += w[1][e];
      sv[3] += w[2][e];
      sv[4] += y[1][e] * p0v[e];
      sv[5] += p0v[e];
      sv[6] += w[1][e] * pc[0][e];
      sv[7] += w[2][e] * pc[0][e];
      sv[8] += y[1][e] * p1v[e];
      sv[9] += p1v[e];
    }
    // the second launch's reverse scans of the two constant weights
    double w2[2][E], t2[2];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      w2[0][e] = w[1][e];
      w2[1][e] = w[2][e];
    }
    scan_arr<2, E, true>(w2, t2, sh);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int j = j0 + e * NT;
      if (j >= M) continue;
      tab[T.lvc + j] = lvc[0][e];
      tab[T.ym + j] = y[1][e];
      tab[T.g1m + j] = w2[0][e];
      tab[T.g1l + j] = w2[1][e];
      tab[T.p2c + j] = pc[0][e];
    }
  }
  btot<NR>(sv, sh);
  if (tid == 0) {
    TR[TJ_LVT * nb + i] = LVt;
    TR[TJ_MS2 * nb + i] = sj[0];
    TR[TJ_MS3 * nb + i] = sj[1];
    TR[TJ_MS4 * nb + i] = sj[2];
    TR[TV_R2M * nb + i] = sv[0];
    TR[TV_R3M * nb + i] = sv[1];
    TR[TV_AM * nb + i] = ty[1];
    TR[TV_AWM * nb + i] = sv[2];
    TR[TV_AWL * nb + i] = sv[3];
    TR[TV_P0M * nb + i] = sv[4];
    TR[TV_P0S * nb + i] = sv[5];
    TR[TV_Q2M * nb + i] = sv[6];
    TR[TV_Q2L * nb + i] = sv[7];
    TR[TV_P2S * nb + i] = tpc[0];
    TR[TV_P1M * nb + i] = sv[8];
    TR[TV_P1S * nb + i] = sv[9];
  }
}

// ------------------------------------------------------------------ launch
static int nblk(long long n, long long per) { return (int)std::max<long long>(1, (n + per - 1) / per); }

// Cross-stream ordering of the calls (the device-global arrival counters and
// the shared workspace make two concurrently running calls corrupt each
// other): a call on a different stream than the previous eager call first
// waits on the host for that stream's work (hipStreamSynchronize), so eager
// calls from any number of streams and host threads execute one after the
// other, and single-stream use -- every call on the hot path -- pays nothing
// on the device (an event recorded after every call measured +5 us per launch
// pair).  g_guard_mu is held from the check through the launches of a call
// (AmpGuard), so two host threads cannot both skip the wait (ctypes releases
// the GIL around these calls).  The previous stream may have been destroyed
// since: a failing stream wait falls back to a device-wide synchronisation.
// A call on a stream under HIP-graph capture is not tracked: a captured graph
// is ordered by its replay stream, so graphs holding these kernels must not
// be replayed concurrently with each other or with eager calls on another
// stream (nifty_amd.h, nft_amp2_jvp).
static std::mutex g_guard_mu;
static hipStream_t g_last_stream = nullptr;
static bool g_any_call = false;
static bool capturing(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(s, &st) == hipSuccess && st != hipStreamCaptureStatusNone;
}
// caller holds g_guard_mu
static int guard_enter(hipStream_t s) {
  if (capturing(s)) return NFT_OK;
  if (g_any_call && s != g_last_stream) {
    if (hipStreamSynchronize(g_last_stream) != hipSuccess) {
      (void)hipGetLastError();
      NFT_HIP_CHECK(hipDeviceSynchronize());
    }
  }
  g_last_stream = s;
  g_any_call = true;
  return NFT_OK;
}

// NFT_AMP2=0: off (the multi-kernel path); nft_amp2_set_enabled overrides
// the environment (tests, A/B)
static int g_override = -1;
static bool enabled() {
  static const int on = getenv("NFT_AMP2") ? atoi(getenv("NFT_AMP2")) : 1;
  return g_override >= 0 ? g_override != 0 : on != 0;
}

// tile count (1024-bin tiles, the same for every batch size), 0: not
// applicable (NFT_AMP2=0, B < 3, too many RHS, or the workspace too small)
static int tiles_of(long long B, int nrhs) {
  if (!enabled() || B < 3 || nrhs < 1 || nrhs > MAXR) return 0;
  const long long wsd = (long long)(nft_amp_workspace(B) / sizeof(double));
  const long long nb = nblk(B - 2, TL);
  if ((V_NROWS + 2) * nb + 8 > wsd || ((B + 63) & ~63LL) + 9 * nb + 10 > wsd) return 0;
  return (int)nb;
}

}  // namespace amp2
}  // namespace nft

using namespace nft;
using namespace nft::amp2;

extern "C" {

int nft_amp2_enabled(void) { return enabled() ? 1 : 0; }

void nft_amp2_set_enabled(int on) { g_override = on < 0 ? -1 : (on != 0); }

int nft_amp2_tiles(int64_t B, int nrhs, int item_mode) {
  (void)item_mode;
  return tiles_of(B, nrhs);
}

int64_t nft_amp2_tab_size(int64_t B) {
  if (B < 3) return 0;
  return (int64_t)tab_size(B, nblk(B - 2, TL));
}

int nft_amp2_prepare(const nft_amp_const* c, const nft_amp_const* item_consts, int item_mode, double* tab,
                     hipStream_t stream) {
  if (!c || !tab || c->B < 3 || (item_mode != 0 && item_mode != 2) || (item_mode == 2 && !item_consts)) {
    set_last_error("nft_amp2_prepare: invalid arguments (item_mode 0 or 2)");
    return NFT_ERR_ARG;
  }
  const int nb = nblk(c->B - 2, TL);
  prof_mark(stream, "amp_prep");
  if (item_mode == 2) hipLaunchKernelGGL((prep_kernel<2>), dim3(nb), dim3(NT), 0, stream, *c, item_consts, nb, tab);
  else hipLaunchKernelGGL((prep_kernel<0>), dim3(nb), dim3(NT), 0, stream, *c, nullptr, nb, tab);
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

}  // extern "C"

namespace {
// TB (a constant-scan table) with modes 0 and 2 only
#define NFT_AMP2_LAUNCH(KERN, VT, MODE, TB, GRID, S, ARGS)                                     \
  do {                                                                                         \
    if ((MODE) == 1) hipLaunchKernelGGL((KERN<VT, 1, false>), GRID, dim3(NT), 0, S, ARGS);     \
    else if ((MODE) == 2 && (TB)) hipLaunchKernelGGL((KERN<VT, 2, true>), GRID, dim3(NT), 0, S, ARGS); \
    else if ((MODE) == 2) hipLaunchKernelGGL((KERN<VT, 2, false>), GRID, dim3(NT), 0, S, ARGS); \
    else if (TB) hipLaunchKernelGGL((KERN<VT, 0, true>), GRID, dim3(NT), 0, S, ARGS);          \
    else hipLaunchKernelGGL((KERN<VT, 0, false>), GRID, dim3(NT), 0, S, ARGS);                 \
  } while (0)

template <typename VT>
int amp2_jvp_impl(const nft_amp_const* cst_, const nft_amp_const* item_consts, int item_mode, void* const* t,
                  const void* const* r, int64_t lat_stride, void* da, int64_t da_stride, int64_t da_elem_stride,
                  double* ws, int nrhs, const double* sc, double* part, int64_t pstride, double shift, int nb,
                  const double* tab, hipStream_t stream) {
  Jvp2Args<VT> a{};
  a.c = *cst_;
  a.dcs = item_mode == 1 ? item_consts : nullptr;
  a.dc1 = item_mode == 2 ? item_consts : nullptr;
  for (int q = 0; q < 6; ++q) {
    a.t[q] = (VT*)t[q];
    a.r[q] = r ? (const VT*)r[q] : nullptr;
  }
  a.ls = lat_stride;
  a.da = (VT*)da;
  a.vs = da_stride;
  a.des = da_elem_stride > 0 ? da_elem_stride : 1;
  a.ws = ws;
  a.wsd = (long long)(nft_amp_workspace(cst_->B) / sizeof(double));
  a.nrhs = nrhs;
  a.nb = nb;
  a.dir = r != nullptr;
  a.sc = sc;
  a.part = part;
  a.pstride = pstride;
  a.shift = shift;
  a.tab = tab;
  const bool tb = tab != nullptr;
  const dim3 grid(grid_of(nb, nrhs));
  std::lock_guard<std::mutex> lk(g_guard_mu);
  if (int st = guard_enter(stream)) return st;
  prof_mark(stream, a.dir ? "amp_jvp2a+dir" : "amp_jvp2a");
  NFT_AMP2_LAUNCH(jvp2a_kernel, VT, item_mode, tb, grid, stream, a);
  prof_mark(stream, "amp_jvp2b");
  NFT_AMP2_LAUNCH(jvp2b_kernel, VT, item_mode, tb, grid, stream, a);
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

template <typename VT>
int amp2_vjp_impl(const nft_amp_const* cst_, const nft_amp_const* item_consts, int item_mode, const void* g,
                  int64_t g_stride, void* const* out, void* const* out2, const void* const* d, int64_t lat_stride,
                  double shift, double* ws, int nrhs, double* sc, double* part, int64_t pstride, const double* gpart,
                  int64_t gp_stride, int64_t gp_row, int ngp, int nb, const double* tab, hipStream_t stream) {
  Vjp2Args<VT> a{};
  a.c = *cst_;
  a.dcs = item_mode == 1 ? item_consts : nullptr;
  a.dc1 = item_mode == 2 ? item_consts : nullptr;
  a.g = (const VT*)g;
  a.gs = g_stride;
  for (int q = 0; q < 6; ++q) {
    a.o[q] = (VT*)out[q];
    a.o2[q] = out2 ? (VT*)out2[q] : nullptr;
    a.d[q] = d ? (const VT*)d[q] : nullptr;
  }
  a.ls = lat_stride;
  a.shift = shift;
  a.ws = ws;
  a.wsd = (long long)(nft_amp_workspace(cst_->B) / sizeof(double));
  a.nrhs = nrhs;
  a.nb = nb;
  a.cg = out2 != nullptr;
  a.sc = sc;
  a.part = part;
  a.pstride = pstride;
  a.gpart = gpart;
  a.gps = gp_stride;
  a.gpr = gp_row;
  a.ngp = a.cg ? ngp : 0;
  a.tab = tab;
  const bool tb = tab != nullptr;
  const dim3 grid(grid_of(nb, nrhs));
  std::lock_guard<std::mutex> lk(g_guard_mu);
  if (int st = guard_enter(stream)) return st;
  prof_mark(stream, a.cg ? "amp_vjp2a+cg" : "amp_vjp2a");
  NFT_AMP2_LAUNCH(vjp2a_kernel, VT, item_mode, tb, grid, stream, a);
  prof_mark(stream, a.cg ? "amp_vjp2b+cg" : "amp_vjp2b");
  NFT_AMP2_LAUNCH(vjp2b_kernel, VT, item_mode, tb, grid, stream, a);
  if (a.cg) {
    prof_mark(stream, "amp_fin");
    hipLaunchKernelGGL((fin_kernel<VT>), dim3((unsigned)nrhs), dim3(NT), 0, stream, a);
  }
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}
}  // namespace

extern "C" {

int nft_amp2_jvp(const nft_amp_const* cst_, const nft_amp_const* item_consts, int item_mode, void* const* t,
                 const void* const* r, int64_t lat_stride, void* da, int64_t da_stride, int64_t da_elem_stride,
                 double* ws, int nrhs, const double* sc, double* part, int64_t pstride, double shift, int dtype,
                 const double* tab, hipStream_t stream) {
  if (!cst_ || !t || !da || !ws || nrhs < 1 || cst_->B < 3 || (cst_->has_flex && !t[KSPEC]) ||
      (r && (!sc || !part)) || (dtype != 0 && dtype != 1) || (tab && item_mode == 1)) {
    set_last_error("nft_amp2_jvp: invalid arguments");
    return NFT_ERR_ARG;
  }
  if (item_mode < 0 || item_mode > 2 || (item_mode != 0 && !item_consts)) {
    set_last_error("nft_amp2_jvp: invalid item_mode / item_consts");
    return NFT_ERR_ARG;
  }
  for (int q = 0; q < 6; ++q)
    if (r && t[q] && !r[q]) {
      set_last_error("nft_amp2_jvp: a direction key without its residual");
      return NFT_ERR_ARG;
    }
  const int nb = tiles_of(cst_->B, nrhs);
  if (!nb) return NFT_AMP2_FALLBACK;
  if (dtype == 1)
    return amp2_jvp_impl<float>(cst_, item_consts, item_mode, t, r, lat_stride, da, da_stride, da_elem_stride, ws,
                                nrhs, sc, part, pstride, shift, nb, tab, stream);
  return amp2_jvp_impl<double>(cst_, item_consts, item_mode, t, r, lat_stride, da, da_stride, da_elem_stride, ws,
                               nrhs, sc, part, pstride, shift, nb, tab, stream);
}

int nft_amp2_vjp(const nft_amp_const* cst_, const nft_amp_const* item_consts, int item_mode, const void* g,
                 int64_t g_stride, void* const* out, void* const* out2, const void* const* d, int64_t lat_stride,
                 double shift, double* ws, int nrhs, double* sc, double* part, int64_t pstride, const double* gpart,
                 int64_t gp_stride, int64_t gp_row, int ngp, int dtype, const double* tab, hipStream_t stream) {
  if (!cst_ || !g || !out || !ws || nrhs < 1 || cst_->B < 3 || (cst_->has_flex && !out[KSPEC]) ||
      (out2 && (!d || !sc || !part || (ngp > 0 && !gpart))) || (dtype != 0 && dtype != 1) ||
      (tab && item_mode == 1)) {
    set_last_error("nft_amp2_vjp: invalid arguments");
    return NFT_ERR_ARG;
  }
  if (item_mode < 0 || item_mode > 2 || (item_mode != 0 && !item_consts)) {
    set_last_error("nft_amp2_vjp: invalid item_mode / item_consts");
    return NFT_ERR_ARG;
  }
  for (int q = 0; q < 6; ++q)
    if (out2 && out[q] && (!out2[q] || !d[q])) {
      set_last_error("nft_amp2_vjp: a CG key without its residual / direction");
      return NFT_ERR_ARG;
    }
  const int nb = tiles_of(cst_->B, nrhs);
  if (!nb) return NFT_AMP2_FALLBACK;
  if (dtype == 1)
    return amp2_vjp_impl<float>(cst_, item_consts, item_mode, g, g_stride, out, out2, d, lat_stride, shift, ws, nrhs,
                                sc, part, pstride, gpart, gp_stride, gp_row, ngp, nb, tab, stream);
  return amp2_vjp_impl<double>(cst_, item_consts, item_mode, g, g_stride, out, out2, d, lat_stride, shift, ws, nrhs,
                               sc, part, pstride, gpart, gp_stride, gp_row, ngp, nb, tab, stream);
}

}  // extern "C"
