// Row-staged prologue carrying the CG direction, fused with the R2C row pass
// of the forward transform (nft_hartley_fused with dir_* set, 2-D grids,
// A / xi0 shared by the items).
//
// The forward transform of the CF Jacobian (reference: the chain
// HarmonicTransformOperator o PowerDistributor o amplitude of
// src/library/correlated_fields_simple.py:86-127, applied inside the sampling
// metric of src/operators/sandwich_operator.py:41-95) starts with
// u = A * d + xi0 * dA[bin]; the carried CG iteration forms the direction
// d = beta d + r in the same pass.  Split, that is pro_rows_kernel (which
// writes u) and the persistent R2C pass (which reads it back).  Here one
// workgroup per (mirror row group, item) forms the group's two rows g and
// n0 - g (for group 0 the two self-mirror rows 0 and n0 / 2) exactly as
// pro_rows_kernel forms them (d written back, u = A d + xi0 dA[cell]: bitwise
// the same u and d), packs them as the real and imaginary parts of ONE
// complex line and runs the R2C pass's FFT and half-spectrum split on it
// (fast::fft, store_r2c's arithmetic): u never goes to memory, 2 x 8 B per
// pixel and item less traffic.  The R2C pass pairs rows 2l, 2l + 1 instead,
// so the half spectra differ from the split path in the last bits (an FFT
// mixes the rounding of its two packed rows); per item the result does not
// depend on the batch (single == batched, compaction bitwise).
// d.d partials: thread t sums positions t, t + NT, ... of row g, then those
// of row n0 - g (pro_rows_kernel's order at NT = 256), the waves folded in
// order, one slot per mirror row group (nft_hartley_dir_blocks).
#include <cstdlib>

#include "fast_dispatch.hpp"
#include "nft_api_internal.hpp"

namespace nft {

template <typename T, int N>
__global__ __launch_bounds__(N / 8) void pro_r2c_kernel(fast::FuseArgs f, const cplx_t<T>* __restrict__ tw,
                                                        cplx_t<T>* __restrict__ hs, int n0) {
  using C = cplx_t<T>;
  // HS: row stride of the half-spectrum workspace (nft_fft.hip half_shape:
  // N / 2 + 1 rounded up to a multiple of 8)
  constexpr int NT = N / 8, NW = NT / 64, VP = 8, HV = VP / 2, HL = N / 2 + 1, HS = (HL + 7) / 8 * 8;
  extern __shared__ __align__(16) unsigned char prc_smem[];
  C* line = (C*)prc_smem;
  C* twq = line + N;
  __shared__ double dsh[2][NW];
  const int tid = threadIdx.x;
  // workgroup -> (group gi, item b): the items of one group on consecutive
  // slots of one XCD, so the shared A / xi0 rows are read from its L2
  const int nb = f.nb, ngr = n0 / 2;
  const int w = blockIdx.x, xg = w & 7, slot = w >> 3;
  const int rl = slot / nb, b = slot - rl * nb;
  const int gi = rl * 8 + xg;
  if (gi >= ngr) return;
  for (int q = tid; q < N / 4; q += NT) twq[q] = tw[q];
  const int rowA = gi, rowB = gi == 0 ? ngr : n0 - gi;
  const int crB = gi == 0 ? ngr : gi;  // cell row of row B (row A: gi)
  const T* __restrict__ px = (const T*)f.px;
  const T* __restrict__ pa = (const T*)f.pa;
  const T* __restrict__ pb = (const T*)f.pb;
  const T* __restrict__ pc = (const T*)f.pc;
  const T* __restrict__ pr = (const T*)f.dr;
  const int* __restrict__ pidx = f.pidx;
  T* pd = const_cast<T*>(px);
  const double* scb = f.dsc + b * NFT_CG_NSCALARS;
  const bool live = scb[NFT_CG_DONE] == 0.0;
  double beta = scb[NFT_CG_GAMMA] / scb[NFT_CG_GPREV];
  if (!(beta > 0.0)) beta = 0.0;
  const T bt = (T)beta;
  const long long jA = (long long)rowA * N, jB = (long long)rowB * N;
  const long long ib = (long long)b * f.sx, ic = (long long)b * f.sc;
  // deferred iterate (nft_hartley_fuse.lazy_*): the previous direction from
  // ring slot s (0: px), the new one (a stopped item's copied) into slot s + 1
  const T* pxs = px;
  T* pds = pd;
  if (f.lazy) {
    // (clamped: a counter out of range never addresses outside the ring)
    const long long sl = min(max((long long)scb[NFT_CG_LAZY], 0LL), f.lnslot - 1);
    pxs = sl == 0 ? px : (const T*)f.lring + (sl - 1) * f.lss;
    pds = (T*)f.lring + sl * f.lss;
  }
  double dA = 0.0;
  T vbk[VP];  // d of row B, summed after every position of row A
  // two halves of the thread's positions, each with every load of both rows
  // issued before the first store (d is stored back into the array x is read
  // from); the halves keep the live registers below 128
#pragma unroll 1
  for (int h = 0; h < 2; ++h) {
    T xa[HV], xb[HV], ra[HV], rb[HV], aa[HV], ab[HV], ba[HV], bb[HV], ca[HV], cb[HV];
#pragma unroll
    for (int i = 0; i < HV; ++i) {
      const int p = tid + (h * HV + i) * NT;
      const int c1 = p == 0 ? 0 : (p <= N - p ? p : N - p);
      xa[i] = pxs[ib + jA + p];
      xb[i] = pxs[ib + jB + p];
      ra[i] = rb[i] = (T)0;
      if (live) {
        ra[i] = pr[ib + jA + p];
        rb[i] = pr[ib + jB + p];
      }
      aa[i] = ab[i] = (T)1;
      if (pa) {
        aa[i] = pa[jA + p];
        ab[i] = pa[jB + p];
      }
      ba[i] = pb[jA + p];
      bb[i] = pb[jB + p];
      ca[i] = pc[ic + (long long)pidx[gi * HL + c1] * f.ce];
      cb[i] = pc[ic + (long long)pidx[crB * HL + c1] * f.ce];
    }
#pragma unroll
    for (int i = 0; i < HV; ++i) {
      const int p = tid + (h * HV + i) * NT;
      T va = xa[i], vb = xb[i];
      if (live) {
        va = bt * va + ra[i];
        vb = bt * vb + rb[i];
        pds[ib + jA + p] = va;
        pds[ib + jB + p] = vb;
        dA += (double)va * (double)va;
      } else if (f.lazy) {
        pds[ib + jA + p] = va;
        pds[ib + jB + p] = vb;
      }
      vbk[h * HV + i] = vb;
      if (pa) {
        va *= aa[i];
        vb *= ab[i];
      }
      va += ba[i] * ca[i];
      vb += bb[i] * cb[i];
      line[p] = C{va, vb};
    }
  }
  double dB = 0.0;
  if (live) {
    if (gi == 0) {  // two groups of one row each
#pragma unroll
      for (int i = 0; i < VP; ++i) dB += (double)vbk[i] * (double)vbk[i];
    } else {
#pragma unroll
      for (int i = 0; i < VP; ++i) dA += (double)vbk[i] * (double)vbk[i];
    }
  }
  __syncthreads();
  fast::fft<T, N, NT, 1, N, -1>(line, twq, tid);
  // half-spectrum split (store_r2c's arithmetic, scale 1): row A from the
  // real part, row B from the imaginary part
  {
    const T hh = (T)0.5;
    C* oA = hs + ((long long)b * n0 + rowA) * HS;
    C* oB = hs + ((long long)b * n0 + rowB) * HS;
    for (int k = tid; k < HL; k += NT) {
      const C zk = line[k];
      const C zm = line[(N - k) & (N - 1)];
      oA[k] = C{hh * (zk.x + zm.x), hh * (zk.y - zm.y)};
      oB[k] = C{hh * (zk.y + zm.y), -hh * (zk.x - zm.x)};
    }
  }
  // d.d partials of the group(s): wave trees, then the waves in order
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    dA += __shfl_down(dA, off, 64);
    dB += __shfl_down(dB, off, 64);
  }
  if ((tid & 63) == 0) {
    dsh[0][tid >> 6] = dA;
    dsh[1][tid >> 6] = dB;
  }
  __syncthreads();
  if (tid < (gi == 0 ? 2 : 1)) {
    double t = dsh[tid][0];
#pragma unroll
    for (int q = 1; q < NW; ++q) t += dsh[tid][q];
    const int grp = tid == 0 ? gi : ngr;
    f.dpart[b * f.dps + f.dblk0 + grp] = live ? f.dshift * t : 0.0;
  }
}

// Measured against the split passes (pro_rows_kernel + the persistent R2C
// pass; tools/ab_pror2c.sh, 4 RHS, same box): 1024^2 fp64 (C2) 53.5 -> 37.6 us,
// CG iteration 276.5 -> 243.3 us; 2048^2 fp64 (C3) 191 -> 195 us; 4096^2 fp32
// (C5) 426 -> 502 us.  The fused pass moves 2/3 of the bytes but runs each
// workgroup's load, FFT and store phases back to back (the persistent R2C
// prefetches the next tile during the FFT; here five operand streams per
// position would need five times its prefetch registers) and re-reads the
// shared A / xi0 rows once per item (PMC 1.25x / 1.55x of its bytes at C3 /
// C5).  Also measured and removed: one workgroup per row group looping over
// every item with A / xi0 and the next item's operands in registers (C3 223 /
// 361 us at 4 / 2 positions per thread: 196 VGPRs, or spills), and item pairs
// transformed as two lines of one workgroup (A / xi0 read once per pair: C3
// 189 us, C5 606 us, C2 40 us).  So the fused pass runs for rows up to 1024.
//
// NFT_PRO_R2C: 0 off, 2 on for every supported row length (tests), default
// (1): rows of at most 1024.  Read at every call (a graph keeps the choice
// made at its capture).
static int pro_r2c_mode() {
  const char* e = getenv("NFT_PRO_R2C");
  if (e && (e[0] == '0' || e[0] == '2')) return e[0] - '0';
  return 1;
}

template <typename T, int N>
static int launch_pro_r2c_n(const fast::FuseArgs& f, void* ws, int n0, hipStream_t s) {
  const void* tw = nullptr;
  int st = get_twiddles(N, sizeof(T) == 8 ? 0 : 1, &tw);
  if (st != NFT_OK) return st;
  const size_t lds = (size_t)(N + N / 4) * sizeof(cplx_t<T>);
  if (lds > 65536) {
    static bool set = false;
    if (!set) {
      NFT_HIP_CHECK(hipFuncSetAttribute((const void*)pro_r2c_kernel<T, N>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      set = true;
    }
  }
  prof_mark(s, "pro_r2c+dir");
  hipLaunchKernelGGL((pro_r2c_kernel<T, N>), dim3((unsigned)((n0 / 2) * f.nb)), dim3(N / 8), lds, s, f,
                     (const cplx_t<T>*)tw, (cplx_t<T>*)ws, n0);
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

template <typename T>
static int launch_pro_r2c(const fast::FuseArgs& f, long long n1, void* ws, int n0, hipStream_t s, int mode,
                          bool* done) {
  if (mode == 1 && n1 > 1024) return NFT_OK;
  int st;
  switch (n1) {
    case 512: st = launch_pro_r2c_n<T, 512>(f, ws, n0, s); break;
    case 1024: st = launch_pro_r2c_n<T, 1024>(f, ws, n0, s); break;
    case 2048: st = launch_pro_r2c_n<T, 2048>(f, ws, n0, s); break;
    case 4096: st = launch_pro_r2c_n<T, 4096>(f, ws, n0, s); break;
    default: return NFT_OK;
  }
  if (st == NFT_OK) *done = true;
  return st;
}

// The geometry the fused pass covers: a batch (nb, n0, n1) transformed over
// both grid axes, n1 in {512 ... 4096}, n0 / 2 a multiple of 8, the direction
// carried and A / xi0 shared by the items.  Otherwise *done stays false and
// the caller runs the split passes.
int pro_r2c_try(const fast::FuseArgs& f, int dtype, int nd, const long long* shape, int naxes, const int* ax,
                void* ws, size_t hws, hipStream_t s, bool* done) {
  *done = false;
  const int mode = pro_r2c_mode();
  if (mode == 0 || !f.dr || f.fnd != 2 || f.sa != 0 || f.sb != 0 || !f.pb || !f.pidx || f.nb < 1)
    return NFT_OK;
  if (nd != 3 || naxes != 2 || ax[0] != 1 || ax[1] != 2 || shape[0] != f.nb) return NFT_OK;
  const long long n0 = shape[1], n1 = shape[2];
  if (f.fn[0] != n0 || f.fn[1] != n1 || f.P != n0 * n1 || f.sx < f.P) return NFT_OK;
  if (n0 < 16 || (n0 / 2) % 8 != 0) return NFT_OK;
  const size_t es = dtype == 0 ? sizeof(double2) : sizeof(float2);
  if (hws < (size_t)(f.nb * n0 * ((n1 / 2 + 1 + 7) / 8 * 8)) * es) return NFT_OK;
  if (dtype == 0) return launch_pro_r2c<double>(f, n1, ws, (int)n0, s, mode, done);
  if (dtype == 1) return launch_pro_r2c<float>(f, n1, ws, (int)n0, s, mode, done);
  return NFT_OK;
}

}  // namespace nft
