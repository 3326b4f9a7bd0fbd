// R2C row pass with the batched correlated-field prologue (engine v2).
//
// The CF Jacobian's forward transform starts from
//   u_b[j] = A[j] * x_b[j] + xi0[j] * dA_b[pindex[j]]      (item b, pixel j)
// where A, xi0 and pindex are shared by all right-hand sides b.  One
// workgroup takes one PAIR of real rows (2 rho, 2 rho + 1) of L items at once:
// it reads the shared operands of those two rows once, forms u for all L
// items (the dA gathers of a pixel are one contiguous run of the bin-major
// interleaved dA), and transforms L complex lines u_b[2 rho] + i u_b[2 rho+1]
// -- exactly the row pairing of the plain R2C pass, so every item's
// half spectrum is bit for bit what the split path (pro_batch + R2C)
// produces, whatever L and the number of items are.  This replaces a
// separate prologue pass that wrote u to HBM and an R2C pass that read it
// back (the fused form of MI355X_MICROARCH "keep tensors resident").
#pragma once
#include "fast_passes.hpp"

namespace nft {
namespace fast {

template <int N, int L>
constexpr size_t pro_pairs_lds() {
  return (size_t)L * N * 16 + (size_t)(N / 4) * 16;
}

// grid: (row pairs, item groups); out: half spectra, item stride ostride
// and row pitch opitch (complex elements; the workspace pads rows to a
// multiple of 8); item b = blockIdx.y * L + l.
template <typename T, int N, int L>
__global__ __launch_bounds__(L* N / VPT) void r2c_pro_pairs(FuseArgs f, cplx_t<T>* __restrict__ out,
                                                            const cplx_t<T>* __restrict__ tw, long long nrows,
                                                            long long ostride, long long opitch) {
  using C = cplx_t<T>;
  constexpr int NT = L * N / VPT;
  constexpr int PX = VPT / L;  // pixels of each row per thread (x = tid + NT*m)
  constexpr int NH = N / 2 + 1;
  static_assert(VPT % L == 0, "L must divide VPT");
  extern __shared__ __align__(16) unsigned char smem[];
  C* lds = (C*)smem;
  C* twq = (C*)(smem + (size_t)L * N * sizeof(C));
  const int tid = threadIdx.x;
  for (int r = tid; r < N / 4; r += NT) twq[r] = tw[r];
  const long long row0 = 2 * (long long)blockIdx.x;  // real rows row0, row0 + 1 of every item
  const int b0 = blockIdx.y * L;
  const T* __restrict__ px = (const T*)f.px;
  const T* __restrict__ pa = (const T*)f.pa;
  const T* __restrict__ pb = (const T*)f.pb;
  const T* __restrict__ pc = (const T*)f.pc;
  const bool has1 = row0 + 1 < nrows;
  // every load of the tile is issued before the first use (the x values and
  // the dA gathers of all L items), so one workgroup keeps ~40 loads per
  // thread in flight instead of one dependent chain per item
  T a[2][PX], c[2][PX];
  long long g[2][PX];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int m = 0; m < PX; ++m) {
      const long long j = (row0 + h) * N + tid + NT * m;
      const bool ok = h == 0 || has1;
      a[h][m] = (pa && ok) ? pa[j] : (T)1;
      c[h][m] = (pb && ok) ? pb[j] : (T)0;
      g[h][m] = (pb && ok) ? pro_cidx(f, j) : 0;
    }
  T xv[L][2][PX], cv[L][2][PX];
#pragma unroll
  for (int l = 0; l < L; ++l)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int m = 0; m < PX; ++m) {
        const long long b = b0 + l;
        const long long j = (row0 + h) * N + tid + NT * m;
        const bool ok = h == 0 || has1;
        xv[l][h][m] = ok ? px[b * f.sx + j] : (T)0;
        cv[l][h][m] = (pb && ok) ? pc[b * f.sc + g[h][m]] : (T)0;
      }
#pragma unroll
  for (int l = 0; l < L; ++l)
#pragma unroll
    for (int m = 0; m < PX; ++m) {
      T v[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        T x = xv[l][h][m];
        if (pa) x *= a[h][m];
        if (pb) x += c[h][m] * cv[l][h][m];
        v[h] = x;
      }
      lds[l * N + tid + NT * m] = C{v[0], v[1]};
    }
  __syncthreads();
  fft<T, N, NT, L, N>(lds, twq, tid);
  const T hh = (T)0.5;
  for (int e = tid; e < L * NH; e += NT) {
    const int l = e / NH;
    const int k = e - l * NH;
    const C zk = lds[l * N + k];
    const C zm = lds[l * N + ((N - k) & (N - 1))];
    const C xa = C{hh * (zk.x + zm.x), hh * (zk.y - zm.y)};
    const C xb = C{hh * (zk.y + zm.y), -hh * (zk.x - zm.x)};
    C* o = out + (b0 + l) * ostride + row0 * opitch + k;
    o[0] = xa;
    if (has1) o[opitch] = xb;
  }
}

// launcher: N = row length (power of two 256..4096), nb items, P pixels per
// item (nrows = P / N rows each); the prologue operands shared by all items.
template <typename T, int N, int L>
static int launch_pro_pairs_nl(const FuseArgs& f, void* out, long long nrows, int nb, long long ostride,
                               long long opitch, hipStream_t s) {
  constexpr int NT = L * N / VPT;
  constexpr size_t lds = pro_pairs_lds<N, L>() / (sizeof(T) == 8 ? 1 : 2);
  static_assert(NT <= 1024, "workgroup too large");
  const void* tw = nullptr;
  int st = get_twiddles(N, sizeof(T) == 8 ? 0 : 1, &tw);
  if (st != NFT_OK) return st;
  if (lds > 65536) {
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)r2c_pro_pairs<T, N, L>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds);
      attr = true;
    }
  }
  prof_mark(s, "fft_r2c+pro");
  hipLaunchKernelGGL((r2c_pro_pairs<T, N, L>), dim3((unsigned)((nrows + 1) / 2), (unsigned)(nb / L)), dim3(NT), lds, s,
                     f, (cplx_t<T>*)out, (const cplx_t<T>*)tw, nrows, ostride, opitch);
  NFT_HIP_CHECK(hipGetLastError());
  return NFT_OK;
}

// items per workgroup: the largest of 4, 3, 2, 1 dividing nb with the
// workgroup within 1024 threads
inline int pro_pairs_group(int N, int nb) {
  static const int lmax = getenv("NFT_PRO_PAIRS_L") ? atoi(getenv("NFT_PRO_PAIRS_L")) : 4;
  for (int L = lmax; L >= 1; --L)
    if (nb % L == 0 && L * N / VPT <= 1024 && VPT % L == 0) return L;
  return 0;
}

template <typename T, int N>
static int launch_pro_pairs_n(const FuseArgs& f, void* out, long long nrows, int nb, long long ostride,
                              long long opitch, hipStream_t s) {
  switch (pro_pairs_group(N, nb)) {
    case 4:
      if constexpr (4 * N / VPT <= 1024) return launch_pro_pairs_nl<T, N, 4>(f, out, nrows, nb, ostride, opitch, s);
      break;
    case 2:
      if constexpr (2 * N / VPT <= 1024) return launch_pro_pairs_nl<T, N, 2>(f, out, nrows, nb, ostride, opitch, s);
      break;
    case 1:
      return launch_pro_pairs_nl<T, N, 1>(f, out, nrows, nb, ostride, opitch, s);
  }
  return 1;  // not handled
}

template <typename T>
static int launch_pro_pairs(int N, const FuseArgs& f, void* out, long long nrows, int nb, long long ostride,
                            long long opitch, hipStream_t s) {
  switch (N) {
    case 256: return launch_pro_pairs_n<T, 256>(f, out, nrows, nb, ostride, opitch, s);
    case 512: return launch_pro_pairs_n<T, 512>(f, out, nrows, nb, ostride, opitch, s);
    case 1024: return launch_pro_pairs_n<T, 1024>(f, out, nrows, nb, ostride, opitch, s);
    case 2048: return launch_pro_pairs_n<T, 2048>(f, out, nrows, nb, ostride, opitch, s);
    case 4096: return launch_pro_pairs_n<T, 4096>(f, out, nrows, nb, ostride, opitch, s);
  }
  return 1;
}

}  // namespace fast
}  // namespace nft
