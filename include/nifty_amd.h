/* nifty_amd — C ABI of the MI355X (gfx950) geoVI/MGVI sampling hot path.
 *
 * Every entry point takes plain device pointers, sizes and a hipStream_t,
 * launches asynchronously on that stream, never synchronises the device and
 * never allocates device memory except the per-length twiddle tables it caches
 * (released by nft_release_caches).  Return value: 0 on success, a negative
 * NFT_ERR_* code on failure; nft_last_error() then describes the failure
 * (thread-local).  Caller owns every buffer (workspace sizes are queried with
 * the *_workspace functions).
 *
 * dtype codes: 0 = float64 (complex128 for complex buffers), 1 = float32
 * (complex64).  Hartley convention: 0 = non-canonical (Re F + Im F, the
 * reference default), 1 = canonical (Re F - Im F)  (src/config.py:3-40).
 *
 * Reference seams replaced (paths relative to the NIFTy 8.5 tree):
 *   nft_hartley        src/ducc_dispatch.py:46-50 (_scipy_hartley), :75-78 (ducc0
 *                      genuine_hartley / genuine_fht) as called from
 *                      HartleyOperator._apply_cartesian, src/operators/harmonic_operators.py:208-217
 *   nft_fft_c2c        src/ducc_dispatch.py:38-43, :66-72 (fftn / ifftn) as called
 *                      from FFTOperator.apply, harmonic_operators.py:106-123
 *   nft_dot            src/ducc_dispatch.py:53-58, :81-86 (vdot), via Field.s_vdot
 *                      src/field.py:296-347
 *   nft_cg_*           ConjugateGradient.__call__ vector algebra,
 *                      src/minimization/conjugate_gradient.py:78-126 and
 *                      QuadraticEnergy, src/minimization/quadratic_energy.py:31-39
 *   nft_bin_gather     DOFDistributor._times, src/operators/distributors.py:114-119
 *   nft_bin_scatter    DOFDistributor._adjoint_times + utilities.special_add_at,
 *                      distributors.py:105-112, src/utilities.py:223-242
 *   nft_cf_*           the correlated-field Jacobian / sampling-metric matvec built
 *                      from HarmonicTransformOperator o (PowerDistributor(A) * xi)
 *                      (src/library/correlated_fields_simple.py:155-160) sandwiched as
 *                      in src/minimization/kl_energies.py:115-123
 *   nft_spmv_*         LOSResponse.apply (scipy COO matvec / rmatvec),
 *                      src/library/los_response.py:226-233
 */
#ifndef NIFTY_AMD_H
#define NIFTY_AMD_H

#include <stddef.h>
#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NFT_OK 0
#define NFT_ERR_ARG (-1)
#define NFT_ERR_UNSUPPORTED (-2)
#define NFT_ERR_HIP (-3)
#define NFT_ERR_ALLOC (-4)

/* device-resident CG scalar block (double[NFT_CG_NSCALARS]) */
#define NFT_CG_GAMMA 0 /* r.r of the current residual (previous_gamma for the next step) */
#define NFT_CG_GPREV 1 /* gamma of the step before */
#define NFT_CG_CURV 2  /* d.q */
#define NFT_CG_ALPHA 3
#define NFT_CG_XR 4 /* x.r */
#define NFT_CG_XB 5 /* x.b */
#define NFT_CG_FLAG 6 /* 1.0: curvature/alpha guard tripped, x and r left unchanged */
#define NFT_CG_DD 7   /* d.d (fused sampling metric) */
#define NFT_CG_NSCALARS 16

const char* nft_last_error(void);
void nft_release_caches(void);

/* ---- transforms ------------------------------------------------------ */
int nft_fft_prepare(int n, int dtype);
int nft_hartley_workspace(int ndim, const int64_t* shape, int naxes, const int* axes, int dtype,
                          size_t* bytes);
/* out = scale * H_axes(in), real -> real, C-contiguous; in == out allowed. */
int nft_hartley(const void* in, void* out, int ndim, const int64_t* shape, int naxes,
                const int* axes, int dtype, int convention, double scale, void* workspace,
                size_t ws_bytes, hipStream_t stream);
/* complex -> complex, forward (e^-i) or backward (e^+i, unnormalised) times scale */
int nft_fft_c2c(const void* in, void* out, int ndim, const int64_t* shape, int naxes,
                const int* axes, int dtype, int forward, double scale, hipStream_t stream);

/* ---- reductions / CG primitives -------------------------------------- */
size_t nft_reduce_workspace(int64_t n);
/* *out (device) = sum a[i]*b[i], fp64 accumulation, deterministic */
int nft_dot(const void* a, const void* b, int64_t n, int dtype, double* out, void* ws,
            hipStream_t stream);
int nft_scale(void* x, int64_t n, int dtype, double scale, hipStream_t stream);
/* alpha = sc[GAMMA]/sc[CURV]; x -= alpha d; r -= alpha q; sc[GAMMA,XR,XB] <- r.r, x.r, x.b */
int nft_cg_update(void* x, void* r, const void* d, const void* q, const void* b, int64_t n,
                  int dtype, double* sc, void* ws, hipStream_t stream);
/* d = max(0, sc[GAMMA]/sc[GPREV]) d + r */
int nft_cg_direction(void* d, const void* r, int64_t n, int dtype, const double* sc,
                     hipStream_t stream);
/* r = ax - b; sc[GPREV] <- sc[GAMMA]; sc[GAMMA,XR,XB] <- r.r, x.r, x.b */
int nft_cg_residual(void* r, const void* ax, const void* x, const void* b, int64_t n, int dtype,
                    double* sc, void* ws, hipStream_t stream);

/* ---- power-bin distributor -------------------------------------------- */
/* out[p,i,q] = in[p, pindex[i], q]; in: [pre, nbins, post], out: [pre, npix, post] */
int nft_bin_gather(const void* in, const int* pindex, void* out, int64_t pre, int64_t npix,
                   int64_t nbins, int64_t post, int dtype, hipStream_t stream);
/* out[p,b,q] = sum_{j in [offsets[b], offsets[b+1])} in[p, perm[j], q], summed in
 * ascending j (perm = stable argsort of pindex: np.bincount order, bit-exact) */
int nft_bin_scatter(const void* in, const int* perm, const int* offsets, void* out, int64_t pre,
                    int64_t npix, int64_t nbins, int64_t post, int dtype, hipStream_t stream);

/* ---- sparse LOS response --------------------------------------------- */
/* y[r] = scale * sum_j weights[j] * x[indices[j]], j in [indptr[r], indptr[r+1]) */
int nft_spmv_csr(const int64_t* indptr, const int* indices, const float* weights, const void* x,
                 void* y, int64_t nrows, int dtype, double scale, int64_t nnz, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* NIFTY_AMD_H */
