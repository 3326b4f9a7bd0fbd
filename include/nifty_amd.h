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
 *   nft_amp_*          Jacobian of the non-parametric amplitude subtree of the CF
 *                      model: _TwoLogIntegrations, _SlopeRemover, _Normalization,
 *                      fluctuation/zero-mode scaling (src/library/correlated_fields.py:
 *                      91-201, correlated_fields_simple.py:86-127), linearised
 *   nft_los_*          LOSResponse.apply on a box-blocked layout of the same COO
 *                      matrix, src/library/los_response.py:180-233
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
#define NFT_CG_DONE 8 /* this right-hand side has stopped (batched solves): set by the host when
                        * its controller stops, by the update's finalize (value 2) when the
                        * step is terminal whatever the controller says (curvature/alpha guard
                        * tripped; with NFT_CG_AUTO also a zero, negative or NaN new gamma) */
#define NFT_CG_ITER 9 /* steps finalized since the solve started (the host may queue several
                       * steps between reads) */
#define NFT_CG_AUTO 10 /* set by the host while it queues several steps: a zero, negative or
                        * NaN new gamma freezes the RHS too (DONE = 2; the guard always does) */
#define NFT_CG_LAZY 11 /* deferred-iterate CG (nft_hartley_fuse.lazy_*): the ring slot of this
                        * step's previous direction; set by the host, advanced by the
                        * carried iteration's finalize */
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
/* v = 0.5 + 0.5 tanh(x), d = 0.5 (1 - tanh(x)^2) for n values (dtype 0
 * fp64, 1 fp32): the value and derivative of the `sigmoid` pointwise map
 * (src/pointwise.py) in one pass, bitwise the separate elementwise passes. */
int nft_sigmoid_pair(const void* x, void* v, void* d, int64_t n, int dtype, hipStream_t stream);
/* For the metric shift*1 + M' with q = M' d formed without the shift:
 * sc[CURV] = sum d*(q + shift*d) */
int nft_cg_curv(const void* d, const void* q, int64_t n, int dtype, double shift, double* sc,
                void* ws, hipStream_t stream);
/* alpha = sc[GAMMA]/sc[CURV]; x -= alpha d; r -= alpha (q + shift d);
 * sc[GAMMA,XR,XB] <- r.r, x.r, x.b */
int nft_cg_update(void* x, void* r, const void* d, const void* q, const void* b, int64_t n,
                  int dtype, double shift, double* sc, void* ws, hipStream_t stream);
/* d = max(0, sc[GAMMA]/sc[GPREV]) d + r */
int nft_cg_direction(void* d, const void* r, int64_t n, int dtype, const double* sc,
                     hipStream_t stream);
/* r = (ax + shift x) - b; sc[GPREV] <- sc[GAMMA]; sc[GAMMA,XR,XB] <- r.r, x.r, x.b */
int nft_cg_residual(void* r, const void* ax, const void* x, const void* b, int64_t n, int dtype,
                    double shift, double* sc, void* ws, hipStream_t stream);
/* Batched forms: nrhs independent right-hand sides, vectors vstride elements
 * apart, scalar blocks NFT_CG_NSCALARS apart in sc, workspace nrhs times
 * nft_reduce_workspace(n).  Per RHS bitwise identical to the single forms;
 * a RHS with sc[NFT_CG_DONE] != 0 is left unchanged. */
int nft_dot_batched(const void* a, const void* b, int64_t n, int64_t vstride, int nrhs, int dtype,
                    double* out, int64_t out_stride, void* ws, hipStream_t stream);
int nft_cg_curv_batched(const void* d, const void* q, int64_t n, int64_t vstride, int nrhs,
                        int dtype, double shift, double* sc, void* ws, hipStream_t stream);
int nft_cg_update_batched(void* x, void* r, const void* d, const void* q, const void* b, int64_t n,
                          int64_t vstride, int nrhs, int dtype, double shift, double* sc, void* ws,
                          hipStream_t stream);
int nft_cg_direction_batched(void* d, const void* r, int64_t n, int64_t vstride, int nrhs, int dtype,
                             const double* sc, hipStream_t stream);
int nft_cg_residual_batched(void* r, const void* ax, const void* x, const void* b, int64_t n,
                            int64_t vstride, int nrhs, int dtype, double shift, double* sc, void* ws,
                            hipStream_t stream);

/* ---- power-bin distributor -------------------------------------------- */
/* out[p,i,q] = in[p, pindex[i], q]; in: [pre, nbins, post], out: [pre, npix, post] */
int nft_bin_gather(const void* in, const int* pindex, void* out, int64_t pre, int64_t npix,
                   int64_t nbins, int64_t post, int dtype, hipStream_t stream);
/* out[p,b,q] = sum_{j in [offsets[b], offsets[b+1])} in[p, perm[j], q], summed in
 * ascending j (perm = stable argsort of pindex: np.bincount order, bit-exact) */
int nft_bin_scatter(const void* in, const int* perm, const int* offsets, void* out, int64_t pre,
                    int64_t npix, int64_t nbins, int64_t post, int dtype, hipStream_t stream);
/* Same result (bitwise), faster gathers for post == 1: the sorted positions are
 * processed in chunks of nft_bin_chunk() entries; gpix / gslot list every
 * chunk's entries in ascending PIXEL order (gpix = the pixel, gslot = its
 * position in the chunk, uint16), so a wavefront's gathers touch nearby
 * memory; values are staged in LDS by gslot and each bin is still summed in
 * ascending j.  chunk_bins (nchunks + 1 entries, or NULL): first bin owned by
 * each chunk (the first bin whose offset is >= c * chunk; the last entry
 * nbins) -- precomputed instead of a binary search per workgroup.
 * gpix / gslot NULL: the plain sorted gathers of nft_bin_scatter. */
int nft_bin_chunk(void);
int nft_bin_scatter_ordered(const void* in, const int* perm, const int* offsets, const int* gpix,
                            const uint16_t* gslot, const int* chunk_bins, void* out, int64_t pre,
                            int64_t npix, int64_t nbins, int64_t post, int dtype, hipStream_t stream);
/* Mirror fold onto the fundamental cell of a harmonic grid (replaces, with
 * nft_bin_scatter on the folded grid, DOFDistributor._adjoint_times for
 * PowerSpace bins, src/operators/distributors.py:105-112: |k| and hence the bin
 * is invariant under k_a -> -k_a, rg_space.py:101-121):
 *   out[p, q] = sum of in[p, i] over the distinct images i_a in {q_a, n_a - q_a}
 * in: (pre, shape[0..ndim-1]); out: (pre, shape[a]/2 + 1 ...); 1 <= ndim <= 3.
 * Fixed summation order (deterministic), not np.bincount's order: the bin sums
 * agree with the reference to rounding (rtol ~1e-15), not bitwise. */
/* The mirror fold of nft_bin_fold from point-mirror pair sums on the half
 * grid (nft_hartley_fuse.epi_out2_pairs; shape = the FULL grid): per
 * fundamental cell the sum of the half-grid entries at the sign flips of all
 * but the last axis (2^(d-1) reads instead of 2^d).  Equal to nft_bin_fold to
 * rounding (the images are added in pairs). */
int nft_bin_fold_half(const void* in, void* out, int64_t pre, int ndim, const int64_t* shape, int dtype,
                      hipStream_t stream);
/* The half-grid fold of nft_bin_fold_half written in bin-sorted order, the
 * pre items of a cell adjacent: out[cpos[cell] * pre + p], cpos the inverse
 * of the folded bin index's stable bin -> cell permutation (1 <= pre <= 8). */
int nft_bin_fold_half_sorted(const void* in, void* out, const int* cpos, int64_t pre, int ndim,
                             const int64_t* shape, int dtype, hipStream_t stream);
/* cpos = NULL in nft_bin_fold_half_sorted: the fold in cell order with the
 * pre items interleaved, out[cell * pre + p]; nft_bin_scatter_il then sums
 * the bins of that layout (pre in {2, 4, 8}), one 8 pre-byte gather per
 * cell for all items -- bitwise nft_bin_fold_half + nft_bin_scatter. */
/* It works in chunks of nft_bin_scatter_il_chunk(pre) sorted positions;
 * chunk_bins (nchunks + 1 entries, or NULL: a binary search of offsets per
 * workgroup): the first bin whose offset is >= c * chunk, last entry nbins
 * -- a plan-time table as for nft_bin_scatter_ordered. */
/* The bin sums of a PLANAR mirror fold (pre, npix) -- nft_bin_fold /
 * nft_bin_fold_half output -- in the arithmetic of nft_bin_scatter_il: bins
 * of up to 64 positions summed in ascending position, longer bins (3-D
 * grids) one wave each (lane-strided partials, fixed shuffle tree).  Bitwise
 * nft_bin_scatter_il on the interleaved fold for every item, so a batch of k
 * right-hand sides gives the k = 1 sums (DOFDistributor._adjoint_times inside
 * the fused CF Jacobian adjoint, src/operators/distributors.py:105-112).
 * chunk_bins: the nft_bin_chunk() table of nft_bin_scatter_ordered, or NULL. */
int nft_bin_scatter_folded(const void* in, const int* perm, const int* offsets, const int* chunk_bins, void* out,
                           int64_t pre, int64_t npix, int64_t nbins, int dtype, hipStream_t stream);
int nft_bin_scatter_il_chunk(int64_t pre);
int nft_bin_scatter_il(const void* in, const int* perm, const int* offsets, const int* chunk_bins, void* out,
                       int64_t pre, int64_t npix, int64_t nbins, int dtype, hipStream_t stream);
int nft_bin_fold(const void* in, void* out, int64_t pre, int ndim, const int64_t* shape, int dtype,
                 hipStream_t stream);

/* ---- sparse LOS response --------------------------------------------- */
/* y[r] = scale * sum_j weights[j] * x[indices[j]], j in [indptr[r], indptr[r+1]) */
int nft_spmv_csr(const int64_t* indptr, const int* indices, const float* weights, const void* x,
                 void* y, int64_t nrows, int dtype, double scale, int64_t nnz, hipStream_t stream);
/* Host helper: partition CSR rows into CSR-stream blocks (<= 256 rows and
 * <= 2048 nonzeros each; a longer single row gets its own block).  indptr is
 * HOST memory; blocks[0..nblocks] receives the block row boundaries. */
int nft_csr_rowblocks(const int64_t* indptr, int64_t nrows, int* blocks, int64_t cap,
                      int64_t* nblocks);
/* y[r] = scale * rowscale[r] * sum_j weights[j] * colscale[c_j] * x[c_j]
 * (colscale / rowscale may be NULL = 1).  rowblocks (device, from
 * nft_csr_rowblocks) selects the CSR-stream kernel for short rows; NULL
 * selects one wave per row.  Fuses the diagonal factors around R in
 * sampling metrics (e.g. sigmoid' and the noise weights). */
int nft_spmv_scaled(const int64_t* indptr, const int* indices, const float* weights,
                    const int* rowblocks, int64_t nblocks, const void* x, const void* colscale,
                    const void* rowscale, void* y, int64_t nrows, int dtype, double scale,
                    hipStream_t stream);

/* ---- Hartley transform with fused elementwise prologue / epilogue ------ */
/* Flat real indices i (input) and j (output) of the C-contiguous arrays:
 *   u[i]    = (pro_a ? pro_a[i] : 1) * pro_x[i] + (pro_b ? pro_b[i] * pro_c[pro_index[i]] : 0)
 *             (u = in when pro_x is NULL)
 *   h       = scale * Hartley(u)
 *   out[j]  = (epi_a ? epi_a[j] : 1) * h[j] + (epi_d ? epi_shift * epi_d[j] : 0)
 *   epi_out2[j] = epi_b[j] * h[j]     (if epi_out2)
 * On the compile-time-planned power-of-two paths the prologue runs inside the
 * first axis pass and the epilogue inside the last one (no extra HBM pass);
 * other shapes run them as separate elementwise kernels.  This is the
 * correlated-field Jacobian's  HT[A*xi + xi0*dA[pindex]]  and its adjoint's
 * (A*v + shift*d, xi0*v)  (src/library/correlated_fields_simple.py:155-160),
 * optionally for a batch of right-hand sides sharing A, xi0 and pindex. */
typedef struct nft_hartley_fuse {
  const void *pro_a, *pro_x, *pro_b, *pro_c;
  const int* pro_index;
  const void *epi_a, *epi_d, *epi_b;
  void* epi_out2;
  double epi_shift;
  /* batch of transforms along a leading axis (0: no batch): elements per item,
   * and the per-item strides of pro_x, pro_c, out, epi_d, epi_out2 (0: the
   * item size, resp. B = pro_c's length for pro_c).  pro_a, pro_b,
   * pro_index, epi_a, epi_b are shared by all items. */
  int64_t batch_period;
  int64_t x_bstride, c_bstride, out_bstride, d_bstride, out2_bstride;
  /* element stride of pro_c (0: 1).  A batch may interleave its dA vectors
   * (c_bstride = 1, c_estride = nitems): the bin gather of element j then
   * reads one contiguous run pro_c[pindex[j] * nitems ...] for all items. */
  int64_t c_estride;
  /* per-item strides of pro_a, pro_b, epi_a, epi_b (0: shared by the batch,
   * the default) -- a batch of different linearisation points */
  int64_t a_bstride, b_bstride, ea_bstride, eb_bstride;
  /* 1: pro_index holds one bin per cell of the FUNDAMENTAL CELL of the
   * harmonic grid (n_a / 2 + 1 per transform axis, C order) instead of one
   * per element: element j reads pro_c[pro_index[cell(j)] * c_estride +
   * item * c_bstride], cell(j) = (min(k_a, n_a - k_a))_a -- the |k| mirror
   * image, which has j's bin.  The batched prologue then gathers dA once per
   * mirror class and writes all 2^d images (4x fewer scattered gathers at
   * d = 2, no per-element index read).  Requires the transform axes to be
   * all of an item's axes. */
  int64_t pro_folded;
  /* CG update carried by the epilogue (cg_x != NULL; batched adjoint of the
   * sampling metric with the curvature already known, nft_hartley_cg_blocks
   * > 0 for the geometry): for every output element j of item b, with
   * q = epi_a[j] * h (the value the epilogue would store in out, which is
   * then NOT written) and alpha = sc[GAMMA] / sc[CURV] of item b (scalar
   * block b * NFT_CG_NSCALARS of cg_sc, guards as nft_cg_update_batched):
   *   x[b * cg_stride + j] -= alpha d[..];  r[..] -= alpha (q + cg_shift d[..])
   * and per transform tile the partials r.r, x.r (x.b = 0) land at
   * cg_part[b * 3 * cg_nbtot + c * cg_nbtot + cg_blk0 + tile] for c = 0, 1, 2
   * -- nft_cg_finalize_batched folds them with the other segments'. */
  void *cg_x, *cg_r;
  const void* cg_d;
  const double* cg_sc;
  double* cg_part;
  int64_t cg_stride;
  double cg_shift;
  int32_t cg_nbtot, cg_blk0;
  /* CG direction carried by the folded prologue (dir_r != NULL, pro_folded,
   * batched): pro_x holds each item's previous direction d and is
   * overwritten with d = max(0, gamma / gprev) d + r (item b's scalar block
   * b * NFT_CG_NSCALARS of dir_sc; unchanged, partial 0, when its DONE is set)
   * before the prologue reads it, and dir_part[b * dir_pstride + dir_blk0 +
   * block] = dir_shift * (the block's sum of d^2), block <
   * nft_hartley_dir_blocks(item grid) -- the d.d partials of
   * nft_cg_direction_dd_batched for the grid segment. */
  const void* dir_r;
  const double* dir_sc;
  double* dir_part;
  int64_t dir_pstride;
  double dir_shift;
  int32_t dir_blk0, dir_pad;
  /* 1: epi_out2 receives point-mirror PAIR SUMS on the half grid (the
   * transform's last axis n -> n/2 + 1): out2[item][row][c] = epi_b * h at
   * (row, c) + epi_b * h at its point mirror (-row, -c), c <= n/2; a column
   * that is its own mirror (c = 0, n/2) holds the single value.  Half the
   * second output's bytes; nft_bin_fold_half completes the mirror fold from
   * it (engine-v2 strided unpack pass only). */
  int64_t epi_out2_pairs;
  /* quadratic form of a pointwise weight carried by the epilogue
   * (quad_part != NULL; batched, epi_a the only epilogue operand, no CG
   * epilogue; the same geometries as the CG epilogue): out = epi_a * h is
   * stored as usual and per transform tile of item b the fp64 sum of
   * h * out over the tile's elements lands at quad_part[b * quad_pstride +
   * quad_blk0 + tile], tile < nft_hartley_cg_blocks.  With epi_a = W this is
   * the data-space curvature (J d).W(J d) of a sampling metric
   * J^T W J with a pointwise W (Gaussian / Poisson likelihoods), formed
   * while the forward transform writes W J d -- the partials that
   * nft_fold_partials folds into the CG curvature (src/minimization/
   * conjugate_gradient.py:96-101 computes it as d.(A d)). */
  double* quad_part;
  int64_t quad_pstride;
  int32_t quad_blk0, quad_pad;
  /* deferred iterate of the carried CG (lazy_ring != NULL; the direction of
   * the row-staged or R2C-fused prologue and the CG epilogue, count-only
   * solves): step s =
   * dir_sc / cg_sc[b * NFT_CG_NSCALARS + NFT_CG_LAZY] of item b reads its
   * previous direction from ring slot s (slot 0: pro_x itself) and the
   * prologue writes the new one to slot s + 1, at lazy_ring + s *
   * lazy_sstride (rows x_bstride / cg_stride apart, as pro_x / cg_d), also
   * for a stopped item (its direction copied); the CG epilogue reads d from
   * that slot, leaves x as it is (x.r partial 0) and records the step's
   * alpha (NaN where the guards leave x unchanged) at lazy_alpha[b *
   * lazy_nslot + s].  nft_cg_lazy_flush then applies the recorded steps to x
   * in order -- bitwise the per-step update -- and copies the last
   * direction back: per step one 8-byte read of d in place of x's 16-byte
   * read and write. */
  void* lazy_ring;
  int64_t lazy_sstride;
  double* lazy_alpha;
  int64_t lazy_nslot;
  /* curvature fold carried by the transform (fold_nrhs > 0): fold_out[r *
   * fold_ostride] = the sum of fold_part[r * fold_nb + b] over b < fold_nb
   * for r < fold_nrhs, bitwise nft_fold_partials, formed by the first
   * workgroups of the R2C row pass (any other geometry, or with a prologue:
   * by nft_fold_partials launched first).  It lets the adjoint transform of
   * a sampling metric with a pointwise W fold the quad_part partials of the
   * forward one on its way (conjugate_gradient.py:101's d.q). */
  const double* fold_part;
  int64_t fold_nb;
  double* fold_out;
  int64_t fold_ostride;
  int64_t fold_nrhs;
} nft_hartley_fuse;

/* Partial blocks per item of the CG-carrying epilogue for a batched
 * Hartley transform of this geometry (leading batch axis not among `axes`),
 * or 0 when its last pass cannot carry the update. */
int nft_hartley_cg_blocks(int ndim, const int64_t* shape, int naxes, const int* axes, int dtype);

/* Blocks of the folded prologue over an item grid of ndim (1..3) axes -- the
 * number of dir_part entries per item of nft_hartley_fuse.dir_*; 0 for a bad
 * shape.  ndim >= 2 with n_last / 2 + 1 <= 2560: one block per group of
 * mirror rows, prod over the first ndim - 1 axes of (n_a / 2 + 1) (the
 * row-staged prologue: the cell row's dA runs in LDS, every row streamed
 * with aligned loads and stores); otherwise the fundamental cell
 * prod(n_a / 2 + 1) with its last axis padded to a multiple of 64, 256 cells
 * per block. */
int nft_hartley_dir_blocks(int ndim, const int64_t* shape);

int nft_hartley_fused_workspace(int ndim, const int64_t* shape, int naxes, const int* axes,
                                int dtype, size_t* bytes);
int nft_hartley_fused(const nft_hartley_fuse* fuse, const void* in, void* out, int ndim,
                      const int64_t* shape, int naxes, const int* axes, int dtype, int convention,
                      double scale, void* workspace, size_t ws_bytes, hipStream_t stream);

/* ---- box-blocked LOS response ----------------------------------------- */
/* Device arrays of a line-of-sight response regrouped by 256-pixel boxes
 * (16x16 over the last two grid axes, 1x256 for 1-D grids; the grid is
 * viewed as [L, H, W]).  Built on the host from the COO triplets
 * (LOSResponse._box_plan); all index arrays int32 unless noted.
 *   forward:  nitems work items (box item_box[i], segments item_seg[i]..[i+1],
 *             entries item_ent[i]..[i+1]);
 *             a segment is the run of one line of sight inside one box:
 *             entries seg_ent[s]..[s+1] with 8-bit local pixel ent_loc and fp32
 *             weight ent_wf; its partial goes to slot seg_slot[s]; line l owns
 *             slots los_ptr[l]..[l+1] (in box order).  The forward workspace
 *             holds the partial of vector v in slot k at ws[k * nvec + v].
 *   adjoint:  box b owns entries box_ent[b]..[b+1], sorted by local pixel;
 *             pixel t of the box owns pix_off[257*b+t]..[257*b+t+1] (uint16,
 *             relative to box_ent[b]); the lines crossing box b are
 *             box_lines[box_lptr[b]..box_lptr[b+1]) (ascending); each entry
 *             holds its line as an index into that list (ent_lidx: uint8 if
 *             lidx8 else uint16) and an fp32 weight ent_wa. */
typedef struct nft_los_plan {
  int64_t H, W;
  int bh, bw, nby, nbx;
  int64_t nbox, nlos, nitems, nseg;
  const int *item_box, *item_seg, *item_ent, *seg_ent, *seg_slot;
  const uint8_t* ent_loc;
  const float* ent_wf;
  const int* los_ptr;
  const int* box_ent;
  const uint16_t* pix_off;
  const int *box_lptr, *box_lines;
  const void* ent_lidx;
  int lidx8;
  const float* ent_wa;
  /* optional (NULL: one workgroup per work item): the work items of every
   * box, items box_item[b] .. box_item[b+1] - 1 (nbox + 1 entries).  Then the
   * batched forward runs one workgroup per box, the pixel tile staged once
   * for all of the box's items (same products and order: bitwise).  The
   * per-box forward stages aligned 16-entry chunks of ent_loc / ent_wf: both
   * arrays must hold 16 entries of padding past the last item. */
  const int* box_item;
  /* optional (NULL: box_ent): the start of every box's adjoint entries
   * (ent_lidx / ent_wa) when each box's run is padded to a multiple of 16
   * entries (8-bit line indices; padding never summed: the pixel runs end
   * before it).  The batched adjoint then stages them with 16-byte loads. */
  const int* box_ent_adj;
} nft_los_plan;

size_t nft_los_workspace(const nft_los_plan* plan);
/* y[l] = scale * rowscale[l] * sum_{(l,p)} w * colscale[p] * x[p]   (R x) */
int nft_los_forward(const nft_los_plan* plan, const void* x, const void* colscale,
                    const void* rowscale, void* y, void* ws, int dtype, double scale,
                    hipStream_t stream);
/* out[p] = scale * rowscale[p] * sum_{(l,p)} w * colscale[l] * y[l]   (R^T y) */
int nft_los_adjoint(const nft_los_plan* plan, const void* y, const void* colscale,
                    const void* rowscale, void* out, int dtype, double scale, hipStream_t stream);
/* Batched over 1 <= nvec <= 8 vectors (x / y / out advance by their strides;
 * the forward workspace holds nvec partial vectors: nvec * nft_los_workspace).
 * The matrix entries are read once per launch for all vectors; per vector
 * the results are bitwise those of the single forms. */
int nft_los_forward_batched(const nft_los_plan* plan, const void* x, const void* colscale,
                            const void* rowscale, void* y, void* ws, int dtype, double scale,
                            int nvec, int64_t x_stride, int64_t y_stride, hipStream_t stream);
int nft_los_quad_blocks(const nft_los_plan* plan);
int nft_los_forward_quad_batched(const nft_los_plan* plan, const void* x, const void* colscale,
                                 const void* rowscale, void* y, void* ws, int dtype, double scale,
                                 int nvec, int64_t x_stride, int64_t y_stride, double* qpart,
                                 int64_t qstride, hipStream_t stream);
int nft_los_adjoint_batched(const nft_los_plan* plan, const void* y, const void* colscale,
                            const void* rowscale, void* out, int dtype, double scale, int nvec,
                            int64_t y_stride, int64_t out_stride, hipStream_t stream);
/* Pixel-side scales per vector: the pixel-side factor of vector v is
 * colscale + v * colscale_stride (forward) / rowscale + v * rowscale_stride
 * (adjoint); stride 0 shares one factor as in the _batched forms.  This is the
 * chain rule of a pointwise nonlinearity in front of the response
 * (R diag(f'(s_v)) in the forward, diag(f'(s_v)) R^T in the adjoint,
 * src/operators/operator.py:_OpChain jacobians), applied while the pixels are
 * loaded / stored instead of as a separate pass over every vector.
 * nft_los_forward_ex takes the optional curvature partials of
 * nft_los_forward_quad_batched (qpart = NULL: none). */
int nft_los_forward_ex(const nft_los_plan* plan, const void* x, const void* colscale,
                       int64_t colscale_stride, const void* rowscale, void* y, void* ws, int dtype,
                       double scale, int nvec, int64_t x_stride, int64_t y_stride, double* qpart,
                       int64_t qstride, hipStream_t stream);
int nft_los_adjoint_ex(const nft_los_plan* plan, const void* y, const void* colscale,
                       const void* rowscale, int64_t rowscale_stride, void* out, int dtype,
                       double scale, int nvec, int64_t y_stride, int64_t out_stride,
                       hipStream_t stream);

/* ---- curvature from the data space ------------------------------------ */
/* For a CG metric shift * 1 + J^T R^T C R J (the LOS sampling metric) the
 * curvature d.(shift d + q) equals shift * d.d + (R J d).C (R J d): the first
 * term is summed while the direction is formed, the second while the LOS
 * forward reduces each line, and nft_fold_partials adds the two partial
 * vectors in a fixed order -- no separate pass over q and d.
 *   nft_cg_direction_dd_batched: d = max(0, gamma/gprev) d + r (as
 *     nft_cg_direction_batched) and part[rhs * pstride + b] = shift * (block b's
 *     sum of d_i^2), b < nft_cg_dd_blocks(n).
 *   nft_los_forward_quad_batched: nft_los_forward_batched plus
 *     qpart[v * qstride + b] = sum over the lines of block b of t_l * y_l
 *     (t = R (colscale x) before scale * rowscale, y the output), b <
 *     nft_los_quad_blocks(plan).
 *   nft_fold_partials: out[rhs * out_stride] = fixed-order sum of part[rhs * nb
 *     .. rhs * nb + nb). */
int nft_cg_dd_blocks(int64_t n);
int nft_cg_direction_dd_batched(void* d, const void* r, int64_t n, int64_t vstride, int nrhs, int dtype,
                                const double* sc, double shift, double* part, int64_t pstride,
                                hipStream_t stream);
/* nft_cg_direction_dd_batched over two segments in one launch: [0, n1) with
 * partials at part[rhs * pstride + b] and [o2, o2 + n2) (o2 >= n1) at
 * part[rhs * pstride + poff2 + b] (poff2 >= nft_cg_dd_blocks(n1)); per
 * block the work of two separate calls. */
int nft_cg_direction_dd2_batched(void* d, const void* r, int64_t n1, int64_t o2, int64_t n2, int64_t vstride,
                                 int nrhs, int dtype, const double* sc, double shift, double* part, int64_t poff2,
                                 int64_t pstride, hipStream_t stream);
int nft_fold_partials(const double* part, int nb, int nrhs, double* out, int64_t out_stride,
                      hipStream_t stream);
/* The deferred iterate's flush (nft_hartley_fuse.lazy_*): for every row b <
 * nrhs and element i < n, x[b * vstride + i] -= alpha_t d_t[b * vstride + i]
 * for the recorded steps t < nsteps in order (alpha_t = alpha[b * nslot + t],
 * skipped when NaN; d_t = ring slot t + 1 at ring + t * sstride), then d[b *
 * vstride + i] = slot nsteps (the current direction back in place). */
int nft_cg_lazy_flush(void* x, void* d, const void* ring, int64_t sstride, const double* alpha, int64_t nslot,
                      int nsteps, int64_t n, int64_t vstride, int nrhs, int dtype, hipStream_t stream);
/* nft_los_adjoint_batched and nft_fold_partials(fold_part, fold_nb,
 * fold_nrhs, fold_out, fold_ostride) in ONE launch (the fold runs as the first
 * fold_nrhs workgroups of the adjoint's grid, bitwise the separate call): the
 * carried CG's curvature, needed only by the adjoint transform's last pass,
 * without a launch of its own between the two LOS passes and the transform. */
int nft_los_adjoint_fold(const nft_los_plan* plan, const void* y, const void* colscale,
                         const void* rowscale, void* out, int dtype, double scale, int nvec,
                         int64_t y_stride, int64_t out_stride, const double* fold_part, int fold_nb,
                         int fold_nrhs, double* fold_out, int64_t fold_ostride, hipStream_t stream);
/* The CG update split over segments of the packed vectors (pointers offset by
 * the caller), so that the update of one segment can run while another
 * segment's q is still being formed (the amplitude keys' VJP on a second
 * stream while the grid segment updates).  The segment's nft_cg_dd_blocks(n)
 * partial blocks land at [blk0, blk0 + nb) of each RHS's 3 x nbtot partial
 * array (r.r, x.r, x.b rows); nft_cg_finalize_batched folds all nbtot in
 * index order and records gamma / alpha / flags as nft_cg_update_batched
 * does.  Per element the arithmetic is that of nft_cg_update_batched. */
int nft_cg_update_seg_batched(void* x, void* r, const void* d, const void* q, const void* b, int64_t n,
                              int64_t vstride, int nrhs, int dtype, double shift, const double* sc,
                              double* part, int nbtot, int blk0, hipStream_t stream);
/* The same over two segments in one launch (the amplitude keys before and
 * after the grid segment): elements [0, n1) with partial blocks at blk1 and
 * [o2, o2 + n2) (o2 >= n1) at blk2, the block ranges disjoint; b = NULL.
 * Per block the work (and so every partial) of two separate
 * nft_cg_update_seg_batched calls. */
int nft_cg_update_seg2_batched(void* x, void* r, const void* d, const void* q, int64_t n1, int blk1, int64_t o2,
                               int64_t n2, int blk2, int64_t vstride, int nrhs, int dtype, double shift,
                               const double* sc, double* part, int nbtot, hipStream_t stream);
int nft_cg_finalize_batched(const double* part, int nbtot, int nrhs, double* sc, hipStream_t stream);

/* ---- correlated-field amplitude Jacobian ------------------------------ */
/* Constants of the amplitude linearisation at one expansion point (all device
 * pointers, fp64).  B = number of power bins, M = B - 2.
 *   c0 = sf*sq0, sf, p0, p1, p2, lv          [M]   (spectrum/flex/asp coefficients)
 *   vslope, sc, Qf, Qa, mspec = mult*spec, An [B]
 * Qf/Qa: SlopeRemove(TwoLog(.)) of the flexibility/asperity coefficients. */
typedef struct nft_amp_const {
  const double *c0, *sf, *p0, *p1, *p2, *lv;
  const double *vslope, *sc, *Qf, *Qa, *mspec, *An;
  double fl, S, ls_f, sig_s, zm, ls_o, total_volume;
  int64_t B;
  int has_flex, has_asp, has_zm;
} nft_amp_const;

/* Cotangent outputs of the VJP (device pointers; NULL for absent keys):
 * out = shift * d + J_amp^T g, d pointers may be NULL (then shift * d = 0). */
typedef struct nft_amp_out {
  double *fl, *sl, *flex, *asp, *zm, *spec;
  const double *dfl, *dsl, *dflex, *dasp, *dzm, *dspec;
  double shift;
} nft_amp_out;

size_t nft_amp_workspace(int64_t B);
/* da[B] = J_amp [t_fl, t_sl, t_flex, t_asp, t_zm, t_spec(2,M)] */
int nft_amp_jvp(const nft_amp_const* c, const double* t_fl, const double* t_sl,
                const double* t_flex, const double* t_asp, const double* t_zm,
                const double* t_spec, double* da, double* ws, hipStream_t stream);
int nft_amp_vjp(const nft_amp_const* c, const double* g, const nft_amp_out* out, double* ws,
                hipStream_t stream);
/* Batched: nrhs right-hand sides; tangent / cotangent pointers (and d) advance
 * by lat_stride elements per RHS, da / g by da_stride (g_stride); bin b of
 * RHS r is written to da[r * da_stride + b * da_elem_stride] (da_elem_stride
 * 0: 1; da_stride 1 with da_elem_stride nrhs interleaves the RHS, see
 * nft_hartley_fuse.c_estride); workspace nrhs * nft_amp_workspace(B).  Per
 * RHS identical to the single forms.  item_consts: NULL (every RHS uses *c)
 * or a DEVICE array of nrhs nft_amp_const, one linearisation point per RHS
 * (same B and flags as *c; batched geoVI refinement of several samples). */
int nft_amp_jvp_batched(const nft_amp_const* c, const nft_amp_const* item_consts, const double* t_fl,
                        const double* t_sl, const double* t_flex, const double* t_asp,
                        const double* t_zm, const double* t_spec, double* da, double* ws, int nrhs,
                        int64_t lat_stride, int64_t da_stride, int64_t da_elem_stride,
                        hipStream_t stream);
int nft_amp_vjp_batched(const nft_amp_const* c, const nft_amp_const* item_consts, const double* g,
                        const nft_amp_out* out, double* ws, int nrhs, int64_t lat_stride,
                        int64_t g_stride, hipStream_t stream);

/* Two-phase amplitude JVP / VJP (csrc/nft_amp2.hip: two launches each; the
 * first forms per-tile dot products of the tangent / cotangent with constant
 * vectors, the second the tile carries in a fixed order, the tile-local scans
 * and the outputs); the batched forms above take this path when it applies.
 * These kernels keep device-global arrival counters, so calls must not
 * overlap: a call on another stream than the previous (eager) call first
 * waits on the host for that stream's work, under a library mutex held from
 * that check through the call's launches, so eager calls from any number of
 * streams and host threads run one after the other.  Calls on a stream under
 * HIP-graph capture are not tracked: graphs holding them must not be replayed
 * concurrently with each other or with eager calls on other streams (the
 * caller's rule; the library cannot see a replay).  Key arrays are indexed fl, sl, flex, asp, zm, spec (NULL:
 * absent key), pointing at right-hand side 0, rows lat_stride elements apart.
 * item_mode: 0 = every RHS uses *c; 1 = item_consts is a DEVICE array of nrhs
 * constant sets (one per RHS); 2 = item_consts is ONE device constant set
 * shared by every RHS (read once per workgroup for up to 4 RHS).  *c gives B
 * and the flags in every mode.  Returns NFT_AMP2_FALLBACK (nothing launched)
 * when NFT_AMP2=0 or B is too small / large; the caller then uses the
 * multi-kernel path.  Workspace: nrhs * nft_amp_workspace(B) bytes.
 *
 * nft_amp2_jvp: da[r * da_stride + b * da_elem_stride] = J_amp t_r.  With
 * r != NULL (residual keys) the tangent t is the CG direction and is first
 * updated in place, d = max(0, gamma/gprev) d + r (per RHS scalars in sc,
 * unchanged when sc[NFT_CG_DONE] != 0), and part[r * pstride + tile] =
 * shift * d.d of the amplitude keys per tile (nft_amp2_tiles tiles; tile 0
 * includes the scalar keys; 0 for a finished RHS) -- the identity part of the
 * data-space curvature.
 *
 * nft_amp2_vjp: out[key] = shift * d[key] + J_amp^T g_r (d may be NULL), or,
 * with out2 != NULL, the CG update of the amplitude keys carried instead:
 * out = x keys, out2 = r keys, d = direction keys, x -= alpha d,
 * r -= alpha (J_amp^T g + shift d) with alpha = sc[GAMMA] / sc[CURV] and the
 * guards of nft_cg_update_batched; then the iteration's finalize
 * (nft_cg_finalize_batched semantics, x.b = 0) over the r.r / x.r partials of
 * the amplitude keys (part: 2 * nft_amp2_tiles per RHS, pstride apart) and of
 * the grid segment (gpart: ngp r.r partials at gpart[r * gp_stride + t], the
 * x.r ones gp_row after them), folded in a fixed order. */
#define NFT_AMP2_FALLBACK 1
int nft_amp2_enabled(void);
/* on = 0 / 1: force the two-phase path off / on for later calls (A/B and
 * tests); on < 0: back to the environment (NFT_AMP2) */
void nft_amp2_set_enabled(int on);
int nft_amp2_tiles(int64_t B, int nrhs, int item_mode);
/* Constant-scan table of one linearisation (item_mode 0: *c, 2: the device
 * set item_consts; not per-RHS sets): the tile-local scans and tile sums that
 * involve the constants only, formed once by nft_amp2_prepare
 * (nft_amp2_tab_size(B) doubles, device) with the kernels' own scan and sum
 * code, so that the JVP / VJP given `tab` skip them and produce bitwise the
 * same results.  Valid while the constants it was made from are unchanged. */
int64_t nft_amp2_tab_size(int64_t B);
int nft_amp2_prepare(const nft_amp_const* c, const nft_amp_const* item_consts, int item_mode, double* tab,
                     hipStream_t stream);
/* dtype (0 fp64, 1 fp32): the element type of the key arrays, da and g
 * (the fp32-storage CG); constants, workspace, sums, part and sc stay fp64 and
 * every sum accumulates in fp64.  tab: NULL, or the table of nft_amp2_prepare
 * for the same constants and item_mode (0 or 2). */
int nft_amp2_jvp(const nft_amp_const* c, const nft_amp_const* item_consts, int item_mode, void* const* t,
                 const void* const* r, int64_t lat_stride, void* da, int64_t da_stride, int64_t da_elem_stride,
                 double* ws, int nrhs, const double* sc, double* part, int64_t pstride, double shift, int dtype,
                 const double* tab, hipStream_t stream);
int nft_amp2_vjp(const nft_amp_const* c, const nft_amp_const* item_consts, int item_mode, const void* g,
                 int64_t g_stride, void* const* out, void* const* out2, const void* const* d, int64_t lat_stride,
                 double shift, double* ws, int nrhs, double* sc, double* part, int64_t pstride, const double* gpart,
                 int64_t gp_stride, int64_t gp_row, int ngp, int dtype, const double* tab, hipStream_t stream);



/* Amplitude model (device pointers, fp64; M = B - 2): the operator chain of
 * src/library/correlated_fields_simple.py:85-127 (_Normalization, _SlopeRemover,
 * _TwoLogIntegrations, the LognormalTransform / NormalTransform scalings) with
 * its fixed per-bin vectors:
 *   vslope = relative log k-lengths, sc = vslope / vslope[B-1], mult = mode
 *   multiplicity                                          [B]
 *   lv = log-volumes, sqrt_lv = sqrt(lv), shift0 = lv^2/12  [M]  (has_flex) */
typedef struct nft_amp_model {
  const double *vslope, *sc, *mult, *lv, *sqrt_lv, *shift0;
  double lm_f, ls_f, mu_s, sig_s, lm_x, ls_x, lm_a, ls_a, lm_o, ls_o, total_volume;
  int64_t B;
  int has_flex, has_asp, has_zm;
} nft_amp_model;
/* Amplitude value at nrow latent points (lat pointers advance by lat_stride
 * per row; a NULL key is an absent model component) and, for each row, the
 * constants of its linearisation: a[r * a_stride + b] (B values),
 * buf[r * buf_stride ..] = c0, sf, p0, p1, p2 [M each], Qf, Qa, mspec, An [B
 * each] (buf_stride >= nft_amp_forward_buf(B)), and item_consts[r] -- a DEVICE
 * nft_amp_const pointing into buf and the model, with fl, S and zm set: the
 * item_consts argument of nft_amp_jvp_batched / nft_amp_vjp_batched.  No value
 * goes through the host.  ws: nrow * nft_amp_workspace(B) bytes. */
int64_t nft_amp_forward_buf(int64_t B);
int nft_amp_forward_batched(const nft_amp_model* model, const double* x_fl, const double* x_sl,
                            const double* x_flex, const double* x_asp, const double* x_zm,
                            const double* x_spec, int64_t lat_stride, int nrow, double* a,
                            int64_t a_stride, double* buf, int64_t buf_stride,
                            nft_amp_const* item_consts, double* ws, hipStream_t stream);

/* ---- launch profiler (HIP events) -------------------------------------- */
/* Between nft_prof_begin and nft_prof_end every hot-path kernel launch
 * records a HIP event on its stream just before the launch; nft_prof_end
 * returns the per-launch durations (ms) in launch order, nft_prof_label(i) the
 * kernel family of launch i.  Not for use during HIP graph capture. */
int nft_prof_begin(int capacity);
int nft_prof_end(hipStream_t stream, float* ms, int cap, int* n);
const char* nft_prof_label(int i);

#ifdef __cplusplus
}
#endif
#endif /* NIFTY_AMD_H */
