/*
 * nerf_amd.h — C-ABI of the MI355X (gfx950) NeRF ray-marching hot path.
 *
 * Every entry point is stateless, works on caller-owned device pointers and
 * enqueues its kernels on the caller's HIP stream (passed as `void*`, i.e. a
 * hipStream_t; NULL = the default stream).  Nothing here allocates device
 * memory, synchronises the stream, or keeps global mutable state, so every
 * call can be captured in a hipGraph.  All tensors are fp32 unless stated.
 *
 * Return value: NERF_OK (0) or a negative status (see nerf_status_string).
 *
 * Reference interfaces replaced (sarphiv/nerf-experiments, read-only copy):
 *   - composite  : NerfInterpolation._render_rays        barf/model_interpolation.py:316-353
 *                  (copies: naive-to-vanilla/model_interpolation.py:198-235,
 *                   mip_NeRF/model_interpolation.py:192-229, 3d-ingp/model.py:347-380)
 *   - resample   : NerfInterpolation._sample_t_pdf_weighted barf/model_interpolation.py:193-277
 *                  (round/argmax variant: naive-to-vanilla/model_interpolation.py:128-169)
 *   - sampling   : _sample_t_stratified_uniform + _get_intervals
 *                                                        barf/model_interpolation.py:114-180
 *   - encoding   : FourierFeatures / BarfPositionalEncoding / IntegratedFourierFeatures
 *                  (+ IntegratedBarfFourierFeatures)     barf/positional_encodings.py:28-282
 *                  fused with _compute_positions         barf/model_interpolation.py:288-312
 *   - hash grid  : INGPTable / INGPEncoding              3d-ingp/model.py:14-121
 *   - linear     : the nn.Linear (addmm) chain of NerfModel.forward
 *                                                        barf/model_interpolation_architecture.py:96-141
 *                  and its autograd backward (dX, dW, db)
 *
 * The reference has no FFI for this path (it is pure PyTorch); INTEGRATION.md
 * shows the ctypes binding a maintainer would add, which is exactly what
 * nerf-experiments_amd/nerf_amd/_lib.py does.
 */
#ifndef NERF_AMD_H
#define NERF_AMD_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NERF_OK 0
#define NERF_ERR_INVALID_ARG (-1)
#define NERF_ERR_UNSUPPORTED (-2)
#define NERF_ERR_LAUNCH (-3)
#define NERF_ERR_WORKSPACE (-4)

/* Library / ABI version (bumped on any signature or data-layout change; 6: NERF_FUSED_MASK;
 * 7: nerf_fused_composite / nerf_mlp_fused_render; 8: nerf_hashgrid_workspace_n, fused compositing
 * of 256-sample rays; 9: nerf_hashgrid_bwd_pos, seg_gen on later layers of the fused forward;
 * 10: nerf_mlp_fused_run (single-pass bf16 flag), the passes argument of nerf_linear_wgrad_x3*). */
int nerf_abi_version(void);
const char* nerf_status_string(int status);
/* sizeof of the argument structs, for bindings to check their layouts against:
 * 0 nerf_pe_params, 1 nerf_fused_layer, 2 nerf_fused_encoding, 3 nerf_hashgrid_params,
 * 4 nerf_adam_batch, 5 nerf_seg, 6 nerf_fused_composite; -1 for an unknown index. */
int64_t nerf_struct_size(int32_t which);
/* Build flags of the loaded library: 0 for a product build.  Bit 0 (NERF_BUILD_DIAG_FUSED): the
 * fused field-MLP kernels were compiled with a NERF_FUSED_DIAG_* switch; bit 1
 * (NERF_BUILD_DIAG_WGRAD): the streamed weight gradient with a NERF_WS_DIAG_* switch.  Those
 * switches drop work for profiling ablations and give wrong results by construction; bindings
 * refuse a library with any bit set (nerf_amd/_lib.py load()). */
#define NERF_BUILD_DIAG_FUSED 1
#define NERF_BUILD_DIAG_WGRAD 2
int32_t nerf_build_flags(void);

/* ---------------------------------------------------------------------------
 * Alpha compositing (a4).  One wavefront per ray, exclusive prefix sum of
 * b_s = ((-sigma_s * delta_s) * scale_a) * scale_b accumulated in fp64 (the
 * reference's CPU cumsum accumulates fp32 input in double).
 *   T_s = exp(sum_{j<s} b_j),  alpha_s = 1 - exp(b_s),  w_s = T_s * alpha_s,
 *   rgb = sum_s w_s * c_s.
 * Reference factor: scale_a = 3, scale_b = MAGIC_NUMBER (barf: 1/3, n2v/mip: 7);
 * 3d-ingp uses scale_a = scale_b = 1.
 * act = 0: density/color are already activated (the _render_rays contract).
 * act = 1: density is raw, sigma = softplus(raw - density_shift, beta=1,
 *          threshold=8) and color is raw, c = sigmoid(raw)  (NerfModel heads
 *          fused in; model_interpolation_architecture.py:137-138).
 * Addressing: sample n = ray*S + s; density[n*density_stride],
 * color[n*color_stride + 0..2], dist[n], rgb_out[ray*3 + c], weights_out[n]
 * (weights_out may be NULL).  S <= 1024.
 * ------------------------------------------------------------------------- */
int nerf_composite_fwd(const float* density, int64_t density_stride,
                       const float* color, int64_t color_stride,
                       const float* dist, int64_t n_rays, int32_t samples_per_ray,
                       float scale_a, float scale_b, int32_t act, float density_shift,
                       float* rgb_out, float* weights_out, void* stream);

/* Backward of nerf_composite_fwd.  grad_rgb [n_rays,3]; grad_weights [n] or
 * NULL.  Writes grad_density[n*gd_stride] and grad_color[n*gc_stride+0..2]
 * (w.r.t. the raw inputs when act = 1).  Either output may be NULL. */
int nerf_composite_bwd(const float* density, int64_t density_stride,
                       const float* color, int64_t color_stride,
                       const float* dist, int64_t n_rays, int32_t samples_per_ray,
                       float scale_a, float scale_b, int32_t act, float density_shift,
                       const float* grad_rgb, const float* grad_weights,
                       float* grad_density, int64_t gd_stride,
                       float* grad_color, int64_t gc_stride, void* stream);

/* ---------------------------------------------------------------------------
 * Stratified / equidistant t sampling (a6) + _get_intervals.
 *   t_s = linspace(near, far - D, S)[s]  (D = (far-near)/S)
 *         + (stratified ? U_{r,s} * D : 0) + (offset != 0 ? U_r * D * offset : 0)
 *   t_start = t; t_end[s] = t[s+1], t_end[S-1] = far.
 * U are Philox-4x32-10 uniforms in [0,1) keyed by (seed, offset_counter).
 * ------------------------------------------------------------------------- */
int nerf_sample_uniform(int64_t n_rays, int32_t samples_per_ray, float near_, float far_,
                        int32_t stratified, float offset_size,
                        uint64_t seed, uint64_t counter,
                        float* t_start, float* t_end, void* stream);

/* ---------------------------------------------------------------------------
 * PDF-weighted fine resampling (a5).  One wavefront per ray, n_bins <= 64.
 * mode 0 (barf): largest-remainder integer allocation of n_samples - n_bins
 *   fine samples (ties by index, as argsort().argsort() on CPU), +1 per bin,
 *   exclusive scan, t_j = t_coarse_i + ((j - c_i) * dist_i) / n_i.
 * mode 1 (naive-to-vanilla / 3d-ingp): round(w * (n_samples - n_bins)) with the
 *   remainder added to the first argmax bin.
 * If any ray's allocation is invalid (non-finite weights, wrong total) the
 * whole batch falls back — as the reference does after its retry loop — to
 * equidistant sampling with a per-ray offset of -U_r * D (model_interpolation.py:274-275),
 * using (seed, counter) for U_r.  status (device int32, caller-zeroed) gets
 * bit 0 set in that case.
 * mode 2 (nerf-siren/model.py:106-112, _sample_t_fine(linspace=False); the multinomial
 *   branch of 3d-ingp/model.py:306-312): n_fine = n_samples - n_bins bins drawn with
 *   replacement with probability w_i / sum w (inverse of the fp64 cumulative weights at
 *   U_j * sum, U_j = Philox(seed, counter, ray * n_fine + j)), t = t_coarse[bin] +
 *   U'_j * dist[bin] (U' from counter ^ 2^62), concatenated with t_coarse and sorted
 *   ascending (stable).  n_samples <= 512.  A row torch.multinomial would reject (negative /
 *   non-finite weight, zero sum) draws its bins uniformly and sets bit 1 of status.
 * ------------------------------------------------------------------------- */
int nerf_resample_pdf(const float* t_coarse, const float* weights, const float* dist_coarse,
                      int64_t n_rays, int32_t n_bins, int32_t n_samples, int32_t mode,
                      float near_, float far_, uint64_t seed, uint64_t counter,
                      float* t_start, float* t_end, int32_t* status, void* stream);

/* ---------------------------------------------------------------------------
 * Positional encodings (a1-a3), fused with sample-position generation.
 *
 * Sample n (= ray*S + s).  Position source:
 *   - x != NULL : position = x[n*3 .. n*3+2]   (S is ignored for positions)
 *   - x == NULL : position = o[ray] + tq * d[ray], tq = t_start[n] (query=0,
 *                 "left") or (t_start[n]+t_end[n])/2 (query=1, "middle").
 * kind 0 = Fourier / BARF: args = p_d * (scale * 2^k) (fp32), out =
 *   [p (if identity) | mask_k*cos(args) (d-major, k-minor) | mask_k*sin(args)].
 *   use_mask == 0 means all ones (plain FourierFeatures).  levels <= 16.
 * kind 1 = integrated (mip-NeRF IPE, positional_encodings.py:170-240); needs
 *   dir (per ray, or the direction itself when x != NULL via xdir),
 *   pixel_width (pw_mode 0: pw[ray]; 1: pw[n % n_rays] — the reference's
 *   (B,)-shaped .repeat quirk; 2: pw[n]), t_start, t_end; variance
 *   distributed if distribute_variance.  Optional BARF mask (IntegratedBarf...).
 * out row stride out_ld >= output_dim; columns [output_dim, out_ld) are zeroed.
 * ------------------------------------------------------------------------- */
typedef struct nerf_pe_params {
    int32_t kind;               /* 0 fourier/barf, 1 integrated (2 hash grid: nerf_fused_encoding only) */
    int32_t levels;             /* L */
    int32_t include_identity;   /* 0/1 */
    int32_t query;              /* 0 left, 1 middle (ray mode) */
    float scale;                /* base scale (2*pi, 1.0, ...) */
    float pixel_width_sigma;    /* IPE extra variance when > 0.25 */
    int32_t distribute_variance;/* IPE */
    int32_t pw_mode;            /* IPE pixel width addressing */
    int32_t use_mask;           /* 0: plain Fourier features */
    float mask[16];             /* BARF coarse-to-fine mask values (by value: no
                                   device copy and no int(alpha) sync per step) */
} nerf_pe_params;

int nerf_encode_fwd(const nerf_pe_params* params,
                    const float* x, const float* xdir,
                    const float* ray_o, const float* ray_d,
                    const float* t_start, const float* t_end, const float* pixel_width,
                    int64_t n_samples, int32_t samples_per_ray, int64_t n_rays,
                    float* out, int64_t out_ld, void* stream);

/* Backward of kind-0 encodings w.r.t. an explicit position input x:
 *   dx[n,d] = g_id + sum_k mask_k*scale*2^k*(-g_cos*sin(a) + g_sin*cos(a)).
 * grad_out has row stride g_ld. If accumulate, dx += ... */
int nerf_encode_bwd(const nerf_pe_params* params, const float* x,
                    const float* grad_out, int64_t g_ld, int64_t n_samples,
                    float* dx, int32_t accumulate, void* stream);

/* Backward of kind-1 (integrated) encodings w.r.t. the position x and the direction xdir
 * (autograd of positional_encodings.py:186-235 and of the masked variant :274-282), one
 * thread per sample.  Inputs as nerf_encode_fwd with x != NULL and pw_mode 2 (per-sample
 * pixel_width[n]).  dx / ddir [n,3] (either may be NULL; accumulate: +=).  t_start, t_end and
 * pixel_width receive no gradient. */
int nerf_encode_bwd_integrated(const nerf_pe_params* params, const float* x, const float* xdir,
                               const float* t_start, const float* t_end, const float* pixel_width,
                               const float* grad_out, int64_t g_ld, int64_t n_samples,
                               float* dx, float* ddir, int32_t accumulate, void* stream);

/* Backward of a ray-mode encoding (nerf_encode_fwd with x == NULL: positions o + tq*d
 * generated in-kernel) w.r.t. the rays:
 *   d_origs[r] = sum_s g_pos(r,s),  d_dirs[r] = sum_s (tq(r,s) * g_pos(r,s) + g_dir(r,s)),
 * g_pos / g_dir = the encoding's gradient w.r.t. the sample position / direction (g_dir = 0 for
 * kind 0).  This is the gradient pose refinement takes through _compute_positions
 * (barf/model_interpolation.py:288-312) into CameraExtrinsics (model_camera_extrinsics.py:77-85).
 * One wavefront per ray, fp64 accumulation in a fixed order.  Same params / inputs as the
 * forward; either output may be NULL; accumulate: +=. */
int nerf_encode_bwd_rays(const nerf_pe_params* params, const float* ray_o, const float* ray_d,
                         const float* t_start, const float* t_end, const float* pixel_width,
                         const float* grad_out, int64_t g_ld, int64_t n_rays, int32_t samples_per_ray,
                         float* d_origs, float* d_dirs, int32_t accumulate, void* stream);

/* Per-ray direction encoding (dir PE evaluated once per ray instead of once
 * per sample; the MLP reads row n / samples_per_ray).  kind 0 only. */
int nerf_encode_rays(const nerf_pe_params* params, const float* ray_d, int64_t n_rays,
                     float* out, int64_t out_ld, void* stream);

/* ---------------------------------------------------------------------------
 * Linear layers on fp32 MFMA (v_mfma_f32_32x32x2_f32, exact fp32 FMA chains).
 *
 * An operand is a column-concatenation of up to 4 row-major segments.  Segment
 * j has k_j valid columns (k_j % 4 == 0, ld % 4 == 0, 16-byte aligned ptr) and
 * occupies kp_j = roundup(k_j, 32) columns [koff_j, koff_j + kp_j) of the packed
 * K dimension (columns past k_j read as zero); row m of the operand is row
 * m / row_div_j of segment j (row_div > 1 broadcasts a per-ray tensor over its
 * samples).  M < 2^31.
 * ------------------------------------------------------------------------- */
typedef struct nerf_seg {
    const float* ptr;
    int64_t ld;
    int32_t k;
    int32_t row_div;
} nerf_seg;

#define NERF_EPI_BIAS  1   /* + bias[n] */
#define NERF_EPI_RELU  2   /* max(., 0) */
#define NERF_EPI_MASK  4   /* * (aux[m, n] > 0): ReLU backward */
#define NERF_EPI_ACCUM 8   /* out += result */
#define NERF_EPI_MASKBITS 16 /* with MASK: aux is the bit mask written by MASKOUT */
#define NERF_EPI_MASKOUT  32 /* also write (out > 0) as a bit mask into aux (N <= 256): row m
                                is 8 uint32 words at (char*)aux + m*ld_aux (ld_aux >= 32 bytes,
                                multiple of 16); bit b of word 2e+h <-> column 4(32h+b)+e */
#define NERF_EPI_NO_PERSIST 256  /* tuning: one tile per workgroup instead of a persistent grid */
#define NERF_EPI_NARROW_TILE 512 /* tuning: force the 128-column tile of the split-precision kernel for N > 128 */
#define NERF_EPI_TANH      4096  /* tanh(.) after the bias (2d-reconstruction/model.py:48-56) */
#define NERF_EPI_TANH_BWD  8192  /* * (1 - y*y), y = aux[m, n] (fp32, row stride ld_aux): tanh backward;
                                    not with MASK (both read aux) */
#define NERF_EPI_GAUSS     1024  /* internal (nerf_linear_gauss_x3): Gaussian activation forward */
#define NERF_EPI_GAUSS_BWD 2048  /* internal (nerf_linear_gauss_x3): Gaussian activation backward */

/* out[m, n] = epi( sum_k A[m, k] * W[n, k] ),  m < M, n < N.
 * W: packed row-major [ceil(N/128)*128][ldw], ldw = sum_j kp_j (zero padding
 * rows/cols).  out row stride ldo.  N <= 32 uses a 128 x 32 tile. */
int nerf_linear_fwd(const nerf_seg* segs, int32_t n_segs, int64_t M,
                    const float* W, int32_t ldw, int32_t N, const float* bias,
                    float* out, int64_t ldo, int32_t epilogue,
                    const float* aux, int64_t ld_aux, void* stream);

/* Weight-gradient partials: for a grid of split-M slices,
 *   slab[s][n][k] = sum_{m in slice s} dY[m, n] * X[m, k],
 *   db_slab[s][n] = sum_{m in slice s} dY[m, n].
 * workspace must hold nerf_linear_wgrad_workspace(...) bytes.  Then
 * nerf_linear_wgrad_reduce (same M, N, K) sums the slices in a fixed order
 * (deterministic) and scatters rows n < n_valid into dW[n, col_map[k]]
 * (row stride ld_dw; col_map[k] < 0 skips; col_map NULL = identity) and db[n]
 * (db may be NULL); accumulate != 0 adds the rounded sums onto dW / db instead (the second
 * pass of a field used twice per step lands in the same gradient).  dY needs N % 4 == 0 and ld_dy % 4 == 0: pass N rounded up
 * to 4 over a zero-padded dY and the true row count as n_valid. */
size_t nerf_linear_wgrad_workspace(int64_t M, int32_t N, int32_t K);
int nerf_linear_wgrad(const float* dY, int64_t ld_dy, int32_t N,
                      const nerf_seg* segs, int32_t n_segs, int64_t M,
                      void* workspace, size_t workspace_bytes, void* stream);
int nerf_linear_wgrad_reduce(int64_t M, int32_t N, int32_t K, int32_t n_valid,
                             const void* workspace, const int32_t* col_map,
                             float* dW, int64_t ld_dw, float* db, int32_t accumulate, void* stream);

/* Pack an nn.Linear weight W[N][K_orig] into the kernel layouts:
 *   Wp [ceil(N/128)*128][Kp]         Wp[n][k] = W[n][col_map[k]] (0 if map < 0 or n >= N)
 *   Wt [ceil(Kp/128)*128 + 128][ldwt] Wt[k][n] = Wp[n][k] for n < N, 0 otherwise,
 *                                    ldwt = ceil(N/32)*32 (the extra 128 zero
 *                                    rows let any 32-aligned row window of Wt
 *                                    be used as a 128-row-tiled B operand).
 * Either output may be NULL. */
int nerf_pack_weight(const float* W, int32_t N, int32_t K_orig, const int32_t* col_map,
                     int32_t Kp, float* Wp, float* Wt, int32_t ldwt, void* stream);

/* ---------------------------------------------------------------------------
 * Split-precision variants ("3 x bf16"): same contracts as the fp32 entry points,
 * each product formed as lo*hi + hi*lo + hi*hi on bf16 MFMA with fp32
 * accumulation (x = hi + lo, hi = bf16(x), lo = bf16(x - hi)): ~2^-17 relative
 * error per product at 5.3x the fp32 MFMA rate.  Selected by the host when
 * torch.get_float32_matmul_precision() != "highest" (the reference sets "high",
 * barf/run_barf.py:101).  Weights are pre-split by nerf_pack_weight_x3 into an
 * interleaved layout of the fp32 packed matrices: element (r, c) of a [rows][ld]
 * matrix is stored at Wx[r][c/32][c%32] (hi) and Wx[r][c/32][32 + c%32] (lo), so
 * every 32-column chunk of a row is 128 contiguous bytes (ld % 32 == 0; Wp_x has
 * ceil(N/128)*128 rows of ld = Kp, Wt_x has ceil(Kp/128)*128 + 128 rows of ld = ldwt).
 * 32 < N <= 256 runs a 256-row tile staged by LDS-DMA; other N a 128 x 128 tile.
 * nerf_linear_wgrad_x3 writes the same workspace as nerf_linear_wgrad (reduce with
 * nerf_linear_wgrad_reduce, same M, K and N rounded up to 4); its N may be the true row count
 * (ld_dy >= pad4(N)): N <= 257 with N or K above 128 and K <= 256 runs as one 256 x 256 tile
 * per M split, row 256 on the vector ALUs in fp32.
 * passes (ABI 10): 3 = the 3 x bf16 split products (matmul precision "high"), 1 = one bf16 pass
 * bf16(dY) * bf16(X) with fp32 accumulation ("medium", as NERF_FUSED_BF16).
 * ------------------------------------------------------------------------- */
int nerf_linear_fwd_x3(const nerf_seg* segs, int32_t n_segs, int64_t M,
                       const void* W_x, int32_t ldw, int32_t N, const float* bias,
                       float* out, int64_t ldo, int32_t epilogue,
                       const float* aux, int64_t ld_aux, void* stream);
int nerf_linear_wgrad_x3(const float* dY, int64_t ld_dy, int32_t N,
                         const nerf_seg* segs, int32_t n_segs, int64_t M,
                         void* workspace, size_t workspace_bytes, int32_t passes, void* stream);
/* The same over two blocks of rows summed into one gradient (the two passes of a field used
 * twice per step: one launch and one reduce instead of two each): rows [0, M0) of (dY, segs),
 * then rows [0, M1) of (dY1, segs1), whose segments have the same widths; workspace and reduce
 * for M = M0 + M1.  M1 = 0: nerf_linear_wgrad_x3. */
int nerf_linear_wgrad_x3_rows(const float* dY, int64_t ld_dy, const nerf_seg* segs, int64_t M0,
                              const float* dY1, int64_t ld_dy1, const nerf_seg* segs1, int64_t M1,
                              int32_t n_segs, int32_t N, void* workspace, size_t workspace_bytes,
                              int32_t passes, void* stream);
/* nerf_linear_wgrad_x3_rows that also writes the per-ray sums of dY, raysum[ray][n] (n < N; rays of
 * samples_per_ray0 rows in block 0, then of samples_per_ray1 rows in block 1), from the streamed
 * single-tile kernel (N <= 256, 128 < N or 128 < K <= 256; 16 <= S <= 128 with S | 128, M0 % 128 = 0).
 * A layer input that is per ray (the direction encoding of NerfModel's colour layer, row divisor S)
 * then takes its weight gradient from the B rays instead of the M samples: sum_m dY[m] x[ray(m)] =
 * sum_ray raysum[ray] x[ray] (barf/model_interpolation_architecture.py:88-92, 132-135). */
int nerf_linear_wgrad_x3_rays(const float* dY, int64_t ld_dy, const nerf_seg* segs, int64_t M0,
                              const float* dY1, int64_t ld_dy1, const nerf_seg* segs1, int64_t M1,
                              int32_t n_segs, int32_t N, void* workspace, size_t workspace_bytes,
                              float* raysum, int32_t samples_per_ray0, int32_t samples_per_ray1,
                              int32_t passes, void* stream);
int nerf_pack_weight_x3(const float* W, int32_t N, int32_t K_orig, const int32_t* col_map,
                        int32_t Kp, void* Wp_x, void* Wt_x, int32_t ldwt, void* stream);

/* ---------------------------------------------------------------------------
 * Fused field-MLP forward (a7: NerfModel.forward, barf/model_interpolation_architecture.py:96-141,
 * every Linear + bias + ReLU of the network in ONE launch, split precision as above).
 *
 * A workgroup of 8 waves owns 128 samples, a wave 16 of them, whose activations stay in
 * registers from layer to layer (the B operand of v_mfma_f32_16x16x32_bf16, bf16 hi/lo): only
 * the HBM-fed inputs are read and only the outputs the backward needs are written.  Weights
 * stream through LDS by LDS-DMA in "chunks" (16 output rows of one layer: its 32-deep k-blocks as
 * ready-to-use MFMA fragments, 2 KB each), all packed into one image by nerf_fused_pack together
 * with the biases.  Layer l's input is [previous layer's output (kbr 32-wide blocks, none for the
 * first layer) | up to 2 HBM-fed segments (kbh blocks in all)]; type = 3*(kbr/4) + kbh with kbr in
 * {0, 4, 8}, kbh in {0, 1, 2}.  A segment is read from seg_ptr, or GENERATED in-kernel
 * (seg_gen): the position encoding of the samples o + tq d of rays, or the encoding of the
 * rays' directions, exactly as nerf_encode_fwd computes them (the first layer reading it also
 * stores the rows for the weight gradients).  out[m, n] for n < ldo (columns >= N are written as
 * 0), ReLU mask bits in the NERF_FUSED_MASK layout (N <= 256), column col_idx (a multiple of 32)
 * additionally into col_out[m].  Buffers: byte extents < 2^31.
 * The same launch runs the input-gradient chain of the backward (layers in reverse, images of
 * W^T, no bias, mask_in instead of ReLU): each step's output is the previous layer's
 * pre-activation gradient, kept in registers for the next step and stored for the weight gradients.
 * ------------------------------------------------------------------------- */
/* NERF_FUSED_MASK: row m of a fused mask buffer is 8 uint32 words at (char*)mask + 32 m; column
 * n = 16 c + 4 g + r (c < 16, g, r < 4) is bit 4 (7 - (c & 7)) + r of word 2 g + (c >> 3) (each
 * MFMA lane's own bits: the forward sets them and the chain reads them with no cross-lane step).
 * A set bit marks a dead unit: !(out > 0).  It is not the NERF_EPI_MASKOUT layout (set bit =
 * out > 0, other positions) of the layer-by-layer kernels. */
#define NERF_FUSED_MAX_LAYERS 16
typedef struct nerf_fused_layer {
    int32_t type;          /* 3*(kbr/4) + kbh */
    int32_t N;             /* output columns */
    int32_t nb;            /* ceil(N / 32), <= 16 (chunks >= 8 are written, never fed forward) */
    int32_t relu;
    int32_t nseg;          /* HBM segments, 0..2 */
    int32_t seg_kb[2];     /* 32-column blocks of each segment (sum = kbh) */
    int32_t seg_k[2];      /* valid columns of each segment (multiple of 4; the rest reads 0) */
    int32_t seg_rd[2];     /* row divisor (row m reads row m / rd) */
    int32_t seg_rows[2];   /* rows of each segment buffer */
    int32_t chunk_units;   /* 1 KB units per chunk = 4*(kbr + kbh) */
    int32_t col_idx;       /* -1 or the column copied to col_out */
    int64_t seg_ld[2];
    const float* seg_ptr[2];
    float* out;            /* [M][ldo] fp32; NULL with ldo 0 drops the layer's stores */
    int64_t ldo;
    uint8_t* mask;         /* [M][32] ReLU bits (NERF_FUSED_MASK) or NULL */
    float* col_out;        /* [M] or NULL */
    int64_t img_off;       /* byte offset of the layer's first chunk in the image */
    int64_t bias_off;      /* byte offset of the layer's [nb][32] fp32 biases in the image */
    const uint8_t* mask_in;/* NULL, or [M][32] ReLU bits (NERF_FUSED_MASK layout) multiplied into the
                              output (the input-gradient chain: dL/dz_{l-1} = (dL/dz_l W_l) * (z_{l-1} > 0)) */
    float* out2;           /* chunks >= n1 (input-gradient chain: the rows of an encoding input) go to
                              out2[m, 32 (chunk - n1) + ...] (row stride ldo2), unmasked, not fed forward */
    int64_t ldo2;
    int32_t n1;            /* chunks written to out (= nb when out2 is unused) */
    int32_t hbm_off;       /* byte offset of the layer's HBM-fed weight fragments in the image */
    int32_t seg_gen[2];    /* 0: segment s is read from seg_ptr; 1 + e (first layer, one segment):
                              the rows of encodings[e] generated at the tile start, read from LDS;
                              3 / 4 (input-gradient chain): the composite's head / density gradient
                              from its coefficient rows (nerf_mlp_fused_render) */
} nerf_fused_layer;

/* An encoding generated inside the fused forward: every entry with out_dim > 0 is computed at the
 * start of each 128-sample tile (exactly as nerf_encode_fwd computes it) and its rows are stored
 * to out (required), where later layers (seg_ptr = out) and the weight gradients read them; the
 * first layer may take them straight from LDS (seg_gen).
 * params.kind 2 (ABI 8): the multiresolution hash-grid features of ray-mode positions, exactly as
 * nerf_hashgrid_fwd computes them (out_dim = levels * features <= 64, levels <= 16, features 1, 2
 * or 4; params.query as hash->query): `hash` points to the host-side parameters (copied at the
 * launch), `hash_table` to the packed device table; at most one kind-2 entry per launch. */
struct nerf_hashgrid_params;
typedef struct nerf_fused_encoding {
    nerf_pe_params params;     /* as nerf_encode_fwd takes it (ray mode: query, pw_mode) */
    const float* ray_o;        /* [n_rays][3] */
    const float* ray_d;        /* [n_rays][3] */
    const float* t_start;      /* [M] (position encodings) */
    const float* t_end;        /* [M] (midpoint queries, IPE) */
    const float* pixel_width;  /* IPE, addressed by params.pw_mode */
    float* out;                /* the rows: [M][ld], or [n_rays][ld] when per_ray (ld <= 64) */
    int64_t ld;
    int64_t n_rays;
    int32_t samples_per_ray;   /* sample m belongs to ray m / samples_per_ray */
    int32_t per_ray;           /* 0: position encoding of o + tq d; 1: encoding of the ray direction */
    int32_t out_dim;           /* encoding columns (the rest of a 32-column block reads 0) */
    int32_t reserved;
    const struct nerf_hashgrid_params* hash;  /* kind 2: host pointer, read at the launch */
    const float* hash_table;   /* kind 2: [sum_l rows_l][features] device table */
} nerf_fused_encoding;

/* encodings: NULL, or 2 entries (generated segments index them) */
int nerf_mlp_fused_fwd(const nerf_fused_layer* layers, int32_t n_layers, const void* image, int64_t M,
                       const nerf_fused_encoding* encodings, void* stream);

/* Alpha compositing fused into the field MLP (a4 inside a7: barf/model_interpolation.py:316-353 on
 * the heads of model_interpolation_architecture.py:128-141, replacing nerf_composite_fwd/bwd with
 * act = 1 for rays whose samples fill whole 128-sample tiles: 128 % S == 0, 16 <= S <= 128, with
 * 128 / S rays per tile, or S == 256, one ray per two tiles that one workgroup runs back to back;
 * M = n_rays * S).
 *
 * Forward (the forward launch): at the end of every tile the waves hand their samples' raw heads
 * (rgb = rows 0..2 of layer head_layer, which has one 16-row chunk; sigma = the column output of
 * sigma_layer, or row 3 of the head layer when sigma_layer < 0) to one wave per ray through LDS,
 * which composites the ray exactly as nerf_composite_fwd (the same instructions: rgb and weights
 * bitwise equal) and writes rgb[ray][3], weights[n] (or not, NULL) and the backward's per-sample
 * coefficients coef[n][8] (or not, NULL):
 *   coef[n][0..2] = dL/d rgb-raw_n,ch per unit grad_rgb_ch = w_n * c_n,ch * (1 - c_n,ch)
 *   coef[n][4..6] = dL/d sigma-raw_n per unit grad_rgb_ch
 *                 = -(((A_n,ch * sb) * sa) * delta_n) * softplus'(raw - shift),
 *     A_n,ch = (-c_n,ch T_n e^{b_n}) + sum_{i > n} c_i,ch w_i   (fp64 suffix sums), [3], [7] = 0,
 * so that the backward of the compositing is linear in grad_rgb per sample: no scan.
 * Input-gradient chain (the chain launch, grad_rgb != NULL): a step whose HBM segment has seg_gen 3
 * takes, per sample, [g_0 coef0, g_1 coef1, g_2 coef2, sigma_layer < 0 ? <g, coef4..6> : 0]
 * (g = grad_rgb of the sample's ray; seg_ptr = coef, seg_ld = seg_k = 8) as its input rows and
 * stores them to grad_head[n * ld_head + 0..3] (the head layer's dY for its weight gradient); seg_gen
 * 4 takes [<g, coef4..6>, 0, 0, 0] (the density column) and stores it to grad_sigma[n * ld_sigma +
 * 0..3] (the density layer's dY columns 256..259).  The weights output is non-differentiable
 * (the renderer only resamples from it). */
typedef struct nerf_fused_composite {
    const float* dist;         /* forward: [M] interval lengths t_end - t_start */
    float* rgb;                /* forward: [n_rays][3] */
    float* weights;            /* forward: [M] or NULL */
    float* coef;               /* forward: [M][8] backward coefficients or NULL */
    const float* grad_rgb;     /* chain: [n_rays][3] */
    float* grad_head;          /* chain: seg_gen 3 rows, or NULL */
    int64_t ld_head;
    float* grad_sigma;         /* chain: seg_gen 4 rows (16-B aligned), or NULL */
    int64_t ld_sigma;
    int32_t samples_per_ray;
    int32_t head_layer;        /* forward: the layer whose rows 0..2 (3) are the raw rgb (sigma) */
    int32_t sigma_layer;       /* the layer whose column output is the raw density, or -1 (head row 3) */
    float scale_a, scale_b;    /* density factor (reference: 3 * MAGIC_NUMBER) */
    float density_shift;       /* sigma = softplus(raw - shift, threshold 8), c = sigmoid(raw) */
    int32_t reserved;
} nerf_fused_composite;

/* nerf_mlp_fused_fwd with compositing fused in (composite: NULL = nerf_mlp_fused_fwd). */
int nerf_mlp_fused_render(const nerf_fused_layer* layers, int32_t n_layers, const void* image, int64_t M,
                          const nerf_fused_encoding* encodings, const nerf_fused_composite* composite,
                          void* stream);

/* nerf_mlp_fused_render with flags (ABI 10).  NERF_FUSED_BF16: every product in one bf16 pass
 * (bf16(w) * bf16(x), fp32 accumulate: matmul precision "medium", the single-pass products of the
 * reference's naive-to-vanilla/main.py:53,58 "medium" / 16-mixed C2 configuration) instead of the
 * 3 x bf16 split (hi*hi + hi*lo + lo*hi, ~2^-17 per product).  Same image, descriptors and outputs. */
#define NERF_FUSED_BF16 1
int nerf_mlp_fused_run(const nerf_fused_layer* layers, int32_t n_layers, const void* image, int64_t M,
                       const nerf_fused_encoding* encodings, const nerf_fused_composite* composite, int32_t flags,
                       void* stream);

/* Gather + split packer for the fused image: for i < n, v = srcs[map_src[i] >> 24][map_src[i] & 0xffffff]
 * (0 if map_src[i] < 0); map_dst[i] >= 0: bf16 element index of hi = bf16(v) (lo = bf16(v - hi)
 * at +512 elements); map_dst[i] < 0: fp32 word ~map_dst[i] = v.  Up to 64 sources. */
#define NERF_FUSED_MAX_SRCS 64
int nerf_fused_pack(const float* const* srcs, int32_t n_srcs, const int32_t* map_src, const int32_t* map_dst,
                    int64_t n, void* image, void* stream);

/* ---------------------------------------------------------------------------
 * Gaussian activation with a learnable per-channel inverse standard deviation (a8, GARF
 * field MLPs): GaussActivation / GaussAct, garf/gaussian.py:8-63 (copy: barf/gaussian.py).
 * v_n = inv_std_n^2 + 1e-6;  y[m,n] = exp((-(z*z)) * v_n)  over z [M][N] (row stride ld_z).
 * Backward: ge = grad_y * exp((-(z*z)) * v);  grad_z = (((-ge) * 2) * z) * v (grad_z may
 * alias grad_y);  grad_inv_std_n = (sum_m (-ge) * z^2) * (2 * inv_std_n), the column sum
 * accumulated in fp64 per slab of rows and the slabs summed in a fixed order (deterministic).
 * workspace: nerf_gauss_act_workspace(M, N) bytes.  accumulate: grad_inv_std += result.
 * ------------------------------------------------------------------------- */
size_t nerf_gauss_act_workspace(int64_t M, int32_t N);

/* Split-precision linear layer with the Gaussian activation in its epilogue (no separate
 * activation pass over HBM).  inv_std [N]; v_n = inv_std_n^2 + 1e-6; every element formula and
 * rounding as nerf_gauss_act_fwd / _bwd.
 *   mode NERF_GAUSS_FWD: z = A W^T + bias -> out (the pre-activation the backward needs) and
 *     y = exp((-(z*z)) * v) -> y (row stride ld_y).  grad_inv_std / workspace unused.
 *   mode NERF_GAUSS_BWD: g = A W^T (the gradient w.r.t. this layer's activation, bias must be
 *     NULL); z = this layer's pre-activation (row stride ld_z); out = grad_z = (((-ge)*2)*z)*v
 *     with ge = g * exp((-(z*z)) * v); grad_inv_std_n (+)= (sum_m (-ge) z^2) * (2 inv_std_n),
 *     the column sums formed per row tile in fp64 in a fixed order and the tiles summed in a
 *     fixed order (deterministic).  workspace: nerf_linear_gauss_workspace(M, N) bytes.
 * Requires N % 4 == 0, 16-byte aligned out / y / z / bias rows (row strides multiples of 4);
 * returns NERF_ERR_UNSUPPORTED otherwise (callers then use nerf_linear_fwd_x3 +
 * nerf_gauss_act_fwd / _bwd). */
#define NERF_GAUSS_FWD 0
#define NERF_GAUSS_BWD 1
size_t nerf_linear_gauss_workspace(int64_t M, int32_t N);
int nerf_linear_gauss_x3(const nerf_seg* segs, int32_t n_segs, int64_t M, const void* W_x, int32_t ldw,
                         int32_t N, const float* bias, float* out, int64_t ldo, int32_t mode,
                         const float* inv_std, float* y, int64_t ld_y, const float* z, int64_t ld_z,
                         float* grad_inv_std, int32_t accumulate, void* workspace, size_t workspace_bytes,
                         void* stream);
int nerf_gauss_act_fwd(const float* z, int64_t ld_z, const float* inv_std, int64_t M, int32_t N,
                       float* y, int64_t ld_y, void* stream);
int nerf_gauss_act_bwd(const float* grad_y, int64_t ld_g, const float* z, int64_t ld_z,
                       const float* inv_std, int64_t M, int32_t N, float* grad_z, int64_t ld_dz,
                       float* grad_inv_std, int32_t accumulate, void* workspace, size_t workspace_bytes,
                       void* stream);

/* ---------------------------------------------------------------------------
 * Fused Adam step (the optimizer of every reference experiment: torch.optim.Adam(eps=1e-5),
 * barf/model_interpolation.py:543-584) for up to NERF_ADAM_MAX_TENSORS tensors in ONE launch.
 * Per element, in torch's fp32 operation order:
 *   g = grad (+ weight_decay*param);  m = m + (1-beta1)*(g-m);  v = v*beta2 + ((1-beta2)*g)*g;
 *   param = param + step_size*(m / (sqrt(v)/bc2_sqrt + eps)),
 * step_size = -lr/(1-beta1^t), bc2_sqrt = sqrt(1-beta2^t) (host scalars per tensor).  The
 * table is copied by value into the kernel arguments: no device table, no copy per step.
 * ------------------------------------------------------------------------- */
#define NERF_ADAM_MAX_TENSORS 48
typedef struct nerf_adam_batch {
    int32_t n_tensors;
    float beta1, beta2, eps;
    float one_minus_beta1, one_minus_beta2;   /* 1 - beta as the host forms it (double -> fp32) */
    float* param[NERF_ADAM_MAX_TENSORS];
    const float* grad[NERF_ADAM_MAX_TENSORS];
    float* exp_avg[NERF_ADAM_MAX_TENSORS];
    float* exp_avg_sq[NERF_ADAM_MAX_TENSORS];
    int64_t numel[NERF_ADAM_MAX_TENSORS];
    float step_size[NERF_ADAM_MAX_TENSORS];
    float bc2_sqrt[NERF_ADAM_MAX_TENSORS];
    float weight_decay[NERF_ADAM_MAX_TENSORS];
} nerf_adam_batch;
int nerf_adam_step(const nerf_adam_batch* batch, void* stream);

/* ---------------------------------------------------------------------------
 * On-device training-batch feed.  Replaces, for one batch of dataset
 * indices, ImagePoseDataset.__getitem__ (barf/dataset.py:613-637) over the dataset's
 * precomputed rays (_get_directions_meshgrid :417-451, _meshgrid_to_world :453-481,
 * _apply_noise :512-557), the DataLoader's collation, and
 * ImagePoseDataModule.get_blurred_pixel_colors (barf/data_module.py:276-367).
 *   indices [B] int64: dataset index = image * H*W + row * W + col (the sampler's order)
 *   c2w [n_img][4][4]; noise_rot [n_img][3][3] / noise_trans [n_img][3] or NULL
 *   images [n_img][H][W][n_sigma][3] fp32 (blur levels, most blurred first)
 * Outputs ([B][3] unless noted; NULL skips): o_raw, d_raw, o_noisy + d_noisy (together),
 * colors_raw [B][n_sigma][3], colors_pair [B][2][3] = (blurred, original) with
 * blur_mode 1: (last, last), 2: (level 0, last), 3: (level lo * coef_lo + level hi * coef_hi,
 * last); img_idx [B] int64.  status (device int32, caller-zeroed): bit 0 = an index was out
 * of range (that ray reads index 0).
 * ------------------------------------------------------------------------- */
int nerf_ray_batch(const int64_t* indices, int64_t B, int32_t H, int32_t W, float focal,
                   const float* c2w, const float* noise_rot, const float* noise_trans, int32_t n_img,
                   const float* images, int32_t n_sigma, int32_t blur_mode, int32_t blur_lo, int32_t blur_hi,
                   float coef_lo, float coef_hi, float* o_raw, float* o_noisy, float* d_raw, float* d_noisy,
                   float* colors_raw, float* colors_pair, int64_t* img_idx, int32_t* status, void* stream);

/* ---------------------------------------------------------------------------
 * Multiresolution hash-grid encoding (a9, config C5): INGPTable.forward / INGPEncoding.forward,
 * 3d-ingp/model.py:14-121 (interface per VERDICT r2; arithmetic per SURVEY.md §8(a) a9, its 2-D
 * statement 2d-ingp/model.py:13-115 pinned by tests/golden/hashgrid2d.npz).
 * Level l has resolution res[l] and its own table of rows_l = (r+1)^3 rows when bijective
 * ((r+1)^3 <= table_size) and table_size rows otherwise; the levels' tables are packed back to
 * back, table = [sum_l rows_l][features] fp32 (nerf_hashgrid_table_rows).
 * Per level: x_hat = (x / 8 + 0.5) * r (normalize = 1, INGPEncoding) or x * r (normalize = 0,
 * INGPTable on normalised points); corners floor(x_hat) + {0,1}^3 in the reference's stacking order
 * (0,0,0), (0,0,1), (0,1,0), ..., (1,1,1) (z fastest); row = x + (r+1) y + (r+1)^2 z of the corner
 * clipped to [0, r] when bijective, else ((x*pi1) ^ (y*pi2) ^ (z*pi3)) mod table_size in 64-bit
 * integers (wrapping products, non-negative remainder); weight prod_d (1 - |x_hat_d - corner_d|)
 * on the unclipped corner; out[n, l*F + f] = sum over the corners in that order of
 * w * table[level l][row][f] (products rounded, then added).
 * Positions: x [n][3], or (x == NULL) o[ray] + tq * d[ray] with ray = n / samples_per_ray and
 * tq = t_start[n] (query 0) or (t_start[n] + t_end[n]) / 2 (query 1).
 * ------------------------------------------------------------------------- */
#define NERF_HASHGRID_MAX_LEVELS 32
#define NERF_HASHGRID_MAX_FEATURES 8
typedef struct nerf_hashgrid_params {
    int32_t levels;
    int32_t table_size;
    int32_t features;
    int32_t query;
    int32_t normalize;          /* 1: x / 8 + 0.5 first (INGPEncoding); 0: points already in [0, 1) */
    int32_t reserved;
    int64_t primes[3];          /* pi1, pi2, pi3 (the reference's defaults 1, 2654435761, 805459861) */
    int32_t res[NERF_HASHGRID_MAX_LEVELS];
} nerf_hashgrid_params;

/* Rows of level `level`'s table, or of the whole packed table when level < 0 (-1 on bad params). */
int64_t nerf_hashgrid_table_rows(const nerf_hashgrid_params* params, int32_t level);

int nerf_hashgrid_fwd(const nerf_hashgrid_params* params, const float* x, const float* ray_o,
                      const float* ray_d, const float* t_start, const float* t_end, int64_t n_samples,
                      int32_t samples_per_ray, const float* table, float* out, int64_t out_ld, void* stream);

/* Gradient of sum(out * grad_out) w.r.t. the packed table (positions get none): every
 * contribution w * g rounded to a 64-bit fixed-point grid 2^-s chosen from the batch's max |g| (no
 * entry can overflow) and added with integer atomics, so the result does not depend on their order
 * (deterministic); then grad_table = acc * 2^-s (+= if accumulate).  A non-finite grad_out gives
 * NaN.  workspace: nerf_hashgrid_workspace(params) bytes, 256-byte aligned; zeroed by the call
 * itself (no state is carried between calls). */
size_t nerf_hashgrid_workspace(const nerf_hashgrid_params* params);
/* (ABI 8) workspace for n_samples: nerf_hashgrid_workspace(params) rounded up to 256 bytes, room for
 * grad_out restaged level-major (n_samples * levels * features fp32) and per-sample position
 * records, and the buckets of the hashed levels' corner contributions (about 12 B x 8 corners x
 * 1.25 per (sample, hashed level): ~2.1 GB for 1.31 M samples x 13 hashed levels).  With a workspace
 * of at least this size the call restages grad_out and takes the hashed levels through the bucketed
 * passes (NERF_HG_BUCKET, default on); with only nerf_hashgrid_workspace(params) bytes every level
 * is walked once per 160 KB part, reading the [n][g_ld] rows in place.  Same result either way
 * (bitwise: integer sums).  The bucketed passes take a hashed level of at most 64 parts of 80 KB
 * (table_size * features <= 64 * 10 240 entries: T <= 327 680 at F = 2, so not the 2^19 tables of
 * instant-ngp); a larger table takes the per-part walk for every level, with the same result.
 * With 8-byte packed entries (the default whenever the sample index and row fit 32 bits) the
 * buckets need two 4-byte arrays' room, not three. */
size_t nerf_hashgrid_workspace_n(const nerf_hashgrid_params* params, int64_t n_samples);
int nerf_hashgrid_bwd(const nerf_hashgrid_params* params, const float* x, const float* ray_o,
                      const float* ray_d, const float* t_start, const float* t_end, int64_t n_samples,
                      int32_t samples_per_ray, const float* grad_out, int64_t g_ld, float* grad_table,
                      int32_t accumulate, void* workspace, size_t workspace_bytes, void* stream);
/* (ABI 9) Gradient of sum(out * grad_out) w.r.t. the positions, through the multilinear weights
 * (w_k = prod_d (1 - |x_hat_d - c_kd|) on the unclipped corner, x_hat = (p / 8 + 0.5) r, or p r
 * unnormalised; torch's abs backward: sign(0) = 0; corners and rows are constants of p):
 *   dL/dp_d = sum_l ((sum_k G_lk (-sign(x_hat_d - c_kd)) prod_{e != d} (1 - |x_hat_e - c_ke|)) r_l) / 8,
 * G_lk = sum_f grad_out[n][l F + f] table[l][row_k][f], levels and corners in order (deterministic).
 * x != NULL: grad_x [n][3] (ray pointers NULL).  Ray form (x == NULL, samples p = o + t_q d,
 * n_samples a multiple of samples_per_ray): grad_o / grad_d [n_rays][3] (either may be NULL) =
 * sum over each ray's samples of dL/dp / of t_q dL/dp; workspace >= n_samples * 12 bytes, 16-byte
 * aligned.  accumulate: += into the outputs. */
int nerf_hashgrid_bwd_pos(const nerf_hashgrid_params* params, const float* x, const float* ray_o,
                          const float* ray_d, const float* t_start, const float* t_end, int64_t n_samples,
                          int32_t samples_per_ray, const float* table, const float* grad_out, int64_t g_ld,
                          float* grad_x, float* grad_o, float* grad_d, int32_t accumulate, void* workspace,
                          size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * Camera-pose alignment: CameraCalibrationModel.kabsch_algorithm
 * (barf/model_camera_calibration.py:69-156) and compute_pose_error (:340-345).
 * from, to: [n][3] fp32 device points, 3 <= n <= NERF_KABSCH_MAX_POINTS.  Writes R [3][3]
 * (row-major), t [3], c [1] with R from_i c + t ~ to_i: centred clouds, c = |to_c| / |from_c|,
 * R from the SVD of from_c^T to_c with the reflection fix on the smallest singular value,
 * t = mean_to - c R mean_from.  remove_outliers: keep the points whose aligned distance is below
 * the 0.9 quantile (torch.quantile's linear interpolation) and solve again.  err (optional):
 * mean_i |to_i - (R from_i c + t)| over all n points — compute_pose_error with from = predicted
 * and to = raw camera origins.  One workgroup, fp64 fixed-order sums (deterministic).
 * ------------------------------------------------------------------------- */
#define NERF_KABSCH_MAX_POINTS 4096

/* ---------------------------------------------------------------------------
 * Proposal-network sampling and interlevel loss: nerfacc's
 * PropNetEstimator.sampling / compute_loss as GARF calls them (garf/model_garf.py:81,210-230,257).
 * nerfacc is not vendored (environment.yml:26, unpinned): restated from its published algorithm,
 * parity unpinned.  One wave per ray; rows of at most NERF_PROP_MAX_EDGES edges.
 *
 * nerf_prop_cdf: cdf [R][K+1] of weights w [R][K]: cdf[0] = 0, cdf[i] = sum_{j<i} w[j] (fp64),
 *   cdf[K] = 1 — nerfacc's 1 - [trans, 0] with trans = 1 - the exclusive weight sum.
 * nerf_prop_sample: n intervals (n + 1 edges) per ray by inverting the piecewise-linear cdf over
 *   the ray's edges vals [R][K+1] (s-space, increasing) at u_0 = 0, u_n = 1 and u_i = i/n, or
 *   (i - 1/2 + U_i)/n when stratified (Philox(seed, counter)); s_out = the s edges, t_out =
 *   transform(s): 0 uniform t = s far + (1-s) near, 1 lindisp 1/t = s/far + (1-s)/near.
 * nerf_prop_loss: interlevel loss between query intervals (q_vals, q_cdf [R][n+1], no gradient)
 *   and key intervals (k_vals, k_cdf [R][K+1]): per query interval j, w = q_cdf[j+1] - q_cdf[j],
 *   w_outer = k_cdf[right(q_vals[j+1])] - k_cdf[left(q_vals[j])] (right = #k_vals <= x clamped to
 *   K, left = that - 1 clamped to 0), loss_j = max(w - w_outer, 0)^2 / (w + eps).  loss_ray [R]
 *   (optional) = sum_j loss_j (fp64, fixed order).  grad_k_w (optional) [R][K] = d(grad_scale *
 *   sum loss) / d key weights (k_cdf as nerf_prop_cdf forms it), gathered in a fixed order.
 * ------------------------------------------------------------------------- */
#define NERF_PROP_MAX_EDGES 512
int nerf_prop_cdf(const float* w, int64_t ld_w, int64_t n_rays, int32_t K, float* cdf, int64_t ld_cdf,
                  void* stream);
int nerf_prop_sample(const float* vals, int64_t ld_vals, const float* cdf, int64_t ld_cdf, int64_t n_rays,
                     int32_t K, int32_t n, int32_t stratified, uint64_t seed, uint64_t counter, int32_t transform,
                     float near_plane, float far_plane, float* s_out, float* t_out, int64_t ld_out, void* stream);
int nerf_prop_loss(const float* q_vals, const float* q_cdf, int64_t ld_q, const float* k_vals, const float* k_cdf,
                   int64_t ld_k, int64_t n_rays, int32_t n, int32_t K, float eps, float* loss_ray,
                   float grad_scale, float* grad_k_w, int64_t ld_gw, void* stream);
int nerf_kabsch(const float* from, const float* to, int32_t n, int32_t remove_outliers, float* R, float* t,
                float* c, float* err, void* stream);

/* ---------------------------------------------------------------------------
 * BARF camera refinement in front of the ray path:
 * CameraExtrinsics.forward (barf/model_camera_extrinsics.py:61-85, so3_to_SO3 :23-43).
 * Replaces the torch chain matrix_exp([rotation]_x) -> [img_idx] gather -> R @ d, o + t / MAGIC
 * and its autograd backward (index_add + matrix_exp's block-matrix backward).
 *
 * nerf_pose_rays_fwd: rotation, translation [n_images][3] (so3 / translation parameters),
 *   img_idx [n_rays] int64, o, d [n_rays][3].  Writes new_o = o + translation[i] / magic,
 *   new_d = R_i d (R_i = exp of the skew matrix of rotation[i], Rodrigues in fp64 rounded to fp32),
 *   and optionally R [n_rays][3][3] (row-major) and t [n_rays][3] = translation[i] / magic.
 *   An out-of-range image index yields NaN outputs for that ray.
 * nerf_pose_rays_bwd: gradients of the per-ray outputs (g_new_o, g_new_d, g_R, g_t; any may be
 *   NULL = zero) to g_rotation, g_translation [n_images][3] (overwritten; zero for images without
 *   rays).  One workgroup per image, fixed-order fp64 sums, the analytic derivative of Rodrigues'
 *   formula: deterministic.  ray_order / image_start (both NULL, or both set): the rays bucketed by
 *   image — ray_order [n_rays] the ray indices stably sorted by img_idx, image_start [n_images + 1]
 *   the first position of each image in it — so each workgroup reads only its own rays (O(n_rays)
 *   work instead of O(n_images * n_rays)); without them every workgroup tests every ray's index.
 * ------------------------------------------------------------------------- */
int nerf_pose_rays_fwd(const float* rotation, const float* translation, int32_t n_images, const int64_t* img_idx,
                       const float* o, const float* d, int64_t n_rays, float magic, float* new_o, float* new_d,
                       float* R, float* t, void* stream);
int nerf_pose_rays_bwd(const float* rotation, int32_t n_images, const int64_t* img_idx, const float* d,
                       int64_t n_rays, float magic, const float* g_new_o, const float* g_new_d, const float* g_R,
                       const float* g_t, const int64_t* ray_order, const int64_t* image_start, float* g_rotation,
                       float* g_translation, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* NERF_AMD_H */
