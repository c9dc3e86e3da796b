// Positional encodings fused with sample-position generation.
//
// References (barf/positional_encodings.py):
//   FourierFeatures.forward              :42-57   args = x.repeat_interleave(L) * (scale*2^k)
//   BarfPositionalEncoding.compute_mask  :105-122 (mask values are computed on the host from
//                                                   the alpha scalar and passed in: no int(alpha) sync)
//   BarfPositionalEncoding.forward       :124-148 [x | mask*cos | mask*sin]
//   IntegratedFourierFeatures.forward    :170-240 (mip-NeRF IPE)
//   IntegratedBarfFourierFeatures        :266-282
//   NerfInterpolation._compute_positions barf/model_interpolation.py:288-312 (o + t*d)
//
// Design: the forward is an HBM-store-bound kernel (≈250 B written per sample vs ≈8 B
// read).  Rows of <= 128 columns go through encode_fwd_lds_kernel: 64 samples per block,
// positions computed once per sample, ONE sin/cos evaluation per (sample, d, k) feeding both
// the cos and the sin column, the row image staged in LDS and written with coalesced 16-byte
// stores.  sin/cos use sincos_enc (fp64 Cody-Waite reduction + fp32 minimax, ~1e-7 abs) —
// libm sincosf made the kernel VALU-bound.  Wider / unaligned rows: one thread per 4 columns.
// Floating-point contraction is off so every other fp32 operation rounds exactly where the
// reference's does.
#include <stddef.h>

#include "common.h"
#include "encode_common.h"

using namespace nerf;

namespace {

struct EncArgs {
    nerf_pe_params p;
    const float* x; const float* xdir;
    const float* o; const float* d;
    const float* t0; const float* t1; const float* pw;
    int64_t n; int S; int64_t n_rays;
    float* out; int64_t ld;
    int out_dim;
    int vec;     // out 16-byte aligned and ld % 4 == 0: float4 stores
};

// One thread per 4 consecutive output columns (one 16-byte store) of one sample: the Q = ld/4
// threads of a row write it contiguously, rows_per_block = 256 / Q rows per block, so a wave
// stores 1 KB of consecutive rows per instruction.  The position (o + t d, or x), and for the
// integrated encoding the per-sample variance terms, are computed once per thread.
__global__ __launch_bounds__(256) void encode_fwd_kernel(EncArgs a, int Q, int RB) {
#pragma clang fp contract(off)
    const int t = threadIdx.x;
    const int rloc = t / Q;
    const int qd = t - rloc * Q;
    if (rloc >= RB) return;
    const int64_t n = (int64_t)blockIdx.x * RB + rloc;
    if (n >= a.n) return;
    const int L = a.p.levels;
    const int id = a.p.include_identity ? 3 : 0;
    float p[3], dv[3];
    load_pos_dir(a, n, p, dv);
    IpeSample q;
    const float* pm = p;
    if (a.p.kind == 1) {
        q = ipe_sample(a.p, p, dv, a.t0[n], a.t1[n], a.pw ? pixel_width_at(a, n) : 0.f);
        pm = q.pm;
    }
    const int c0 = 4 * qd;
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = (c0 + e < a.out_dim) ? enc_column(a.p, L, id, c0 + e, pm, q) : 0.0f;
    float* o = a.out + n * a.ld + c0;
    if (a.vec) {
        *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (c0 + e < a.ld) o[e] = v[e];
    }
}

// LDS-staged variant for rows of <= 128 columns (every encoding of the reference's configs):
// a block encodes 64 samples in three phases —
//   0. one thread per sample: position (and the IPE variance terms) into LDS, identity and
//      zero-pad columns into the row image;
//   1. one thread per (sample, d, k): ONE sincos per argument, writing both the cos and the sin
//      column (half the transcendental work of a per-column mapping);
//   2. the 64-row image leaves LDS as coalesced 16-byte stores (ld/4 consecutive lanes per row).
#ifndef NERF_ENC_ROWS
#define NERF_ENC_ROWS 64
#endif
#ifndef NERF_ENC_NT
#define NERF_ENC_NT 0
#endif
constexpr int kEncRows = NERF_ENC_ROWS;
constexpr int kEncMaxLd = 128;

// NERF_ENC_PERSIST=1: a grid of at most 8 blocks per CU walks the 64-row tiles instead of one tile
// per block — measured slower at a full 800 x 800 frame (2.62 vs 3.50 TB/s, profiles/r05e), and so
// was a barrier-free form with each wave encoding its own 16 rows in a private LDS image (2.70 TB/s,
// profiles/r05f): the dispatch of ~1 M short blocks does not pace this kernel
#ifndef NERF_ENC_PERSIST
#define NERF_ENC_PERSIST 0
#endif
__global__ __launch_bounds__(256) void encode_fwd_lds_kernel(EncArgs a) {
#pragma clang fp contract(off)
    extern __shared__ float img[];      // kEncRows x (ld + 4) floats (dynamic: sized to the row)
    __shared__ float spm[kEncRows][3];
    __shared__ float svb[kEncRows][3];
    const int t = threadIdx.x;
    const int L = a.p.levels;
    const int id = a.p.include_identity ? 3 : 0;
    const int ld = (int)a.ld;
    const int lds_ld = ld + 4;          // 16-byte aligned rows, staggered banks
    const int64_t ntiles = (a.n + kEncRows - 1) / kEncRows;
    const int tl = 3 * L;
    const int TPR = tl <= 32 ? 32 : 64;
    const int j = t & (TPR - 1);
    const int dd = j >= 2 * L ? 2 : (j >= L ? 1 : 0);
    const int k = j < tl ? j - dd * L : 0;                 // (threads past the tasks: unused)
    const float s = a.p.scale * (float)(1u << k);
    const float m = a.p.use_mask ? a.p.mask[k] : 1.0f;
    const float sc4 = (float)(1u << (2 * k));
    const int Q = ld >> 2;
    const bool pow2 = (Q & (Q - 1)) == 0;
    const int qsh = __builtin_ctz((unsigned)Q);
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += (NERF_ENC_PERSIST ? (int64_t)gridDim.x : ntiles)) {
        const int64_t n0 = tile * kEncRows;
        const int rows = a.n - n0 < kEncRows ? (int)(a.n - n0) : kEncRows;
        if (t < rows) {
            const int64_t n = n0 + t;
            float p[3], dv[3];
            load_pos_dir(a, n, p, dv);
            float* row = img + t * lds_ld;
            if (a.p.kind == 1) {
                const IpeSample q = ipe_sample(a.p, p, dv, a.t0[n], a.t1[n], a.pw ? pixel_width_at(a, n) : 0.f);
#pragma unroll
                for (int d = 0; d < 3; ++d) {
                    spm[t][d] = q.pm[d];
                    svb[t][d] = q.vb[d];
                }
            } else {
#pragma unroll
                for (int d = 0; d < 3; ++d) spm[t][d] = p[d];
            }
            for (int c = 0; c < id; ++c) row[c] = spm[t][c];
            for (int c = a.out_dim; c < ld; ++c) row[c] = 0.0f;
        }
        __syncthreads();
        // phase 1: thread t owns argument column j = t % TPR (fixed d, k, scale, mask for the whole
        // block) and walks the rows r = t / TPR, + 256/TPR, ...: no per-task index arithmetic
        if (j < tl) {
            for (int r = t / TPR; r < rows; r += 256 / TPR) {
                float sn, cs;
                sincos_enc(spm[r][dd] * s, &sn, &cs);
                if (a.p.kind == 1) {
                    const float w = expf((-(svb[r][dd] * sc4)) / 2.0f);
                    cs = cs * w;
                    sn = sn * w;
                }
                if (a.p.use_mask) {
                    cs = m * cs;
                    sn = m * sn;
                }
                float* row = img + r * lds_ld;
                row[id + j] = cs;
                row[id + tl + j] = sn;
            }
        }
        __syncthreads();
        const int stores = rows * Q;
        for (int i = t; i < stores; i += 256) {
            const int r = pow2 ? i >> qsh : i / Q;
            const int qd = i - r * Q;
#if NERF_ENC_NT
            typedef float f4v __attribute__((ext_vector_type(4)));
            const f4v v = *reinterpret_cast<const f4v*>(img + r * lds_ld + 4 * qd);
            __builtin_nontemporal_store(v, reinterpret_cast<f4v*>(a.out + (n0 + r) * a.ld + 4 * qd));
#else
            const float4 v = *reinterpret_cast<const float4*>(img + r * lds_ld + 4 * qd);
            *reinterpret_cast<float4*>(a.out + (n0 + r) * a.ld + 4 * qd) = v;
#endif
        }
        if (NERF_ENC_PERSIST) __syncthreads();      // the image is rewritten by the next tile
    }
}

// Gradient of one integrated-encoding row g w.r.t. the sample's position (gpm) and direction
// (gdd).  Used by the per-sample kernel below and by the per-ray kernel of nerf_encode_bwd_rays.
__device__ __forceinline__ void ipe_grad(const nerf_pe_params& p, const float pos[3], const float dv[3], float t0,
                                         float t1, float pwv, const float* gr, float gpm[3], float gdd[3]) {
#pragma clang fp contract(off)
    const int L = p.levels;
    const int id = p.include_identity ? 3 : 0;
    const IpeSample q = ipe_sample(p, pos, dv, t0, t1, pwv);
    float gvb[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        float apm = id ? gr[d] : 0.0f;
        float avb = 0.0f;
        for (int k = 0; k < L; ++k) {
            const float m = p.use_mask ? p.mask[k] : 1.0f;
            const float sc4 = (float)(1u << (2 * k));
            const float w = expf((-(q.vb[d] * sc4)) / 2.0f);
            const float s = p.scale * (float)(1u << k);
            float sn, cs;
            sincos_enc(q.pm[d] * s, &sn, &cs);
            const float gc = gr[id + d * L + k] * m;
            const float gs = gr[id + 3 * L + d * L + k] * m;
            apm += (((-gc) * sn + gs * cs) * w) * s;
            avb += ((gc * cs + gs * sn) * w) * (-(sc4 / 2.0f));
        }
        gpm[d] = apm;
        gvb[d] = avb;
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) gdd[j] = gpm[j] * q.mu_diff;
    if (!p.distribute_variance) {
        const float S = q.ssum;
        const float cross = ((gvb[0] * (dv[0] * dv[0]) + gvb[1] * (dv[1] * dv[1])) + gvb[2] * (dv[2] * dv[2])) *
                            ((2.0f * q.sr) / (S * S));
#pragma unroll
        for (int j = 0; j < 3; ++j)
            gdd[j] += (2.0f * dv[j]) * ((q.st - q.sr / S) * gvb[j]) + dv[j] * cross;
    }
}

// Gradient of one Fourier/BARF row g w.r.t. coordinate d of the position:
//   g_id + sum_k mask_k * s_k * (-g_cos * sin(a) + g_sin * cos(a))
__device__ __forceinline__ float fourier_grad(const nerf_pe_params& p, float xv, int dd, const float* gr) {
#pragma clang fp contract(off)
    const int L = p.levels;
    const int id = p.include_identity ? 3 : 0;
    float acc = id ? gr[dd] : 0.0f;
    for (int k = 0; k < L; ++k) {
        const float s = p.scale * (float)(1u << k);
        float sn, cs;
        sincos_enc(xv * s, &sn, &cs);
        const float m = p.use_mask ? p.mask[k] : 1.0f;
        const float gc = gr[id + dd * L + k];
        const float gs = gr[id + 3 * L + dd * L + k];
        acc += ((-(gc * m) * sn) + (gs * m) * cs) * s;
    }
    return acc;
}

// dx[n, d] for Fourier/BARF encodings of an explicit position input, one thread per (n, d).
__global__ __launch_bounds__(256) void encode_bwd_kernel(nerf_pe_params p, const float* __restrict__ x,
                                                         const float* __restrict__ g, int64_t g_ld, int64_t n_total,
                                                         float* __restrict__ dx, int accumulate) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= n_total * 3) return;
    const int64_t n = idx / 3;
    const int dd = (int)(idx - n * 3);
    float acc = fourier_grad(p, x[n * 3 + dd], dd, g + n * g_ld);
    if (accumulate) acc += dx[idx];
    dx[idx] = acc;
}

// Backward of the integrated encoding (autograd of positional_encodings.py:186-235, and of the
// masked variant :274-282) w.r.t. the position and the direction, one thread per sample:
//   out_cos(d,k) = m_k * (cos(a) * w),  out_sin(d,k) = m_k * (sin(a) * w),
//   a = pm_d * scale * 2^k,  w = exp(-(vb_d * 4^k) / 2),  pm = pos + mu_diff * dir.
//   g_pm_d = g_id_d + sum_k s_k * w * (-m g_cos sin a + m g_sin cos a)
//   g_vb_d = sum_k -(4^k / 2) * w * (m g_cos cos a + m g_sin sin a)
//   dpos = g_pm;  ddir_j = g_pm_j * mu_diff + [diagonal variance only]
//          2 d_j (st - sr / S) g_vb_j + 2 d_j sr / S^2 * sum_d g_vb_d d_d^2   (S = |d|^2)
// t_start / t_end / pixel_width receive no gradient (the reference's samplers never need one).
__global__ __launch_bounds__(256) void encode_bwd_integrated_kernel(
    nerf_pe_params p, const float* __restrict__ x, const float* __restrict__ xdir, const float* __restrict__ t0,
    const float* __restrict__ t1, const float* __restrict__ pw, const float* __restrict__ g, int64_t g_ld,
    int64_t n_total, float* __restrict__ dx, float* __restrict__ ddir, int accumulate) {
#pragma clang fp contract(off)
    const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= n_total) return;
    float pos[3], dv[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        pos[d] = x[n * 3 + d];
        dv[d] = xdir[n * 3 + d];
    }
    float gpm[3], dd[3];
    ipe_grad(p, pos, dv, t0[n], t1[n], pw[n], g + n * g_ld, gpm, dd);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        if (dx) dx[n * 3 + j] = accumulate ? dx[n * 3 + j] + gpm[j] : gpm[j];
        if (ddir) ddir[n * 3 + j] = accumulate ? ddir[n * 3 + j] + dd[j] : dd[j];
    }
}

// Ray-mode backward (positions generated in-kernel from rays, nerf_encode_fwd with x == NULL):
//   pos_s = o + tq_s * d  =>  dL/do = sum_s g_pos_s,  dL/dd = sum_s (tq_s * g_pos_s + g_dir_s)
// where g_dir_s is the integrated encoding's own direction gradient (0 for Fourier/BARF).
// This is the gradient the reference's pose refinement takes through _compute_positions
// (barf/model_interpolation.py:288-312) into CameraExtrinsics (model_camera_extrinsics.py:77-85).
//
// One wavefront per ray, LANES OVER THE ENCODING'S COLUMNS: for every sample the wave reads the
// gradient row as one coalesced 256-byte access, each lane evaluates the sin/cos of its own
// column's argument and adds its column's share of g_pos (and, for the integrated encoding, of
// the variance gradient) into per-lane fp64 accumulators; everything that follows is linear in
// those shares, so the per-sample coefficients (tq, mu_diff, st, sr) are folded in per lane and
// one fixed-order wave reduction per output component ends the ray.  Columns of an encoding
// wider than 64 are strided over the lanes.
__global__ __launch_bounds__(256) void encode_bwd_rays_kernel(EncArgs a, const float* __restrict__ g, int64_t g_ld,
                                                              float* __restrict__ d_o, float* __restrict__ d_d,
                                                              int accumulate) {
#pragma clang fp contract(off)
    const int lane = threadIdx.x & 63;
    const int64_t ray = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (ray >= a.n_rays) return;
    const nerf_pe_params& p = a.p;
    const int L = p.levels;
    const int id = p.include_identity ? 3 : 0;
    const int tl = 3 * L;
    float dv[3], ov[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        dv[j] = a.d[ray * 3 + j];
        ov[j] = a.o[ray * 3 + j];
    }
    // per lane: accumulated contributions to dL/do_dd, dL/dd_dd (own coordinate) and the
    // cross term of the diagonal variance (multiplied by d_j for every j at the end); one set per
    // column slot the lane owns (two slots cover out_dim <= 128)
    double acc_o[2] = {0.0, 0.0}, acc_d[2] = {0.0, 0.0}, acc_x[2] = {0.0, 0.0};
    int slot_d[2] = {-1, -1};
    for (int s = 0; s < a.S; ++s) {
        const int64_t n = ray * a.S + s;
        const float t0 = a.t0[n];
        const float t1 = (p.query != 0 || p.kind == 1) ? a.t1[n] : t0;
        const float tq = (p.query == 0) ? t0 : (t0 + t1) / 2.0f;
        float pos[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) pos[j] = ov[j] + tq * dv[j];
        IpeSample q;
        const float* pm = pos;
        if (p.kind == 1) {
            q = ipe_sample(p, pos, dv, t0, t1, pixel_width_at(a, n));
            pm = q.pm;
        }
        const float* gr = g + n * g_ld;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int c = lane + 64 * u;
            if (c >= a.out_dim) continue;
            const float gv = gr[c];
            int dd;
            float cpos, cvb = 0.0f;       // this column's share of g_pos[dd] / g_vb[dd]
            if (c < id) {
                dd = c;
                cpos = gv;
            } else {
                const int j = c - id;
                const bool is_sin = j >= tl;
                const int jj = is_sin ? j - tl : j;
                dd = jj >= 2 * L ? 2 : (jj >= L ? 1 : 0);
                const int k = jj - dd * L;
                const float m = p.use_mask ? p.mask[k] : 1.0f;
                const float sc = p.scale * (float)(1u << k);
                float sn, cs;
                sincos_enc(sel3(pm, dd) * sc, &sn, &cs);
                const float gm = gv * m;
                float w = 1.0f;
                if (p.kind == 1) w = expf((-(sel3(q.vb, dd) * (float)(1u << (2 * k)))) / 2.0f);
                cpos = (is_sin ? gm * cs : (-gm) * sn) * w * sc;
                if (p.kind == 1) cvb = (is_sin ? gm * sn : gm * cs) * w * (-((float)(1u << (2 * k)) / 2.0f));
            }
            slot_d[u] = dd;
            acc_o[u] += (double)cpos;
            double dterm = (double)(tq * cpos);
            if (p.kind == 1) {
                dterm += (double)(cpos * q.mu_diff);
                if (!p.distribute_variance) {
                    const float S = q.ssum;
                    dterm += (double)((2.0f * sel3(dv, dd)) * ((q.st - q.sr / S) * cvb));
                    acc_x[u] += (double)((cvb * (sel3(dv, dd) * sel3(dv, dd))) * ((2.0f * q.sr) / (S * S)));
                }
            }
            acc_d[u] += dterm;
        }
    }
    double cross = wave_sum(acc_x[0] + acc_x[1]);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        double so = 0.0, sd = 0.0;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            if (slot_d[u] == j) {
                so += acc_o[u];
                sd += acc_d[u];
            }
        }
        so = wave_sum(so);
        sd = wave_sum(sd) + cross * (double)dv[j];
        if (lane == 0) {
            if (d_o) d_o[ray * 3 + j] = accumulate ? d_o[ray * 3 + j] + (float)so : (float)so;
            if (d_d) d_d[ray * 3 + j] = accumulate ? d_d[ray * 3 + j] + (float)sd : (float)sd;
        }
    }
}

int enc_num_cus() {
    static int n = 0;
    if (n == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
    }
    return n;
}

int out_dim_of(const nerf_pe_params& p) { return (2 * p.levels + (p.include_identity ? 1 : 0)) * 3; }

}  // namespace

extern "C" int nerf_encode_fwd(const nerf_pe_params* params, const float* x, const float* xdir,
                               const float* ray_o, const float* ray_d, const float* t_start, const float* t_end,
                               const float* pixel_width, int64_t n_samples, int32_t samples_per_ray,
                               int64_t n_rays, float* out, int64_t out_ld, void* stream) {
    NERF_REQUIRE(params && out && n_samples >= 0);
    if (n_samples == 0) return NERF_OK;
    const nerf_pe_params& p = *params;
    NERF_REQUIRE(p.levels >= 0 && p.levels <= 16 && (p.kind == 0 || p.kind == 1));
    const int od = out_dim_of(p);
    NERF_REQUIRE(out_ld >= od && od > 0);
    if (!x) NERF_REQUIRE(ray_o && ray_d && t_start && samples_per_ray >= 1 && (p.query == 0 || t_end));
    if (p.kind == 1) {
        NERF_REQUIRE(t_start && t_end && pixel_width && (x ? xdir != nullptr : ray_d != nullptr));
        NERF_REQUIRE(p.pw_mode >= 0 && p.pw_mode <= 2);
        if (p.pw_mode != 2 && !x) NERF_REQUIRE(samples_per_ray >= 1 && n_rays >= 1);
        if (p.pw_mode == 1) NERF_REQUIRE(n_rays >= 1);
        if (p.pw_mode == 0) NERF_REQUIRE(samples_per_ray >= 1);
    }
    NERF_REQUIRE(n_samples < (1ll << 31) && out_ld <= 1024);
    const int vec = aligned16(out) && (out_ld % 4) == 0;
    EncArgs a{p, x, xdir, ray_o, ray_d, t_start, t_end, pixel_width, n_samples,
              samples_per_ray > 0 ? samples_per_ray : 1, n_rays, out, out_ld, od, vec};
    if (vec && out_ld <= kEncMaxLd) {
        int64_t blocks = (n_samples + kEncRows - 1) / kEncRows;
        if (NERF_ENC_PERSIST) blocks = blocks < 8 * enc_num_cus() ? blocks : 8 * enc_num_cus();
        const size_t lds = (size_t)kEncRows * (size_t)(out_ld + 4) * sizeof(float);
        hipLaunchKernelGGL(encode_fwd_lds_kernel, dim3((unsigned)blocks), dim3(256), lds, as_stream(stream), a);
    } else {
        const int Q = (int)((out_ld + 3) / 4);      // threads per row (4 columns each)
        const int RB = 256 / Q;                     // rows per block
        const int64_t blocks = (n_samples + RB - 1) / RB;
        hipLaunchKernelGGL(encode_fwd_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), a, Q, RB);
    }
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}

extern "C" int nerf_encode_bwd(const nerf_pe_params* params, const float* x, const float* grad_out, int64_t g_ld,
                               int64_t n_samples, float* dx, int32_t accumulate, void* stream) {
    NERF_REQUIRE(params && x && grad_out && dx && n_samples >= 0);
    if (n_samples == 0) return NERF_OK;
    if (params->kind != 0) return NERF_ERR_UNSUPPORTED;
    NERF_REQUIRE(g_ld >= out_dim_of(*params));
    const int64_t total = n_samples * 3;
    hipLaunchKernelGGL(encode_bwd_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, as_stream(stream),
                       *params, x, grad_out, g_ld, n_samples, dx, accumulate);
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}

extern "C" int nerf_encode_bwd_integrated(const nerf_pe_params* params, const float* x, const float* xdir,
                                          const float* t_start, const float* t_end, const float* pixel_width,
                                          const float* grad_out, int64_t g_ld, int64_t n_samples, float* dx,
                                          float* ddir, int32_t accumulate, void* stream) {
    NERF_REQUIRE(params && n_samples >= 0);
    if (n_samples == 0) return NERF_OK;
    NERF_REQUIRE(params->kind == 1 && params->levels >= 0 && params->levels <= 16);
    NERF_REQUIRE(x && xdir && t_start && t_end && pixel_width && grad_out && (dx || ddir));
    NERF_REQUIRE(g_ld >= out_dim_of(*params));
    hipLaunchKernelGGL(encode_bwd_integrated_kernel, dim3((unsigned)((n_samples + 255) / 256)), dim3(256), 0,
                       as_stream(stream), *params, x, xdir, t_start, t_end, pixel_width, grad_out, g_ld, n_samples,
                       dx, ddir, accumulate);
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}

extern "C" int nerf_encode_bwd_rays(const nerf_pe_params* params, const float* ray_o, const float* ray_d,
                                    const float* t_start, const float* t_end, const float* pixel_width,
                                    const float* grad_out, int64_t g_ld, int64_t n_rays, int32_t samples_per_ray,
                                    float* d_origs, float* d_dirs, int32_t accumulate, void* stream) {
    NERF_REQUIRE(params && n_rays >= 0 && samples_per_ray >= 1);
    if (n_rays == 0) return NERF_OK;
    const nerf_pe_params& p = *params;
    NERF_REQUIRE(p.levels >= 0 && p.levels <= 16 && (p.kind == 0 || p.kind == 1));
    NERF_REQUIRE(ray_o && ray_d && t_start && grad_out && (d_origs || d_dirs));
    NERF_REQUIRE(g_ld >= out_dim_of(p) && out_dim_of(p) <= 128);
    if (p.query != 0 || p.kind == 1) NERF_REQUIRE(t_end != nullptr);
    if (p.kind == 1) NERF_REQUIRE(pixel_width != nullptr && p.pw_mode >= 0 && p.pw_mode <= 2);
    const int64_t n = n_rays * (int64_t)samples_per_ray;
    NERF_REQUIRE(n < (1ll << 31));
    EncArgs a{p, nullptr, nullptr, ray_o, ray_d, t_start, t_end, pixel_width, n, samples_per_ray, n_rays,
              nullptr, g_ld, out_dim_of(p), 0};
    hipLaunchKernelGGL(encode_bwd_rays_kernel, dim3((unsigned)((n_rays + 3) / 4)), dim3(256), 0, as_stream(stream), a,
                       grad_out, g_ld, d_origs, d_dirs, accumulate);
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}

extern "C" int nerf_encode_rays(const nerf_pe_params* params, const float* ray_d, int64_t n_rays, float* out,
                                int64_t out_ld, void* stream) {
    NERF_REQUIRE(params && params->kind == 0);
    nerf_pe_params p = *params;
    return nerf_encode_fwd(&p, ray_d, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, n_rays, 1, n_rays, out,
                           out_ld, stream);
}
