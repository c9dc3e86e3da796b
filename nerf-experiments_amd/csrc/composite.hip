// Alpha compositing (volume rendering quadrature) — forward and backward.
//
// Reference: NerfInterpolation._render_rays, barf/model_interpolation.py:316-353
//   blocking_neg = (-densities * distances) * 3 * MAGIC_NUMBER
//   alpha        = 1 - exp(blocking_neg)
//   alpha_int    = [1, exp(cumsum(blocking_neg[:, :-1]))]
//   weights      = alpha_int * alpha;  rgb = sum(weights[..., None] * colors, 1)
//
// Design: one 64-lane wavefront per ray; lane l owns the R samples s = 64 r + l,
// so every load and store instruction covers 64 consecutive samples (256 B of a
// per-sample scalar, 1 KB of 16-byte colour rows: the round-1 layout, R consecutive
// samples per lane, touched 8x the cache lines per instruction and streamed at
// 2.6 TB/s on a full 800x800 frame).  The exclusive prefix of b is one fp64 wave
// scan per 64-sample segment plus the running segment total (torch's CPU cumsum
// accumulates fp32 input in double, which is what the reference's CPU path
// computes).  No LDS, no atomics; HBM traffic = the algorithmic bytes (sigma,
// rgb, delta in; w, rgb out).
#include "common.h"
#include "composite_common.h"

using namespace nerf;

namespace {

struct CompositeArgs {
    const float* density; int64_t ds;
    const float* color; int64_t cs;
    const float* dist;
    int64_t n_rays; int S;
    float sa, sb; int act; float shift;
};

// The next ray is prefetched (and the grid capped at one residency, kMaxBlocks) for up to
// 128 samples per ray; longer rays would double an already large register footprint.
constexpr bool prefetch_rays(int R) { return R <= 2; }
constexpr int64_t kMaxBlocks = 2048;  // 256 CUs x 32 waves / 4 waves per block

// One ray's samples into registers: raw density, interval length, raw colour (zeros past S).
// PK: [rgb | sigma] rows; C4: colour rows of stride 4, 16-byte aligned (one dwordx4 each).
template <int R, bool PK, bool C4>
__device__ __forceinline__ void load_samples(const CompositeArgs& a, int64_t ray, int lane, float (&rd)[R],
                                             float (&del)[R], float (&rc)[R][3]) {
    const int64_t base = ray * a.S;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int s = r * NERF_WAVE + lane;
        rd[r] = 0.f; del[r] = 0.f;
        rc[r][0] = rc[r][1] = rc[r][2] = 0.f;
        if (s < a.S) {
            const int64_t n = base + s;
            del[r] = a.dist[n];
            if (PK) {  // [rgb | sigma] rows of 16 B: one dwordx4 load per sample
                const float4 v = *reinterpret_cast<const float4*>(a.color + n * 4);
                rc[r][0] = v.x; rc[r][1] = v.y; rc[r][2] = v.z; rd[r] = v.w;
            } else {
                rd[r] = a.density[n * a.ds];
                if (C4) {
                    const float4 v = *reinterpret_cast<const float4*>(a.color + n * 4);
                    rc[r][0] = v.x; rc[r][1] = v.y; rc[r][2] = v.z;
                } else {
                    const float* cp = a.color + n * a.cs;
                    rc[r][0] = cp[0]; rc[r][1] = cp[1]; rc[r][2] = cp[2];
                }
            }
        }
    }
}

template <int R>
__device__ __forceinline__ void composite_fwd_ray(const CompositeArgs& a, int64_t ray, int lane, const float (&rd)[R],
                                                  const float (&del)[R], const float (&rc)[R][3],
                                                  float* __restrict__ rgb_out, float* __restrict__ w_out) {
    const int64_t base = ray * a.S;
    float w[R], rgb[3], cc[R][3], cs[R][3];
    composite_ray<R, false>(a.S, a.sa, a.sb, a.act, a.shift, lane, rd, del, rc, w, rgb, cc, cs);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int s = r * NERF_WAVE + lane;
        if (s < a.S && w_out) w_out[base + s] = w[r];
    }
    if (lane == 0) {
        rgb_out[ray * 3 + 0] = rgb[0];
        rgb_out[ray * 3 + 1] = rgb[1];
        rgb_out[ray * 3 + 2] = rgb[2];
    }
}

// Each wave walks rays ray, ray + 4*gridDim.x, ... and loads the next ray's samples before
// compositing the current one, so the loads of one ray overlap the scan of the previous one
// (prefetch_rays; otherwise one ray per wave, as the grid is not capped).
template <int R, bool PK, bool C4>
__global__ __launch_bounds__(256) void composite_fwd_kernel(CompositeArgs a, float* __restrict__ rgb_out,
                                                            float* __restrict__ w_out) {
    const int lane = lane_id();
    int64_t ray = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (ray >= a.n_rays) return;
    float rd[R], del[R], rc[R][3];
    load_samples<R, PK, C4>(a, ray, lane, rd, del, rc);
    if constexpr (!prefetch_rays(R)) {
        composite_fwd_ray<R>(a, ray, lane, rd, del, rc, rgb_out, w_out);
    } else {
        const int64_t step = (int64_t)gridDim.x * 4;
        for (;;) {
            const int64_t next = ray + step;
            const bool more = next < a.n_rays;
            float nd[R], ndel[R], nc[R][3];
            load_samples<R, PK, C4>(a, more ? next : ray, lane, nd, ndel, nc);
            composite_fwd_ray<R>(a, ray, lane, rd, del, rc, rgb_out, w_out);
            if (!more) break;
            ray = next;
            for (int r = 0; r < R; ++r) {  // R <= 2: unrolled by the compiler
                rd[r] = nd[r]; del[r] = ndel[r];
                rc[r][0] = nc[r][0]; rc[r][1] = nc[r][1]; rc[r][2] = nc[r][2];
            }
        }
    }
}

// Backward.  With g_w(s) = <g_rgb, c_s> + g_weights(s):
//   dL/db_k = -g_w(k) * T_k * exp(b_k) + sum_{i>k} g_w(i) * w_i
//   dL/dsigma_k = dL/db_k * (-(delta_k) * sa * sb) ;  dL/dc_k = w_k * g_rgb
// Same ray walk and next-ray prefetch as the forward.
template <int R, bool PKG>
__device__ __forceinline__ void composite_bwd_ray(const CompositeArgs& a, int64_t ray, int lane, const float (&rawd)[R],
                                                  const float (&del)[R], const float (&rawc)[R][3], float g0,
                                                  float g1, float g2, const float* __restrict__ g_w,
                                                  float* __restrict__ gd, int64_t gds, float* __restrict__ gc,
                                                  int64_t gcs) {
#pragma clang fp contract(off)
    const int64_t base = ray * a.S;

    float c[R][3], T[R], w[R], e[R], gw[R];
    double qincl[R];               // inclusive prefix of q = g_w * w over the ray, in sample order
    double carry = 0.0, qcarry = 0.0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int s = r * NERF_WAVE + lane;
        float sig;
        if (a.act) {
            sig = comp_softplus(rawd[r] - a.shift);
            c[r][0] = comp_sigmoid(rawc[r][0]);
            c[r][1] = comp_sigmoid(rawc[r][1]);
            c[r][2] = comp_sigmoid(rawc[r][2]);
        } else {
            sig = rawd[r];
            c[r][0] = rawc[r][0]; c[r][1] = rawc[r][1]; c[r][2] = rawc[r][2];
        }
        float bb = ((-sig) * del[r]) * a.sa;
        bb = bb * a.sb;
        if (s >= a.S) bb = 0.f;
        e[r] = comp_exp(bb);
        const double incl = wave_inclusive_scan((double)bb);
        const double ex = carry + (incl - (double)bb);
        carry += __shfl(incl, NERF_WAVE - 1, NERF_WAVE);
        T[r] = (s == 0) ? 1.0f : comp_exp((float)ex);
        w[r] = T[r] * (1.0f - e[r]);
        float gwr = 0.f;
        if (s < a.S) {
            gwr = g0 * c[r][0] + g1 * c[r][1] + g2 * c[r][2];
            if (g_w) gwr += g_w[base + s];
        }
        gw[r] = gwr;
        const double qi = wave_inclusive_scan((double)gwr * (double)w[r]);
        qincl[r] = qcarry + qi;
        qcarry += __shfl(qi, NERF_WAVE - 1, NERF_WAVE);
    }
    // suffix sums: sum_{i>k} q_i = total - inclusive_prefix(k)
    const double qtotal = qcarry;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int s = r * NERF_WAVE + lane;
        if (s >= a.S) continue;
        const double suffix = qtotal - qincl[r];
        const int64_t n = base + s;
        const float dldb = (float)((double)(-gw[r] * T[r] * e[r]) + suffix);
        float dsig = 0.f;
        if (PKG || gd) {
            dsig = -(((dldb * a.sb) * a.sa) * del[r]);
            if (a.act) dsig = dsig * softplus_thr8_grad(rawd[r] - a.shift);
            if (!PKG) gd[n * gds] = dsig;
        }
        if (PKG || gc) {
            float d0 = w[r] * g0, d1 = w[r] * g1, d2 = w[r] * g2;
            if (a.act) {
                d0 = d0 * (1.0f - c[r][0]) * c[r][0];
                d1 = d1 * (1.0f - c[r][1]) * c[r][1];
                d2 = d2 * (1.0f - c[r][2]) * c[r][2];
            }
            if (PKG) {  // [d rgb | d sigma] rows: one dwordx4 store per sample
                *reinterpret_cast<float4*>(gc + n * 4) = make_float4(d0, d1, d2, dsig);
            } else {
                float* gp = gc + n * gcs;
                gp[0] = d0; gp[1] = d1; gp[2] = d2;
            }
        }
    }
}

template <int R, bool PK, bool C4, bool PKG>
__global__ __launch_bounds__(256) void composite_bwd_kernel(CompositeArgs a, const float* __restrict__ g_rgb,
                                                            const float* __restrict__ g_w,
                                                            float* __restrict__ gd, int64_t gds,
                                                            float* __restrict__ gc, int64_t gcs) {
    const int lane = lane_id();
    int64_t ray = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (ray >= a.n_rays) return;
    float rawd[R], del[R], rawc[R][3];
    load_samples<R, PK, C4>(a, ray, lane, rawd, del, rawc);
    float g0 = g_rgb[ray * 3 + 0], g1 = g_rgb[ray * 3 + 1], g2 = g_rgb[ray * 3 + 2];
    if constexpr (!prefetch_rays(R)) {
        composite_bwd_ray<R, PKG>(a, ray, lane, rawd, del, rawc, g0, g1, g2, g_w, gd, gds, gc, gcs);
    } else {
        const int64_t step = (int64_t)gridDim.x * 4;
        for (;;) {
            const int64_t next = ray + step;
            const bool more = next < a.n_rays;
            const int64_t pf = more ? next : ray;
            float nd[R], ndel[R], nc[R][3];
            load_samples<R, PK, C4>(a, pf, lane, nd, ndel, nc);
            const float ng0 = g_rgb[pf * 3 + 0], ng1 = g_rgb[pf * 3 + 1], ng2 = g_rgb[pf * 3 + 2];
            composite_bwd_ray<R, PKG>(a, ray, lane, rawd, del, rawc, g0, g1, g2, g_w, gd, gds, gc, gcs);
            if (!more) break;
            ray = next;
            g0 = ng0; g1 = ng1; g2 = ng2;
            for (int r = 0; r < R; ++r) {
                rawd[r] = nd[r]; del[r] = ndel[r];
                rawc[r][0] = nc[r][0]; rawc[r][1] = nc[r][1]; rawc[r][2] = nc[r][2];
            }
        }
    }
}

// Interleaved [rgb | sigma] rows (the colour head's output, 16-B aligned): the kernel loads
// (stores) each sample's four values with one 16-byte access instead of four strided ones.
bool packed_rows(const float* density, int64_t ds, const float* color, int64_t cs) {
    return density && color && ds == 4 && cs == 4 && density == color + 3 &&
           (reinterpret_cast<uintptr_t>(color) & 15) == 0;
}

int pick_r(int S) {
    int r = (S + NERF_WAVE - 1) / NERF_WAVE;
    if (r <= 6) return r;
    if (r <= 8) return 8;
    if (r <= 16) return 16;
    return -1;
}

}  // namespace

extern "C" int nerf_composite_fwd(const float* density, int64_t density_stride, const float* color,
                                  int64_t color_stride, const float* dist, int64_t n_rays,
                                  int32_t samples_per_ray, float scale_a, float scale_b, int32_t act,
                                  float density_shift, float* rgb_out, float* weights_out, void* stream) {
    NERF_REQUIRE(n_rays >= 0 && samples_per_ray >= 1);
    if (n_rays == 0) return NERF_OK;
    NERF_REQUIRE(density && color && dist && rgb_out);
    const int R = pick_r(samples_per_ray);
    if (R < 0) return NERF_ERR_UNSUPPORTED;
    CompositeArgs a{density, density_stride, color, color_stride, dist, n_rays, samples_per_ray,
                    scale_a, scale_b, act, density_shift};
    dim3 grid((unsigned)((n_rays + 3) / 4)), block(256);
    if (R <= 2) grid.x = (unsigned)std::min<int64_t>(grid.x, kMaxBlocks);
    hipStream_t st = as_stream(stream);
    const bool pk = packed_rows(density, density_stride, color, color_stride);
    const bool c4 = !pk && color_stride == 4 && aligned16(color);
    switch (R) {
#define CASE(RR) case RR: if (pk) hipLaunchKernelGGL((composite_fwd_kernel<RR, true, false>), grid, block, 0, st, a, rgb_out, weights_out); \
                          else if (c4) hipLaunchKernelGGL((composite_fwd_kernel<RR, false, true>), grid, block, 0, st, a, rgb_out, weights_out); \
                          else hipLaunchKernelGGL((composite_fwd_kernel<RR, false, false>), grid, block, 0, st, a, rgb_out, weights_out); break;
        CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(8) CASE(16)
#undef CASE
        default: return NERF_ERR_UNSUPPORTED;
    }
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}

extern "C" int nerf_composite_bwd(const float* density, int64_t density_stride, const float* color,
                                  int64_t color_stride, const float* dist, int64_t n_rays,
                                  int32_t samples_per_ray, float scale_a, float scale_b, int32_t act,
                                  float density_shift, const float* grad_rgb, const float* grad_weights,
                                  float* grad_density, int64_t gd_stride, float* grad_color,
                                  int64_t gc_stride, void* stream) {
    NERF_REQUIRE(n_rays >= 0 && samples_per_ray >= 1);
    if (n_rays == 0) return NERF_OK;
    NERF_REQUIRE(density && color && dist && grad_rgb);
    const int R = pick_r(samples_per_ray);
    if (R < 0) return NERF_ERR_UNSUPPORTED;
    CompositeArgs a{density, density_stride, color, color_stride, dist, n_rays, samples_per_ray,
                    scale_a, scale_b, act, density_shift};
    dim3 grid((unsigned)((n_rays + 3) / 4)), block(256);
    if (R <= 2) grid.x = (unsigned)std::min<int64_t>(grid.x, kMaxBlocks);
    hipStream_t st = as_stream(stream);
    const bool pk = packed_rows(density, density_stride, color, color_stride);
    const bool pkg = packed_rows(grad_density, gd_stride, grad_color, gc_stride);
    const bool c4 = !pk && color_stride == 4 && aligned16(color);
    switch (R) {
#define LAUNCH(RR, P, C, PG) hipLaunchKernelGGL((composite_bwd_kernel<RR, P, C, PG>), grid, block, 0, st, a, grad_rgb, grad_weights, grad_density, gd_stride, grad_color, gc_stride)
#define CASE(RR) case RR: if (pk && pkg) LAUNCH(RR, true, false, true); else if (pk) LAUNCH(RR, true, false, false); \
                          else if (c4 && pkg) LAUNCH(RR, false, true, true); else if (c4) LAUNCH(RR, false, true, false); \
                          else if (pkg) LAUNCH(RR, false, false, true); else LAUNCH(RR, false, false, false); break;
        CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(8) CASE(16)
#undef CASE
#undef LAUNCH
        default: return NERF_ERR_UNSUPPORTED;
    }
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}
