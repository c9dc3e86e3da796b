// Alpha compositing (volume rendering quadrature) — forward and backward.
//
// Reference: NerfInterpolation._render_rays, barf/model_interpolation.py:316-353
//   blocking_neg = (-densities * distances) * 3 * MAGIC_NUMBER
//   alpha        = 1 - exp(blocking_neg)
//   alpha_int    = [1, exp(cumsum(blocking_neg[:, :-1]))]
//   weights      = alpha_int * alpha;  rgb = sum(weights[..., None] * colors, 1)
//
// Design: one 64-lane wavefront per ray; lane l owns R consecutive samples
// s = l*R + r.  The exclusive prefix of b is a per-lane serial scan plus a
// wave shuffle scan, both in fp64 (torch's CPU cumsum accumulates fp32 input
// in double, which is what the reference's CPU path computes).  No LDS, no
// atomics; HBM traffic = the algorithmic bytes (sigma, rgb, delta in; w, rgb out).
#include "common.h"

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
template <int R, bool PK>
__device__ __forceinline__ void load_samples(const CompositeArgs& a, int64_t ray, int lane, float (&rd)[R],
                                             float (&del)[R], float (&rc)[R][3]) {
    const int64_t base = ray * a.S;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int s = lane * R + r;
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
                const float* cp = a.color + n * a.cs;
                rc[r][0] = cp[0]; rc[r][1] = cp[1]; rc[r][2] = cp[2];
            }
        }
    }
}

template <int R, bool PK>
__device__ __forceinline__ void composite_fwd_ray(const CompositeArgs& a, int64_t ray, int lane, const float (&rd)[R],
                                                  const float (&del)[R], const float (&rc)[R][3],
                                                  float* __restrict__ rgb_out, float* __restrict__ w_out) {
#pragma clang fp contract(off)
    const int64_t base = ray * a.S;

    float b[R], e[R], c[R][3];
    double pre[R];
    double run = 0.0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int s = lane * R + r;
        float sig = rd[r];
        c[r][0] = rc[r][0]; c[r][1] = rc[r][1]; c[r][2] = rc[r][2];
        if (a.act && s < a.S) {
            sig = softplus_thr8(sig - a.shift);
            c[r][0] = sigmoidf_(c[r][0]);
            c[r][1] = sigmoidf_(c[r][1]);
            c[r][2] = sigmoidf_(c[r][2]);
        }
        // ((-sigma * delta) * 3) * MAGIC — two fp32 multiplies, as the reference.
        float bb = ((-sig) * del[r]) * a.sa;
        bb = bb * a.sb;
        if (s >= a.S) bb = 0.f;
        b[r] = bb;
        e[r] = expf(bb);
        pre[r] = run;            // exclusive within lane
        run += (double)bb;
    }
    const double incl = wave_inclusive_scan(run);
    const double lane_off = incl - run;

    float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int s = lane * R + r;
        const double ex = lane_off + pre[r];
        const float T = (s == 0) ? 1.0f : expf((float)ex);
        const float alpha = 1.0f - e[r];
        const float w = T * alpha;
        if (s < a.S) {
            if (w_out) w_out[base + s] = w;
            acc0 += w * c[r][0];
            acc1 += w * c[r][1];
            acc2 += w * c[r][2];
        }
    }
    acc0 = wave_sum_f(acc0);
    acc1 = wave_sum_f(acc1);
    acc2 = wave_sum_f(acc2);
    if (lane == 0) {
        rgb_out[ray * 3 + 0] = acc0;
        rgb_out[ray * 3 + 1] = acc1;
        rgb_out[ray * 3 + 2] = acc2;
    }
}

// Each wave walks rays ray, ray + 4*gridDim.x, ... and loads the next ray's samples before
// compositing the current one, so the loads of one ray overlap the scan of the previous one
// (prefetch_rays; otherwise one ray per wave, as the grid is not capped).
template <int R, bool PK>
__global__ __launch_bounds__(256) void composite_fwd_kernel(CompositeArgs a, float* __restrict__ rgb_out,
                                                            float* __restrict__ w_out) {
    const int lane = lane_id();
    int64_t ray = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (ray >= a.n_rays) return;
    float rd[R], del[R], rc[R][3];
    load_samples<R, PK>(a, ray, lane, rd, del, rc);
    if constexpr (!prefetch_rays(R)) {
        composite_fwd_ray<R, PK>(a, ray, lane, rd, del, rc, rgb_out, w_out);
    } else {
        const int64_t step = (int64_t)gridDim.x * 4;
        for (;;) {
            const int64_t next = ray + step;
            const bool more = next < a.n_rays;
            float nd[R], ndel[R], nc[R][3];
            load_samples<R, PK>(a, more ? next : ray, lane, nd, ndel, nc);
            composite_fwd_ray<R, PK>(a, ray, lane, rd, del, rc, rgb_out, w_out);
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
template <int R, bool PK, bool PKG>
__device__ __forceinline__ void composite_bwd_ray(const CompositeArgs& a, int64_t ray, int lane, const float (&rawd)[R],
                                                  const float (&del)[R], const float (&rawc)[R][3], float g0,
                                                  float g1, float g2, const float* __restrict__ g_w,
                                                  float* __restrict__ gd, int64_t gds, float* __restrict__ gc,
                                                  int64_t gcs) {
#pragma clang fp contract(off)
    const int64_t base = ray * a.S;

    float sig[R], c[R][3], b[R], e[R];
    double pre[R];
    double run = 0.0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int s = lane * R + r;
        if (a.act) {
            sig[r] = softplus_thr8(rawd[r] - a.shift);
            c[r][0] = sigmoidf_(rawc[r][0]);
            c[r][1] = sigmoidf_(rawc[r][1]);
            c[r][2] = sigmoidf_(rawc[r][2]);
        } else {
            sig[r] = rawd[r];
            c[r][0] = rawc[r][0]; c[r][1] = rawc[r][1]; c[r][2] = rawc[r][2];
        }
        float bb = ((-sig[r]) * del[r]) * a.sa;
        bb = bb * a.sb;
        if (s >= a.S) bb = 0.f;
        b[r] = bb;
        e[r] = expf(bb);
        pre[r] = run;
        run += (double)bb;
    }
    const double incl = wave_inclusive_scan(run);
    const double lane_off = incl - run;

    float T[R], w[R], gw[R];
    double q[R];
    double qrun = 0.0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int s = lane * R + r;
        T[r] = (s == 0) ? 1.0f : expf((float)(lane_off + pre[r]));
        w[r] = T[r] * (1.0f - e[r]);
        float gwr = 0.f;
        if (s < a.S) {
            gwr = g0 * c[r][0] + g1 * c[r][1] + g2 * c[r][2];
            if (g_w) gwr += g_w[base + s];
        }
        gw[r] = gwr;
        q[r] = (double)gwr * (double)w[r];
        qrun += q[r];
    }
    // suffix sums: sum_{i>k} q_i = total - inclusive_prefix(k)
    const double qincl = wave_inclusive_scan(qrun);
    const double qtotal = __shfl(qincl, NERF_WAVE - 1, NERF_WAVE);
    double qpre = qincl - qrun;  // exclusive lane offset
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int s = lane * R + r;
        qpre += q[r];
        const double suffix = qtotal - qpre;
        if (s >= a.S) continue;
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

template <int R, bool PK, bool PKG>
__global__ __launch_bounds__(256) void composite_bwd_kernel(CompositeArgs a, const float* __restrict__ g_rgb,
                                                            const float* __restrict__ g_w,
                                                            float* __restrict__ gd, int64_t gds,
                                                            float* __restrict__ gc, int64_t gcs) {
    const int lane = lane_id();
    int64_t ray = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (ray >= a.n_rays) return;
    float rawd[R], del[R], rawc[R][3];
    load_samples<R, PK>(a, ray, lane, rawd, del, rawc);
    float g0 = g_rgb[ray * 3 + 0], g1 = g_rgb[ray * 3 + 1], g2 = g_rgb[ray * 3 + 2];
    if constexpr (!prefetch_rays(R)) {
        composite_bwd_ray<R, PK, PKG>(a, ray, lane, rawd, del, rawc, g0, g1, g2, g_w, gd, gds, gc, gcs);
    } else {
        const int64_t step = (int64_t)gridDim.x * 4;
        for (;;) {
            const int64_t next = ray + step;
            const bool more = next < a.n_rays;
            const int64_t pf = more ? next : ray;
            float nd[R], ndel[R], nc[R][3];
            load_samples<R, PK>(a, pf, lane, nd, ndel, nc);
            const float ng0 = g_rgb[pf * 3 + 0], ng1 = g_rgb[pf * 3 + 1], ng2 = g_rgb[pf * 3 + 2];
            composite_bwd_ray<R, PK, PKG>(a, ray, lane, rawd, del, rawc, g0, g1, g2, g_w, gd, gds, gc, gcs);
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
    switch (R) {
#define CASE(RR) case RR: if (pk) hipLaunchKernelGGL((composite_fwd_kernel<RR, true>), grid, block, 0, st, a, rgb_out, weights_out); \
                          else hipLaunchKernelGGL((composite_fwd_kernel<RR, false>), grid, block, 0, st, a, rgb_out, weights_out); break;
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
    switch (R) {
#define LAUNCH(RR, P, PG) hipLaunchKernelGGL((composite_bwd_kernel<RR, P, PG>), grid, block, 0, st, a, grad_rgb, grad_weights, grad_density, gd_stride, grad_color, gc_stride)
#define CASE(RR) case RR: if (pk && pkg) LAUNCH(RR, true, true); else if (pk) LAUNCH(RR, true, false); \
                          else if (pkg) LAUNCH(RR, false, true); else LAUNCH(RR, false, false); break;
        CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(8) CASE(16)
#undef CASE
#undef LAUNCH
        default: return NERF_ERR_UNSUPPORTED;
    }
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}
