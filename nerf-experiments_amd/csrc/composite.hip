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

template <int R>
__global__ __launch_bounds__(256) void composite_fwd_kernel(CompositeArgs a, float* __restrict__ rgb_out,
                                                            float* __restrict__ w_out) {
#pragma clang fp contract(off)
    const int lane = lane_id();
    const int64_t ray = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (ray >= a.n_rays) return;
    const int64_t base = ray * a.S;

    float b[R], e[R], c[R][3];
    double pre[R];
    double run = 0.0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int s = lane * R + r;
        float sig = 0.f, del = 0.f;
        c[r][0] = c[r][1] = c[r][2] = 0.f;
        if (s < a.S) {
            const int64_t n = base + s;
            sig = a.density[n * a.ds];
            del = a.dist[n];
            const float* cp = a.color + n * a.cs;
            c[r][0] = cp[0]; c[r][1] = cp[1]; c[r][2] = cp[2];
            if (a.act) {
                sig = softplus_thr8(sig - a.shift);
                c[r][0] = sigmoidf_(c[r][0]);
                c[r][1] = sigmoidf_(c[r][1]);
                c[r][2] = sigmoidf_(c[r][2]);
            }
        }
        // ((-sigma * delta) * 3) * MAGIC — two fp32 multiplies, as the reference.
        float bb = ((-sig) * del) * a.sa;
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

// Backward.  With g_w(s) = <g_rgb, c_s> + g_weights(s):
//   dL/db_k = -g_w(k) * T_k * exp(b_k) + sum_{i>k} g_w(i) * w_i
//   dL/dsigma_k = dL/db_k * (-(delta_k) * sa * sb) ;  dL/dc_k = w_k * g_rgb
template <int R>
__global__ __launch_bounds__(256) void composite_bwd_kernel(CompositeArgs a, const float* __restrict__ g_rgb,
                                                            const float* __restrict__ g_w,
                                                            float* __restrict__ gd, int64_t gds,
                                                            float* __restrict__ gc, int64_t gcs) {
#pragma clang fp contract(off)
    const int lane = lane_id();
    const int64_t ray = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (ray >= a.n_rays) return;
    const int64_t base = ray * a.S;
    const float g0 = g_rgb[ray * 3 + 0], g1 = g_rgb[ray * 3 + 1], g2 = g_rgb[ray * 3 + 2];

    float rawd[R], rawc[R][3], sig[R], del[R], c[R][3], b[R], e[R];
    double pre[R];
    double run = 0.0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int s = lane * R + r;
        rawd[r] = 0.f; del[r] = 0.f;
        rawc[r][0] = rawc[r][1] = rawc[r][2] = 0.f;
        if (s < a.S) {
            const int64_t n = base + s;
            rawd[r] = a.density[n * a.ds];
            del[r] = a.dist[n];
            const float* cp = a.color + n * a.cs;
            rawc[r][0] = cp[0]; rawc[r][1] = cp[1]; rawc[r][2] = cp[2];
        }
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
        if (gd) {
            float dsig = -(((dldb * a.sb) * a.sa) * del[r]);
            if (a.act) dsig = dsig * softplus_thr8_grad(rawd[r] - a.shift);
            gd[n * gds] = dsig;
        }
        if (gc) {
            float d0 = w[r] * g0, d1 = w[r] * g1, d2 = w[r] * g2;
            if (a.act) {
                d0 = d0 * (1.0f - c[r][0]) * c[r][0];
                d1 = d1 * (1.0f - c[r][1]) * c[r][1];
                d2 = d2 * (1.0f - c[r][2]) * c[r][2];
            }
            float* gp = gc + n * gcs;
            gp[0] = d0; gp[1] = d1; gp[2] = d2;
        }
    }
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
    hipStream_t st = as_stream(stream);
    switch (R) {
#define CASE(RR) case RR: hipLaunchKernelGGL(composite_fwd_kernel<RR>, grid, block, 0, st, a, rgb_out, weights_out); break;
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
    hipStream_t st = as_stream(stream);
    switch (R) {
#define CASE(RR) case RR: hipLaunchKernelGGL(composite_bwd_kernel<RR>, grid, block, 0, st, a, grad_rgb, grad_weights, grad_density, gd_stride, grad_color, gc_stride); break;
        CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(8) CASE(16)
#undef CASE
        default: return NERF_ERR_UNSUPPORTED;
    }
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}
