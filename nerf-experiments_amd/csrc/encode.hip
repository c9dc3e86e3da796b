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
// Design: one thread per output column of one sample, so a row of the
// encoding (e.g. 64 floats for BARF L=10 + identity, padded) is written by 64
// consecutive lanes — every store is a fully coalesced 256-byte wave write.
// Each thread recomputes the sample's position (o, d, t are L1/L2 hits) and one
// sincos; the kernel is store-bound by design.  Floating-point contraction is
// off so every fp32 operation rounds exactly where the reference's does.
#include "common.h"

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
};

__device__ __forceinline__ void load_pos_dir(const EncArgs& a, int64_t n, float p[3], float dv[3]) {
#pragma clang fp contract(off)
    if (a.x) {
        p[0] = a.x[n * 3 + 0]; p[1] = a.x[n * 3 + 1]; p[2] = a.x[n * 3 + 2];
        if (a.xdir) { dv[0] = a.xdir[n * 3 + 0]; dv[1] = a.xdir[n * 3 + 1]; dv[2] = a.xdir[n * 3 + 2]; }
        else { dv[0] = dv[1] = dv[2] = 0.f; }
    } else {
        const int64_t ray = n / a.S;
        const float tq = (a.p.query == 0) ? a.t0[n] : (a.t0[n] + a.t1[n]) / 2.0f;
        dv[0] = a.d[ray * 3 + 0]; dv[1] = a.d[ray * 3 + 1]; dv[2] = a.d[ray * 3 + 2];
        p[0] = a.o[ray * 3 + 0] + tq * dv[0];
        p[1] = a.o[ray * 3 + 1] + tq * dv[1];
        p[2] = a.o[ray * 3 + 2] + tq * dv[2];
    }
}

__device__ __forceinline__ float sel3(const float v[3], int i) {
    return i == 0 ? v[0] : (i == 1 ? v[1] : v[2]);
}

__device__ __forceinline__ float pixel_width_at(const EncArgs& a, int64_t n) {
    if (a.p.pw_mode == 0) return a.pw[n / a.S];
    if (a.p.pw_mode == 1) return a.pw[n % a.n_rays];
    return a.pw[n];
}

__global__ __launch_bounds__(256) void encode_fwd_kernel(EncArgs a) {
#pragma clang fp contract(off)
    const int64_t total = a.n * a.ld;
    const int L = a.p.levels;
    const int id = a.p.include_identity ? 3 : 0;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int64_t n = idx / a.ld;
        const int c = (int)(idx - n * a.ld);
        float val = 0.0f;
        if (c < a.out_dim) {
            float p[3], dv[3];
            load_pos_dir(a, n, p, dv);
            if (a.p.kind == 1) {
                // mip-NeRF integrated encoding (positional_encodings.py:186-235)
                const float t0 = a.t0[n], t1 = a.t1[n];
                const float tm = (t0 + t1) / 2.0f;
                const float td = (t1 - t0) / 2.0f;
                const float tm2 = tm * tm, td2 = td * td;
                const float td4 = powf(td, 4.0f);
                const float mu_diff = ((2.0f * tm) * td2) / ((3.0f * tm2) + td2);
                float pm[3];
                pm[0] = p[0] + mu_diff * dv[0];
                pm[1] = p[1] + mu_diff * dv[1];
                pm[2] = p[2] + mu_diff * dv[2];
                if (c < id) {
                    val = sel3(pm, c);
                } else {
                    const int j = c - id;
                    const int blk = j / (3 * L);       // 0 cos, 1 sin
                    const int jj = j - blk * 3 * L;
                    const int dd = jj / L, k = jj - dd * L;
                    const float pwv = pixel_width_at(a, n);
                    const float r_dot = (pwv * 2.0f) / 3.4641016151377544f;
                    const float q3 = (3.0f * tm2) + td2;
                    float st = (td2 / 3.0f) - (((4.0f * td4) * ((12.0f * tm2) - td2)) / (15.0f * (q3 * q3)));
                    float sr = (r_dot * r_dot) *
                               (((tm2 / 4.0f) + ((5.0f * td2) / 12.0f)) - ((4.0f * td4) / (15.0f * q3)));
                    if (a.p.pixel_width_sigma > 0.25f) {
                        const float as_ = (a.p.pixel_width_sigma * pwv) * tm;
                        const float add = as_ * as_;
                        st = st + add;
                        sr = sr + add;
                    }
                    const float sc4 = (float)(1u << (2 * k));   // 4^k (exact)
                    float sig;
                    if (a.p.distribute_variance) {
                        sig = ((st + sr * 2.0f) / 3.0f) * sc4;
                    } else {
                        const float dsel = sel3(dv, dd);
                        const float d2 = dsel * dsel;
                        const float ssum = (dv[0] * dv[0] + dv[1] * dv[1]) + dv[2] * dv[2];
                        const float diag = (st * d2) + (sr * (1.0f - (d2 / ssum)));
                        sig = diag * sc4;
                    }
                    const float wgt = expf((-sig) / 2.0f);
                    const float s = a.p.scale * (float)(1u << k);
                    const float arg = sel3(pm, dd) * s;
                    float sn, cs;
                    sincosf(arg, &sn, &cs);
                    val = (blk == 0 ? cs : sn) * wgt;
                    if (a.p.use_mask) val = a.p.mask[k] * val;
                }
            } else {
                if (c < id) {
                    val = sel3(p, c);
                } else {
                    const int j = c - id;
                    const int blk = j / (3 * L);
                    const int jj = j - blk * 3 * L;
                    const int dd = jj / L, k = jj - dd * L;
                    const float s = a.p.scale * (float)(1u << k);
                    const float arg = sel3(p, dd) * s;
                    float sn, cs;
                    sincosf(arg, &sn, &cs);
                    val = (blk == 0) ? cs : sn;
                    if (a.p.use_mask) val = a.p.mask[k] * val;
                }
            }
        }
        a.out[n * a.ld + c] = val;
    }
}

// dx[n, d] = g_id + sum_k mask_k * s_k * (-g_cos * sin(a) + g_sin * cos(a))
__global__ __launch_bounds__(256) void encode_bwd_kernel(nerf_pe_params p, const float* __restrict__ x,
                                                         const float* __restrict__ g, int64_t g_ld, int64_t n_total,
                                                         float* __restrict__ dx, int accumulate) {
#pragma clang fp contract(off)
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= n_total * 3) return;
    const int64_t n = idx / 3;
    const int dd = (int)(idx - n * 3);
    const int L = p.levels;
    const int id = p.include_identity ? 3 : 0;
    const float xv = x[n * 3 + dd];
    const float* gr = g + n * g_ld;
    float acc = id ? gr[dd] : 0.0f;
    for (int k = 0; k < L; ++k) {
        const float s = p.scale * (float)(1u << k);
        const float arg = xv * s;
        float sn, cs;
        sincosf(arg, &sn, &cs);
        const float m = p.use_mask ? p.mask[k] : 1.0f;
        const float gc = gr[id + dd * L + k];
        const float gs = gr[id + 3 * L + dd * L + k];
        acc += ((-(gc * m) * sn) + (gs * m) * cs) * s;
    }
    if (accumulate) acc += dx[idx];
    dx[idx] = acc;
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
    EncArgs a{p, x, xdir, ray_o, ray_d, t_start, t_end, pixel_width, n_samples,
              samples_per_ray > 0 ? samples_per_ray : 1, n_rays, out, out_ld, od};
    const int64_t total = n_samples * out_ld;
    int64_t blocks = (total + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(encode_fwd_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), a);
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

extern "C" int nerf_encode_rays(const nerf_pe_params* params, const float* ray_d, int64_t n_rays, float* out,
                                int64_t out_ld, void* stream) {
    NERF_REQUIRE(params && params->kind == 0);
    nerf_pe_params p = *params;
    return nerf_encode_fwd(&p, ray_d, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, n_rays, 1, n_rays, out,
                           out_ld, stream);
}
