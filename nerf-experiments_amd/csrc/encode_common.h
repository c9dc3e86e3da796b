// Encoding math shared by the encoding kernels (encode.hip) and the fused field MLP, which
// generates its encoding inputs in-kernel (mlp_fused.hip): positions from rays, the mip-NeRF
// integrated-encoding terms and one encoding column, in the reference's fp32 operation order
// (barf/positional_encodings.py:42-57, 124-148, 170-240; model_interpolation.py:288-312), so
// both produce bitwise the same values.  The argument structs provide p (nerf_pe_params), x,
// xdir, o, d, t0, t1, pw, S, n_rays (p: nerf_pe_params or an address-space-qualified reference).
#pragma once
#include "common.h"

namespace nerf {

template <class A>
__device__ __forceinline__ void load_pos_dir(const A& a, int64_t n, float p[3], float dv[3]) {
#pragma clang fp contract(off)
    if (a.x) {
        p[0] = a.x[n * 3 + 0]; p[1] = a.x[n * 3 + 1]; p[2] = a.x[n * 3 + 2];
        if (a.xdir) { dv[0] = a.xdir[n * 3 + 0]; dv[1] = a.xdir[n * 3 + 1]; dv[2] = a.xdir[n * 3 + 2]; }
        else { dv[0] = dv[1] = dv[2] = 0.f; }
    } else {
        const int64_t ray = (int64_t)((uint32_t)n / (uint32_t)a.S);   // n < 2^31 (host check)
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

template <class A>
__device__ __forceinline__ float pixel_width_at(const A& a, int64_t n) {
    if (a.p.pw_mode == 0) return a.pw[(uint32_t)n / (uint32_t)a.S];
    if (a.p.pw_mode == 1) return a.pw[(uint32_t)n % (uint32_t)a.n_rays];
    return a.pw[n];
}

// Per-sample quantities of the mip-NeRF integrated encoding (positional_encodings.py:186-226),
// in the reference's fp32 operation order:
//   pm      = pos + mu_diff * dir                         (eq 8, :190-191)
//   vb[d]   = variance of coordinate d before the 4^k level scale: (st + 2 sr) / 3 when the
//             variance is distributed (:213-215), st d_d^2 + sr (1 - d_d^2 / |d|^2) otherwise
//             (eq 16, :219); weight(d, k) = exp(-(vb[d] * 4^k) / 2).
// st, sr (eq 7, :201-207) and mu_diff are returned for the backward.
struct IpeSample {
    float pm[3], vb[3];
    float st, sr, mu_diff, ssum;
};

template <class P>
__device__ __forceinline__ IpeSample ipe_sample(const P& p, const float pos[3], const float dv[3], float t0, float t1,
                                                float pwv) {
#pragma clang fp contract(off)
    IpeSample r;
    const float tm = (t0 + t1) / 2.0f;
    const float td = (t1 - t0) / 2.0f;
    const float tm2 = tm * tm, td2 = td * td;
    const float td4 = powf(td, 4.0f);
    r.mu_diff = ((2.0f * tm) * td2) / ((3.0f * tm2) + td2);
    r.pm[0] = pos[0] + r.mu_diff * dv[0];
    r.pm[1] = pos[1] + r.mu_diff * dv[1];
    r.pm[2] = pos[2] + r.mu_diff * dv[2];
    const float r_dot = (pwv * 2.0f) / 3.4641016151377544f;
    const float q3 = (3.0f * tm2) + td2;
    float st = (td2 / 3.0f) - (((4.0f * td4) * ((12.0f * tm2) - td2)) / (15.0f * (q3 * q3)));
    float sr = (r_dot * r_dot) * (((tm2 / 4.0f) + ((5.0f * td2) / 12.0f)) - ((4.0f * td4) / (15.0f * q3)));
    if (p.pixel_width_sigma > 0.25f) {
        const float as_ = (p.pixel_width_sigma * pwv) * tm;
        const float add = as_ * as_;
        st = st + add;
        sr = sr + add;
    }
    r.st = st;
    r.sr = sr;
    r.ssum = (dv[0] * dv[0] + dv[1] * dv[1]) + dv[2] * dv[2];
    if (p.distribute_variance) {
        const float v = (st + sr * 2.0f) / 3.0f;
        r.vb[0] = r.vb[1] = r.vb[2] = v;
    } else {
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            const float d2 = dv[d] * dv[d];
            r.vb[d] = (st * d2) + (sr * (1.0f - (d2 / r.ssum)));
        }
    }
    return r;
}

// Value of encoding column c (< out_dim) of one sample.  pm = the (mean-shifted, for kind 1)
// position; q = the IPE per-sample terms (kind 1 only).  P: nerf_pe_params, or its copy in the
// kernel-argument segment (address space 4: uniform fields by scalar loads, no private copy).
template <class P>
__device__ __forceinline__ float enc_column(const P& p, int L, int id, int c, const float pm[3], const IpeSample& q) {
#pragma clang fp contract(off)
    if (c < id) return sel3(pm, c);
    const int j = c - id;
    const int blk = j >= 3 * L ? 1 : 0;              // 0 cos, 1 sin
    const int jj = j - blk * 3 * L;
    const int dd = jj >= 2 * L ? 2 : (jj >= L ? 1 : 0);
    const int k = jj - dd * L;
    const float s = p.scale * (float)(1u << k);
    const float arg = sel3(pm, dd) * s;
    float sn, cs;
    sincos_enc(arg, &sn, &cs);
    float val = blk == 0 ? cs : sn;
    if (p.kind == 1) {
        // mip-NeRF weight exp(-(var_d * 4^k) / 2) (positional_encodings.py:213-232)
        const float sc4 = (float)(1u << (2 * k));   // 4^k (exact)
        val = val * expf((-(sel3(q.vb, dd) * sc4)) / 2.0f);
    }
    if (p.use_mask) val = p.mask[k] * val;
    return val;
}


}  // namespace nerf
