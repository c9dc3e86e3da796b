// Per-ray compositing arithmetic shared by the stand-alone kernels (composite.hip) and the
// compositing fused into the field MLP's forward (mlp_fused.hip): the same instructions, so both
// produce bitwise the same rgb and weights.
//
// Reference: NerfInterpolation._render_rays, barf/model_interpolation.py:316-353
//   b_s = ((-sigma_s * delta_s) * scale_a) * scale_b,  T_s = exp(sum_{j<s} b_j) (fp64 prefix),
//   w_s = T_s * (1 - exp(b_s)),  rgb = sum_s w_s c_s.
// One wavefront per ray; lane l owns the R samples s = 64 r + l.  Prefix sums: fp64 DPP wave scans.
#pragma once
#include "common.h"

namespace nerf {

// NERF_COMP_FASTEXP=1 (off): e^x from the hardware 2^x with the exponent product split (~2 ulp),
// sigmoid through the hardware reciprocal, in the compositing (stand-alone and fused).  At a full
// 800 x 800 frame composite_fwd 2.84 -> 3.17-3.26 TB/s, composite_bwd 2.84 -> 2.93-3.00 (profiles/
// r05e, r05f); off because the parity bars of the compositing are set on the libm results and the
// training step composites inside the fused MLP launches, where these kernels do not run.  Neither a
// second ray's loads in flight nor two rays composited per iteration changed the rates (r05f, r05h):
// the kernel waits on its instruction dependencies (SQ_WAIT_INST_ANY 53 % of wave cycles, r05g).
#ifndef NERF_COMP_FASTEXP
#define NERF_COMP_FASTEXP 0
#endif
#if NERF_COMP_FASTEXP
__device__ __forceinline__ float comp_exp(float x) {
    const float L = 1.44269502162933349609375f;              // log2(e) rounded to fp32
    const float p = x * L;
    const float lo = __builtin_fmaf(x, L, -p) + x * 1.925963033500011e-08f;   // x (log2 e - L)
    return __builtin_amdgcn_exp2f(p) * __builtin_fmaf(lo, 0.693147182464599609375f, 1.0f);
}
__device__ __forceinline__ float comp_sigmoid(float x) { return __builtin_amdgcn_rcpf(1.0f + comp_exp(-x)); }
__device__ __forceinline__ float comp_softplus(float x) { return x > 8.0f ? x : log1pf(comp_exp(x)); }
#else
__device__ __forceinline__ float comp_exp(float x) { return expf(x); }
__device__ __forceinline__ float comp_sigmoid(float x) { return sigmoidf_(x); }
__device__ __forceinline__ float comp_softplus(float x) { return softplus_thr8(x); }
#endif

// rd / del / rc: raw density, interval length, raw (act) or activated colour of the lane's samples
// (anything past S is ignored).  Outputs: w[r] (valid for s < S), rgb (every lane: the wave sum).
// COEF: also the per-sample backward coefficients of the act = 1 form (include/nerf_amd.h,
// nerf_fused_composite): cc[r][ch] = w c (1 - c), cs[r][ch] = d sigma-raw / d grad_rgb_ch.
template <int R, bool COEF>
__device__ __forceinline__ void composite_ray(int S, float sa, float sb, int act, float shift, int lane,
                                              const float (&rd)[R], const float (&del)[R], const float (&rc)[R][3],
                                              float (&w)[R], float (&rgb)[3], float (&cc)[R][3],
                                              float (&cs)[R][3]) {
#pragma clang fp contract(off)
    float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f;
    double carry = 0.0;            // sum of b over the previous 64-sample segments
    float c[R][3], T[R], e[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int s = r * NERF_WAVE + lane;
        float sig = rd[r];
        c[r][0] = rc[r][0]; c[r][1] = rc[r][1]; c[r][2] = rc[r][2];
        if (act && s < S) {
            sig = comp_softplus(sig - shift);
            c[r][0] = comp_sigmoid(c[r][0]);
            c[r][1] = comp_sigmoid(c[r][1]);
            c[r][2] = comp_sigmoid(c[r][2]);
        }
        // ((-sigma * delta) * 3) * MAGIC — two fp32 multiplies, as the reference.
        float bb = ((-sig) * del[r]) * sa;
        bb = bb * sb;
        if (s >= S) bb = 0.f;
        const double incl = wave_inclusive_scan_dpp((double)bb);
        const double ex = carry + (incl - (double)bb);      // exclusive prefix
        carry += wave_last_d(incl);
        T[r] = (s == 0) ? 1.0f : comp_exp((float)ex);
        e[r] = comp_exp(bb);
        w[r] = T[r] * (1.0f - e[r]);
        if (s < S) {
            acc0 += w[r] * c[r][0];
            acc1 += w[r] * c[r][1];
            acc2 += w[r] * c[r][2];
        }
    }
    rgb[0] = wave_sum_f(acc0);
    rgb[1] = wave_sum_f(acc1);
    rgb[2] = wave_sum_f(acc2);
    if constexpr (COEF) {
        // dL/db_n = sum_ch g_ch A_n,ch with A_n,ch = -c_n,ch T_n e^{b_n} + sum_{i>n} c_i,ch w_i
        // (nerf_composite_bwd with gw = <g, c> split per channel), suffix sums in fp64
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
            double qincl[R];
            double qcarry = 0.0;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int s = r * NERF_WAVE + lane;
                const double q = s < S ? (double)c[r][ch] * (double)w[r] : 0.0;
                const double qi = wave_inclusive_scan_dpp(q);
                qincl[r] = qcarry + qi;
                qcarry += wave_last_d(qi);
            }
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int s = r * NERF_WAVE + lane;
                const float a = (float)((double)((-c[r][ch] * T[r]) * e[r]) + (qcarry - qincl[r]));
                float d = -(((a * sb) * sa) * del[r]);
                if (act && s < S) d = d * softplus_thr8_grad(rd[r] - shift);
                cs[r][ch] = d;
                cc[r][ch] = act ? (w[r] * (1.0f - c[r][ch])) * c[r][ch] : w[r];
            }
        }
    }
}

}  // namespace nerf
