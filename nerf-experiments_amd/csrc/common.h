// Shared device helpers for the gfx950 NeRF kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "nerf_amd.h"

#define NERF_WAVE 64

#define NERF_CHECK_LAUNCH()                                   \
    do {                                                      \
        hipError_t e_ = hipGetLastError();                    \
        if (e_ != hipSuccess) return NERF_ERR_LAUNCH;         \
    } while (0)

#define NERF_REQUIRE(cond)                                    \
    do {                                                      \
        if (!(cond)) return NERF_ERR_INVALID_ARG;             \
    } while (0)

// Diagnostic ablation switches (profiling builds only, wrong results by construction).  Every
// NERF_*_DIAG_* macro tested in csrc/ must be listed here (tests/test_capi.py checks the list): a
// translation unit compiled with one reports it through nerf_build_flags(), which load() refuses.
#if defined(NERF_FUSED_DIAG_NOFRAG) || defined(NERF_FUSED_DIAG_MFMAONLY) || defined(NERF_FUSED_DIAG_NOMASK) || \
    defined(NERF_FUSED_DIAG_NOSPLIT) || defined(NERF_FUSED_DIAG_NOSTORE) || defined(NERF_FUSED_DIAG_NOMASKIN) || \
    defined(NERF_FUSED_DIAG_DROPSTORE) || defined(NERF_FUSED_DIAG_NODMA) || defined(NERF_FUSED_DIAG_NOEPI) || \
    defined(NERF_FUSED_DIAG_NOBARRIER) || defined(NERF_FUSED_DIAG_NOCOMP) || defined(NERF_FUSED_DIAG_NOGEN) || \
    defined(NERF_FUSED_DIAG_COMP2) || defined(NERF_FUSED_DIAG_GEN2) || defined(NERF_FUSED_DIAG_BAR2)
#define NERF_TU_DIAG_FUSED NERF_BUILD_DIAG_FUSED
#else
#define NERF_TU_DIAG_FUSED 0
#endif
#if defined(NERF_WS_DIAG_YD_FIXED) || defined(NERF_WS_DIAG_NOCONV) || defined(NERF_WS_DIAG_NOMFMA) || \
    defined(NERF_WT_DIAG_NOMFMA) || defined(NERF_WT_DIAG_NOLOAD)
#define NERF_TU_DIAG_WGRAD NERF_BUILD_DIAG_WGRAD
#else
#define NERF_TU_DIAG_WGRAD 0
#endif
#define NERF_TU_BUILD_FLAGS (NERF_TU_DIAG_FUSED | NERF_TU_DIAG_WGRAD)

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

static inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

namespace nerf {

// ---------------------------------------------------------------------------
// Wave-level scans/reductions (64 lanes).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ double wave_inclusive_scan(double v) {
    const int lane = lane_id();
#pragma unroll
    for (int off = 1; off < NERF_WAVE; off <<= 1) {
        double o = __shfl_up(v, off, NERF_WAVE);
        if (lane >= off) v += o;
    }
    return v;
}

// The same inclusive scan on DPP lane shifts, no LDS round trip per step (the __shfl_up form is a
// ds_bpermute per 32-bit half and step): row_shr 1, 2, 4, 8 inside each 16-lane row, then row_bcast
// 15 / 31 carry the row totals (lanes without a source add 0).  A different summation tree than
// wave_inclusive_scan: use one or the other consistently.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ double dpp_shift_d(double v) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)b, CTRL, ROW_MASK, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(b >> 32), CTRL, ROW_MASK, 0xf, false);
    return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double wave_inclusive_scan_dpp(double v) {
    v += dpp_shift_d<0x111, 0xf>(v);     // row_shr:1
    v += dpp_shift_d<0x112, 0xf>(v);     // row_shr:2
    v += dpp_shift_d<0x114, 0xf>(v);     // row_shr:4
    v += dpp_shift_d<0x118, 0xf>(v);     // row_shr:8
    v += dpp_shift_d<0x142, 0xa>(v);     // row_bcast:15 into rows 1, 3
    v += dpp_shift_d<0x143, 0xc>(v);     // row_bcast:31 into rows 2, 3
    return v;
}
// lane 63's value in every lane (two readlanes: scalar registers, no LDS)
__device__ __forceinline__ double wave_last_d(double v) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, 63);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), 63);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

__device__ __forceinline__ int wave_inclusive_scan_int(int v) {
    const int lane = lane_id();
#pragma unroll
    for (int off = 1; off < NERF_WAVE; off <<= 1) {
        int o = __shfl_up(v, off, NERF_WAVE);
        if (lane >= off) v += o;
    }
    return v;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = NERF_WAVE / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, NERF_WAVE);
    return v;
}

__device__ __forceinline__ float wave_sum_f(float v) {
#pragma unroll
    for (int off = NERF_WAVE / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, NERF_WAVE);
    return v;
}

// ---------------------------------------------------------------------------
// Activations with the exact torch semantics used by NerfModel
// (nn.Softplus(beta=1, threshold=8), nn.Sigmoid).
// ---------------------------------------------------------------------------
__device__ __forceinline__ float softplus_thr8(float x) {
    return (x > 8.0f) ? x : log1pf(expf(x));
}
__device__ __forceinline__ float softplus_thr8_grad(float x) {
    if (x > 8.0f) return 1.0f;
    float z = expf(x);
    return z / (z + 1.0f);
}
__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

// ---------------------------------------------------------------------------
// sin and cos of one fp32 argument for the encodings (|x| up to scale * 2^15 * |p|):
// k = rint(x * 2/pi); r = x - k * pi/2 by a three-term fp32 Cody-Waite reduction with fused
// multiply-adds (each k * c_i exact inside its FMA: |r| error ~1e-7 for |k| < 2^24), then fp32
// minimax polynomials on [-pi/4, pi/4] (Cephes sinf/cosf, ~1 ulp) and the quadrant swap.  About
// a third of the instructions of the libm sincosf, within ~1e-7 absolute of the correctly
// rounded values; larger or non-finite arguments take sincosf.  (-DNERF_SINCOS_FP64_REDUCTION:
// the same with a two-term fp64 reduction, measured 2 % slower in the encoding kernel.)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void sincos_enc(float x, float* s, float* c) {
    if (!(fabsf(x) < 1073741824.0f)) {
        sincosf(x, s, c);
        return;
    }
    const float kf = rintf(x * 0.636619772367581343f);
#ifndef NERF_SINCOS_FP64_REDUCTION
    // three-term fp32 Cody-Waite with fused multiply-adds (each product exact inside the FMA)
    float r = __builtin_fmaf(kf, -1.57079637050628662109375f, x);
    r = __builtin_fmaf(kf, 4.3711388286737929e-08f, r);
    r = __builtin_fmaf(kf, 1.7763568394002505e-15f, r);
#else
    double rd = __builtin_fma((double)kf, -1.5707963267948966, (double)x);
    rd = __builtin_fma((double)kf, -6.123233995736766e-17, rd);
    const float r = (float)rd;
#endif
    const float r2 = r * r;
    float sp = __builtin_fmaf(r2, -1.9515295891e-4f, 8.3321608736e-3f);
    sp = __builtin_fmaf(r2, sp, -1.6666654611e-1f);
    sp = __builtin_fmaf(r * r2, sp, r);
    float cp = __builtin_fmaf(r2, 2.443315711809948e-5f, -1.388731625493765e-3f);
    cp = __builtin_fmaf(r2, cp, 4.166664568298827e-2f);
    cp = __builtin_fmaf(r2 * r2, cp, __builtin_fmaf(r2, -0.5f, 1.0f));
    const int q = (int)kf & 3;
    const float ss = (q & 1) ? cp : sp;
    const float cc = (q & 1) ? sp : cp;
    *s = (q & 2) ? -ss : ss;
    *c = ((q + 1) & 2) ? -cc : cc;
}

// ---------------------------------------------------------------------------
// Philox-4x32-10 counter-based RNG -> uniform float in [0, 1) (24-bit).
// ---------------------------------------------------------------------------
struct Philox4 {
    uint32_t v[4];
};

__device__ __forceinline__ Philox4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                                 uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        uint32_t hi0 = __umulhi(M0, c0), lo0 = M0 * c0;
        uint32_t hi1 = __umulhi(M1, c2), lo1 = M1 * c2;
        uint32_t n0 = hi1 ^ c1 ^ k0;
        uint32_t n1 = lo1;
        uint32_t n2 = hi0 ^ c3 ^ k1;
        uint32_t n3 = lo0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += W0; k1 += W1;
    }
    Philox4 r;
    r.v[0] = c0; r.v[1] = c1; r.v[2] = c2; r.v[3] = c3;
    return r;
}

__device__ __forceinline__ float u32_to_unit(uint32_t x) {
    return (float)(x >> 8) * (1.0f / 16777216.0f);
}

// uniform for element `idx` of stream (seed, counter)
__device__ __forceinline__ float philox_uniform(uint64_t seed, uint64_t counter, uint64_t idx) {
    Philox4 r = philox4x32_10((uint32_t)idx, (uint32_t)(idx >> 32), (uint32_t)counter,
                              (uint32_t)(counter >> 32), (uint32_t)seed, (uint32_t)(seed >> 32));
    return u32_to_unit(r.v[0]);
}

// torch.linspace(start, end, steps) element (CPU float kernel formula).
__device__ __forceinline__ float linspace_at(float start, float end, int steps, int idx) {
#pragma clang fp contract(off)
    if (steps == 1) return start;
    const float step = (end - start) / (float)(steps - 1);
    const int halfway = steps / 2;
    return (idx < halfway) ? start + step * (float)idx : end - step * (float)(steps - idx - 1);
}

// ---------------------------------------------------------------------------
// Epilogue of one output quad (columns n .. n+3 of row m) of the NT linear kernels
// (nerf_linear_fwd / nerf_linear_fwd_x3), in a fixed operation order:
//   v (+ bias) (ReLU) (* ReLU-backward mask) (+ out) -> out, then (MASKOUT) mask bits.
// With NERF_EPI_MASKBITS / NERF_EPI_MASKOUT, aux is a bit mask (N <= 256): row m is 8 uint32
// words at (char*)aux + m * ld_aux; bit b of word 2e + h is (activation at column
// 4 (32 h + b) + e) > 0 — component-major, so that a wave's ballot over its lanes' quads is
// one word.  Otherwise aux is the fp32 activation itself.
typedef float epi_f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned quad_bits(epi_f4 v) {
    return (v.x > 0.f ? 1u : 0u) | (v.y > 0.f ? 2u : 0u) | (v.z > 0.f ? 4u : 0u) | (v.w > 0.f ? 8u : 0u);
}
__device__ __forceinline__ epi_f4 apply_bits(epi_f4 v, unsigned b) {
    v.x = (b & 1u) ? v.x : 0.f; v.y = (b & 2u) ? v.y : 0.f;
    v.z = (b & 4u) ? v.z : 0.f; v.w = (b & 8u) ? v.w : 0.f;
    return v;
}
__device__ __forceinline__ epi_f4 apply_sign(epi_f4 v, epi_f4 x) {
    v.x = x.x > 0.f ? v.x : 0.f; v.y = x.y > 0.f ? v.y : 0.f;
    v.z = x.z > 0.f ? v.z : 0.f; v.w = x.w > 0.f ? v.w : 0.f;
    return v;
}
// 4-bit mask of quad q of a bit-mask row (vector loads)
__device__ __forceinline__ unsigned load_quad_bits(const unsigned char* row, int q) {
    const unsigned* w = reinterpret_cast<const unsigned*>(row) + (q >> 5);
    const int b = q & 31;
    return ((w[0] >> b) & 1u) | (((w[2] >> b) & 1u) << 1) | (((w[4] >> b) & 1u) << 2) | (((w[6] >> b) & 1u) << 3);
}
// Write the bits of a group of G consecutive lanes (G = 64, 32 or 8) holding consecutive
// quads q0 .. q0+G-1 (q0 a multiple of G) of one row.  Every lane of the wave must call it.
template <int G>
__device__ __forceinline__ void store_quad_bits(unsigned char* row, bool row_ok, int q0, unsigned nib) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const unsigned long long b = __ballot((nib >> e) & 1u);
        if (row_ok && (lane & (G - 1)) == 0) {
            unsigned* w = reinterpret_cast<unsigned*>(row) + 2 * e + (q0 >> 5);
            if (G == 64) {
                w[0] = (unsigned)b;
                w[1] = (unsigned)(b >> 32);
            } else if (G == 32) {
                w[0] = (unsigned)(b >> (lane & 32));
            } else {
                reinterpret_cast<unsigned char*>(w)[(q0 & 31) >> 3] = (unsigned char)(b >> (lane & 56));
            }
        }
    }
}

struct EpiOut {
    float* out; int64_t ldo;
    const float* bias;
    const void* aux; int64_t ldaux;
    int M; int N; int epi; int vec_ok;
};

// torch's tanh_backward: g * (1 - y * y), no contraction
__device__ __forceinline__ float tanh_bwd(float g, float y) {
#pragma clang fp contract(off)
    const float yy = y * y;
    return g * (1.0f - yy);
}

// Epilogue of one lane's quad (ok: the quad is in range); returns its (out > 0) bits.  Layer
// outputs are stored nontemporal: they are read back by a later launch, never from these caches,
// and default-policy stores slowed the kernels' counted waits on their own loads (GARF step
// 25.3 -> 24.3 ms; the fused MLP kernel, mlp_fused.hip ST_AUX, far more).
__device__ __forceinline__ unsigned epi_quad_lane(const EpiOut& E, int m, int n, epi_f4 v) {
    const bool bits = (E.epi & (NERF_EPI_MASKBITS | NERF_EPI_MASKOUT)) != 0;
    const unsigned char* mrow = (const unsigned char*)E.aux + (int64_t)m * E.ldaux;
    float* o = E.out + (int64_t)m * E.ldo + n;
    if (E.vec_ok && n + 4 <= E.N) {
        if (E.epi & NERF_EPI_BIAS) v += *reinterpret_cast<const epi_f4*>(E.bias + n);
        if (E.epi & NERF_EPI_RELU) {
            v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
        }
        if (E.epi & NERF_EPI_TANH) {
            v.x = tanhf(v.x); v.y = tanhf(v.y); v.z = tanhf(v.z); v.w = tanhf(v.w);
        }
        if (E.epi & NERF_EPI_TANH_BWD) {
            const epi_f4 y = *reinterpret_cast<const epi_f4*>((const float*)E.aux + (int64_t)m * E.ldaux + n);
            v.x = tanh_bwd(v.x, y.x); v.y = tanh_bwd(v.y, y.y); v.z = tanh_bwd(v.z, y.z); v.w = tanh_bwd(v.w, y.w);
        }
        if (E.epi & NERF_EPI_MASK)
            v = bits ? apply_bits(v, load_quad_bits(mrow, n >> 2))
                     : apply_sign(v, *reinterpret_cast<const epi_f4*>((const float*)E.aux + (int64_t)m * E.ldaux + n));
        if (E.epi & NERF_EPI_ACCUM) v = *reinterpret_cast<const epi_f4*>(o) + v;
        __builtin_nontemporal_store(v, reinterpret_cast<epi_f4*>(o));
        return quad_bits(v);
    }
    const unsigned mb = (bits && (E.epi & NERF_EPI_MASK)) ? load_quad_bits(mrow, n >> 2) : 0u;
    unsigned ob = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        if (n + e >= E.N) break;
        float x = e == 0 ? v.x : (e == 1 ? v.y : (e == 2 ? v.z : v.w));
        if (E.epi & NERF_EPI_BIAS) x = x + E.bias[n + e];
        if (E.epi & NERF_EPI_RELU) x = fmaxf(x, 0.f);
        if (E.epi & NERF_EPI_TANH) x = tanhf(x);
        if (E.epi & NERF_EPI_TANH_BWD) x = tanh_bwd(x, ((const float*)E.aux)[(int64_t)m * E.ldaux + n + e]);
        if (E.epi & NERF_EPI_MASK)
            x = (bits ? ((mb >> e) & 1u) != 0u : ((const float*)E.aux)[(int64_t)m * E.ldaux + n + e] > 0.f) ? x : 0.f;
        if (E.epi & NERF_EPI_ACCUM) x = o[e] + x;
        o[e] = x;
        ob |= (x > 0.f ? 1u : 0u) << e;
    }
    return ob;
}

// Quad epilogue for kernels whose epilogue maps G consecutive lanes to G consecutive quads
// of one row (G-aligned).  Every lane of the wave calls it; ok = this lane's quad is in range.
template <int G>
__device__ __forceinline__ void epi_quad(const EpiOut& E, bool ok, int m, int n, epi_f4 v) {
    const unsigned nib = ok ? epi_quad_lane(E, m, n, v) : 0u;
    if (E.epi & NERF_EPI_MASKOUT)
        store_quad_bits<G>((unsigned char*)E.aux + (int64_t)m * E.ldaux, m < E.M, (n >> 2) & ~(G - 1), nib);
}

// Column sums of per-row-tile fp64 partials [slabs][N] for the Gaussian activation's
// inverse-std gradient (gauss.hip): ds_n (+)= (float)(sum_i partial[i][n]) * (2 * s_n), summed in
// a fixed order (chunks of slabs in parallel, then the chunks in order).  scratch holds
// gauss_reduce_scratch(N) bytes.
size_t gauss_reduce_scratch(int N);
int gauss_reduce(const double* partial, int64_t slabs, int N, const float* s, float* ds, int accumulate,
                 double* scratch, hipStream_t stream);

}  // namespace nerf
