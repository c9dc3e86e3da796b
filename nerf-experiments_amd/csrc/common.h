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

}  // namespace nerf
