// Per-level corner arithmetic of the multiresolution hash grid (a9: INGPTable / INGPEncoding,
// 3d-ingp/model.py:14-121 as SURVEY.md §8(a) a9 restates it; oracle/hashgrid_oracle.py), shared by
// the stand-alone kernels (hashgrid.hip) and the features generated inside the fused field-MLP
// forward (mlp_fused.hip): the same instructions, so both produce bitwise the same features.
#pragma once
#include "common.h"

namespace nerf {

struct Corners {
    int idx[8];           // table rows (< T < 2^31)
    float w[8];
};

// rows of a level's table: (r+1)^3 when bijective, else T
__host__ __device__ inline int64_t level_rows(int r, int T) {
    const int64_t r1 = r + 1;
    return r1 * r1 * r1 <= T ? r1 * r1 * r1 : T;
}

// the hash of one corner: int64 (x*pi1) ^ (y*pi2) ^ (z*pi3) with wrap-around products and the
// non-negative remainder modulo T (torch.remainder); modulo a power of two that is the low bits,
// which only the low 32 bits of corners and primes determine (two's complement): 32-bit arithmetic
__device__ __forceinline__ int hash_row(const long long* cc, long long pr0, long long pr1, long long pr2, int T,
                                        bool pow2) {
    if (pow2) {
        const unsigned h = ((unsigned)cc[0] * (unsigned)pr0) ^ ((unsigned)cc[1] * (unsigned)pr1) ^
                           ((unsigned)cc[2] * (unsigned)pr2);
        return (int)(h & (unsigned)(T - 1));
    }
    const unsigned long long h = ((unsigned long long)cc[0] * (unsigned long long)pr0) ^
                                 ((unsigned long long)cc[1] * (unsigned long long)pr1) ^
                                 ((unsigned long long)cc[2] * (unsigned long long)pr2);
    const long long m = (long long)h % (long long)T;
    return (int)(m < 0 ? m + T : m);
}

// x_hat = (x / 8 + 0.5) * r (normalize) or x * r; corners floor(x_hat) + {0,1}^3 in the reference's
// stacking order (z fastest), their rows (bijective: clipped x + (r+1) y + (r+1)^2 z; else the
// hash) and weights prod_d (1 - |x_hat_d - corner_d|) on the unclipped corner.
// The corner coordinates are the reference's int64 floor values; while |x_hat| < 2^30 (any position
// within 2^26 of the scene at r <= 2^20, normalised by 8) they are carried in 32-bit integers, whose
// sums, conversions to float and low 32 bits of the hash products equal the 64-bit ones exactly, and
// the two per-dimension weight factors are formed once (the same expressions); beyond that, or for a
// table size that is not a power of two (64-bit remainder), the 64-bit form.
template <typename PR>
__device__ __forceinline__ Corners level_corners(const float* p, int normalize, int r, int T, const PR& primes) {
#pragma clang fp contract(off)
    Corners c;
    float xh[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) xh[j] = (normalize ? (p[j] / 8.0f + 0.5f) : p[j]) * (float)r;
    const bool bij = (long long)(r + 1) * (r + 1) * (r + 1) <= (long long)T;
    const bool pow2 = (T & (T - 1)) == 0;
    const bool small = fabsf(xh[0]) < 1073741824.0f && fabsf(xh[1]) < 1073741824.0f && fabsf(xh[2]) < 1073741824.0f;
    if (small && (bij || pow2)) {
        int b[3];
        float f0[3], f1[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            b[j] = (int)floorf(xh[j]);
            f0[j] = 1.0f - fabsf(xh[j] - (float)b[j]);
            f1[j] = 1.0f - fabsf(xh[j] - (float)(b[j] + 1));
        }
        // the row form is uniform per level: one branch for all eight corners
        if (bij) {
            const int r1 = r + 1;
            int qx[2], qy[2], qz[2];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int vx = b[0] + e, vy = b[1] + e, vz = b[2] + e;
                qx[e] = vx < 0 ? 0 : (vx > r ? r : vx);
                qy[e] = r1 * (vy < 0 ? 0 : (vy > r ? r : vy));
                qz[e] = r1 * r1 * (vz < 0 ? 0 : (vz > r ? r : vz));
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) c.idx[k] = qx[(k >> 2) & 1] + qy[(k >> 1) & 1] + qz[k & 1];
        } else {
            const unsigned pr0 = (unsigned)(long long)primes[0], pr1 = (unsigned)(long long)primes[1],
                           pr2 = (unsigned)(long long)primes[2];
            unsigned hxy[4], hz[2];
#pragma unroll
            for (int e = 0; e < 2; ++e) hz[e] = (unsigned)(b[2] + e) * pr2;
#pragma unroll
            for (int e = 0; e < 4; ++e) hxy[e] = ((unsigned)(b[0] + (e >> 1)) * pr0) ^ ((unsigned)(b[1] + (e & 1)) * pr1);
#pragma unroll
            for (int k = 0; k < 8; ++k) c.idx[k] = (int)((hxy[k >> 1] ^ hz[k & 1]) & (unsigned)(T - 1));
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int ex = (k >> 2) & 1, ey = (k >> 1) & 1, ez = k & 1;   // z fastest
            c.w[k] = ((ex ? f1[0] : f0[0]) * (ey ? f1[1] : f0[1])) * (ez ? f1[2] : f0[2]);
        }
        return c;
    }
    long long base[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) base[j] = (long long)floorf(xh[j]);
    const long long pr0 = (long long)primes[0], pr1 = (long long)primes[1], pr2 = (long long)primes[2];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        long long cc[3];
        float dw[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            cc[j] = base[j] + ((k >> (2 - j)) & 1);         // z fastest: the reference's stacking order
            dw[j] = 1.0f - fabsf(xh[j] - (float)cc[j]);
        }
        c.w[k] = (dw[0] * dw[1]) * dw[2];
        if (bij) {
            const int r1 = r + 1;
            int q[3];
#pragma unroll
            for (int j = 0; j < 3; ++j) q[j] = cc[j] < 0 ? 0 : (cc[j] > r ? r : (int)cc[j]);
            c.idx[k] = q[0] + r1 * q[1] + r1 * r1 * q[2];
        } else {
            c.idx[k] = hash_row(cc, pr0, pr1, pr2, T, pow2);
        }
    }
    return c;
}

}  // namespace nerf
