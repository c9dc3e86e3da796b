// Multiresolution hash-grid encoding (a9, config C5): INGPTable / INGPEncoding of the
// reference's 3d-ingp/model.py:14-121 (the interface VERDICT r2 states; the arithmetic restated
// from SURVEY.md §8(a) a9 and pinned on its 2-D copy, 2d-ingp/model.py:13-115 — see
// oracle/hashgrid_oracle.py).  Contract in include/nerf_amd.h.
//
// Table layout = the reference's parameters: one [rows_l][F] table per level, rows_l = (r+1)^3 for
// a bijective level ((r+1)^3 <= T), T otherwise, the levels packed back to back (row offsets
// computed on the host from (res, T)), so INGPEncoding's per-level Parameters are views of one
// buffer.
//
// Forward: one thread per (sample, level), consecutive threads = consecutive levels of one sample,
// so a sample's L*F features are written by L adjacent threads as one contiguous row.  Per level:
// x_hat = (x / 8 + 0.5) * r (INGPEncoding; x * r for INGPTable on normalised points), the 8
// corners floor(x_hat) + {0,1}^3, their table rows (bijective: x + (r+1) y + (r+1)^2 z of the corner
// clipped to [0, r]; else the product-xor hash with primes (pi1, pi2, pi3) modulo T computed as the
// reference's int64 tensor arithmetic with a non-negative remainder), weights prod_d (1 - |x_hat_d -
// corner_d|) on the unclipped corner, features summed over the corners in the reference's stacking
// order (i, j, k) = (0,0,0), (0,0,1), (0,1,0), ... — z fastest, corner c = 4 dx + 2 dy + dz — with
// separate multiplies and adds (no contraction), as th.sum over the stacked corners adds them.
//
// Backward (the table gradient; positions receive none): every contribution w * g is rounded to a
// 64-bit fixed-point integer at a scale 2^s chosen from the batch's max |g| so that no table entry
// can overflow, and added with integer atomics; integer addition is associative, so the result is
// independent of the order in which the atomics land (deterministic, unlike float atomics).
#include <stdlib.h>

#include "common.h"
#include "hashgrid_common.h"

namespace {
using namespace nerf;

struct HashArgs {
    nerf_hashgrid_params p;
    int64_t off[NERF_HASHGRID_MAX_LEVELS];          // first row of each level in the packed table
    const float* x;
    const float* o;
    const float* d;
    const float* t0;
    const float* t1;
    int64_t n;
    int spr;
    const float4* pos;                              // backward: position records (or null)
};

__device__ __forceinline__ void sample_position(const HashArgs& a, int64_t n, float* p) {
#pragma clang fp contract(off)
    if (a.x != nullptr) {
        p[0] = a.x[n * 3 + 0];
        p[1] = a.x[n * 3 + 1];
        p[2] = a.x[n * 3 + 2];
        return;
    }
    const int64_t ray = n / a.spr;
    const float tq = (a.p.query == 0) ? a.t0[n] : (a.t0[n] + a.t1[n]) / 2.0f;
#pragma unroll
    for (int j = 0; j < 3; ++j) p[j] = a.o[ray * 3 + j] + tq * a.d[ray * 3 + j];
}

__global__ __launch_bounds__(256) void hashgrid_fwd_kernel(HashArgs a, const float* __restrict__ table,
                                                           float* __restrict__ out, int64_t ld) {
#pragma clang fp contract(off)
    const int L = a.p.levels, F = a.p.features, T = a.p.table_size;
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t n = t / L;
    const int l = (int)(t - n * L);
    if (n >= a.n) return;
    float p[3];
    sample_position(a, n, p);
    const Corners c = level_corners(p, a.p.normalize, a.p.res[l], T, a.p.primes);
    const float* tab = table + a.off[l] * F;
    float acc[NERF_HASHGRID_MAX_FEATURES];
#pragma unroll
    for (int f = 0; f < NERF_HASHGRID_MAX_FEATURES; ++f) acc[f] = 0.0f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
#pragma unroll
        for (int f = 0; f < NERF_HASHGRID_MAX_FEATURES; ++f)
            if (f < F) acc[f] = acc[f] + c.w[k] * tab[(int64_t)c.idx[k] * F + f];
    }
    float* o = out + n * ld + (int64_t)l * F;
#pragma unroll
    for (int f = 0; f < NERF_HASHGRID_MAX_FEATURES; ++f)
        if (f < F) o[f] = acc[f];
}

// The same features with the threads of a wave on ONE level and 64 consecutive samples (grid y =
// level): a wave's gathers all hit one level's table and, along a ray, neighbouring cells (at the
// coarse levels the same rows), instead of 16 tables per 16 threads; each thread writes its F
// features of one row (rows of a sample complete in L2 from the levels' waves).  Bitwise the
// kernel above (same per-level arithmetic).
__global__ __launch_bounds__(256) void hashgrid_fwd_level_kernel(HashArgs a, const float* __restrict__ table,
                                                                 float* __restrict__ out, int64_t ld) {
#pragma clang fp contract(off)
    const int F = a.p.features, T = a.p.table_size;
    const int l = blockIdx.y;
    const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (n >= a.n) return;
    float p[3];
    sample_position(a, n, p);
    const Corners c = level_corners(p, a.p.normalize, a.p.res[l], T, a.p.primes);
    const float* tab = table + a.off[l] * F;
    float acc[NERF_HASHGRID_MAX_FEATURES];
#pragma unroll
    for (int f = 0; f < NERF_HASHGRID_MAX_FEATURES; ++f) acc[f] = 0.0f;
    if (F == 2) {
        // the 8 rows' feature pairs as 8-byte loads, all issued before the sums
        float2 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = *reinterpret_cast<const float2*>(tab + (int64_t)c.idx[k] * 2);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            acc[0] = acc[0] + c.w[k] * v[k].x;
            acc[1] = acc[1] + c.w[k] * v[k].y;
        }
        *reinterpret_cast<float2*>(out + n * ld + (int64_t)l * 2) = make_float2(acc[0], acc[1]);
        return;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
#pragma unroll
        for (int f = 0; f < NERF_HASHGRID_MAX_FEATURES; ++f)
            if (f < F) acc[f] = acc[f] + c.w[k] * tab[(int64_t)c.idx[k] * F + f];
    }
    float* o = out + n * ld + (int64_t)l * F;
#pragma unroll
    for (int f = 0; f < NERF_HASHGRID_MAX_FEATURES; ++f)
        if (f < F) o[f] = acc[f];
}

// The same features, 64 samples per workgroup with one wave per level (64 L threads): a wave's
// gathers hit one level's table (at the coarse levels neighbouring samples of a ray share rows),
// and the workgroup's results are staged in LDS and written as whole [64][ld] output rows — the
// kernel above writes each 128-B row as 16 scattered 8-B pieces from 16 waves of the level grid,
// which the caches cannot hold together (write amplification).  Bitwise the kernels above.
constexpr int TILE_SAMPLES = 64;
template <int F>
__global__ __launch_bounds__(1024) void hashgrid_fwd_tile_kernel(HashArgs a, const float* __restrict__ table,
                                                                 float* __restrict__ out, int64_t ld) {
#pragma clang fp contract(off)
    __shared__ float rows[TILE_SAMPLES * (16 * F + 1)];
    const int L = a.p.levels, T = a.p.table_size, cols = L * F, rld = cols + 1;
    const int l = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
    const int64_t n0 = (int64_t)blockIdx.x * TILE_SAMPLES;
    const int64_t n = n0 + lane;
    if (n < a.n) {
        float p[3];
        sample_position(a, n, p);
        const Corners c = level_corners(p, a.p.normalize, a.p.res[l], T, a.p.primes);
        const float* tab = table + a.off[l] * F;
        float v[8][F];
#pragma unroll
        for (int k = 0; k < 8; ++k)
#pragma unroll
            for (int f = 0; f < F; ++f) v[k][f] = tab[(int64_t)c.idx[k] * F + f];   // all 8 F loads first
        float acc[F];
#pragma unroll
        for (int f = 0; f < F; ++f) acc[f] = 0.0f;
#pragma unroll
        for (int k = 0; k < 8; ++k)
#pragma unroll
            for (int f = 0; f < F; ++f) acc[f] = acc[f] + c.w[k] * v[k][f];
#pragma unroll
        for (int f = 0; f < F; ++f) rows[lane * rld + l * F + f] = acc[f];
    }
    __syncthreads();
    const int64_t left = a.n - n0;
    const int nr = left < TILE_SAMPLES ? (int)left : TILE_SAMPLES;
    for (int e = threadIdx.x; e < nr * cols; e += blockDim.x) {
        const int r = e / cols, cc = e - r * cols;
        out[(n0 + r) * ld + cc] = rows[r * rld + cc];
    }
}

// max |grad_out| over the batch as the bits of a non-negative float (order-preserving as uint32);
// non-finite values land above every finite one
template <int V>
__global__ __launch_bounds__(256) void hashgrid_gmax_kernel(const float* __restrict__ g, int64_t ld, int64_t n,
                                                            int cols, unsigned* __restrict__ gmax) {
    // V-float vectors of the [n, cols] block of rows of stride ld; 32-bit index math when it fits
    const int cv = cols / V;
    const int64_t total = n * cv;
    const bool small = total < ((int64_t)1 << 31);
    unsigned m = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const int64_t r = small ? (int64_t)((unsigned)i / (unsigned)cv) : i / cv;
        const float* p = g + r * ld + (i - r * cv) * V;
        float v[V];
        if constexpr (V == 4) {
            const float4 q = *reinterpret_cast<const float4*>(p);
            v[0] = q.x, v[1] = q.y, v[2] = q.z, v[3] = q.w;
        } else {
            v[0] = p[0];
        }
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const unsigned b = __float_as_uint(fabsf(v[j]));
            m = b > m ? b : m;
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned o = __shfl_xor(m, off, 64);
        m = o > m ? o : m;
    }
    // one atomic per block: same-address atomics serialise at the memory side (one per wave of
    // 16 K waves took ~190 us)
    __shared__ unsigned wm[4];
    if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        m = wm[0] > wm[1] ? wm[0] : wm[1];
        m = m > wm[2] ? m : wm[2];
        m = m > wm[3] ? m : wm[3];
        if (m != 0) atomicMax(gmax, m);
    }
}

// The max as above, and grad_out restaged level-major, gt[l][n][f] (the backward's part walks read
// one level's F values per sample: from the [n][ld] rows that is 4 F bytes out of every 128-B line,
// re-read by every part of the level; level-major they are contiguous).  64 rows per workgroup:
// coalesced row reads into LDS, coalesced level-run writes out of it.
template <int F>
__global__ __launch_bounds__(256) void hashgrid_gtr_kernel(const float* __restrict__ g, int64_t ld, int64_t n, int L,
                                                           float* __restrict__ gt, unsigned* __restrict__ gmax) {
    __shared__ float rows[TILE_SAMPLES * (NERF_HASHGRID_MAX_LEVELS * F + 1)];
    __shared__ unsigned wm[4];
    const int cols = L * F, rld = cols + 1;
    const int64_t n0 = (int64_t)blockIdx.x * TILE_SAMPLES;
    const int nr = n - n0 < TILE_SAMPLES ? (int)(n - n0) : TILE_SAMPLES;
    unsigned m = 0;
    for (int e = threadIdx.x; e < nr * cols; e += 256) {
        const int r = e / cols, c = e - r * cols;
        const float v = g[(n0 + r) * ld + c];
        rows[r * rld + c] = v;
        const unsigned b = __float_as_uint(fabsf(v));
        m = b > m ? b : m;
    }
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned o = __shfl_xor(m, off, 64);
        m = o > m ? o : m;
    }
    if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        m = wm[0] > wm[1] ? wm[0] : wm[1];
        m = m > wm[2] ? m : wm[2];
        m = m > wm[3] ? m : wm[3];
        // same-address atomics serialise at the memory side (one per block of 20 K blocks: ~0.2 ms):
        // only a block whose max exceeds the running one adds its atomic
        if (m != 0 && m > __hip_atomic_load(gmax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(gmax, m);
    }
    const int run = nr * F;                       // one level's values of the workgroup's rows
    for (int e = threadIdx.x; e < L * run; e += 256) {
        const int l = e / run, q = e - l * run;
        const int r = q / F, f = q - r * F;
        gt[((int64_t)l * n + n0) * F + q] = rows[r * rld + l * F + f];
    }
}

// fixed-point exponent s with 8 * n * gmax * 2^s < 2^62 (no entry can overflow); -1000 flags a
// non-finite gradient
__device__ __forceinline__ int fixed_shift(unsigned gmax_bits, int64_t n) {
    const float gm = __uint_as_float(gmax_bits);
    if (!(gm < INFINITY)) return -1000;
    if (gm == 0.0f) return 60;
    const double bound = 8.0 * (double)n * (double)gm;
    int e;
    frexp(bound, &e);                       // bound < 2^e
    int s = 62 - e;
    return s > 120 ? 120 : s;
}

// Backward as (level, part, slab) workgroups: a part is a run of PART_ENTRIES accumulators of one
// level's table (bijective levels need only (r+1)^3 rows) held in LDS as 64-bit fixed-point sums; the
// workgroup walks its slab of samples, adds every corner contribution whose row falls in its part
// with LDS integer atomics, then adds the part to the global accumulators with one contiguous pass of
// atomics.  Global atomics scattered one lane per row run ~17x below their contiguous rate (they
// execute at the memory side, one request per lane), so the scattered adds stay on chip and only
// coalesced ones leave it; positions and corners are recomputed per part (cheap VALU).
#ifndef NERF_HG_PART_ENTRIES
#define NERF_HG_PART_ENTRIES 20480
#endif
// all 160 KiB of LDS as int64 accumulators (16384: 8 parts per hashed level of 2^16 rows x 2
// features, 20480: 7 — every part re-walks its slab's samples, so fewer parts is less work)
constexpr int PART_ENTRIES = NERF_HG_PART_ENTRIES;
constexpr int BWD_THREADS = 1024;

struct BwdPlan {
    int start[NERF_HASHGRID_MAX_LEVELS + 1];        // prefix of parts per level
    int rows_per_part;
    int parts;                                      // parts of all levels (workgroups per slab)
    int64_t slab;                                   // samples per slab
    int64_t nslab;                                  // slabs (the persistent walk's items: parts x nslab)
};


// Each thread takes BWD_UNROLL samples per trip and issues all their loads (positions or ray
// origin / direction / interval, and the F gradient values) before any is used, so a trip costs one
// memory round trip instead of one per load.
constexpr int BWD_UNROLL = 4;

// round-to-nearest-even of |x| < 2^51 to int64 (llrint's value): adding 1.5 * 2^52 rounds x to an
// integer in the binade [2^52, 2^53), whose mantissa bits then hold it — 3 instructions, not ~8
__device__ __forceinline__ long long rint_fixed(double x) {
#pragma clang fp contract(off)
    const double m = 6755399441055744.0;
    return __builtin_bit_cast(long long, x + m) - __builtin_bit_cast(long long, m);
}

// Sample positions as float4 records (x, y, z, 0), computed once per backward call for the ray
// form — as sample_position computes them — instead of once per part walk (97 parts at C5)
__global__ __launch_bounds__(256) void hashgrid_pos_kernel(HashArgs a, float4* __restrict__ pos) {
    const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (n >= a.n) return;
    float p[3];
    sample_position(a, n, p);
    pos[n] = make_float4(p[0], p[1], p[2], 0.0f);
}

#ifndef NERF_HG_SKIPZERO
#define NERF_HG_SKIPZERO 0
#endif
#ifndef NERF_HG_QUEUE
#define NERF_HG_QUEUE 0
#endif

// One trip's corner contributions of BWD_UNROLL samples (nb + u BWD_THREADS) whose rows fall in the
// part [row0, row0 + prow), added to the LDS accumulators.  SMALL: a.n >= 256, so that every
// contribution |w g 2^s| <= gmax 2^s < 2^62 / (8 n) <= 2^51 rounds with rint_fixed.
template <int F, bool SMALL>
__device__ __forceinline__ void add_trip(const HashArgs& a, int res, int64_t row0, int prow, double scale, int64_t nb,
                                         int64_t n_end, const float (&p)[BWD_UNROLL][3],
                                         const float (&gv)[BWD_UNROLL][F], unsigned long long* part) {
#pragma clang fp contract(off)
#pragma unroll
    for (int u = 0; u < BWD_UNROLL; ++u) {
        if (nb + u * BWD_THREADS >= n_end) continue;
        const Corners c = level_corners(p[u], a.p.normalize, res, a.p.table_size, a.p.primes);
        // w g 2^s = w (g 2^s): both products exact in fp64 (24-bit mantissas, power-of-two scale)
        double gs[F];
#pragma unroll
        for (int f = 0; f < F; ++f) gs[f] = (double)gv[u][f] * scale;
        int rel[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) rel[k] = c.idx[k] - (int)row0;     // rows, part bounds < T < 2^31
        if (NERF_HG_QUEUE) {
            // each lane queues its in-range corners and the wave issues one add per queued-corner
            // round (its longest queue), selecting the corner's row and weight per round
            unsigned pend = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if ((unsigned)rel[k] < (unsigned)prow) pend |= 1u << k;
            while (pend != 0u) {
                const int k = __builtin_ctz(pend);
                pend &= pend - 1u;
                int rk = rel[0];
                float wk = c.w[0];
#pragma unroll
                for (int j = 1; j < 8; ++j)
                    if (k == j) {
                        rk = rel[j];
                        wk = c.w[j];
                    }
#pragma unroll
                for (int f = 0; f < F; ++f) {
                    // one rounding to the fixed-point grid
                    const double x = (double)wk * gs[f];
                    const long long q = SMALL ? rint_fixed(x) : llrint(x);
                    if (q != 0) atomicAdd(&part[rk * F + f], (unsigned long long)q);
                }
            }
        } else {
            // corner by corner, the lanes whose corner falls in the part (a corner no lane holds is
            // skipped): no per-round selection of the row and weight
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                if ((unsigned)rel[k] < (unsigned)prow) {
                    const double wk = (double)c.w[k];
#pragma unroll
                    for (int f = 0; f < F; ++f) {
                        const double x = wk * gs[f];
                        const long long q = SMALL ? rint_fixed(x) : llrint(x);
                        if (!NERF_HG_SKIPZERO || q != 0) atomicAdd(&part[rel[k] * F + f], (unsigned long long)q);
                    }
                }
            }
        }
    }
}

#ifndef NERF_HG_PIPE
#define NERF_HG_PIPE 1
#endif

// One part's walk over the samples [n_begin, n_end): every corner contribution whose row falls in
// the part [row0, row0 + prow) of level l, added to the LDS accumulators.  g: the level's F values of
// sample n at gt[n F + f] when restaged level-major (gt != null), else at g[n ld + l F + f].
// Positions from the float4 records (a.pos, hashgrid_pos_kernel; NERF_HG_POS=1) when present: two
// loads per sample, the next trip's issued before this trip's corners (NERF_HG_PIPE); measured no
// faster than the walks' own position arithmetic (profiles/r04n: the walk is not load-latency
// bound); else from the inputs (x, or ray o / d and the interval).
template <int F, bool SMALL>
__device__ __forceinline__ void walk_part(const HashArgs& a, int l, int res, int64_t row0, int prow, double scale,
                                          int64_t n_begin, int64_t n_end, const float* __restrict__ g, int64_t ld,
                                          const float* __restrict__ gt, unsigned long long* part) {
#pragma clang fp contract(off)
    constexpr int STEP = BWD_UNROLL * BWD_THREADS;
    const bool rays = a.x == nullptr, mid = a.p.query != 0, small = a.n < ((int64_t)1 << 31);
    if (a.pos != nullptr) {
        float4 qn[BWD_UNROLL];
        float gn[BWD_UNROLL][F];
        // indices clamped into the range, so every load is in bounds; samples past it are masked
        auto load = [&](int64_t base) __attribute__((always_inline)) {
#pragma unroll
            for (int u = 0; u < BWD_UNROLL; ++u) {
                const int64_t n = base + threadIdx.x + u * BWD_THREADS < n_end ? base + threadIdx.x + u * BWD_THREADS
                                                                               : n_end - 1;
                qn[u] = a.pos[n];
#pragma unroll
                for (int f = 0; f < F; ++f) gn[u][f] = gt ? gt[n * F + f] : g[n * ld + (int64_t)l * F + f];
            }
        };
        load(n_begin);
        for (int64_t base = n_begin; base < n_end; base += STEP) {
            float p[BWD_UNROLL][3], gv[BWD_UNROLL][F];
#pragma unroll
            for (int u = 0; u < BWD_UNROLL; ++u) {
                p[u][0] = qn[u].x, p[u][1] = qn[u].y, p[u][2] = qn[u].z;
#pragma unroll
                for (int f = 0; f < F; ++f) gv[u][f] = gn[u][f];
            }
            if (NERF_HG_PIPE && base + STEP < n_end) load(base + STEP);
            add_trip<F, SMALL>(a, res, row0, prow, scale, base + threadIdx.x, n_end, p, gv, part);
            if (!NERF_HG_PIPE && base + STEP < n_end) load(base + STEP);
        }
        return;
    }
    for (int64_t base = n_begin; base < n_end; base += STEP) {
        const int64_t nb = base + threadIdx.x;
        float p[BWD_UNROLL][3], gv[BWD_UNROLL][F];
        // loads first (indices clamped into the range, so every load is in bounds) ...
        if (rays) {
            float t0[BWD_UNROLL], t1[BWD_UNROLL], o[BWD_UNROLL][3], d[BWD_UNROLL][3];
#pragma unroll
            for (int u = 0; u < BWD_UNROLL; ++u) {
                const int64_t n = nb + u * BWD_THREADS < n_end ? nb + u * BWD_THREADS : n_end - 1;
                const int64_t ray = small ? (int64_t)((unsigned)n / (unsigned)a.spr) : n / a.spr;
                t0[u] = a.t0[n];
                t1[u] = mid ? a.t1[n] : 0.0f;
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    o[u][j] = a.o[ray * 3 + j];
                    d[u][j] = a.d[ray * 3 + j];
                }
#pragma unroll
                for (int f = 0; f < F; ++f) gv[u][f] = gt ? gt[n * F + f] : g[n * ld + (int64_t)l * F + f];
            }
            // ... then the positions, as sample_position computes them
#pragma unroll
            for (int u = 0; u < BWD_UNROLL; ++u) {
                const float tq = mid ? (t0[u] + t1[u]) / 2.0f : t0[u];
#pragma unroll
                for (int j = 0; j < 3; ++j) p[u][j] = o[u][j] + tq * d[u][j];
            }
        } else {
#pragma unroll
            for (int u = 0; u < BWD_UNROLL; ++u) {
                const int64_t n = nb + u * BWD_THREADS < n_end ? nb + u * BWD_THREADS : n_end - 1;
#pragma unroll
                for (int j = 0; j < 3; ++j) p[u][j] = a.x[n * 3 + j];
#pragma unroll
                for (int f = 0; f < F; ++f) gv[u][f] = gt ? gt[n * F + f] : g[n * ld + (int64_t)l * F + f];
            }
        }
        add_trip<F, SMALL>(a, res, row0, prow, scale, nb, n_end, p, gv, part);
    }
}

// The same walk with each thread on BWD_UNROLL CONSECUTIVE samples (one ray's neighbours) and a
// run-length merge per corner slot: a corner whose row equals the previous sample's corner k adds
// its fixed-point contribution to a register sum, which goes to the LDS accumulator once the row
// changes (or at the end).  At the coarse levels the samples of a ray share cells, so most of their
// LDS atomics — same-address atomics, serialised by the LDS — disappear; the integer sums are
// associative, so the result is bitwise that of walk_part.
template <int F>
__device__ __forceinline__ void walk_part_merged(const HashArgs& a, int l, int res, int64_t row0, int prow, double scale,
                                                 int64_t n_begin, int64_t n_end, const float* __restrict__ g,
                                                 int64_t ld, const float* __restrict__ gt, unsigned long long* part) {
#pragma clang fp contract(off)
    const int T = a.p.table_size;
    const bool rays = a.x == nullptr, mid = a.p.query != 0, small = a.n < ((int64_t)1 << 31);
    for (int64_t base = n_begin; base < n_end; base += BWD_UNROLL * BWD_THREADS) {
        const int64_t nb = base + (int64_t)threadIdx.x * BWD_UNROLL;
        float p[BWD_UNROLL][3], gv[BWD_UNROLL][F];
        if (rays) {
            float t0[BWD_UNROLL], t1[BWD_UNROLL], o[BWD_UNROLL][3], d[BWD_UNROLL][3];
#pragma unroll
            for (int u = 0; u < BWD_UNROLL; ++u) {
                const int64_t n = nb + u < n_end ? nb + u : n_end - 1;
                const int64_t ray = small ? (int64_t)((unsigned)n / (unsigned)a.spr) : n / a.spr;
                t0[u] = a.t0[n];
                t1[u] = mid ? a.t1[n] : 0.0f;
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    o[u][j] = a.o[ray * 3 + j];
                    d[u][j] = a.d[ray * 3 + j];
                }
#pragma unroll
                for (int f = 0; f < F; ++f) gv[u][f] = gt ? gt[n * F + f] : g[n * ld + (int64_t)l * F + f];
            }
#pragma unroll
            for (int u = 0; u < BWD_UNROLL; ++u) {
                const float tq = mid ? (t0[u] + t1[u]) / 2.0f : t0[u];
#pragma unroll
                for (int j = 0; j < 3; ++j) p[u][j] = o[u][j] + tq * d[u][j];
            }
        } else {
#pragma unroll
            for (int u = 0; u < BWD_UNROLL; ++u) {
                const int64_t n = nb + u < n_end ? nb + u : n_end - 1;
#pragma unroll
                for (int j = 0; j < 3; ++j) p[u][j] = a.x[n * 3 + j];
#pragma unroll
                for (int f = 0; f < F; ++f) gv[u][f] = gt ? gt[n * F + f] : g[n * ld + (int64_t)l * F + f];
            }
        }
        // run-length slots per corner: the row (relative to the part; -1 = none) and its sums
        int srow[8];
        long long sq[8][F];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            srow[k] = -1;
#pragma unroll
            for (int f = 0; f < F; ++f) sq[k][f] = 0;
        }
        auto flush = [&](unsigned pend) __attribute__((always_inline)) {
            // one LDS add per queued round (the wave's longest queue), as walk_part
            while (pend != 0u) {
                const int k = __builtin_ctz(pend);
                pend &= pend - 1u;
                int rk = srow[0];
                long long qk[F];
#pragma unroll
                for (int f = 0; f < F; ++f) qk[f] = sq[0][f];
#pragma unroll
                for (int j = 1; j < 8; ++j)
                    if (k == j) {
                        rk = srow[j];
#pragma unroll
                        for (int f = 0; f < F; ++f) qk[f] = sq[j][f];
                    }
#pragma unroll
                for (int f = 0; f < F; ++f)
                    if (qk[f] != 0) atomicAdd(&part[rk * F + f], (unsigned long long)qk[f]);
            }
        };
#pragma unroll
        for (int u = 0; u < BWD_UNROLL; ++u) {
            if (nb + u >= n_end) break;
            const Corners c = level_corners(p[u], a.p.normalize, res, T, a.p.primes);
            int rel[8];
            unsigned change = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int64_t r = (int64_t)c.idx[k] - row0;
                rel[k] = (uint64_t)r < (uint64_t)prow ? (int)r : -1;
                if (rel[k] != srow[k] && srow[k] >= 0) change |= 1u << k;
            }
            flush(change);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const bool same = rel[k] == srow[k];
#pragma unroll
                for (int f = 0; f < F; ++f) {
                    // w * g is exact in fp64 (two 24-bit mantissas); one rounding to the fixed-point grid
                    const long long q = rel[k] >= 0 ? llrint((double)c.w[k] * (double)gv[u][f] * scale) : 0;
                    sq[k][f] = same ? sq[k][f] + q : q;
                }
                srow[k] = rel[k];
            }
        }
        unsigned rest = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (srow[k] >= 0) rest |= 1u << k;
        flush(rest);
    }
}

// the part's accumulators out to the global ones: one contiguous pass of atomics
template <int F>
__device__ __forceinline__ void flush_part(const HashArgs& a, int l, int64_t row0, int prow,
                                           const unsigned long long* part, unsigned long long* __restrict__ acc) {
    unsigned long long* dst = acc + (a.off[l] + row0) * F;
    for (int e = threadIdx.x; e < prow * F; e += BWD_THREADS) {
        const unsigned long long v = part[e];
        if (v != 0ull) atomicAdd(dst + e, v);
    }
}

__device__ __forceinline__ void part_of(const HashArgs& a, const BwdPlan& pl, int w, int& l, int64_t& row0, int& prow) {
    l = 0;
    while (w >= pl.start[l + 1]) ++l;
    row0 = (int64_t)(w - pl.start[l]) * pl.rows_per_part;
    const int64_t rows = level_rows(a.p.res[l], a.p.table_size) - row0;
    prow = (int)(rows < pl.rows_per_part ? rows : pl.rows_per_part);
}

// One workgroup per (part, slab).  MERGED: walk_part_merged (consecutive samples per thread).
template <int F, bool MERGED>
__global__ __launch_bounds__(BWD_THREADS) void hashgrid_bwd_kernel(HashArgs a, BwdPlan pl, const float* __restrict__ g,
                                                                   int64_t ld, const float* __restrict__ gt,
                                                                   const unsigned* __restrict__ gmax,
                                                                   unsigned long long* __restrict__ acc) {
    __shared__ unsigned long long part[PART_ENTRIES];
    const int w = (int)(blockIdx.x % (unsigned)pl.parts);
    const int64_t slab = blockIdx.x / (unsigned)pl.parts;
    int l, prow;
    int64_t row0;
    part_of(a, pl, w, l, row0, prow);
    const int s = fixed_shift(*gmax, a.n);
    if (s == -1000) return;                         // uniform: the finish pass writes NaN
    const double scale = ldexp(1.0, s);
    for (int e = threadIdx.x; e < prow * F; e += BWD_THREADS) part[e] = 0ull;
    __syncthreads();
    const int64_t n1 = (slab + 1) * pl.slab < a.n ? (slab + 1) * pl.slab : a.n;
    if constexpr (MERGED)
        walk_part_merged<F>(a, l, a.p.res[l], row0, prow, scale, slab * pl.slab, n1, g, ld,
                            gt ? gt + (int64_t)l * a.n * F : nullptr, part);
    else if (a.n >= 256)
        walk_part<F, true>(a, l, a.p.res[l], row0, prow, scale, slab * pl.slab, n1, g, ld,
                           gt ? gt + (int64_t)l * a.n * F : nullptr, part);
    else
        walk_part<F, false>(a, l, a.p.res[l], row0, prow, scale, slab * pl.slab, n1, g, ld,
                            gt ? gt + (int64_t)l * a.n * F : nullptr, part);
    __syncthreads();
    flush_part<F>(a, l, row0, prow, part, acc);
}

// Persistent form: one workgroup per CU walks a contiguous run of the (part, slab) items, part-major,
// so that every workgroup gets the same number of slabs (the per-item grid ran ~4.2 waves of
// workgroups: the last one 1/5 full) and keeps a part in LDS across its consecutive slabs (one flush
// per part change, not one per item).
template <int F>
__global__ __launch_bounds__(BWD_THREADS) void hashgrid_bwd_walk_kernel(HashArgs a, BwdPlan pl, const float* __restrict__ g,
                                                                        int64_t ld, const float* __restrict__ gt,
                                                                        const unsigned* __restrict__ gmax,
                                                                        unsigned long long* __restrict__ acc) {
    __shared__ unsigned long long part[PART_ENTRIES];
    const int s = fixed_shift(*gmax, a.n);
    if (s == -1000) return;                         // uniform: the finish pass writes NaN
    const double scale = ldexp(1.0, s);
    const int64_t items = (int64_t)pl.parts * pl.nslab;
    const int64_t i0 = items * blockIdx.x / gridDim.x, i1 = items * (blockIdx.x + 1) / gridDim.x;
    int cur = -1, l = 0, prow = 0;
    int64_t row0 = 0;
    for (int64_t i = i0; i < i1; ++i) {
        const int w = (int)(i / pl.nslab);
        const int64_t slab = i - (int64_t)w * pl.nslab;
        if (w != cur) {
            if (cur >= 0) {
                __syncthreads();
                flush_part<F>(a, l, row0, prow, part, acc);
                __syncthreads();
            }
            cur = w;
            part_of(a, pl, w, l, row0, prow);
            for (int e = threadIdx.x; e < prow * F; e += BWD_THREADS) part[e] = 0ull;
            __syncthreads();
        }
        const int64_t n0 = slab * pl.slab;
        const int64_t n1 = n0 + pl.slab < a.n ? n0 + pl.slab : a.n;
        if (n0 < n1 && a.n >= 256)
            walk_part<F, true>(a, l, a.p.res[l], row0, prow, scale, n0, n1, g, ld,
                               gt ? gt + (int64_t)l * a.n * F : nullptr, part);
        else if (n0 < n1)
            walk_part<F, false>(a, l, a.p.res[l], row0, prow, scale, n0, n1, g, ld,
                                gt ? gt + (int64_t)l * a.n * F : nullptr, part);
    }
    if (cur >= 0) {
        __syncthreads();
        flush_part<F>(a, l, row0, prow, part, acc);
    }
}

// ---- Bucketed backward for the hashed levels (NERF_HG_BUCKET): the walk above re-derives every
// sample's corners once per 160 KB part (7 parts per 2^16-row level at C5).  Instead one pass
// derives each (sample, hashed level)'s corners once and files the (sample, row in part, weight)
// contributions into per-(level, part) buckets of the workspace; a second pass per bucket chunk adds
// them to its part in LDS with every lane active, and flushes the part as the walk does.  Integer
// fixed-point sums: bitwise the walk's result in any order.  A bucket's contributions past its
// capacity (sized 1.25x the uniform share plus a margin; the hash spreads rows evenly) go straight
// to the global accumulators, so no input can lose one.
constexpr int BUCKET_MAXP = 64;
// pass B's part: NERF_HG_BUCKET_PART entries (default 10240 = 80 KB: two workgroups share a CU, with
// twice the parts — 1.68 vs 1.81 ms per ingp step against 20480 = 160 KB, profiles/r04z)
#ifndef NERF_HG_BUCKET_PART
#define NERF_HG_BUCKET_PART 10240
#endif
constexpr int BUCKET_PART_ENTRIES = NERF_HG_BUCKET_PART;
// Every bucket is split into BUCKET_SUB sub-buckets with their own fill counters: pass-A workgroup w
// files into sub-bucket w % BUCKET_SUB, so a counter takes the atomics of 1/16 of the workgroups, all
// on one XCD (workgroups are dealt to the 8 XCDs round-robin) — one shared counter per bucket took
// one same-address global atomic per workgroup (5120 at C5's fine pass), serialised in L2
constexpr int BUCKET_SUB = 16;

struct BucketPlan {
    int first;              // first hashed level: levels first .. L-1 are bucketed
    int nparts;             // parts per hashed level (ceil(T / rpp))
    int rpp;                // rows per part
    int chunks;             // pass-B workgroups per bucket (one per sub-bucket)
    int64_t cap;            // entries per sub-bucket
    int pack_bits;          // > 0: entries packed into 8 B (uint2 {local sample << bits | row, weight}) — the
                            // sample as its index among the sub-bucket's workgroups' samples; 0: 3 arrays
    unsigned* count;        // [(L - first) * nparts][BUCKET_SUB] entries filed (zeroed per call)
    unsigned* en;           // [bucket][sub][cap] sample
    unsigned* er;           // [bucket][sub][cap] row within the part
    float* ew;              // [bucket][sub][cap] corner weight
};

#ifndef NERF_HG_BUCKET_LOOP
#define NERF_HG_BUCKET_LOOP 1
#endif
#ifndef NERF_HG_ADD_UNROLL
#define NERF_HG_ADD_UNROLL 4
#endif
#ifndef NERF_HG_PACK_DEFAULT
#define NERF_HG_PACK_DEFAULT 1
#endif
#ifndef NERF_HG_BUCKET_RANK
#define NERF_HG_BUCKET_RANK 1
#endif

// Pass A.  NERF_HG_BUCKET_LOOP (default 1): each workgroup's 256 samples through every hashed level
// (positions derived once); 0: one level per workgroup (grid y).
template <int F>
__global__ __launch_bounds__(256) void hashgrid_bucket_kernel(HashArgs a, BucketPlan bp, const float* __restrict__ g,
                                                              int64_t ld, const unsigned* __restrict__ gmax,
                                                              unsigned long long* __restrict__ acc) {
#pragma clang fp contract(off)
    __shared__ unsigned cnt[BUCKET_MAXP], base[BUCKET_MAXP], cntw[4][BUCKET_MAXP];
    const int s = fixed_shift(*gmax, a.n);
    if (s == -1000) return;                         // uniform: the finish pass writes NaN
    const int P = bp.nparts;
    const int wave = threadIdx.x >> 6;
    const int l_begin = NERF_HG_BUCKET_LOOP ? bp.first : bp.first + (int)blockIdx.y;
    const int l_end = NERF_HG_BUCKET_LOOP ? a.p.levels : l_begin + 1;
    const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const bool valid = n < a.n;
    const int lane = threadIdx.x & 63;
    const int sub = (int)(blockIdx.x % BUCKET_SUB);
    const double scale = ldexp(1.0, s);
    float p[3] = {0.0f, 0.0f, 0.0f};
    if (valid) sample_position(a, n, p);
    for (int l = l_begin; l < l_end; ++l) {
        if (threadIdx.x < P) cnt[threadIdx.x] = 0u;
        if (NERF_HG_BUCKET_RANK && threadIdx.x < 4 * P) cntw[threadIdx.x / P][threadIdx.x % P] = 0u;
        __syncthreads();
        Corners c;
        int pk[8];
        unsigned slot[8];
        if (valid) c = level_corners(p, a.p.normalize, a.p.res[l], a.p.table_size, a.p.primes);
        if (NERF_HG_BUCKET_RANK) {
            // slots from per-wave LDS counters (returning adds: a wave instruction's lanes on a
            // handful of addresses, no cross-wave contention), wave offsets by a prefix after the sync.
            // Default: the fine pass's 16 levels 1298 vs 1468 us with the ballot grouping below
            // (NERF_HG_BUCKET_RANK=0; profiles/r04w)
            if (valid) {
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    pk[k] = (int)((unsigned)c.idx[k] / (unsigned)bp.rpp);
                    slot[k] = atomicAdd(&cntw[wave][pk[k]], 1u);
                }
            }
            __syncthreads();
            if (threadIdx.x < P) {
                unsigned run = 0;
#pragma unroll
                for (int w = 0; w < 4; ++w) {
                    const unsigned c_w = cntw[w][threadIdx.x];
                    cntw[w][threadIdx.x] = run;
                    run += c_w;
                }
                cnt[threadIdx.x] = run;
            }
            __syncthreads();
            if (valid) {
#pragma unroll
                for (int k = 0; k < 8; ++k) slot[k] += cntw[wave][pk[k]];
            }
        } else {
        // slots: per corner, the wave's lanes grouped by part (one ballot per part present), ranks
        // and per-part running counts in registers (lane p holds part p's), then ONE LDS add per wave
        // for all its parts — no atomic round trip inside the loop
        unsigned runv = 0;                          // lane p: this wave's entries for part p so far
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            pk[k] = valid ? (int)((unsigned)c.idx[k] / (unsigned)bp.rpp) : -1;
            unsigned long long rest = __ballot(valid);
            while (rest != 0ull) {
                const int leader = __builtin_ctzll(rest);
                const int pp = __builtin_amdgcn_readlane(pk[k], leader);
                const unsigned long long m = __ballot(pk[k] == pp);
                const unsigned rank =
                    __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
                const unsigned run = __builtin_amdgcn_readlane(runv, pp);
                if (pk[k] == pp) slot[k] = run + rank;
                if (lane == pp) runv += (unsigned)__builtin_popcountll(m);
                rest &= ~m;
            }
        }
        const unsigned wbase = (lane < P && runv != 0u) ? atomicAdd(&cnt[lane], runv) : 0u;
#pragma unroll
        for (int k = 0; k < 8; ++k) slot[k] += (unsigned)__shfl((int)wbase, pk[k] < 0 ? 0 : pk[k], 64);
        __syncthreads();
        }
        unsigned* const gcount = bp.count + (int64_t)(l - bp.first) * P * BUCKET_SUB + sub;
        if (threadIdx.x < P && cnt[threadIdx.x] != 0u)
            base[threadIdx.x] = atomicAdd(&gcount[threadIdx.x * BUCKET_SUB], cnt[threadIdx.x]);
        __syncthreads();
        if (valid) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const unsigned pos = base[pk[k]] + slot[k];
                const int64_t b = ((int64_t)(l - bp.first) * P + pk[k]) * BUCKET_SUB + sub;
                if (pos < (uint64_t)bp.cap) {
                    const int64_t e = b * bp.cap + pos;
                    const unsigned row = (unsigned)(c.idx[k] - pk[k] * bp.rpp);
                    if (bp.pack_bits > 0) {
                        const unsigned li = (blockIdx.x / BUCKET_SUB) * 256u + threadIdx.x;
                        reinterpret_cast<uint2*>(bp.en)[e] =
                            make_uint2((li << bp.pack_bits) | row, __float_as_uint(c.w[k]));
                    } else {
                        bp.en[e] = (unsigned)n;
                        bp.er[e] = row;
                        bp.ew[e] = c.w[k];
                    }
                } else {
                    // past the sub-bucket's capacity: straight to the global accumulator
#pragma unroll
                    for (int f = 0; f < F; ++f) {
                        const double x = (double)c.w[k] * ((double)g[n * ld + (int64_t)l * F + f] * scale);
                        const long long q = a.n >= 256 ? rint_fixed(x) : llrint(x);
                        if (q != 0) atomicAdd(&acc[(a.off[l] + c.idx[k]) * F + f], (unsigned long long)q);
                    }
                }
            }
        }
    }
}

// g: grad_out restaged level-major (gt[l][n][f], hashgrid_gtr_kernel): a bucket's entries come in
// runs of nearby samples, whose F values are then adjacent (from the [n][ld] rows every entry would
// fetch its own line, and the 7 parts' buckets are not walked together to share it in L2)
template <int F>
__global__ __launch_bounds__(BWD_THREADS) void hashgrid_bucket_add_kernel(HashArgs a, BucketPlan bp,
                                                                          const float* __restrict__ gt,
                                                                          const unsigned* __restrict__ gmax,
                                                                          unsigned long long* __restrict__ acc) {
#pragma clang fp contract(off)
    __shared__ unsigned long long part[BUCKET_PART_ENTRIES];
    const int s = fixed_shift(*gmax, a.n);
    if (s == -1000) return;
    const double scale = ldexp(1.0, s);
    const int b = (int)(blockIdx.x / (unsigned)bp.chunks), ch = (int)(blockIdx.x % (unsigned)bp.chunks);
    const int l = bp.first + b / bp.nparts, pi = b % bp.nparts;
    const int64_t row0 = (int64_t)pi * bp.rpp;
    const int64_t rows = (int64_t)a.p.table_size - row0;
    const int prow = (int)(rows < bp.rpp ? rows : bp.rpp);
    for (int e = threadIdx.x; e < prow * F; e += BWD_THREADS) part[e] = 0ull;
    __syncthreads();
    const int64_t sb = (int64_t)b * BUCKET_SUB + ch;         // chunks == BUCKET_SUB: this sub-bucket
    const unsigned cnt = bp.count[sb];
    const int64_t e0 = 0, e1 = cnt < (uint64_t)bp.cap ? (int64_t)cnt : bp.cap;
    const unsigned* __restrict__ en = bp.en + sb * bp.cap;
    const unsigned* __restrict__ er = bp.er + sb * bp.cap;
    const float* __restrict__ ew = bp.ew + sb * bp.cap;
    const bool fast = a.n >= 256;
    const float* __restrict__ gl = gt + (int64_t)l * a.n * F;
    // NERF_HG_ADD_UNROLL entries per thread per trip, all their loads issued before any is used
    constexpr int U = NERF_HG_ADD_UNROLL;
    for (int64_t e = e0 + threadIdx.x; e < e1; e += U * BWD_THREADS) {
        unsigned nn[U], row[U];
        float w[U], gv[U][F];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t eu = e + u * BWD_THREADS < e1 ? e + u * BWD_THREADS : e1 - 1;
            if (bp.pack_bits > 0) {
                typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
                const u32x2 kw = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(bp.en) + sb * bp.cap + eu);
                const unsigned kx = kw[0], ky = kw[1];      // scalar copies (ext-vector elements)
                const unsigned li = kx >> bp.pack_bits;
                nn[u] = ((li >> 8) * BUCKET_SUB + (unsigned)ch) * 256u + (li & 255u);
                row[u] = kx & ((1u << bp.pack_bits) - 1u);
                w[u] = __uint_as_float(ky);
            } else {
                nn[u] = __builtin_nontemporal_load(en + eu);
                row[u] = __builtin_nontemporal_load(er + eu);
                w[u] = __builtin_nontemporal_load(ew + eu);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int f = 0; f < F; ++f) gv[u][f] = gl[(int64_t)nn[u] * F + f];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (e + u * BWD_THREADS >= e1) break;
#pragma unroll
            for (int f = 0; f < F; ++f) {
                // the walk's arithmetic: w (g 2^s), one rounding to the fixed-point grid
                const double x = (double)w[u] * ((double)gv[u][f] * scale);
                const long long q = fast ? rint_fixed(x) : llrint(x);
                atomicAdd(&part[row[u] * F + f], (unsigned long long)q);
            }
        }
    }
    __syncthreads();
    flush_part<F>(a, l, row0, prow, part, acc);
}

template <int F>
void launch_bucket(hipStream_t s, const HashArgs& a, const BucketPlan& bp, int nhashed, const float* g, int64_t ld,
                   const float* gt, const unsigned* gmax, unsigned long long* acc) {
    hipLaunchKernelGGL(hashgrid_bucket_kernel<F>, dim3((unsigned)((a.n + 255) / 256), NERF_HG_BUCKET_LOOP ? 1u : (unsigned)nhashed),
                       dim3(256), 0, s,
                       a, bp, g, ld, gmax, acc);
    hipLaunchKernelGGL(hashgrid_bucket_add_kernel<F>, dim3((unsigned)((int64_t)nhashed * bp.nparts * bp.chunks)),
                       dim3(BWD_THREADS), 0, s, a, bp, gt, gmax, acc);
}

template <int F>
void launch_bwd(bool walk, bool merged, int64_t blocks, hipStream_t s, const HashArgs& a, const BwdPlan& pl, const float* g, int64_t ld,
                const float* gt, const unsigned* gmax, unsigned long long* acc) {
    if (walk)
        hipLaunchKernelGGL(hashgrid_bwd_walk_kernel<F>, dim3((unsigned)blocks), dim3(BWD_THREADS), 0, s, a, pl, g, ld, gt,
                           gmax, acc);
    else if (merged)
        hipLaunchKernelGGL((hashgrid_bwd_kernel<F, true>), dim3((unsigned)blocks), dim3(BWD_THREADS), 0, s, a, pl, g, ld, gt,
                           gmax, acc);
    else
        hipLaunchKernelGGL((hashgrid_bwd_kernel<F, false>), dim3((unsigned)blocks), dim3(BWD_THREADS), 0, s, a, pl, g, ld, gt,
                           gmax, acc);
}

template <int F>
void launch_fwd_tile(hipStream_t s, const HashArgs& a, const float* table, float* out, int64_t ld) {
    hipLaunchKernelGGL(hashgrid_fwd_tile_kernel<F>, dim3((unsigned)((a.n + TILE_SAMPLES - 1) / TILE_SAMPLES)),
                       dim3(64 * a.p.levels), 0, s, a, table, out, ld);
}

template <int F>
void launch_gtr(hipStream_t s, const float* g, int64_t ld, int64_t n, int L, float* gt, unsigned* gmax) {
    hipLaunchKernelGGL(hashgrid_gtr_kernel<F>, dim3((unsigned)((n + TILE_SAMPLES - 1) / TILE_SAMPLES)), dim3(256), 0, s,
                       g, ld, n, L, gt, gmax);
}

int env_mode(const char* name, int dflt) {
    const char* e = getenv(name);
    return (e && e[0] >= '0' && e[0] <= '9') ? e[0] - '0' : dflt;
}

int num_cus() {
    static int n = 0;
    if (n == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
    }
    return n;
}

// table gradient = accumulator * 2^-s (or NaN after a non-finite gradient)
__global__ __launch_bounds__(256) void hashgrid_finish_kernel(unsigned long long* __restrict__ acc, int64_t count,
                                                              const unsigned* __restrict__ gmax, int64_t n,
                                                              float* __restrict__ grad, int accumulate) {
    const int s = fixed_shift(*gmax, n);
    const double inv = s == -1000 ? 0.0 : ldexp(1.0, -s);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < count; i += (int64_t)gridDim.x * 256) {
        const long long q = (long long)acc[i];
        const float v = s == -1000 ? NAN : (float)((double)q * inv);
        grad[i] = accumulate ? grad[i] + v : v;
    }
}

// ------------------------------------------------------------------- position gradient
// dL/dp of the features' positions through the multilinear weights (3d-ingp/model.py:58-121 as
// SURVEY §8(a) a9 restates it: w_k = prod_d (1 - |x_hat_d - c_kd|) on the unclipped corner c_k,
// x_hat = (p / 8 + 0.5) r; autograd of torch.abs takes sign(0) = 0; the corners and rows are
// constants of p).  With G_k = sum_f g[l F + f] table[l][row_k][f]:
//   dL/dx_hat_d = sum_k G_k (-sign(x_hat_d - c_kd)) prod_{e != d} (1 - |x_hat_e - c_ke|),
//   dL/dp_d     = sum_l (dL/dx_hat_d r_l) / 8  (r_l without normalisation),
// levels and corners added in order (fp32, fixed order: deterministic).  One thread per sample.
__global__ __launch_bounds__(256) void hashgrid_bwd_pos_kernel(HashArgs a, const float* __restrict__ table,
                                                               const float* __restrict__ g, int64_t g_ld,
                                                               float* __restrict__ dpos, int accumulate) {
#pragma clang fp contract(off)
    const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (n >= a.n) return;
    const int L = a.p.levels, F = a.p.features, T = a.p.table_size;
    float p[3];
    sample_position(a, n, p);
    float acc[3] = {0.0f, 0.0f, 0.0f};
    for (int l = 0; l < L; ++l) {
        const int r = a.p.res[l];
        const Corners c = level_corners(p, a.p.normalize, r, T, a.p.primes);
        // per dimension: the factor 1 - |u| and its derivative -sign(u), u = x_hat - corner, for the
        // corner offsets 0 / 1 (the corner coordinates as level_corners forms them: int64 floor)
        float fac[3][2], dfac[3][2];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const float xh = (a.p.normalize ? (p[j] / 8.0f + 0.5f) : p[j]) * (float)r;
            const long long b = (long long)floorf(xh);
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const float u = xh - (float)(b + e);
                fac[j][e] = 1.0f - fabsf(u);
                dfac[j][e] = u > 0.0f ? -1.0f : (u < 0.0f ? 1.0f : 0.0f);
            }
        }
        const float* tab = table + a.off[l] * F;
        const float* gl = g + n * g_ld + (int64_t)l * F;
        float gx[3] = {0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int ex = (k >> 2) & 1, ey = (k >> 1) & 1, ez = k & 1;   // z fastest
            float G = 0.0f;
            for (int f = 0; f < F; ++f) G = G + gl[f] * tab[(int64_t)c.idx[k] * F + f];
            gx[0] = gx[0] + G * (dfac[0][ex] * (fac[1][ey] * fac[2][ez]));
            gx[1] = gx[1] + G * (dfac[1][ey] * (fac[0][ex] * fac[2][ez]));
            gx[2] = gx[2] + G * (dfac[2][ez] * (fac[0][ex] * fac[1][ey]));
        }
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const float gr = gx[j] * (float)r;
            acc[j] = acc[j] + (a.p.normalize ? gr / 8.0f : gr);
        }
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) dpos[n * 3 + j] = accumulate ? dpos[n * 3 + j] + acc[j] : acc[j];
}

// Ray form: p = o + t_q d, so dL/do = sum_s dL/dp_s and dL/dd = sum_s t_q,s dL/dp_s over each ray's
// samples — one wave per ray, lane-strided partial sums then a fixed-order wave sum.
__global__ __launch_bounds__(256) void hashgrid_pos_rays_kernel(HashArgs a, const float* __restrict__ dpos,
                                                                int64_t n_rays, float* __restrict__ d_o,
                                                                float* __restrict__ d_d, int accumulate) {
#pragma clang fp contract(off)
    const int64_t ray = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (ray >= n_rays) return;
    float so[3] = {0.0f, 0.0f, 0.0f}, sd[3] = {0.0f, 0.0f, 0.0f};
    for (int s = lane; s < a.spr; s += 64) {
        const int64_t n = ray * a.spr + s;
        if (n >= a.n) break;
        const float tq = (a.p.query == 0) ? a.t0[n] : (a.t0[n] + a.t1[n]) / 2.0f;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const float gp = dpos[n * 3 + j];
            so[j] = so[j] + gp;
            sd[j] = sd[j] + gp * tq;
        }
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const float to = wave_sum_f(so[j]), td = wave_sum_f(sd[j]);
        if (lane == 0) {
            if (d_o) d_o[ray * 3 + j] = accumulate ? d_o[ray * 3 + j] + to : to;
            if (d_d) d_d[ray * 3 + j] = accumulate ? d_d[ray * 3 + j] + td : td;
        }
    }
}

bool valid_params(const nerf_hashgrid_params* p) {
    if (p == nullptr || p->levels < 1 || p->levels > NERF_HASHGRID_MAX_LEVELS) return false;
    if (p->features < 1 || p->features > NERF_HASHGRID_MAX_FEATURES || p->table_size < 1) return false;
    if ((int64_t)p->levels * p->table_size * p->features >= ((int64_t)1 << 31)) return false;
    for (int l = 0; l < p->levels; ++l)
        if (p->res[l] < 1 || p->res[l] > (1 << 20)) return false;
    if (p->normalize != 0 && p->normalize != 1) return false;
    return p->query == 0 || p->query == 1;
}

int64_t total_rows(const nerf_hashgrid_params* p) {
    int64_t rows = 0;
    for (int l = 0; l < p->levels; ++l) rows += level_rows(p->res[l], p->table_size);
    return rows;
}

HashArgs make_args(const nerf_hashgrid_params* p, const float* x, const float* o, const float* d, const float* t0,
                   const float* t1, int64_t n, int spr) {
    HashArgs a{};
    a.p = *p;
    int64_t r = 0;
    for (int l = 0; l < p->levels; ++l) {
        a.off[l] = r;
        r += level_rows(p->res[l], p->table_size);
    }
    a.x = x, a.o = o, a.d = d, a.t0 = t0, a.t1 = t1, a.n = n, a.spr = spr;
    return a;
}

}  // namespace

extern "C" int nerf_hashgrid_fwd(const nerf_hashgrid_params* params, const float* x, const float* ray_o,
                                 const float* ray_d, const float* t_start, const float* t_end, int64_t n_samples,
                                 int32_t samples_per_ray, const float* table, float* out, int64_t out_ld,
                                 void* stream) {
    NERF_REQUIRE(valid_params(params) && table != nullptr && out != nullptr && n_samples >= 0);
    NERF_REQUIRE(out_ld >= (int64_t)params->levels * params->features);
    NERF_REQUIRE(x != nullptr || (ray_o && ray_d && t_start && samples_per_ray >= 1 &&
                                  (params->query == 0 || t_end)));
    if (n_samples == 0) return NERF_OK;
    const HashArgs a = make_args(params, x, ray_o, ray_d, t_start, t_end, n_samples, samples_per_ray);
    // NERF_HG_FWD: 1 (default) the level grid; 2 64-sample tiles, one wave per level, whole output
    // rows; 0 one thread per (sample, level) — bitwise the same features (1.31 M samples x 16 levels:
    // 361 / 375 / 764 us, profiles/r04e/hg_*.txt)
    static const int mode = env_mode("NERF_HG_FWD", 1);
    const int F = params->features, L = params->levels;
    const bool f2_aligned = F != 2 || ((reinterpret_cast<uintptr_t>(out) & 7) == 0 && out_ld % 2 == 0 &&
                                       (reinterpret_cast<uintptr_t>(table) & 7) == 0);
    hipStream_t st = as_stream(stream);
    if (mode == 2 && L <= 16 && (F == 1 || F == 2 || F == 4) && (n_samples + TILE_SAMPLES - 1) / TILE_SAMPLES < (1ll << 31)) {
        if (F == 1) launch_fwd_tile<1>(st, a, table, out, out_ld);
        else if (F == 2) launch_fwd_tile<2>(st, a, table, out, out_ld);
        else launch_fwd_tile<4>(st, a, table, out, out_ld);
    } else if (mode >= 1 && f2_aligned && (n_samples + 255) / 256 < (1ll << 31)) {
        hipLaunchKernelGGL(hashgrid_fwd_level_kernel, dim3((unsigned)((n_samples + 255) / 256), (unsigned)L),
                           dim3(256), 0, st, a, table, out, out_ld);
    } else {
        const int64_t threads = n_samples * L;
        hipLaunchKernelGGL(hashgrid_fwd_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, a, table,
                           out, out_ld);
    }
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}

extern "C" int nerf_hashgrid_bwd_pos(const nerf_hashgrid_params* params, const float* x, const float* ray_o,
                                     const float* ray_d, const float* t_start, const float* t_end, int64_t n_samples,
                                     int32_t samples_per_ray, const float* table, const float* grad_out, int64_t g_ld,
                                     float* grad_x, float* grad_o, float* grad_d, int32_t accumulate, void* workspace,
                                     size_t workspace_bytes, void* stream) {
    NERF_REQUIRE(valid_params(params) && table != nullptr && grad_out != nullptr && n_samples >= 0);
    NERF_REQUIRE(g_ld >= (int64_t)params->levels * params->features);
    if (x != nullptr) {
        NERF_REQUIRE(grad_x != nullptr && grad_o == nullptr && grad_d == nullptr);
    } else {
        NERF_REQUIRE(ray_o && ray_d && t_start && samples_per_ray >= 1 && (params->query == 0 || t_end));
        NERF_REQUIRE(grad_x == nullptr && (grad_o != nullptr || grad_d != nullptr));
        NERF_REQUIRE(n_samples % samples_per_ray == 0);
        if (workspace == nullptr || workspace_bytes < (size_t)n_samples * 3 * sizeof(float)) return NERF_ERR_WORKSPACE;
        NERF_REQUIRE(aligned16(workspace));
    }
    if (n_samples == 0) return NERF_OK;
    NERF_REQUIRE((n_samples + 255) / 256 < (1ll << 31));
    const HashArgs a = make_args(params, x, ray_o, ray_d, t_start, t_end, n_samples, samples_per_ray);
    hipStream_t st = as_stream(stream);
    float* dpos = x != nullptr ? grad_x : static_cast<float*>(workspace);
    hipLaunchKernelGGL(hashgrid_bwd_pos_kernel, dim3((unsigned)((n_samples + 255) / 256)), dim3(256), 0, st, a, table,
                       grad_out, g_ld, dpos, x != nullptr ? accumulate : 0);
    NERF_CHECK_LAUNCH();
    if (x == nullptr) {
        const int64_t rays = n_samples / samples_per_ray;
        NERF_REQUIRE((rays + 3) / 4 < (1ll << 31));
        hipLaunchKernelGGL(hashgrid_pos_rays_kernel, dim3((unsigned)((rays + 3) / 4)), dim3(256), 0, st, a, dpos, rays,
                           grad_o, grad_d, accumulate);
        NERF_CHECK_LAUNCH();
    }
    return NERF_OK;
}

extern "C" int64_t nerf_hashgrid_table_rows(const nerf_hashgrid_params* params, int32_t level) {
    if (!valid_params(params) || level >= params->levels) return -1;
    return level < 0 ? total_rows(params) : level_rows(params->res[level], params->table_size);
}

extern "C" size_t nerf_hashgrid_workspace(const nerf_hashgrid_params* params) {
    if (!valid_params(params)) return 0;
    return 256 + (size_t)total_rows(params) * params->features * sizeof(unsigned long long);
}

namespace {
using namespace nerf;
size_t gt_offset(const nerf_hashgrid_params* params) { return (nerf_hashgrid_workspace(params) + 255) & ~(size_t)255; }
size_t round256(size_t v) { return (v + 255) & ~(size_t)255; }

// The bucketed backward's share of the workspace: the hashed levels from `first` on (a level whose
// (r+1)^3 > T; the walk keeps every level before it), nparts parts of rpp rows each, buckets of cap
// entries per sub-bucket (1.25x the uniform share of a level's 8 n corner contributions, plus 4096).  bytes = 0:
// not eligible (no hashed level, more than BUCKET_MAXP parts a level, or n outside [1, 2^31)).
struct BucketLayout {
    int first = 0, nparts = 0, rpp = 0;
    int pack_bits = 0;      // > 0: 8-byte packed entries (two arrays' room), else three 4-byte arrays
    int64_t cap = 0;
    size_t bytes = 0;
};
BucketLayout bucket_layout(const nerf_hashgrid_params* p, int64_t n) {
    BucketLayout b;
    const int L = p->levels;
    const int64_t T = p->table_size;
    auto hashed = [&](int l) {
        const int64_t r1 = (int64_t)p->res[l] + 1;
        return r1 * r1 * r1 > T;
    };
    int first = L;
    while (first > 0 && hashed(first - 1)) --first;
    b.first = first;
    b.rpp = BUCKET_PART_ENTRIES / p->features;
    b.nparts = (int)((T + b.rpp - 1) / b.rpp);
    if (first == L || b.nparts > BUCKET_MAXP || n < 1 || n >= ((int64_t)1 << 31)) return b;
    b.cap = ((8 * n * 5 / 4) / ((int64_t)b.nparts * BUCKET_SUB) + 4096 + 63) / 64 * 64;
    const int64_t nb = (int64_t)(L - first) * b.nparts * BUCKET_SUB;       // sub-buckets
    // 8-byte entries when the sample index among a sub-bucket's workgroups and the row fit 32 bits
    // together (C5's fine pass: 82 176 x 10 240 rows); NERF_HG_PACK=0: 12-byte entries (1538 vs
    // 1474 us with the ballot grouping, profiles/r04v).  The packed form needs two arrays' room, not
    // three (~0.7 GB less workspace per C5 fine-pass backward)
    int rb = 0;
    while ((1 << rb) < b.rpp) ++rb;
    const int64_t li_max = ((n + 255) / 256 + BUCKET_SUB - 1) / BUCKET_SUB * 256;
    b.pack_bits = (env_mode("NERF_HG_PACK", NERF_HG_PACK_DEFAULT) == 1 && rb < 32 && li_max <= ((int64_t)1 << (32 - rb)))
                      ? rb : 0;
    b.bytes = round256((size_t)nb * sizeof(unsigned)) +
              (b.pack_bits > 0 ? 2 : 3) * round256((size_t)nb * b.cap * sizeof(unsigned));
    return b;
}
size_t bucket_offset(const nerf_hashgrid_params* p, int64_t n) {
    return gt_offset(p) + round256((size_t)n * sizeof(float4) + (size_t)n * p->levels * p->features * sizeof(float));
}
}  // namespace

// [header + accumulators][position records: n float4][grad_out restaged level-major: L n F floats]
// [bucketed backward: counts | samples | rows | weights]
extern "C" size_t nerf_hashgrid_workspace_n(const nerf_hashgrid_params* params, int64_t n_samples) {
    if (!valid_params(params) || n_samples < 0) return 0;
    return bucket_offset(params, n_samples) + bucket_layout(params, n_samples).bytes;
}

extern "C" int nerf_hashgrid_bwd(const nerf_hashgrid_params* params, const float* x, const float* ray_o,
                                 const float* ray_d, const float* t_start, const float* t_end, int64_t n_samples,
                                 int32_t samples_per_ray, const float* grad_out, int64_t g_ld, float* grad_table,
                                 int32_t accumulate, void* workspace, size_t workspace_bytes, void* stream) {
    NERF_REQUIRE(valid_params(params) && grad_out != nullptr && grad_table != nullptr && workspace != nullptr);
    NERF_REQUIRE(n_samples >= 0 && g_ld >= (int64_t)params->levels * params->features);
    NERF_REQUIRE(x != nullptr || (ray_o && ray_d && t_start && samples_per_ray >= 1 &&
                                  (params->query == 0 || t_end)));
    if (workspace_bytes < nerf_hashgrid_workspace(params)) return NERF_ERR_WORKSPACE;
    NERF_REQUIRE((reinterpret_cast<uintptr_t>(workspace) & 255) == 0);
    unsigned* gmax = static_cast<unsigned*>(workspace);
    unsigned long long* acc = reinterpret_cast<unsigned long long*>(static_cast<char*>(workspace) + 256);
    const int64_t count = total_rows(params) * params->features;
    hipStream_t s = as_stream(stream);
    // header and accumulators zeroed by every call (no state carried between calls)
    if (hipMemsetAsync(workspace, 0, 256 + (size_t)count * sizeof(unsigned long long), s) != hipSuccess)
        return NERF_ERR_LAUNCH;
    HashArgs a = make_args(params, x, ray_o, ray_d, t_start, t_end, n_samples, samples_per_ray);
    if (n_samples > 0) {
        const int cols = params->levels * params->features;
        const bool room = workspace_bytes >= nerf_hashgrid_workspace_n(params, n_samples);
        char* const tail = static_cast<char*>(workspace) + gt_offset(params);
        // NERF_HG_POS=1: the ray form's positions computed once into float4 records when the workspace
        // has room (nerf_hashgrid_workspace_n), instead of in every part walk; bitwise the same, and
        // measured no faster (2.68 vs 2.65 ms per ingp step, profiles/r04n): off by default
        static const int pos_mode = env_mode("NERF_HG_POS", 0);
        if (pos_mode == 1 && room && x == nullptr && (n_samples + 255) / 256 < (1ll << 31)) {
            float4* pos = reinterpret_cast<float4*>(tail);
            hipLaunchKernelGGL(hashgrid_pos_kernel, dim3((unsigned)((n_samples + 255) / 256)), dim3(256), 0, s, a, pos);
            NERF_CHECK_LAUNCH();
            a.pos = pos;
        }
        // grad_out restaged level-major (with its max) when the workspace has room for it
        // (nerf_hashgrid_workspace_n) and the walks read it (NERF_HG_BWD: 0 (default) the per-item grid
        // on the rows; 1 the per-item grid over the restaged values; 2 the persistent walk over them).
        // Measured (1.31 M samples x 16 levels, profiles/r04e/hg_*.txt): 2807 / 3042 / 5586 us — the
        // 97 concurrent parts of a slab share its rows in L2, so the strided reads cost nothing, and
        // the part-major walk loses that sharing
        static const int mode = env_mode("NERF_HG_BWD", 0);
        const int F = params->features;
        // NERF_HG_BUCKET (default 1): the hashed levels through the bucketed passes when the workspace
        // has room (nerf_hashgrid_workspace_n), F is 1, 2 or 4 (grad_out restaged level-major for
        // them) and the walks read the rows (NERF_HG_BWD=0, no merge); the walk keeps the levels
        // before them.  Bitwise the walk's result; 1.31 M samples x 16 levels 1610 vs 2083 us, the
        // ingp step 23.4 vs 24.3 ms (profiles/r04r)
        static const int bucket_mode = env_mode("NERF_HG_BUCKET", 1);
        static const int merge = env_mode("NERF_HG_MERGE", 0);
        const BucketLayout bl = bucket_layout(params, n_samples);
        const bool tile_ok = (F == 1 || F == 2 || F == 4) && (n_samples + TILE_SAMPLES - 1) / TILE_SAMPLES < (1ll << 31);
        const bool bucket = bucket_mode == 1 && room && bl.bytes > 0 && mode == 0 && merge == 0 && tile_ok;
        float* gt = nullptr;
        float* gt_bucket = nullptr;
        if (bucket) {
            gt_bucket = reinterpret_cast<float*>(tail + (size_t)n_samples * sizeof(float4));
            if (F == 1) launch_gtr<1>(s, grad_out, g_ld, n_samples, params->levels, gt_bucket, gmax);
            else if (F == 2) launch_gtr<2>(s, grad_out, g_ld, n_samples, params->levels, gt_bucket, gmax);
            else launch_gtr<4>(s, grad_out, g_ld, n_samples, params->levels, gt_bucket, gmax);
        } else if (mode >= 1 && room && tile_ok) {
            gt = reinterpret_cast<float*>(tail + (size_t)n_samples * sizeof(float4));
            if (F == 1) launch_gtr<1>(s, grad_out, g_ld, n_samples, params->levels, gt, gmax);
            else if (F == 2) launch_gtr<2>(s, grad_out, g_ld, n_samples, params->levels, gt, gmax);
            else launch_gtr<4>(s, grad_out, g_ld, n_samples, params->levels, gt, gmax);
        }
        if (gt == nullptr && gt_bucket == nullptr) {
            const bool vec = cols % 4 == 0 && g_ld % 4 == 0 && (reinterpret_cast<uintptr_t>(grad_out) & 15) == 0;
            int64_t blocks = (n_samples * (vec ? cols / 4 : cols) + 255) / 256;
            blocks = blocks < 1024 ? blocks : 1024;
            if (vec)
                hipLaunchKernelGGL(hashgrid_gmax_kernel<4>, dim3((unsigned)blocks), dim3(256), 0, s, grad_out, g_ld,
                                   n_samples, cols, gmax);
            else
                hipLaunchKernelGGL(hashgrid_gmax_kernel<1>, dim3((unsigned)blocks), dim3(256), 0, s, grad_out, g_ld,
                                   n_samples, cols, gmax);
        }
        NERF_CHECK_LAUNCH();
        BwdPlan pl{};
        pl.rows_per_part = PART_ENTRIES / params->features;
        for (int l = 0; l < params->levels; ++l) {
            const int64_t rows = level_rows(params->res[l], params->table_size);
            pl.start[l + 1] = pl.start[l] + (int)((rows + pl.rows_per_part - 1) / pl.rows_per_part);
        }
        pl.parts = pl.start[params->levels];
        if (bucket) pl.parts = pl.start[bl.first];
        const bool walk = mode == 2 && gt != nullptr;
        int64_t blocks;
        if (walk) {
            // ~16 slabs per CU-resident workgroup, slabs of at least one 4096-sample trip
            const int64_t G = num_cus();
            int64_t slabs = (16 * G + pl.parts - 1) / pl.parts;
            const int64_t most = (n_samples + 4095) / 4096;
            slabs = slabs < most ? slabs : most;
            pl.slab = (n_samples + slabs - 1) / slabs;
            pl.nslab = (n_samples + pl.slab - 1) / pl.slab;
            const int64_t items = (int64_t)pl.parts * pl.nslab;
            blocks = items < G ? items : G;
        } else {
            // slabs of at least 4096 samples; the grid runs one 1024-thread workgroup per CU at a time,
            // so its time goes as ceil(slabs parts / CUs) rounds of 1/slabs of the samples each: the
            // slab count minimising that (the fewest slabs within 1 %: fewer flushes of parts) from
            // three rounds up to twice four workgroups per CU (97 parts at C5: 13 slabs, 1261 workgroups =
            // 4.93 rounds; four per CU gave 11, 1067 = 4.17 rounds, the last one a sixth full).
            // NERF_HG_SLABS=0: four per CU; =k: k slabs.
            static const int slab_env = [] {
                const char* e = getenv("NERF_HG_SLABS");
                return e ? atoi(e) : -1;
            }();
            const int64_t most = (n_samples + 4095) / 4096;
            const int64_t parts = pl.parts > 0 ? pl.parts : 1;     // (0: every level bucketed)
            const int64_t G = num_cus(), four = (1024 + parts - 1) / parts;
            int64_t slabs = four;
            if (slab_env > 0) {
                slabs = slab_env;
            } else if (slab_env < 0) {
                double best = 1e30;
                const int64_t k0 = (3 * G + parts - 1) / parts, k1 = k0 > 2 * four ? k0 : 2 * four;
                for (int64_t k = k0; k <= k1; ++k) {
                    const double c = (double)((k * parts + G - 1) / G) / (double)k;
                    if (c < 0.99 * best) best = c, slabs = k;
                }
            }
            slabs = slabs < most ? slabs : most;
            pl.slab = (n_samples + slabs - 1) / slabs;
            pl.nslab = slabs;
            blocks = slabs * pl.parts;
        }
        void (*launch)(bool, bool, int64_t, hipStream_t, const HashArgs&, const BwdPlan&, const float*, int64_t,
                       const float*, const unsigned*, unsigned long long*) = nullptr;
        switch (params->features) {
            case 1: launch = launch_bwd<1>; break;
            case 2: launch = launch_bwd<2>; break;
            case 3: launch = launch_bwd<3>; break;
            case 4: launch = launch_bwd<4>; break;
            case 5: launch = launch_bwd<5>; break;
            case 6: launch = launch_bwd<6>; break;
            case 7: launch = launch_bwd<7>; break;
            default: launch = launch_bwd<8>; break;
        }
        // NERF_HG_MERGE=1: consecutive samples per thread with run-length merged corner contributions
        // (walk_part_merged); default 0, samples strided by the workgroup (walk_part).  Bitwise equal;
        // measured (profiles/r04g): the merge saves a fifth at the coarsest level (98 vs 125 us) but
        // costs 60 % at the hashed ones (283 vs 175 us): 3261 vs 2845 us over 16 levels
        if (pl.parts > 0) {
            launch(walk, merge != 0, blocks, s, a, pl, grad_out, g_ld, gt, gmax, acc);
            NERF_CHECK_LAUNCH();
        }
        if (bucket) {
            char* const bb = static_cast<char*>(workspace) + bucket_offset(params, n_samples);
            const int nh = params->levels - bl.first;
            const int64_t nb = (int64_t)nh * bl.nparts * BUCKET_SUB;           // sub-buckets
            BucketPlan bp{};
            bp.first = bl.first;
            bp.nparts = bl.nparts;
            bp.rpp = bl.rpp;
            bp.cap = bl.cap;
            bp.count = reinterpret_cast<unsigned*>(bb);
            bp.en = reinterpret_cast<unsigned*>(bb + round256((size_t)nb * sizeof(unsigned)));
            bp.er = bp.en + round256((size_t)nb * bl.cap * sizeof(unsigned)) / sizeof(unsigned);
            // (the packed form stores uint2 entries over en and er and never touches ew)
            bp.ew = bl.pack_bits > 0 ? nullptr
                                     : reinterpret_cast<float*>(bp.er + round256((size_t)nb * bl.cap * sizeof(unsigned)) /
                                                                            sizeof(unsigned));
            if (hipMemsetAsync(bp.count, 0, (size_t)nb * sizeof(unsigned), s) != hipSuccess) return NERF_ERR_LAUNCH;
            bp.chunks = BUCKET_SUB;
            bp.pack_bits = bl.pack_bits;
            switch (params->features) {
                case 1: launch_bucket<1>(s, a, bp, nh, grad_out, g_ld, gt_bucket, gmax, acc); break;
                case 2: launch_bucket<2>(s, a, bp, nh, grad_out, g_ld, gt_bucket, gmax, acc); break;
                case 4: launch_bucket<4>(s, a, bp, nh, grad_out, g_ld, gt_bucket, gmax, acc); break;
                default: break;                         // (bucket requires F = 1, 2 or 4)
            }
            NERF_CHECK_LAUNCH();
        }
    }
    int64_t fb = (count + 255) / 256;
    fb = fb < 4096 ? fb : 4096;
    hipLaunchKernelGGL(hashgrid_finish_kernel, dim3((unsigned)fb), dim3(256), 0, s, acc, count, gmax,
                       n_samples > 0 ? n_samples : 1, grad_table, accumulate);
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}
