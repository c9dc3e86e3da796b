// Split-precision ("3 x bf16") MFMA linear layers: fp32 operands, fp32 accumulation,
// each operand split as x = hi + lo with hi = bf16(x), lo = bf16(x - hi) (both
// round-to-nearest-even), and every product formed as lo*hi + hi*lo + hi*hi on
// v_mfma_f32_32x32x16_bf16.  The representation error of hi + lo is <= 2^-18 |x|
// and the dropped lo*lo term is <= 2^-18 |x y|, so each product carries ~2^-17
// relative error (fp32: 2^-24; the TF32 the reference trains with on A100,
// run_barf.py:101 set_float32_matmul_precision("high"): 2^-11).  Three bf16
// MFMAs cost 96 cycles per 32x32x16 block against 512 for eight fp32
// 32x32x2 MFMAs: 5.3x the fp32 MFMA rate.
//
// Same contracts and operand conventions as linear.hip (segments, epilogues,
// packed weights); the weights arrive pre-split (nerf_pack_weight_x3).
//
// NT (forward / input gradient): 128 x 128 tile, 4 waves of 64 x 64, K in
// 32-wide chunks.  A (fp32 in HBM) is split while it is staged into LDS;
// LDS planes are [row][32 + 8] bf16 (80-byte rows: the 16 rows a ds_read_b128
// lane group touches hit 16 distinct 16-byte bank slots).  Lane (r, h) of the
// 32x32x16 MFMA holds row r, k = 8h .. 8h+7 of both operands: one ds_read_b128
// per plane and block.
//
// TN (weight gradient): slab[s][n][k] = sum_m dY[m][n] X[m][k]; the sample index
// is the MFMA reduction dimension, so dY and X are staged TRANSPOSED ([n][m],
// [k][m]): a thread loads 8 rows x 4 columns and writes four 8-sample bf16
// vectors per plane (ds_write_b128).
#include "common.h"

using namespace nerf;

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

namespace {

constexpr int BK = 32;
constexpr int LDB = BK + 8;   // bf16 elements per LDS row (80 bytes)
constexpr int MAX_SEGS = 4;

struct SegList {
    const float* ptr[MAX_SEGS];
    int64_t ld[MAX_SEGS];
    int k[MAX_SEGS];
    int kp[MAX_SEGS];
    int row_div[MAX_SEGS];
    int koff[MAX_SEGS];
    int n;
    int ktot;
};

template <typename T>
__device__ __forceinline__ T pick4(const T (&v)[MAX_SEGS], int i) {
    T r = v[0];
    r = (i == 1) ? v[1] : r;
    r = (i == 2) ? v[2] : r;
    r = (i == 3) ? v[3] : r;
    return r;
}

__device__ __forceinline__ f32x16 mfma16(bf16x8 a, bf16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// acc += a*b with both operands split hi/lo; small terms first
__device__ __forceinline__ f32x16 mfma_x3(bf16x8 ah, bf16x8 al, bf16x8 bh, bf16x8 bl, f32x16 c) {
    c = mfma16(al, bh, c);
    c = mfma16(ah, bl, c);
    return mfma16(ah, bh, c);
}

__device__ __forceinline__ void split4(f4 v, bf16x4& hi, bf16x4& lo) {
    hi = __builtin_convertvector(v, bf16x4);
    lo = __builtin_convertvector(v - __builtin_convertvector(hi, f4), bf16x4);
}

__device__ __forceinline__ bool tile_coords(int tile, int ntm, int ntn, int& tm, int& tn) {
    const int grp = 8 * ntn;
    const int g = tile / grp, r = tile - g * grp;
    tn = r / 8;
    tm = g * 8 + (r - tn * 8);
    return tm < ntm;
}

struct NTArgs {
    SegList A;
    int M;
    const __bf16* Wh; const __bf16* Wl; int ldw; int N;
    const float* bias;
    float* out; int64_t ldo;
    int epi;
    const float* aux; int64_t ldaux;
    int vec_ok;
};

// ------------------------------------------------------------------------- NT
__global__ __launch_bounds__(256, 2) void linear_nt_x3_kernel(NTArgs a, int ntm, int ntiles) {
    constexpr int BM = 128, BN = 128;
    constexpr int PL = BM * LDB;                 // one bf16 plane (128 rows)
    constexpr int BUFB = 4 * PL;                 // A hi, A lo, W hi, W lo (bf16 elements)
    constexpr int LDC = BN + 4;
    constexpr int HR = 64;
    static_assert(HR * LDC * 4 <= BUFB * 2, "epilogue half-tile must fit one staging buffer");
    __shared__ __attribute__((aligned(16))) __bf16 smem[2 * BUFB];

    const int ntn = (a.N + BN - 1) / BN;
    const int t = threadIdx.x;
    const int wave = t >> 6, lane = t & 63;
    const int wr = wave >> 1, wc = wave & 1;
    const int li = lane & 31, lh = lane >> 5;
    const int c4 = t & 7, rbase = t >> 3;          // A staging: 8 threads x 4 floats per row
    const int w8 = (t & 3) * 8, wrow = t >> 2;     // W staging: 4 threads x 8 bf16 per row

    int tile = blockIdx.x, tm = 0, tn = 0;
    while (tile < ntiles && !tile_coords(tile, ntm, ntn, tm, tn)) tile += gridDim.x;
    if (tile >= ntiles) return;
    int m0 = tm * BM, n0 = tn * BN;

    int seg = 0;
    const float* sp = nullptr;
    int sk = 0, skp = 0, skoff = 0;
    int64_t aoff[4];
    unsigned aok = 0;
    auto set_seg = [&](int s, int mbase) __attribute__((always_inline)) {
        sp = pick4(a.A.ptr, s);
        const int64_t ld = pick4(a.A.ld, s);
        const unsigned rd = (unsigned)pick4(a.A.row_div, s);
        sk = pick4(a.A.k, s);
        skp = pick4(a.A.kp, s);
        skoff = pick4(a.A.koff, s);
        aok = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int m = mbase + i * 32 + rbase;
            const bool ok = m < a.M;
            const unsigned mc = (unsigned)(ok ? m : a.M - 1);
            const unsigned src = (rd == 1u) ? mc : mc / rd;
            aoff[i] = (int64_t)src * ld;
            aok |= (ok ? 1u : 0u) << i;
        }
    };
    int64_t woff[2];
    auto set_w = [&](int nbase) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < 2; ++j) woff[j] = (int64_t)(nbase + j * 64 + wrow) * a.ldw + w8;
    };

    f4 ra[4];
    u16x8 rwh[2], rwl[2];
    unsigned rmask = 0;
    auto load_chunk = [&](int kc) __attribute__((always_inline)) {
        const int col = kc + c4 * 4;
        const bool cok = col < sk;
        const int acol = cok ? col : 0;
        rmask = cok ? aok : 0u;
#pragma unroll
        for (int i = 0; i < 4; ++i) ra[i] = *reinterpret_cast<const f4*>(sp + aoff[i] + acol);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            rwh[j] = *reinterpret_cast<const u16x8*>(a.Wh + woff[j] + skoff + kc);
            rwl[j] = *reinterpret_cast<const u16x8*>(a.Wl + woff[j] + skoff + kc);
        }
    };
    auto store_chunk = [&](int buf) __attribute__((always_inline)) {
        __bf16* Ah = smem + buf * BUFB;
        __bf16* Al = Ah + PL;
        __bf16* Whp = Ah + 2 * PL;
        __bf16* Wlp = Ah + 3 * PL;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const f4 v = ((rmask >> i) & 1u) ? ra[i] : f4{0.f, 0.f, 0.f, 0.f};
            bf16x4 h, l;
            split4(v, h, l);
            const int o = (i * 32 + rbase) * LDB + c4 * 4;
            *reinterpret_cast<bf16x4*>(Ah + o) = h;
            *reinterpret_cast<bf16x4*>(Al + o) = l;
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int o = (j * 64 + wrow) * LDB + w8;
            *reinterpret_cast<u16x8*>(Whp + o) = rwh[j];
            *reinterpret_cast<u16x8*>(Wlp + o) = rwl[j];
        }
    };

    set_seg(0, m0);
    set_w(n0);
    int kc = 0;
    load_chunk(0);
    store_chunk(0);
    __syncthreads();
    const int nchunks = a.A.ktot / BK;
    int cur = 0;

    while (true) {
        int ntile = tile + gridDim.x, ntm_ = 0, ntn_ = 0;
        while (ntile < ntiles && !tile_coords(ntile, ntm, ntn, ntm_, ntn_)) ntile += gridDim.x;
        const bool has_next_tile = ntile < ntiles;

        f32x16 acc[2][2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

        for (int c = 0; c < nchunks; ++c) {
            if (c + 1 < nchunks) {
                kc += BK;
                if (kc >= skp) {
                    ++seg;
                    set_seg(seg, m0);
                    kc = 0;
                }
            } else {
                seg = 0;
                kc = 0;
                set_seg(0, has_next_tile ? ntm_ * BM : m0);
                set_w(has_next_tile ? ntn_ * BN : n0);
            }
            load_chunk(kc);
            __builtin_amdgcn_sched_barrier(0);

            const __bf16* Ah = smem + cur * BUFB + (wr * 64 + li) * LDB + lh * 8;
            const __bf16* Wb = smem + cur * BUFB + 2 * PL + (wc * 64 + li) * LDB + lh * 8;
#pragma unroll
            for (int s = 0; s < BK / 16; ++s) {
                bf16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    ah[i] = *reinterpret_cast<const bf16x8*>(Ah + i * 32 * LDB + s * 16);
                    al[i] = *reinterpret_cast<const bf16x8*>(Ah + PL + i * 32 * LDB + s * 16);
                    bh[i] = *reinterpret_cast<const bf16x8*>(Wb + i * 32 * LDB + s * 16);
                    bl[i] = *reinterpret_cast<const bf16x8*>(Wb + PL + i * 32 * LDB + s * 16);
                }
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) acc[i][j] = mfma_x3(ah[i], al[i], bh[j], bl[j], acc[i][j]);
            }
            store_chunk(cur ^ 1);
            __syncthreads();
            cur ^= 1;
        }

        float* Cs = reinterpret_cast<float*>(smem + (cur ^ 1) * BUFB);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (wr == h) {
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            const int row = i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                            Cs[row * LDC + wc * 64 + j * 32 + li] = acc[i][j][r];
                        }
            }
            __syncthreads();
            constexpr int Q = BN / 4;
            constexpr int ITER = HR * Q / 256;
#pragma unroll 4
            for (int it = 0; it < ITER; ++it) {
                const int q = it * 256 + t;
                const int row = q / Q, cq = q - (q / Q) * Q;
                const int m = m0 + h * HR + row;
                const int n = n0 + cq * 4;
                if (m >= a.M || n >= a.N) continue;
                f4 v = *reinterpret_cast<const f4*>(Cs + row * LDC + cq * 4);
                float* o = a.out + (int64_t)m * a.ldo + n;
                if (a.vec_ok && n + 4 <= a.N) {
                    if (a.epi & NERF_EPI_BIAS) v += *reinterpret_cast<const f4*>(a.bias + n);
                    if (a.epi & NERF_EPI_RELU) {
                        v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
                    }
                    if (a.epi & NERF_EPI_MASK) {
                        const f4 x = *reinterpret_cast<const f4*>(a.aux + (int64_t)m * a.ldaux + n);
                        v.x = x.x > 0.f ? v.x : 0.f; v.y = x.y > 0.f ? v.y : 0.f;
                        v.z = x.z > 0.f ? v.z : 0.f; v.w = x.w > 0.f ? v.w : 0.f;
                    }
                    if (a.epi & NERF_EPI_ACCUM) v = *reinterpret_cast<const f4*>(o) + v;
                    *reinterpret_cast<f4*>(o) = v;
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        if (n + e >= a.N) break;
                        float x = e == 0 ? v.x : (e == 1 ? v.y : (e == 2 ? v.z : v.w));
                        if (a.epi & NERF_EPI_BIAS) x = x + a.bias[n + e];
                        if (a.epi & NERF_EPI_RELU) x = fmaxf(x, 0.f);
                        if (a.epi & NERF_EPI_MASK) x = (a.aux[(int64_t)m * a.ldaux + n + e] > 0.f) ? x : 0.f;
                        if (a.epi & NERF_EPI_ACCUM) x = o[e] + x;
                        o[e] = x;
                    }
                }
            }
            __syncthreads();
        }

        if (!has_next_tile) break;
        tile = ntile;
        m0 = ntm_ * BM;
        n0 = ntn_ * BN;
    }
}

// ------------------------------------------------------------------------- TN
constexpr int TB = 128, TBM = 32;

struct TNArgs {
    const float* dY; int64_t lddy; int N;
    SegList X;
    int M;
    int m_per_split;
    int splits;
    float* slab;
    float* db_slab;
};

__global__ __launch_bounds__(256, 2) void linear_wgrad_x3_kernel(TNArgs a) {
    constexpr int PL = TB * LDB;          // one transposed bf16 plane: 128 rows x (32 samples + pad)
    constexpr int BUFB = 4 * PL;          // dY^T hi, lo, X^T hi, lo
    __shared__ __attribute__((aligned(16))) __bf16 smem[2 * BUFB];

    const int ntn = (a.N + TB - 1) / TB;
    const int ntk = (a.X.ktot + TB - 1) / TB;
    const int tiles = ntn * ntk;
    const int bid = blockIdx.x;
    const int split = bid / tiles;
    const int tile = bid - split * tiles;
    const int tn = tile / ntk, tk = tile - (tile / ntk) * ntk;
    const int n0 = tn * TB, k0 = tk * TB;
    const int mbeg = split * a.m_per_split;
    int mend = mbeg + a.m_per_split;
    if (mend > a.M) mend = a.M;

    const int t = threadIdx.x;
    const int wave = t >> 6, lane = t & 63;
    const int wr = wave >> 1, wc = wave & 1;
    const int li = lane & 31, lh = lane >> 5;

    // staging role: threads 0..127 stage dY, 128..255 stage X; each owns 4 columns x 8 rows
    const bool isx = t >= 128;
    const int st = t & 127;
    const int cg = st & 31;              // column group (4 columns)
    const int rg = st >> 5;              // row group (8 samples) of the 32-sample stage
    const float* gptr;
    int64_t gld;
    unsigned grd = 1;
    bool col_ok;
    int gcol;
    if (!isx) {
        gcol = n0 + cg * 4;
        col_ok = gcol < a.N;
        gptr = a.dY;
        gld = a.lddy;
    } else {
        const int kx = k0 + cg * 4;
        int xs = -1, xoff = 0;
#pragma unroll
        for (int s = 0; s < MAX_SEGS; ++s)
            if (s < a.X.n && kx >= a.X.koff[s] && kx < a.X.koff[s] + a.X.kp[s]) { xs = s; xoff = kx - a.X.koff[s]; }
        col_ok = xs >= 0 && xoff < (xs >= 0 ? pick4(a.X.k, xs) : 0);
        gptr = col_ok ? pick4(a.X.ptr, xs) : a.dY;
        gld = col_ok ? pick4(a.X.ld, xs) : 0;
        grd = col_ok ? (unsigned)pick4(a.X.row_div, xs) : 1u;
        gcol = xoff;
    }
    if (!col_ok) gcol = 0;

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    f4 dbacc = f4{0.f, 0.f, 0.f, 0.f};

    f4 rv[8];
    unsigned mmask = 0;
    auto gload = [&](int mc) __attribute__((always_inline)) {
        mmask = 0;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const int m = mc + rg * 8 + r;
            const bool mok = m < mend;
            mmask |= (mok ? 1u : 0u) << r;
            const unsigned mm = (unsigned)(mok ? m : mbeg);
            rv[r] = *reinterpret_cast<const f4*>(gptr + (int64_t)(grd == 1u ? mm : mm / grd) * gld + gcol);
        }
    };
    auto sstore = [&](int buf) __attribute__((always_inline)) {
        __bf16* Ph = smem + buf * BUFB + (isx ? 2 * PL : 0);
        __bf16* Pl = Ph + PL;
        f4 v[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) v[r] = (col_ok && ((mmask >> r) & 1u)) ? rv[r] : f4{0.f, 0.f, 0.f, 0.f};
        if (!isx) {
#pragma unroll
            for (int r = 0; r < 8; ++r) dbacc += v[r];
        }
        // transpose: column e of the 8 rows -> one 8-sample vector per plane
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            bf16x8 h, l;
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const float x = e == 0 ? v[r].x : (e == 1 ? v[r].y : (e == 2 ? v[r].z : v[r].w));
                const __bf16 hb = (__bf16)x;
                h[r] = hb;
                l[r] = (__bf16)(x - (float)hb);
            }
            const int o = (cg * 4 + e) * LDB + rg * 8;
            *reinterpret_cast<bf16x8*>(Ph + o) = h;
            *reinterpret_cast<bf16x8*>(Pl + o) = l;
        }
    };

    if (mbeg < mend) {
        gload(mbeg);
        sstore(0);
        __syncthreads();
        int cur = 0;
        for (int mc = mbeg; mc < mend; mc += TBM) {
            const bool has_next = mc + TBM < mend;
            gload(has_next ? mc + TBM : mc);
            __builtin_amdgcn_sched_barrier(0);
            const __bf16* Yb = smem + cur * BUFB + (wr * 64 + li) * LDB + lh * 8;
            const __bf16* Xb = smem + cur * BUFB + 2 * PL + (wc * 64 + li) * LDB + lh * 8;
#pragma unroll
            for (int s = 0; s < TBM / 16; ++s) {
                bf16x8 yh[2], yl[2], xh[2], xl[2];
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    yh[i] = *reinterpret_cast<const bf16x8*>(Yb + i * 32 * LDB + s * 16);
                    yl[i] = *reinterpret_cast<const bf16x8*>(Yb + PL + i * 32 * LDB + s * 16);
                    xh[i] = *reinterpret_cast<const bf16x8*>(Xb + i * 32 * LDB + s * 16);
                    xl[i] = *reinterpret_cast<const bf16x8*>(Xb + PL + i * 32 * LDB + s * 16);
                }
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) acc[i][j] = mfma_x3(yh[i], yl[i], xh[j], xl[j], acc[i][j]);
            }
            if (has_next) sstore(cur ^ 1);
            __syncthreads();
            cur ^= 1;
        }
    }

    const int npad = ntn * TB, kpad = ntk * TB;
    float* slab = a.slab + (size_t)split * npad * kpad;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int n = n0 + wr * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                const int k = k0 + wc * 64 + j * 32 + li;
                slab[(size_t)n * kpad + k] = acc[i][j][r];
            }
    // bias gradient: the 4 row groups of the dY stagers reduce through LDS (fixed order);
    // the staging buffers are free here (the loop ended on a barrier)
    if (tk == 0) {
        float* dbred = reinterpret_cast<float*>(smem);   // [4][TB]
        if (!isx) {
            dbred[rg * TB + cg * 4 + 0] = dbacc.x;
            dbred[rg * TB + cg * 4 + 1] = dbacc.y;
            dbred[rg * TB + cg * 4 + 2] = dbacc.z;
            dbred[rg * TB + cg * 4 + 3] = dbacc.w;
        }
        __syncthreads();
        if (t < TB)
            a.db_slab[(size_t)split * npad + n0 + t] =
                ((dbred[t] + dbred[TB + t]) + dbred[2 * TB + t]) + dbred[3 * TB + t];
    }
}

__global__ void pack_weight_x3_kernel(const float* __restrict__ W, int N, int K_orig, const int32_t* __restrict__ col_map,
                                      int Kp, int npad, __bf16* __restrict__ Wph, __bf16* __restrict__ Wpl,
                                      __bf16* __restrict__ Wth, __bf16* __restrict__ Wtl, int ldwt, int kpad_rows) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)npad * Kp;
    if (idx < total) {
        const int n = (int)(idx / Kp), k = (int)(idx - (idx / Kp) * Kp);
        const int src = col_map[k];
        const float v = (n < N && src >= 0 && src < K_orig) ? W[(int64_t)n * K_orig + src] : 0.f;
        const __bf16 h = (__bf16)v;
        const __bf16 l = (__bf16)(v - (float)h);
        if (Wph) { Wph[idx] = h; Wpl[idx] = l; }
        if (Wth && n < ldwt) { Wth[(int64_t)k * ldwt + n] = h; Wtl[(int64_t)k * ldwt + n] = l; }
    }
    if (Wth) {
        const int64_t pad_total = (int64_t)(kpad_rows - Kp) * ldwt;
        if (idx < pad_total) {
            Wth[(int64_t)Kp * ldwt + idx] = (__bf16)0.f;
            Wtl[(int64_t)Kp * ldwt + idx] = (__bf16)0.f;
        }
    }
}

bool build_segs(const nerf_seg* segs, int n, SegList& L) {
    if (!segs || n < 1 || n > MAX_SEGS) return false;
    int koff = 0;
    for (int i = 0; i < n; ++i) {
        const nerf_seg& s = segs[i];
        if (!s.ptr || s.k <= 0 || (s.k % 4) != 0 || s.ld < s.k || (s.ld % 4) != 0 || s.row_div < 1) return false;
        if (!aligned16(s.ptr)) return false;
        const int kp = (s.k + BK - 1) / BK * BK;
        L.ptr[i] = s.ptr; L.ld[i] = s.ld; L.k[i] = s.k; L.kp[i] = kp; L.row_div[i] = s.row_div; L.koff[i] = koff;
        koff += kp;
    }
    for (int i = n; i < MAX_SEGS; ++i) {
        L.ptr[i] = nullptr; L.ld[i] = 0; L.k[i] = 0; L.kp[i] = 0; L.row_div[i] = 1; L.koff[i] = koff;
    }
    L.n = n;
    L.ktot = koff;
    return true;
}

int cu_count_x3() {
    static int cached[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (cached[dev] == 0) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        cached[dev] = n;
    }
    return cached[dev];
}

}  // namespace

// same split policy as the fp32 weight-gradient (shared workspace / reduce kernel)
extern "C" size_t nerf_linear_wgrad_workspace(int64_t M, int32_t N, int32_t K);
int nerf_wgrad_choose_splits(int64_t M, int tiles);

extern "C" int nerf_linear_fwd_x3(const nerf_seg* segs, int32_t n_segs, int64_t M, const void* W_hi, const void* W_lo,
                                  int32_t ldw, int32_t N, const float* bias, float* out, int64_t ldo,
                                  int32_t epilogue, const float* aux, int64_t ld_aux, void* stream) {
    NERF_REQUIRE(M >= 0 && M < (1ll << 31) && N >= 1);
    if (M == 0) return NERF_OK;
    SegList L;
    NERF_REQUIRE(build_segs(segs, n_segs, L));
    NERF_REQUIRE(W_hi && W_lo && out && aligned16(W_hi) && aligned16(W_lo) && ldw == L.ktot && (ldw % 8) == 0 &&
                 ldo >= N);
    if (epilogue & NERF_EPI_BIAS) NERF_REQUIRE(bias != nullptr);
    if (epilogue & NERF_EPI_MASK) NERF_REQUIRE(aux != nullptr && ld_aux >= N);
    const int vec_ok = aligned16(out) && (ldo % 4) == 0 && (!(epilogue & NERF_EPI_BIAS) || aligned16(bias)) &&
                       (!(epilogue & NERF_EPI_MASK) || (aligned16(aux) && (ld_aux % 4) == 0));
    NTArgs a{L, (int)M, reinterpret_cast<const __bf16*>(W_hi), reinterpret_cast<const __bf16*>(W_lo), ldw, N, bias,
             out, ldo, epilogue, aux, ld_aux, vec_ok};
    const int ntm = (int)((M + 127) / 128);
    const int ntn = (N + 127) / 128;
    const int ntiles = (ntm + 7) / 8 * 8 * ntn;
    int grid = ntiles;
    if (!(epilogue & NERF_EPI_NO_PERSIST)) {
        const int cap = 2 * cu_count_x3();
        if (grid > cap) grid = cap;
    }
    hipLaunchKernelGGL(linear_nt_x3_kernel, dim3((unsigned)grid), dim3(256), 0, as_stream(stream), a, ntm, ntiles);
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}

extern "C" int nerf_linear_wgrad_x3(const float* dY, int64_t ld_dy, int32_t N, const nerf_seg* segs, int32_t n_segs,
                                    int64_t M, void* workspace, size_t workspace_bytes, void* stream) {
    NERF_REQUIRE(dY && N >= 1 && M >= 0 && M < (1ll << 31) && aligned16(dY) && (ld_dy % 4) == 0 && (N % 4) == 0 &&
                 ld_dy >= N);
    SegList L;
    NERF_REQUIRE(build_segs(segs, n_segs, L));
    const int ntn = (N + TB - 1) / TB, ntk = (L.ktot + TB - 1) / TB;
    const int splits = nerf_wgrad_choose_splits(M, ntn * ntk);
    const size_t need = nerf_linear_wgrad_workspace(M, N, L.ktot);
    if (!workspace || workspace_bytes < need || !aligned16(workspace)) return NERF_ERR_WORKSPACE;
    float* slab = reinterpret_cast<float*>(workspace);
    float* db_slab = slab + (size_t)splits * ntn * TB * (size_t)ntk * TB;
    int64_t mps = (M + splits - 1) / splits;
    mps = ((mps + TBM - 1) / TBM) * TBM;
    TNArgs a{dY, ld_dy, N, L, (int)M, (int)mps, splits, slab, db_slab};
    const int64_t blocks = (int64_t)splits * ntn * ntk;
    hipLaunchKernelGGL(linear_wgrad_x3_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), a);
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}

extern "C" int nerf_pack_weight_x3(const float* W, int32_t N, int32_t K_orig, const int32_t* col_map, int32_t Kp,
                                   void* Wp_hi, void* Wp_lo, void* Wt_hi, void* Wt_lo, int32_t ldwt, void* stream) {
    NERF_REQUIRE(W && col_map && N >= 1 && K_orig >= 1 && Kp >= 1 && (Kp % BK) == 0);
    NERF_REQUIRE((Wp_hi == nullptr) == (Wp_lo == nullptr) && (Wt_hi == nullptr) == (Wt_lo == nullptr));
    const int npad = ((N + 127) / 128) * 128;
    if (Wt_hi) NERF_REQUIRE(ldwt >= ((N + 31) / 32) * 32);
    const int kpad_rows = ((Kp + 127) / 128) * 128 + 128;
    int64_t total = (int64_t)npad * Kp;
    const int64_t pad_total = (int64_t)(kpad_rows - Kp) * (Wt_hi ? ldwt : 0);
    if (pad_total > total) total = pad_total;
    hipLaunchKernelGGL(pack_weight_x3_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, as_stream(stream), W,
                       N, K_orig, col_map, Kp, npad, reinterpret_cast<__bf16*>(Wp_hi), reinterpret_cast<__bf16*>(Wp_lo),
                       reinterpret_cast<__bf16*>(Wt_hi), reinterpret_cast<__bf16*>(Wt_lo), ldwt, kpad_rows);
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}
