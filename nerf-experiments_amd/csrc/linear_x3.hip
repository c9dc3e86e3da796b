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
// 32-wide chunks.  A (fp32 in HBM) is split while it is staged into LDS.
// LDS planes are [row][32] bf16 (64-byte rows, no padding) with the 16-byte
// slots of each row PAIR permuted (swz below): the 16 rows a ds_read_b128 lane
// group reads and the 128 contiguous bytes a ds_write_b64 / ds_write_b128 lane
// group writes (two rows, or one column of 8 rows 4 apart in the transposed TN
// staging) all land on distinct bank slots.  Lane (r, h) of the 32x32x16 MFMA
// holds row r, k = 8h .. 8h+7 of both operands: one ds_read_b128 per plane and block.
//
// TN (weight gradient): slab[s][n][k] = sum_m dY[m][n] X[m][k]; the sample index
// is the MFMA reduction dimension, so dY and X are staged TRANSPOSED ([n][m],
// [k][m]): a thread loads 8 rows x 4 columns and writes four 8-sample bf16
// vectors per plane (ds_write_b128).  Layers with N, K <= 256 take one 256 x 256 tile whose
// operands stream through an LDS-DMA ring (linear_wgrad_x3_stream_kernel).
#include "common.h"

using namespace nerf;

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

namespace {

constexpr int BK = 32;
constexpr int LDB = BK;       // bf16 elements per LDS row (64 bytes)

// bf16 element offset of 16-byte slot `slot` (0..3) of row `row` in a swizzled plane:
// rows 2p and 2p+1 share a 128-byte line whose 8 slots are XOR-permuted by (row >> 2) & 7.
__device__ __forceinline__ int swz(int row, int slot) {
    return (row >> 1) * 64 + ((((row & 1) << 2) | slot) ^ ((row >> 2) & 7)) * 8;
}
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
// the weight gradients' products: the 3 x bf16 split, or (X1: matmul precision "medium") one bf16 pass
template <bool X1>
__device__ __forceinline__ f32x16 mfma_w(bf16x8 ah, bf16x8 al, bf16x8 bh, bf16x8 bl, f32x16 c) {
    if constexpr (X1)
        return mfma16(ah, bh, c);
    else
        return mfma_x3(ah, al, bh, bl, c);
}

__device__ __forceinline__ void split4(f4 v, bf16x4& hi, bf16x4& lo) {
    hi = __builtin_convertvector(v, bf16x4);
    lo = __builtin_convertvector(v - __builtin_convertvector(hi, f4), bf16x4);
}

// 8 values -> their bf16 hi and lo halves (hi = bf16(x), lo = bf16(x - hi), both RNE), one packed
// conversion per PAIR: hi of (x, y) in one v_cvt_pk_bf16_f32, its halves read back as fp32 by a
// shift / a mask, x - hi and y - hi in one v_pk_add_f32, lo in one more conversion (5 VALU per pair)
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void split8_pairs(const float (&x)[8], bf16x8& hi, bf16x8& lo) {
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
    typedef float f2 __attribute__((ext_vector_type(2)));
    u32x4 h, l;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const f2 v = {x[2 * p], x[2 * p + 1]};
        const unsigned hp = __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2));
        const f2 hv = {__builtin_bit_cast(float, hp << 16), __builtin_bit_cast(float, hp & 0xffff0000u)};
        h[p] = hp;
        l[p] = __builtin_bit_cast(unsigned, __builtin_convertvector(v - hv, bf16x2));
    }
    hi = __builtin_bit_cast(bf16x8, h);
    lo = __builtin_bit_cast(bf16x8, l);
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
    const __bf16* Wx; int ldw; int N;      // weights, interleaved [row][ldw/32][hi 32 | lo 32]
    const float* bias;
    float* out; int64_t ldo;
    int epi;
    const float* aux; int64_t ldaux;
    int vec_ok;
    // Gaussian-activation epilogues (nerf_linear_gauss_x3): inverse std, activation output,
    // per-row-tile fp64 column partials of the inverse-std gradient
    const float* gs; float* y2; int64_t ldy2; double* part;
};

// Gaussian activation (garf/gaussian.py:8-31) on a column quad, with exactly the element
// formulas of gauss.hip: v = s^2 + 1e-6, y = exp((-(z*z)) * v); backward ge = g * exp((-(z*z)) v),
// dz = (((-ge) * 2) * z) * v, column partial += (double)((-ge) * z^2).
__device__ __forceinline__ f4 gauss_v4(const float* s, int n) {
#pragma clang fp contract(off)
    const f4 sv = *reinterpret_cast<const f4*>(s + n);
    return sv * sv + 1e-6f;
}

__device__ __forceinline__ void gauss_fwd_store(float* o, float* yo, f4 z, f4 v) {
#pragma clang fp contract(off)
    __builtin_nontemporal_store(z, reinterpret_cast<f4*>(o));
    f4 y;
    y.x = expf((-(z.x * z.x)) * v.x);
    y.y = expf((-(z.y * z.y)) * v.y);
    y.z = expf((-(z.z * z.z)) * v.z);
    y.w = expf((-(z.w * z.w)) * v.w);
    __builtin_nontemporal_store(y, reinterpret_cast<f4*>(yo));
}

__device__ __forceinline__ float gauss_bwd1(float g, float zz, float v, double& acc) {
#pragma clang fp contract(off)
    const float z2 = zz * zz;
    const float ge = g * expf((-z2) * v);
    acc += (double)((-ge) * z2);
    return (((-ge) * 2.0f) * zz) * v;
}

__device__ __forceinline__ void gauss_bwd_store(float* o, f4 g, f4 z, f4 v, double (&acc)[4]) {
    f4 dz;
    dz.x = gauss_bwd1(g.x, z.x, v.x, acc[0]);
    dz.y = gauss_bwd1(g.y, z.y, v.y, acc[1]);
    dz.z = gauss_bwd1(g.z, z.z, v.z, acc[2]);
    dz.w = gauss_bwd1(g.w, z.w, v.w, acc[3]);
    __builtin_nontemporal_store(dz, reinterpret_cast<f4*>(o));
}

// ------------------------------------------------------------------------- NT
__global__ __launch_bounds__(256, 2) void linear_nt_x3_kernel(NTArgs a, int ntm, int ntiles) {
    const EpiOut E{a.out, a.ldo, a.bias, a.aux, a.ldaux, a.M, a.N, a.epi, a.vec_ok};
    constexpr int BM = 128, BN = 128;
    constexpr int PL = BM * LDB;                 // one bf16 plane (128 rows)
    constexpr int BUFB = 4 * PL;                 // A hi, A lo, W hi, W lo (bf16 elements)
    constexpr int LDC = BN;                      // 32-lane row writes / 16-byte row reads: conflict-free
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
        for (int j = 0; j < 2; ++j) woff[j] = (int64_t)(nbase + j * 64 + wrow) * a.ldw * 2 + w8;
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
            rwh[j] = *reinterpret_cast<const u16x8*>(a.Wx + woff[j] + 2 * (skoff + kc));
            rwl[j] = *reinterpret_cast<const u16x8*>(a.Wx + woff[j] + 2 * (skoff + kc) + 32);
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
            const int o = swz(i * 32 + rbase, c4 >> 1) + (c4 & 1) * 4;
            *reinterpret_cast<bf16x4*>(Ah + o) = h;
            *reinterpret_cast<bf16x4*>(Al + o) = l;
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int o = swz(j * 64 + wrow, w8 >> 3);
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

#pragma unroll
            for (int s = 0; s < BK / 16; ++s) {
                const __bf16* Ah = smem + cur * BUFB + swz(wr * 64 + li, 2 * s + lh);
                const __bf16* Wb = smem + cur * BUFB + 2 * PL + swz(wc * 64 + li, 2 * s + lh);
                bf16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    ah[i] = *reinterpret_cast<const bf16x8*>(Ah + i * 32 * LDB);
                    al[i] = *reinterpret_cast<const bf16x8*>(Ah + PL + i * 32 * LDB);
                    bh[i] = *reinterpret_cast<const bf16x8*>(Wb + i * 32 * LDB);
                    bl[i] = *reinterpret_cast<const bf16x8*>(Wb + PL + i * 32 * LDB);
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
        const bool gmode = (a.epi & (NERF_EPI_GAUSS | NERF_EPI_GAUSS_BWD)) != 0;
        double gp[4] = {0.0, 0.0, 0.0, 0.0};
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
                const f4 c = *reinterpret_cast<const f4*>(Cs + row * LDC + cq * 4);
                if (gmode) {
                    // N % 4 == 0 and 16-byte rows (nerf_linear_gauss_x3 checks): whole quads
                    if (m < a.M && n < a.N) {
                        const f4 v = gauss_v4(a.gs, n);
                        if (a.epi & NERF_EPI_GAUSS) {
                            f4 z = c;
                            if (a.epi & NERF_EPI_BIAS) z += *reinterpret_cast<const f4*>(a.bias + n);
                            gauss_fwd_store(a.out + (int64_t)m * a.ldo + n, a.y2 + (int64_t)m * a.ldy2 + n, z, v);
                        } else {
                            gauss_bwd_store(a.out + (int64_t)m * a.ldo + n, c,
                                            *reinterpret_cast<const f4*>(a.aux + (int64_t)m * a.ldaux + n), v, gp);
                        }
                    }
                } else {
                    epi_quad<BN / 4>(E, m < a.M && n < a.N, m, n, c);
                }
            }
            __syncthreads();
        }
        if (a.epi & NERF_EPI_GAUSS_BWD) {
            // the tile's column partials: thread t holds rows = t / 32 (mod 8) of column quad t % 32;
            // the 8 row groups are added in order, one fp64 row per 128-row tile
            static_assert(256 % (BN / 4) == 0, "fixed column quad per thread");
            double* R = reinterpret_cast<double*>(Cs);
            const int grp = t / (BN / 4), cq = t % (BN / 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) R[grp * BN + cq * 4 + e] = gp[e];
            __syncthreads();
            if (t < BN && n0 + t < a.N) {
                double sum = 0.0;
#pragma unroll
                for (int g = 0; g < 256 / (BN / 4); ++g) sum += R[g * BN + t];
                a.part[(int64_t)(m0 / BM) * a.N + n0 + t] = sum;
            }
            __syncthreads();
        }

        if (!has_next_tile) break;
        tile = ntile;
        m0 = ntm_ * BM;
        n0 = ntn_ * BN;
    }
}

// ------------------------------------------------------------------- NT glds
// 32 < N <= 256: 256-row x BN-column tile (BN = 128 JN), 8 waves (2 x 4) of 128 x 32 JN,
// every operand staged by LDS-DMA (global_load_lds_dwordx4: no VGPR round trip, no
// ds_write pass).  A is staged as raw fp32 and split into bf16 hi/lo as the fragments
// are read out of LDS; the weights arrive pre-split and interleaved ([row][k/32][hi 32 | lo 32]).
// Both LDS images have 128-byte rows whose 16-byte slots are XOR-permuted by (row >> 1) & 7;
// the permutation is applied to the per-lane SOURCE address (the DMA destination is
// lane-linear) and to the fragment reads, which it makes bank-conflict-free.
// Pipeline: A (streamed from HBM) runs two chunks ahead in a 3-stage ring, W (L2-resident)
// one chunk ahead in a 2-stage ring — 64 KB of A in flight per CU; all LDS is this ring
// (160 KB for BN = 256).  In-loop waits are counted vmcnt, barriers raw, so the prefetch is
// never drained by a __syncthreads().
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

__device__ __forceinline__ int swz128(int row, int slot) { return row * 128 + ((slot ^ ((row >> 1) & 7)) << 4); }

template <int EPI, int JN>
__global__ __launch_bounds__(512, 1) void linear_nt_x3_glds_kernel(NTArgs a, int ntiles) {
    constexpr int BM = 256, BN = 128 * JN;
    constexpr int ABYTES = BM * 128, WBYTES = BN * 128;
    constexpr int LW = 8;                       // waves issuing the DMA (all; a 4/4 loader/storer split measured slower)
    constexpr int EW = LW == 8 ? 8 : 8 - LW;    // waves running the epilogue's global phase
    constexpr int QA = BM / (8 * LW);           // A DMA instructions per loader wave per chunk (8 rows each)
    constexpr int QW = BN / (8 * LW);           // W DMA instructions per loader wave per chunk
    // ONE __shared__ array (a second LDS object makes hipcc drain the DMA before ds_reads)
    __shared__ __attribute__((aligned(16))) char smem[3 * ABYTES + 2 * WBYTES];
    char* const Aring = smem;
    char* const Wring = smem + 3 * ABYTES;

    const int t = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6), lane = t & 63;
    const int wr = wave >> 2, wc = wave & 3;
    const int li = lane & 31, lh = lane >> 5;
    const int lrow = lane >> 3, lphys = lane & 7;        // DMA lane -> (row in 8-row group, physical slot)

    if ((int)blockIdx.x >= ntiles) return;
    const int nchunks = a.A.ktot / BK;
    const int my_tiles = (ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
    const int total = my_tiles * nchunks;

    // segment table in scalar registers; the empty asm keeps the compiler from turning the
    // selects of pick4 back into an indexed load of the by-value argument (which it would
    // then copy to scratch)
    // segment fields indexed by the (wave-uniform) segment number are read straight from the
    // kernel-argument segment with scalar loads: indexing the by-value argument (or selecting
    // among its fields, which the optimizer folds into an indexed load) makes hipcc copy the
    // whole argument to scratch
    typedef __attribute__((address_space(4))) const char kchar_t;
    kchar_t* kargs = (kchar_t*)__builtin_amdgcn_kernarg_segment_ptr();
#define NERF_SEGF(T, field, i)                                                                         \
    (*(const __attribute__((address_space(4))) T*)(kargs + offsetof(NTArgs, A) + offsetof(SegList, field) + \
                                                    (size_t)(i) * sizeof(T)))
    typedef const float* cfptr_t;

    // ---- A DMA cursor.  Each tile walks its K chunks starting at chunk (tile % nchunks),
    // wrapping around, so workgroups reach their epilogues (store bursts) at different
    // times; the summation order is a function of the tile index only (grid-independent).
    int a_tile = blockIdx.x, a_i = 0, a_seg = -1, a_kc = 0;
    const float* sp = nullptr;
    int sk = 0;
    int64_t sld = 0;
    unsigned asrc[QA];            // source row of each A DMA instruction of this lane
    // rows of instruction q are q*8 + lrow (mod 64): the swizzle term only depends on q & 1
    const int alog0 = lphys ^ ((lrow >> 1) & 7), alog1 = lphys ^ (4 + ((lrow >> 1) & 7));
    auto a_locate = [&](bool new_tile) __attribute__((always_inline)) {
        int c = a_i + a_tile % nchunks;
        c = c >= nchunks ? c - nchunks : c;
        int sgi = 0;
        while (sgi + 1 < a.A.n && c * BK >= NERF_SEGF(int, koff, sgi + 1)) ++sgi;
        a_kc = c * BK - NERF_SEGF(int, koff, sgi);
        if (new_tile || sgi != a_seg) {
            a_seg = sgi;
            sp = NERF_SEGF(cfptr_t, ptr, sgi);
            sld = NERF_SEGF(int64_t, ld, sgi);
            sk = NERF_SEGF(int, k, sgi);
            const unsigned rd = (unsigned)NERF_SEGF(int, row_div, sgi);
            const int m0 = a_tile * BM;
#pragma unroll
            for (int q = 0; q < QA; ++q) {
                int m = m0 + (wave * QA + q) * 8 + lrow;
                m = m < a.M ? m : a.M - 1;                // rows past M: any valid row (discarded)
                asrc[q] = (rd == 1u) ? (unsigned)m : (unsigned)m / rd;
            }
        }
    };
    a_locate(true);
    const bool loader = wave < LW;
    auto issue_a = [&](int stage) __attribute__((always_inline)) {
        char* base = Aring + stage * ABYTES;
        if (loader)
#pragma unroll
        for (int q = 0; q < QA; ++q) {
            const int col = a_kc + ((q & 1) ? alog1 : alog0) * 4;
            const float* src = sp + (int64_t)asrc[q] * sld + (col < sk ? col : 0);   // past k: finite data x zero weights
            __builtin_amdgcn_global_load_lds((glb_void_t*)src, (lds_void_t*)(base + (wave * QA + q) * 1024), 16, 0, 0);
        }
        if (++a_i == nchunks) {
            a_i = 0;
            a_tile += gridDim.x;
            if (a_tile < ntiles) a_locate(true);
        } else {
            a_locate(false);
        }
    };
    // ---- W DMA cursor
    const int nkc = a.ldw / BK;                          // 32-wide chunks per weight row
    unsigned woff[QW];                                   // bf16 element offsets (weights are small)
#pragma unroll
    for (int q = 0; q < QW; ++q) {
        const int row = (wave * QW + q) * 8 + lrow;
        const int n = row < a.N ? row : a.N - 1;         // rows past N: any valid row (discarded)
        woff[q] = (unsigned)n * nkc * 64 + ((lphys ^ ((row >> 1) & 7)) << 3);
    }
    int w_tile = blockIdx.x, w_i = 0;
    auto issue_w = [&](int stage) __attribute__((always_inline)) {
        char* base = Wring + stage * WBYTES;
        int c = w_i + w_tile % nchunks;
        c = c >= nchunks ? c - nchunks : c;
        if (loader)
#pragma unroll
        for (int q = 0; q < QW; ++q) {
            const __bf16* src = a.Wx + woff[q] + (unsigned)c * 64u;
            __builtin_amdgcn_global_load_lds((glb_void_t*)src, (lds_void_t*)(base + (wave * QW + q) * 1024), 16, 0, 0);
        }
        if (++w_i == nchunks) {
            w_i = 0;
            w_tile += gridDim.x;
        }
    };

    f32x16 acc[4][JN];
    auto zero_acc = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < JN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    };
    auto compute = [&](int astage, int wstage) __attribute__((always_inline)) {
        const char* Ab = Aring + astage * ABYTES;
        const char* Wb = Wring + wstage * WBYTES;
#pragma unroll
        for (int s = 0; s < BK / 16; ++s) {
            bf16x8 bh[JN], bl[JN];
#pragma unroll
            for (int j = 0; j < JN; ++j) {
                const int row = wc * (BN / 4) + j * 32 + li;
                bh[j] = *reinterpret_cast<const bf16x8*>(Wb + swz128(row, 2 * s + lh));
                bl[j] = *reinterpret_cast<const bf16x8*>(Wb + swz128(row, 4 + 2 * s + lh));
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = wr * 128 + i * 32 + li;
                const f4 x0 = *reinterpret_cast<const f4*>(Ab + swz128(row, 4 * s + 2 * lh));
                const f4 x1 = *reinterpret_cast<const f4*>(Ab + swz128(row, 4 * s + 2 * lh + 1));
                bf16x4 h0, l0, h1, l1;
                split4(x0, h0, l0);
                split4(x1, h1, l1);
                const bf16x8 ah = __builtin_shufflevector(h0, h1, 0, 1, 2, 3, 4, 5, 6, 7);
                const bf16x8 al = __builtin_shufflevector(l0, l1, 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
                for (int j = 0; j < JN; ++j) acc[i][j] = mfma_x3(ah, al, bh[j], bl[j], acc[i][j]);
            }
        }
    };

    // bias of this thread's epilogue column quad (N <= BN: one column tile), loaded before
    // any DMA is in flight
    constexpr int C4 = BN / 4;                    // float4 columns per row
    constexpr int RS = 64 * EW / C4;              // rows per epilogue sweep
    const int et = t & (64 * EW - 1);
    const int ec4 = et % C4, erow = et / C4;
    const int en = ec4 * 4;
    f4 bias4 = f4{0.f, 0.f, 0.f, 0.f};
    if ((EPI & NERF_EPI_BIAS) && a.vec_ok && en + 4 <= a.N) bias4 = *reinterpret_cast<const f4*>(a.bias + en);
    constexpr bool GF = (EPI & NERF_EPI_GAUSS) != 0, GB = (EPI & NERF_EPI_GAUSS_BWD) != 0;
    f4 gv4 = f4{0.f, 0.f, 0.f, 0.f};
    if ((GF || GB) && en + 4 <= a.N) gv4 = gauss_v4(a.gs, en);
    double gp[4] = {0.0, 0.0, 0.0, 0.0};          // GB: this thread's column-quad partials of the tile
    const EpiOut E{a.out, a.ldo, a.bias, a.aux, a.ldaux, a.M, a.N,
                   EPI | (a.epi & (NERF_EPI_MASKBITS | NERF_EPI_MASKOUT)), a.vec_ok};
    const bool mbits = (a.epi & NERF_EPI_MASKBITS) != 0, mout = (a.epi & NERF_EPI_MASKOUT) != 0;
    unsigned char* mask8 = (unsigned char*)a.aux;
    auto barrier = []() __attribute__((always_inline)) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    // epilogue: 64 rows per pass, rows 0-31 in the free A stage, 32-63 in the free W stage
    int c_tile = blockIdx.x, c_chunk = 0;
    // Epilogue: PR rows per pass through the free A stage (C0, rows 0-31) and the free W stage
    // (C1, rows 32-63 of a 64-row pass).  Masked variants use 32-row passes and stage the tile's
    // 256 rows of ReLU mask bits (8 KB) in C1 with one LDS-DMA per thread up front: one memory
    // round trip per tile instead of one per batch of rows.
    constexpr bool MSK = (EPI & NERF_EPI_MASK) != 0;
    constexpr int PR = MSK ? 32 : 64;
    static_assert(32 * BN * 4 <= ABYTES && 32 * BN * 4 <= WBYTES && BM * 32 <= WBYTES, "epilogue staging");
    auto epilogue = [&](int astage, int wstage) __attribute__((always_inline)) {
        float* C0 = reinterpret_cast<float*>(Aring + astage * ABYTES);
        float* C1 = reinterpret_cast<float*>(Wring + wstage * WBYTES);
        const unsigned* mbits_lds = reinterpret_cast<const unsigned*>(C1);
        const int tm0 = c_tile * BM;
        const bool vec = a.vec_ok && en + 4 <= a.N;
        if (MSK && mbits) {
            int m = tm0 + (t >> 1);
            m = m < a.M ? m : a.M - 1;
            const char* src = reinterpret_cast<const char*>(a.aux) + (int64_t)m * a.ldaux + (t & 1) * 16;
            __builtin_amdgcn_global_load_lds((glb_void_t*)src, (lds_void_t*)(reinterpret_cast<char*>(C1) + wave * 1024),
                                             16, 0, 0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        // rows r0 .. r0+PR-1 of the tile; acc blocks c (rows 0-31) and d (rows 32-63, PR = 64)
        auto pass = [&](int r0, int wr_owner, const f32x16 (&c)[JN], const f32x16 (&d)[JN]) __attribute__((always_inline)) {
            if (wr == wr_owner) {
#pragma unroll
                for (int j = 0; j < JN; ++j)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int row = (r & 3) + 8 * (r >> 2) + 4 * lh;
                        C0[row * BN + wc * (BN / 4) + j * 32 + li] = c[j][r];
                        if (PR == 64) C1[row * BN + wc * (BN / 4) + j * 32 + li] = d[j][r];
                    }
            }
            barrier();
            // aux / out reads of a batch of rows are issued together (one memory round trip
            // per batch instead of one per row)
            constexpr int UB = PR / RS < 4 ? PR / RS : 4;       // rows per batch
#pragma unroll
            for (int qb = 0; qb < PR / RS; qb += UB) {
                f4 xa[UB], xo[UB];
                unsigned xb[UB];
                if (vec && (EPI & (NERF_EPI_MASK | NERF_EPI_ACCUM | NERF_EPI_GAUSS_BWD))) {
#pragma unroll
                    for (int u = 0; u < UB; ++u) {
                        int m = tm0 + r0 + erow + RS * (qb + u);
                        m = m < a.M ? m : a.M - 1;
                        if ((MSK && !mbits) || GB) xa[u] = *reinterpret_cast<const f4*>(a.aux + (int64_t)m * a.ldaux + en);
                        if (EPI & NERF_EPI_ACCUM) xo[u] = *reinterpret_cast<const f4*>(a.out + (int64_t)m * a.ldo + en);
                    }
                }
                if (MSK && mbits) {
#pragma unroll
                    for (int u = 0; u < UB; ++u) {
                        const unsigned* wrow = mbits_lds + (r0 + erow + RS * (qb + u)) * 8 + (ec4 >> 5);
                        const int b = ec4 & 31;
                        xb[u] = ((wrow[0] >> b) & 1u) | (((wrow[2] >> b) & 1u) << 1) | (((wrow[4] >> b) & 1u) << 2) |
                                (((wrow[6] >> b) & 1u) << 3);
                    }
                }
#pragma unroll
                for (int u = 0; u < UB; ++u) {
                    const int row = erow + RS * (qb + u);
                    const int m = tm0 + r0 + row;
                    const bool ok = m < a.M && en < a.N;
                    const float* Cr = row < 32 ? C0 + row * BN : C1 + (row - 32) * BN;
                    f4 v = *reinterpret_cast<const f4*>(Cr + en);
                    unsigned nib = 0;
                    if (ok && vec && GF) {
                        // pre-activation to out (kept for the backward), activation to y2
                        if (EPI & NERF_EPI_BIAS) v += bias4;
                        gauss_fwd_store(a.out + (int64_t)m * a.ldo + en, a.y2 + (int64_t)m * a.ldy2 + en, v, gv4);
                    } else if (ok && vec && GB) {
                        gauss_bwd_store(a.out + (int64_t)m * a.ldo + en, v, xa[u], gv4, gp);
                    } else if (ok && vec) {
                        float* o = a.out + (int64_t)m * a.ldo + en;
                        if (EPI & NERF_EPI_BIAS) v += bias4;
                        if (EPI & NERF_EPI_RELU) {
                            v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
                        }
                        if (MSK) v = mbits ? apply_bits(v, xb[u]) : apply_sign(v, xa[u]);
                        if (EPI & NERF_EPI_ACCUM) v = xo[u] + v;
                        __builtin_nontemporal_store(v, reinterpret_cast<f4*>(o));
                        nib = quad_bits(v);
                    } else if (ok) {
                        nib = epi_quad_lane(E, m, en, v);      // partial / unaligned quads (bias from memory)
                    }
                    if (mout) store_quad_bits<C4>(mask8 + (int64_t)m * a.ldaux, m < a.M, 0, nib);
                }
            }
            barrier();
        };
        if (PR == 64) {
            pass(0, 0, acc[0], acc[1]);
            pass(64, 0, acc[2], acc[3]);
            pass(128, 1, acc[0], acc[1]);
            pass(192, 1, acc[2], acc[3]);
        } else {
#pragma unroll
            for (int p = 0; p < 8; ++p) {
                // compile-time acc indices once unrolled
                pass(32 * p, p >> 2, acc[p & 3], acc[p & 3]);
            }
        }
        if (GB) {
            // the tile's inverse-std gradient column partials: the RS row groups of each column
            // quad added in order through the free A stage, one fp64 row per 256-row tile
            double* R = reinterpret_cast<double*>(C0);
            static_assert(RS * BN * 8 <= ABYTES, "partials staging");
#pragma unroll
            for (int e = 0; e < 4; ++e) R[erow * BN + en + e] = gp[e];
            barrier();
            if (t < BN && t < a.N) {
                double sum = 0.0;
#pragma unroll
                for (int r = 0; r < RS; ++r) sum += R[r * BN + t];
                a.part[(int64_t)c_tile * a.N + t] = sum;
            }
            barrier();
#pragma unroll
            for (int e = 0; e < 4; ++e) gp[e] = 0.0;
        }
    };

    // prologue: A(0), W(0), A(1); iteration g issues W(g+1), A(g+2) and waits for A(g), W(g)
    // (a loop, not three call sites: fewer inlined copies of the cursor code)
    for (int q = 0; q < 3; ++q) {
        if (q == 1) issue_w(0);
        else if (q / 2 < total) issue_a(q / 2);
    }
    zero_acc();
    int as = 0, ws = 0;                 // ring slots of chunk g
    for (int g = 0; g < total; ++g) {
        const int as2 = as == 0 ? 2 : as - 1;           // (g + 2) % 3
        if (g + 2 < total) {
            issue_w(ws ^ 1);
            issue_a(as2);
            if (loader) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * QA + QW) : "memory");
        } else if (g + 1 < total) {
            issue_w(ws ^ 1);
            if (loader) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(QA + QW) : "memory");
        } else if (loader) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        barrier();                      // chunk g visible to every wave
        compute(as, ws);
        barrier();                      // every wave done reading chunk g's stages
        if (++c_chunk == nchunks) {
            epilogue(as, ws);
            zero_acc();
            c_chunk = 0;
            c_tile += gridDim.x;
        }
        as = as == 2 ? 0 : as + 1;
        ws ^= 1;
    }
#undef NERF_SEGF
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
    // a second block of rows (the other pass of a field used twice per step): rows m >= M0 read
    // dY1 / X1 row m - M0 (M0 = M and the block unused for a single block); X1 has X's segment
    // structure, only its pointers, row strides and row divisors differ
    int M0;
    const float* dY1; int64_t lddy1;
    const float* x1ptr[MAX_SEGS]; int64_t x1ld[MAX_SEGS]; int x1rd[MAX_SEGS];
    // streamed kernel only: per-ray sums of dY (raysum[ray][n], rays of rs_S0 / rs_S1 samples in the
    // two blocks, block 1's rays after block 0's rs_B0) for a per-ray input's weight gradient, or null
    float* raysum; int rs_S0, rs_S1, rs_B0;
};

template <bool X1>
__global__ __launch_bounds__(256, 2) void linear_wgrad_x3_kernel(TNArgs a) {
    constexpr int PL = TB * LDB;          // one transposed bf16 plane: 128 rows x 32 samples (swizzled)
    constexpr int BUFB = 4 * PL;          // dY^T hi, lo, X^T hi, lo
    __shared__ __attribute__((aligned(16))) __bf16 smem[2 * BUFB];

    const int ntn = (a.N + TB - 1) / TB;
    const int ntk = (a.X.ktot + TB - 1) / TB;
    const int tiles = ntn * ntk;
    // XCD-aware block order (speed only): the tiles of one M split read the same dY / X rows, so
    // they are given consecutive logical ids on blocks that share an XCD (blockIdx % 8, dealt
    // round-robin) and meet in that XCD's L2 instead of each fetching the rows from HBM (bijective
    // for any grid size: MI355X guide, XCD swizzle)
    const int bid = [] {
        const int nwg = (int)gridDim.x, orig = (int)blockIdx.x, xcd = orig % 8, q = nwg / 8, r = nwg % 8;
        return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
    }();
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
    const float *gptr, *gptr1;
    int64_t gld, gld1;
    unsigned grd = 1, grd1 = 1;
    bool col_ok;
    int gcol;
    if (!isx) {
        gcol = n0 + cg * 4;
        col_ok = gcol < a.N;
        gptr = a.dY;
        gld = a.lddy;
        gptr1 = a.dY1;
        gld1 = a.lddy1;
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
        gptr1 = col_ok ? pick4(a.x1ptr, xs) : a.dY;
        gld1 = col_ok ? pick4(a.x1ld, xs) : 0;
        grd1 = col_ok ? (unsigned)pick4(a.x1rd, xs) : 1u;
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
    // waves whose lanes all read one source row per sample take the pointer walk below (decided
    // per wave: a wave mixing the two forms would run both)
    const bool wave_rd1 = __ballot(grd != 1u || grd1 != 1u) == 0;
    auto gload = [&](int mc) __attribute__((always_inline)) {
        const int m0 = mc + rg * 8;
        const bool in1 = m0 >= a.M0;                    // the 8 rows' block (when they share one)
        if (wave_rd1 && m0 + 8 <= mend && (in1 || m0 + 8 <= a.M0)) {
            // all 8 rows inside the split and one block, one source row per sample: a pointer walk
            const int64_t ld = in1 ? gld1 : gld;
            const float* p = (in1 ? gptr1 : gptr) + (int64_t)(in1 ? m0 - a.M0 : m0) * ld + gcol;
            mmask = 0xffu;
#pragma unroll
            for (int r = 0; r < 8; ++r, p += ld) rv[r] = *reinterpret_cast<const f4*>(p);
        } else {
            mmask = 0;
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const int m = m0 + r;
                const bool mok = m < mend;
                mmask |= (mok ? 1u : 0u) << r;
                const int mm = mok ? m : mbeg;
                const bool b1 = mm >= a.M0;
                const unsigned row = (unsigned)(b1 ? mm - a.M0 : mm), rd = b1 ? grd1 : grd;
                rv[r] = *reinterpret_cast<const f4*>((b1 ? gptr1 : gptr) + (int64_t)(rd == 1u ? row : row / rd) *
                                                                              (b1 ? gld1 : gld) + gcol);
            }
        }
    };
    auto sstore = [&](int buf) __attribute__((always_inline)) {
        __bf16* Ph = smem + buf * BUFB + (isx ? 2 * PL : 0);
        __bf16* Pl = Ph + PL;
        f4 v[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) v[r] = rv[r];
        if (!(col_ok && mmask == 0xffu)) {                 // padded column or the split's last rows
#pragma unroll
            for (int r = 0; r < 8; ++r) v[r] = (col_ok && ((mmask >> r) & 1u)) ? rv[r] : f4{0.f, 0.f, 0.f, 0.f};
        }
        if (!isx) {
#pragma unroll
            for (int r = 0; r < 8; ++r) dbacc += v[r];
        }
        // transpose: column e of the 8 rows -> one 8-sample vector per plane
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            bf16x8 h, l;
            float x[8];
#pragma unroll
            for (int r = 0; r < 8; ++r) x[r] = e == 0 ? v[r].x : (e == 1 ? v[r].y : (e == 2 ? v[r].z : v[r].w));
            split8_pairs(x, h, l);
            const int o = swz(cg * 4 + e, rg);
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
#pragma unroll
            for (int s = 0; s < TBM / 16; ++s) {
                const __bf16* Yb = smem + cur * BUFB + swz(wr * 64 + li, 2 * s + lh);
                const __bf16* Xb = smem + cur * BUFB + 2 * PL + swz(wc * 64 + li, 2 * s + lh);
                bf16x8 yh[2], yl[2], xh[2], xl[2];
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    yh[i] = *reinterpret_cast<const bf16x8*>(Yb + i * 32 * LDB);
                    yl[i] = *reinterpret_cast<const bf16x8*>(Yb + PL + i * 32 * LDB);
                    xh[i] = *reinterpret_cast<const bf16x8*>(Xb + i * 32 * LDB);
                    xl[i] = *reinterpret_cast<const bf16x8*>(Xb + PL + i * 32 * LDB);
                }
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) acc[i][j] = mfma_w<X1>(yh[i], yl[i], xh[j], xl[j], acc[i][j]);
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

// ------------------------------------------------------------------- TN stream
// The 256 x 256 weight-gradient tile (N, K <= 256: one tile per layer, dY and X each read from
// HBM once per M split) with the operands streamed by LDS-DMA.  (It replaced a register-staged
// kernel — 8-sample loads, split, transposed LDS writes — that had 64 KB per CU in flight only
// while its MFMAs ran: 343-368 vs 326-336 us at M = 524 288, bitwise equal weight gradients;
// tools/wgrad_ab.py.)  The raw fp32
// rows (16 samples x 256 columns of dY and of X: 32 KB per step) land in a 3-stage ring two
// steps ahead of the step being multiplied, so two steps (64 KB) are always in flight; the only
// vector-memory ops in the loop are these DMAs, so the counted waits track them alone.  Each
// step, thread (operand, column c) reads its column's 16 samples from the ring (conflict-free:
// a wave reads 64 consecutive columns of a row), splits them into bf16 hi/lo and writes one
// 64-byte image row [hi 0-7 | hi 8-15 | lo 0-7 | lo 8-15] (the swz layout of the 128-tile
// kernel) while the waves multiply the other image stage.  The MFMA sequence is that of the
// register-staged kernel (16-sample k-steps in sample order, lo*hi + hi*lo + hi*hi): identical slabs.  The
// bias gradient is the dY thread's own column sum over the split, in sample order.
// LDS: 3 x 32 KB ring + 2 x 32 KB images = 160 KB.
constexpr int WS_T = 16;                        // samples per step
constexpr int WS_RAW = 2 * WS_T * 1024;         // ring stage: dY rows then X rows, 1 KB each
constexpr int WS_IMG = 2 * 256 * 64;            // image stage: Y rows then X rows, 64 B each
template <int NRAW, int NIMG, bool X1>
__global__ __launch_bounds__(512, 1) __attribute__((amdgpu_waves_per_eu(2, 2))) void linear_wgrad_x3_stream_kernel(TNArgs a, int npad, int kpad) {
    static_assert(NRAW * WS_RAW + NIMG * WS_IMG <= 160 * 1024, "LDS");
    __shared__ __attribute__((aligned(16))) char smem[NRAW * WS_RAW + NIMG * WS_IMG];
    char* const ring = smem;
    char* const img = smem + NRAW * WS_RAW;

    const int split = blockIdx.x;
#ifndef NERF_WS_INTERLEAVE
    const int mbeg = split * a.m_per_split;
    int mend = mbeg + a.m_per_split;
    if (mend > a.M) mend = a.M;
    const int steps = mbeg < mend ? (mend - mbeg + WS_T - 1) / WS_T : 0;
    // first row of step i, rows of the split past mend read any valid row (zeroed)
#define WS_ROW0(i) (mbeg + (i) * WS_T)
#define WS_VALID(i) (mend - WS_ROW0(i))
#else
    // tuning: 16-row steps dealt round-robin over the splits (split s: steps s, s + splits, ...)
    const int mbeg = split * WS_T;
    const int nst = (a.M + WS_T - 1) / WS_T;
    const int steps = split < nst ? (nst - split + (int)gridDim.x - 1) / (int)gridDim.x : 0;
    const int mend = a.M;
#define WS_ROW0(i) ((split + (i) * (int)gridDim.x) * WS_T)
#define WS_VALID(i) (a.M - WS_ROW0(i))
#endif

    const int t = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6), lane = t & 63;
    const int wr = wave >> 2, wc = wave & 3;
    const int li = lane & 31, lh = lane >> 5;

    // X segment of packed column kx (segments span multiples of 32 columns)
    auto x_seg = [&](int kx, int& xs, int& xoff) __attribute__((always_inline)) {
        xs = -1;
        xoff = 0;
#pragma unroll
        for (int q = 0; q < MAX_SEGS; ++q)
            if (q < a.X.n && kx >= a.X.koff[q] && kx < a.X.koff[q] + a.X.kp[q]) { xs = q; xoff = kx - a.X.koff[q]; }
    };
    // ---- DMA sources of this lane: columns 4 lane .. 4 lane + 3 of dY and of X (invalid
    // columns read column 0: finite data, zeroed when converted)
    const int ycol = 4 * lane < a.N ? 4 * lane : 0;
    int dxs, dxoff;
    x_seg(4 * lane, dxs, dxoff);
    const bool dx_ok = dxs >= 0 && dxoff < pick4(a.X.k, dxs);
    const float* dxp = dx_ok ? pick4(a.X.ptr, dxs) + dxoff : a.X.ptr[0];
    const int64_t dxld = dx_ok ? pick4(a.X.ld, dxs) : a.X.ld[0];
    const unsigned dxrd = dx_ok ? (unsigned)pick4(a.X.row_div, dxs) : (unsigned)a.X.row_div[0];
    const float* dxp1 = dx_ok ? pick4(a.x1ptr, dxs) + dxoff : a.x1ptr[0];     // the second block's
    const int64_t dxld1 = dx_ok ? pick4(a.x1ld, dxs) : a.x1ld[0];
    const unsigned dxrd1 = dx_ok ? (unsigned)pick4(a.x1rd, dxs) : (unsigned)a.x1rd[0];
    // wave w brings rows 2w, 2w + 1 of both operands.  Lanes whose 4 columns lie past N / the
    // packed K fetch nothing (their LDS bytes keep stale values, zeroed by the conversion's column
    // mask): a 64-column X (the first layer) moves 256 B per row, not 1 KB.  Lane 0's columns are
    // always valid, so every DMA instruction issues (the counted waits count them).
    const bool y_fetch = 4 * lane < a.N;
    const bool x_fetch = dx_ok;
    auto issue = [&](int step) __attribute__((always_inline)) {
        char* st = ring + (step % NRAW) * WS_RAW;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int r = 2 * wave + q;
            int m = WS_ROW0(step) + r;
            m = m < mend && r < WS_VALID(step) ? m : mbeg;   // past the split: any valid row (zeroed)
            const bool b1 = m >= a.M0;                     // wave-uniform: the row's block
            const int mr = b1 ? m - a.M0 : m;
            const float* ys = (b1 ? a.dY1 : a.dY) + (int64_t)mr * (b1 ? a.lddy1 : a.lddy) + ycol;
            if (y_fetch) __builtin_amdgcn_global_load_lds((glb_void_t*)ys, (lds_void_t*)(st + r * 1024), 16, 0, 0);
            const unsigned rd = b1 ? dxrd1 : dxrd;
            const unsigned xr = rd == 1u ? (unsigned)mr : (unsigned)mr / rd;
            const float* xsrc = (b1 ? dxp1 : dxp) + (int64_t)xr * (b1 ? dxld1 : dxld);
            if (x_fetch)
                __builtin_amdgcn_global_load_lds((glb_void_t*)xsrc, (lds_void_t*)(st + (WS_T + r) * 1024), 16, 0, 0);
        }
    };

    // ---- conversion role: operand op (0 dY, 1 X), column c
    const int op = t >> 8, c = t & 255;
    bool c_ok;
    if (op == 0) {
        c_ok = c < a.N;
    } else {
        int xs, xoff;
        x_seg(c, xs, xoff);
        c_ok = xs >= 0 && xoff < pick4(a.X.k, xs);
    }
    float db = 0.f;
    float ray_acc = 0.f;      // raysum: this dY column's sum over the current ray's rows so far
    // N = 257 (NerfModel's density + feature layer): row 256 of dW / db on the X conversion threads,
    // dW[256][c] = sum over the split's samples (in order) of dY[m][256] * X[m][c] as fp32 FMAs; the
    // step's 16 dY[m][256] values by scalar loads (uniform addresses), issued with the ring reads
    const bool xrow = a.N > 256 && op == 1;
    float dacc = 0.f, dbx = 0.f;
    float yd[WS_T];
    auto yd_load = [&](int step) __attribute__((always_inline)) {
#pragma unroll
        for (int r = 0; r < WS_T; ++r) {
            int m = WS_ROW0(step) + r;
            m = m < mend && r < WS_VALID(step) ? m : mbeg;
#ifdef NERF_WS_DIAG_YD_FIXED      // diagnostic builds only: every row-256 load from one row (cache hits)
            m = mbeg;
#endif
            const bool b1 = m >= a.M0;
            yd[r] = *(const __attribute__((address_space(4))) float*)((b1 ? a.dY1 : a.dY) +
                                                                       (int64_t)(b1 ? m - a.M0 : m) * (b1 ? a.lddy1 : a.lddy) + 256);
        }
    };
    // the conversion in two halves, so that a step's ring reads can be issued ahead of the MFMAs
    // and its split / image writes scheduled between them (one basic block: no branch inside);
    // past the last step it converts stale ring rows into an image stage nobody reads again, all
    // masked to zero (no bias-gradient contribution).  db accumulates in every thread, only the
    // dY threads' sums are written.
    auto conv_load = [&](int step, float (&v)[WS_T]) __attribute__((always_inline)) {
        const float* src = reinterpret_cast<const float*>(ring + (step % NRAW) * WS_RAW + op * WS_T * 1024) + c;
#pragma unroll
        for (int r = 0; r < WS_T; ++r) v[r] = src[r * 256];
        if (xrow) yd_load(step);
    };
    auto conv_store = [&](int step, float (&v)[WS_T]) __attribute__((always_inline)) {
        __bf16* dst = reinterpret_cast<__bf16*>(img + (step % NIMG) * WS_IMG + op * 256 * 64);
        const int valid = WS_VALID(step);                   // rows of this step inside the split
        // masking only where a row or the column is invalid (the split's last step, padded
        // columns: a branch around it that full steps skip)
        if (!(c_ok && valid >= WS_T)) {
            const unsigned cm = c_ok ? ~0u : 0u;
#pragma unroll
            for (int r = 0; r < WS_T; ++r)
                v[r] = __builtin_bit_cast(float, __builtin_bit_cast(unsigned, v[r]) & (r < valid ? cm : 0u));
        }
        if (op == 0) {                                      // wave-uniform: the dY threads
#pragma unroll
            for (int r = 0; r < WS_T; ++r) db += v[r];
            if (a.raysum != nullptr && valid > 0) {
                // rays end at step ends (16 | S, ray starts and splits at multiples of 128 rows)
                float sv = 0.f;
#pragma unroll
                for (int r = 0; r < WS_T; ++r) sv += v[r];
                ray_acc += sv;
                const int last = WS_ROW0(step) + (valid < WS_T ? valid : WS_T) - 1;
                const bool b1 = last >= a.M0;
                const int rel = b1 ? last - a.M0 : last;
                const int S = b1 ? a.rs_S1 : a.rs_S0;
                if ((rel + 1) % S == 0) {
                    const int ray = (b1 ? a.rs_B0 : 0) + rel / S;
                    if (c < a.N) a.raysum[(size_t)ray * a.N + c] = ray_acc;
                    ray_acc = 0.f;
                }
            }
        }
        if (xrow) {                                         // wave-uniform: the X threads of N = 257
#pragma unroll
            for (int r = 0; r < WS_T; ++r) dacc = __builtin_fmaf(yd[r], v[r], dacc);   // v is 0 past the split
#pragma unroll
            for (int r = 0; r < WS_T; ++r) dbx += r < valid ? yd[r] : 0.f;
        }
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
            bf16x8 h, l;
            float x[8];
#pragma unroll
            for (int r = 0; r < 8; ++r) x[r] = v[8 * hh + r];
            split8_pairs(x, h, l);
            *reinterpret_cast<bf16x8*>(dst + swz(c, hh)) = h;
            *reinterpret_cast<bf16x8*>(dst + swz(c, 2 + hh)) = l;
        }
    };
    auto convert = [&](int step) __attribute__((always_inline)) {
#ifndef NERF_WS_DIAG_NOCONV       // diagnostic builds only: no conversion (the images keep stale bytes)
        float v[WS_T];
        conv_load(step, v);
        conv_store(step, v);
#endif
    };
    auto barrier = []() __attribute__((always_inline)) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };

    f32x16 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    // waves whose k columns lie wholly past the packed K skip the MFMAs (wave-uniform)
    const bool active = wc * 64 < a.X.ktot && wr * 128 < a.N;

    // wait until at most `ahead` steps' DMAs (4 per wave each) are outstanding
    auto wait_dma = [](int ahead) __attribute__((always_inline)) {
        if (ahead >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else if (ahead == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    };
    auto mfma_step = [&](int i) __attribute__((always_inline)) {
        const __bf16* Yb = reinterpret_cast<const __bf16*>(img + (i % NIMG) * WS_IMG);
        const __bf16* Xb = Yb + 256 * 32;
        bf16x8 xh[2], xl[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int row = wc * 64 + j * 32 + li;
            xh[j] = *reinterpret_cast<const bf16x8*>(Xb + swz(row, lh));
            xl[j] = *reinterpret_cast<const bf16x8*>(Xb + swz(row, 2 + lh));
        }
        // every fragment read issued before the first MFMA (one LDS latency per step, not one per
        // reuse of a fragment register)
        bf16x8 yh[4], yl[4];
#pragma unroll
        for (int ii = 0; ii < 4; ++ii) {
            const int row = wr * 128 + ii * 32 + li;
            yh[ii] = *reinterpret_cast<const bf16x8*>(Yb + swz(row, lh));
            yl[ii] = *reinterpret_cast<const bf16x8*>(Yb + swz(row, 2 + lh));
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int ii = 0; ii < 4; ++ii)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[ii][j] = mfma_w<X1>(yh[ii], yl[ii], xh[j], xl[j], acc[ii][j]);
    };
    if (steps > 0) {
        // prologue: steps 0 .. NRAW-1 issued, step 0 converted, step 1 landed
        for (int q = 0; q < NRAW - 1 && q < steps; ++q) issue(q);
        wait_dma(min(steps, NRAW - 1) - 1);
        barrier();
        convert(0);
        if (NRAW - 1 < steps) issue(NRAW - 1);
        wait_dma(min(steps, NRAW) - 2);
        barrier();
        for (int i = 0; i < steps; ++i) {
            // the stage step i held was converted before the previous barrier: refill it now, so
            // that two steps (i + 2, i + 3) stream in while step i multiplies and i + 1 converts
            if (i + NRAW < steps) issue(i + NRAW);
            // NIMG = 2: step i + 1's conversion overlaps step i's MFMAs (other image stage)
            if (NIMG == 2) {
                if (active) {
#ifndef NERF_WS_DIAG_NOCONV
                    float v[WS_T];
                    conv_load(i + 1, v);
#endif
                    __builtin_amdgcn_sched_barrier(0);      // the ring reads fly while the MFMAs run
#ifndef NERF_WS_DIAG_NOMFMA       // diagnostic builds only: no MFMA step
                    mfma_step(i);
#endif
                    __builtin_amdgcn_sched_barrier(0);
#ifndef NERF_WS_DIAG_NOCONV
                    conv_store(i + 1, v);
#endif
                } else {
                    convert(i + 1);
                }
            } else {
                if (active) mfma_step(i);
                barrier();                                  // the single image stage is free
                convert(i + 1);
            }
            // step i + 2 landed (it is converted in the next iteration)
            wait_dma(min(steps - 1, i + NRAW) - (i + 2));
            barrier();
        }
    }

#undef WS_ROW0
#undef WS_VALID
    float* slab = a.slab + (size_t)split * npad * kpad;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int k = wc * 64 + j * 32 + li;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int n = wr * 128 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                if (n < npad && k < kpad) slab[(size_t)n * kpad + k] = acc[i][j][r];
            }
        }
    if (op == 0 && c < npad) a.db_slab[(size_t)split * npad + c] = db;
    if (xrow) {
        slab[(size_t)256 * kpad + c] = dacc;
        if (c == 0) a.db_slab[(size_t)split * npad + 256] = dbx;
    }
}

// ------------------------------------------------------------------- TN register-staged, transposed reads
// The same 256 x 256 weight-gradient tile as linear_wgrad_x3_stream_kernel (one workgroup per M
// split, dY and X read from HBM once, 16-sample MFMA steps in sample order, lo*hi + hi*lo + hi*hi on
// v_mfma_f32_32x32x16_bf16: slabs bitwise equal), with the operand stream rebuilt around what the
// hardware does fastest (tools/stream_bench.hip, profiles/r04b): plain nontemporal
// global_load_dwordx4 rows into VGPRs stream 1 GB at 6.45-6.6 TB/s after the forward's writes,
// where the LDS-DMA ring of the stream kernel reads the same rows at 4.2-4.4 TB/s.
//
// Waves 0-3 load dY rows 4w .. 4w + 3 of a step, waves 4-7 the X rows; lane l holds columns
// 4l .. 4l + 3 of each (one coalesced 1 KB row per wave-instruction), two steps ahead of the step
// being converted.  Each lane splits its own 16 values into bf16 hi / lo and writes them ROW-major
// ([op][hi|lo][16 samples][256 columns], 64-byte blocks XOR-permuted by row & 3) with ds_write_b64;
// the MFMA operands, which need 8 consecutive SAMPLES per lane, come back through
// ds_read_b64_tr_b16 (the gfx950 transposed read; MI355X guide T10) — no raw ring, no column reads,
// no DMA.  Per step: 32 KB of image, two stages (64 KB of LDS); both conflict-free.
// Bias gradients, the 257th row (NerfModel's density + feature layer) and the per-ray dY sums of the
// colour layer come from per-wave partials over the wave's rows, added in a fixed order (same values
// as the stream kernel up to fp32 summation order).
constexpr int WT_T = 16;                          // samples per step
constexpr int WT_IMG = 4 * WT_T * 512;            // image stage: [op][hi | lo][16 rows][256 cols] bf16
constexpr int WT_RS = 4 * 256 * 4;                // per-ray partials of the 4 dY waves
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4_t;

// byte offset of columns col .. col + 3 (8-byte aligned) of image row `row` of plane (op, pl)
__device__ __forceinline__ unsigned wt_off(int op, int pl, int row, int col) {
    return (unsigned)(((op * 2 + pl) * WT_T + row) * 512 + ((2 * col) ^ ((row & 3) << 6)));
}

typedef const __attribute__((address_space(1))) float* wt_gfp;
// source of relative row `rel` of the split (rows past its end read its first row): block 1 (rows
// >= M0) from s1 / ld1 / rd1, block 0 from s0 / ld0 / rd0
__device__ __forceinline__ wt_gfp wt_src_row(wt_gfp s0, wt_gfp s1, int64_t ld0, int64_t ld1, unsigned rd0,
                                             unsigned rd1, bool rd_one, int M0, int mbeg, int mend, int rel) {
    int m = mbeg + rel;
    m = m < mend ? m : mbeg;
    const bool b1 = m >= M0;                                // wave-uniform
    const unsigned r = (unsigned)(b1 ? m - M0 : m);
    const unsigned rr = rd_one ? r : r / (b1 ? rd1 : rd0);
    return (b1 ? s1 : s0) + (int64_t)rr * (b1 ? ld1 : ld0);
}

template <bool ROW257, bool RAYS, bool X1, int JN>
__global__ __launch_bounds__(512, 1) __attribute__((amdgpu_waves_per_eu(2, 2))) void linear_wgrad_x3_tr_kernel(
    TNArgs a, int npad, int kpad) {
    __shared__ __attribute__((aligned(16))) char smem[2 * WT_IMG + (RAYS ? 2 * WT_RS : 0)];
    // every argument the loop uses in registers (a lambda reading the by-value argument through a
    // reference puts it in scratch), global pointers in the global address space (flat loads would
    // share lgkmcnt with the LDS traffic)
    typedef wt_gfp gfp;
    typedef const __attribute__((address_space(1))) f4* gf4p;
    const int split = blockIdx.x;
    const int mbeg = split * a.m_per_split;
    const int mend = min(mbeg + a.m_per_split, a.M);
    const int M0 = a.M0, N = a.N;
    const gfp dY0 = (gfp)a.dY, dY1 = (gfp)a.dY1;
    const int64_t lddy0 = a.lddy, lddy1 = a.lddy1;
    const int rs_S0 = a.rs_S0, rs_S1 = a.rs_S1, rs_B0 = a.rs_B0;
    float* const raysum = a.raysum;
    const int steps = mbeg < mend ? (mend - mbeg + WT_T - 1) / WT_T : 0;
    const int t = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6), lane = t & 63;
    const int op = wave >> 2;                 // this wave loads and converts 0: dY rows, 1: X rows
    const int lr = 4 * (wave & 3);            // its first row of each step

    // ---- this lane's source columns 4 lane .. 4 lane + 3 (segments span multiples of 32 columns);
    // invalid columns read column 0 of the operand (finite data) and are zeroed when converted
    gfp s0, s1;
    int64_t ld0, ld1;
    unsigned rd0 = 1, rd1 = 1, cmask = 0;
    if (op == 0) {
        const int nval = N < 256 ? N : 256;
#pragma unroll
        for (int e = 0; e < 4; ++e) cmask |= (4 * lane + e < nval ? 1u : 0u) << e;
        const int col = 4 * lane < nval ? 4 * lane : 0;
        s0 = dY0 + col;
        s1 = dY1 + col;
        ld0 = lddy0;
        ld1 = lddy1;
    } else {
        int xs = -1, xoff = 0;
#pragma unroll
        for (int q = 0; q < MAX_SEGS; ++q)
            if (q < a.X.n && 4 * lane >= a.X.koff[q] && 4 * lane < a.X.koff[q] + a.X.kp[q]) {
                xs = q;
                xoff = 4 * lane - a.X.koff[q];
            }
        const int kk = xs >= 0 ? pick4(a.X.k, xs) : 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) cmask |= (xoff + e < kk ? 1u : 0u) << e;
        const bool ok = cmask != 0;
        s0 = (gfp)(ok ? pick4(a.X.ptr, xs) + xoff : a.X.ptr[0]);
        ld0 = ok ? pick4(a.X.ld, xs) : a.X.ld[0];
        rd0 = ok ? (unsigned)pick4(a.X.row_div, xs) : (unsigned)a.X.row_div[0];
        s1 = (gfp)(ok ? pick4(a.x1ptr, xs) + xoff : a.x1ptr[0]);
        ld1 = ok ? pick4(a.x1ld, xs) : a.x1ld[0];
        rd1 = ok ? (unsigned)pick4(a.x1rd, xs) : (unsigned)a.x1rd[0];
    }
    // one source row per sample in every lane of the wave (the row divisor is the per-ray input's,
    // absent from this kernel's layers in practice): no per-lane division
    const bool rd_one = __ballot(rd0 != 1u || rd1 != 1u) == 0;
    // (rows are computed by free functions of values: through a lambda's captures `b1 ? x : y`
    // becomes a select of the captured variables' addresses, which keeps them in scratch)
#define WT_SRC_ROW(i, q) wt_src_row(s0, s1, ld0, ld1, rd0, rd1, rd_one, M0, mbeg, mend, (i) * WT_T + lr + (q))
#define WT_YD_ROW(i, q) wt_src_row(dY0 + 256, dY1 + 256, lddy0, lddy1, 1u, 1u, true, M0, mbeg, mend, (i) * WT_T + lr + (q))
    f4 ra[4], rb[4];                          // the two register stages: steps in flight
    float ya[4], yb[4];
    auto issue = [&](int i, f4 (&r)[4], float (&y)[4]) __attribute__((always_inline)) {
#ifdef NERF_WT_DIAG_NOLOAD     // diagnostic builds only: no row loads (converts the registers' stale values)
        if (i < 2)
#endif
#pragma unroll
        for (int q = 0; q < 4; ++q) r[q] = __builtin_nontemporal_load((gf4p)WT_SRC_ROW(i, q));
        if constexpr (ROW257) {
#pragma unroll
            for (int q = 0; q < 4; ++q) y[q] = *WT_YD_ROW(i, q);
        }
    };

    // ---- per-wave partial sums (fixed order: rows of the wave in sample order)
    f4 dbp = {0.f, 0.f, 0.f, 0.f};            // dY waves: bias gradient of columns 4 lane ..
    f4 rp = {0.f, 0.f, 0.f, 0.f};             // dY waves: the current ray's dY sums
    f4 dacc = {0.f, 0.f, 0.f, 0.f};           // X waves (ROW257): dW[256][4 lane ..]
    float dbx = 0.f;                          // X waves (ROW257): db[256]
    int pend_ray = -1;                        // a ray whose partials wait in rs[pend_ray & 1]
    char* const rs = smem + 2 * WT_IMG;

    // image offsets of this lane's row writes
    unsigned woff[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) woff[q] = wt_off(op, 0, lr + q, 4 * lane);

    const bool cols_full = __ballot(cmask != 0xfu) == 0;   // wave-uniform: no padded column in the wave
    auto convert = [&](int i, const f4 (&r)[4], const float (&y)[4]) __attribute__((always_inline)) {
        const int valid = mend - (mbeg + i * WT_T);          // rows of step i inside the split
        char* const img = smem + (i & 1) * WT_IMG;
        f4 rv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) rv[q] = r[q];
        if (!(cols_full && valid >= WT_T)) {                 // padded columns or the split's last rows
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const unsigned rm = lr + q < valid ? cmask : 0u;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    // through a scalar: __builtin_bit_cast of the vector element lvalue rv[q][e] reads
                    // element 0 (hipcc), which filled the masked rows' columns 1-3 with column 0
                    const float xe = rv[q][e];
                    rv[q][e] = __builtin_bit_cast(float, __builtin_bit_cast(int, xe) &
                                                             __builtin_amdgcn_sbfe((int)rm, (unsigned)e, 1u));
                }
            }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const f4 v = rv[q];
            if (op == 0) {
                dbp += v;
                if constexpr (RAYS) rp += v;
            } else if constexpr (ROW257) {
                const float yq = lr + q < valid ? y[q] : 0.f;
#pragma unroll
                for (int e = 0; e < 4; ++e) dacc[e] = __builtin_fmaf(yq, v[e], dacc[e]);
                dbx += yq;
            }
            typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
            typedef float f2 __attribute__((ext_vector_type(2)));
            typedef unsigned u2 __attribute__((ext_vector_type(2)));
            u2 h, l;
#pragma unroll
            for (int pp = 0; pp < 2; ++pp) {
                const f2 x2 = {v[2 * pp], v[2 * pp + 1]};
                const unsigned hp = __builtin_bit_cast(unsigned, __builtin_convertvector(x2, bf16x2));
                const f2 hv = {__builtin_bit_cast(float, hp << 16), __builtin_bit_cast(float, hp & 0xffff0000u)};
                h[pp] = hp;
                l[pp] = __builtin_bit_cast(unsigned, __builtin_convertvector(x2 - hv, bf16x2));
            }
            *reinterpret_cast<u2*>(img + woff[q]) = h;
            *reinterpret_cast<u2*>(img + woff[q] + WT_T * 512) = l;
        }
        if constexpr (RAYS) {
            if (op == 0 && valid > 0) {
                // rays end at step ends (16 | S; ray starts and splits at multiples of 128 rows)
                const int last = mbeg + i * WT_T + (valid < WT_T ? valid : WT_T) - 1;
                const bool b1 = last >= M0;
                const int rel = b1 ? last - M0 : last;
                const int S = b1 ? rs_S1 : rs_S0;
                if ((rel + 1) % S == 0) {
                    const int ray = (b1 ? rs_B0 : 0) + rel / S;
                    *reinterpret_cast<f4*>(rs + (ray & 1) * WT_RS + ((wave & 3) * 256 + 4 * lane) * 4) = rp;
                    rp = f4{0.f, 0.f, 0.f, 0.f};
                }
            }
        }
    };
    // the ray completed in the previous step: its 4 wave partials, added in wave order, to raysum
    auto flush_ray = [&]() __attribute__((always_inline)) {
        if constexpr (RAYS) {
            if (pend_ray >= 0 && op == 0) {
                const int c = 64 * (wave & 3) + lane;
                const float* p = reinterpret_cast<const float*>(rs + (pend_ray & 1) * WT_RS);
                const float s = ((p[c] + p[256 + c]) + p[512 + c]) + p[768 + c];
                if (c < N) raysum[(size_t)pend_ray * N + c] = s;
            }
        }
    };
    // the ray (if any) whose last rows are in step i
    auto ray_of_step = [=](int i) __attribute__((always_inline)) {
        const int valid = mend - (mbeg + i * WT_T);
        if (valid <= 0) return -1;
        const int last = mbeg + i * WT_T + (valid < WT_T ? valid : WT_T) - 1;
        const bool b1 = last >= M0;
        const int rel = b1 ? last - M0 : last;
        const int S = b1 ? rs_S1 : rs_S0;
        return (rel + 1) % S == 0 ? (b1 ? rs_B0 : 0) + rel / S : -1;
    };

    // ---- MFMA role: wave (wr, wc) owns dW rows wr*128 .. +127 (4 x 32) and columns wc*32JN ..
    // +32JN-1 (JN x 32; JN = 1 for inputs of <= 128 columns, so that all four SIMDs multiply)
    const int wr = wave >> 2, wc = wave & 3;
#ifndef NERF_WT_DIAG_NOMFMA     // diagnostic builds only: no MFMA step (loads, conversion, barriers)
    const bool active = wc * 32 * JN < a.X.ktot && wr * 128 < N;
#else
    const bool active = false;
#endif
    // transposed-read addresses: lane 4q + p of 16-lane group G supplies row 8 (G >> 1) + q (+ 4 for
    // the fragment's second half), columns c0 + 16 (G & 1) + 4 p of the 32-column block c0
    const int G = lane >> 4, qq = (lane & 15) >> 2, pq = lane & 3;
    unsigned ya_off[4], xa_off[JN];
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) ya_off[ii] = wt_off(0, 0, 8 * (G >> 1) + qq, wr * 128 + 32 * ii + 16 * (G & 1) + 4 * pq);
#pragma unroll
    for (int j = 0; j < JN; ++j) xa_off[j] = wt_off(1, 0, 8 * (G >> 1) + qq, wc * 32 * JN + 32 * j + 16 * (G & 1) + 4 * pq);
    auto frag = [&](const char* img, unsigned off) __attribute__((always_inline)) {
        const s16x4 lo4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(img + off));
        const s16x4 hi4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(img + off + 4 * 512));
        return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo4, hi4, 0, 1, 2, 3, 4, 5, 6, 7));
    };
    f32x16 acc[4][JN];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    // the MFMAs of step i over row blocks ii0 .. ii1 - 1
    auto mfma_step = [&](int i, int ii0 = 0, int ii1 = 4) __attribute__((always_inline)) {
        const char* img = smem + (i & 1) * WT_IMG;
        bf16x8 xh[JN], xl[JN], yh[4], yl[4];
#pragma unroll
        for (int j = 0; j < JN; ++j) {
            xh[j] = frag(img, xa_off[j]);
            xl[j] = frag(img, xa_off[j] + WT_T * 512);
        }
#pragma unroll
        for (int ii = ii0; ii < ii1; ++ii) {
            yh[ii] = frag(img, ya_off[ii]);
            yl[ii] = frag(img, ya_off[ii] + WT_T * 512);
        }
#pragma unroll
        for (int ii = ii0; ii < ii1; ++ii)
#pragma unroll
            for (int j = 0; j < JN; ++j) acc[ii][j] = mfma_w<X1>(yh[ii], yl[ii], xh[j], xl[j], acc[ii][j]);
    };
    // The two waves of a SIMD (wave w loads dY rows, wave w + 4 X rows) multiply at different times:
    // the X-loading wave runs step i's MFMAs before converting step i + 1, its partner after, so one
    // wave's conversion (VALU) runs under the other's MFMAs (profiles/r06k: the kernel 1.5-2 % faster
    // in the mip step than both converting first; the roles swapped, or half of every wave's MFMAs
    // before the conversion, no better).  Same products in the same order per accumulator.
    auto mfma_pre = [&](int i) __attribute__((always_inline)) {
        if (op == 1 && active) mfma_step(i);
    };
    auto mfma_post = [&](int i) __attribute__((always_inline)) {
        if (op == 0 && active) mfma_step(i);
    };
    auto barrier = []() __attribute__((always_inline)) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's LDS writes / reads done
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };

    if (steps > 0) {
        // prologue: steps 0 and 1 in flight, step 0 converted, step 2 issued
        issue(0, ra, ya);
        issue(1, rb, yb);
        convert(0, ra, ya);
        issue(2, ra, ya);
        if constexpr (RAYS) pend_ray = op == 0 ? ray_of_step(0) : -1;
        barrier();
        // iteration i: convert step i + 1 (landed: issued two iterations ago), refill its registers
        // with step i + 3, multiply step i; unrolled by two so the register stages are compile-time
        // (loads past the last step re-read the split's first rows and conversions past it fill a
        // stage nobody reads, masked to zero: no branch around them, so the counted waits are exact)
        int i = 0;
        for (; i + 1 < steps; i += 2) {
            mfma_pre(i);
            convert(i + 1, rb, yb);
            issue(i + 3, rb, yb);
            flush_ray();
            if constexpr (RAYS) pend_ray = op == 0 ? ray_of_step(i + 1) : -1;
            mfma_post(i);
            barrier();
            mfma_pre(i + 1);
            convert(i + 2, ra, ya);
            issue(i + 4, ra, ya);
            flush_ray();
            if constexpr (RAYS) pend_ray = i + 2 < steps && op == 0 ? ray_of_step(i + 2) : -1;
            mfma_post(i + 1);
            barrier();
        }
        if (i < steps) {                       // odd step count: the last step, converted already
            flush_ray();
            if constexpr (RAYS) pend_ray = -1;
            if (active) mfma_step(i);
            barrier();
        }
        flush_ray();
    }

    float* slab = a.slab + (size_t)split * npad * kpad;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j) {
            const int k = wc * 32 * JN + j * 32 + (lane & 31);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int n = wr * 128 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                if (n < npad && k < kpad) slab[(size_t)n * kpad + k] = acc[i][j][r];
            }
        }
    // per-wave partials through LDS (the image stages are free: the loop ended on a barrier), added
    // in wave order
    float* red = reinterpret_cast<float*>(smem);          // [4 dY waves][256] | [4 X waves][256]
    *reinterpret_cast<f4*>(red + (op * 4 + (wave & 3)) * 256 + 4 * lane) = op == 0 ? dbp : dacc;
    if (ROW257 && op == 1 && lane == 0) red[2048 + (wave & 3)] = dbx;
    __syncthreads();
    if (t < 256) {
        const float s = ((red[t] + red[256 + t]) + red[512 + t]) + red[768 + t];
        if (t < npad) a.db_slab[(size_t)split * npad + t] = s;
    } else if (ROW257) {
        const int c = t - 256;
        const float* x = red + 1024;
        slab[(size_t)256 * kpad + c] = ((x[c] + x[256 + c]) + x[512 + c]) + x[768 + c];
        if (c == 0)
            a.db_slab[(size_t)split * npad + 256] = ((red[2048] + red[2049]) + red[2050]) + red[2051];
    }
#undef WT_SRC_ROW
#undef WT_YD_ROW
}

// ------------------------------------------------------------------- TN small N
// Weight gradient of a layer with few outputs (N <= 16: the colour head's last Linear(128, 3 or 4),
// barf/model_interpolation_architecture.py:88-92), where the tile kernels would run a 128-row MFMA
// tile for 4 rows.  One workgroup per M split streams the split's rows once (dY: 4 N4 bytes, X:
// 4 ktot bytes per row); thread (row group g, column quad q) accumulates exact fp32 products of the
// rows m = mbeg + g, g + RG, ... in sample order (SN_U rows' loads in flight per thread), and the RG
// row groups' partial sums are added in a fixed order through LDS: deterministic, and finer than the
// 3 x bf16 products of the tile kernels.  Same slab / bias-slab layout and reduce.
constexpr int SN_T = 512;
constexpr int SN_U = 8;
template <int N4>
__global__ __launch_bounds__(SN_T) void linear_wgrad_smalln_kernel(TNArgs a, int kpad) {
    extern __shared__ __attribute__((aligned(16))) float sn_part[];     // [RG][N4][ktot] + [RG][N4]
    const int split = blockIdx.x;
    const int mbeg = split * a.m_per_split;
    const int mend = min(mbeg + a.m_per_split, a.M);
    const int ktot = a.X.ktot;
    const int qw = ktot >> 2;                       // column quads per row
    const int rg = SN_T / qw;                       // row groups
    const int t = threadIdx.x;
    const int g = t / qw, q = t - g * qw;
    const bool live = g < rg;
    // this thread's four packed columns 4 q .. 4 q + 3: one segment (segments span multiples of 32)
    int xs = 0, xoff = 0;
#pragma unroll
    for (int i = 0; i < MAX_SEGS; ++i)
        if (i < a.X.n && 4 * q >= a.X.koff[i] && 4 * q < a.X.koff[i] + a.X.kp[i]) { xs = i; xoff = 4 * q - a.X.koff[i]; }
    const bool col_ok = live && xoff < pick4(a.X.k, xs);
    const float* xp0 = pick4(a.X.ptr, xs) + xoff;
    const int64_t xld0 = pick4(a.X.ld, xs);
    const unsigned xrd0 = (unsigned)pick4(a.X.row_div, xs);
    const float* xp1 = pick4(a.x1ptr, xs) + xoff;
    const int64_t xld1 = pick4(a.x1ld, xs);
    const unsigned xrd1 = (unsigned)pick4(a.x1rd, xs);
    f4 acc[N4];
    f4 dbs[N4 / 4];
#pragma unroll
    for (int n = 0; n < N4; ++n) acc[n] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < N4 / 4; ++j) dbs[j] = f4{0.f, 0.f, 0.f, 0.f};
    if (live) {
        for (int m0 = mbeg + g; m0 < mend; m0 += SN_U * rg) {
            f4 y[SN_U][N4 / 4], x[SN_U];
#pragma unroll
            for (int u = 0; u < SN_U; ++u) {
                const int m = m0 + u * rg;
                const bool ok = m < mend;
                const bool b1 = m >= a.M0;
                const int mr = ok ? (b1 ? m - a.M0 : m) : 0;
                const float* yr = (b1 ? a.dY1 : a.dY) + (int64_t)mr * (b1 ? a.lddy1 : a.lddy);
#pragma unroll
                for (int j = 0; j < N4 / 4; ++j)
                    y[u][j] = ok ? *reinterpret_cast<const f4*>(yr + 4 * j) : f4{0.f, 0.f, 0.f, 0.f};
                const unsigned rd = b1 ? xrd1 : xrd0;
                const unsigned xr = rd == 1u ? (unsigned)mr : (unsigned)mr / rd;
                const float* xr_p = (b1 ? xp1 : xp0) + (int64_t)xr * (b1 ? xld1 : xld0);
                x[u] = ok && col_ok ? *reinterpret_cast<const f4*>(xr_p) : f4{0.f, 0.f, 0.f, 0.f};
            }
#pragma unroll
            for (int u = 0; u < SN_U; ++u) {
#pragma unroll
                for (int n = 0; n < N4; ++n) {
                    const float yn = y[u][n >> 2][n & 3];
#pragma unroll
                    for (int c = 0; c < 4; ++c) acc[n][c] = __builtin_fmaf(yn, x[u][c], acc[n][c]);
                }
#pragma unroll
                for (int j = 0; j < N4 / 4; ++j) dbs[j] += y[u][j];
            }
        }
        float* p = sn_part + (size_t)g * N4 * ktot;
#pragma unroll
        for (int n = 0; n < N4; ++n) *reinterpret_cast<f4*>(p + (size_t)n * ktot + 4 * q) = acc[n];
        if (q == 0) {
            float* d = sn_part + (size_t)rg * N4 * ktot + g * N4;
#pragma unroll
            for (int j = 0; j < N4 / 4; ++j) *reinterpret_cast<f4*>(d + 4 * j) = dbs[j];
        }
    }
    __syncthreads();
    float* slab = a.slab + (size_t)split * (size_t)((a.N + TB - 1) / TB * TB) * kpad;
    for (int o = t; o < N4 * ktot; o += SN_T) {
        float v = 0.f;
        for (int gg = 0; gg < rg; ++gg) v += sn_part[(size_t)gg * N4 * ktot + o];
        const int n = o / ktot, k = o - n * ktot;
        slab[(size_t)n * kpad + k] = v;
    }
    if (t < N4) {
        float v = 0.f;
        for (int gg = 0; gg < rg; ++gg) v += sn_part[(size_t)rg * N4 * ktot + gg * N4 + t];
        a.db_slab[(size_t)split * ((a.N + TB - 1) / TB * TB) + t] = v;
    }
}

// Interleaved split weights: element (r, c) of a [rows][ld] matrix goes to
// Wx[r][c / 32][c % 32] (hi) and Wx[r][c / 32][32 + c % 32] (lo), i.e. each 32-column
// chunk of a row is 128 contiguous bytes: 32 hi then 32 lo.
__device__ __forceinline__ int64_t xoff(int64_t r, int c, int ld) { return r * ld * 2 + (c >> 5) * 64 + (c & 31); }

__global__ void pack_weight_x3_kernel(const float* __restrict__ W, int N, int K_orig, const int32_t* __restrict__ col_map,
                                      int Kp, int npad, __bf16* __restrict__ Wpx, __bf16* __restrict__ Wtx, int ldwt,
                                      int kpad_rows) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)npad * Kp;
    if (idx < total) {
        const int n = (int)(idx / Kp), k = (int)(idx - (idx / Kp) * Kp);
        const int src = col_map[k];
        const float v = (n < N && src >= 0 && src < K_orig) ? W[(int64_t)n * K_orig + src] : 0.f;
        const __bf16 h = (__bf16)v;
        const __bf16 l = (__bf16)(v - (float)h);
        if (Wpx) { const int64_t o = xoff(n, k, Kp); Wpx[o] = h; Wpx[o + 32] = l; }
        if (Wtx && n < ldwt) { const int64_t o = xoff(k, n, ldwt); Wtx[o] = h; Wtx[o + 32] = l; }
    }
    if (Wtx) {
        // rows Kp .. kpad_rows of the transposed matrix are zero (columns N .. ldwt: n >= N above)
        const int64_t pad_total = (int64_t)(kpad_rows - Kp) * ldwt;
        if (idx < pad_total) {
            const int64_t o = xoff(Kp + idx / ldwt, (int)(idx % ldwt), ldwt);
            Wtx[o] = (__bf16)0.f;
            Wtx[o + 32] = (__bf16)0.f;
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
int nerf_wgrad_split_tiles(int N, int K);

// Layers wider than 256 outputs (GARF's Linear(3, 1024), Linear(131, 512) and the input gradients
// into them) as column blocks of <= 256 on the 256-row tile kernel, A re-read per block, instead of
// the 128 x 128-tile kernel.  NERF_NT_NBLOCK=0: the 128-tile kernel (A/B switch, read once).
static const bool NT_NBLOCK = [] {
    const char* e = getenv("NERF_NT_NBLOCK");
    return !(e && e[0] == '0');
}();

extern "C" int nerf_linear_fwd_x3(const nerf_seg* segs, int32_t n_segs, int64_t M, const void* W_x, int32_t ldw,
                                  int32_t N, const float* bias, float* out, int64_t ldo, int32_t epilogue,
                                  const float* aux, int64_t ld_aux, void* stream) {
    NERF_REQUIRE(M >= 0 && M < (1ll << 31) && N >= 1);
    if (M == 0) return NERF_OK;
    SegList L;
    NERF_REQUIRE(build_segs(segs, n_segs, L));
    NERF_REQUIRE(W_x && out && aligned16(W_x) && ldw == L.ktot && (ldw % BK) == 0 && ldo >= N);
    if (epilogue & NERF_EPI_BIAS) NERF_REQUIRE(bias != nullptr);
    const bool mbits = (epilogue & (NERF_EPI_MASKBITS | NERF_EPI_MASKOUT)) != 0;
    if (mbits) NERF_REQUIRE(aux != nullptr && N <= 256 && ld_aux >= 32 && (ld_aux % 16) == 0 && aligned16(aux));
    if (epilogue & NERF_EPI_MASK) NERF_REQUIRE(aux != nullptr && (mbits || ld_aux >= N));
    if (epilogue & NERF_EPI_MASKOUT) NERF_REQUIRE(!(epilogue & NERF_EPI_MASK));
    if (epilogue & NERF_EPI_TANH_BWD) NERF_REQUIRE(aux != nullptr && ld_aux >= N && !(epilogue & (NERF_EPI_MASK | NERF_EPI_MASKBITS | NERF_EPI_MASKOUT)));
    NERF_REQUIRE(!(epilogue & (NERF_EPI_GAUSS | NERF_EPI_GAUSS_BWD)));     // nerf_linear_gauss_x3 only
    const int vec_ok = aligned16(out) && (ldo % 4) == 0 && (!(epilogue & NERF_EPI_BIAS) || aligned16(bias)) &&
                       (!(epilogue & NERF_EPI_MASK) || mbits || (aligned16(aux) && (ld_aux % 4) == 0)) &&
                       (!(epilogue & NERF_EPI_TANH_BWD) || (aligned16(aux) && (ld_aux % 4) == 0));
    NTArgs a{L, (int)M, reinterpret_cast<const __bf16*>(W_x), ldw, N, bias, out, ldo, epilogue, aux, ld_aux, vec_ok};
    hipStream_t st = as_stream(stream);
    // tanh epilogues run on the 128 x 128 tile kernel (runtime epilogue flags); mask bits need N <= 256
    if ((N <= 256 || (NT_NBLOCK && !mbits)) && !(epilogue & (NERF_EPI_NARROW_TILE | NERF_EPI_TANH | NERF_EPI_TANH_BWD))) {
        const int ntiles = (int)((M + 255) / 256);
        int grid = cu_count_x3();
        if (grid > ntiles) grid = ntiles;
        const dim3 g3((unsigned)grid), b3(512);
        for (int n0 = 0; n0 < N; n0 += 256) {          // column blocks of <= 256 (one when N <= 256)
            NTArgs b = a;
            b.N = N - n0 < 256 ? N - n0 : 256;
            b.Wx = a.Wx + (size_t)n0 * 2 * ldw;
            b.bias = bias ? bias + n0 : nullptr;
            b.out = out + n0;
            b.aux = aux && !mbits ? aux + n0 : aux;
#define NERF_GLDS_LAUNCH(E)                                                                            \
    do {                                                                                              \
        if (b.N > 128) hipLaunchKernelGGL((linear_nt_x3_glds_kernel<E, 2>), g3, b3, 0, st, b, ntiles); \
        else hipLaunchKernelGGL((linear_nt_x3_glds_kernel<E, 1>), g3, b3, 0, st, b, ntiles);         \
    } while (0)
            switch (epilogue & 15) {
                case NERF_EPI_BIAS | NERF_EPI_RELU: NERF_GLDS_LAUNCH(NERF_EPI_BIAS | NERF_EPI_RELU); break;
                case NERF_EPI_BIAS: NERF_GLDS_LAUNCH(NERF_EPI_BIAS); break;
                case NERF_EPI_BIAS | NERF_EPI_ACCUM: NERF_GLDS_LAUNCH(NERF_EPI_BIAS | NERF_EPI_ACCUM); break;
                case 0: NERF_GLDS_LAUNCH(0); break;
                case NERF_EPI_MASK: NERF_GLDS_LAUNCH(NERF_EPI_MASK); break;
                case NERF_EPI_MASK | NERF_EPI_ACCUM: NERF_GLDS_LAUNCH(NERF_EPI_MASK | NERF_EPI_ACCUM); break;
                case NERF_EPI_ACCUM: NERF_GLDS_LAUNCH(NERF_EPI_ACCUM); break;
                default: return NERF_ERR_UNSUPPORTED;
            }
#undef NERF_GLDS_LAUNCH
            NERF_CHECK_LAUNCH();
        }
        return NERF_OK;
    }
    const int ntm = (int)((M + 127) / 128);
    const int ntn = (N + 127) / 128;
    const int ntiles = (ntm + 7) / 8 * 8 * ntn;
    int grid = ntiles;
    if (!(epilogue & NERF_EPI_NO_PERSIST)) {
        const int cap = 2 * cu_count_x3();
        if (grid > cap) grid = cap;
    }
    hipLaunchKernelGGL(linear_nt_x3_kernel, dim3((unsigned)grid), dim3(256), 0, st, a, ntm, ntiles);
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}

extern "C" size_t nerf_linear_gauss_workspace(int64_t M, int32_t N) {
    if (M <= 0 || N <= 0) return 0;
    // one fp64 row per 128-row tile (the 256-row tile kernel uses half) + the reduction's chunk sums
    return (size_t)((M + 127) / 128) * (size_t)N * sizeof(double) + nerf::gauss_reduce_scratch(N);
}

extern "C" int nerf_linear_gauss_x3(const nerf_seg* segs, int32_t n_segs, int64_t M, const void* W_x, int32_t ldw,
                                    int32_t N, const float* bias, float* out, int64_t ldo, int32_t mode,
                                    const float* inv_std, float* y, int64_t ld_y, const float* z, int64_t ld_z,
                                    float* grad_inv_std, int32_t accumulate, void* workspace, size_t workspace_bytes,
                                    void* stream) {
    NERF_REQUIRE(M >= 0 && M < (1ll << 31) && N >= 1 && (mode == NERF_GAUSS_FWD || mode == NERF_GAUSS_BWD));
    NERF_REQUIRE(inv_std != nullptr && out != nullptr);
    const bool fwd = mode == NERF_GAUSS_FWD;
    if (fwd) NERF_REQUIRE(y != nullptr && ld_y >= N);
    else NERF_REQUIRE(bias == nullptr && z != nullptr && ld_z >= N && grad_inv_std != nullptr);
    hipStream_t st = as_stream(stream);
    if (M == 0) {
        if (!fwd && !accumulate && hipMemsetAsync(grad_inv_std, 0, (size_t)N * sizeof(float), st) != hipSuccess)
            return NERF_ERR_LAUNCH;
        return NERF_OK;
    }
    // whole 16-byte quads everywhere, or the caller takes the unfused path
    if ((N % 4) != 0 || !aligned16(out) || (ldo % 4) != 0 || ldo < N || !aligned16(inv_std) ||
        (bias && !aligned16(bias)) || (fwd && (!aligned16(y) || (ld_y % 4) != 0)) ||
        (!fwd && (!aligned16(z) || (ld_z % 4) != 0)))
        return NERF_ERR_UNSUPPORTED;
    if (!fwd && (workspace == nullptr || workspace_bytes < nerf_linear_gauss_workspace(M, N) ||
                 (reinterpret_cast<uintptr_t>(workspace) & 7) != 0))
        return NERF_ERR_WORKSPACE;
    SegList L;
    NERF_REQUIRE(build_segs(segs, n_segs, L));
    NERF_REQUIRE(W_x && aligned16(W_x) && ldw == L.ktot && (ldw % BK) == 0);
    const int epi = fwd ? (NERF_EPI_GAUSS | (bias ? NERF_EPI_BIAS : 0)) : NERF_EPI_GAUSS_BWD;
    double* part = static_cast<double*>(workspace);
    NTArgs a{L, (int)M, reinterpret_cast<const __bf16*>(W_x), ldw, N, bias, out, ldo, epi, z, ld_z, 1,
             inv_std, y, ld_y, part};
    int64_t slabs;
    if (N > 256 && NT_NBLOCK) {
        // wider layers (GARF's Linear(3, 1024), Linear(131, 512) and the input gradients into them):
        // column blocks of <= 256 on the 256-row tile kernel, each re-reading A, with the fp64
        // column partials of block n0 in their own [tiles][nb] slab block (part + n0 * tiles)
        const int ntiles = (int)((M + 255) / 256);
        int grid = cu_count_x3();
        if (grid > ntiles) grid = ntiles;
        const dim3 g3((unsigned)grid), b3(512);
        for (int n0 = 0; n0 < N; n0 += 256) {
            NTArgs b = a;
            b.N = N - n0 < 256 ? N - n0 : 256;
            b.Wx = a.Wx + (size_t)n0 * 2 * ldw;
            b.bias = bias ? bias + n0 : nullptr;
            b.out = out + n0;
            b.gs = inv_std + n0;
            if (fwd) b.y2 = y + n0;
            else b.aux = z + n0;
            b.part = part + (size_t)n0 * ntiles;
            if (b.N > 128) {
                if (epi == (NERF_EPI_GAUSS | NERF_EPI_BIAS)) hipLaunchKernelGGL((linear_nt_x3_glds_kernel<NERF_EPI_GAUSS | NERF_EPI_BIAS, 2>), g3, b3, 0, st, b, ntiles);
                else if (epi == NERF_EPI_GAUSS) hipLaunchKernelGGL((linear_nt_x3_glds_kernel<NERF_EPI_GAUSS, 2>), g3, b3, 0, st, b, ntiles);
                else hipLaunchKernelGGL((linear_nt_x3_glds_kernel<NERF_EPI_GAUSS_BWD, 2>), g3, b3, 0, st, b, ntiles);
            } else {
                if (epi == (NERF_EPI_GAUSS | NERF_EPI_BIAS)) hipLaunchKernelGGL((linear_nt_x3_glds_kernel<NERF_EPI_GAUSS | NERF_EPI_BIAS, 1>), g3, b3, 0, st, b, ntiles);
                else if (epi == NERF_EPI_GAUSS) hipLaunchKernelGGL((linear_nt_x3_glds_kernel<NERF_EPI_GAUSS, 1>), g3, b3, 0, st, b, ntiles);
                else hipLaunchKernelGGL((linear_nt_x3_glds_kernel<NERF_EPI_GAUSS_BWD, 1>), g3, b3, 0, st, b, ntiles);
            }
            NERF_CHECK_LAUNCH();
        }
        if (fwd) return NERF_OK;
        for (int n0 = 0; n0 < N; n0 += 256) {
            const int nb = N - n0 < 256 ? N - n0 : 256;
            const int rc = nerf::gauss_reduce(part + (size_t)n0 * ntiles, ntiles, nb, inv_std + n0, grad_inv_std + n0,
                                              accumulate, part + (size_t)ntiles * N, st);
            if (rc != NERF_OK) return rc;
        }
        return NERF_OK;
    }
    if (N <= 256) {
        const int ntiles = (int)((M + 255) / 256);
        int grid = cu_count_x3();
        if (grid > ntiles) grid = ntiles;
        const dim3 g3((unsigned)grid), b3(512);
#define NERF_GLDS_LAUNCH(E)                                                                          \
    do {                                                                                            \
        if (N > 128) hipLaunchKernelGGL((linear_nt_x3_glds_kernel<E, 2>), g3, b3, 0, st, a, ntiles); \
        else hipLaunchKernelGGL((linear_nt_x3_glds_kernel<E, 1>), g3, b3, 0, st, a, ntiles);         \
    } while (0)
        if (epi == (NERF_EPI_GAUSS | NERF_EPI_BIAS)) NERF_GLDS_LAUNCH(NERF_EPI_GAUSS | NERF_EPI_BIAS);
        else if (epi == NERF_EPI_GAUSS) NERF_GLDS_LAUNCH(NERF_EPI_GAUSS);
        else NERF_GLDS_LAUNCH(NERF_EPI_GAUSS_BWD);
#undef NERF_GLDS_LAUNCH
        slabs = ntiles;
    } else {
        const int ntm = (int)((M + 127) / 128);
        const int ntn = (N + 127) / 128;
        const int ntiles = (ntm + 7) / 8 * 8 * ntn;
        int grid = ntiles;
        const int cap = 2 * cu_count_x3();
        if (grid > cap) grid = cap;
        hipLaunchKernelGGL(linear_nt_x3_kernel, dim3((unsigned)grid), dim3(256), 0, st, a, ntm, ntiles);
        slabs = ntm;
    }
    NERF_CHECK_LAUNCH();
    if (fwd) return NERF_OK;
    return nerf::gauss_reduce(part, slabs, N, inv_std, grad_inv_std, accumulate, part + slabs * N, st);
}

// NERF_WGRAD_SMALLN=0: layers with N <= 16 on the 128-tile kernel (A/B switch, read once)
static const bool SMALLN_ON = [] {
    const char* e = getenv("NERF_WGRAD_SMALLN");
    return !(e && e[0] == '0');
}();

// NERF_WGRAD_TR=0: the single-tile layers on the LDS-DMA stream kernel instead of the register-staged
// transposed-read kernel (A/B switch, read once).  The two are bitwise equal (tests/
// test_gpu_wgrad_tr.py); the transposed-read kernel runs 313 vs 363 us at M = 524 288, N = K = 256
// and 264 vs 349 us for the 257-row layer (profiles/r04e/ab_*.txt)
static const bool WGRAD_TR = [] {
    const char* e = getenv("NERF_WGRAD_TR");
    return !(e && e[0] == '0');
}();

static int wgrad_x3_rows_impl(const float* dY, int64_t ld_dy, const nerf_seg* segs, int64_t M0,
                              const float* dY1, int64_t ld_dy1, const nerf_seg* segs1, int64_t M1,
                              int32_t n_segs, int32_t N, void* workspace, size_t workspace_bytes,
                              float* raysum, int32_t S0, int32_t S1, int32_t passes, void* stream) {
    NERF_REQUIRE(passes == 1 || passes == 3);
    const bool x1 = passes == 1;
    // N need not be a multiple of 4: the kernels read dY in 4-column pieces up to pad4(N) <= ld_dy;
    // slab rows past N are left unspecified (nerf_linear_wgrad_reduce's n_valid <= N)
    const int64_t M = M0 + M1;
    NERF_REQUIRE(dY && N >= 1 && M0 >= 0 && M1 >= 0 && M < (1ll << 31) && aligned16(dY) && (ld_dy % 4) == 0 &&
                 ld_dy >= (N + 3) / 4 * 4);
    SegList L;
    NERF_REQUIRE(build_segs(segs, n_segs, L));
    const int ntn = (N + TB - 1) / TB, ntk = (L.ktot + TB - 1) / TB;
    const int splits = nerf_wgrad_choose_splits(M, nerf_wgrad_split_tiles(N, L.ktot));
    const size_t need = nerf_linear_wgrad_workspace(M, N, L.ktot);
    if (!workspace || workspace_bytes < need || !aligned16(workspace)) return NERF_ERR_WORKSPACE;
    float* slab = reinterpret_cast<float*>(workspace);
    float* db_slab = slab + (size_t)splits * ntn * TB * (size_t)ntk * TB;
    int64_t mps = (M + splits - 1) / splits;
    mps = ((mps + TBM - 1) / TBM) * TBM;
    if (raysum != nullptr) {
        // per-ray sums of dY from the streamed kernel: rays of 16..128 samples (S | 128) or of a multiple
        // of 128 samples (3d-ingp's 256-sample fine pass) that no step or split cuts (splits and block 1
        // start at multiples of lcm(128, S0, S1) rows)
        auto s_ok = [](int S) { return S >= 16 && S <= 4096 && (128 % S == 0 || S % 128 == 0); };
        auto lcm = [](int64_t x, int64_t y) {
            int64_t g = x, h = y;
            while (h) { const int64_t t = g % h; g = h; h = t; }
            return x / g * y;
        };
        NERF_REQUIRE(s_ok(S0) && (M1 == 0 || s_ok(S1)));
        const int64_t R = lcm(lcm(128, S0), M1 ? S1 : 1);
        NERF_REQUIRE((M1 == 0 || M0 % R == 0) && M0 % S0 == 0 && M1 % (M1 ? S1 : 1) == 0);
        NERF_REQUIRE((N > 128 || L.ktot > 128) && N <= 256 && L.ktot <= 256);
        mps = ((mps + R - 1) / R) * R;
    }
    TNArgs a{dY, ld_dy, N, L, (int)M, (int)mps, splits, slab, db_slab, (int)M0, dY, ld_dy, {}, {}, {},
             raysum, S0 > 0 ? S0 : 1, S1 > 0 ? S1 : 1, S0 > 0 ? (int)(M0 / S0) : 0};
    for (int i = 0; i < MAX_SEGS; ++i) {
        a.x1ptr[i] = L.ptr[i];
        a.x1ld[i] = L.ld[i];
        a.x1rd[i] = L.row_div[i];
    }
    if (M1 > 0) {
        // the second block: the same segment structure (widths, packed offsets), its own rows
        NERF_REQUIRE(dY1 && aligned16(dY1) && (ld_dy1 % 4) == 0 && ld_dy1 >= (N + 3) / 4 * 4);
        SegList L1;
        NERF_REQUIRE(build_segs(segs1, n_segs, L1) && L1.n == L.n && L1.ktot == L.ktot);
        for (int i = 0; i < L.n; ++i) NERF_REQUIRE(L1.k[i] == L.k[i] && L1.kp[i] == L.kp[i]);
        a.dY1 = dY1;
        a.lddy1 = ld_dy1;
        for (int i = 0; i < MAX_SEGS; ++i) {
            a.x1ptr[i] = L1.ptr[i];
            a.x1ld[i] = L1.ld[i];
            a.x1rd[i] = L1.row_div[i];
        }
    } else {
        a.M0 = (int)M;
    }
    // (M = 0 still launches: every split writes its zero slab, which the reduce reads)
    if (N <= 16 && L.ktot <= 4 * SN_T && SMALLN_ON) {                  // few output rows: vector-ALU stream
        const int n4 = (N + 3) / 4 * 4;
        const int rg = SN_T / (L.ktot / 4);
        const size_t lds = ((size_t)rg * n4 * L.ktot + (size_t)rg * n4) * sizeof(float);
        if (lds <= 160 * 1024) {
            const dim3 grid((unsigned)splits), block(SN_T);
            switch (n4) {
                case 4: hipLaunchKernelGGL(linear_wgrad_smalln_kernel<4>, grid, block, lds, as_stream(stream), a, ntk * TB); break;
                case 8: hipLaunchKernelGGL(linear_wgrad_smalln_kernel<8>, grid, block, lds, as_stream(stream), a, ntk * TB); break;
                case 12: hipLaunchKernelGGL(linear_wgrad_smalln_kernel<12>, grid, block, lds, as_stream(stream), a, ntk * TB); break;
                default: hipLaunchKernelGGL(linear_wgrad_smalln_kernel<16>, grid, block, lds, as_stream(stream), a, ntk * TB); break;
            }
            NERF_CHECK_LAUNCH();
            return NERF_OK;
        }
    }
    if ((N > 128 || L.ktot > 128) && N <= 257 && L.ktot <= 256) {   // one 256 x 256 tile (+ row 256)
        const dim3 grid((unsigned)splits), block(512);
        hipStream_t st = as_stream(stream);
        if (WGRAD_TR) {
            // register-staged rows, transposed LDS reads (linear_wgrad_x3_tr_kernel); inputs of <= 128
            // columns spread their 4 column blocks over the 4 SIMDs (JN = 1)
            const bool narrow = L.ktot <= 128 && !raysum;
#define NERF_WT_LAUNCH(R257, RAYS, X1, JN) \
    hipLaunchKernelGGL((linear_wgrad_x3_tr_kernel<R257, RAYS, X1, JN>), grid, block, 0, st, a, ntn * TB, ntk * TB)
            if (x1) {
                if (narrow && N > 256) NERF_WT_LAUNCH(true, false, true, 1);
                else if (narrow) NERF_WT_LAUNCH(false, false, true, 1);
                else if (N > 256) NERF_WT_LAUNCH(true, false, true, 2);
                else if (raysum) NERF_WT_LAUNCH(false, true, true, 2);
                else NERF_WT_LAUNCH(false, false, true, 2);
            } else {
                if (narrow && N > 256) NERF_WT_LAUNCH(true, false, false, 1);
                else if (narrow) NERF_WT_LAUNCH(false, false, false, 1);
                else if (N > 256) NERF_WT_LAUNCH(true, false, false, 2);
                else if (raysum) NERF_WT_LAUNCH(false, true, false, 2);
                else NERF_WT_LAUNCH(false, false, false, 2);
            }
#undef NERF_WT_LAUNCH
        } else if (x1) {
            hipLaunchKernelGGL((linear_wgrad_x3_stream_kernel<3, 2, true>), grid, block, 0, st, a, ntn * TB, ntk * TB);
        } else {
            hipLaunchKernelGGL((linear_wgrad_x3_stream_kernel<3, 2, false>), grid, block, 0, st, a, ntn * TB, ntk * TB);
        }
        NERF_CHECK_LAUNCH();
        return NERF_OK;
    }
    const int64_t blocks = (int64_t)splits * ntn * ntk;
    if (x1)
        hipLaunchKernelGGL(linear_wgrad_x3_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), a);
    else
        hipLaunchKernelGGL(linear_wgrad_x3_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), a);
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}

extern "C" int nerf_linear_wgrad_x3_rows(const float* dY, int64_t ld_dy, const nerf_seg* segs, int64_t M0,
                                         const float* dY1, int64_t ld_dy1, const nerf_seg* segs1, int64_t M1,
                                         int32_t n_segs, int32_t N, void* workspace, size_t workspace_bytes,
                                         int32_t passes, void* stream) {
    return wgrad_x3_rows_impl(dY, ld_dy, segs, M0, dY1, ld_dy1, segs1, M1, n_segs, N, workspace, workspace_bytes,
                              nullptr, 0, 0, passes, stream);
}

extern "C" int nerf_linear_wgrad_x3_rays(const float* dY, int64_t ld_dy, const nerf_seg* segs, int64_t M0,
                                         const float* dY1, int64_t ld_dy1, const nerf_seg* segs1, int64_t M1,
                                         int32_t n_segs, int32_t N, void* workspace, size_t workspace_bytes,
                                         float* raysum, int32_t samples_per_ray0, int32_t samples_per_ray1,
                                         int32_t passes, void* stream) {
    NERF_REQUIRE(raysum != nullptr);
    return wgrad_x3_rows_impl(dY, ld_dy, segs, M0, dY1, ld_dy1, segs1, M1, n_segs, N, workspace, workspace_bytes,
                              raysum, samples_per_ray0, samples_per_ray1, passes, stream);
}

extern "C" int nerf_linear_wgrad_x3(const float* dY, int64_t ld_dy, int32_t N, const nerf_seg* segs, int32_t n_segs,
                                    int64_t M, void* workspace, size_t workspace_bytes, int32_t passes, void* stream) {
    return nerf_linear_wgrad_x3_rows(dY, ld_dy, segs, M, nullptr, 0, nullptr, 0, n_segs, N, workspace,
                                     workspace_bytes, passes, stream);
}

extern "C" int nerf_pack_weight_x3(const float* W, int32_t N, int32_t K_orig, const int32_t* col_map, int32_t Kp,
                                   void* Wp_x, void* Wt_x, int32_t ldwt, void* stream) {
    NERF_REQUIRE(W && col_map && N >= 1 && K_orig >= 1 && Kp >= 1 && (Kp % BK) == 0);
    const int npad = ((N + 127) / 128) * 128;
    if (Wt_x) NERF_REQUIRE(ldwt >= ((N + 31) / 32) * 32 && (ldwt % BK) == 0);
    const int kpad_rows = ((Kp + 127) / 128) * 128 + 128;
    int64_t total = (int64_t)npad * Kp;
    if (Wt_x) {
        const int64_t pad_total = (int64_t)(kpad_rows - Kp) * ldwt;
        if (pad_total > total) total = pad_total;
    }
    hipLaunchKernelGGL(pack_weight_x3_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, as_stream(stream), W,
                       N, K_orig, col_map, Kp, npad, reinterpret_cast<__bf16*>(Wp_x), reinterpret_cast<__bf16*>(Wt_x),
                       ldwt, kpad_rows);
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}

extern "C" __attribute__((visibility("hidden"))) int32_t nerf_tu_build_flags_linear_x3(void) {
    return NERF_TU_BUILD_FLAGS;
}
