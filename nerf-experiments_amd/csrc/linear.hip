// fp32 MFMA linear layers for the NeRF field MLPs (forward, input-gradient and
// weight-gradient), replacing the addmm chain of NerfModel.forward
// (barf/model_interpolation_architecture.py:96-141) and its autograd backward.
//
// Numerics: v_mfma_f32_32x32x2_f32 is an exact fp32 FMA chain (no TF32 on
// gfx950), so results differ from CPU BLAS only by summation order.
//
// Forward / input-gradient ("NT"): out[M,N] = epi(A[M,K] . W[N,K]^T)
//   256 threads = 4 waves.  BN = 128: 128 x 128 tile, waves 2 x 2, each 64 x 64
//   (2 x 2 MFMA blocks of 32 x 32).  BN = 32 (narrow layers, N <= 32): 128 x 32
//   tile, 4 waves stacked in M, each 32 x 32.
//   K streams in 32-wide chunks through a double-buffered LDS tile (rows
//   padded to 36 floats: the 16 distinct rows of a ds_read_b128 lane group hit
//   16 distinct 16-byte bank slots).  In a chunk, MFMA k-step s (0..15) pairs
//   columns s and 16 + s: lane half h reads columns h*16 + 4g .. +3 with one
//   ds_read_b128 per operand block, which feeds four k-steps.
//   A is a column-concatenation of up to 4 segments (activations | position
//   encoding | per-ray direction encoding), so the reference's th.cat copies
//   never exist; per-thread row pointers are recomputed only at segment
//   boundaries (row_div broadcasts per-ray rows over their samples).
//   The epilogue stages the accumulator tile through LDS so bias, ReLU, the
//   ReLU-backward mask (aux) and accumulation run on coalesced 16-byte rows.
//
// Weight gradient ("TN"): slab[s][n][k] = sum_{m in slice s} dY[m,n] X[m,k]
//   tile 128(n) x 128(k), split over M; 32-row M chunks staged in LDS; the
//   MFMA reduction index is the sample index.  A second kernel sums the
//   slices in a fixed order (deterministic) and scatters into the nn.Linear
//   gradient layout through a column map.
#include <cstdlib>

#include "common.h"

using namespace nerf;

typedef float f32x16 __attribute__((ext_vector_type(16)));
// native 4-wide vector (HIP's f4 is a struct: copies of it become memcpys that
// defeat register promotion of the staging arrays)
typedef float f4 __attribute__((ext_vector_type(4)));

namespace {

constexpr int BK = 32, LDP = BK + 4;  // chunk width and padded LDS row (floats)
constexpr int MAX_SEGS = 4;

struct SegList {
    const float* ptr[MAX_SEGS];
    int64_t ld[MAX_SEGS];
    int k[MAX_SEGS];        // valid columns (multiple of 4)
    int kp[MAX_SEGS];       // padded width in the packed weight layout (multiple of 32)
    int row_div[MAX_SEGS];
    int koff[MAX_SEGS];     // first packed column of the segment
    int n;
    int ktot;               // sum of kp
};

struct NTArgs {
    SegList A;
    int M;
    const float* W; int ldw; int N;
    const float* bias;
    float* out; int64_t ldo;
    int epi;
    const float* aux; int64_t ldaux;
    int vec_ok;             // out/aux/bias 16-byte aligned with ld % 4 == 0
};

// Runtime segment selection without dynamic indexing of the by-value kernel
// argument (which would force a private-memory copy of the struct).
template <typename T>
__device__ __forceinline__ T pick4(const T (&v)[MAX_SEGS], int i) {
    T r = v[0];
    r = (i == 1) ? v[1] : r;
    r = (i == 2) ? v[2] : r;
    r = (i == 3) ? v[3] : r;
    return r;
}

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

template <int BN>
struct TileCfg;
template <>
struct TileCfg<128> {
    static constexpr int WAVES_N = 2, WM = 64, WN = 64, BM = 128;
};
template <>
struct TileCfg<32> {
    static constexpr int WAVES_N = 1, WM = 32, WN = 32, BM = 128;
};

// XCD-aware tile order: blocks b and b + 8 are dealt to the same XCD, so the ntn
// column tiles of one row tile (which share the A rows) are placed 8 apart and
// read A once from HBM into that XCD's L2.  Returns false for padding tiles.
__device__ __forceinline__ bool tile_coords(int tile, int ntm, int ntn, int& tm, int& tn) {
    const int grp = 8 * ntn;
    const int g = tile / grp, r = tile - g * grp;
    tn = r / 8;
    tm = g * 8 + (r - tn * 8);
    return tm < ntm;
}

// Persistent over output tiles: a workgroup walks tiles blockIdx.x, +gridDim.x, ...
// and stages the NEXT tile's first K chunk during the current tile's last chunk,
// so the HBM latency of a tile start is hidden behind MFMA work.  The epilogue
// stages the accumulators through the idle LDS buffer, 64 rows at a time.
template <int BN>
__global__ __launch_bounds__(256, 2) void linear_nt_kernel(NTArgs a, int ntm, int ntiles) {
    const EpiOut E{a.out, a.ldo, a.bias, a.aux, a.ldaux, a.M, a.N, a.epi, a.vec_ok};
    using Cfg = TileCfg<BN>;
    constexpr int BM = Cfg::BM, WM = Cfg::WM, WN = Cfg::WN;
    constexpr int MB = WM / 32, NB = WN / 32;   // MFMA blocks per wave
    constexpr int NA = BM / 32, NW = BN / 32;   // f4 staging loads per thread per chunk
    constexpr int LDC = BN + 4;
    constexpr int BUF = (BM + BN) * LDP;
    constexpr int HR = BM / 2;                  // epilogue rows per half
    static_assert(HR * LDC <= BUF, "epilogue half-tile must fit one staging buffer");
    __shared__ __attribute__((aligned(16))) float smem[2 * BUF];

    const int ntn = (a.N + BN - 1) / BN;
    const int t = threadIdx.x;
    const int wave = t >> 6, lane = t & 63;
    const int wr = wave / Cfg::WAVES_N, wc = wave % Cfg::WAVES_N;
    const int li = lane & 31, lh = lane >> 5;
    const int c4 = t & 7, rbase = t >> 3;

    // find this workgroup's first real tile
    int tile = blockIdx.x, tm = 0, tn = 0;
    while (tile < ntiles && !tile_coords(tile, ntm, ntn, tm, tn)) tile += gridDim.x;
    if (tile >= ntiles) return;
    int m0 = tm * BM, n0 = tn * BN;

    // ---- segment state: scalar parameters + per-thread row offsets
    int seg = 0;
    const float* sp = nullptr;
    int sk = 0, skp = 0, skoff = 0;
    int64_t aoff[NA];
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
        for (int i = 0; i < NA; ++i) {
            const int m = mbase + i * 32 + rbase;
            const bool ok = m < a.M;
            const unsigned mc = (unsigned)(ok ? m : a.M - 1);
            const unsigned src = (rd == 1u) ? mc : mc / rd;
            aoff[i] = (int64_t)src * ld;  // row start; the column is added per chunk
            aok |= (ok ? 1u : 0u) << i;
        }
    };
    int64_t woff[NW];
    auto set_w = [&](int nbase) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < NW; ++j) woff[j] = (int64_t)(nbase + j * 32 + rbase) * a.ldw + c4 * 4;
    };

    f4 ra[NA], rw[NW];
    unsigned rmask = 0;  // rows/columns of the staged chunk to zero-fill (applied at the LDS write,
                         // so the loads stay in flight under the MFMAs)
    auto load_chunk = [&](int kc) __attribute__((always_inline)) {
        const int col = kc + c4 * 4;
        const bool cok = col < sk;
        const int acol = cok ? col : 0;  // columns past k are never addressed (zero-filled)
        rmask = cok ? aok : 0u;
#pragma unroll
        for (int i = 0; i < NA; ++i) ra[i] = *reinterpret_cast<const f4*>(sp + aoff[i] + acol);
#pragma unroll
        for (int j = 0; j < NW; ++j) rw[j] = *reinterpret_cast<const f4*>(a.W + woff[j] + skoff + kc);
    };
    auto store_chunk = [&](int buf) __attribute__((always_inline)) {
        float* As = smem + buf * BUF;
        float* Ws = As + BM * LDP;
#pragma unroll
        for (int i = 0; i < NA; ++i)
            *reinterpret_cast<f4*>(As + (i * 32 + rbase) * LDP + c4 * 4) =
                ((rmask >> i) & 1u) ? ra[i] : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < NW; ++j) *reinterpret_cast<f4*>(Ws + (j * 32 + rbase) * LDP + c4 * 4) = rw[j];
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
        // next tile of this workgroup (if any)
        int ntile = tile + gridDim.x, ntm_ = 0, ntn_ = 0;
        while (ntile < ntiles && !tile_coords(ntile, ntm, ntn, ntm_, ntn_)) ntile += gridDim.x;
        const bool has_next_tile = ntile < ntiles;

        f32x16 acc[MB][NB];
#pragma unroll
        for (int i = 0; i < MB; ++i)
#pragma unroll
            for (int j = 0; j < NB; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

        for (int c = 0; c < nchunks; ++c) {
            // stage the next chunk: of this tile, else the first chunk of the next tile
            // (else re-stage chunk 0 into the idle buffer, never read: branch-free registers)
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
            // keep the staging loads here, ahead of the MFMAs: left alone, the scheduler
            // sinks them to the end of the block (register reuse) and the chunk then
            // waits on a full HBM round trip before its ds_write
            __builtin_amdgcn_sched_barrier(0);

            const float* Ab = smem + cur * BUF + (wr * WM + li) * LDP + lh * 16;
            const float* Bb = smem + cur * BUF + BM * LDP + (wc * WN + li) * LDP + lh * 16;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                f4 av[MB], bv[NB];
#pragma unroll
                for (int i = 0; i < MB; ++i) av[i] = *reinterpret_cast<const f4*>(Ab + i * 32 * LDP + g * 4);
#pragma unroll
                for (int j = 0; j < NB; ++j) bv[j] = *reinterpret_cast<const f4*>(Bb + j * 32 * LDP + g * 4);
#pragma unroll
                for (int i = 0; i < MB; ++i)
#pragma unroll
                    for (int j = 0; j < NB; ++j) {
                        acc[i][j] = mfma32(av[i].x, bv[j].x, acc[i][j]);
                        acc[i][j] = mfma32(av[i].y, bv[j].y, acc[i][j]);
                        acc[i][j] = mfma32(av[i].z, bv[j].z, acc[i][j]);
                        acc[i][j] = mfma32(av[i].w, bv[j].w, acc[i][j]);
                    }
            }
            store_chunk(cur ^ 1);
            __syncthreads();
            cur ^= 1;
        }
        // now `cur` holds the next tile's first chunk; buffer cur ^ 1 is idle

        // ---- epilogue: accumulators -> idle LDS buffer (64 rows at a time) -> 16-byte rows
        // C/D map of the 32x32 MFMA: col = lane & 31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
        float* Cs = smem + (cur ^ 1) * BUF;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if ((wr * WM) / HR == h) {
#pragma unroll
                for (int i = 0; i < MB; ++i)
#pragma unroll
                    for (int j = 0; j < NB; ++j)
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            const int row = wr * WM - h * HR + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                            Cs[row * LDC + wc * WN + j * 32 + li] = acc[i][j][r];
                        }
            }
            __syncthreads();
            constexpr int Q = BN / 4;               // f4 per tile row
            constexpr int ITER = HR * Q / 256;
#pragma unroll 4
            for (int it = 0; it < ITER; ++it) {
                const int q = it * 256 + t;
                const int row = q / Q, cq = q - (q / Q) * Q;
                const int m = m0 + h * HR + row;
                const int n = n0 + cq * 4;
                epi_quad<BN / 4>(E, m < a.M && n < a.N, m, n, *reinterpret_cast<const f4*>(Cs + row * LDC + cq * 4));
            }
            __syncthreads();
        }

        if (!has_next_tile) break;
        tile = ntile;
        m0 = ntm_ * BM;
        n0 = ntn_ * BN;
    }
}

// ------------------------------- weight gradient ---------------------------
constexpr int TB = 128;  // n and k tile of the weight-gradient kernel
constexpr int TBM = 32;  // samples per LDS stage

struct TNArgs {
    const float* dY; int64_t lddy; int N;
    SegList X;
    int M;
    int m_per_split;
    int splits;
    float* slab;      // [splits][ntn*128][ntk*128]
    float* db_slab;   // [splits][ntn*128]
};

__global__ __launch_bounds__(256, 2) void linear_wgrad_kernel(TNArgs a) {
    __shared__ __attribute__((aligned(16))) float sY[2][TBM][TB];
    __shared__ __attribute__((aligned(16))) float sX[2][TBM][TB];

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
    const int wr = wave >> 1, wc = wave & 1;   // wr: n half, wc: k half
    const int li = lane & 31, lh = lane >> 5;

    // this thread's fixed load column (f4 granule) for both tiles
    const int c4 = t & 31;
    const int rr = t >> 5;  // 0..7: rows rr, rr+8, rr+16, rr+24 of each stage
    const int ny = n0 + c4 * 4;
    const bool ny_ok = ny < a.N;
    const int kx = k0 + c4 * 4;
    int xs = -1, xoff = 0;
#pragma unroll
    for (int s = 0; s < MAX_SEGS; ++s)
        if (s < a.X.n && kx >= a.X.koff[s] && kx < a.X.koff[s] + a.X.kp[s]) { xs = s; xoff = kx - a.X.koff[s]; }
    const bool x_ok = xs >= 0 && xoff < (xs >= 0 ? pick4(a.X.k, xs) : 0);
    const float* xptr = x_ok ? pick4(a.X.ptr, xs) : a.dY;
    const int64_t xld = x_ok ? pick4(a.X.ld, xs) : 0;
    const unsigned xrd = x_ok ? (unsigned)pick4(a.X.row_div, xs) : 1u;

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    float dbacc = 0.f;

    f4 ry[4], rx[4];
    unsigned mmask = 0;  // staged rows inside the slice (zero-fill applied at the LDS write)
    auto gload = [&](int mc) __attribute__((always_inline)) {
        mmask = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int m = mc + rr + 8 * i;
            const bool mok = m < mend;
            mmask |= (mok ? 1u : 0u) << i;
            const unsigned mm = (unsigned)(mok ? m : mbeg);
            ry[i] = *reinterpret_cast<const f4*>(a.dY + (int64_t)mm * a.lddy + (ny_ok ? ny : 0));
            rx[i] = *reinterpret_cast<const f4*>(xptr + (int64_t)(xrd == 1u ? mm : mm / xrd) * xld + (x_ok ? xoff : 0));
        }
    };
    auto sstore = [&](int buf) __attribute__((always_inline)) {
        const f4 z = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const bool mok = (mmask >> i) & 1u;
            *reinterpret_cast<f4*>(&sY[buf][rr + 8 * i][c4 * 4]) = (mok && ny_ok) ? ry[i] : z;
            *reinterpret_cast<f4*>(&sX[buf][rr + 8 * i][c4 * 4]) = (mok && x_ok) ? rx[i] : z;
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
            __builtin_amdgcn_sched_barrier(0);  // issue the next stage's loads before the MFMAs
#pragma unroll
            for (int s = 0; s < 16; ++s) {
                const int mr = lh * 16 + s;
                float av[2], bv[2];
                av[0] = sY[cur][mr][wr * 64 + li];
                av[1] = sY[cur][mr][wr * 64 + 32 + li];
                bv[0] = sX[cur][mr][wc * 64 + li];
                bv[1] = sX[cur][mr][wc * 64 + 32 + li];
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) acc[i][j] = mfma32(av[i], bv[j], acc[i][j]);
            }
            if (tk == 0 && t < TB) {
#pragma unroll
                for (int r = 0; r < TBM; ++r) dbacc += sY[cur][r][t];
            }
            sstore(cur ^ 1);
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
    if (tk == 0 && t < TB) a.db_slab[(size_t)split * npad + n0 + t] = dbacc;
}

// Sum the split slabs.  Block = 64 consecutive outputs x 4 split groups; each
// thread sums splits g, g+4, ... (independent loads in flight), then the 4
// partial sums are added in a fixed order through LDS: deterministic.
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(int splits, int n_valid, int K, int npad, int kpad,
                                                           const float* __restrict__ slab,
                                                           const float* __restrict__ db_slab,
                                                           const int32_t* __restrict__ col_map,
                                                           float* __restrict__ dW, int64_t ld_dw,
                                                           float* __restrict__ db, int accumulate) {
    __shared__ double part[4][64];
    const int t = threadIdx.x;
    const int o = t & 63, g = t >> 6;
    const int64_t total = (int64_t)n_valid * K;
    const int64_t nblk_w = (total + 63) / 64;
    const bool is_db = (int64_t)blockIdx.x >= nblk_w;
    const int64_t idx = is_db ? ((int64_t)blockIdx.x - nblk_w) * 64 + o : (int64_t)blockIdx.x * 64 + o;
    const int64_t lim = is_db ? n_valid : total;
    double s0 = 0.0, s1 = 0.0;
    if (idx < lim) {
        size_t off, stride;
        if (is_db) {
            off = (size_t)idx;
            stride = (size_t)npad;
        } else {
            const int n = (int)(idx / K), k = (int)(idx - (idx / K) * K);
            off = (size_t)n * kpad + k;
            stride = (size_t)npad * kpad;
        }
        const float* base = (is_db ? db_slab : slab) + off;
#ifndef NERF_REDUCE_ILP2
        // eight slabs' loads in flight per thread (the slabs were just written: the sum runs at the
        // cache's bandwidth only with enough loads outstanding), summed in a fixed order
        double q[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
        int sp = g;
        for (; sp + 28 < splits; sp += 32) {
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = base[(size_t)(sp + 4 * j) * stride];
#pragma unroll
            for (int j = 0; j < 8; ++j) q[j] += (double)v[j];
        }
        for (int j = 0; sp < splits; sp += 4, ++j) q[j & 7] += (double)base[(size_t)sp * stride];
        s0 = ((q[0] + q[1]) + (q[2] + q[3]));
        s1 = ((q[4] + q[5]) + (q[6] + q[7]));
#else
        int sp = g;
        for (; sp + 4 < splits; sp += 8) {
            s0 += (double)base[(size_t)sp * stride];
            s1 += (double)base[(size_t)(sp + 4) * stride];
        }
        if (sp < splits) s0 += (double)base[(size_t)sp * stride];
#endif
    }
    part[g][o] = s0 + s1;
    __syncthreads();
    if (g == 0 && idx < lim) {
        const double s = ((part[0][o] + part[1][o]) + part[2][o]) + part[3][o];
        // accumulate: += the rounded sum (an fp32 add, as autograd's accumulation of two passes)
        if (is_db) {
            db[idx] = accumulate ? db[idx] + (float)s : (float)s;
        } else {
            const int n = (int)(idx / K), k = (int)(idx - (idx / K) * K);
            const int dst = col_map ? col_map[k] : k;
            if (dst >= 0) {
                float* p = dW + (int64_t)n * ld_dw + dst;
                *p = accumulate ? *p + (float)s : (float)s;
            }
        }
    }
}

// compute units of the current device (cached per device id)
int cu_count() {
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

// M splits of the weight gradient (a workspace-layout parameter shared by the fp32 and the
// split-precision kernels and the reduce): enough workgroups for the whole chip even with
// the 256 x 256 tiles of the split-precision kernel (one workgroup per CU).
int choose_splits(int64_t M, int tiles) {
    // NERF_WGRAD_SPLITS (read once) overrides the split count, for split-count experiments
    static const int64_t split_override = [] {
        const char* e = getenv("NERF_WGRAD_SPLITS");
        return e ? (int64_t)atoi(e) : (int64_t)0;
    }();
    int64_t target = 1024 / (tiles > 0 ? tiles : 1);
    if (target > 256) target = 256;
    if (split_override > 0) target = split_override;
    if (target < 1) target = 1;
    const int64_t max_splits = (M + TBM - 1) / TBM;
    if (target > max_splits) target = max_splits;
    return (int)target;
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

__global__ void pack_weight_kernel(const float* __restrict__ W, int N, int K_orig, const int32_t* __restrict__ col_map,
                                   int Kp, int npad, float* __restrict__ Wp, float* __restrict__ Wt, int ldwt,
                                   int kpad_rows) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)npad * Kp;
    if (idx < total) {
        const int n = (int)(idx / Kp), k = (int)(idx - (idx / Kp) * Kp);
        const int src = col_map[k];
        const float v = (n < N && src >= 0 && src < K_orig) ? W[(int64_t)n * K_orig + src] : 0.f;
        if (Wp) Wp[idx] = v;
        if (Wt && n < ldwt) Wt[(int64_t)k * ldwt + n] = v;
    }
    // zero the padding rows of Wt (k in [Kp, kpad_rows))
    if (Wt) {
        const int64_t pad_total = (int64_t)(kpad_rows - Kp) * ldwt;
        if (idx < pad_total) Wt[(int64_t)Kp * ldwt + idx] = 0.f;
    }
}

}  // namespace

// shared with linear_x3.hip (same slab layout and reduce)
int nerf_wgrad_choose_splits(int64_t M, int tiles) { return choose_splits(M, tiles); }

// The tile count the M split is chosen for: a layer the split-precision weight gradient runs as one
// 256 x 256 tile (plus, for N = 257, one row on the vector ALUs: NerfModel's density + feature
// layer, whose workspace and reduce see it padded to 260) counts as the four 128 x 128 tiles it
// covers, whatever its 128-tile grid
int nerf_wgrad_split_tiles(int N, int K) {
    if (N <= 260 && K <= 256 && (N > 128 || K > 128)) return 4;
    return ((N + TB - 1) / TB) * ((K + TB - 1) / TB);
}

extern "C" int nerf_linear_fwd(const nerf_seg* segs, int32_t n_segs, int64_t M, const float* W, int32_t ldw, int32_t N,
                               const float* bias, float* out, int64_t ldo, int32_t epilogue, const float* aux,
                               int64_t ld_aux, void* stream) {
    NERF_REQUIRE(M >= 0 && M < (1ll << 31) && N >= 1);
    if (M == 0) return NERF_OK;
    SegList L;
    NERF_REQUIRE(build_segs(segs, n_segs, L));
    NERF_REQUIRE(W && out && aligned16(W) && ldw == L.ktot && (ldw % 4) == 0 && ldo >= N);
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
    NTArgs a{L, (int)M, W, ldw, N, bias, out, ldo, epilogue, aux, ld_aux, vec_ok};
    const int ntm = (int)((M + 127) / 128);
    const int ntn = N <= 32 ? 1 : (N + 127) / 128;
    const int ntiles = (ntm + 7) / 8 * 8 * ntn;        // XCD-aware order pads to groups of 8 row tiles
    int grid = ntiles;
    if (!(epilogue & NERF_EPI_NO_PERSIST)) {
        const int cap = 2 * cu_count();                 // two resident workgroups per CU
        if (grid > cap) grid = cap;
    }
    hipStream_t st = as_stream(stream);
    if (N <= 32) {
        hipLaunchKernelGGL(linear_nt_kernel<32>, dim3((unsigned)grid), dim3(256), 0, st, a, ntm, ntiles);
    } else {
        hipLaunchKernelGGL(linear_nt_kernel<128>, dim3((unsigned)grid), dim3(256), 0, st, a, ntm, ntiles);
    }
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}

extern "C" size_t nerf_linear_wgrad_workspace(int64_t M, int32_t N, int32_t K) {
    const int ntn = (N + TB - 1) / TB, ntk = (K + TB - 1) / TB;
    const int splits = choose_splits(M, nerf_wgrad_split_tiles(N, K));
    return (size_t)splits * ntn * TB * (size_t)ntk * TB * sizeof(float) + (size_t)splits * ntn * TB * sizeof(float);
}

extern "C" int nerf_linear_wgrad(const float* dY, int64_t ld_dy, int32_t N, const nerf_seg* segs, int32_t n_segs,
                                 int64_t M, void* workspace, size_t workspace_bytes, void* stream) {
    NERF_REQUIRE(dY && N >= 1 && M >= 0 && M < (1ll << 31) && aligned16(dY) && (ld_dy % 4) == 0 && (N % 4) == 0 &&
                 ld_dy >= N);
    SegList L;
    NERF_REQUIRE(build_segs(segs, n_segs, L));
    const int ntn = (N + TB - 1) / TB, ntk = (L.ktot + TB - 1) / TB;
    const int splits = choose_splits(M, nerf_wgrad_split_tiles(N, L.ktot));
    const size_t need = nerf_linear_wgrad_workspace(M, N, L.ktot);
    if (!workspace || workspace_bytes < need || !aligned16(workspace)) return NERF_ERR_WORKSPACE;
    float* slab = reinterpret_cast<float*>(workspace);
    float* db_slab = slab + (size_t)splits * ntn * TB * (size_t)ntk * TB;
    int64_t mps = (M + splits - 1) / splits;
    mps = ((mps + TBM - 1) / TBM) * TBM;
    TNArgs a{dY, ld_dy, N, L, (int)M, (int)mps, splits, slab, db_slab};
    const int64_t blocks = (int64_t)splits * ntn * ntk;
    hipLaunchKernelGGL(linear_wgrad_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), a);
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}

extern "C" int nerf_linear_wgrad_reduce(int64_t M, int32_t N, int32_t K, int32_t n_valid, const void* workspace,
                                        const int32_t* col_map, float* dW, int64_t ld_dw, float* db,
                                        int32_t accumulate, void* stream) {
    NERF_REQUIRE(workspace && dW && N >= 1 && K >= 1 && n_valid >= 1 && n_valid <= N);
    const int ntn = (N + TB - 1) / TB, ntk = (K + TB - 1) / TB;
    const int splits = choose_splits(M, nerf_wgrad_split_tiles(N, K));
    const float* slab = reinterpret_cast<const float*>(workspace);
    const float* db_slab = slab + (size_t)splits * ntn * TB * (size_t)ntk * TB;
    const int64_t total = (int64_t)n_valid * K;
    const int64_t blocks = (total + 63) / 64 + (db ? (n_valid + 63) / 64 : 0);
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), splits, n_valid, K,
                       ntn * TB, ntk * TB, slab, db_slab, col_map, dW, ld_dw, db, accumulate != 0 ? 1 : 0);
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}

extern "C" int nerf_pack_weight(const float* W, int32_t N, int32_t K_orig, const int32_t* col_map, int32_t Kp,
                                float* Wp, float* Wt, int32_t ldwt, void* stream) {
    NERF_REQUIRE(W && col_map && N >= 1 && K_orig >= 1 && Kp >= 1 && (Kp % BK) == 0);
    const int npad = ((N + 127) / 128) * 128;
    if (Wt) NERF_REQUIRE(ldwt >= ((N + 31) / 32) * 32);
    const int kpad_rows = ((Kp + 127) / 128) * 128 + 128;
    int64_t total = (int64_t)npad * Kp;
    const int64_t pad_total = (int64_t)(kpad_rows - Kp) * (Wt ? ldwt : 0);
    if (pad_total > total) total = pad_total;
    hipLaunchKernelGGL(pack_weight_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, as_stream(stream), W, N,
                       K_orig, col_map, Kp, npad, Wp, Wt, ldwt, kpad_rows);
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}
