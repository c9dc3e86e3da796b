// fp32 MFMA linear layers for the NeRF field MLPs (forward, input-gradient and
// weight-gradient), replacing the addmm chain of NerfModel.forward
// (barf/model_interpolation_architecture.py:96-141) and its autograd backward.
//
// Numerics: v_mfma_f32_32x32x2_f32 is an exact fp32 FMA chain (no TF32 on
// gfx950), so results differ from CPU BLAS only by summation order.
//
// Forward / input-gradient ("NT"): out[M,N] = epi(A[M,K] . W[N,K]^T)
//   tile 128 x 128, 256 threads = 4 waves in a 2x2 grid, each wave 64 x 64 =
//   2 x 2 MFMA blocks of 32 x 32.  K streamed in 32-wide chunks through a
//   double-buffered LDS tile (rows padded to 36 floats: the 16 distinct rows
//   a ds_read_b128 lane group touches land on 16 distinct 16-byte bank slots).
//   In a chunk, MFMA k-step s (0..15) pairs columns s and 16+s: lane half h
//   reads columns h*16 + 4g .. +3 with one ds_read_b128 per operand block,
//   which feeds four k-steps.  A is a concatenation of up to 4 segments
//   (activations | positional encoding | per-ray direction encoding), so the
//   reference's torch.cat copies are never materialised.
//
// Weight gradient ("TN"): slab[s][n][k] = sum_{m in slice s} dY[m,n] X[m,k]
//   tile 128(n) x 128(k), split over M; 32-row M chunks staged in LDS; the
//   MFMA reduction index is the sample index.  A second kernel sums the slices
//   (fixed order, deterministic) and scatters into the nn.Linear grad layout.
#include "common.h"

using namespace nerf;

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int BM = 128, BN = 128, BK = 32, LDP = BK + 4;  // padded LDS row (floats)
constexpr int MAX_SEGS = 4;

struct SegList {
    const float* ptr[MAX_SEGS];
    int64_t ld[MAX_SEGS];
    int k[MAX_SEGS];
    int row_div[MAX_SEGS];
    int koff[MAX_SEGS];
    int n;
    int ktot;
};

struct NTArgs {
    SegList A;
    int64_t M;
    const float* W; int ldw; int N;
    const float* bias;
    float* out; int64_t ldo;
    int epi;
    const float* aux; int64_t ldaux;
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

// Loads one 128 x 32 A chunk (segment `sg`, column offset kc) and the matching
// 128 x 32 W chunk into registers (4 float4 each per thread).
__device__ __forceinline__ void load_chunk(const NTArgs& a, int sg, int kc, int64_t m0, int n0, float4 ra[4],
                                           float4 rb[4]) {
    const int t = threadIdx.x;
    const int c4 = t & 7;
    const float* sp = pick4(a.A.ptr, sg);
    const int64_t ld = pick4(a.A.ld, sg);
    const int rd = pick4(a.A.row_div, sg);
    const int koff = pick4(a.A.koff, sg);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = i * 32 + (t >> 3);
        const int64_t m = m0 + r;
        const bool ok = m < a.M;
        const int64_t mc = ok ? m : a.M - 1;  // clamp: branch-free load, zeroed below
        const int64_t src = (rd == 1 ? mc : mc / rd);
        float4 v = *reinterpret_cast<const float4*>(sp + src * ld + kc + c4 * 4);
        ra[i] = ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
        const int n = n0 + r;
        rb[i] = *reinterpret_cast<const float4*>(a.W + (int64_t)n * a.ldw + koff + kc + c4 * 4);
    }
}

__device__ __forceinline__ void store_chunk(float* As, float* Bs, const float4 ra[4], const float4 rb[4]) {
    const int t = threadIdx.x;
    const int c4 = t & 7;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = i * 32 + (t >> 3);
        *reinterpret_cast<float4*>(As + r * LDP + c4 * 4) = ra[i];
        *reinterpret_cast<float4*>(Bs + r * LDP + c4 * 4) = rb[i];
    }
}

__global__ __launch_bounds__(256, 2) void linear_nt_kernel(NTArgs a) {
    __shared__ __attribute__((aligned(16))) float smem[2 * 2 * BM * LDP];
    // buffer b: A tile at smem + b*2*BM*LDP, W tile right after it

    const int ntn = (a.N + BN - 1) / BN;
    const int bid = blockIdx.x;
    const int tn = bid % ntn;
    const int64_t tm = bid / ntn;
    const int64_t m0 = tm * BM;
    const int n0 = tn * BN;

    const int t = threadIdx.x;
    const int wave = t >> 6, lane = t & 63;
    const int wr = wave >> 1, wc = wave & 1;
    const int li = lane & 31, lh = lane >> 5;

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // chunk iteration over (segment, kc)
    int sg = 0, kc = 0;
    float4 ra[4], rb[4];
    load_chunk(a, sg, kc, m0, n0, ra, rb);
    store_chunk(smem, smem + BM * LDP, ra, rb);
    __syncthreads();
    const int nchunks = a.A.ktot / BK;
    int cur = 0;
    for (int c = 0; c < nchunks; ++c) {
        // advance to next chunk coordinates
        int nsg = sg, nkc = kc + BK;
        if (nkc >= pick4(a.A.k, nsg)) { nsg++; nkc = 0; }
        const bool has_next = (c + 1 < nchunks);
        // the last iteration re-stages chunk 0 into the idle buffer (never read):
        // keeps the staging registers branch-free
        load_chunk(a, has_next ? nsg : 0, has_next ? nkc : 0, m0, n0, ra, rb);

        const float* Ab = smem + cur * 2 * BM * LDP + (wr * 64 + li) * LDP + lh * 16;
        const float* Bb = smem + cur * 2 * BM * LDP + BM * LDP + (wc * 64 + li) * LDP + lh * 16;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            float4 av[2], bv[2];
            av[0] = *reinterpret_cast<const float4*>(Ab + g * 4);
            av[1] = *reinterpret_cast<const float4*>(Ab + 32 * LDP + g * 4);
            bv[0] = *reinterpret_cast<const float4*>(Bb + g * 4);
            bv[1] = *reinterpret_cast<const float4*>(Bb + 32 * LDP + g * 4);
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    acc[i][j] = mfma32(av[i].x, bv[j].x, acc[i][j]);
                    acc[i][j] = mfma32(av[i].y, bv[j].y, acc[i][j]);
                    acc[i][j] = mfma32(av[i].z, bv[j].z, acc[i][j]);
                    acc[i][j] = mfma32(av[i].w, bv[j].w, acc[i][j]);
                }
        }
        store_chunk(smem + (cur ^ 1) * 2 * BM * LDP, smem + (cur ^ 1) * 2 * BM * LDP + BM * LDP, ra, rb);
        __syncthreads();
        cur ^= 1;
        sg = nsg; kc = nkc;
    }

    // epilogue: C/D map of 32x32 MFMA: col = lane & 31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int n = n0 + wc * 64 + j * 32 + li;
        if (n >= a.N) continue;
        const float bv = (a.epi & NERF_EPI_BIAS) ? a.bias[n] : 0.f;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int64_t m = m0 + wr * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                if (m >= a.M) continue;
                float v = acc[i][j][r];
                if (a.epi & NERF_EPI_BIAS) v = v + bv;
                if (a.epi & NERF_EPI_RELU) v = fmaxf(v, 0.f);
                if (a.epi & NERF_EPI_MASK) v = (a.aux[m * a.ldaux + n] > 0.f) ? v : 0.f;
                float* o = a.out + m * a.ldo + n;
                if (a.epi & NERF_EPI_ACCUM) v = *o + v;
                *o = v;
            }
        }
    }
}

// ------------------------------- weight gradient ---------------------------
constexpr int TBM = 32;  // samples per LDS stage

struct TNArgs {
    const float* dY; int64_t lddy; int N;
    SegList X;
    int64_t M;
    int64_t m_per_split;
    int splits;
    float* slab;      // [splits][ntn*128][ntk*128]
    float* db_slab;   // [splits][ntn*128]
};

__global__ __launch_bounds__(256, 2) void linear_wgrad_kernel(TNArgs a) {
    __shared__ __attribute__((aligned(16))) float sY[2][TBM][BN];
    __shared__ __attribute__((aligned(16))) float sX[2][TBM][BN];

    const int ntn = (a.N + BN - 1) / BN;
    const int ntk = (a.X.ktot + BN - 1) / BN;
    const int tiles = ntn * ntk;
    const int bid = blockIdx.x;
    const int split = bid / tiles;
    const int tile = bid - split * tiles;
    const int tn = tile / ntk, tk = tile - (tile / ntk) * ntk;
    const int n0 = tn * BN, k0 = tk * BN;
    const int64_t mbeg = (int64_t)split * a.m_per_split;
    int64_t mend = mbeg + a.m_per_split;
    if (mend > a.M) mend = a.M;

    const int t = threadIdx.x;
    const int wave = t >> 6, lane = t & 63;
    const int wr = wave >> 1, wc = wave & 1;   // wr: n half, wc: k half
    const int li = lane & 31, lh = lane >> 5;

    // this thread's fixed load column (float4 granule) for both tiles
    const int c4 = t & 31;
    const int rr = t >> 5;  // 0..7, rows rr, rr+8, rr+16, rr+24
    const int ny = n0 + c4 * 4;
    const bool ny_ok = ny < a.N;
    const int kx = k0 + c4 * 4;
    int xs = -1, xoff = 0;
#pragma unroll
    for (int s = 0; s < MAX_SEGS; ++s)
        if (s < a.X.n && kx >= a.X.koff[s] && kx < a.X.koff[s] + a.X.k[s]) { xs = s; xoff = kx - a.X.koff[s]; }
    const float* xptr = xs >= 0 ? pick4(a.X.ptr, xs) : nullptr;
    const int64_t xld = xs >= 0 ? pick4(a.X.ld, xs) : 0;
    const int xrd = xs >= 0 ? pick4(a.X.row_div, xs) : 1;

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    float dbacc = 0.f;

    float4 ry[4], rx[4];
    auto gload = [&](int64_t mc) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int64_t m = mc + rr + 8 * i;
            const bool mok = m < mend;
            ry[i] = (mok && ny_ok) ? *reinterpret_cast<const float4*>(a.dY + m * a.lddy + ny)
                                   : make_float4(0.f, 0.f, 0.f, 0.f);
            rx[i] = (mok && xptr) ? *reinterpret_cast<const float4*>(xptr + (xrd == 1 ? m : m / xrd) * xld + xoff)
                                  : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto sstore = [&](int buf) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            *reinterpret_cast<float4*>(&sY[buf][rr + 8 * i][c4 * 4]) = ry[i];
            *reinterpret_cast<float4*>(&sX[buf][rr + 8 * i][c4 * 4]) = rx[i];
        }
    };

    if (mbeg < mend) {
        gload(mbeg);
        sstore(0);
        __syncthreads();
        int cur = 0;
        for (int64_t mc = mbeg; mc < mend; mc += TBM) {
            const bool has_next = mc + TBM < mend;
            if (has_next) gload(mc + TBM);
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
            if (tk == 0 && t < BN) {
#pragma unroll
                for (int r = 0; r < TBM; ++r) dbacc += sY[cur][r][t];
            }
            if (has_next) sstore(cur ^ 1);
            __syncthreads();
            cur ^= 1;
        }
    }

    const int npad = ntn * BN, kpad = ntk * BN;
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
    if (tk == 0 && t < BN) a.db_slab[(size_t)split * npad + n0 + t] = dbacc;
}

__global__ __launch_bounds__(256) void wgrad_reduce_kernel(int splits, int N, int K, int npad, int kpad,
                                                           const float* __restrict__ slab,
                                                           const float* __restrict__ db_slab,
                                                           const int32_t* __restrict__ col_map,
                                                           float* __restrict__ dW, int64_t ld_dw,
                                                           float* __restrict__ db) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)N * K;
    if (idx < total) {
        const int n = (int)(idx / K), k = (int)(idx - (idx / K) * K);
        const int dst = col_map ? col_map[k] : k;
        if (dst >= 0) {
            double s = 0.0;
            for (int sp = 0; sp < splits; ++sp) s += (double)slab[((size_t)sp * npad + n) * kpad + k];
            dW[(int64_t)n * ld_dw + dst] = (float)s;
        }
    }
    if (db && idx < N) {
        double s = 0.0;
        for (int sp = 0; sp < splits; ++sp) s += (double)db_slab[(size_t)sp * npad + idx];
        db[idx] = (float)s;
    }
}

int choose_splits(int64_t M, int tiles) {
    int64_t target = 1024 / (tiles > 0 ? tiles : 1);
    if (target < 1) target = 1;
    const int64_t max_splits = (M + TBM - 1) / TBM;
    if (target > max_splits) target = max_splits;
    if (target > 4096) target = 4096;
    return (int)target;
}

bool build_segs(const nerf_seg* segs, int n, SegList& L) {
    if (!segs || n < 1 || n > MAX_SEGS) return false;
    int koff = 0;
    for (int i = 0; i < n; ++i) {
        const nerf_seg& s = segs[i];
        if (!s.ptr || s.k <= 0 || (s.k % BK) != 0 || s.ld < s.k || (s.ld % 4) != 0 || s.row_div < 1) return false;
        if (!aligned16(s.ptr)) return false;
        L.ptr[i] = s.ptr; L.ld[i] = s.ld; L.k[i] = s.k; L.row_div[i] = s.row_div; L.koff[i] = koff;
        koff += s.k;
    }
    for (int i = n; i < MAX_SEGS; ++i) { L.ptr[i] = nullptr; L.ld[i] = 0; L.k[i] = 0; L.row_div[i] = 1; L.koff[i] = koff; }
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

extern "C" int nerf_linear_fwd(const nerf_seg* segs, int32_t n_segs, int64_t M, const float* W, int32_t ldw, int32_t N,
                               const float* bias, float* out, int64_t ldo, int32_t epilogue, const float* aux,
                               int64_t ld_aux, void* stream) {
    NERF_REQUIRE(M >= 0 && N >= 1);
    if (M == 0) return NERF_OK;
    SegList L;
    NERF_REQUIRE(build_segs(segs, n_segs, L));
    NERF_REQUIRE(W && out && aligned16(W) && ldw == L.ktot && ldo >= N);
    if (epilogue & NERF_EPI_BIAS) NERF_REQUIRE(bias != nullptr);
    if (epilogue & NERF_EPI_MASK) NERF_REQUIRE(aux != nullptr && ld_aux >= N);
    NTArgs a{L, M, W, ldw, N, bias, out, ldo, epilogue, aux, ld_aux};
    const int64_t ntm = (M + BM - 1) / BM;
    const int64_t ntn = (N + BN - 1) / BN;
    const int64_t blocks = ntm * ntn;
    NERF_REQUIRE(blocks < (1ll << 31));
    hipLaunchKernelGGL(linear_nt_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), a);
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}

extern "C" size_t nerf_linear_wgrad_workspace(int64_t M, int32_t N, int32_t K) {
    const int ntn = (N + BN - 1) / BN, ntk = (K + BN - 1) / BN;
    const int splits = choose_splits(M, ntn * ntk);
    return (size_t)splits * ntn * BN * (size_t)ntk * BN * sizeof(float) + (size_t)splits * ntn * BN * sizeof(float);
}

extern "C" int nerf_linear_wgrad(const float* dY, int64_t ld_dy, int32_t N, const nerf_seg* segs, int32_t n_segs,
                                 int64_t M, void* workspace, size_t workspace_bytes, void* stream) {
    NERF_REQUIRE(dY && N >= 1 && M >= 0 && aligned16(dY) && (ld_dy % 4) == 0 && (N % 4) == 0 && ld_dy >= N);
    SegList L;
    NERF_REQUIRE(build_segs(segs, n_segs, L));
    const int ntn = (N + BN - 1) / BN, ntk = (L.ktot + BN - 1) / BN;
    const int splits = choose_splits(M, ntn * ntk);
    const size_t need = nerf_linear_wgrad_workspace(M, N, L.ktot);
    if (!workspace || workspace_bytes < need) return NERF_ERR_WORKSPACE;
    float* slab = reinterpret_cast<float*>(workspace);
    float* db_slab = slab + (size_t)splits * ntn * BN * (size_t)ntk * BN;
    int64_t mps = (M + splits - 1) / splits;
    mps = ((mps + TBM - 1) / TBM) * TBM;
    TNArgs a{dY, ld_dy, N, L, M, mps, splits, slab, db_slab};
    const int64_t blocks = (int64_t)splits * ntn * ntk;
    hipLaunchKernelGGL(linear_wgrad_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), a);
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}

extern "C" int nerf_linear_wgrad_reduce(int64_t M, int32_t N, int32_t K, int32_t n_valid, const void* workspace,
                                        const int32_t* col_map, float* dW, int64_t ld_dw, float* db, void* stream) {
    NERF_REQUIRE(workspace && dW && N >= 1 && K >= 1 && n_valid >= 1 && n_valid <= N);
    const int ntn = (N + BN - 1) / BN, ntk = (K + BN - 1) / BN;
    const int splits = choose_splits(M, ntn * ntk);
    const float* slab = reinterpret_cast<const float*>(workspace);
    const float* db_slab = slab + (size_t)splits * ntn * BN * (size_t)ntk * BN;
    const int64_t total = (int64_t)n_valid * K;
    const int64_t blocks = (total + 255) / 256;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), splits, n_valid, K,
                       ntn * BN, ntk * BN, slab, db_slab, col_map, dW, ld_dw, db);
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}

extern "C" int nerf_pack_weight(const float* W, int32_t N, int32_t K_orig, const int32_t* col_map, int32_t Kp,
                                float* Wp, float* Wt, int32_t ldwt, void* stream) {
    NERF_REQUIRE(W && col_map && N >= 1 && K_orig >= 1 && Kp >= 1 && (Kp % BK) == 0);
    const int npad = ((N + BN - 1) / BN) * BN;
    if (Wt) NERF_REQUIRE(ldwt >= ((N + 31) / 32) * 32);
    const int kpad_rows = ((Kp + BN - 1) / BN) * BN + BN;
    int64_t total = (int64_t)npad * Kp;
    const int64_t pad_total = (int64_t)(kpad_rows - Kp) * (Wt ? ldwt : 0);
    if (pad_total > total) total = pad_total;
    hipLaunchKernelGGL(pack_weight_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, as_stream(stream), W, N,
                       K_orig, col_map, Kp, npad, Wp, Wt, ldwt, kpad_rows);
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}
