// Proposal-network sampling and interlevel loss: the nerfacc pieces GARF's
// renderer calls — PropNetEstimator.sampling (garf/model_garf.py:210-220), its cdfs
// (1 - [trans, 0]) and compute_loss (:257).  nerfacc is not vendored (environment.yml:26, version
// unpinned, not installed here), so this restates its published algorithm: PARITY UNPINNED
// (oracle/nerfacc_oracle.py restates the same).  Contract in include/nerf_amd.h.
//
// Every kernel is one wave per ray, the ray's edges / cdf staged in LDS.  Sums are fp64 in a
// fixed order; the loss gradient with respect to the key cdf is gathered per key index over the
// contiguous range of query intervals that touch it (the search indices are monotone), so the
// result does not depend on scheduling.
#include "common.h"

using namespace nerf;

namespace {

constexpr int PW = 64;          // one wave per ray
constexpr int PRAYS = 4;        // rays per block

// number of v[0..n) <= x (torch.searchsorted(right=True) on a sorted row)
__device__ __forceinline__ int count_le(const float* v, int n, float x) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (v[mid] <= x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ float stot(float s, int transform, float near, float far) {
#pragma clang fp contract(off)
    if (transform == 0) return s * far + (1.0f - s) * near;                  // uniform
    return 1.0f / (s * (1.0f / far) + (1.0f - s) * (1.0f / near));           // lindisp: 1/t linear in s
}

// cdf[r][0] = 0, cdf[r][i] = sum_{j<i} w[r][j] (fp64 prefix), cdf[r][K] = 1
__global__ __launch_bounds__(PW * PRAYS) void prop_cdf_kernel(const float* __restrict__ w, int64_t ldw, int64_t R,
                                                             int K, float* __restrict__ cdf, int64_t ldc) {
    const int lane = threadIdx.x & (PW - 1);
    const int64_t r = (int64_t)blockIdx.x * PRAYS + (threadIdx.x >> 6);
    if (r >= R) return;
    double carry = 0.0;
    for (int base = 0; base < K; base += PW) {
        const int j = base + lane;
        double v = j < K ? (double)w[r * ldw + j] : 0.0;
        // inclusive wave scan (fixed order)
        for (int off = 1; off < PW; off <<= 1) {
            const double o = __shfl_up(v, off, PW);
            if (lane >= off) v += o;
        }
        if (j < K - 1) cdf[r * ldc + j + 1] = (float)(carry + v);
        carry += __shfl(v, PW - 1, PW);
    }
    if (lane == 0) {
        cdf[r * ldc] = 0.0f;
        cdf[r * ldc + K] = 1.0f;
    }
}

struct SampleArgs {
    const float* vals; int64_t ldv;
    const float* cdf; int64_t ldc;
    int64_t R; int K; int n;
    int stratified; uint64_t seed; uint64_t counter;
    int transform; float near, far;
    float* s_out; float* t_out; int64_t ldo;
};

// inverse CDF of the piecewise-linear cdf over the ray's edges at n + 1 quantiles
__global__ __launch_bounds__(PW * PRAYS) void prop_sample_kernel(SampleArgs a) {
#pragma clang fp contract(off)
    __shared__ float sv[PRAYS][NERF_PROP_MAX_EDGES];
    __shared__ float sc[PRAYS][NERF_PROP_MAX_EDGES];
    const int lane = threadIdx.x & (PW - 1), wv = threadIdx.x >> 6;
    const int64_t r = (int64_t)blockIdx.x * PRAYS + wv;
    const bool live = r < a.R;
    const int E = a.K + 1;
    if (live)
        for (int i = lane; i < E; i += PW) {
            sv[wv][i] = a.vals[r * a.ldv + i];
            sc[wv][i] = a.cdf[r * a.ldc + i];
        }
    __syncthreads();
    if (!live) return;
    for (int i = lane; i <= a.n; i += PW) {
        float u;
        if (i == 0) u = 0.0f;
        else if (i == a.n) u = 1.0f;
        else if (a.stratified) u = ((float)i - 0.5f + philox_uniform(a.seed, a.counter, (uint64_t)(r * (a.n + 1) + i))) / (float)a.n;
        else u = (float)i / (float)a.n;
        int b = count_le(sc[wv], E, u) - 1;          // last edge with cdf <= u
        b = b < 0 ? 0 : (b > a.K - 1 ? a.K - 1 : b);
        const float c0 = sc[wv][b], c1 = sc[wv][b + 1];
        const float den = c1 - c0;
        float f = den > 0.0f ? (u - c0) / den : 0.0f;
        f = f < 0.0f ? 0.0f : (f > 1.0f ? 1.0f : f);
        const float s = sv[wv][b] + f * (sv[wv][b + 1] - sv[wv][b]);
        a.s_out[r * a.ldo + i] = s;
        a.t_out[r * a.ldo + i] = stot(s, a.transform, a.near, a.far);
    }
}

struct LossArgs {
    const float* qv; const float* qc; int64_t ldq;     // query edges / cdf [R][n+1]
    const float* kv; const float* kc; int64_t ldk;     // key edges / cdf [R][K+1]
    int64_t R; int n; int K; float eps;
    float* loss_ray;                                   // [R] sum of the ray's interval losses (or null)
    float gscale;                                      // backward: d total / d each interval loss
    float* dkw; int64_t lddw;                          // backward: d total / d key weights [R][K] (or null)
};

// nerfacc _pdf_loss: w = qc[j+1]-qc[j]; w_outer = kc[right(q[j+1])] - kc[left(q[j])];
// loss_j = max(w - w_outer, 0)^2 / (w + eps); only the key cdf carries a gradient
__global__ __launch_bounds__(PW * PRAYS) void prop_loss_kernel(LossArgs a) {
#pragma clang fp contract(off)
    __shared__ float skv[PRAYS][NERF_PROP_MAX_EDGES];
    __shared__ float skc[PRAYS][NERF_PROP_MAX_EDGES];
    __shared__ float cj[PRAYS][NERF_PROP_MAX_EDGES];      // per query interval: d loss / d w_outer
    __shared__ int rj[PRAYS][NERF_PROP_MAX_EDGES];
    __shared__ int lj[PRAYS][NERF_PROP_MAX_EDGES];
    __shared__ double dcdf[PRAYS][NERF_PROP_MAX_EDGES];
    const int lane = threadIdx.x & (PW - 1), wv = threadIdx.x >> 6;
    const int64_t r = (int64_t)blockIdx.x * PRAYS + wv;
    const bool live = r < a.R;
    const int E = a.K + 1;
    if (live)
        for (int i = lane; i < E; i += PW) {
            skv[wv][i] = a.kv[r * a.ldk + i];
            skc[wv][i] = a.kc[r * a.ldk + i];
        }
    __syncthreads();
    double acc = 0.0;
    if (live)
        for (int j = lane; j < a.n; j += PW) {
            const float q0 = a.qv[r * a.ldq + j], q1 = a.qv[r * a.ldq + j + 1];
            int right = count_le(skv[wv], E, q1);
            right = right > a.K ? a.K : right;
            int left = count_le(skv[wv], E, q0) - 1;
            left = left < 0 ? 0 : (left > a.K ? a.K : left);
            const float w = a.qc[r * a.ldq + j + 1] - a.qc[r * a.ldq + j];
            const float wo = skc[wv][right] - skc[wv][left];
            const float d = fmaxf(w - wo, 0.0f);
            const float den = w + a.eps;
            acc += (double)((d * d) / den);
            cj[wv][j] = -(2.0f * d / den) * a.gscale;           // d loss_j / d w_outer
            rj[wv][j] = right;
            lj[wv][j] = left;
        }
    // fixed-order wave sum of the ray's loss
    for (int off = PW / 2; off > 0; off >>= 1) acc += __shfl_xor(acc, off, PW);
    if (live && lane == 0 && a.loss_ray != nullptr) a.loss_ray[r] = (float)acc;
    if (a.dkw == nullptr) return;
    __syncthreads();
    if (live) {
        // d w_outer_j / d kc[k] = [k == right_j] - [k == left_j]; right / left are non-decreasing
        // in j, so each k gathers a contiguous range of j, summed in order
        for (int k = lane; k < E; k += PW) {
            double g = 0.0;
            int lo = 0, hi = a.n;
            while (lo < hi) {                                     // first j with right_j >= k
                const int mid = (lo + hi) >> 1;
                if (rj[wv][mid] < k) lo = mid + 1;
                else hi = mid;
            }
            for (int j = lo; j < a.n && rj[wv][j] == k; ++j) g += (double)cj[wv][j];
            lo = 0, hi = a.n;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (lj[wv][mid] < k) lo = mid + 1;
                else hi = mid;
            }
            for (int j = lo; j < a.n && lj[wv][j] == k; ++j) g -= (double)cj[wv][j];
            dcdf[wv][k] = g;
        }
    }
    __syncthreads();
    if (live && lane == 0) {
        // kc[i] = sum_{j<i} w[j] for 0 < i < K (kc[0] = 0 and kc[K] = 1 are constants):
        // d w[j] = sum_{i=j+1}^{K-1} d kc[i], a suffix sum in fixed order
        double s = 0.0;
        for (int j = a.K - 1; j >= 0; --j) {
            a.dkw[r * a.lddw + j] = (float)s;
            if (j >= 1) s += dcdf[wv][j];
        }
    }
}

}  // namespace

extern "C" int nerf_prop_cdf(const float* w, int64_t ld_w, int64_t n_rays, int32_t K, float* cdf, int64_t ld_cdf,
                             void* stream) {
    NERF_REQUIRE(n_rays >= 0 && K >= 1 && ld_w >= K && ld_cdf >= K + 1);
    if (n_rays == 0) return NERF_OK;
    NERF_REQUIRE(w && cdf);
    hipLaunchKernelGGL(prop_cdf_kernel, dim3((unsigned)((n_rays + PRAYS - 1) / PRAYS)), dim3(PW * PRAYS), 0,
                       as_stream(stream), w, ld_w, n_rays, K, cdf, ld_cdf);
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}

extern "C" int nerf_prop_sample(const float* vals, int64_t ld_vals, const float* cdf, int64_t ld_cdf, int64_t n_rays,
                                int32_t K, int32_t n, int32_t stratified, uint64_t seed, uint64_t counter,
                                int32_t transform, float near_plane, float far_plane, float* s_out, float* t_out,
                                int64_t ld_out, void* stream) {
    NERF_REQUIRE(n_rays >= 0 && K >= 1 && K + 1 <= NERF_PROP_MAX_EDGES && n >= 1 && ld_vals >= K + 1 &&
                 ld_cdf >= K + 1 && ld_out >= n + 1 && (transform == 0 || transform == 1));
    NERF_REQUIRE(near_plane > 0.0f || transform == 0);
    if (n_rays == 0) return NERF_OK;
    NERF_REQUIRE(vals && cdf && s_out && t_out);
    SampleArgs a{vals, ld_vals, cdf, ld_cdf, n_rays, K, n, stratified, seed, counter, transform, near_plane,
                 far_plane, s_out, t_out, ld_out};
    hipLaunchKernelGGL(prop_sample_kernel, dim3((unsigned)((n_rays + PRAYS - 1) / PRAYS)), dim3(PW * PRAYS), 0,
                       as_stream(stream), a);
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}

extern "C" int nerf_prop_loss(const float* q_vals, const float* q_cdf, int64_t ld_q, const float* k_vals,
                              const float* k_cdf, int64_t ld_k, int64_t n_rays, int32_t n, int32_t K, float eps,
                              float* loss_ray, float grad_scale, float* grad_k_w, int64_t ld_gw, void* stream) {
    NERF_REQUIRE(n_rays >= 0 && n >= 1 && K >= 1 && n + 1 <= NERF_PROP_MAX_EDGES && K + 1 <= NERF_PROP_MAX_EDGES &&
                 ld_q >= n + 1 && ld_k >= K + 1);
    if (n_rays == 0) return NERF_OK;
    NERF_REQUIRE(q_vals && q_cdf && k_vals && k_cdf && (loss_ray || grad_k_w));
    if (grad_k_w) NERF_REQUIRE(ld_gw >= K);
    LossArgs a{q_vals, q_cdf, ld_q, k_vals, k_cdf, ld_k, n_rays, n, K, eps, loss_ray, grad_scale, grad_k_w, ld_gw};
    hipLaunchKernelGGL(prop_loss_kernel, dim3((unsigned)((n_rays + PRAYS - 1) / PRAYS)), dim3(PW * PRAYS), 0,
                       as_stream(stream), a);
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}
