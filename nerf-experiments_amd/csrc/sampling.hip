// Ray-interval sampling: stratified/equidistant coarse t (a6) and the
// pdf-weighted fine resample (a5).
//
// References:
//   _sample_t_stratified_uniform  barf/model_interpolation.py:135-180
//   _get_intervals                barf/model_interpolation.py:114-132
//   _sample_t_pdf_weighted        barf/model_interpolation.py:193-277 (mode 0)
//   _sample_t_fine                naive-to-vanilla/model_interpolation.py:128-169 (mode 1)
//   _sample_t_fine(linspace=False) nerf-siren/model.py:106-112 (mode 2; the multinomial branch
//                                  SURVEY §8(a) a5 names at 3d-ingp/model.py:306-312)
//
// Resample design: one wavefront per ray, lane i = coarse bin i (n_bins <= 64).
// The integer allocation (floor / largest remainder / +1) is done in registers,
// the ranking of fractional parts uses 64 scalar broadcasts (readlane), the
// exclusive scan of counts is a wave shuffle scan, and each fine sample j is
// owned by lane j % 64, which walks the 64 bins' [c_i, c_i+1) ranges from
// scalar registers — the reference's masked accumulation, including its
// behaviour on degenerate counts — and stores coalesced.  A batch-wide fallback (the reference's "pdf sampling
// failed" branch) runs in a second tiny kernel that reads the device status
// word, so there is never a host synchronisation.
#include "common.h"

using namespace nerf;

namespace {

__global__ __launch_bounds__(256) void sample_uniform_kernel(int64_t n_rays, int S, float near_, float far_,
                                                             int stratified, float offset_size,
                                                             uint64_t seed, uint64_t counter,
                                                             float* __restrict__ t_start,
                                                             float* __restrict__ t_end) {
#pragma clang fp contract(off)
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = n_rays * S;
    if (idx >= total) return;
    const int64_t ray = idx / S;
    const int s = (int)(idx - ray * S);
    const float interval = (far_ - near_) / (float)S;
    auto t_at = [&](int ss) -> float {
        float t = linspace_at(near_, far_ - interval, S, ss);
        if (stratified) t = t + philox_uniform(seed, counter, (uint64_t)(ray * S + ss)) * interval;
        if (offset_size != 0.0f) {
            // one uniform per ray, drawn from a disjoint counter stream
            float u = philox_uniform(seed, counter ^ 0x8000000000000000ull, (uint64_t)ray);
            t = t + (u * interval) * offset_size;
        }
        return t;
    };
    const float t0 = t_at(s);
    t_start[idx] = t0;
    t_end[idx] = (s + 1 < S) ? t_at(s + 1) : far_;
}

struct ResampleArgs {
    const float* t_coarse; const float* w; const float* dist;
    int64_t n_rays; int K; int N; int mode;
    float* t_start; float* t_end; int32_t* status;
};

__device__ __forceinline__ float bcast(float v, int lane) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), lane));
}

// one wave per ray, 4 rays per 256-thread block
__global__ __launch_bounds__(256) void resample_kernel(ResampleArgs a) {
#pragma clang fp contract(off)
    const int lane = lane_id();
    const int wid = threadIdx.x >> 6;
    const int64_t ray = (int64_t)blockIdx.x * 4 + wid;
    if (ray >= a.n_rays) return;
    const int K = a.K;
    const bool active = lane < K;
    const int64_t rb = ray * K;
    const float wi = active ? a.w[rb + lane] : 0.0f;
    const float tci = active ? a.t_coarse[rb + lane] : 0.0f;
    const float di = active ? a.dist[rb + lane] : 0.0f;
    const int nfine = a.N - K;

    float cnt;      // fine_samples: a float holding an integer, as in the reference
    bool ok = true;
    if (a.mode == 0) {
        // weights / weights.sum(dim=1): the sum is formed in fp64 and rounded once
        const float ssum = (float)wave_sum((double)wi);
        const float p = wi / ssum;
        const float raw = p * (float)nfine;
        const float fl = floorf(raw);
        const float err = raw - fl;
        const float flsum = (float)wave_sum((double)(active ? fl : 0.0f));
        const float excess = (float)nfine - flsum;
        // rank = position of err in a stable ascending argsort (argsort().argsort())
        int rank = 0;
        bool finite_all = true;
        for (int k = 0; k < 64; ++k) {
            if (k >= K) break;
            const float ek = bcast(err, k);
            if (!isfinite(ek)) finite_all = false;
            rank += (ek < err || (ek == err && k < lane)) ? 1 : 0;
        }
        const bool add = (float)rank >= ((float)K - excess);
        cnt = fl + (add ? 1.0f : 0.0f) + 1.0f;
        ok = finite_all && isfinite(cnt) && cnt >= 0.0f;
    } else {
        // round-half-even(w * n_fine), remainder to the first argmax bin (no renormalisation)
        float f = active ? rintf(wi * (float)nfine) : 0.0f;
        const float fsum = (float)wave_sum((double)f);
        float best = -INFINITY;
        int besti = 0;
        for (int k = 0; k < 64; ++k) {
            if (k >= K) break;
            const float fk = bcast(f, k);
            if (fk > best || (isnan(fk) && !isnan(best))) { best = fk; besti = k; }
        }
        if (lane == besti) f = f + ((float)nfine - fsum);
        cnt = f + 1.0f;
    }
    if (!active) cnt = 0.0f;
    // c_i = exclusive prefix of counts (exact: integers), c_{i+1} = inclusive
    const double cincl = wave_inclusive_scan((double)cnt);
    const float c_hi = (float)cincl;
    const float c_lo = (float)(cincl - (double)cnt);
    if (a.mode == 0) {
        const double total = __shfl(cincl, 63, NERF_WAVE);
        const bool ray_ok = __all(ok || !active) && total == (double)a.N;
        if (!ray_ok) {
            if (lane == 0) atomicOr(a.status, 1);
            return;  // the batch fallback rewrites every ray
        }
    }
    // t_j = sum over bins i (in order) covering j of  t_coarse_i  +  ((j - c_i) * dist_i) / n_i
    const int64_t ob = ray * a.N;
    for (int j = lane; j < a.N; j += NERF_WAVE) {
        const float jf = (float)j;
        float t = 0.0f;
        for (int i = 0; i < 64; ++i) {
            if (i >= K) break;
            const float lo = bcast(c_lo, i), hi = bcast(c_hi, i);
            const float m = (jf >= lo && jf < hi) ? 1.0f : 0.0f;
            t = t + bcast(tci, i) * m;
            t = t + (((jf - lo) * m) * bcast(di, i)) / bcast(cnt, i);
        }
        a.t_start[ob + j] = t;
    }
}

// Mode 2, torch.multinomial(weights, n_fine, replacement=True) -> t_coarse.gather + U * dist.gather
// -> cat with t_coarse -> sort (nerf-siren/model.py:106-112): one wave per ray.  Bin of fine
// sample j: the inverse of the fp64 cumulative weights at u_j * total (u_j = Philox(seed, counter,
// ray * n_fine + j)); offset U = Philox(seed, counter ^ 2^62, same index).  The K coarse and
// n_fine fine values are sorted in LDS by rank counting (ascending, ties by index: a stable
// sort, deterministic).  A row torch.multinomial rejects (a negative or non-finite weight, or a
// zero sum) draws its bins uniformly and sets bit 1 (value 2) of the status word.
constexpr int kMnMax = 512;              // K + n_fine per ray
__device__ __forceinline__ double bcast_d(double v, int lane) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, lane);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), lane);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

__global__ __launch_bounds__(256) void resample_multinomial_kernel(ResampleArgs a, uint64_t seed, uint64_t counter) {
#pragma clang fp contract(off)
    __shared__ float sv[4][kMnMax];      // the ray's K coarse then n_fine fine values
    __shared__ float stc[4][64], sdi[4][64];
    const int lane = lane_id();
    const int wid = threadIdx.x >> 6;
    const int64_t ray = (int64_t)blockIdx.x * 4 + wid;
    if (ray >= a.n_rays) return;        // wave-uniform: only wave-local synchronisation below
    const int K = a.K, N = a.N, nfine = N - K;
    const bool active = lane < K;
    const int64_t rb = ray * K;
    const float wi = active ? a.w[rb + lane] : 0.0f;
    const float tci = active ? a.t_coarse[rb + lane] : 0.0f;
    const float di = active ? a.dist[rb + lane] : 0.0f;
    const bool wok = !active || (isfinite(wi) && wi >= 0.0f);
    const double incl = wave_inclusive_scan((double)wi);
    const double total = __shfl(incl, NERF_WAVE - 1, NERF_WAVE);
    const bool valid = __all(wok) && isfinite(total) && total > 0.0;
    if (!valid && lane == 0) atomicOr(a.status, 2);
    const double cum = valid ? incl : (double)(lane + 1);
    const double tot = valid ? total : (double)K;
    if (active) {
        sv[wid][lane] = tci;
        stc[wid][lane] = tci;
        sdi[wid][lane] = di;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    for (int j = lane; j < nfine; j += NERF_WAVE) {
        const uint64_t id = (uint64_t)ray * (uint64_t)nfine + (uint64_t)j;
        const double target = (double)philox_uniform(seed, counter, id) * tot;
        int bin = 0;
        for (int i = 0; i < 64; ++i) {
            if (i >= K) break;
            bin += bcast_d(cum, i) <= target ? 1 : 0;
        }
        bin = bin < K ? bin : K - 1;
        const float u2 = philox_uniform(seed, counter ^ 0x4000000000000000ull, id);
        sv[wid][K + j] = stc[wid][bin] + u2 * sdi[wid][bin];
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const int64_t ob = ray * N;
    for (int e = lane; e < N; e += NERF_WAVE) {
        const float ve = sv[wid][e];
        int rank = 0;
        for (int f = 0; f < N; ++f) {
            const float vf = sv[wid][f];
            rank += (vf < ve || (vf == ve && f < e)) ? 1 : 0;
        }
        a.t_start[ob + rank] = ve;
    }
}

// t_end = next t_start, far for the last sample; the batch fallback overwrites
// everything when the status word is set.
__global__ __launch_bounds__(256) void resample_finish_kernel(int64_t n_rays, int N, float near_, float far_,
                                                              uint64_t seed, uint64_t counter,
                                                              const int32_t* __restrict__ status,
                                                              float* __restrict__ t_start,
                                                              float* __restrict__ t_end) {
#pragma clang fp contract(off)
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = n_rays * N;
    if (idx >= total) return;
    const int64_t ray = idx / N;
    const int s = (int)(idx - ray * N);
    if (*status & 1) {
        // _sample_t_stratified_uniform(batch, n_samples, "equidistant", offset=-1)
        const float interval = (far_ - near_) / (float)N;
        const float u = philox_uniform(seed, counter ^ 0x8000000000000000ull, (uint64_t)ray);
        auto t_at = [&](int ss) -> float {
            float t = linspace_at(near_, far_ - interval, N, ss);
            return t + (u * interval) * -1.0f;
        };
        t_start[idx] = t_at(s);
        t_end[idx] = (s + 1 < N) ? t_at(s + 1) : far_;
    } else {
        t_end[idx] = (s + 1 < N) ? t_start[idx + 1] : far_;
    }
}

}  // namespace

extern "C" int nerf_sample_uniform(int64_t n_rays, int32_t samples_per_ray, float near_, float far_,
                                   int32_t stratified, float offset_size, uint64_t seed, uint64_t counter,
                                   float* t_start, float* t_end, void* stream) {
    NERF_REQUIRE(n_rays >= 0 && samples_per_ray >= 1);
    if (n_rays == 0) return NERF_OK;
    NERF_REQUIRE(t_start && t_end);
    const int64_t total = n_rays * samples_per_ray;
    dim3 grid((unsigned)((total + 255) / 256)), block(256);
    hipLaunchKernelGGL(sample_uniform_kernel, grid, block, 0, as_stream(stream), n_rays, samples_per_ray,
                       near_, far_, stratified, offset_size, seed, counter, t_start, t_end);
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}

extern "C" int nerf_resample_pdf(const float* t_coarse, const float* weights, const float* dist_coarse,
                                 int64_t n_rays, int32_t n_bins, int32_t n_samples, int32_t mode, float near_,
                                 float far_, uint64_t seed, uint64_t counter, float* t_start, float* t_end,
                                 int32_t* status, void* stream) {
    NERF_REQUIRE(n_rays >= 0);
    if (n_rays == 0) return NERF_OK;
    NERF_REQUIRE(t_coarse && weights && dist_coarse && t_start && t_end && status);
    NERF_REQUIRE(n_bins >= 1 && n_samples >= n_bins && (mode == 0 || mode == 1 || mode == 2));
    if (n_bins > 64 || (mode == 2 && n_samples > kMnMax)) return NERF_ERR_UNSUPPORTED;
    ResampleArgs a{t_coarse, weights, dist_coarse, n_rays, n_bins, n_samples, mode, t_start, t_end, status};
    hipStream_t st = as_stream(stream);
    dim3 grid((unsigned)((n_rays + 3) / 4)), block(256);
    if (mode == 2)
        hipLaunchKernelGGL(resample_multinomial_kernel, grid, block, 0, st, a, seed, counter);
    else
        hipLaunchKernelGGL(resample_kernel, grid, block, 0, st, a);
    NERF_CHECK_LAUNCH();
    const int64_t total = n_rays * n_samples;
    dim3 grid2((unsigned)((total + 255) / 256));
    hipLaunchKernelGGL(resample_finish_kernel, grid2, block, 0, st, n_rays, n_samples, near_, far_, seed, counter,
                       status, t_start, t_end);
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}
