// BARF's per-image camera refinement in front of the ray path:
// CameraExtrinsics.forward (barf/model_camera_extrinsics.py:61-85) — new_o = o + translation[i] /
// MAGIC, new_d = R_i d with R_i = matrix_exp([rotation[i]]_x) (so3_to_SO3, :23-43) — and its
// backward to the so3 / translation parameters.  Contract in include/nerf_amd.h (nerf_pose_rays_*).
//
// The reference exponentiates all n_images skew matrices with torch.matrix_exp, gathers them per
// ray, multiplies R @ d as a batched GEMM, and on the way back index_adds the per-ray gradients
// and runs matrix_exp's block-matrix backward: a dozen launches per step.  Here:
//  * forward: one thread per ray; R from Rodrigues' formula in fp64 (R = I + A K + B K^2,
//    A = sin t / t, B = 2 sin^2(t/2) / t^2, Taylor series below t^2 = 1e-4), rounded to fp32 once;
//  * backward: one workgroup per image gathers its rays' contributions in a fixed order (thread j
//    takes rays j, j + 256, ...; a fixed-shape LDS tree) in fp64 — dL/dt = sum g_o (+ g_t) / MAGIC,
//    G = dL/dR = sum g_d d^T (+ g_R) — then maps G through the analytic derivative of Rodrigues'
//    formula:  dR/dw_m = (A'/t) w_m K + A E_m + (B'/t) w_m K^2 + B (w e_m^T + e_m w^T - 2 w_m I),
//    E_m = [e_m]_x.  Deterministic, no atomics; images without rays get zero gradients, as the
//    reference's dense index_add does.
// A ray whose image index is out of range gets NaN outputs and contributes no gradient (the
// reference raises an IndexError; a device-side check cannot without a host sync).
#include "common.h"

namespace {

constexpr int PT = 256;

struct So3 {
    double A, B, dA, dB;   // A, B of Rodrigues' formula and A'(t)/t, B'(t)/t
};

__device__ __forceinline__ So3 so3_coeffs(double th2) {
    So3 c;
    if (th2 < 1e-4) {
        c.A = 1.0 - th2 / 6.0 + th2 * th2 / 120.0;
        c.B = 0.5 - th2 / 24.0 + th2 * th2 / 720.0;
        c.dA = -1.0 / 3.0 + th2 / 30.0 - th2 * th2 / 840.0;
        c.dB = -1.0 / 12.0 + th2 / 180.0 - th2 * th2 / 6720.0;
    } else {
        const double th = sqrt(th2);
        double s, co;
        sincos(th, &s, &co);
        const double sh = sin(0.5 * th);
        c.A = s / th;
        c.B = 2.0 * sh * sh / th2;
        c.dA = (th * co - s) / (th2 * th);
        c.dB = (th * s - 4.0 * sh * sh) / (th2 * th2);
    }
    return c;
}

// R (row-major) = exp([w]_x) = I + A K + B (w w^T - t^2 I)
__device__ __forceinline__ void so3_to_SO3(const double w[3], const So3& c, double R[9]) {
    const double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    const double K[9] = {0.0, -w[2], w[1], w[2], 0.0, -w[0], -w[1], w[0], 0.0};
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int k = 0; k < 3; ++k)
            R[3 * r + k] = (r == k ? 1.0 : 0.0) + c.A * K[3 * r + k] + c.B * (w[r] * w[k] - (r == k ? th2 : 0.0));
}

__global__ __launch_bounds__(PT) void pose_rays_fwd_kernel(const float* __restrict__ rotation,
                                                           const float* __restrict__ translation, int n_images,
                                                           const int64_t* __restrict__ img_idx,
                                                           const float* __restrict__ o, const float* __restrict__ d,
                                                           int64_t n_rays, float magic, float* __restrict__ new_o,
                                                           float* __restrict__ new_d, float* __restrict__ R_out,
                                                           float* __restrict__ t_out) {
#pragma clang fp contract(off)
    const int64_t j = (int64_t)blockIdx.x * PT + threadIdx.x;
    if (j >= n_rays) return;
    const int64_t i = img_idx[j];
    if (i < 0 || i >= n_images) {
        const float nan = __builtin_nanf("");
        for (int k = 0; k < 3; ++k) {
            new_o[3 * j + k] = nan;
            new_d[3 * j + k] = nan;
            if (t_out) t_out[3 * j + k] = nan;
        }
        if (R_out)
            for (int k = 0; k < 9; ++k) R_out[9 * j + k] = nan;
        return;
    }
    const double w[3] = {rotation[3 * i], rotation[3 * i + 1], rotation[3 * i + 2]};
    double Rd[9];
    so3_to_SO3(w, so3_coeffs(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]), Rd);
    float R[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) R[k] = (float)Rd[k];
    const float dx = d[3 * j], dy = d[3 * j + 1], dz = d[3 * j + 2];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        const float t = translation[3 * i + r] / magic;                 // translation[i] / MAGIC (fp32)
        new_o[3 * j + r] = o[3 * j + r] + t;
        // the fp32 matrix R times d, accumulated in fp64 and rounded once
        new_d[3 * j + r] = (float)((double)R[3 * r] * dx + (double)R[3 * r + 1] * dy + (double)R[3 * r + 2] * dz);
        if (t_out) t_out[3 * j + r] = t;
    }
    if (R_out)
#pragma unroll
        for (int k = 0; k < 9; ++k) R_out[9 * j + k] = R[k];
}

__global__ __launch_bounds__(PT) void pose_rays_bwd_kernel(const float* __restrict__ rotation, int n_images,
                                                           const int64_t* __restrict__ img_idx,
                                                           const int64_t* __restrict__ ray_order,
                                                           const int64_t* __restrict__ image_start,
                                                           const float* __restrict__ d, int64_t n_rays, float magic,
                                                           const float* __restrict__ g_o,
                                                           const float* __restrict__ g_d,
                                                           const float* __restrict__ g_R,
                                                           const float* __restrict__ g_t,
                                                           float* __restrict__ g_rotation,
                                                           float* __restrict__ g_translation) {
    __shared__ double red[12][PT];
    const int img = blockIdx.x;
    const int tid = threadIdx.x;
    double s[12];                                   // dL/dt (3), G = dL/dR row-major (9)
#pragma unroll
    for (int k = 0; k < 12; ++k) s[k] = 0.0;
    // bucketed (ray_order != NULL): this image's rays are ray_order[image_start[img] ..
    // image_start[img + 1]) in increasing index order; otherwise every ray's index is tested
    const int64_t lo = ray_order ? image_start[img] : 0, hi = ray_order ? image_start[img + 1] : n_rays;
    for (int64_t p = lo + tid; p < hi; p += PT) {
        const int64_t j = ray_order ? ray_order[p] : p;
        if (!ray_order && img_idx[j] != img) continue;
        const double gd[3] = {g_d ? g_d[3 * j] : 0.f, g_d ? g_d[3 * j + 1] : 0.f, g_d ? g_d[3 * j + 2] : 0.f};
        const double dd[3] = {d[3 * j], d[3 * j + 1], d[3 * j + 2]};
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            if (g_o) s[r] += g_o[3 * j + r];
            if (g_t) s[r] += g_t[3 * j + r];
#pragma unroll
            for (int k = 0; k < 3; ++k) s[3 + 3 * r + k] += gd[r] * dd[k] + (g_R ? (double)g_R[9 * j + 3 * r + k] : 0.0);
        }
    }
#pragma unroll
    for (int k = 0; k < 12; ++k) red[k][tid] = s[k];
    __syncthreads();
    for (int h = PT / 2; h > 0; h >>= 1) {
        if (tid < h)
#pragma unroll
            for (int k = 0; k < 12; ++k) red[k][tid] += red[k][tid + h];
        __syncthreads();
    }
    if (tid != 0) return;
    for (int r = 0; r < 3; ++r) g_translation[3 * img + r] = (float)(red[r][0] / (double)magic);
    double G[9];
    for (int k = 0; k < 9; ++k) G[k] = red[3 + k][0];
    const double w[3] = {rotation[3 * img], rotation[3 * img + 1], rotation[3 * img + 2]};
    const double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    const So3 c = so3_coeffs(th2);
    // <G, E_m> for E_0, E_1, E_2; <G, K> = sum_m w_m <G, E_m>; <G, K^2> = w^T G w - t^2 tr G
    const double ge[3] = {G[7] - G[5], G[2] - G[6], G[3] - G[1]};
    const double gk = w[0] * ge[0] + w[1] * ge[1] + w[2] * ge[2];
    const double trG = G[0] + G[4] + G[8];
    double wGw = 0.0;
    for (int r = 0; r < 3; ++r)
        for (int k = 0; k < 3; ++k) wGw += w[r] * G[3 * r + k] * w[k];
    const double gk2 = wGw - th2 * trG;
    for (int m = 0; m < 3; ++m) {
        double colm = 0.0, rowm = 0.0;              // sum_r G[r][m] w_r, sum_k G[m][k] w_k
        for (int r = 0; r < 3; ++r) {
            colm += G[3 * r + m] * w[r];
            rowm += G[3 * m + r] * w[r];
        }
        const double v = c.dA * w[m] * gk + c.A * ge[m] + c.dB * w[m] * gk2 + c.B * (colm + rowm - 2.0 * w[m] * trG);
        g_rotation[3 * img + m] = (float)v;
    }
}

}  // namespace

extern "C" int nerf_pose_rays_fwd(const float* rotation, const float* translation, int32_t n_images,
                                  const int64_t* img_idx, const float* o, const float* d, int64_t n_rays, float magic,
                                  float* new_o, float* new_d, float* R, float* t, void* stream) {
    NERF_REQUIRE(n_rays >= 0 && n_images >= 1 && magic != 0.0f);
    if (n_rays == 0) return NERF_OK;
    NERF_REQUIRE(rotation && translation && img_idx && o && d && new_o && new_d);
    const unsigned blocks = (unsigned)((n_rays + PT - 1) / PT);
    hipLaunchKernelGGL(pose_rays_fwd_kernel, dim3(blocks), dim3(PT), 0, as_stream(stream), rotation, translation,
                       n_images, img_idx, o, d, n_rays, magic, new_o, new_d, R, t);
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}

extern "C" int nerf_pose_rays_bwd(const float* rotation, int32_t n_images, const int64_t* img_idx, const float* d,
                                  int64_t n_rays, float magic, const float* g_new_o, const float* g_new_d,
                                  const float* g_R, const float* g_t, const int64_t* ray_order,
                                  const int64_t* image_start, float* g_rotation, float* g_translation, void* stream) {
    NERF_REQUIRE(n_rays >= 0 && n_images >= 1 && magic != 0.0f);
    NERF_REQUIRE(rotation && g_rotation && g_translation);
    NERF_REQUIRE(n_rays == 0 || (img_idx && d));
    NERF_REQUIRE((ray_order == nullptr) == (image_start == nullptr));
    hipLaunchKernelGGL(pose_rays_bwd_kernel, dim3(n_images), dim3(PT), 0, as_stream(stream), rotation, n_images,
                       img_idx, ray_order, image_start, d, n_rays, magic, g_new_o, g_new_d, g_R, g_t, g_rotation,
                       g_translation);
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}
