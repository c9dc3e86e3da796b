// On-device ray-batch feed: the training batch the reference's
// ImagePoseDataset + DataLoader assemble on the host, built per step in one launch from
// HBM-resident images and camera matrices.
//
// References:
//   _get_directions_meshgrid   barf/dataset.py:417-451  (pixel-centre directions, camera space)
//   _meshgrid_to_world         barf/dataset.py:453-481  (R_c2w @ d, origins = c2w[:3, 3])
//   _apply_noise               barf/dataset.py:512-557  (d_noisy = R_noise @ d, o_noisy = o + t_noise)
//   __getitem__                barf/dataset.py:613-637  (index -> image index, pixel index)
//   get_blurred_pixel_colors   barf/data_module.py:276-367 (blur-level selection / interpolation)
//
// One thread per ray.  The reference materialises every ray's origin and direction for the
// whole dataset (2 x 100 x 640 000 x 12 B at 800^2) and gathers from them; here the direction
// is recomputed from the pixel coordinates (a few flops) so a batch reads only its colours
// (n_sigma x 12 B per ray) and the per-image matrices (L2-resident).  Arithmetic follows the
// reference's operation order with contraction off: linspace as torch computes it (both ends),
// negate / divide by the focal length, the 2-norm, then the two 3 x 3 matrix-vector products.
#include "common.h"

using namespace nerf;

namespace {

struct RayBatchArgs {
    const int64_t* indices; int64_t B; int H, W; float focal;
    const float* c2w; const float* noise_rot; const float* noise_trans;
    const float* images; int n_sigma; int n_img;
    int blur_mode, blur_lo, blur_hi; float coef_lo, coef_hi;
    float* o_raw; float* o_noisy; float* d_raw; float* d_noisy;
    float* colors_raw; float* colors_pair; int64_t* img_idx; int32_t* status;
};

__device__ __forceinline__ void matvec3(const float* __restrict__ R, int ld, float x, float y, float z, float* out) {
#pragma clang fp contract(off)
    // torch's CPU matmul of a 3 x 3 by a 3-vector: k = 0, 1, 2 summed in order
    for (int i = 0; i < 3; ++i) out[i] = (R[i * ld + 0] * x + R[i * ld + 1] * y) + R[i * ld + 2] * z;
}

__global__ __launch_bounds__(256) void ray_batch_kernel(RayBatchArgs a) {
#pragma clang fp contract(off)
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= a.B) return;
    const int64_t HW = (int64_t)a.H * a.W;
    int64_t idx = a.indices[r];
    if (idx < 0 || idx >= HW * a.n_img) {
        // an out-of-range index is reported, and the ray reads pixel 0 so nothing faults
        atomicOr(a.status, 1);
        idx = 0;
    }
    const int n = (int)(idx / HW);
    const int64_t p = idx - (int64_t)n * HW;
    const int row = (int)(p / a.W), col = (int)(p - (int64_t)row * a.W);

    // camera-space direction: (x, y, -1) / |(x, y, -1)|, x and y from torch.linspace
    const float x = linspace_at(-(float)(a.W - 1) / 2.0f, (float)(a.W - 1) / 2.0f, a.W, col) / a.focal;
    const float y = (-linspace_at(-(float)(a.H - 1) / 2.0f, (float)(a.H - 1) / 2.0f, a.H, row)) / a.focal;
    const float nrm = sqrtf((x * x + y * y) + 1.0f);
    const float cx = x / nrm, cy = y / nrm, cz = -1.0f / nrm;

    const float* M = a.c2w + (int64_t)n * 16;
    float d[3];
    matvec3(M, 4, cx, cy, cz, d);
    const float o[3] = {M[3], M[7], M[11]};
    for (int i = 0; i < 3; ++i) {
        a.d_raw[r * 3 + i] = d[i];
        a.o_raw[r * 3 + i] = o[i];
    }
    if (a.d_noisy) {
        float dn[3] = {d[0], d[1], d[2]};
        if (a.noise_rot) matvec3(a.noise_rot + (int64_t)n * 9, 3, d[0], d[1], d[2], dn);
        for (int i = 0; i < 3; ++i) {
            a.d_noisy[r * 3 + i] = dn[i];
            a.o_noisy[r * 3 + i] = a.noise_trans ? o[i] + a.noise_trans[n * 3 + i] : o[i];
        }
    }
    if (a.img_idx) a.img_idx[r] = n;

    const float* c = a.images + idx * a.n_sigma * 3;
    if (a.colors_raw)
        for (int k = 0; k < a.n_sigma * 3; ++k) a.colors_raw[r * a.n_sigma * 3 + k] = c[k];
    if (a.colors_pair) {
        const float* last = c + (a.n_sigma - 1) * 3;
        for (int i = 0; i < 3; ++i) {
            float v;
            if (a.blur_mode == 1) v = last[i];                 // sigma <= 0.25: no blur
            else if (a.blur_mode == 2) v = c[i];               // sigma >= max: the most blurred level
            else v = c[a.blur_lo * 3 + i] * a.coef_lo + c[a.blur_hi * 3 + i] * a.coef_hi;
            a.colors_pair[r * 6 + i] = v;
            a.colors_pair[r * 6 + 3 + i] = last[i];
        }
    }
}

}  // namespace

extern "C" int nerf_ray_batch(const int64_t* indices, int64_t B, int32_t H, int32_t W, float focal,
                              const float* c2w, const float* noise_rot, const float* noise_trans, int32_t n_img,
                              const float* images, int32_t n_sigma, int32_t blur_mode, int32_t blur_lo,
                              int32_t blur_hi, float coef_lo, float coef_hi, float* o_raw, float* o_noisy,
                              float* d_raw, float* d_noisy, float* colors_raw, float* colors_pair, int64_t* img_idx,
                              int32_t* status, void* stream) {
    NERF_REQUIRE(B >= 0 && H >= 1 && W >= 1 && n_img >= 1 && n_sigma >= 1 && focal != 0.0f);
    NERF_REQUIRE((int64_t)H * W * n_img < ((int64_t)1 << 62) / (3 * n_sigma));
    if (B == 0) return NERF_OK;
    NERF_REQUIRE(indices && c2w && images && o_raw && d_raw && status);
    NERF_REQUIRE((o_noisy == nullptr) == (d_noisy == nullptr));
    NERF_REQUIRE(blur_mode >= 0 && blur_mode <= 3);
    if (colors_pair) NERF_REQUIRE(blur_mode != 0);
    if (blur_mode == 3) NERF_REQUIRE(blur_lo >= 0 && blur_lo < n_sigma && blur_hi >= 0 && blur_hi < n_sigma);
    RayBatchArgs a{indices, B, H, W, focal, c2w, noise_rot, noise_trans, images, n_sigma, n_img,
                   blur_mode, blur_lo, blur_hi, coef_lo, coef_hi, o_raw, o_noisy, d_raw, d_noisy,
                   colors_raw, colors_pair, img_idx, status};
    hipLaunchKernelGGL(ray_batch_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, as_stream(stream), a);
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}
