// Gaussian activation with a learnable per-channel inverse standard deviation (GARF).
//
// Reference: garf/gaussian.py:8-31 (GaussActivation), :34-63 (GaussAct); identical copy in
// barf/gaussian.py.  With v_n = s_n^2 + 1e-6 (GaussAct.forward, :63):
//   forward   y      = exp((-(z * z)) * v)
//   backward  ge     = g * exp((-(z * z)) * v)
//             dz     = (((-ge) * 2) * z) * v
//             dv_n   = sum_m (-ge) * z^2          (autograd's reduction of the broadcast v)
//             ds_n   = dv_n * (2 * s_n)           (backward of s ** 2)
//
// Layout: z, y, g, dz are [M][N] row-major with their own row strides (the MLP's padded
// activation buffers).  Both kernels map 64 consecutive lanes to 64 consecutive columns of
// one row, so every load/store is a coalesced 256-byte wave access; the backward keeps one
// fp64 column partial per thread over a slab of rows, reduces the 4 row groups of a block
// through LDS and writes one partial row per slab; nerf::gauss_reduce then sums the slabs in
// a fixed order (deterministic, no atomics).  The same reduction serves the fused
// linear + Gaussian-activation epilogue of linear_x3.hip (nerf_linear_gauss_x3).
#include "common.h"

using namespace nerf;

namespace {

constexpr int kCols = 64;     // columns per block
constexpr int kRowGroups = 4; // row groups per block (blockDim = 256)

__device__ __forceinline__ float inv_var(const float* s, int n) {
#pragma clang fp contract(off)
    const float sv = s[n];
    return sv * sv + 1e-6f;
}

__global__ __launch_bounds__(256) void gauss_fwd_kernel(const float* __restrict__ z, int64_t ldz,
                                                        const float* __restrict__ s, int64_t M, int N,
                                                        float* __restrict__ y, int64_t ldy, int64_t rows_per_block) {
#pragma clang fp contract(off)
    const int n = blockIdx.y * kCols + (threadIdx.x & (kCols - 1));
    if (n >= N) return;
    const float v = inv_var(s, n);
    const int64_t m0 = (int64_t)blockIdx.x * rows_per_block;
    const int64_t m1 = m0 + rows_per_block < M ? m0 + rows_per_block : M;
    for (int64_t m = m0 + (threadIdx.x >> 6); m < m1; m += kRowGroups) {
        const float zz = z[m * ldz + n];
        y[m * ldy + n] = expf((-(zz * zz)) * v);
    }
}

// grad_z may alias grad_y (in-place): each element is read and then written by one thread.
__global__ __launch_bounds__(256) void gauss_bwd_kernel(const float* g, int64_t ldg,
                                                        const float* __restrict__ z, int64_t ldz,
                                                        const float* __restrict__ s, int64_t M, int N,
                                                        float* dz, int64_t lddz, int64_t rows_per_block,
                                                        double* __restrict__ partial) {
#pragma clang fp contract(off)
    __shared__ double red[kRowGroups][kCols];
    const int c = threadIdx.x & (kCols - 1);
    const int rg = threadIdx.x >> 6;
    const int n = blockIdx.y * kCols + c;
    double acc = 0.0;
    if (n < N) {
        const float v = inv_var(s, n);
        const int64_t m0 = (int64_t)blockIdx.x * rows_per_block;
        const int64_t m1 = m0 + rows_per_block < M ? m0 + rows_per_block : M;
        for (int64_t m = m0 + rg; m < m1; m += kRowGroups) {
            const float zz = z[m * ldz + n];
            const float z2 = zz * zz;
            const float ge = g[m * ldg + n] * expf((-z2) * v);
            dz[m * lddz + n] = (((-ge) * 2.0f) * zz) * v;
            acc += (double)((-ge) * z2);
        }
    }
    red[rg][c] = acc;
    __syncthreads();
    if (rg == 0 && n < N) {
        const double t = ((red[0][c] + red[1][c]) + red[2][c]) + red[3][c];
        partial[(int64_t)blockIdx.x * N + n] = t;
    }
}

// Column sums of the slab partials in two fixed-order levels: block (column group, chunk) sums
// its chunk's slabs (4 row groups, each a strided run, combined in order), then one thread per
// column sums the chunks in order.
constexpr int kMaxChunks = 64;

__global__ __launch_bounds__(256) void gauss_reduce_chunks_kernel(const double* __restrict__ partial, int64_t slabs,
                                                                  int N, int64_t chunk, double* __restrict__ out2) {
    __shared__ double red[kRowGroups][kCols];
    const int c = threadIdx.x & (kCols - 1);
    const int rg = threadIdx.x >> 6;
    const int n = blockIdx.x * kCols + c;
    const int64_t i0 = (int64_t)blockIdx.y * chunk;
    const int64_t i1 = i0 + chunk < slabs ? i0 + chunk : slabs;
    double acc = 0.0;
    if (n < N)
        for (int64_t i = i0 + rg; i < i1; i += kRowGroups) acc += partial[i * N + n];
    red[rg][c] = acc;
    __syncthreads();
    if (rg == 0 && n < N) out2[(int64_t)blockIdx.y * N + n] = ((red[0][c] + red[1][c]) + red[2][c]) + red[3][c];
}

__global__ __launch_bounds__(256) void gauss_reduce_final_kernel(const double* __restrict__ out2, int chunks, int N,
                                                                 const float* __restrict__ s, float* __restrict__ ds,
                                                                 int accumulate) {
#pragma clang fp contract(off)
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    double t = 0.0;
    for (int i = 0; i < chunks; ++i) t += out2[(int64_t)i * N + n];
    const float sv = s[n];
    const float r = ((float)t) * (2.0f * sv);
    ds[n] = accumulate ? ds[n] + r : r;
}

int64_t slabs_for(int64_t M) {
    // ~512 rows per slab, at most 1024 slabs (the partials stay tiny: slabs * N * 8 bytes)
    int64_t slabs = (M + 511) / 512;
    if (slabs > 1024) slabs = 1024;
    if (slabs < 1) slabs = 1;
    return slabs;
}

}  // namespace

size_t nerf::gauss_reduce_scratch(int N) { return (size_t)kMaxChunks * (size_t)(N > 0 ? N : 0) * sizeof(double); }

int nerf::gauss_reduce(const double* partial, int64_t slabs, int N, const float* s, float* ds, int accumulate,
                       double* scratch, hipStream_t st) {
    int64_t chunks = (slabs + 63) / 64;
    chunks = chunks < 1 ? 1 : (chunks > kMaxChunks ? kMaxChunks : chunks);
    const int64_t chunk = (slabs + chunks - 1) / chunks;
    chunks = (slabs + chunk - 1) / chunk;
    hipLaunchKernelGGL(gauss_reduce_chunks_kernel, dim3((unsigned)((N + kCols - 1) / kCols), (unsigned)chunks),
                       dim3(256), 0, st, partial, slabs, N, chunk, scratch);
    if (hipGetLastError() != hipSuccess) return NERF_ERR_LAUNCH;
    hipLaunchKernelGGL(gauss_reduce_final_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, st, scratch,
                       (int)chunks, N, s, ds, accumulate);
    if (hipGetLastError() != hipSuccess) return NERF_ERR_LAUNCH;
    return NERF_OK;
}

extern "C" size_t nerf_gauss_act_workspace(int64_t M, int32_t N) {
    if (M <= 0 || N <= 0) return 0;
    return (size_t)slabs_for(M) * (size_t)N * sizeof(double) + nerf::gauss_reduce_scratch(N);
}

extern "C" int nerf_gauss_act_fwd(const float* z, int64_t ld_z, const float* inv_std, int64_t M, int32_t N, float* y,
                                  int64_t ld_y, void* stream) {
    NERF_REQUIRE(M >= 0 && N >= 0);
    if (M == 0 || N == 0) return NERF_OK;
    NERF_REQUIRE(z && inv_std && y && ld_z >= N && ld_y >= N);
    const int64_t slabs = slabs_for(M);
    const int64_t rows = (M + slabs - 1) / slabs;
    dim3 grid((unsigned)slabs, (unsigned)((N + kCols - 1) / kCols));
    hipLaunchKernelGGL(gauss_fwd_kernel, grid, dim3(256), 0, as_stream(stream), z, ld_z, inv_std, M, N, y, ld_y,
                       rows);
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}

extern "C" int nerf_gauss_act_bwd(const float* grad_y, int64_t ld_g, const float* z, int64_t ld_z,
                                  const float* inv_std, int64_t M, int32_t N, float* grad_z, int64_t ld_dz,
                                  float* grad_inv_std, int32_t accumulate, void* workspace, size_t workspace_bytes,
                                  void* stream) {
    NERF_REQUIRE(M >= 0 && N >= 0);
    if (N == 0) return NERF_OK;
    NERF_REQUIRE(inv_std && grad_inv_std);
    hipStream_t st = as_stream(stream);
    if (M == 0) {
        if (!accumulate) {
            if (hipMemsetAsync(grad_inv_std, 0, (size_t)N * sizeof(float), st) != hipSuccess) return NERF_ERR_LAUNCH;
        }
        return NERF_OK;
    }
    NERF_REQUIRE(grad_y && z && grad_z && ld_g >= N && ld_z >= N && ld_dz >= N);
    if (!workspace || workspace_bytes < nerf_gauss_act_workspace(M, N)) return NERF_ERR_WORKSPACE;
    const int64_t slabs = slabs_for(M);
    const int64_t rows = (M + slabs - 1) / slabs;
    double* partial = reinterpret_cast<double*>(workspace);
    dim3 grid((unsigned)slabs, (unsigned)((N + kCols - 1) / kCols));
    hipLaunchKernelGGL(gauss_bwd_kernel, grid, dim3(256), 0, st, grad_y, ld_g, z, ld_z, inv_std, M, N, grad_z, ld_dz,
                       rows, partial);
    NERF_CHECK_LAUNCH();
    return nerf::gauss_reduce(partial, slabs, N, inv_std, grad_inv_std, accumulate, partial + slabs * N, st);
}
