// Camera-pose alignment for BARF's validation / pose error:
// CameraCalibrationModel.kabsch_algorithm (barf/model_camera_calibration.py:69-156) and
// compute_pose_error (:340-345).  Contract in include/nerf_amd.h (nerf_kabsch).
//
// One workgroup (the clouds are the training cameras: ~100 points).  Every sum is a fixed-order
// fp64 block reduction (deterministic); the 3x3 SVD of H = from_c^T to_c is one-sided Jacobi in
// fp64 (H V = U S, columns orthogonalised until every pair is orthogonal to 1e-15), singular values
// in descending order as torch.linalg.svd returns them, so the reflection fix
// diag(1, 1, det(V U^T)) lands on the smallest one.  Outlier removal as the reference: distances
// of the aligned points, their 0.9 quantile with torch.quantile's linear interpolation (the sorted
// order by rank counting), keep d < q, solve again.
#include "common.h"

namespace {

constexpr int KT = 256;

// fixed-order block sum of one double per thread (result valid in every thread)
__device__ double block_sum(double v, double* red) {
    red[threadIdx.x] = v;
    __syncthreads();
    for (int s = KT / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    const double r = red[0];
    __syncthreads();
    return r;
}

__device__ double det3(const double* M) {
    return M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6]) + M[2] * (M[3] * M[7] - M[4] * M[6]);
}

// H (row-major) = U diag(S) V^T; R = V diag(1, 1, det(V) det(U)) U^T (row-major out)
__device__ void kabsch_rotation(const double* H, double* R) {
    double A[9], V[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    for (int i = 0; i < 9; ++i) A[i] = H[i];
    for (int sweep = 0; sweep < 60; ++sweep) {
        bool rotated = false;
        for (int pq = 0; pq < 3; ++pq) {
            const int p = pq == 2 ? 1 : 0, q = pq == 0 ? 1 : 2;
            double alpha = 0, beta = 0, gamma = 0;
            for (int i = 0; i < 3; ++i) {
                alpha += A[3 * i + p] * A[3 * i + p];
                beta += A[3 * i + q] * A[3 * i + q];
                gamma += A[3 * i + p] * A[3 * i + q];
            }
            if (fabs(gamma) <= 1e-15 * sqrt(alpha * beta) || gamma == 0.0) continue;
            rotated = true;
            const double zeta = (beta - alpha) / (2.0 * gamma);
            const double tt = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
            const double cs = 1.0 / sqrt(1.0 + tt * tt), sn = cs * tt;
            for (int i = 0; i < 3; ++i) {
                const double ap = A[3 * i + p], aq = A[3 * i + q];
                A[3 * i + p] = cs * ap - sn * aq;
                A[3 * i + q] = sn * ap + cs * aq;
                const double vp = V[3 * i + p], vq = V[3 * i + q];
                V[3 * i + p] = cs * vp - sn * vq;
                V[3 * i + q] = sn * vp + cs * vq;
            }
        }
        if (!rotated) break;
    }
    double S[3];
    int ord[3] = {0, 1, 2};
    for (int j = 0; j < 3; ++j) S[j] = sqrt(A[j] * A[j] + A[3 + j] * A[3 + j] + A[6 + j] * A[6 + j]);
    for (int a = 0; a < 3; ++a)                       // descending singular values
        for (int b = a + 1; b < 3; ++b)
            if (S[ord[b]] > S[ord[a]]) {
                const int x = ord[a];
                ord[a] = ord[b];
                ord[b] = x;
            }
    double U[9], Vs[9];
    for (int j = 0; j < 3; ++j) {
        const int k = ord[j];
        for (int i = 0; i < 3; ++i) {
            Vs[3 * i + j] = V[3 * i + k];
            U[3 * i + j] = S[k] > 0 ? A[3 * i + k] / S[k] : 0.0;
        }
    }
    if (!(S[ord[2]] > 1e-300)) {                       // rank-deficient: complete U by a cross product
        U[2] = U[3] * U[7] - U[6] * U[4];
        U[5] = U[6] * U[1] - U[0] * U[7];
        U[8] = U[0] * U[4] - U[3] * U[1];
    }
    const double d = det3(Vs) * det3(U);
    for (int r = 0; r < 3; ++r)
        for (int cc = 0; cc < 3; ++cc)
            R[3 * r + cc] = Vs[3 * r + 0] * U[3 * cc + 0] + Vs[3 * r + 1] * U[3 * cc + 1] + d * Vs[3 * r + 2] * U[3 * cc + 2];
}

__global__ __launch_bounds__(KT) void kabsch_kernel(const float* __restrict__ from, const float* __restrict__ to,
                                                    int n, int remove_outliers, float* __restrict__ R_out,
                                                    float* __restrict__ t_out, float* __restrict__ c_out,
                                                    float* __restrict__ err_out) {
    __shared__ double red[KT];
    __shared__ double sol[13];                         // R (9), t (3), c
    __shared__ float dist[NERF_KABSCH_MAX_POINTS];
    __shared__ float srt[NERF_KABSCH_MAX_POINTS];
    __shared__ unsigned char keep[NERF_KABSCH_MAX_POINTS];
    const int tid = threadIdx.x;
    for (int i = tid; i < n; i += KT) keep[i] = 1;
    __syncthreads();
    for (int pass = 0; pass < (remove_outliers ? 2 : 1); ++pass) {
        double s[7] = {0, 0, 0, 0, 0, 0, 0};
        for (int i = tid; i < n; i += KT) {
            if (!keep[i]) continue;
            s[0] += 1.0;
            for (int j = 0; j < 3; ++j) {
                s[1 + j] += from[3 * i + j];
                s[4 + j] += to[3 * i + j];
            }
        }
        double tot[7];
        for (int k = 0; k < 7; ++k) tot[k] = block_sum(s[k], red);
        double mf[3], mt[3];
        for (int j = 0; j < 3; ++j) {
            mf[j] = tot[1 + j] / tot[0];
            mt[j] = tot[4 + j] / tot[0];
        }
        double h[11] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};   // H (9), |from_c|^2, |to_c|^2
        for (int i = tid; i < n; i += KT) {
            if (!keep[i]) continue;
            double a[3], b[3];
            for (int j = 0; j < 3; ++j) {
                a[j] = from[3 * i + j] - mf[j];
                b[j] = to[3 * i + j] - mt[j];
            }
            for (int r = 0; r < 3; ++r)
                for (int cc = 0; cc < 3; ++cc) h[3 * r + cc] += a[r] * b[cc];
            h[9] += a[0] * a[0] + a[1] * a[1] + a[2] * a[2];
            h[10] += b[0] * b[0] + b[1] * b[1] + b[2] * b[2];
        }
        double H[11];
        for (int k = 0; k < 11; ++k) H[k] = block_sum(h[k], red);
        if (tid == 0) {
            double R[9];
            kabsch_rotation(H, R);
            const double c = sqrt(H[10]) / sqrt(H[9]);
            for (int k = 0; k < 9; ++k) sol[k] = R[k];
            for (int r = 0; r < 3; ++r) sol[9 + r] = mt[r] - c * (R[3 * r] * mf[0] + R[3 * r + 1] * mf[1] + R[3 * r + 2] * mf[2]);
            sol[12] = c;
        }
        __syncthreads();
        if (pass == 0 && remove_outliers) {
            for (int i = tid; i < n; i += KT) {
                double e2 = 0;
                for (int r = 0; r < 3; ++r) {
                    const double y = (sol[3 * r] * from[3 * i] + sol[3 * r + 1] * from[3 * i + 1] +
                                      sol[3 * r + 2] * from[3 * i + 2]) * sol[12] + sol[9 + r] - to[3 * i + r];
                    e2 += y * y;
                }
                dist[i] = (float)sqrt(e2);
            }
            __syncthreads();
            for (int i = tid; i < n; i += KT) {       // ascending order by rank (ties: index)
                int rank = 0;
                const float di = dist[i];
                for (int j = 0; j < n; ++j) rank += (dist[j] < di || (dist[j] == di && j < i)) ? 1 : 0;
                srt[rank] = di;
            }
            __syncthreads();
            // torch.quantile(d, 0.9): rank 0.9 (n - 1), linear interpolation (torch.lerp's two forms)
            const float pos = 0.9f * (float)(n - 1);
            const int lo = (int)floorf(pos), hi = (int)ceilf(pos);
            const float w = pos - (float)lo;
            const float a = srt[lo], b = srt[hi];
            const float q = w < 0.5f ? a + w * (b - a) : b - (b - a) * (1.0f - w);
            for (int i = tid; i < n; i += KT) keep[i] = dist[i] < q ? 1 : 0;
            __syncthreads();
        }
    }
    if (tid < 9) R_out[tid] = (float)sol[tid];
    if (tid < 3) t_out[tid] = (float)sol[9 + tid];
    if (tid == 0) c_out[0] = (float)sol[12];
    if (err_out != nullptr) {
        // compute_pose_error: mean over ALL points of |to - (R from c + t)|
        double e = 0;
        for (int i = tid; i < n; i += KT) {
            double e2 = 0;
            for (int r = 0; r < 3; ++r) {
                const double y = to[3 * i + r] - ((sol[3 * r] * from[3 * i] + sol[3 * r + 1] * from[3 * i + 1] +
                                                   sol[3 * r + 2] * from[3 * i + 2]) * sol[12] + sol[9 + r]);
                e2 += y * y;
            }
            e += sqrt(e2);
        }
        const double tot = block_sum(e, red);
        if (tid == 0) err_out[0] = (float)(tot / n);
    }
}

}  // namespace

extern "C" int nerf_kabsch(const float* from, const float* to, int32_t n, int32_t remove_outliers, float* R,
                           float* t, float* c, float* err, void* stream) {
    NERF_REQUIRE(from && to && R && t && c && n >= 3 && n <= NERF_KABSCH_MAX_POINTS);
    hipLaunchKernelGGL(kabsch_kernel, dim3(1), dim3(KT), 0, as_stream(stream), from, to, n, remove_outliers ? 1 : 0,
                       R, t, c, err);
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}
