// Fused Adam: one launch updates every parameter tensor of an optimizer step.
//
// Reference: every experiment trains with torch.optim.Adam(eps=1e-5) (configure_optimizers,
// barf/model_interpolation.py:543-584).  torch's per-element update (torch/optim/adam.py,
// amsgrad = maximize = False), restated in fp32 with the same operation order:
//   g = grad (+ weight_decay * param)
//   m = m + (1 - beta1) * (g - m)                  exp_avg.lerp_(grad, 1 - beta1)
//   v = v * beta2 + ((1 - beta2) * g) * g          exp_avg_sq.mul_(beta2).addcmul_(grad, grad, 1 - beta2)
//   p = p + step * (m / (sqrt(v) / bc2_sqrt + eps))
// with step = -lr / (1 - beta1^t) and bc2_sqrt = sqrt(1 - beta2^t) host scalars per tensor
// (formed in double, as torch forms them).
//
// torch's default (foreach) Adam issues ~7 multi-tensor kernels per step; here the tensor
// table travels in the kernel arguments (no device table, no host-to-device copy per step),
// every 256-thread block updates 2048 consecutive elements of one tensor and finds its tensor
// with a scan of the table read by scalar loads from the kernarg segment (indexing the
// by-value argument would make hipcc copy it to scratch).
#include <cstddef>

#include "common.h"

namespace {

constexpr int kAdamPerBlock = 2048;

typedef __attribute__((address_space(4))) const char kchar_t;
typedef float* fptr_t;
typedef const float* cfptr_t;
#define NERF_ADAMF(T, field, i) \
    (*(const __attribute__((address_space(4))) T*)(kargs + offsetof(nerf_adam_batch, field) + (size_t)(i) * sizeof(T)))

__global__ __launch_bounds__(256) void adam_kernel(nerf_adam_batch b) {
#pragma clang fp contract(off)
    kchar_t* kargs = (kchar_t*)__builtin_amdgcn_kernarg_segment_ptr();
    const int64_t bid = blockIdx.x;
    int ti = 0;
    int64_t first = 0;
    for (; ti < b.n_tensors; ++ti) {
        const int64_t nb = (NERF_ADAMF(int64_t, numel, ti) + kAdamPerBlock - 1) / kAdamPerBlock;
        if (bid < first + nb) break;
        first += nb;
    }
    if (ti >= b.n_tensors) return;
    const int64_t n = NERF_ADAMF(int64_t, numel, ti);
    float* p = NERF_ADAMF(fptr_t, param, ti);
    const float* g = NERF_ADAMF(cfptr_t, grad, ti);
    float* m = NERF_ADAMF(fptr_t, exp_avg, ti);
    float* v = NERF_ADAMF(fptr_t, exp_avg_sq, ti);
    const float step = NERF_ADAMF(float, step_size, ti);
    const float bc2 = NERF_ADAMF(float, bc2_sqrt, ti);
    const float wd = NERF_ADAMF(float, weight_decay, ti);
    const int64_t i0 = (bid - first) * kAdamPerBlock;
    const int64_t i1 = i0 + kAdamPerBlock < n ? i0 + kAdamPerBlock : n;
    for (int64_t i = i0 + threadIdx.x; i < i1; i += 256) {
        float pv = p[i];
        float gv = g[i];
        if (wd != 0.0f) gv = gv + wd * pv;
        float mv = m[i];
        mv = mv + b.one_minus_beta1 * (gv - mv);
        float vv = v[i];
        vv = vv * b.beta2 + (b.one_minus_beta2 * gv) * gv;
        const float denom = sqrtf(vv) / bc2 + b.eps;
        pv = pv + step * (mv / denom);
        p[i] = pv;
        m[i] = mv;
        v[i] = vv;
    }
}

}  // namespace

extern "C" int nerf_adam_step(const nerf_adam_batch* batch, void* stream) {
    NERF_REQUIRE(batch && batch->n_tensors >= 0 && batch->n_tensors <= NERF_ADAM_MAX_TENSORS);
    int64_t blocks = 0;
    for (int i = 0; i < batch->n_tensors; ++i) {
        const int64_t n = batch->numel[i];
        NERF_REQUIRE(n >= 0);
        if (n > 0) NERF_REQUIRE(batch->param[i] && batch->grad[i] && batch->exp_avg[i] && batch->exp_avg_sq[i]);
        blocks += (n + kAdamPerBlock - 1) / kAdamPerBlock;
    }
    if (blocks == 0) return NERF_OK;
    NERF_REQUIRE(blocks < (1ll << 31));
    hipLaunchKernelGGL(adam_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), *batch);
    NERF_CHECK_LAUNCH();
    return NERF_OK;
}
