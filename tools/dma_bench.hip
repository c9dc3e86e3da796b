// Microbenchmark of the streamed weight gradient's operand stream (linear_x3.hip
// linear_wgrad_x3_stream_kernel): every workgroup (one per CU) streams 16-row steps of two
// fp32 row buffers (dY, X: 1 KB rows) into an LDS ring by LDS-DMA, with nothing consuming them.
// Variants: who issues the DMA (all 8 waves, 4 instructions each, or one loader wave, 32),
// ring depth (steps in flight), and how the rows are dealt to workgroups (contiguous ranges or
// step-interleaved).  Prints the read rate.
//
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/dma_bench tools/dma_bench.hip && /tmp/dma_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

constexpr int T = 16;              // rows per step and operand
constexpr int STAGE = 2 * T * 1024;

template <int NRAW, bool LOADER, bool INTERLEAVE>
__global__ __launch_bounds__(512, 1) void stream_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                        int M, float* sink) {
    __shared__ __attribute__((aligned(16))) char ring[NRAW * STAGE];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int nsteps_total = M / T;
    const int G = gridDim.x;
    int steps, first;
    if (INTERLEAVE) {
        first = blockIdx.x;
        steps = (nsteps_total - first + G - 1) / G;
    } else {
        const int per = (nsteps_total + G - 1) / G;
        first = blockIdx.x * per;
        steps = min(per, nsteps_total - first);
    }
    auto step_row = [&](int i) { return INTERLEAVE ? (first + i * G) * T : (first + i) * T; };
    auto issue = [&](int i) {
        char* st = ring + (i % NRAW) * STAGE;
        const int r0 = step_row(i);
        if (LOADER) {
            if (wave == 0) {
#pragma unroll
                for (int r = 0; r < T; ++r) {
                    __builtin_amdgcn_global_load_lds((glb_void_t*)(dy + (size_t)(r0 + r) * 256 + 4 * lane),
                                                     (lds_void_t*)(st + r * 1024), 16, 0, 0);
                    __builtin_amdgcn_global_load_lds((glb_void_t*)(x + (size_t)(r0 + r) * 256 + 4 * lane),
                                                     (lds_void_t*)(st + (T + r) * 1024), 16, 0, 0);
                }
            }
        } else {
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int r = 2 * wave + q;
                __builtin_amdgcn_global_load_lds((glb_void_t*)(dy + (size_t)(r0 + r) * 256 + 4 * lane),
                                                 (lds_void_t*)(st + r * 1024), 16, 0, 0);
                __builtin_amdgcn_global_load_lds((glb_void_t*)(x + (size_t)(r0 + r) * 256 + 4 * lane),
                                                 (lds_void_t*)(st + (T + r) * 1024), 16, 0, 0);
            }
        }
    };
    // per-step DMA count of the issuing waves: 4 (all waves) or 32 (loader)
    constexpr int PER = LOADER ? 2 * T : 4;
    float acc = 0.f;
    for (int q = 0; q < NRAW - 1 && q < steps; ++q) issue(q);
    for (int i = 0; i < steps; ++i) {
        if (i + NRAW - 1 < steps) issue(i + NRAW - 1);
        // step i landed: at most NRAW - 1 younger steps outstanding
        const int younger = min(steps - 1, i + NRAW - 1) - i;
        if (younger >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * PER > 63 ? 63 : 3 * PER) : "memory");
        else if (younger == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER > 63 ? 63 : 2 * PER) : "memory");
        else if (younger == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        acc += reinterpret_cast<const float*>(ring + (i % NRAW) * STAGE)[threadIdx.x];
        __builtin_amdgcn_s_barrier();
    }
    if (acc == 1234.5f) sink[threadIdx.x] = acc;
}

__global__ void flush_kernel(float4* p, size_t n, float v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_float4(v, v, v, v);
}

float* g_flush = nullptr;
constexpr size_t FLUSH_BYTES = 512ull << 20;

template <int NRAW, bool LOADER, bool INTERLEAVE>
void run(const char* name, const float* dy, const float* x, int M, float* sink) {
    const int grid = 256;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int w = 0; w < 3; ++w) stream_kernel<NRAW, LOADER, INTERLEAVE><<<grid, 512>>>(dy, x, M, sink);
    const int reps = 10;
    float tot = 0.f;
    for (int w = 0; w < reps; ++w) {
        // a 512 MB write between launches (cold caches / translations, as in the training step)
        flush_kernel<<<2048, 256>>>(reinterpret_cast<float4*>(g_flush), FLUSH_BYTES / 16, (float)w);
        hipEventRecord(e0);
        stream_kernel<NRAW, LOADER, INTERLEAVE><<<grid, 512>>>(dy, x, M, sink);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        tot += ms;
    }
    const double us = tot * 1000.0 / reps;
    const double bytes = 2.0 * M * 1024.0;
    printf("%-34s %8.1f us  %6.2f TB/s\n", name, us, bytes / (us * 1e-6) / 1e12);
}

int main() {
    const int M = 524288;
    float *dy, *x, *sink;
    hipMalloc(&dy, (size_t)M * 1024);
    hipMalloc(&x, (size_t)M * 1024);
    hipMalloc(&sink, 4096);
    hipMalloc(&g_flush, FLUSH_BYTES);
    hipMemset(dy, 0, (size_t)M * 1024);
    hipMemset(x, 0, (size_t)M * 1024);
    run<3, false, false>("all waves, 2 steps ahead, ranges", dy, x, M, sink);
    run<3, true, false>("loader, 2 steps ahead, ranges", dy, x, M, sink);
    run<4, true, false>("loader, 3 steps ahead, ranges", dy, x, M, sink);
    run<3, false, true>("all waves, 2 ahead, interleaved", dy, x, M, sink);
    run<3, true, true>("loader, 2 ahead, interleaved", dy, x, M, sink);
    run<4, true, true>("loader, 3 ahead, interleaved", dy, x, M, sink);
    run<4, false, true>("all waves, 3 ahead, interleaved", dy, x, M, sink);
    run<2, false, true>("all waves, 1 ahead, interleaved", dy, x, M, sink);
    hipFree(dy);
    hipFree(x);
    hipFree(sink);
    return 0;
}
