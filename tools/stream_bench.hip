// Microbenchmark of the streamed weight gradient's operand read (linear_x3.hip
// linear_wgrad_x3_stream_kernel) — VERDICT r3 #4: is the 4.3-4.6 TB/s of its LDS-DMA stream a
// property of LDS-DMA, or of the access pattern / the cache state?  Every variant reads the same
// 2 x 512 MB (dY and X: 524 288 rows of 1 KB each), one 512-thread workgroup per CU (256), and
// puts the rows in a 32 KB-per-step LDS ring that nothing consumes (a token read keeps it live).
//
//   dma      : buffer-less LDS-DMA (global_load_lds_dwordx4), 4 per wave per step, D steps ahead
//   reg      : global_load_dwordx4 into VGPRs (4 per thread per step, D steps in flight, counted
//              vmcnt), then ds_write_b128 into the ring: the register-staged form
//   regnolds : as reg, the rows summed into a register instead of written to LDS (pure read)
//
// Row order: "ranges" (CU s reads rows [s M/256, (s+1) M/256) in 16-row steps — the kernel's
// split layout) or "inter" (16-row step i of CU s is global step s + 256 i: all CUs within a
// 8 MB window at any moment).  Cache state before each timed launch: "wflush" (a 512 MB write,
// as the training step's forward / chain leave it), "rflush" (a 1 GB read of another buffer:
// caches hold clean, unrelated lines) or "warm" (nothing; 1 GB does not fit the 256 MB MALL).
//
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/stream_bench tools/stream_bench.hip && /tmp/stream_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int T = 16;                 // rows per step and operand
constexpr int STAGE = 2 * T * 1024;   // 32 KB per step

enum { DMA = 0, REG = 1, REGNOLDS = 2 };

template <int MODE, int D, bool INTER>
__global__ __launch_bounds__(512, 1) void stream_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                        int M, float* sink) {
    constexpr int NRAW = MODE == DMA ? D + 1 : 2;
    __shared__ __attribute__((aligned(16))) char ring[NRAW * STAGE];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int G = gridDim.x, nst = M / T;
    int steps, first;
    if (INTER) {
        first = blockIdx.x;
        steps = (nst - first + G - 1) / G;
    } else {
        const int per = (nst + G - 1) / G;
        first = blockIdx.x * per;
        steps = min(per, nst - first);
    }
    auto row0 = [&](int i) { return INTER ? (first + i * G) * T : (first + i) * T; };
    // wave w, piece q (0..3): operand q >> 1, row 2 w + (q & 1) of the step
    auto src = [&](int i, int q) {
        const float* b = (q >> 1) ? x : dy;
        return b + (size_t)(row0(i) + 2 * wave + (q & 1)) * 256 + 4 * lane;
    };
    float acc = 0.f;
    if constexpr (MODE == DMA) {
        auto issue = [&](int i) {
            char* st = ring + (i % NRAW) * STAGE;
#pragma unroll
            for (int q = 0; q < 4; ++q)
                __builtin_amdgcn_global_load_lds((glb_void_t*)src(i, q),
                                                 (lds_void_t*)(st + ((q >> 1) * T + 2 * wave + (q & 1)) * 1024), 16, 0, 0);
        };
        for (int q = 0; q < D && q < steps; ++q) issue(q);
        for (int i = 0; i < steps; ++i) {
            const int younger = min(steps - 1, i + D - 1) - i;     // steps issued after i
            if (younger >= 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
            else if (younger == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else if (younger == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            acc += reinterpret_cast<const float*>(ring + (i % NRAW) * STAGE)[threadIdx.x];
            __builtin_amdgcn_s_barrier();
            if (i + D < steps) issue(i + D);
        }
    } else {
        // D steps of 4 dwordx4 per thread in flight; registers indexed at compile time only
        f4 buf[D][4];
#pragma unroll
        for (int s = 0; s < D; ++s)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (s < steps) buf[s][q] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(src(s, q)));
        f4 sum = {0.f, 0.f, 0.f, 0.f};
        for (int i0 = 0; i0 < steps; i0 += D) {
#pragma unroll
            for (int s = 0; s < D; ++s) {
                const int i = i0 + s;
                if (i < steps) {
                    if constexpr (MODE == REG) {
                        char* st = ring + (i & 1) * STAGE;
#pragma unroll
                        for (int q = 0; q < 4; ++q)
                            *reinterpret_cast<f4*>(st + ((q >> 1) * T + 2 * wave + (q & 1)) * 1024 + 16 * lane) = buf[s][q];
                    } else {
#pragma unroll
                        for (int q = 0; q < 4; ++q) sum += buf[s][q];
                    }
                    if (i + D < steps) {
#pragma unroll
                        for (int q = 0; q < 4; ++q)
                            buf[s][q] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(src(i + D, q)));
                    }
                    if constexpr (MODE == REG) {
                        if ((i & 7) == 7) {
                            __syncthreads();
                            acc += reinterpret_cast<const float*>(ring)[threadIdx.x];
                            __syncthreads();
                        }
                    }
                }
            }
        }
        acc += sum.x + sum.y + sum.z + sum.w;
    }
    if (acc == 1234.5f) sink[threadIdx.x] = acc;
}

__global__ void wflush_kernel(f4* p, size_t n, float v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = f4{v, v, v, v};
}
__global__ void rflush_kernel(const f4* p, size_t n, float* sink) {
    f4 s = {0.f, 0.f, 0.f, 0.f};
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        s += p[i];
    if (s.x == 1234.5f) sink[0] = s.y;
}
__global__ void fill_kernel(float* p, size_t n, unsigned seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned h = (unsigned)i * 2654435761u ^ seed;
        h ^= h >> 13;
        h *= 0x5bd1e995u;
        p[i] = (float)(h & 0xffff) * (1.f / 65536.f) - 0.5f;
    }
}

constexpr size_t FLUSH_BYTES = 1024ull << 20;
f4* g_flush = nullptr;
float* g_sink = nullptr;

template <int MODE, int D, bool INTER>
void run(const char* mode, const float* dy, const float* x, int M, int cache) {
    const int grid = 256;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int w = 0; w < 2; ++w) stream_kernel<MODE, D, INTER><<<grid, 512>>>(dy, x, M, g_sink);
    const int reps = 8;
    float tot = 0.f;
    for (int w = 0; w < reps; ++w) {
        if (cache == 0) wflush_kernel<<<4096, 256>>>(g_flush, FLUSH_BYTES / 2 / 16, (float)w);
        if (cache == 1) rflush_kernel<<<4096, 256>>>(g_flush, FLUSH_BYTES / 16, g_sink);
        hipEventRecord(e0);
        stream_kernel<MODE, D, INTER><<<grid, 512>>>(dy, x, M, g_sink);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        tot += ms;
    }
    const double us = tot * 1000.0 / reps;
    const double bytes = 2.0 * M * 1024.0;
    static const char* cn[] = {"wflush", "rflush", "warm"};
    printf("%-9s D=%d %-6s %-6s %8.1f us  %6.2f TB/s\n", mode, D, INTER ? "inter" : "ranges", cn[cache], us,
           bytes / (us * 1e-6) / 1e12);
    fflush(stdout);
}

template <bool INTER>
void sweep(const float* dy, const float* x, int M, int cache) {
    run<DMA, 2, INTER>("dma", dy, x, M, cache);
    run<DMA, 3, INTER>("dma", dy, x, M, cache);
    run<DMA, 4, INTER>("dma", dy, x, M, cache);
    run<REG, 2, INTER>("reg", dy, x, M, cache);
    run<REG, 4, INTER>("reg", dy, x, M, cache);
    run<REGNOLDS, 2, INTER>("regnolds", dy, x, M, cache);
    run<REGNOLDS, 4, INTER>("regnolds", dy, x, M, cache);
}

int main() {
    const int M = 524288;
    float *dy, *x;
    hipMalloc(&dy, (size_t)M * 1024);
    hipMalloc(&x, (size_t)M * 1024);
    hipMalloc(&g_sink, 4096);
    hipMalloc(&g_flush, FLUSH_BYTES);
    fill_kernel<<<4096, 256>>>(dy, (size_t)M * 256, 1u);
    fill_kernel<<<4096, 256>>>(x, (size_t)M * 256, 2u);
    fill_kernel<<<4096, 256>>>(reinterpret_cast<float*>(g_flush), FLUSH_BYTES / 4, 3u);
    hipDeviceSynchronize();
    for (int cache = 0; cache < 3; ++cache) {
        sweep<false>(dy, x, M, cache);
        sweep<true>(dy, x, M, cache);
    }
    hipFree(dy);
    hipFree(x);
    hipFree(g_flush);
    hipFree(g_sink);
    return 0;
}
