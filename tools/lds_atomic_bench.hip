// LDS 64-bit integer atomic throughput on gfx950 under the access shapes the hash-grid backward
// produces: all lanes on distinct rows, 1/8 of the lanes active, runs of lanes on one row.
//   hipcc -O3 --offload-arch=gfx950 tools/lds_atomic_bench.hip -o tools/_lds_atomic_bench && ./tools/_lds_atomic_bench
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ENTRIES = 16384;
constexpr int ITERS = 256;

template <int MODE>
__global__ __launch_bounds__(1024) void k(unsigned long long* out, int salt) {
    __shared__ unsigned long long part[ENTRIES];
    for (int e = threadIdx.x; e < ENTRIES; e += 1024) part[e] = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    unsigned h = threadIdx.x * 2654435761u + salt;
    for (int i = 0; i < ITERS; ++i) {
        h = h * 1664525u + 1013904223u;
        int row;
        bool act = true;
        if (MODE == 0) row = h >> 18;                      // distinct random rows, all lanes
        else if (MODE == 1) { row = h >> 18; act = (h & 7) == 0; }   // 1/8 of lanes
        else if (MODE == 2) row = ((h >> 18) & ~63) | (lane >> 4);  // runs of 16 lanes on a row
        else row = (h >> 18) & ~63;                        // whole wave on one row (per wave random)
        if (MODE == 3) row = __builtin_amdgcn_readfirstlane(row);
        if (MODE == 2) row = __builtin_amdgcn_readfirstlane(row & ~63) | (lane >> 4);
        if (act) atomicAdd(&part[row], 1ull + i);
    }
    __syncthreads();
    unsigned long long s = 0;
    for (int e = threadIdx.x; e < ENTRIES; e += 1024) s += part[e];
    atomicAdd(out, s);
}

template <int MODE>
float run(unsigned long long* d) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(k<MODE>, dim3(1024), dim3(1024), 0, 0, d, 1);
    hipEventRecord(a);
    for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(k<MODE>, dim3(1024), dim3(1024), 0, 0, d, r);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms / 10;
}

int main() {
    unsigned long long* d;
    hipMalloc(&d, 8);
    const char* names[] = {"all lanes, distinct rows", "1/8 lanes active", "runs of 16 lanes", "whole wave one row"};
    float t[4] = {run<0>(d), run<1>(d), run<2>(d), run<3>(d)};
    // wave-instructions per CU (1024 workgroups over 256 CUs, 16 waves each, ITERS each)
    const double instr_per_cu = 1024.0 / 256 * 16 * ITERS;
    for (int m = 0; m < 4; ++m)
        printf("%-28s %8.1f us  %6.1f ns per ds_add_u64 wave-instruction per CU\n", names[m], t[m] * 1e3,
               t[m] * 1e6 / instr_per_cu);
    hipFree(d);
    return 0;
}
