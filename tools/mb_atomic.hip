// Microbenchmark: the final hop's output reservation. Each workgroup of the GO final kernel
// (final_kernels.h finalBody, !ORDERED) reserves its rows with one atomicAdd on a single device-scope
// counter and then stores at the returned offset. At C2 that is ~31 K same-address atomics per launch.
// This times the reservation pattern alone over the same grid:
//   same   one counter (the kernel's pattern)
//   xcd8   one counter per XCD (blockIdx % 8), 256 B apart
//   none   no atomic (offset from the block index)
// each followed by a dependent 256-thread store of 8 B per lane at the offset (as the row stores).
// Usage: mb_atomic [workgroups] [iters]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP %s at %s\n", hipGetErrorString(e_), #x); std::exit(1); } } while (0)

template <int MODE>
__global__ __launch_bounds__(256) void k_reserve(unsigned long long* ctr, long long* out, unsigned per) {
    __shared__ unsigned long long base;
    if (threadIdx.x == 0) {
        if (MODE == 0) base = atomicAdd(ctr, static_cast<unsigned long long>(per));
        else if (MODE == 1) base = atomicAdd(ctr + (blockIdx.x % 8u) * 32u, static_cast<unsigned long long>(per));
        else base = static_cast<unsigned long long>(blockIdx.x) * per;
    }
    __syncthreads();
    // offsets of modes 0 / 1 stay below grid * per (mode 1: each counter below its own share * 8)
    const unsigned long long o = (base % (static_cast<unsigned long long>(gridDim.x) * per)) + threadIdx.x % per;
    out[o] = static_cast<long long>(blockIdx.x);
}

int main(int argc, char** argv) {
    const unsigned grid = argc > 1 ? static_cast<unsigned>(std::atoi(argv[1])) : 31250u;
    const int iters = argc > 2 ? std::atoi(argv[2]) : 20;
    const unsigned per = 256;
    unsigned long long* ctr;
    long long* out;
    CK(hipMalloc(&ctr, 8 * 32 * 8));
    CK(hipMalloc(&out, static_cast<size_t>(grid) * per * 8));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const char* names[3] = {"same", "xcd8", "none"};
    for (int mode = 0; mode < 3; mode++) {
        float total = 0;
        for (int it = 0; it < iters + 2; it++) {
            CK(hipMemset(ctr, 0, 8 * 32 * 8));
            CK(hipEventRecord(a));
            if (mode == 0) hipLaunchKernelGGL(k_reserve<0>, dim3(grid), dim3(256), 0, 0, ctr, out, per);
            else if (mode == 1) hipLaunchKernelGGL(k_reserve<1>, dim3(grid), dim3(256), 0, 0, ctr, out, per);
            else hipLaunchKernelGGL(k_reserve<2>, dim3(grid), dim3(256), 0, 0, ctr, out, per);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            if (it >= 2) total += ms;
        }
        std::printf("%s: %u workgroups, %.1f us per launch (%.2f ns per workgroup)\n", names[mode], grid,
                    1e3 * total / iters, 1e6 * total / iters / grid);
    }
    return 0;
}
