// Microbenchmark: does a small latency-bound kernel pay for the address translations a big kernel
// before it evicted? (The close kernel's header — two dependent loads of a few control words — takes
// ~7 us more than an empty launch even on one workgroup, right after the 300-us final hop that touches
// ~4 GB.)
//   probe      one workgroup; thread 0 loads small[0], then small[that] (a 2-load chain), stores it
//   sweep(S)   one load per 64 KB over S bytes of a big buffer, every CU (touches S / 2 MB pages)
// Timed with HIP events around the probe alone, after: another probe (warm), a sweep of 64 MB, a
// sweep of 6 GB; and the probe over a small buffer inside the big allocation's first page.
// Usage: mb_tlb
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP %s at %s\n", hipGetErrorString(e_), #x); std::exit(1); } } while (0)

__global__ void k_probe(const uint64_t* small, uint64_t* out) {
    if (threadIdx.x == 0) {
        const uint64_t i = small[0];
        out[0] = small[i & 1023] + 1;
    }
}

__global__ void k_sweep(const uint8_t* big, uint64_t bytes, uint64_t* out) {
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
    uint64_t acc = 0;
    for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i * 65536 < bytes; i += stride)
        acc += big[i * 65536];
    if (acc == 0x77) out[1] = acc;
}

int main() {
    const uint64_t bigBytes = 6ULL << 30;
    uint8_t* big = nullptr;
    uint64_t *small = nullptr, *out = nullptr;
    CK(hipMalloc(&big, bigBytes));
    CK(hipMemset(big, 1, bigBytes));
    CK(hipMalloc(&small, 8192));
    CK(hipMemset(small, 0, 8192));
    CK(hipMalloc(&out, 64));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto probeAfter = [&](uint64_t sweepBytes, const uint64_t* target) {
        double sum = 0;
        const int iters = 50;
        for (int it = 0; it < iters; it++) {
            if (sweepBytes) hipLaunchKernelGGL(k_sweep, dim3(1024), dim3(256), 0, 0, big, sweepBytes, out);
            else hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, target, out);
            CK(hipEventRecord(a, 0));
            hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, target, out);
            CK(hipEventRecord(b, 0));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            sum += ms * 1e3;
        }
        return sum / iters;
    };
    const uint64_t* inBig = reinterpret_cast<const uint64_t*>(big);   // small words inside the big allocation
    CK(hipMemset(big, 0, 8192));
    std::printf("{\"probe_warm_us\": %.2f, \"probe_after_64MB_us\": %.2f, \"probe_after_6GB_us\": %.2f, "
                "\"probe_in_big_after_6GB_us\": %.2f}\n",
                probeAfter(0, small), probeAfter(64ULL << 20, small), probeAfter(bigBytes, small),
                probeAfter(bigBytes, inBig));
    CK(hipFree(big));
    CK(hipFree(small));
    CK(hipFree(out));
    return 0;
}
