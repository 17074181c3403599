// Microbenchmark: what one small latency-bound kernel costs on MI355X, to explain the seed hop
// (k_seed_frontier: one 1024-thread workgroup, ~5 dependent loads, 14 us) and the close kernel.
//   empty        an empty 1-workgroup launch (the floor of a kernel on the stream)
//   chase<S, K>  1024 threads, each K dependent random 8-B loads over an S-byte buffer (a pointer
//                chase: the next index comes from the loaded value), for S from 4 MB to 2 GB: the
//                per-load latency once TLB reach is exceeded
//   host         one load per thread from host-mapped page-locked memory, then one store back
// Each configuration: 200 back-to-back launches timed with HIP events, average per launch.
// Usage: mb_latency
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP %s at %s\n", hipGetErrorString(e_), #x); std::exit(1); } } while (0)

__global__ void k_empty() {}

__global__ __launch_bounds__(1024) void k_chase(const uint64_t* buf, uint64_t mask, int k, uint64_t seed, uint64_t* out) {
    uint64_t i = (seed + threadIdx.x * 0x9e3779b97f4a7c15ULL) & mask;
    uint64_t acc = 0;
    for (int j = 0; j < k; j++) {
        const uint64_t v = buf[i];
        acc += v;
        i = (v ^ (i * 0xbf58476d1ce4e5b9ULL)) & mask;
    }
    if (acc == 0x1234567) out[threadIdx.x] = acc;
}

__global__ __launch_bounds__(1024) void k_host(const uint64_t* h, uint64_t* d, uint64_t n) {
    const uint64_t i = threadIdx.x;
    if (i < n) d[i] = h[i] + 1;
}

template <class F>
double timeIt(F launch, int iters = 200) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 10; i++) launch(i);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < iters; i++) launch(i);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ms * 1e3 / iters;
}

int main() {
    uint64_t* out = nullptr;
    CK(hipMalloc(&out, 1024 * 8));
    std::printf("{\"empty_us\": %.2f,\n", timeIt([&](int) { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, 0); }));
    std::printf(" \"chase\": [\n");
    const uint64_t sizes[] = {4ULL << 20, 32ULL << 20, 256ULL << 20, 2048ULL << 20};
    bool first = true;
    for (uint64_t S : sizes) {
        uint64_t* buf = nullptr;
        CK(hipMalloc(&buf, S));
        std::vector<uint64_t> h(S / 8);
        uint64_t x = 88172645463325252ULL;
        for (auto& v : h) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = x; }
        CK(hipMemcpy(buf, h.data(), S, hipMemcpyHostToDevice));
        for (int k : {1, 2, 4, 8}) {
            const double us = timeIt([&](int it) {
                hipLaunchKernelGGL(k_chase, dim3(1), dim3(1024), 0, 0, buf, S / 8 - 1, k, static_cast<uint64_t>(it) * 7919, out);
            });
            std::printf("%s  {\"bytes\": %llu, \"loads\": %d, \"us\": %.2f}", first ? "" : ",\n",
                        static_cast<unsigned long long>(S), k, us);
            first = false;
        }
        CK(hipFree(buf));
    }
    std::printf("\n ],\n");
    uint64_t* hb = nullptr;
    CK(hipHostMalloc(&hb, 1024 * 8, hipHostMallocMapped));
    uint64_t* hd = nullptr;
    CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&hd), hb, 0));
    std::printf(" \"host_read_us\": %.2f}\n", timeIt([&](int) { hipLaunchKernelGGL(k_host, dim3(1), dim3(1024), 0, 0, hd, out, 1000); }));
    CK(hipHostFree(hb));
    CK(hipFree(out));
    return 0;
}
