// Microbenchmark: device -> page-locked host bandwidth on MI355X for the result-delivery path
// (ngx_go host_columnar). Variants: hipMemcpyAsync on 1 / 2 / 4 / 8 streams over equal chunks, into
// hipHostMalloc memory allocated default / non-coherent / write-combined / numa-user, and a copy
// kernel storing into the mapped host buffer. Prints GB/s per variant.
// Build: hipcc -O3 --offload-arch=gfx950 tools/mb_d2h.hip -o tools/mb_d2h
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ void kcopy(const uint4* src, uint4* dst, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) dst[i] = src[i];
}

int main() {
    const size_t bytes = size_t(1277) << 20;
    void* dev = nullptr;
    CK(hipMalloc(&dev, bytes));
    CK(hipMemset(dev, 1, bytes));
    std::vector<hipStream_t> st(8);
    for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    struct Flav { const char* name; unsigned flags; };
    Flav flavs[] = {{"default", hipHostMallocDefault}, {"noncoherent", hipHostMallocNonCoherent},
                    {"writecombined", hipHostMallocWriteCombined}, {"coherent", hipHostMallocCoherent}};
    for (auto& f : flavs) {
        void* host = nullptr;
        if (hipHostMalloc(&host, bytes, f.flags) != hipSuccess) { std::printf("%s: alloc failed\n", f.name); continue; }
        std::memset(host, 0, bytes);
        for (int ns : {1, 2, 4, 8}) {
            double best = 1e9;
            for (int rep = 0; rep < 3; rep++) {
                CK(hipDeviceSynchronize());
                auto t0 = std::chrono::steady_clock::now();
                size_t chunk = (bytes / ns + 4095) & ~size_t(4095);
                for (int k = 0; k < ns; k++) {
                    size_t off = k * chunk;
                    if (off >= bytes) break;
                    size_t n = off + chunk > bytes ? bytes - off : chunk;
                    CK(hipMemcpyAsync(static_cast<char*>(host) + off, static_cast<char*>(dev) + off, n, hipMemcpyDeviceToHost, st[k]));
                }
                for (int k = 0; k < ns; k++) CK(hipStreamSynchronize(st[k]));
                double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                if (s < best) best = s;
            }
            std::printf("%-14s memcpy streams=%d  %.2f ms  %.1f GB/s\n", f.name, ns, best * 1e3, bytes / best / 1e9);
        }
        void* hdev = nullptr;
        if (hipHostGetDevicePointer(&hdev, host, 0) == hipSuccess) {
            for (int grid : {256, 1024, 4096}) {
                double best = 1e9;
                for (int rep = 0; rep < 3; rep++) {
                    CK(hipDeviceSynchronize());
                    auto t0 = std::chrono::steady_clock::now();
                    hipLaunchKernelGGL(kcopy, dim3(grid), dim3(256), 0, st[0], (const uint4*)dev, (uint4*)hdev, bytes / 16);
                    CK(hipStreamSynchronize(st[0]));
                    double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                    if (s < best) best = s;
                }
                std::printf("%-14s kernel grid=%d  %.2f ms  %.1f GB/s\n", f.name, grid, best * 1e3, bytes / best / 1e9);
            }
        }
        CK(hipHostFree(host));
    }
    // pageable memory for reference
    std::vector<char> pageable(bytes);
    double best = 1e9;
    for (int rep = 0; rep < 2; rep++) {
        auto t0 = std::chrono::steady_clock::now();
        CK(hipMemcpy(pageable.data(), dev, bytes, hipMemcpyDeviceToHost));
        double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (s < best) best = s;
    }
    std::printf("pageable       memcpy          %.2f ms  %.1f GB/s\n", best * 1e3, bytes / best / 1e9);
    return 0;
}
