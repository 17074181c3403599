// Microbenchmark: the intermediate-hop kernels of kernels.hip (compaction count + write, pull head +
// segment pass) on a synthetic shard shaped like the C2 bench (V rows, RMAT-like skewed degrees), run
// back to back with warm caches and, separately, right after a kernel that dirties the mark array the
// way the push expansion does; plus an empty launch as the floor. Separates what a kernel costs by
// itself from what it pays for its place in the hop sequence (cold lines, dirty lines, clocks).
// Usage: mb_hops [V_millions] [marked_fraction] [iters]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../nebula_amd/csrc/kernels.hip"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP %s at %s\n", hipGetErrorString(e_), #x); std::exit(1); } } while (0)

__global__ void k_empty() {}
__global__ void k_dirty(uint8_t* marks, uint64_t V, uint8_t ep, uint32_t step) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    const uint64_t r = (i * 2654435761ULL + step) % V;
    if (i < V / 16) marks[r] = static_cast<uint8_t>(marks[r] == ep ? ep : marks[r]);
}

template <typename T>
T* dev(const std::vector<T>& h) {
    T* p = nullptr;
    CK(hipMalloc(&p, h.size() * sizeof(T) + 64));
    CK(hipMemcpy(p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
    return p;
}

int main(int argc, char** argv) {
    using namespace ngx;
    const double vm = argc > 1 ? std::atof(argv[1]) : 2.4;
    const double frac = argc > 2 ? std::atof(argv[2]) : 0.017;
    const int iters = argc > 3 ? std::atoi(argv[3]) : 50;
    const uint64_t V = static_cast<uint64_t>(vm * 1e6);
    std::mt19937_64 rng(42);
    // degrees: a power-law-ish mix (mean ~27)
    std::vector<uint64_t> off(V + 1, 0);
    for (uint64_t r = 0; r < V; r++) {
        const double u = std::uniform_real_distribution<double>(0, 1)(rng);
        off[r + 1] = off[r] + static_cast<uint64_t>(std::min(20000.0, 4.0 / std::pow(u + 1e-6, 0.7)));
    }
    std::vector<uint8_t> marks(V, 0);
    for (uint64_t r = 0; r < V; r++) marks[r] = std::uniform_real_distribution<double>(0, 1)(rng) < frac ? 1 : 0;
    const uint64_t E = off[V];
    std::printf("V %lu, E %lu, marked %.3f\n", V, E, frac);
    uint64_t* dOff = dev(off);
    uint8_t* dMarks = dev(marks);
    const uint64_t nt = (V + TILE - 1) / TILE;
    std::vector<uint32_t> F(V);
    std::vector<uint64_t> est(V + 1), cf(E / kChunk + 2), tile(nt + 1), wave(4 * nt + 4), bits(V / 64 + 2), misc(4096);
    uint32_t* dF = dev(F);
    uint64_t *dEst = dev(est), *dCf = dev(cf), *dTile = dev(tile), *dWave = dev(wave), *dBits = dev(bits), *dMisc = dev(misc);
    uint32_t* dErr = reinterpret_cast<uint32_t*>(dMisc + 1024);
    CompactArgs a{};
    a.visited = dMarks; a.V = V;
    a.hs.n = 1; a.hs.off[0] = dOff;
    a.outF = dF; a.estart = dEst; a.chunkFirst = dCf; a.cfCap = cf.size(); a.tileSum = dTile; a.waveSum = dWave;
    a.total = dMisc; a.pub = Publish{nullptr, 0}; a.zero = dMisc + 8; a.nzero = 0; a.err = dErr; a.epoch = 1;
    a.bits = dBits;
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeIt = [&](const char* what, auto&& f) {
        for (int i = 0; i < 3; i++) f(i);
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < iters; i++) f(i);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("  %-44s %8.2f us per iteration\n", what, ms * 1e3 / iters);
    };
    timeIt("empty launch (1 WG)", [&](int) { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s); });
    timeIt("empty launch (586 WG)", [&](int) { hipLaunchKernelGGL(k_empty, dim3(nt), dim3(256), 0, s); });
    timeIt("dirty kernel alone", [&](int i) {
        hipLaunchKernelGGL(k_dirty, dim3((V / 16 + 255) / 256), dim3(256), 0, s, dMarks, V, 1, i);
    });
    timeIt("compact count", [&](int) { hipLaunchKernelGGL(k_compact_count<true>, dim3(nt), dim3(WG), 0, s, a); });
    timeIt("compact write", [&](int) { hipLaunchKernelGGL(k_compact_write<true>, dim3(nt), dim3(WG), 0, s, a); });
    timeIt("compact count + write", [&](int) { launchCompactLb(a, s); });
    timeIt("dirty + compact count + write", [&](int i) {
        hipLaunchKernelGGL(k_dirty, dim3((V / 16 + 255) / 256), dim3(256), 0, s, dMarks, V, 1, i);
        launchCompactLb(a, s);
    });
    CK(hipMemcpy(misc.data(), dMisc, 64, hipMemcpyDeviceToHost));
    std::printf("  total rows %lu, edges %lu\n", misc[0] >> kFdShift, misc[0] & kFdMask);
    return 0;
}
