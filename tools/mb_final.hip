// Microbenchmark of the final-hop access pattern (C2 shape): E edges, four columns read per edge
// (dst, rank, filter prop p0, yielded prop p1), filter p0 < 50 (~50 %), the passing edges' rows
// (src, dst, rank, p0, p1 as int64) written densely per chunk. Variants differ only in how the columns
// are stored and loaded, to decide the final kernel's layout:
//   0  strided  : 2048-edge chunks, thread t loads edges t + 256k (8 per thread), 8-byte columns
//   1  strided  : same mapping, narrow columns (dst int32, rank int8, p0 int8, p1 int64)
//   2  blocked  : 1024-edge chunks, thread t loads edges 4t..4t+3 with 16-byte vector loads, 8-byte
//                 columns; passing rows staged in LDS and written coalesced
//   3  blocked  : as 2 with narrow columns (dst 16 B, rank 4 B, p0 4 B, p1 2 x 16 B per thread)
// The CSR here is one contiguous segment (best case: no entry boundaries inside a thread's run).
// Usage: mb_final [E_millions] [iters]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP %s at %s\n", hipGetErrorString(e_), #x); std::exit(1); } } while (0)

struct Out { int64_t *src, *dst, *rank, *p0, *p1; unsigned long long* counter; };

template <int WD, int WR, int WP>
__device__ __forceinline__ int64_t ld(const void* p, uint64_t i) {
    if constexpr (WD == 1) return static_cast<const int8_t*>(p)[i];
    else if constexpr (WD == 4) return static_cast<const int32_t*>(p)[i];
    else return static_cast<const int64_t*>(p)[i];
}

// ---------------------------------------------------------------------------------- strided
template <int WDST, int WRANK, int WP0>
__global__ __launch_bounds__(256) void k_strided(const void* dst, const void* rank, const void* p0, const int64_t* p1,
                                                 uint64_t E, Out o) {
    __shared__ uint64_t words[32];
    __shared__ uint32_t wordPre[32];
    __shared__ uint64_t sBase;
    const uint64_t base = static_cast<uint64_t>(blockIdx.x) * 2048;
    int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int64_t d[8], r[8], a[8], b[8];
    bool pass[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        uint64_t p = base + threadIdx.x + k * 256;
        pass[k] = false;
        if (p < E) {
            d[k] = ld<WDST, 0, 0>(dst, p);
            r[k] = ld<WRANK, 0, 0>(rank, p);
            a[k] = ld<WP0, 0, 0>(p0, p);
            b[k] = p1[p];
            pass[k] = a[k] < 50;
        }
    }
#pragma unroll
    for (int k = 0; k < 8; k++) {
        uint64_t bal = __ballot(pass[k]);
        if (lane == 0) words[k * 4 + wid] = bal;
    }
    __syncthreads();
    if (wid == 0) {
        uint64_t w = lane < 32 ? words[lane] : 0;
        uint32_t c = __popcll(w), x = c;
        for (int off = 1; off < 64; off <<= 1) { uint32_t y = __shfl_up(x, off, 64); if (lane >= off) x += y; }
        if (lane < 32) wordPre[lane] = x - c;
        uint32_t total = __shfl(x, 63, 64);
        if (lane == 0) sBase = atomicAdd(o.counter, static_cast<unsigned long long>(total));
    }
    __syncthreads();
    const uint64_t below = (1ULL << lane) - 1;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        if (!pass[k]) continue;
        int w = k * 4 + wid;
        uint64_t q = sBase + wordPre[w] + __popcll(words[w] & below);
        o.src[q] = static_cast<int64_t>(base + threadIdx.x + k * 256) >> 5;
        o.dst[q] = d[k];
        o.rank[q] = r[k];
        o.p0[q] = a[k];
        o.p1[q] = b[k];
    }
}

// ---------------------------------------------------------------------------------- blocked
template <int W> struct Vec4 {};                       // four consecutive elements of a W-byte column
template <> struct Vec4<8> {
    static __device__ __forceinline__ void load(const void* p, uint64_t i, int64_t* v) {
        const int4* q = reinterpret_cast<const int4*>(static_cast<const int64_t*>(p) + i);
        int4 x = q[0], y = q[1];
        v[0] = (static_cast<int64_t>(static_cast<uint32_t>(x.y)) << 32) | static_cast<uint32_t>(x.x);
        v[1] = (static_cast<int64_t>(static_cast<uint32_t>(x.w)) << 32) | static_cast<uint32_t>(x.z);
        v[2] = (static_cast<int64_t>(static_cast<uint32_t>(y.y)) << 32) | static_cast<uint32_t>(y.x);
        v[3] = (static_cast<int64_t>(static_cast<uint32_t>(y.w)) << 32) | static_cast<uint32_t>(y.z);
    }
};
template <> struct Vec4<4> {
    static __device__ __forceinline__ void load(const void* p, uint64_t i, int64_t* v) {
        int4 x = *reinterpret_cast<const int4*>(static_cast<const int32_t*>(p) + i);
        v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
    }
};
template <> struct Vec4<1> {
    static __device__ __forceinline__ void load(const void* p, uint64_t i, int64_t* v) {
        int32_t x = *reinterpret_cast<const int32_t*>(static_cast<const int8_t*>(p) + i);
        v[0] = static_cast<int8_t>(x); v[1] = static_cast<int8_t>(x >> 8);
        v[2] = static_cast<int8_t>(x >> 16); v[3] = static_cast<int8_t>(x >> 24);
    }
};

template <int WDST, int WRANK, int WP0>
__global__ __launch_bounds__(256) void k_blocked(const void* dst, const void* rank, const void* p0, const int64_t* p1,
                                                 uint64_t E, Out o) {
    constexpr int CH = 1024;
    __shared__ int64_t stage[5][CH];
    __shared__ uint32_t wsum[4];
    __shared__ uint64_t sBase;
    __shared__ uint32_t sTotal;
    const uint64_t base = static_cast<uint64_t>(blockIdx.x) * CH;
    const uint64_t p = base + threadIdx.x * 4;
    int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int64_t d[4], r[4], a[4], b[4];
    uint32_t passBits = 0;
    if (p + 4 <= E) {
        Vec4<WDST>::load(dst, p, d);
        Vec4<WRANK>::load(rank, p, r);
        Vec4<WP0>::load(p0, p, a);
        Vec4<8>::load(p1, p, b);
#pragma unroll
        for (int k = 0; k < 4; k++) passBits |= (a[k] < 50 ? 1u : 0u) << k;
    }
    uint32_t c = __popc(passBits), x = c;
    for (int off = 1; off < 64; off <<= 1) { uint32_t y = __shfl_up(x, off, 64); if (lane >= off) x += y; }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    uint32_t pre = x - c;
    for (int w = 0; w < wid; w++) pre += wsum[w];
    if (threadIdx.x == 0) {
        uint32_t t = wsum[0] + wsum[1] + wsum[2] + wsum[3];
        sTotal = t;
        sBase = atomicAdd(o.counter, static_cast<unsigned long long>(t));
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
        if (!(passBits >> k & 1)) continue;
        stage[0][pre] = static_cast<int64_t>(p + k) >> 5;
        stage[1][pre] = d[k];
        stage[2][pre] = r[k];
        stage[3][pre] = a[k];
        stage[4][pre] = b[k];
        pre++;
    }
    __syncthreads();
    const uint32_t n = sTotal;
    const uint64_t ob = sBase;
    for (uint32_t i = threadIdx.x; i < n; i += 256) {
        o.src[ob + i] = stage[0][i];
        o.dst[ob + i] = stage[1][i];
        o.rank[ob + i] = stage[2][i];
        o.p0[ob + i] = stage[3][i];
        o.p1[ob + i] = stage[4][i];
    }
}

template <typename T>
T* devFill(uint64_t n, int w, uint64_t seed, int64_t mod) {
    std::vector<T> h(n);
    uint64_t s = seed;
    for (uint64_t i = 0; i < n; i++) {
        s = s * 6364136223846793005ULL + 1442695040888963407ULL;
        int64_t v = static_cast<int64_t>(s >> 17);
        h[i] = static_cast<T>(mod ? v % mod : v);
    }
    (void)w;
    T* d;
    CK(hipMalloc(&d, n * sizeof(T)));
    CK(hipMemcpy(d, h.data(), n * sizeof(T), hipMemcpyHostToDevice));
    return d;
}

int main(int argc, char** argv) {
    uint64_t E = (argc > 1 ? std::atoll(argv[1]) : 64) * 1000000ULL;
    int iters = argc > 2 ? std::atoi(argv[2]) : 20;
    E = E / 2048 * 2048;
    int64_t* dst8 = devFill<int64_t>(E, 8, 1, 1 << 22);
    int32_t* dst4 = devFill<int32_t>(E, 4, 1, 1 << 22);
    int64_t* rank8 = devFill<int64_t>(E, 8, 2, 1);
    int8_t* rank1 = devFill<int8_t>(E, 1, 2, 1);
    int64_t* p08 = devFill<int64_t>(E, 8, 3, 100);
    int8_t* p01 = devFill<int8_t>(E, 1, 3, 100);
    int64_t* p1 = devFill<int64_t>(E, 8, 4, 0);
    Out o;
    CK(hipMalloc(&o.src, E * 8)); CK(hipMalloc(&o.dst, E * 8)); CK(hipMalloc(&o.rank, E * 8));
    CK(hipMalloc(&o.p0, E * 8)); CK(hipMalloc(&o.p1, E * 8)); CK(hipMalloc(&o.counter, 8));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    const char* names[] = {"strided-8B", "strided-narrow", "blocked-8B", "blocked-narrow"};
    for (int v = 0; v < 4; v++) {
        float best = 1e30f, sum = 0;
        unsigned long long rows = 0;
        for (int it = 0; it < iters + 3; it++) {
            CK(hipMemset(o.counter, 0, 8));
            CK(hipEventRecord(a));
            if (v == 0) hipLaunchKernelGGL((k_strided<8, 8, 8>), dim3(E / 2048), dim3(256), 0, 0, dst8, rank8, p08, p1, E, o);
            if (v == 1) hipLaunchKernelGGL((k_strided<4, 1, 1>), dim3(E / 2048), dim3(256), 0, 0, dst4, rank1, p01, p1, E, o);
            if (v == 2) hipLaunchKernelGGL((k_blocked<8, 8, 8>), dim3(E / 1024), dim3(256), 0, 0, dst8, rank8, p08, p1, E, o);
            if (v == 3) hipLaunchKernelGGL((k_blocked<4, 1, 1>), dim3(E / 1024), dim3(256), 0, 0, dst4, rank1, p01, p1, E, o);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (it >= 3) { sum += ms; best = ms < best ? ms : best; }
            CK(hipMemcpy(&rows, o.counter, 8, hipMemcpyDeviceToHost));
        }
        int rb = (v == 0 || v == 2) ? 32 : 14;
        double bytes = static_cast<double>(E) * rb + rows * 40.0;
        double algo = static_cast<double>(E) * 24 + rows * 40.0;
        std::printf("%-16s E=%llu rows=%llu avg %.1f us best %.1f us  moved %.2f GB -> %.2f TB/s  algo-frac %.3f\n",
                    names[v], static_cast<unsigned long long>(E), rows, sum / iters * 1e3, best * 1e3, bytes / 1e9,
                    bytes / (sum / iters * 1e-3) / 1e12, algo / (sum / iters * 1e-3) / 8e12);
    }
    return 0;
}
