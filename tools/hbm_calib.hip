// HBM counter calibration for the final hop's access widths.
//
// MI355X_MICROARCH.md (HBM section) calibrates FETCH_SIZE only for 16-B-per-lane streaming reads (it
// reports half the bytes) and WRITE_SIZE only for 16-B streaming stores; every other width is
// "uncalibrated". The final hop (final_kernels.h) reads 4-B dst / 1-B p0 columns per lane in CSR order,
// 8-B p1 values for the ~half of the edges that pass the filter, and writes 1/4/8-B row columns in
// order. This program runs each of those patterns as its own kernel over buffers far larger than the
// 256 MiB Infinity Cache, with a known byte count, so that one rocprofv3 --pmc pass per counter gives
// counter / known bytes per pattern (tools/calib_summary.py). It also prints the HIP-event bandwidth
// of each pattern: the ceiling a kernel built from that access can reach.
//
// Build: tools/build_calib.sh (hipcc --offload-arch=gfx950). Run: tools/calib.sh on the GPU box.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                \
        }                                                                                \
    } while (0)

constexpr int WG = 256;

__device__ __forceinline__ uint32_t passHash(uint64_t i) {     // ~half the positions pass
    uint64_t x = i * 0x9e3779b97f4a7c15ULL;
    x ^= x >> 29;
    return static_cast<uint32_t>(x >> 40) & 1u;
}

// streaming reads, T per lane, consecutive lanes on consecutive elements, grid-stride; the xor of the
// values is stored only if it equals a key the compiler cannot see (the caller passes one no xor
// reaches), so no load is dead
template <class T>
__device__ __forceinline__ uint64_t fold(const T& v) { return static_cast<uint64_t>(v); }
template <>
__device__ __forceinline__ uint64_t fold<uint4>(const uint4& v) { return (static_cast<uint64_t>(v.x ^ v.z) << 32) | (v.y ^ v.w); }

#define READ_KERNEL(NAME, T)                                                                 \
    __global__ __launch_bounds__(WG) void NAME(const T* __restrict__ p, uint64_t n, uint64_t* sink, uint64_t key) { \
        uint64_t acc = 0;                                                                    \
        const uint64_t stride = static_cast<uint64_t>(gridDim.x) * WG;                        \
        uint64_t i = static_cast<uint64_t>(blockIdx.x) * WG + threadIdx.x;                    \
        for (; i + 3 * stride < n; i += 4 * stride) {                                        \
            T a = p[i], b = p[i + stride], c = p[i + 2 * stride], d = p[i + 3 * stride];     \
            acc ^= fold(a) ^ fold(b) ^ fold(c) ^ fold(d);                                    \
        }                                                                                    \
        for (; i < n; i += stride) acc ^= fold(p[i]);                                        \
        if (acc == key) sink[0] = acc;                                                       \
    }
READ_KERNEL(k_calib_read16, uint4)
READ_KERNEL(k_calib_read8, uint64_t)
READ_KERNEL(k_calib_read4, uint32_t)
READ_KERNEL(k_calib_read1, uint8_t)

// the p1 pattern: 8-B values at the ~half of the positions that pass (lanes in order, holes random)
__global__ __launch_bounds__(WG) void k_calib_gather8_half(const uint64_t* __restrict__ p, uint64_t n, uint64_t* sink, uint64_t key) {
    uint64_t acc = 0;
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * WG;
    for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * WG + threadIdx.x; i < n; i += stride)
        if (passHash(i)) acc ^= p[i];
    if (acc == key) sink[0] = acc;
}

#define WRITE_KERNEL(NAME, T)                                                                \
    __global__ __launch_bounds__(WG) void NAME(T* __restrict__ p, uint64_t n, uint64_t seed) { \
        const uint64_t stride = static_cast<uint64_t>(gridDim.x) * WG;                        \
        for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * WG + threadIdx.x; i < n; i += stride) \
            p[i] = static_cast<T>(i ^ seed);                                                 \
    }
WRITE_KERNEL(k_calib_write8, uint64_t)
WRITE_KERNEL(k_calib_write4, uint32_t)
WRITE_KERNEL(k_calib_write1, uint8_t)

__global__ __launch_bounds__(WG) void k_calib_write16(uint4* __restrict__ p, uint64_t n, uint64_t seed) {
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * WG;
    for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * WG + threadIdx.x; i < n; i += stride) {
        const uint32_t v = static_cast<uint32_t>(i ^ seed);
        p[i] = make_uint4(v, v + 1, v + 2, v + 3);
    }
}

// the final hop's access mix without its chunk map or row reservation: per edge a 4-B dst and a 1-B p0
// in CSR order; the ~half of the edges that pass read their 8-B p1 and write an 18-B row (4-B src, 4-B
// dst, 1-B rank, 1-B p0, 8-B p1) into five column arrays, contiguous inside the workgroup's 4096-edge
// chunk (each chunk owns the output range of its edges: no global allocation). The time of this kernel
// at C2's last-hop size is the ceiling the final hop could reach with its bytes.
constexpr int MIX_ITEMS = 16, MIX_CHUNK = WG * MIX_ITEMS;
__global__ __launch_bounds__(WG) void k_calib_finalmix(const uint32_t* __restrict__ dst, const uint8_t* __restrict__ p0,
                                                       const uint64_t* __restrict__ p1, uint64_t n,
                                                       uint32_t* oSrc, uint32_t* oDst, uint8_t* oRank, uint8_t* oP0,
                                                       uint64_t* oP1) {
    __shared__ uint32_t cnt[MIX_ITEMS][WG / 64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint64_t base = static_cast<uint64_t>(blockIdx.x) * MIX_CHUNK;
    uint32_t d[MIX_ITEMS];
    uint8_t q[MIX_ITEMS];
    bool pass[MIX_ITEMS];
#pragma unroll
    for (int k = 0; k < MIX_ITEMS; k++) {
        const uint64_t e = base + k * WG + threadIdx.x;
        const uint64_t c = e < n ? e : n - 1;
        d[k] = dst[c];
        q[k] = p0[c];
    }
#pragma unroll
    for (int k = 0; k < MIX_ITEMS; k++) {
        const uint64_t e = base + k * WG + threadIdx.x;
        pass[k] = e < n && (((q[k] ^ passHash(e)) & 1u) != 0);
        const uint64_t b = __ballot(pass[k]);
        if (lane == 0) cnt[k][wid] = static_cast<uint32_t>(__popcll(b));
    }
    __syncthreads();
    uint32_t run = 0, start[MIX_ITEMS];
    for (int k = 0; k < MIX_ITEMS; k++)
        for (int w = 0; w < WG / 64; w++) {
            if (w == wid) start[k] = run;
            run += cnt[k][w];
        }
    const uint64_t below = (1ULL << lane) - 1;
    uint64_t v[MIX_ITEMS];
#pragma unroll
    for (int k = 0; k < MIX_ITEMS; k++) v[k] = pass[k] ? p1[base + k * WG + threadIdx.x] : 0;
#pragma unroll
    for (int k = 0; k < MIX_ITEMS; k++) {
        const uint64_t b = __ballot(pass[k]);
        if (!pass[k]) continue;
        const uint64_t r = base + start[k] + __popcll(b & below);
        oSrc[r] = static_cast<uint32_t>(base >> 4);
        oDst[r] = d[k];
        oRank[r] = 0;
        oP0[r] = q[k];
        oP1[r] = v[k];
    }
}

// The same mix with wide accesses: a lane takes 4 consecutive edges per round (dst as one 16-B load,
// p0 as one 4-B load), and the chunk's rows are staged in LDS, then copied out column by column with
// 16-B stores (the real final hop cannot use the wide loads across entry boundaries, so this bounds
// what access width alone could buy).
constexpr int WMIX_CHUNK = 2048, WMIX_R = WMIX_CHUNK / (WG * 4);     // 2 rounds of 4 edges per lane
__global__ __launch_bounds__(WG) void k_calib_finalmix_wide(const uint32_t* __restrict__ dst, const uint8_t* __restrict__ p0,
                                                            const uint64_t* __restrict__ p1, uint64_t n,
                                                            uint32_t* oSrc, uint32_t* oDst, uint8_t* oRank, uint8_t* oP0,
                                                            uint64_t* oP1) {
    __shared__ uint64_t sP1[WMIX_CHUNK];
    __shared__ uint32_t sDst[WMIX_CHUNK];
    __shared__ uint8_t sP0[WMIX_CHUNK];
    __shared__ uint32_t cnt[WG];
    const uint64_t base = static_cast<uint64_t>(blockIdx.x) * WMIX_CHUNK;
    if (base + WMIX_CHUNK > n) return;                        // whole chunks only (n is a multiple)
    uint4 d[WMIX_R];
    uint32_t q[WMIX_R];
#pragma unroll
    for (int j = 0; j < WMIX_R; j++) {
        const uint64_t e = base + (static_cast<uint64_t>(j) * WG + threadIdx.x) * 4;
        d[j] = *reinterpret_cast<const uint4*>(dst + e);
        q[j] = *reinterpret_cast<const uint32_t*>(p0 + e);
    }
    uint32_t passBits = 0, c = 0;
#pragma unroll
    for (int j = 0; j < WMIX_R; j++)
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint64_t e = base + (static_cast<uint64_t>(j) * WG + threadIdx.x) * 4 + k;
            const uint32_t b = (((q[j] >> (8 * k)) ^ passHash(e)) & 1u);
            passBits |= b << (j * 4 + k);
            c += b;
        }
    uint64_t v[WMIX_R * 4];
#pragma unroll
    for (int j = 0; j < WMIX_R; j++)
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint64_t e = base + (static_cast<uint64_t>(j) * WG + threadIdx.x) * 4 + k;
            v[j * 4 + k] = (passBits >> (j * 4 + k)) & 1u ? p1[e] : 0;
        }
    // block exclusive scan of the per-thread counts (rows leave in thread order)
    cnt[threadIdx.x] = c;
    __syncthreads();
    for (int o = 1; o < WG; o <<= 1) {
        const uint32_t y = threadIdx.x >= static_cast<unsigned>(o) ? cnt[threadIdx.x - o] : 0;
        __syncthreads();
        cnt[threadIdx.x] += y;
        __syncthreads();
    }
    const uint32_t total = cnt[WG - 1];
    uint32_t r = cnt[threadIdx.x] - c;
#pragma unroll
    for (int j = 0; j < WMIX_R; j++)
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if (!((passBits >> (j * 4 + k)) & 1u)) continue;
            const uint32_t dv = k == 0 ? d[j].x : k == 1 ? d[j].y : k == 2 ? d[j].z : d[j].w;
            sDst[r] = dv;
            sP0[r] = static_cast<uint8_t>(q[j] >> (8 * k));
            sP1[r] = v[j * 4 + k];
            r++;
        }
    __syncthreads();
    // copy out, 16 B per lane per column (rows [base, base + total) of the chunk's own range)
    const uint64_t o = base;
    const uint32_t src = static_cast<uint32_t>(base >> 4);
    for (uint32_t i = threadIdx.x * 4; i < total; i += WG * 4) {
        if (i + 4 <= total) {
            *reinterpret_cast<uint4*>(oDst + o + i) = *reinterpret_cast<const uint4*>(sDst + i);
            *reinterpret_cast<uint4*>(oSrc + o + i) = make_uint4(src, src, src, src);
        } else {
            for (uint32_t t = i; t < total; t++) { oDst[o + t] = sDst[t]; oSrc[o + t] = src; }
        }
    }
    for (uint32_t i = threadIdx.x * 16; i < total; i += WG * 16) {
        if (i + 16 <= total) {
            *reinterpret_cast<uint4*>(oP0 + o + i) = *reinterpret_cast<const uint4*>(sP0 + i);
            *reinterpret_cast<uint4*>(oRank + o + i) = make_uint4(0, 0, 0, 0);
        } else {
            for (uint32_t t = i; t < total; t++) { oP0[o + t] = sP0[t]; oRank[o + t] = 0; }
        }
    }
    for (uint32_t i = threadIdx.x * 2; i < total; i += WG * 2) {
        if (i + 2 <= total) *reinterpret_cast<uint4*>(oP1 + o + i) = *reinterpret_cast<const uint4*>(sP1 + i);
        else oP1[o + i] = sP1[i];
    }
}

int main(int argc, char** argv) {
    const uint64_t bytes = (argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 2048ULL) << 20;   // MiB
    const int reps = argc > 2 ? std::atoi(argv[2]) : 3;
    const uint64_t key = argc > 3 ? std::strtoull(argv[3], nullptr, 16) : 0x5a5a5a5a5a5a5a5aULL;
    const unsigned grid = 256 * 8 * 4;                     // 8 workgroups per CU... x4: far more than 256 CUs
    uint8_t *src = nullptr, *dst = nullptr;
    uint64_t* sink = nullptr;
    CK(hipMalloc(&src, bytes));
    CK(hipMalloc(&dst, bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(src, 0x11, bytes));
    CK(hipMemset(dst, 0, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    struct Pat { const char* name; int kind; };            // kind: read width, 100 + write width, 200 gather
    const Pat pats[] = {{"k_calib_read16", 16}, {"k_calib_read8", 8}, {"k_calib_read4", 4}, {"k_calib_read1", 1},
                        {"k_calib_gather8_half", 200}, {"k_calib_write16", 116}, {"k_calib_write8", 108},
                        {"k_calib_write4", 104}, {"k_calib_write1", 101}};
    std::printf("{\"buffer_bytes\": %llu, \"reps\": %d, \"patterns\": [\n", static_cast<unsigned long long>(bytes), reps);
    bool first = true;
    for (const Pat& pt : pats) {
        float best = 1e30f;
        for (int r = 0; r < reps; r++) {
            CK(hipEventRecord(e0, 0));
            switch (pt.kind) {
                case 16: hipLaunchKernelGGL(k_calib_read16, grid, WG, 0, 0, reinterpret_cast<uint4*>(src), bytes / 16, sink, key); break;
                case 8: hipLaunchKernelGGL(k_calib_read8, grid, WG, 0, 0, reinterpret_cast<uint64_t*>(src), bytes / 8, sink, key); break;
                case 4: hipLaunchKernelGGL(k_calib_read4, grid, WG, 0, 0, reinterpret_cast<uint32_t*>(src), bytes / 4, sink, key); break;
                case 1: hipLaunchKernelGGL(k_calib_read1, grid, WG, 0, 0, src, bytes, sink, key); break;
                case 200: hipLaunchKernelGGL(k_calib_gather8_half, grid, WG, 0, 0, reinterpret_cast<uint64_t*>(src), bytes / 8, sink, key); break;
                case 116: hipLaunchKernelGGL(k_calib_write16, grid, WG, 0, 0, reinterpret_cast<uint4*>(dst), bytes / 16, r); break;
                case 108: hipLaunchKernelGGL(k_calib_write8, grid, WG, 0, 0, reinterpret_cast<uint64_t*>(dst), bytes / 8, r); break;
                case 104: hipLaunchKernelGGL(k_calib_write4, grid, WG, 0, 0, reinterpret_cast<uint32_t*>(dst), bytes / 4, r); break;
                case 101: hipLaunchKernelGGL(k_calib_write1, grid, WG, 0, 0, dst, bytes, r); break;
            }
            CK(hipGetLastError());
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
        }
        // known bytes: every element once; the gather's compulsory bytes are the 128-B lines it touches
        // (all of them at a 1/2 pass rate) and its requested bytes are half the buffer
        const bool write = pt.kind > 100 && pt.kind < 200;
        std::printf("%s {\"kernel\": \"%s\", \"dir\": \"%s\", \"width\": %d, \"known_bytes\": %llu, "
                    "\"requested_bytes\": %llu, \"best_ms\": %.4f, \"GBps\": %.1f}",
                    first ? " " : ",\n ", pt.name, write ? "write" : "read", pt.kind == 200 ? 8 : pt.kind % 100,
                    static_cast<unsigned long long>(bytes),
                    static_cast<unsigned long long>(pt.kind == 200 ? bytes / 2 : bytes), best,
                    bytes / (best * 1e-3) / 1e9);
        first = false;
    }
    {
        // the mix at C2's last hop: 64 M edges
        const uint64_t n = 64ULL << 20;
        uint32_t *dd = nullptr, *os = nullptr, *od = nullptr;
        uint8_t *pp0 = nullptr, *orank = nullptr, *op0 = nullptr;
        uint64_t *pp1 = nullptr, *op1 = nullptr;
        CK(hipMalloc(&dd, n * 4));
        CK(hipMalloc(&pp0, n));
        CK(hipMalloc(&pp1, n * 8));
        CK(hipMalloc(&os, n * 4));
        CK(hipMalloc(&od, n * 4));
        CK(hipMalloc(&orank, n));
        CK(hipMalloc(&op0, n));
        CK(hipMalloc(&op1, n * 8));
        CK(hipMemset(dd, 0x22, n * 4));
        CK(hipMemset(pp0, 0x11, n));
        CK(hipMemset(pp1, 0x33, n * 8));
        const unsigned g = static_cast<unsigned>((n + MIX_CHUNK - 1) / MIX_CHUNK);
        float best = 1e30f;
        for (int r = 0; r < reps; r++) {
            CK(hipMemset(dst, r, 256ULL << 20));              // evict: the mix's arrays leave the Infinity Cache
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(k_calib_finalmix, g, WG, 0, 0, dd, pp0, pp1, n, os, od, orank, op0, op1);
            CK(hipGetLastError());
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
        }
        // compulsory: dst + p0 streamed, every p1 line touched, 18 B per passing row (~n / 2)
        const uint64_t rd = n * 4 + n + n * 8, wr = n / 2 * 18;
        std::printf(",\n  {\"kernel\": \"k_calib_finalmix\", \"dir\": \"mix\", \"width\": 0, \"edges\": %llu, "
                    "\"known_read_bytes\": %llu, \"known_write_bytes\": %llu, \"best_ms\": %.4f, \"GBps\": %.1f}",
                    static_cast<unsigned long long>(n), static_cast<unsigned long long>(rd),
                    static_cast<unsigned long long>(wr), best, (rd + wr) / (best * 1e-3) / 1e9);
        best = 1e30f;
        const unsigned gw = static_cast<unsigned>(n / WMIX_CHUNK);
        for (int r = 0; r < reps; r++) {
            CK(hipMemset(dst, r, 256ULL << 20));
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(k_calib_finalmix_wide, gw, WG, 0, 0, dd, pp0, pp1, n, os, od, orank, op0, op1);
            CK(hipGetLastError());
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
        }
        std::printf(",\n  {\"kernel\": \"k_calib_finalmix_wide\", \"dir\": \"mix\", \"width\": 16, \"edges\": %llu, "
                    "\"known_read_bytes\": %llu, \"known_write_bytes\": %llu, \"best_ms\": %.4f, \"GBps\": %.1f}",
                    static_cast<unsigned long long>(n), static_cast<unsigned long long>(rd),
                    static_cast<unsigned long long>(wr), best, (rd + wr) / (best * 1e-3) / 1e9);
        for (void* p : {static_cast<void*>(dd), static_cast<void*>(pp0), static_cast<void*>(pp1), static_cast<void*>(os),
                        static_cast<void*>(od), static_cast<void*>(orank), static_cast<void*>(op0), static_cast<void*>(op1)})
            CK(hipFree(p));
    }
    std::printf("\n]}\n");
    CK(hipFree(src));
    CK(hipFree(dst));
    CK(hipFree(sink));
    return 0;
}
