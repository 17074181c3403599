// Microbenchmark: the real final-hop body (final_kernels.h finalBody, edge-balanced chunk map) on a
// synthetic CSR shaped like the C2 bench's last hop (E edges over nEnt frontier entries with a skewed
// degree distribution), with an evaluator equivalent to the generated one for
// `WHERE e.p0 < 50 YIELD e._dst, e._rank, e.p0, e.p1` (p0 int8, p1 int64, dst int32, rank int8),
// against the map-free strided kernel of tools/mb_final.hip reading the same bytes. The difference
// is the cost of the chunk map (entry lookup, CSR position, source vid) in the real kernel.
// Usage: mb_map [E_millions] [nEnt_thousands] [iters]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#include "../nebula_amd/csrc/final_kernels.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP %s at %s\n", hipGetErrorString(e_), #x); std::exit(1); } } while (0)

namespace ngx {

template <bool SRC>
struct MicroEv {
    static constexpr bool kPos32 = true;
    static constexpr bool kMask = false;
    static constexpr int kDstW = 4, kRankW = 1;
    static constexpr bool kDrow = false;
    static constexpr bool kFlat = SRC;
    static constexpr bool kEflags = false, kTtl = false;
    static constexpr int kEtype = 1;
    static constexpr int kEager = 2;
    static __device__ __forceinline__ bool hasP(const FinalArgs&) { return true; }
    static __device__ __forceinline__ bool hasW(const FinalArgs&) { return true; }
    static __device__ __forceinline__ Val P(const FinalArgs& a, const EdgeCtx& ec) {
        Val v0 = opEcolT<2, 1, false>(a.env, ec, 0, 1, 0, mkInt(0));
        return opRel(OP_LT, v0, Val{a.kc[0], 0u, 1});
    }
    static __device__ __forceinline__ Val W(const FinalArgs& a, const EdgeCtx& ec) { return P(a, ec); }
    static __device__ __forceinline__ void YV(const FinalArgs& a, const EdgeCtx& ec, Val* v) {
        v[0] = opEcolT<2, 1, false>(a.env, ec, 0, 1, 3, mkInt(0));
        v[1] = opEcolT<2, 8, false>(a.env, ec, 1, 1, 3, mkInt(0));
    }
    static __device__ __forceinline__ void YS(const FinalArgs& a, const Val* yv, uint64_t o, uint32_t& errs) {
        (void)errs;
        gst<int64_t>(a.oCols[2].x, o, yv[0].x);
        gst<int64_t>(a.oCols[3].x, o, yv[1].x);
    }
    static __device__ __forceinline__ void Y(const FinalArgs&, const EdgeCtx&, uint64_t, uint32_t&) {}
};

}  // namespace ngx

using namespace ngx;

template <int WAVES, bool FLAT = true>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WAVES))) void k_map(FinalArgs a) {
    finalBody<MicroEv<FLAT>, true, false, false>(a);
}
// buildMap alone (what the final kernel does before any edge load)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) void k_maponly(FinalArgs a, uint32_t* sink) {
    __shared__ ChunkMap<true, false, true> m;
    const uint64_t base = static_cast<uint64_t>(blockIdx.x) * CE;
    const uint32_t cnt = static_cast<uint32_t>(a.E - base < CE ? a.E - base : CE);
    buildMap<true, false, true>(a.estart, a.chunkFirst, a.nEnt, blockIdx.x, gridDim.x, base, cnt, a.F, a.hs, m);
    if (threadIdx.x == 0) sink[blockIdx.x] = m.at[threadIdx.x * 7] + m.row[m.at[2047]];
}

// map built; LDSPOS: per-edge CSR position from the map (else pos = base + p); VID: per-edge source vid
// gathered from vid[row] (else the first record's)
template <bool LDSPOS, bool VID>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) void k_mapdirect(FinalArgs a, int64_t* o0, int64_t* o1,
                                                                                          int64_t* o2, int64_t* o3, int64_t* o4,
                                                                                          unsigned long long* counter) {
    __shared__ ChunkMap<true, false, true> m;
    __shared__ uint64_t words[32];
    __shared__ uint32_t wordPre[32];
    __shared__ uint64_t sBase;
    const uint64_t base = static_cast<uint64_t>(blockIdx.x) * CE;
    const uint32_t cnt = static_cast<uint32_t>(a.E - base < CE ? a.E - base : CE);
    buildMap<true, false, true>(a.estart, a.chunkFirst, a.nEnt, blockIdx.x, gridDim.x, base, cnt, a.F, a.hs, m);
    const int32_t* dst = static_cast<const int32_t*>(a.hs.dst[0]);
    const int8_t* rank = static_cast<const int8_t*>(a.hs.rank[0]);
    const DCol* cols = a.env.cols;
    const int8_t* p0 = static_cast<const int8_t*>(cols[0].data);
    const int64_t* p1 = static_cast<const int64_t*>(cols[1].data);
    int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int64_t d[8], r[8], x[8], y[8];
    bool pass[8];
    int64_t src0 = a.vid[m.row[0]];
    int64_t sv[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        uint32_t pl = threadIdx.x + k * 256;
        uint64_t p = base + pl;
        pass[k] = false;
        sv[k] = src0;
        if (pl < cnt) {
            uint32_t q = m.at[pl];
            if (LDSPOS) p = static_cast<uint64_t>(static_cast<uint32_t>(p) + static_cast<uint32_t>(m.pb[q]));
            if (VID) sv[k] = a.vid[m.row[q]];
            d[k] = gld<int32_t>(dst, p); r[k] = gld<int8_t>(rank, p); x[k] = gld<int8_t>(p0, p); y[k] = gld<int64_t>(p1, p); pass[k] = x[k] < 50;
        }
    }
#pragma unroll
    for (int k = 0; k < 8; k++) { uint64_t b = __ballot(pass[k]); if (lane == 0) words[k * 4 + wid] = b; }
    __syncthreads();
    if (wid == 0) {
        uint64_t w = lane < 32 ? words[lane] : 0;
        uint32_t c = __popcll(w), xx = c;
        for (int off = 1; off < 64; off <<= 1) { uint32_t yy = __shfl_up(xx, off, 64); if (lane >= off) xx += yy; }
        if (lane < 32) wordPre[lane] = xx - c;
        uint32_t total = __shfl(xx, 63, 64);
        if (lane == 0) sBase = atomicAdd(counter, static_cast<unsigned long long>(total));
    }
    __syncthreads();
    const uint64_t below = (1ULL << lane) - 1;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        if (!pass[k]) continue;
        int w = k * 4 + wid;
        uint64_t q = sBase + wordPre[w] + __popcll(words[w] & below);
        o0[q] = sv[k]; o1[q] = d[k]; o2[q] = r[k]; o3[q] = x[k]; o4[q] = y[k];
    }
}

template <int WAVES>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WAVES))) void k_plain(const int32_t* dst, const int8_t* rank,
                                                                                           const int8_t* p0, const int64_t* p1,
                                                                                           uint64_t E, int64_t* o0, int64_t* o1,
                                                                                           int64_t* o2, int64_t* o3, int64_t* o4,
                                                                                           unsigned long long* counter) {
    __shared__ uint64_t words[32];
    __shared__ uint32_t wordPre[32];
    __shared__ uint64_t sBase;
    const uint64_t base = static_cast<uint64_t>(blockIdx.x) * 2048;
    int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int64_t d[8], r[8], x[8], y[8];
    bool pass[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        uint64_t p = base + threadIdx.x + k * 256;
        pass[k] = false;
        if (p < E) { d[k] = dst[p]; r[k] = rank[p]; x[k] = p0[p]; y[k] = p1[p]; pass[k] = x[k] < 50; }
    }
#pragma unroll
    for (int k = 0; k < 8; k++) { uint64_t b = __ballot(pass[k]); if (lane == 0) words[k * 4 + wid] = b; }
    __syncthreads();
    if (wid == 0) {
        uint64_t w = lane < 32 ? words[lane] : 0;
        uint32_t c = __popcll(w), xx = c;
        for (int off = 1; off < 64; off <<= 1) { uint32_t yy = __shfl_up(xx, off, 64); if (lane >= off) xx += yy; }
        if (lane < 32) wordPre[lane] = xx - c;
        uint32_t total = __shfl(xx, 63, 64);
        if (lane == 0) sBase = atomicAdd(counter, static_cast<unsigned long long>(total));
    }
    __syncthreads();
    const uint64_t below = (1ULL << lane) - 1;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        if (!pass[k]) continue;
        int w = k * 4 + wid;
        uint64_t q = sBase + wordPre[w] + __popcll(words[w] & below);
        o0[q] = static_cast<int64_t>(base + threadIdx.x + k * 256) >> 5;
        o1[q] = d[k]; o2[q] = r[k]; o3[q] = x[k]; o4[q] = y[k];
    }
}

template <typename T>
T* up(const std::vector<T>& h) {
    T* d;
    CK(hipMalloc(&d, std::max<size_t>(h.size(), 1) * sizeof(T)));
    if (!h.empty()) CK(hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
    return d;
}

int main(int argc, char** argv) {
    uint64_t E = (argc > 1 ? std::atoll(argv[1]) : 64) * 1000000ULL;
    uint64_t nEnt = (argc > 2 ? std::atoll(argv[2]) : 1900) * 1000ULL;
    int iters = argc > 3 ? std::atoi(argv[3]) : 20;
    std::mt19937_64 rng(42);
    // skewed degrees summing to ~E: Zipf-like weights, shuffled
    std::vector<double> w(nEnt);
    for (uint64_t i = 0; i < nEnt; i++) w[i] = 1.0 / std::pow(static_cast<double>(i + 1), 0.75);
    double ws = std::accumulate(w.begin(), w.end(), 0.0);
    std::vector<uint64_t> deg(nEnt);
    uint64_t tot = 0;
    for (uint64_t i = 0; i < nEnt; i++) { deg[i] = std::max<uint64_t>(1, static_cast<uint64_t>(w[i] / ws * E)); tot += deg[i]; }
    std::shuffle(deg.begin(), deg.end(), rng);
    E = tot;
    // CSR over V = nEnt rows (frontier = every row), off, dst int32, rank int8, p0 int8, p1 int64
    std::vector<uint64_t> off(nEnt + 1, 0);
    for (uint64_t i = 0; i < nEnt; i++) off[i + 1] = off[i] + deg[i];
    std::vector<int32_t> dst(E);
    std::vector<int8_t> rank(E, 0), p0(E);
    std::vector<int64_t> p1(E), vid(nEnt);
    std::vector<uint32_t> dgid(E);
    for (uint64_t e = 0; e < E; e++) {
        uint64_t r = rng();
        dst[e] = static_cast<int32_t>(r % (1u << 22));
        dgid[e] = static_cast<uint32_t>(r % nEnt);
        p0[e] = static_cast<int8_t>((r >> 24) % 100);
        p1[e] = static_cast<int64_t>(rng());
    }
    for (uint64_t i = 0; i < nEnt; i++) vid[i] = static_cast<int64_t>(i * 7 + 3);
    std::vector<uint32_t> F(nEnt);
    std::iota(F.begin(), F.end(), 0u);
    std::vector<uint64_t> estart(nEnt + 1);
    for (uint64_t i = 0; i <= nEnt; i++) estart[i] = off[i];
    uint64_t chunks = (E + kChunk - 1) / kChunk;
    std::vector<uint64_t> chunkFirst(chunks);
    for (uint64_t i = 0; i < nEnt; i++)
        for (uint64_t c = (estart[i] + kChunk - 1) / kChunk; c * kChunk < estart[i + 1]; c++) chunkFirst[c] = i;

    DCol cols[2] = {};
    cols[0].type = 2; cols[0].width = 1; cols[0].data = up(p0);
    cols[1].type = 2; cols[1].width = 8; cols[1].data = up(p1);
    FinalArgs a{};
    a.F = up(F); a.estart = up(estart); a.chunkFirst = up(chunkFirst); a.nEnt = nEnt; a.E = E;
    a.hs.n = 1; a.hs.slotIdx[0] = 0; a.hs.etype[0] = 1; a.hs.off[0] = up(off); a.hs.dgid[0] = up(dgid);
    a.hs.dst[0] = up(dst); a.hs.rank[0] = up(rank); a.hs.dstW[0] = 4; a.hs.rankW[0] = 1; a.hs.eflags[0] = nullptr;
    a.hs.colBase[0] = 0;
    a.vid = up(vid); a.V = nEnt; a.gbase = 0;
    a.env.cols = up(std::vector<DCol>(cols, cols + 2));
    a.propsMask = 1; a.ttlCol[0] = -1; a.wIsP = 1; a.kc[0] = 50;
    uint32_t* err; CK(hipMalloc(&err, 16)); a.err = err; a.env.unsupported = err + 1;
    int64_t *oSrc, *oDst, *oRank, *oP0, *oP1;
    CK(hipMalloc(&oSrc, E * 8)); CK(hipMalloc(&oDst, E * 8)); CK(hipMalloc(&oRank, E * 8));
    CK(hipMalloc(&oP0, E * 8)); CK(hipMalloc(&oP1, E * 8));
    OutCol oc[4] = {{oDst, nullptr, nullptr}, {oRank, nullptr, nullptr}, {oP0, nullptr, nullptr}, {oP1, nullptr, nullptr}};
    a.oCols = up(std::vector<OutCol>(oc, oc + 4));
    a.oSrc = oSrc; a.oDst = oDst; a.oRank = oRank; a.oType = nullptr; a.oEntry = nullptr;
    uint64_t* lb; CK(hipMalloc(&lb, (chunks + 2) * 8)); a.lbStatus = lb;
    hipEvent_t t0, t1;
    CK(hipEventCreate(&t0)); CK(hipEventCreate(&t1));
    const char* names[] = {"final flat", "maponly", "mapdirect", "plain w5", "map+pos", "map+vid", "map+pos+vid", "final branchy"};
    uint32_t* sink; CK(hipMalloc(&sink, chunks * 4));
    for (int v = 0; v < 8; v++) {
        double sum = 0;
        uint64_t rows = 0;
        for (int it = 0; it < iters + 3; it++) {
            CK(hipMemset(lb, 0, (chunks + 2) * 8));
            CK(hipEventRecord(t0));
            if (v == 0) hipLaunchKernelGGL((k_map<5, true>), dim3(chunks), dim3(256), 0, 0, a);
            if (v == 7) hipLaunchKernelGGL((k_map<5, false>), dim3(chunks), dim3(256), 0, 0, a);
            if (v == 1) hipLaunchKernelGGL(k_maponly, dim3(chunks), dim3(256), 0, 0, a, sink);
            auto* lbc = reinterpret_cast<unsigned long long*>(lb);
            if (v == 2) hipLaunchKernelGGL((k_mapdirect<false, false>), dim3(chunks), dim3(256), 0, 0, a, oSrc, oDst, oRank, oP0, oP1, lbc);
            if (v == 4) hipLaunchKernelGGL((k_mapdirect<true, false>), dim3(chunks), dim3(256), 0, 0, a, oSrc, oDst, oRank, oP0, oP1, lbc);
            if (v == 5) hipLaunchKernelGGL((k_mapdirect<false, true>), dim3(chunks), dim3(256), 0, 0, a, oSrc, oDst, oRank, oP0, oP1, lbc);
            if (v == 6) hipLaunchKernelGGL((k_mapdirect<true, true>), dim3(chunks), dim3(256), 0, 0, a, oSrc, oDst, oRank, oP0, oP1, lbc);
            if (v == 3) {
                const int32_t* dd = static_cast<const int32_t*>(a.hs.dst[0]);
                const int8_t* rr = static_cast<const int8_t*>(a.hs.rank[0]);
                const int8_t* pp = static_cast<const int8_t*>(cols[0].data);
                const int64_t* qq = static_cast<const int64_t*>(cols[1].data);
                unsigned long long* cnt = reinterpret_cast<unsigned long long*>(lb);
                hipLaunchKernelGGL((k_plain<5>), dim3(chunks), dim3(256), 0, 0, dd, rr, pp, qq, E, oSrc, oDst, oRank, oP0, oP1, cnt);
            }
            CK(hipEventRecord(t1));
            CK(hipEventSynchronize(t1));
            float ms;
            CK(hipEventElapsedTime(&ms, t0, t1));
            if (it >= 3) sum += ms;
            CK(hipMemcpy(&rows, lb, 8, hipMemcpyDeviceToHost));
        }
        double us = sum / iters * 1e3;
        double moved = E * 14.0 + rows * 40.0;
        std::printf("%-10s E=%llu nEnt=%llu rows=%llu avg %.1f us  moved(min) %.2f GB -> %.2f TB/s  algo-frac %.3f\n",
                    names[v], (unsigned long long)E, (unsigned long long)nEnt, (unsigned long long)rows, us, moved / 1e9,
                    moved / (us * 1e-6) / 1e12, (E * 24.0 + rows * 40.0) / (us * 1e-6) / 8e12);
    }
    return 0;
}
