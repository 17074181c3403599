// HIP kernels of the GetNeighbors / GO path on gfx950 (MI355X), and their host launchers.
//
//  * k_lookup           seed (part, vid) -> vertex row, binary search of the sorted vertex table
//  * tile scans         3-phase reduce-then-scan (tile = 256 threads x 16 items) used for entry
//                       degrees (CSR offsets of the frontier) and for frontier compaction
//  * k_chunk_first      per 2048-edge chunk of a hop: the frontier entry holding its first edge
//  * k_expand_mark      intermediate hop: edge-balanced expansion. A workgroup owns 2048 consecutive
//                       frontier edges whatever their vertices' degrees (a supernode spreads over
//                       many workgroups, a thread never loops over a whole adjacency); the entry
//                       records of the chunk are staged in LDS (final_kernels.h buildMap); each
//                       edge reads one 4-byte destination row id (coalesced) and marks the
//                       destination in an epoch byte array = the hop's frontier dedup
//  * k_compact          visited[row] == epoch -> next frontier (ballot-free tile compaction)
//  * k_final            last hop in one pass: storage filter (pushdown) + graphd WHERE through the
//                       bytecode VM, wave-ballot pass masks, decoupled look-back over the chunks'
//                       pass counts, rows + columnar YIELD cells of passing edges written densely
//                       (deterministic order)
//  * k_pack / k_merge   multi-GPU frontier exchange: epoch marks -> per-peer bitmaps and back
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <algorithm>

#include "kernels.h"
#include "final_kernels.h"
#include "rowcodec.h"

namespace ngx {

// ------------------------------------------------------------------------------ 3-phase scans
struct DegreeIn {                // degree of frontier entry i = (frontier row i / ns, slot i % ns)
    const uint32_t* F;
    HopSlots hs;
    __device__ __forceinline__ uint64_t operator()(uint64_t i) const {
        uint32_t r = F[i / hs.n];
        if (r == kNoRow) return 0;
        const uint64_t* off = hs.off[i % hs.n];
        return off[r + 1] - off[r];
    }
};
struct FlagIn {                  // visited[gbase + r] == epoch
    const uint8_t* visited;
    uint64_t gbase;
    uint8_t epoch;
    __device__ __forceinline__ uint64_t operator()(uint64_t r) const { return visited[gbase + r] == epoch ? 1 : 0; }
};
struct WriteEstart {
    uint64_t* estart;
    __device__ __forceinline__ void operator()(uint64_t i, uint64_t v, uint64_t pre) const { (void)v; estart[i] = pre; }
};
struct WriteCompact {
    uint32_t* out;
    __device__ __forceinline__ void operator()(uint64_t i, uint64_t v, uint64_t pre) const { if (v) out[pre] = static_cast<uint32_t>(i); }
};

// Fused compaction + next-hop degree scan: one scan over the shard's rows of the pair
// (1 if visited[row] == epoch, the row's degree over the hop's slots), packed as count << kFdShift | degree
// (host guarantees V < 2^(64 - kFdShift) rows and E < 2^kFdShift edges). The write phase stores the
// next frontier row AND its entries' estart, so the next hop needs no separate degree scan and the
// host reads |F| and E together in one round trip.
struct FlagDegIn {
    const uint8_t* visited;
    uint64_t gbase;
    uint8_t epoch;
    HopSlots hs;
    __device__ __forceinline__ uint64_t operator()(uint64_t r) const {
        if (visited[gbase + r] != epoch) return 0;
        uint64_t d = 0;
        for (int s = 0; s < hs.n; s++) d += hs.off[s][r + 1] - hs.off[s][r];
        return (1ULL << kFdShift) | d;
    }
};
struct WriteCompactEstart {
    uint32_t* out;
    uint64_t* estart;
    HopSlots hs;
    __device__ __forceinline__ void operator()(uint64_t r, uint64_t v, uint64_t pre) const {
        if (!v) return;
        uint64_t f = pre >> kFdShift, e = pre & kFdMask;
        out[f] = static_cast<uint32_t>(r);
        for (int s = 0; s < hs.n; s++) {
            estart[f * hs.n + s] = e;
            e += hs.off[s][r + 1] - hs.off[s][r];
        }
    }
};

template <class In>
__global__ __launch_bounds__(WG) void k_tile_reduce(In in, uint64_t n, uint64_t* tileSums) {
    __shared__ uint64_t sm[NW + 1];
    uint64_t base = static_cast<uint64_t>(blockIdx.x) * TILE + static_cast<uint64_t>(threadIdx.x) * ITEMS;
    uint64_t s = 0;
#pragma unroll 4
    for (int k = 0; k < ITEMS; k++) if (base + k < n) s += in(base + k);
    uint64_t t = blockSum(s, sm);
    if (threadIdx.x == 0) tileSums[blockIdx.x] = t;
}

// tail != nullptr (fused compaction): also writes estart[|F| * ns] = E from the packed total
// pub.slot != nullptr: the total is also published to host-mapped memory (value, then the sequence
// number with a system-scope release store), so the host learns it while the scan's last phase runs
__global__ __launch_bounds__(1024) void k_scan_tiles(uint64_t* sums, uint64_t nt, uint64_t* total, uint64_t* tail, int ns,
                                                     Publish pub) {
    __shared__ uint64_t sm[1024 / 64 + 1];
    uint64_t per = (nt + 1023) / 1024;
    uint64_t lo = threadIdx.x * per, hi = lo + per < nt ? lo + per : nt;
    uint64_t s = 0;
    for (uint64_t i = lo; i < hi; i++) s += sums[i];
    // block exclusive scan over 1024 threads
    int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint64_t x = s;
    for (int o = 1; o < 64; o <<= 1) {
        uint64_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) sm[wid] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t acc = 0;
        for (int w = 0; w < 16; w++) { uint64_t t = sm[w]; sm[w] = acc; acc += t; }
        sm[16] = acc;
    }
    __syncthreads();
    uint64_t pre = sm[wid] + x - s;
    for (uint64_t i = lo; i < hi; i++) { uint64_t t = sums[i]; sums[i] = pre; pre += t; }
    if (threadIdx.x == 0) {
        *total = sm[16];
        if (tail) tail[(sm[16] >> kFdShift) * static_cast<uint64_t>(ns)] = sm[16] & kFdMask;
        if (pub.slot) publishWords(pub.slot, pub.seq, sm[16], 0);
    }
}

template <class In, class Out>
__global__ __launch_bounds__(WG) void k_tile_scan(In in, uint64_t n, const uint64_t* tileOff, Out out) {
    __shared__ uint64_t sm[NW + 1];
    uint64_t base = static_cast<uint64_t>(blockIdx.x) * TILE + static_cast<uint64_t>(threadIdx.x) * ITEMS;
    uint64_t v[ITEMS];
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < ITEMS; k++) { v[k] = base + k < n ? in(base + k) : 0; s += v[k]; }
    uint64_t tot;
    uint64_t pre = blockExScan(s, tot, sm) + tileOff[blockIdx.x];
#pragma unroll
    for (int k = 0; k < ITEMS; k++) {
        if (base + k < n) out(base + k, v[k], pre);
        pre += v[k];
    }
}

template <class In, class Out>
static int scan3(In in, uint64_t n, Out out, uint64_t* tileSums, uint64_t* total, hipStream_t s,
                 uint64_t* tail = nullptr, int ns = 0, Publish pub = Publish{nullptr, 0}) {
    uint64_t nt = (n + TILE - 1) / TILE;
    if (nt == 0) {                       // empty input: the 1-tile scan of nothing publishes 0 below
        nt = 1;
        n = 0;
    }
    hipLaunchKernelGGL(k_tile_reduce<In>, dim3(static_cast<unsigned>(nt)), dim3(WG), 0, s, in, n, tileSums);
    hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(1024), 0, s, tileSums, nt, total, tail, ns, pub);
    hipLaunchKernelGGL((k_tile_scan<In, Out>), dim3(static_cast<unsigned>(nt)), dim3(WG), 0, s, in, n, tileSums, out);
    return static_cast<int>(hipGetLastError());
}

// ------------------------------------------------------------------------------ seeds
__global__ void k_lookup(const int32_t* qpart, const int64_t* qvid, uint64_t n, const int32_t* vpart,
                         const int64_t* vid, uint64_t V, uint32_t* out) {
    uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int32_t p = qpart[i];
    int64_t v = qvid[i];
    uint64_t lo = 0, hi = V;
    while (lo < hi) {
        uint64_t mid = (lo + hi) >> 1;
        bool less = vpart[mid] < p || (vpart[mid] == p && vid[mid] < v);
        if (less) lo = mid + 1; else hi = mid;
    }
    out[i] = (lo < V && vpart[lo] == p && vid[lo] == v) ? static_cast<uint32_t>(lo) : kNoRow;
}

// linear probing, two slots per round trip: both loads issue before either is compared (most keys
// resolve in the first pair at the index's load factor)
// Two slots per round trip, each one 16-byte load, both issued before either is examined, and the
// outcome picked by selects (a probe written with early returns let the compiler split each slot
// into a row load and a key load behind branches: four dependent loads per probe pair, r04 ISA).
__device__ __forceinline__ uint4 vindexSlot(const VIndex& idx, uint64_t h) {
    return reinterpret_cast<const uint4*>(idx.slots)[h];
}
__device__ __forceinline__ uint32_t vindexFind(const VIndex& idx, int32_t part, int64_t vid) {
    uint64_t h = vindexHash(part, vid) & idx.mask;
    const uint32_t vlo = static_cast<uint32_t>(vid), vhi = static_cast<uint32_t>(static_cast<uint64_t>(vid) >> 32);
    for (uint64_t probe = 0; probe <= idx.mask; probe += 2) {
        const uint4 a = vindexSlot(idx, h), b = vindexSlot(idx, (h + 1) & idx.mask);
        const bool aHit = a.x == vlo && a.y == vhi && a.z == static_cast<uint32_t>(part) && a.w != kNoRow;
        const bool bHit = b.x == vlo && b.y == vhi && b.z == static_cast<uint32_t>(part) && b.w != kNoRow;
        const bool done = aHit || a.w == kNoRow || bHit || b.w == kNoRow;   // found, or an empty slot ends the run
        const uint32_t r = aHit ? a.w : a.w == kNoRow ? kNoRow : bHit ? b.w : kNoRow;
        if (done) return r;
        h = (h + 2) & idx.mask;
    }
    return kNoRow;
}

// seed (part, vid) -> vertex row through the commit-time hash index (GetNeighbors requests)
__global__ void k_index_lookup(const int32_t* qpart, const int64_t* qvid, uint64_t n, VIndex idx, uint32_t* out) {
    uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = vindexFind(idx, qpart[i], qvid[i]);
}

// chunk heads of entry i (hop edges [e, e + d)): every chunk whose first edge c * CE lies in the range
__device__ __forceinline__ void writeChunkHeads(uint64_t* cf, uint64_t cap, uint64_t i, uint64_t e, uint64_t d, uint32_t* err) {
    for (uint64_t c = (e + CE - 1) / CE; c * CE < e + d; c++) {
        if (c >= cap) { atomicOr(err + 3, 1u); return; }
        cf[c] = i;
    }
}

// Seed hop in two launches. A single workgroup doing the lookups measured ~1.5 us per dependent step
// (tools/mb_latency.hip: 1024 random loads from one CU queue behind its own miss handling), 14 us in
// all; spread over 64-thread workgroups on as many CUs each step costs about one memory latency.
// Launch 1 (a thread per seed): (part, vid) -> row through the index, F[i], and per entry its degree
// (into estart, turned into offsets by launch 2) and CSR base (ebase); block 0 clears zero[] / zero8.
__global__ __launch_bounds__(64) void k_seed_lookup(const int32_t* qpart, const int64_t* qvid, uint64_t n, VIndex idx,
                                                    HopSlots hs, uint32_t* F, uint64_t* deg, uint64_t* ebase,
                                                    uint64_t* zero, uint32_t nzero, uint64_t* zero8) {
    if (blockIdx.x == 0) {
        if (threadIdx.x < nzero) zero[threadIdx.x * kDoneOff] = 0;
        if (zero8 != nullptr && threadIdx.x < 8) zero8[threadIdx.x] = 0;
    }
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 64 + threadIdx.x;
    if (i >= n) return;
    const uint32_t r = vindexFind(idx, qpart[i], qvid[i]);
    F[i] = r;
    const uint64_t rr = r == kNoRow ? 0 : r;                    // every load issued, the result selected
    for (int s = 0; s < hs.n; s++) {
        const uint64_t o0 = hs.off[s][rr], o1 = hs.off[s][rr + 1];
        deg[i * hs.n + s] = r == kNoRow ? 0 : o1 - o0;
        if (ebase) ebase[i * hs.n + s] = o0;
    }
}

// Launch 2 (one 256-thread workgroup, nEnt <= kSeedFuseMax): the entries' degrees -> exclusive offsets
// in place, E = estart[nEnt], the hop's chunk heads, E published (and packed with |F| for dyn hops). (A
// 1024-thread workgroup waited up to 200 us for a CU with 16 free wave slots beside another query's final
// hop in a pipelined batch.)
constexpr int kSeedScanWG = 256;
__global__ __launch_bounds__(kSeedScanWG) void k_seed_scan(uint64_t n, int ns, uint64_t* estart, Publish pub,
                                                           uint64_t* chunkFirst, uint64_t cfCap, uint32_t* err,
                                                           uint64_t* packedOut) {
    constexpr int NW = kSeedScanWG / 64;
    __shared__ uint64_t sm[NW + 1];
    constexpr int kPer = static_cast<int>(kSeedFuseMax / kSeedScanWG);
    const uint64_t nEnt = n * static_cast<uint64_t>(ns);
    const uint64_t lo = threadIdx.x * static_cast<uint64_t>(kPer);
    uint64_t d[kPer];
    uint64_t sum = 0;
#pragma unroll
    for (int k = 0; k < kPer; k++) {
        d[k] = lo + k < nEnt ? estart[lo + k] : 0;
        sum += d[k];
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint64_t x = sum;
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) sm[wid] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t acc = 0;
        for (int w = 0; w < NW; w++) { const uint64_t t = sm[w]; sm[w] = acc; acc += t; }
        sm[NW] = acc;
    }
    __syncthreads();
    uint64_t pre = sm[wid] + x - sum;
#pragma unroll
    for (int k = 0; k < kPer; k++) {
        if (lo + k >= nEnt) break;
        estart[lo + k] = pre;
        writeChunkHeads(chunkFirst, cfCap, lo + k, pre, d[k], err);
        pre += d[k];
    }
    if (threadIdx.x == 0) {
        estart[nEnt] = sm[NW];
        if (packedOut) *packedOut = (n << kDynShift) | sm[NW];       // device-driven hops read this
        if (pub.slot) publishWords(pub.slot, pub.seq, sm[NW], 0);
    }
}

// ------------------------------------------------------------------------------ chunk -> first entry
// chunkFirst[c] = the entry holding edge c * CE (the only entry with estart[i] <= c*CE < estart[i+1])
// zero[0 .. nzero) is cleared on the way (the next final launch's look-back words: no memset launch)
__global__ void k_chunk_first(const uint64_t* estart, uint64_t nEnt, uint64_t* chunkFirst, uint64_t* zero,
                              uint64_t nzero) {
    uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    for (uint64_t z = i; z < nzero; z += static_cast<uint64_t>(gridDim.x) * blockDim.x) zero[z] = 0;
    if (i >= nEnt) return;
    uint64_t s = estart[i], t = estart[i + 1];
    for (uint64_t c = (s + CE - 1) / CE; c * CE < t; c++) chunkFirst[c] = i;
}

// ------------------------------------------------------------------------------ intermediate hop
// Edge-balanced expansion: every edge of the hop reads its 4-byte destination row and stores the
// hop's epoch into visited[] (the frontier dedup of GoExecutor::getDstIdsFromResp, a set of dsts).
// The store is unconditional: a byte store needs no read and duplicates write the same value.
// P32: CSR positions fit 32 bits (20 KiB chunk map instead of 28, see ChunkMap)
// MASK: only edges with mask[e] != 0 (the storage outcome of a hop with TTL or a max-edges cap)
// dyn (device-driven hop): E and the frontier size come from *dyn (packed, written by the kernel that
// built the frontier); the fixed grid strides over the chunks; a hop with E >= pullMinE is the pull
// kernels' (they run instead).
template <bool ONE, bool P32, bool MASK>
__global__ __launch_bounds__(WG) void k_expand_mark(const uint32_t* F, const uint64_t* estart, const uint64_t* chunkFirst,
                                                    uint64_t nEnt, uint64_t E, HopSlots hs, uint8_t* visited,
                                                    uint8_t epoch, const uint8_t* mask, const uint64_t* dyn,
                                                    uint64_t pullMinE, const uint64_t* ebase) {
    __shared__ ChunkMap<ONE, false, P32, false> m;      // (no src rows: the expansion marks destinations)
    // direct-mapped LDS filter of the rows this workgroup already marked: a repeated destination
    // (hubs of a power-law graph) costs an LDS probe instead of another L2 byte-store transaction
    constexpr int kSeenBits = 11;
    __shared__ uint32_t seen[1 << kSeenBits];
    uint32_t nChunks = gridDim.x;
    if (dyn != nullptr) {
        const uint64_t t = *dyn;
        E = t & kDynMask;
        if (E >= pullMinE) return;
        nEnt = (t >> kDynShift) * static_cast<uint64_t>(hs.n);
        nChunks = static_cast<uint32_t>((E + CE - 1) / CE);
    }
    for (int p = threadIdx.x; p < (1 << kSeenBits); p += WG) seen[p] = kNoRow;
    for (uint32_t chunk = blockIdx.x; chunk < nChunks; chunk += gridDim.x) {
    const uint64_t base = static_cast<uint64_t>(chunk) * CE;
    const uint32_t cnt = static_cast<uint32_t>(E - base < CE ? E - base : CE);
    buildMap<ONE, false, P32, false>(estart, chunkFirst, nEnt, chunk, nChunks, base, cnt, F, hs, m, ebase);
    uint32_t g[CITEMS];
#pragma unroll
    for (int k = 0; k < CITEMS; k++) {
        uint32_t p = threadIdx.x + k * WG;
        g[k] = kNoRow;
        if (p < cnt && (!MASK || mask[base + p])) {
            uint32_t q = m.at[p];
            int s = ONE ? 0 : m.slot[q];
            uint64_t pos = P32 ? static_cast<uint64_t>(static_cast<uint32_t>(base + p) + static_cast<uint32_t>(m.pb[q]))
                               : static_cast<uint64_t>(static_cast<int64_t>(base + p) + static_cast<int64_t>(m.pb[q]));
            g[k] = hs.dgid[s][pos];
        }
    }
#pragma unroll
    for (int k = 0; k < CITEMS; k++) {
        if (g[k] == kNoRow) continue;
        uint32_t h = (g[k] * 2654435761u) >> (32 - kSeenBits);
        if (seen[h] == g[k]) continue;                  // marked by this workgroup already (its store is issued)
        seen[h] = g[k];
        visited[g[k]] = epoch;
    }
    if (dyn == nullptr) break;
    __syncthreads();                                    // the chunk map is rebuilt for the next chunk
    }
}

// ------------------------------------------------------------------------------ compaction
// visited[row] == epoch -> next frontier + its entries' estart + the next hop's chunk heads, two
// launches (kernels.h CompactArgs). Wave w of tile t owns rows t * 1024 CIT + w * 64 CIT + k * 64 +
// lane, k < CIT, so the marks (1 B per lane) and the CSR offsets (8 B per lane) of one k are one coalesced
// wave access, and rows leave in row order (k-major, ballot prefix inside k).
// (r02 gave each thread 16 consecutive rows: its offset loads put the 64 lanes of a wave on 64 cache
// lines, 16 times, and the address unit bounded the pass; a single-pass decoupled look-back over
// tiles taken by ticket then spent 20-38 us per launch on the 586 ticket atomics and the polling.)
// 1024-thread workgroups: a 4096-row tile over 16 waves of 4 rows per lane (r03's 4 waves of 16
// rows left 2.3 waves per SIMD at C2, each wave issuing 16 scans one after the other)
// CIT rows per lane (4 by default; 8 or 16 by the flag compact_lane_rows, tested for parity)
constexpr int CWG = 1024;
__device__ __forceinline__ uint64_t waveInclScan(uint64_t x, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    return x;
}

// Loads in these kernels are issued unconditionally (an unwanted lane reads a valid dummy address and
// its value is discarded by a select): a load under a divergent branch gets its own `s_waitcnt
// vmcnt(0)` at the branch's end, which serialized the 16 mark loads and 32 offset loads of a wave
// into 48 round trips (r03 ISA; 7 + 13 us per compaction at C2 instead of ~3).
template <bool ONE>
__device__ __forceinline__ uint64_t rowDegree(const HopSlots& hs, uint64_t r) {
    if (ONE) return hs.off[0][r + 1] - hs.off[0][r];
    uint64_t d = 0;
    for (int s = 0; s < hs.n; s++) d += hs.off[s][r + 1] - hs.off[s][r];
    return d;
}

// the wave's 16 mark flags (bit k: row wbase + 64 k + lane)
template <int CIT>
__device__ __forceinline__ uint32_t waveFlags(const CompactArgs& a, uint64_t wbase, int lane) {
    uint8_t mk[CIT];
#pragma unroll
    for (int k = 0; k < CIT; k++) {
        const uint64_t r = wbase + k * 64 + lane;
        mk[k] = a.visited[r < a.V ? r : a.V - 1];
    }
    uint32_t flags = 0;
#pragma unroll
    for (int k = 0; k < CIT; k++) flags |= (mk[k] == a.epoch && wbase + k * 64 + lane < a.V ? 1u : 0u) << k;
    return flags;
}

// degrees of the wave's flagged rows (0 elsewhere), every load issued before the first use
// (ONE: also each row's CSR base in ob[], for the write launch's ebase[])
template <bool ONE, int CIT>
__device__ __forceinline__ void waveDegrees(const CompactArgs& a, uint64_t wbase, int lane, uint32_t flags,
                                            uint64_t (&deg)[CIT], uint64_t* ob = nullptr) {
#pragma unroll
    for (int k = 0; k < CIT; k++) {
        const bool m = (flags >> k) & 1u;
        const uint64_t r = m ? wbase + k * 64 + lane : 0;
        if (ONE) {
            const uint64_t o0 = a.hs.off[0][r], o1 = a.hs.off[0][r + 1];
            deg[k] = m ? o1 - o0 : 0;
            if (ob) ob[k] = o0;
        } else {
            const uint64_t d = rowDegree<ONE>(a.hs, r);
            deg[k] = m ? d : 0;
        }
    }
}

// launch 1: per tile and per wave the packed (rows << kFdShift | degrees) total; the bitmap words
// (WGS = CWG threads per workgroup; r05 measured 256 threads x 16 rows per lane, the same tile, in a
// pipelined batch beside another query's final hop: 0.370 vs 0.366 ms per C2 step, alone 27.8 vs 25.8 us)
template <bool ONE, int CIT, int WGS>
__global__ __launch_bounds__(WGS) void k_compact_count(CompactArgs a) {
    constexpr int NW = WGS / 64;
    __shared__ uint64_t sWave[NW];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint64_t wbase = static_cast<uint64_t>(blockIdx.x) * (WGS * CIT) + static_cast<uint64_t>(wid) * (64 * CIT);
    if (blockIdx.x == 0 && threadIdx.x == 0 && a.clear32 != nullptr) *a.clear32 = 0;
    const uint32_t flags = waveFlags<CIT>(a, wbase, lane);
    uint64_t deg[CIT];
    waveDegrees<ONE, CIT>(a, wbase, lane, flags, deg);
    uint64_t dsum = 0;
#pragma unroll
    for (int k = 0; k < CIT; k++) dsum += deg[k];
    if (a.bits != nullptr) {
        // word k of the wave = rows wbase + 64 k .. + 63; lane k stores it
        uint64_t w = 0;
#pragma unroll
        for (int k = 0; k < CIT; k++) {
            const uint64_t b = __ballot((flags >> k) & 1u);
            if (lane == k) w = b;
        }
        if (lane < CIT && wbase + static_cast<uint64_t>(lane) * 64 < a.V) a.bits[(wbase >> 6) + lane] = a.bitsZero ? 0 : w;
    }
    uint64_t packed = (static_cast<uint64_t>(__popc(flags)) << kFdShift) | dsum;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) packed += __shfl_xor(packed, o, 64);
    if (lane == 0) {
        sWave[wid] = packed;
        a.waveSum[static_cast<uint64_t>(blockIdx.x) * NW + wid] = packed;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
#pragma unroll
        for (int w = 0; w < NW; w++) t += sWave[w];
        a.tileSum[blockIdx.x] = t;
    }
}

// launch 2: the wave's start = the tiles before it + the waves before it in its tile (summed from
// launch 1's words, nothing waited for), then the rows in order: positions from each k's ballot and a
// wave scan of its degrees. The last tile writes the totals (estart[|F| * ns] = E, *total, publish).
template <bool ONE, int CIT, int WGS>
__global__ __launch_bounds__(WGS) void k_compact_write(CompactArgs a) {
    constexpr int NW = WGS / 64;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint64_t tile = blockIdx.x;
    const uint64_t wbase = tile * (WGS * CIT) + static_cast<uint64_t>(wid) * (64 * CIT);
    const int ns = a.hs.n;
    const uint32_t flags = waveFlags<CIT>(a, wbase, lane);
    // the totals of the tiles before this one: 8 loads in flight per lane (a dependent loop of loads
    // cost 10 us at C2's 586 tiles)
    uint64_t pre = lane < wid ? a.waveSum[tile * NW + lane] : 0;
    for (uint64_t t0 = 0; t0 < tile; t0 += 8 * 64) {
        uint64_t v[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint64_t t = t0 + j * 64 + lane;
            v[j] = t < tile ? a.tileSum[t] : 0;
        }
#pragma unroll
        for (int j = 0; j < 8; j++) pre += v[j];
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) pre += __shfl_xor(pre, o, 64);
    if (tile == gridDim.x - 1 && wid == NW - 1 && lane == 0) {
        const uint64_t incl = pre + a.waveSum[tile * NW + wid];
        a.estart[(incl >> kFdShift) * static_cast<uint64_t>(ns)] = incl & kFdMask;
        *a.total = incl;
        if (a.pub.slot) publishWords(a.pub.slot, a.pub.seq, incl, 0);
    }
    if (tile == 0 && threadIdx.x < a.nzero) a.zero[threadIdx.x * kDoneOff] = 0;
    if (__ballot(flags != 0) == 0) return;              // wave-uniform: every lane stays for the scans below
    uint64_t deg[CIT], ob[CIT];
    waveDegrees<ONE, CIT>(a, wbase, lane, flags, deg, ONE ? ob : nullptr);
    uint64_t fk = pre >> kFdShift, ek = pre & kFdMask;     // running start of group k
    const uint64_t below = (1ULL << lane) - 1;
#pragma unroll
    for (int k = 0; k < CIT; k++) {
        const bool m = (flags >> k) & 1u;
        const uint64_t ball = __ballot(m);
        if (ball == 0) continue;
        const uint64_t r = wbase + k * 64 + lane;
        const uint64_t incl = waveInclScan(deg[k], lane);
        const uint64_t f = fk + static_cast<uint64_t>(__popcll(ball & below));
        uint64_t e = ek + incl - deg[k];
        fk += static_cast<uint64_t>(__popcll(ball));
        ek += __shfl(incl, 63, 64);
        if (!m) continue;
        a.outF[f] = static_cast<uint32_t>(r);
        if (ONE) {
            a.estart[f] = e;
            if (a.ebase) a.ebase[f] = ob[k];
            writeChunkHeads(a.chunkFirst, a.cfCap, f, e, deg[k], a.err);
        } else {
            for (int s = 0; s < ns; s++) {
                const uint64_t o = a.hs.off[s][r];
                const uint64_t d = a.hs.off[s][r + 1] - o;
                a.estart[f * ns + s] = e;
                if (a.ebase) a.ebase[f * ns + s] = o;
                writeChunkHeads(a.chunkFirst, a.cfCap, f * ns + s, e, d, a.err);
                e += d;
            }
        }
    }
}

// ------------------------------------------------------------------------------ sparse intermediate hop
// kernels.h SparseArgs. The same edge-balanced chunk map as k_expand_mark, but kSparseSub workgroups
// per 2048-edge chunk, each taking one 256-edge slice of it (one edge per thread): the hop's atomics
// spread over kSparseSub times as many CUs. The atomics execute at the memory side and a CU issues them
// at a bounded rate — with 8 per thread on 24 CUs (C2 hop 1) they took ~10 of 21 us (device
// timestamps, r05). A destination's first edge (the one whose atomicOr set its bit) makes it a row of
// the next frontier. Loads and atomics are issued for every lane and selected afterwards (no memory
// operation under a divergent branch, see the compaction's note below).
constexpr int kSparseSub = CE / WG;                     // 8 slices of 256 edges per chunk
template <bool ONE, bool P32>
__global__ __launch_bounds__(WG) void k_expand_sparse(SparseArgs a) {
    __shared__ ChunkMap<ONE, false, P32, false> m;      // (no src rows: the expansion marks destinations)
    __shared__ uint64_t sm[NW + 1];
    __shared__ uint64_t sBase;
    // direct-mapped LDS filter of the destinations this workgroup already sent an atomic for (as in
    // k_expand_mark): a hub's repeats cost an LDS probe, not another atomic on the hub's word
    constexpr int kSeenBits = 9;
    __shared__ uint32_t seen[1 << kSeenBits];
    for (int p = threadIdx.x; p < (1 << kSeenBits); p += WG) seen[p] = kNoRow;
    // the hop's edges: from the arguments, or (dynIn, a hop launched before its size is known on the
    // host) from the packed (|F|, E) word the kernel that built the frontier wrote; the grid then strides
    // over the slices
    uint64_t E = a.E, nEnt = a.nEnt;
    if (a.dynIn != nullptr) {
        const uint64_t t = gld<uint64_t>(a.dynIn, 0);
        E = t & kDynMask;
        nEnt = (t >> kDynShift) * static_cast<uint64_t>(a.hs.n);
    }
    const uint32_t nChunks = static_cast<uint32_t>((E + CE - 1) / CE);
    const int ns = a.hs.n;
    // workgroups past the hop's slices leave at once, without counting themselves done (a same-address
    // atomic per workgroup of a 1024-workgroup grid cost ~9 us); an empty hop is finished by workgroup 0
    const uint32_t items = nChunks * kSparseSub;
    const uint32_t active = items < gridDim.x ? (items ? items : 1u) : gridDim.x;
    if (blockIdx.x >= active) return;
    for (uint32_t item = blockIdx.x; item < items; item += gridDim.x) {
        const uint32_t chunk = item / kSparseSub, sub = item % kSparseSub;
        const uint64_t base = static_cast<uint64_t>(chunk) * CE;
        const uint32_t cnt = static_cast<uint32_t>(E - base < CE ? E - base : CE);
        buildMap<ONE, false, P32, false>(a.estart, a.chunkFirst, nEnt, chunk, nChunks, base, cnt, a.F, a.hs, m, a.ebase);
        const uint32_t p = sub * WG + threadIdx.x;          // this lane's edge of the chunk
        uint32_t g = kNoRow;
        if (p < cnt) {
            const uint32_t q = m.at[p];
            const int s = ONE ? 0 : m.slot[q];
            const uint64_t pos = P32 ? static_cast<uint64_t>(static_cast<uint32_t>(base + p) + static_cast<uint32_t>(m.pb[q]))
                                     : static_cast<uint64_t>(static_cast<int64_t>(base + p) + static_cast<int64_t>(m.pb[q]));
            g = a.hs.dgid[s][pos];
        }
        bool need = false;                                   // the destination not yet seen in this workgroup
        if (g != kNoRow) {
            const uint32_t h = (g * 2654435761u) >> (32 - kSeenBits);
            if (seen[h] != g) { seen[h] = g; need = true; }
        }
        // the atomic and the row's CSR offsets issued together; a lane without one ORs 0 into a word of its
        // own (no queue on one address). 32-bit words of the 64-bit bitmap (little-endian halves).
        uint32_t* const bits32 = reinterpret_cast<uint32_t*>(a.bits);
        const uint64_t r = need ? g : 0;
        const uint64_t w = need ? (r >> 5) : (static_cast<uint64_t>(blockIdx.x) * WG + threadIdx.x) % (2 * a.bitWords);
        const uint32_t old = atomicOr(bits32 + w, need ? 1u << (r & 31) : 0u);
        uint64_t deg, ob;
        if (ONE) {
            const uint64_t o0 = a.hs.off[0][r], o1 = a.hs.off[0][r + 1];
            deg = o1 - o0;
            ob = o0;
        } else {
            deg = rowDegree<false>(a.hs, r);
            ob = 0;
        }
        const bool first = need && !(old & (1u << (r & 31)));
        deg = first ? deg : 0;
        uint64_t tot;
        const uint64_t pre = blockExScan(first ? ((1ULL << kFdShift) | deg) : 0, tot, sm);
        if (threadIdx.x == 0) {
            sBase = tot ? static_cast<uint64_t>(atomicAdd(reinterpret_cast<unsigned long long*>(a.ctl),
                                                          static_cast<unsigned long long>(tot)))
                        : 0;
        }
        __syncthreads();
        if (first) {
            const uint64_t at = sBase + pre;
            const uint64_t f = at >> kFdShift;
            uint64_t e = at & kFdMask;
            a.outF[f] = g;
            if (ONE) {
                a.outEst[f] = e;
                if (a.outEbase) a.outEbase[f] = ob;
                writeChunkHeads(a.outCf, a.cfCap, f, e, deg, a.err);
            } else {
                for (int s = 0; s < ns; s++) {
                    const uint64_t o = a.hs.off[s][g];
                    const uint64_t d = a.hs.off[s][g + 1] - o;
                    a.outEst[f * ns + s] = e;
                    if (a.outEbase) a.outEbase[f * ns + s] = o;
                    writeChunkHeads(a.outCf, a.cfCap, f * ns + s, e, d, a.err);
                    e += d;
                }
            }
        }
        __syncthreads();                                // the chunk map and sBase are rebuilt for the next slice
    }
    // the last workgroup to finish writes the totals: every workgroup's reservation returned before its
    // done increment was issued, so the count it reads is final. No fence: the rows, estart and heads
    // are read by later launches only (a kernel boundary orders them; an agent-scope fence here would
    // write back the XCD's L2)
    if (threadIdx.x == 0) {
        const uint64_t done = atomicAdd(reinterpret_cast<unsigned long long*>(a.ctl + 1), 1ULL);
        if (done == active - 1) {
            const uint64_t t = __hip_atomic_load(a.ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            a.outEst[(t >> kFdShift) * static_cast<uint64_t>(ns)] = t & kFdMask;
            *a.total = t;
            a.ctl[0] = 0;
            a.ctl[1] = 0;
            if (a.pub.slot) publishWords(a.pub.slot, a.pub.seq, t, 0);
        }
    }
}

// ------------------------------------------------------------------------------ pull (direction-optimizing) hop
// Segment word: k (28 bits: segment index in the row's remaining in-list) | slot (4) | row (32).
__device__ __forceinline__ uint64_t pullSegWord(uint32_t row, int s, uint64_t k) {
    return (k << 36) | (static_cast<uint64_t>(s) << 32) | row;
}

// Row pass over the head image (kernels.h PullArgs): one wave per 64-row slice, grid-stride over the
// slices of every hop slot. Round k loads head[slice][k][*] (coalesced) and probes the frontier mark
// of that in-neighbour for the lanes still open; the first kPullK / 2 rounds are loaded together. A
// lane closes on a hit, on a kNoRow entry (its in-list ended) or after its last head entry; lanes of
// rows with a longer in-list that are still open reserve segment words for k_pull_segments (their
// whole in-list, from the mirror CSR).
__device__ __forceinline__ bool inFrontier(const PullArgs& a, uint32_t g) {
    return (a.curBits[g >> 6] >> (g & 63)) & 1ULL;
}
// the probe of a lane that may not need it: an unconditional load (row 0's word for the others) so the
// probes of a round issue together (see rowDegree's note)
__device__ __forceinline__ bool probe(const PullArgs& a, bool want, uint32_t g) {
    const uint32_t x = want ? g : 0u;
    const uint64_t w = a.curBits[x >> 6];
    return static_cast<bool>(static_cast<uint32_t>(want) & static_cast<uint32_t>((w >> (x & 63)) & 1ULL));
}

// one slice's first loads: its rows, round count and first KH head rounds (independent loads; rounds
// past the slice's count hold kNoRow: the image is kPullK rounds deep everywhere)
constexpr int kPullKB = 4;                             // head rounds per batch after the first KH
template <int KH>
struct PullSlice {
    uint32_t pw;
    int nk;
    uint32_t u[KH];
};
template <bool ONE, int KH>
__device__ __forceinline__ void pullLoad(const PullArgs& a, uint64_t j, int lane, int& s, uint64_t& js, PullSlice<KH>& p) {
    s = 0;
    if (!ONE) while (j >= a.sliceEnd[s]) s++;
    js = (ONE || s == 0) ? j : j - a.sliceEnd[s - 1];
    const uint32_t* hp = a.head[s] + js * (kPullK * 64) + lane;
    p.pw = a.perm[s][js * 64 + lane];
    p.nk = a.nk[s][js];
#pragma unroll
    for (int k = 0; k < KH; k++) p.u[k] = hp[k * 64];
}

// probes of N consecutive head rounds held in u[off .. off + N), for the lanes still open: every probe
// issued before the first is resolved, then the rounds resolved in order
template <int N>
__device__ __forceinline__ void pullProbe(const PullArgs& a, const uint32_t* u, bool& open, bool& hit) {
    // bit k of `ev`: round k ends the lane's search (a hit, or kNoRow: its in-list ended); straight-line
    // selects, no branch per round (a branch would wait for each probe in turn)
    uint32_t hits = 0, ends = 0;
#pragma unroll
    for (int k = 0; k < N; k++) {
        hits |= static_cast<uint32_t>(probe(a, open && u[k] != kNoRow, u[k])) << k;
        ends |= static_cast<uint32_t>(u[k] == kNoRow) << k;
    }
    const uint32_t ev = hits | ends;
    const uint32_t first = ev & (0u - ev);                  // lowest set bit: the round that decides
    hit = hit || (open && (first & hits) != 0);
    open = open && ev == 0;
}

// One slice's search: true for a lane whose row has an in-neighbour in the frontier among its head
// rounds (round 0 alone first: most reached rows hit there; then batches for the lanes still open).
// A lane left open on a long row reserves the segments of its in-list past the head (one atomic per
// wave) for the segment pass.
template <int KH>
__device__ __forceinline__ bool pullSliceHit(const PullArgs& a, const PullSlice<KH>& cur, int s, uint64_t js, int lane,
                                             uint32_t& row) {
    const uint32_t* hp = a.head[s] + js * (kPullK * 64) + lane;
    bool hit = probe(a, cur.u[0] != kNoRow, cur.u[0]);
    bool open = cur.pw != kNoRow && !hit && cur.u[0] != kNoRow && cur.nk > 1;
    if (__any(open)) {
        if constexpr (KH > 1) pullProbe<KH - 1>(a, cur.u + 1, open, hit);   // rounds 1 .. KH - 1
        uint32_t u[kPullKB];
        for (int k0 = KH; k0 < cur.nk && __any(open); k0 += kPullKB) {
            // a batch reaching past the image re-probes its last round (kNoRow would end the lane's
            // search, and a long row's in-list continues past the head)
#pragma unroll
            for (int k = 0; k < kPullKB; k++) u[k] = hp[(k0 + k < kPullK ? k0 + k : kPullK - 1) * 64];
            pullProbe<kPullKB>(a, u, open, hit);
        }
    }
    row = cur.pw & ~kPullLong;
    const bool more = open && cur.pw != kNoRow && (cur.pw & kPullLong) != 0;
    uint32_t nseg = 0;
    if (more) nseg = static_cast<uint32_t>((a.ioff[s][row + 1] - a.ioff[s][row] + kPullSeg - 1) / kPullSeg);
    if (__any(nseg != 0)) {
        const uint64_t incl = waveInclScan(nseg, lane);
        uint32_t base = 0;
        if (lane == 63) base = atomicAdd(&a.ctl[0], static_cast<uint32_t>(incl));
        base = __shfl(base, 63, 64);
        uint64_t at = base + incl - nseg;
        for (uint32_t k = 0; k < nseg; k++, at++) {
            if (at < a.segCap) a.seg[at] = pullSegWord(row, s, k);
            else atomicOr(a.err + 3, 1u);
        }
    }
    return hit && cur.pw != kNoRow;
}

// A wave per slice of the head image (the grid covers the slices: r03 measured a grid of 2048
// workgroups striding over the slices and loading the next one before probing the current 56 vs 52 us,
// and one LDS-gathered mark write per 2048-row window 45 vs 33 us); KH = 2 head rounds loaded with the
// slice before its first probe (48 us at C2 against 50 for 4 and 51 for 1).
constexpr int kPullKH = 2;
template <bool ONE>
__global__ __launch_bounds__(WG) void k_pull_head(PullArgs a) {
    if (a.dyn != nullptr && (*a.dyn & kDynMask) < a.minE) return;   // a push hop (k_expand_mark takes it)
    const int lane = threadIdx.x & 63;
    const uint64_t total = a.sliceEnd[ONE ? 0 : a.n - 1];
    // workgroups are dispatched to the 8 XCDs round robin (b % 8): logical workgroup (b % 8) * (G / 8) +
    // b / 8 keeps consecutive logical workgroups — the 32 slices of a 2048-row window, whose mark bytes
    // share 16 cache lines — on one XCD, so each line is dirtied in one L2 and written back whole
    // instead of partially from up to 8 L2s (33 vs 44 us at C2)
    const uint64_t b = (blockIdx.x % 8u) * (gridDim.x / 8u) + blockIdx.x / 8u;
    const uint64_t j = (b * WG + threadIdx.x) >> 6;
    if (j >= total) return;
    int s;
    uint64_t js;
    PullSlice<kPullKH> cur;
    pullLoad<ONE, kPullKH>(a, j, lane, s, js, cur);
    uint32_t row;
    if (pullSliceHit<kPullKH>(a, cur, s, js, lane, row)) a.out[row] = a.ep;
}

// Segment pass (the next launch on the stream, so every segment word is visible): a workgroup per
// segment of kPullSeg in-edges of a long row's in-list, grid-stride; any hit marks the row. The
// compaction's count launch after it clears the segment counter for the next hop (CompactArgs::clear32).
__global__ __launch_bounds__(WG) void k_pull_segments(PullArgs a) {
    const uint32_t nres = __hip_atomic_load(&a.ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t n = nres < a.segCap ? nres : a.segCap;
    for (uint64_t i = blockIdx.x; i < n; i += gridDim.x) {
        const uint64_t w = a.seg[i];
        const uint32_t row = static_cast<uint32_t>(w);
        const int s = static_cast<int>((w >> 32) & 0xF);
        const uint64_t k = w >> 36;
        const uint64_t e = a.ioff[s][row + 1];
        const uint64_t b = a.ioff[s][row] + k * kPullSeg;
        const uint64_t be = b + kPullSeg < e ? b + kPullSeg : e;
        const uint32_t* in = a.isrc[s];
        uint32_t u[kPullSeg / WG];
#pragma unroll
        for (int j = 0; j < static_cast<int>(kPullSeg / WG); j++) {
            const uint64_t p = b + threadIdx.x + static_cast<uint64_t>(j) * WG;
            u[j] = p < be ? in[p] : kNoRow;
        }
        bool hit = false;
#pragma unroll
        for (int j = 0; j < static_cast<int>(kPullSeg / WG); j++) hit |= u[j] != kNoRow && inFrontier(a, u[j]);
        if (hit) a.out[row] = a.ep;
    }
}

// the end of a GO query: the error words (bit k = err[k] != 0) and `nExtra` device words published to
// host-mapped memory, sequence number last (system-scope release), so the host learns the outcome by
// polling instead of an event synchronisation plus a copy (~20 us of host time per query)
__global__ void k_publish_tail(const uint32_t* err, const uint64_t* extra, int nExtra, uint64_t* slot, uint64_t seq) {
    if (threadIdx.x != 0) return;
    uint64_t bits = 0;
    for (int k = 0; k < 4; k++) bits |= static_cast<uint64_t>(err[k] != 0) << k;
    __hip_atomic_store(slot + 1, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    for (int i = 0; i < nExtra; i++) __hip_atomic_store(slot + 2 + i, extra[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(slot, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void k_mark_bits(const uint32_t* F, uint64_t n, uint64_t* bits) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n && F[i] != kNoRow) atomicOr(reinterpret_cast<unsigned long long*>(bits + (F[i] >> 6)), 1ULL << (F[i] & 63));
}

// The global frontier bitmap from the all-gathered per-shard ones: shard q's segment (segWords words,
// bit i = its local row i) lands at global rows [sb[q], sb[q + 1]). Output word w collects the 64
// global rows [64 w, 64 w + 64) from every shard overlapping them (a funnel shift of two words).
__global__ void k_repack_bits(RepackArgs a) {
    const uint64_t w = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (w >= a.outWords) return;
    const uint64_t g0 = w * 64, g1 = g0 + 64;
    uint64_t out = 0;
    for (int q = 0; q < a.world; q++) {
        const uint64_t lo = a.sb[q] > g0 ? a.sb[q] : g0;
        const uint64_t hi = a.sb[q + 1] < g1 ? a.sb[q + 1] : g1;
        if (lo >= hi) continue;
        const uint64_t* seg = a.seg + static_cast<uint64_t>(q) * a.segWords;
        // local bits [lo - sb[q], hi - sb[q]) -> output bits [lo - g0, hi - g0)
        const uint64_t l0 = lo - a.sb[q];
        const uint64_t wi = l0 >> 6, sh = l0 & 63;
        uint64_t x = seg[wi] >> sh;
        if (sh && wi + 1 < a.segWords) x |= seg[wi + 1] << (64 - sh);
        const uint64_t n = hi - lo;
        const uint64_t m = n == 64 ? ~0ULL : ((1ULL << n) - 1);
        out |= (x & m) << (lo - g0);
    }
    a.out[w] = out;
}

// ------------------------------------------------------------------------------ multi-root walk
// A pipe's sentence from many roots in one walk (engine.cpp runPipe): each frontier row carries the
// set of roots (bit j = root j of a batch of 64) that reach it at this hop, the reference's
// VertexBackTracker (GoExecutor.h:189-207) as a bitmask. A wave per frontier entry, lanes striding
// over its edges: every destination ORs in the source's roots and is marked for the compaction.
__global__ __launch_bounds__(WG) void k_expand_roots(const uint32_t* F, uint64_t nEnt, HopSlots hs, const uint64_t* rootsCur,
                                                     unsigned long long* rootsNext, uint8_t* visited, uint8_t epoch) {
    const int lane = threadIdx.x & 63;
    const uint64_t nw = static_cast<uint64_t>(gridDim.x) * NW;
    for (uint64_t w = (static_cast<uint64_t>(blockIdx.x) * WG + threadIdx.x) >> 6; w < nEnt; w += nw) {
        const uint32_t row = F[w / hs.n];
        const int s = static_cast<int>(w % hs.n);
        if (row == kNoRow) continue;
        const unsigned long long m = rootsCur[row];
        if (m == 0) continue;
        const uint64_t b = hs.off[s][row], e = hs.off[s][row + 1];
        for (uint64_t p = b + lane; p < e; p += 64) {
            const uint32_t g = hs.dgid[s][p];
            if (g == kNoRow) continue;
            atomicOr(rootsNext + g, m);
            visited[g] = epoch;
        }
    }
}

// roots[F[i]] |= bits[i] (the seed frontier's roots; a vid may repeat) and out[i] = roots of F[i]
__global__ void k_scatter_roots(const uint32_t* F, uint64_t n, const uint64_t* bits, unsigned long long* roots) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n && F[i] != kNoRow) atomicOr(roots + F[i], static_cast<unsigned long long>(bits[i]));
}
__global__ void k_gather_roots(const uint32_t* F, uint64_t n, const uint64_t* roots, uint64_t* out) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n) out[i] = F[i] == kNoRow ? 0 : roots[F[i]];
}

__global__ void k_merge_roots(const uint64_t* own, const uint64_t* recv, uint64_t stride, uint64_t n, int world, int rank,
                              uint64_t* out) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t m = own[i];
    for (int q = 0; q < world; q++)
        if (q != rank) m |= recv[q * stride + i];
    out[i] = m;
}

__global__ void k_mark_rows(const uint32_t* F, uint64_t n, uint8_t* marks, uint8_t ep) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n && F[i] != kNoRow) marks[F[i]] = ep;
}

// ------------------------------------------------------------------------------ YIELD DISTINCT
__device__ __forceinline__ uint64_t dmix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint8_t dType(const DistinctArgs& a, const OutCol& c, int y, uint64_t r) {
    const uint8_t t = c.t ? c.t[r] : a.vt[y];
    return (t == V_INT || t == V_DBL || t == V_BOOL || t == V_STR) ? t : 0;
}
__device__ __forceinline__ uint64_t dBits(uint8_t t, int64_t x) {
    if (t == 0) return 0;
    if (t == V_DBL) {
        const double d = __longlong_as_double(x);
        if (d == 0.0) return 0;                           // -0.0 == 0.0
        if (d != d) return 0x7FF8000000000000ULL;         // every NaN alike
    }
    return static_cast<uint64_t>(x);
}
__device__ uint64_t rowHash(const DistinctArgs& a, uint64_t r) {
    uint64_t h = 0x9E3779B97F4A7C15ULL;
    for (int y = 0; y < a.nY; y++) {
        const OutCol& c = a.cols[y];
        const uint8_t t = dType(a, c, y, r);
        h = dmix(h ^ t);
        if (t == V_STR) {
            const uint32_t len = c.len ? c.len[r] : 0;
            const char* p = reinterpret_cast<const char*>(c.x[r]);
            uint64_t w = len;
            for (uint32_t i = 0; i < len; i++) w = (w ^ static_cast<uint8_t>(p[i])) * 0x100000001B3ULL;
            h = dmix(h ^ w);
        } else {
            h = dmix(h ^ dBits(t, c.x[r]));
        }
    }
    return h;
}
__device__ bool rowsEqual(const DistinctArgs& a, uint64_t r, uint64_t o) {
    for (int y = 0; y < a.nY; y++) {
        const OutCol& c = a.cols[y];
        const uint8_t t = dType(a, c, y, r);
        if (t != dType(a, c, y, o)) return false;
        if (t == V_STR) {
            const uint32_t l1 = c.len ? c.len[r] : 0, l2 = c.len ? c.len[o] : 0;
            if (l1 != l2) return false;
            const char* p1 = reinterpret_cast<const char*>(c.x[r]);
            const char* p2 = reinterpret_cast<const char*>(c.x[o]);
            for (uint32_t i = 0; i < l1; i++) if (p1[i] != p2[i]) return false;
        } else if (dBits(t, c.x[r]) != dBits(t, c.x[o])) {
            return false;
        }
    }
    return true;
}
__global__ __launch_bounds__(256) void k_distinct_mark(DistinctArgs a) {
    const uint64_t r = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (r >= a.n) return;
    const uint64_t h = rowHash(a, r);
    const uint64_t tag = (h >> 32) << 32;
    const uint64_t mine = tag | (r + 1);
    uint64_t slot = h & a.mask;
    for (uint64_t probes = 0; probes <= a.mask; probes++) {
        uint64_t cur = atomicCAS(reinterpret_cast<unsigned long long*>(a.table + slot), 0ULL,
                                 static_cast<unsigned long long>(mine));
        if (cur == 0) { a.keep[r] = 1; return; }
        if ((cur >> 32) << 32 == tag && rowsEqual(a, r, (cur & 0xFFFFFFFFULL) - 1)) { a.keep[r] = 0; return; }
        slot = (slot + 1) & a.mask;
    }
    a.keep[r] = 1;                                        // unreachable: the table has >= 2n slots
}
__global__ __launch_bounds__(256) void k_scatter_kept(ScatterArgs a) {
    const uint64_t r = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (r >= a.n || !a.keep[r]) return;
    const uint64_t to = a.pre[r];
    for (int k = 0; k < a.k; k++) {
        switch (a.esz[k]) {
            case 1: a.dst[k][to] = a.src[k][r]; break;
            case 4: reinterpret_cast<uint32_t*>(a.dst[k])[to] = reinterpret_cast<const uint32_t*>(a.src[k])[r]; break;
            default: reinterpret_cast<uint64_t*>(a.dst[k])[to] = reinterpret_cast<const uint64_t*>(a.src[k])[r]; break;
        }
    }
}

// 16-byte units of a batch of arrays, grid-stride; unit u of array k covers bytes [16 (u - start[k]) ..)
__global__ __launch_bounds__(256) void k_copy_batch(CopyBatch b) {
    const uint64_t total = b.start[b.n];
    for (uint64_t u = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; u < total;
         u += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
        int k = 0;
        while (k + 1 < b.n && b.start[k + 1] <= u) k++;
        const uint64_t off = (u - b.start[k]) * 16;
        const uint64_t left = b.bytes[k] - off;
        if (left >= 16 && ((reinterpret_cast<uintptr_t>(b.src[k]) | reinterpret_cast<uintptr_t>(b.dst[k])) & 15) == 0) {
            const uint4 v = *reinterpret_cast<const uint4*>(b.src[k] + off);
            *reinterpret_cast<uint4*>(b.dst[k] + off) = v;
        } else {
            const uint64_t m = left < 16 ? left : 16;
            for (uint64_t i = 0; i < m; i++) b.dst[k][off + i] = b.src[k][off + i];
        }
    }
}


// ------------------------------------------------------------------------------ final hop (interpreter)
struct VmEv {
    static constexpr int kEager = -1;                 // YIELD evaluated in the write pass
    static constexpr bool kRankConst = false;         // rank columns read per slot (or its constant)
    static constexpr bool kPos32 = false;             // 64-bit CSR positions in the chunk map
    static constexpr bool kMask = true;               // reads FinalArgs::mask when set
    static constexpr int kDstW = 0, kRankW = 0;       // key column widths read per slot
    static constexpr bool kDrow = true;               // programs may read $$ props
    static constexpr bool kFlat = false;              // branchy passes(): programs evaluated only when needed
    static constexpr bool kEflags = true, kTtl = true; // per-edge flags / TTL read when the slot has them
    static constexpr int kEtype = 0;                  // edge type read per slot
    static constexpr int kRowMask = 7;                // row arrays: written where FinalArgs::o* is set
    static constexpr bool kNeedRow = true;            // programs may read the src row ($^ props, e._src)
    static constexpr bool kNtStore = false;
    static constexpr int kOutSrcW = 0, kOutDstW = 0, kOutRankW = 0;   // row array widths from FinalArgs
    static __device__ __forceinline__ void YV(const FinalArgs&, const EdgeCtx&, Val*) {}
    static __device__ __forceinline__ void YS(const FinalArgs&, const Val*, uint64_t, uint32_t&) {}
    static __device__ __forceinline__ bool hasP(const FinalArgs& a) { return a.P != nullptr; }
    static __device__ __forceinline__ bool hasW(const FinalArgs& a) { return a.W != nullptr; }
    static __device__ __forceinline__ Val P(const FinalArgs& a, const EdgeCtx& ec) { return vmEval(a.P, a.env, ec); }
    static __device__ __forceinline__ Val W(const FinalArgs& a, const EdgeCtx& ec) { return vmEval(a.W, a.env, ec); }
    static __device__ __forceinline__ void Y(const FinalArgs& a, const EdgeCtx& ec, uint64_t o, uint32_t& errs) {
        for (int y = 0; y < a.nY; y++) {
            const OutCol& oc = outCol(a, y);
            Val v;
            if (a.ySlotType != nullptr && a.ySlotType[y] != 0 && a.ySlotType[y] != ec.etype) {
                v.t = 0xFF; v.len = 0; v.x = 0;              // column of another edge type (GetNeighbors)
            } else {
                const uint32_t sb = y < 32 ? (a.strOutMask >> y) & 1u : 0u;
                v = vmEval(a.yCode + a.yOff[y], a.env, ec,
                           sb ? strSlot(a, o, __popc(a.strOutMask & ((1u << y) - 1u))) : nullptr);
                if (v.t == V_ERR) errs |= 1u;
                else if (a.yColType != nullptr && !cellTypeOk(a.yColType[y], v.t)) errs |= 4u;
            }
            if (oc.x) storeW(oc.x, oc.w, o, v.x);         // no array: a constant column (aliased rank)
            if (oc.len) gst<uint32_t>(oc.len, o, v.len);
            if (oc.t) gst<uint8_t>(oc.t, o, v.t);
        }
    }
};

template <bool ONE, bool FIDX>
__global__ __launch_bounds__(WG) void k_final(FinalArgs a) { finalBody<VmEv, ONE, FIDX, FIDX>(a); }
// a GO whose frontier entries carry input rows (FinalArgs::fin: multi-root pipe walks reading $-)
template <bool ONE>
__global__ __launch_bounds__(WG) void k_final_in(FinalArgs a) { finalBody<VmEv, ONE, true, false>(a); }

// ------------------------------------------------------------------------------ GO final hop: close
// After the final kernel (kargs.h resv*): every group's last block is partly empty, so physical rows
// [0, P) hold R rows with at most resvG holes. The i-th occupied row at or past R moves to the i-th
// hole below R (as many of one as of the other; a thread per moved row), then [0, R) is dense.
// Workgroup 0 publishes R and the error bits to host-mapped memory at once (the final kernel has
// ended, so every error atomic of it has landed), keeps R in the control words and clears the other
// set of counters for the next launch: no count of finished workgroups (another same-address stream).
// The moves complete in the stream's order, before any later work on the context's stream.
struct CloseHead {
    uint64_t hLo[kResvMaxGroups], hHi[kResvMaxGroups], gV[kResvMaxGroups];
    uint64_t R, P, M;
    uint64_t tsum[NW];                  // a.dynTiles: per-wave partial sums (workgroup 0)
    int nh;
};
// every workgroup: the groups' counts and last blocks (one load round trip), the holes sorted, R and
// M; workgroup (0, 0) also publishes R and clears the next launch's counters. Plain loads: the words
// were last written by the final kernel (an earlier launch on the stream), and every workgroup reads
// the same 17 of them — as device-scope atomic loads each went to the memory side, one same-address
// queue for ~1300 workgroups (r04 SQ pass: 10 us per wave, 13 us per close)
template <class A>
__device__ __forceinline__ void closeHead(const A& a, CloseHead& h, bool first) {
    const uint64_t B = 1ULL << a.resvShift, st = a.resvStride;
    const uint32_t G = a.resvG;
    if (threadIdx.x < G) {
        const uint32_t g = threadIdx.x;
        const uint64_t v = gld<uint64_t>(a.resvCtl, (1 + g) * st);
        h.gV[g] = v;
        h.hLo[g] = h.hHi[g] = 0;
        if (v & (B - 1)) {
            const uint64_t k = v >> a.resvShift;
            const uint64_t e = k < a.resvTB ? gld<uint64_t>(a.resvTab, static_cast<uint64_t>(g) * a.resvTB + k) : 0;
            if ((e >> 32) != a.resvSeq) {
                atomicOr(a.err + 3, 1u);                    // every reserved block is published: cannot happen
            } else {
                h.hLo[g] = ((e & 0xFFFFFFFFULL) << a.resvShift) + (v & (B - 1));
                h.hHi[g] = ((e & 0xFFFFFFFFULL) + 1) << a.resvShift;
            }
        }
    }
    if (threadIdx.x == WG - 1) h.P = gld<uint64_t>(a.resvCtl, 0);
    if (first && a.dynTiles != nullptr) {                   // the dense final hop's frontier total (its
        uint64_t t = 0;                                     // count launch's tiles, written before the final)
        for (uint64_t i = threadIdx.x; i < a.nDynTiles; i += WG) t += gld<uint64_t>(a.dynTiles, i);
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) t += __shfl_xor(t, o, 64);
        if ((threadIdx.x & 63) == 0) h.tsum[threadIdx.x >> 6] = t;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t R = 0;
        int nh = 0;
        for (uint32_t g = 0; g < G; g++) {                  // holes sorted by position (insertion sort)
            R += h.gV[g];
            if (h.hHi[g] == 0) continue;
            const uint64_t lo = h.hLo[g], hi = h.hHi[g];
            int j = nh++;
            while (j > 0 && h.hLo[j - 1] > lo) { h.hLo[j] = h.hLo[j - 1]; h.hHi[j] = h.hHi[j - 1]; j--; }
            h.hLo[j] = lo;
            h.hHi[j] = hi;
        }
        uint64_t M = 0;
        for (int j = 0; j < nh; j++) M += h.hLo[j] < R ? (h.hHi[j] < R ? h.hHi[j] : R) - h.hLo[j] : 0;
        h.R = R;
        h.M = M;
        h.nh = nh;
        if (first) {
            // the hop's packed (|F|, E): summed here from the count launch's tiles (dense final hop, whose
            // kernel never reads it; the word is the device copy the final kernel would otherwise take), or
            // as the compaction left it
            uint64_t tot = 0;
            if (a.dynTiles != nullptr) {
                for (int w = 0; w < NW; w++) tot += h.tsum[w];
                *const_cast<uint64_t*>(a.dynTotal) = tot;
            } else if (a.dynTotal != nullptr) {
                tot = gld<uint64_t>(a.dynTotal, 0);
            }
            lbStore(a.resvCtl + (1 + G) * st, R);           // the row count (device copy; dyn hops read it)
            for (uint32_t g = 0; g <= G; g++) lbStore(a.resvNext + g * st, 0);   // the next launch's counters
            if (a.rowsPub != nullptr) {
                uint64_t bits = 0;
                for (int k = 0; k < 4; k++)
                    bits |= static_cast<uint64_t>(__hip_atomic_load(a.err + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) << k;
                publishWords(a.rowsPub, a.rowsSeq, R, bits, tot);
            }
        }
    }
    __syncthreads();
}

// move i (< M): the i-th hole row below R (to) and the i-th occupied row in [R, P) (from); false if
// the counts disagree (cannot happen)
__device__ __forceinline__ bool closePair(const CloseHead& h, uint64_t i, uint64_t& to, uint64_t& from) {
    const uint64_t R = h.R;
    to = ~0ULL;
    uint64_t acc = 0;
    for (int j = 0; j < h.nh && h.hLo[j] < R; j++) {
        const uint64_t len = (h.hHi[j] < R ? h.hHi[j] : R) - h.hLo[j];
        if (i < acc + len) { to = h.hLo[j] + (i - acc); break; }
        acc += len;
    }
    from = ~0ULL;
    uint64_t cur = R, left = i;
    for (int j = 0; j <= h.nh; j++) {
        if (j < h.nh && h.hHi[j] <= R) continue;
        const uint64_t segEnd = j < h.nh ? h.hLo[j] : h.P;
        if (segEnd > cur) {
            if (left < segEnd - cur) { from = cur + left; break; }
            left -= segEnd - cur;
        }
        if (j < h.nh && h.hHi[j] > cur) cur = h.hHi[j];
    }
    return to != ~0ULL && from != ~0ULL;
}

__device__ __forceinline__ void closeMove(const FinalArgs& a, uint64_t from, uint64_t to);
// fallback (more columns than CloseCols holds): a thread per moved row, every column of it
__global__ __launch_bounds__(WG) void k_final_close(FinalArgs a) {
    __shared__ CloseHead h;
    closeHead(a, h, blockIdx.x == 0);
    for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * WG + threadIdx.x; i < h.M; i += static_cast<uint64_t>(gridDim.x) * WG) {
        uint64_t to, from;
        if (!closePair(h, i, to, from)) { atomicOr(a.err + 3, 1u); return; }
        closeMove(a, from, to);
    }
}

// A workgroup column (blockIdx.y) of one moved array: each thread moves kCloseBatch rows of it, every
// load of the batch issued before its stores (one width per launch row, no branch between them).
constexpr int kCloseBatch = 8;
template <typename T, int KIND>
__device__ __forceinline__ void closeColumn(const CloseArgs& a, const CloseHead& h, const CloseCol& col) {
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * WG;
    for (uint64_t i0 = static_cast<uint64_t>(blockIdx.x) * WG + threadIdx.x; i0 < h.M; i0 += stride * kCloseBatch) {
        uint64_t to[kCloseBatch], from[kCloseBatch];
        T v[kCloseBatch];
        bool ok = true;
#pragma unroll
        for (int k = 0; k < kCloseBatch; k++) {
            const uint64_t i = i0 + k * stride;
            to[k] = from[k] = 0;
            if (i < h.M) ok = closePair(h, i, to[k], from[k]) && ok;
            to[k] += a.oBase;
            from[k] += a.oBase;
        }
        if (!ok) { atomicOr(a.err + 3, 1u); return; }
#pragma unroll
        for (int k = 0; k < kCloseBatch; k++) {
            const uint64_t i = i0 + k * stride;
            if (KIND == 2) v[k] = i < h.M ? gld<T>(a.strOut, ((from[k] - a.oBase) * a.nStrOut * kStrBuildBytes) / 8 + col.w) : T(0);
            else v[k] = i < h.M ? gld<T>(col.p, from[k]) : T(0);
        }
#pragma unroll
        for (int k = 0; k < kCloseBatch; k++) {
            const uint64_t i = i0 + k * stride;
            if (i >= h.M) continue;
            if (KIND == 2) {
                gst<T>(a.strOut, ((to[k] - a.oBase) * a.nStrOut * kStrBuildBytes) / 8 + col.w, v[k]);
            } else if (KIND == 1) {
                // a string value pointing into the row's own arena slots moves with them
                uint64_t ux = static_cast<uint64_t>(v[k]);
                const uint64_t slotBytes = static_cast<uint64_t>(a.nStrOut) * kStrBuildBytes;
                const uint64_t sFrom = reinterpret_cast<uint64_t>(a.strOut) + (from[k] - a.oBase) * slotBytes;
                const uint64_t sTo = reinterpret_cast<uint64_t>(a.strOut) + (to[k] - a.oBase) * slotBytes;
                if (ux >= sFrom && ux < sFrom + slotBytes) ux = ux - sFrom + sTo;
                gst<T>(col.p, to[k], static_cast<T>(ux));
            } else {
                gst<T>(col.p, to[k], v[k]);
            }
        }
    }
}

// (its own small argument block: the fields sit in two cache lines, where FinalArgs spreads the ones
// the close reads over 2.3 KB of kernel arguments, each line a scalar-cache miss on every CU)
__global__ __launch_bounds__(WG) void k_final_close_cols(CloseArgs a, CloseCols cc) {
    __shared__ CloseHead h;
    closeHead(a, h, blockIdx.x == 0 && blockIdx.y == 0);
    const CloseCol col = cc.c[blockIdx.y];
    if (col.kind == 2) closeColumn<uint64_t, 2>(a, h, col);
    else if (col.kind == 1) closeColumn<uint64_t, 1>(a, h, col);
    else if (col.w == 1) closeColumn<uint8_t, 0>(a, h, col);
    else if (col.w == 2) closeColumn<uint16_t, 0>(a, h, col);
    else if (col.w == 4) closeColumn<uint32_t, 0>(a, h, col);
    else closeColumn<uint64_t, 0>(a, h, col);
}

__device__ __forceinline__ void closeMove(const FinalArgs& a, uint64_t from, uint64_t to) {
    from += a.oBase;
    to += a.oBase;
    // every load of the row issued before its first store (a load after a store to another array
    // waits for it: the compiler cannot tell the arrays apart), in batches of registers
    const uint64_t slotBytes = static_cast<uint64_t>(a.nStrOut) * kStrBuildBytes;
    char* const sFrom = a.strOut ? strSlot(a, from, 0) : nullptr;
    char* const sTo = a.strOut ? strSlot(a, to, 0) : nullptr;
    {
        const int64_t v0 = a.oSrc ? loadW(a.oSrc, a.oSrcW, from) : 0;
        const int64_t v1 = a.oDst ? loadW(a.oDst, a.oDstW, from) : 0;
        const int64_t v2 = a.oRank ? loadW(a.oRank, a.oRankW, from) : 0;
        const int32_t v3 = a.oType ? gld<int32_t>(a.oType, from) : 0;
        const uint32_t v4 = a.oEntry ? gld<uint32_t>(a.oEntry, from) : 0;
        const uint8_t v5 = a.oFlags ? gld<uint8_t>(a.oFlags, from) : 0;
        if (a.oSrc) storeW(a.oSrc, a.oSrcW, to, v0);
        if (a.oDst) storeW(a.oDst, a.oDstW, to, v1);
        if (a.oRank) storeW(a.oRank, a.oRankW, to, v2);
        if (a.oType) gst<int32_t>(a.oType, to, v3);
        if (a.oEntry) gst<uint32_t>(a.oEntry, to, v4);
        if (a.oFlags) gst<uint8_t>(a.oFlags, to, v5);
    }
    // strings the row's YIELD columns built live in its slots of the result string arena: they move
    // with the row, and a value pointing into them is rebased
    for (uint64_t b = 0; sFrom && b < slotBytes; b += 64) {
        uint64_t w[8];
#pragma unroll
        for (int k = 0; k < 8; k++) w[k] = b + 8 * k < slotBytes ? gld<uint64_t>(sFrom, b / 8 + k) : 0;
#pragma unroll
        for (int k = 0; k < 8; k++) if (b + 8 * k < slotBytes) gst<uint64_t>(sTo, b / 8 + k, w[k]);
    }
    constexpr int kB = 4;                                   // YIELD columns per batch
    for (int y0 = 0; y0 < a.nY; y0 += kB) {
        int64_t x[kB];
        uint32_t len[kB];
        uint8_t t[kB];
#pragma unroll
        for (int k = 0; k < kB; k++) {
            x[k] = 0; len[k] = 0; t[k] = 0;
            if (y0 + k >= a.nY) continue;
            const OutCol& oc = outCol(a, y0 + k);
            // a key column aliased to a row array moved with it
            if (oc.x && oc.x != a.oSrc && oc.x != a.oDst && oc.x != a.oRank) x[k] = loadW(oc.x, oc.w, from);
            if (oc.len) len[k] = gld<uint32_t>(oc.len, from);
            if (oc.t) t[k] = gld<uint8_t>(oc.t, from);
        }
#pragma unroll
        for (int k = 0; k < kB; k++) {
            if (y0 + k >= a.nY) continue;
            const OutCol& oc = outCol(a, y0 + k);
            if (oc.x && oc.x != a.oSrc && oc.x != a.oDst && oc.x != a.oRank) {
                const uint64_t ux = static_cast<uint64_t>(x[k]);
                if (oc.len && sFrom && ux >= reinterpret_cast<uint64_t>(sFrom) && ux < reinterpret_cast<uint64_t>(sFrom) + slotBytes)
                    x[k] = static_cast<int64_t>(ux - reinterpret_cast<uint64_t>(sFrom) + reinterpret_cast<uint64_t>(sTo));
                storeW(oc.x, oc.w, to, x[k]);
            }
            if (oc.len) gst<uint32_t>(oc.len, to, len[k]);
            if (oc.t) gst<uint8_t>(oc.t, to, t[k]);
        }
    }
}

// ------------------------------------------------------------------------------ max_edge_returned_per_vertex
// Storage outcome of every hop edge (bad row / TTL / pushed filter; the interpreter evaluates the
// filter) -> out[e] = 1 if the processor would emit it, before the per-vertex cap.
template <bool ONE>
__global__ __launch_bounds__(WG) void k_storage_pass(FinalArgs a, uint8_t* out) {
    __shared__ ChunkMap<ONE, false, false> m;
    const uint64_t base = static_cast<uint64_t>(blockIdx.x) * CE;
    const uint32_t cnt = static_cast<uint32_t>(a.E - base < CE ? a.E - base : CE);
    buildMap<ONE, false, false>(a.estart, a.chunkFirst, a.nEnt, blockIdx.x, gridDim.x, base, cnt, a.F, a.hs, m, a.ebase);
    for (int k = 0; k < CITEMS; k++) {
        uint32_t p = threadIdx.x + k * WG;
        if (p >= cnt) continue;
        EdgeCtx ec;
        int s;
        edgeCtxAt<VmEv, ONE, false, false>(a, m, base, p, ec, s);
        bool pe = false;
        out[base + p] = storagePass<VmEv>(a, ec, s, pe) ? 1 : 0;
    }
}

// collectEdgeProps stops once `cap` edges of the (vertex, type) prefix were emitted, in key order
// (QueryBaseProcessor.inl:501-505, ++cnt at :606): keep the first `cap` set flags of every frontier
// entry (its hop edges estart[i] .. estart[i + 1] - 1, in key order), clear the rest.
__global__ void k_cap(const uint64_t* estart, uint64_t nEnt, uint8_t* mask, int64_t cap) {
    uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= nEnt) return;
    uint64_t lo = estart[i], hi = estart[i + 1];
    if (hi - lo <= static_cast<uint64_t>(cap)) return;
    int64_t kept = 0;
    for (uint64_t e = lo; e < hi; e++) {
        if (!mask[e]) continue;
        if (kept < cap) kept++;
        else mask[e] = 0;
    }
}

// ------------------------------------------------------------------------------ vertex cells
__global__ void k_vertex_cells(VertexCellArgs a) {
    uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    uint32_t r = a.rows[i];
    for (int c = 0; c < a.ncols; c++) {
        OutCell out{0, 0, 0xFF};
        int tslot = a.tagSlot[c];
        if (tslot >= 0 && r != kNoRow) {
            const DTag& t = a.env.tags[tslot];
            if (!tagAbsent(a.env, t, r)) {
                const DCol& col = a.env.cols[t.colBase + a.col[c]];
                Val v = (col.valid != nullptr && col.valid[r] == 0) ? defaultOfType(col.type) : loadCol(col, r);
                out.t = v.t; out.len = v.len; out.x = v.x;
            }
        }
        a.out[i * a.ncols + c] = out;
    }
}

// ------------------------------------------------------------------------------ response rows
// RowWriter rows of response schemas (rowcodec.h), one thread per returned edge
// the data part of row i of slot sl; offs gets the block offsets (their count returned in nb)
__device__ __forceinline__ void rowCord(const RowEncArgs& a, uint64_t i, int sl, RowSink& s, uint64_t* offs, int& nb) {
    const int b = a.cbeg[sl], nf = a.cbeg[sl + 1] - b;
    const bool reader = !(a.oFlags != nullptr && (a.oFlags[i] & EF_EMPTY_VALUE));
    int col = 0;
    nb = 0;
    for (int j = 0; j < nf; j++) {
        const int32_t src = a.rcSrc[b + j];
        const int32_t ft = a.rcType[b + col];            // the field the next write lands in
        if (src == kRcSrc) rowField(s, V_INT, a.oSrc[i], 0, ft);
        else if (src == kRcRank) rowField(s, V_INT, a.oRank[i], 0, ft);
        else if (src == kRcType) rowField(s, V_INT, a.oType[i], 0, ft);
        else if (!reader) continue;                      // collectProps without a RowReader: not collected
        else {
            const OutCol& oc = a.cols[src];
            rowField(s, oc.t != nullptr ? oc.t[i] : V_INT, oc.x[i], oc.len != nullptr ? oc.len[i] : 0u, ft);
        }
        col++;
        if ((col & 15) == 0) offs[nb++] = s.n;         // RW_CLEAN_UP_WRITE: every 16 fields written
    }
    for (int k = col; k < nf; k++) {                    // encode(): Skip the fields never written
        rowDefault(s, a.rcType[b + k]);
        if (k != 0 && (k & 15) == 0) offs[nb++] = s.n;  // Skip's own block check (on the field index)
    }
}

__global__ void k_encode_rows(RowEncArgs a, int write) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    int sl = -1;
    for (int s = 0; s < a.nslots; s++) if (a.etype[s] == a.oType[i]) sl = s;
    if (sl < 0 || a.cbeg[sl + 1] == a.cbeg[sl]) {        // onlyStructure type: no props
        if (!write) a.rowLen[i] = 0;
        return;
    }
    uint64_t offs[kMaxRespCols / 16 + 2];
    int nb = 0;
    RowSink cs{nullptr, 0};
    rowCord(a, i, sl, cs, offs, nb);
    const int ob = rowOffsetBytes(cs.n);
    if (!write) {
        a.rowLen[i] = 1 + static_cast<uint64_t>(nb) * ob + cs.n;
        return;
    }
    uint8_t* dst = a.out + a.rowOff[i];
    RowSink hs{dst, 0};
    hs.put(static_cast<uint8_t>(ob - 1));
    for (int k = 0; k < nb; k++) hs.le(offs[k], ob);
    RowSink ws{dst + hs.n, 0};
    rowCord(a, i, sl, ws, offs, nb);
}

// ------------------------------------------------------------------------------ result digest
__device__ __forceinline__ uint64_t digestMix(uint64_t z) {        // splitmix64's finalizer
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

// a grid-stride pass over the rows; per wave one atomic per word
__global__ __launch_bounds__(256) void k_row_digest(DigestArgs a) {
    uint64_t sum = 0, x = 0, cnt = 0;
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
    for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < a.n; i += stride) {
        uint64_t h = kDigestSeed;
        for (int k = 0; k <= a.ncols; k++) {
            const int64_t v = a.w[k] == 0 ? a.c[k] : loadW(a.x[k], a.w[k], i);
            h = digestMix(h ^ static_cast<uint64_t>(v));
        }
        sum += h;
        x ^= h;
        cnt++;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        sum += __shfl_xor(sum, o, 64);
        x ^= __shfl_xor(x, o, 64);
        cnt += __shfl_xor(cnt, o, 64);
    }
    if ((threadIdx.x & 63) == 0 && cnt) {
        atomicAdd(reinterpret_cast<unsigned long long*>(a.out), static_cast<unsigned long long>(sum));
        atomicXor(reinterpret_cast<unsigned long long*>(a.out + 1), static_cast<unsigned long long>(x));
        atomicAdd(reinterpret_cast<unsigned long long*>(a.out + 2), static_cast<unsigned long long>(cnt));
    }
}

int launchRowDigest(const DigestArgs& a, hipStream_t s) {
    if (hipMemsetAsync(a.out, 0, 24, s) != hipSuccess) return 1;
    if (a.n == 0) return 0;
    const uint64_t blocks = std::min<uint64_t>((a.n + 255) / 256, 4096);
    hipLaunchKernelGGL(k_row_digest, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, s, a);
    return static_cast<int>(hipGetLastError());
}

struct ArrIn {
    const uint64_t* v;
    __device__ __forceinline__ uint64_t operator()(uint64_t i) const { return v[i]; }
};
struct WriteArr {
    uint64_t* out;
    __device__ __forceinline__ void operator()(uint64_t i, uint64_t v, uint64_t pre) const { (void)v; out[i] = pre; }
};

// ------------------------------------------------------------------------------ multi-GPU exchange
// pack this shard's marks for peer q's rows into a bitmap: one row byte per lane (coalesced), the
// wave's ballot is the 64-bit word of its 64 rows; merge received bitmaps into visited
// grid.y = peer; a wave's ballot is one bitmap word (the whole block leaves together for q == rank)
__global__ __launch_bounds__(256) void k_pack(const ExchangeArgs a) {
    const int q = blockIdx.y;
    if (q == a.rank) return;
    const uint64_t lo = a.sb[q], n = a.sb[q + 1] - lo;
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    const bool mark = i < n && a.visited[lo + i] == a.epoch;
    const uint64_t word = __ballot(mark);
    if ((threadIdx.x & 63) == 0 && i < n) a.bits[q * a.words + (i >> 6)] = word;
}
// one thread per own row: the OR over the peers' words (each a wave-wide broadcast load), one store
__global__ __launch_bounds__(256) void k_merge(const ExchangeArgs a) {
    const uint64_t lo = a.sb[a.rank], n = a.sb[a.rank + 1] - lo;
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t any = 0;
    for (int q = 0; q < a.world; q++)
        if (q != a.rank) any |= a.bits[q * a.words + (i >> 6)];
    if ((any >> (i & 63)) & 1) a.visited[lo + i] = a.epoch;
}

// ------------------------------------------------------------------------------ launchers
int launchLookup(const int32_t* qpart, const int64_t* qvid, uint64_t n, const int32_t* vpart, const int64_t* vid,
                 uint64_t V, uint32_t* out, hipStream_t s) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_lookup, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, s, qpart, qvid, n, vpart, vid, V, out);
    return static_cast<int>(hipGetLastError());
}

int launchIndexLookup(const int32_t* qpart, const int64_t* qvid, uint64_t n, VIndex idx, uint32_t* out, hipStream_t s) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_index_lookup, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, s, qpart, qvid, n, idx, out);
    return static_cast<int>(hipGetLastError());
}

int launchDegreeScan(const uint32_t* F, uint64_t nEnt, const HopSlots& hs, uint64_t* estart, uint64_t* tileSums,
                     hipStream_t s, Publish pub) {
    return scan3(DegreeIn{F, hs}, nEnt, WriteEstart{estart}, tileSums, estart + nEnt, s, nullptr, 0, pub);
}

int launchSeedFrontierCf(const int32_t* qpart, const int64_t* qvid, uint64_t n, VIndex idx, const HopSlots& hs,
                         uint32_t* F, uint64_t* estart, Publish pub, uint64_t* chunkFirst, uint64_t cfCap,
                         uint64_t* zero, uint32_t nzero, uint32_t* err, hipStream_t s, uint64_t* packedOut,
                         uint64_t* zero8, uint64_t* ebase) {
    if (n * static_cast<uint64_t>(hs.n) > kSeedFuseMax || n > kSeedFuseMax || idx.slots == nullptr || nzero > 64) return 1;
    const unsigned g = static_cast<unsigned>(std::max<uint64_t>((n + 63) / 64, 1));   // block 0 also clears
    hipLaunchKernelGGL(k_seed_lookup, dim3(g), dim3(64), 0, s, qpart, qvid, n, idx, hs,
                       F, estart, ebase, zero, nzero, zero8);
    hipLaunchKernelGGL(k_seed_scan, dim3(1), dim3(kSeedScanWG), 0, s, n, hs.n, estart, pub, chunkFirst, cfCap, err, packedOut);
    return static_cast<int>(hipGetLastError());
}

int launchChunkFirst(const uint64_t* estart, uint64_t nEnt, uint64_t* chunkFirst, hipStream_t s, uint64_t* zero,
                     uint64_t nzero) {
    if (nEnt == 0 && nzero == 0) return 0;
    uint64_t n = nEnt > nzero ? nEnt : nzero;
    hipLaunchKernelGGL(k_chunk_first, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, s, estart, nEnt, chunkFirst,
                       zero, nzero);
    return static_cast<int>(hipGetLastError());
}

int launchExpandSparse(const SparseArgs& a, bool pos32, hipStream_t s) {
    if (a.E == 0 && a.dynIn == nullptr) return 1;       // the host handles an empty hop
    // dynIn: the hop's size is on the device; a fixed grid (4 workgroups per CU) strides over its slices
    const dim3 grid(a.dynIn != nullptr ? 1024u : static_cast<unsigned>((a.E + CE - 1) / CE * kSparseSub));
    if (a.hs.n == 1 && pos32) hipLaunchKernelGGL((k_expand_sparse<true, true>), grid, dim3(WG), 0, s, a);
    else if (a.hs.n == 1) hipLaunchKernelGGL((k_expand_sparse<true, false>), grid, dim3(WG), 0, s, a);
    else if (pos32) hipLaunchKernelGGL((k_expand_sparse<false, true>), grid, dim3(WG), 0, s, a);
    else hipLaunchKernelGGL((k_expand_sparse<false, false>), grid, dim3(WG), 0, s, a);
    return static_cast<int>(hipGetLastError());
}

int launchExpandMark(const uint32_t* F, const uint64_t* estart, const uint64_t* chunkFirst, uint64_t nEnt, uint64_t E,
                     const HopSlots& hs, uint8_t* visited, uint8_t epoch, bool pos32, hipStream_t s, const uint8_t* mask,
                     const uint64_t* dyn, uint64_t pullMinE, const uint64_t* ebase) {
    if (E == 0) return 0;
    // dyn: E is an upper bound here; the grid strides (kDynGrid workgroups at most)
    dim3 grid(static_cast<unsigned>(std::min<uint64_t>((E + CE - 1) / CE, dyn ? kDynGrid : ~0u)));
#define NGX_EXPAND(ONE, P32, MASK) hipLaunchKernelGGL((k_expand_mark<ONE, P32, MASK>), grid, dim3(WG), 0, s, F, estart, \
                                                    chunkFirst, nEnt, E, hs, visited, epoch, mask, dyn, pullMinE, ebase)
    if (mask) {
        if (hs.n == 1) NGX_EXPAND(true, false, true);
        else NGX_EXPAND(false, false, true);
    } else if (hs.n == 1 && pos32) NGX_EXPAND(true, true, false);
    else if (hs.n == 1) NGX_EXPAND(true, false, false);
    else if (pos32) NGX_EXPAND(false, true, false);
    else NGX_EXPAND(false, false, false);
#undef NGX_EXPAND
    return static_cast<int>(hipGetLastError());
}

int launchStoragePass(const FinalArgs& a, uint8_t* out, hipStream_t s) {
    if (a.E == 0) return 0;
    dim3 grid(static_cast<unsigned>((a.E + CE - 1) / CE));
    if (a.hs.n == 1) hipLaunchKernelGGL((k_storage_pass<true>), grid, dim3(WG), 0, s, a, out);
    else hipLaunchKernelGGL((k_storage_pass<false>), grid, dim3(WG), 0, s, a, out);
    return static_cast<int>(hipGetLastError());
}

int launchCap(const uint64_t* estart, uint64_t nEnt, uint8_t* mask, int64_t cap, hipStream_t s) {
    if (nEnt == 0) return 0;
    hipLaunchKernelGGL(k_cap, dim3(static_cast<unsigned>((nEnt + 255) / 256)), dim3(256), 0, s, estart, nEnt, mask, cap);
    return static_cast<int>(hipGetLastError());
}

int launchCompact(const uint8_t* visited, uint64_t gbase, uint64_t V, uint8_t epoch, uint32_t* outF, uint64_t* tileSums,
                  uint64_t* count, hipStream_t s) {
    return scan3(FlagIn{visited, gbase, epoch}, V, WriteCompact{outF}, tileSums, count, s);
}

int launchCompactDegrees(const uint8_t* visited, uint64_t gbase, uint64_t V, uint8_t epoch, const HopSlots& hs,
                         uint32_t* outF, uint64_t* estart, uint64_t* tileSums, uint64_t* packedTotal, hipStream_t s,
                         Publish pub) {
    return scan3(FlagDegIn{visited, gbase, epoch, hs}, V, WriteCompactEstart{outF, estart, hs}, tileSums, packedTotal,
                 s, estart, hs.n, pub);
}

// the packed (rows << kFdShift | degrees) total of the count launch's tiles (countOnly: the frontier the
// dense final hop reads from the marks, its size and edges for the statistics)
__global__ __launch_bounds__(256) void k_tile_total(const uint64_t* tileSum, uint64_t tiles, uint64_t* total, Publish pub) {
    __shared__ uint64_t sm[4];
    uint64_t t = 0;
    for (uint64_t i = threadIdx.x; i < tiles; i += 256) t += tileSum[i];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) t += __shfl_xor(t, o, 64);
    if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = t;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint64_t t4 = sm[0] + sm[1] + sm[2] + sm[3];
        *total = t4;
        if (pub.slot) publishWords(pub.slot, pub.seq, t4, 0);      // a host-sized final hop (world > 1)
    }
}

uint64_t compactLbTiles(const CompactArgs& a) {
    const bool small = a.wgThreads == 256;
    const int cit = small ? 16 : a.laneRows != 0 ? a.laneRows : 4;
    const uint64_t tile = static_cast<uint64_t>(small ? 256 : CWG) * cit;
    return std::max<uint64_t>((a.V + tile - 1) / tile, 1);
}

int launchCompactLb(const CompactArgs& a, hipStream_t s) {
    if (a.V >= kCompactLbMaxV || a.nzero > WG) return 1;
    if (a.totalByClose && !a.countOnly) return 1;
    // rows per lane: 4 unless the flag forces 8 or 16 (measured at C2: 8 rows per lane, every wave
    // resident at once, 48 vs 46 us per step for 4 with a second round of waves)
    // 256-thread workgroups (a pipelined batch: one finds room on a CU beside the other query's final-hop
    // workgroups, where a 1024-thread one waits for 16 free wave slots — r05 trace: the count launch 185 us
    // beside the final hop, starved until it drained) take 16 rows per lane, the same 4096-row tile
    const bool small = a.wgThreads == 256;
    const int cit = small ? 16 : a.laneRows != 0 ? a.laneRows : 4;
    const uint64_t tile = static_cast<uint64_t>(small ? 256 : CWG) * cit;
    const dim3 grid(static_cast<unsigned>(std::max<uint64_t>((a.V + tile - 1) / tile, 1)));
#define NGX_COMPACT(ONE, CIT, WGS)                                                              \
    do {                                                                                        \
        hipLaunchKernelGGL((k_compact_count<ONE, CIT, WGS>), grid, dim3(WGS), 0, s, a);         \
        if (a.countOnly && !a.totalByClose)                                                     \
            hipLaunchKernelGGL(k_tile_total, dim3(1), dim3(256), 0, s, a.tileSum, static_cast<uint64_t>(grid.x), a.total, a.pub); \
        else if (a.countOnly) {}                                                                \
        else                                                                                    \
            hipLaunchKernelGGL((k_compact_write<ONE, CIT, WGS>), grid, dim3(WGS), 0, s, a);     \
    } while (0)
    if (small) {
        if (a.hs.n == 1) NGX_COMPACT(true, 16, 256);
        else NGX_COMPACT(false, 16, 256);
    } else if (a.hs.n == 1) {
        if (cit == 4) NGX_COMPACT(true, 4, CWG);
        else if (cit == 8) NGX_COMPACT(true, 8, CWG);
        else NGX_COMPACT(true, 16, CWG);
    } else {
        if (cit == 4) NGX_COMPACT(false, 4, CWG);
        else if (cit == 8) NGX_COMPACT(false, 8, CWG);
        else NGX_COMPACT(false, 16, CWG);
    }
#undef NGX_COMPACT
    return static_cast<int>(hipGetLastError());
}

int launchEncodeRows(const RowEncArgs& a, bool write, hipStream_t s) {
    if (a.n == 0) return 0;
    hipLaunchKernelGGL(k_encode_rows, dim3(static_cast<unsigned>((a.n + 255) / 256)), dim3(256), 0, s, a, write ? 1 : 0);
    return static_cast<int>(hipGetLastError());
}

int launchScanInPlace(uint64_t* v, uint64_t n, hipStream_t s) {
    hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(1024), 0, s, v, n, v + n, nullptr, 0, Publish{nullptr, 0});
    return static_cast<int>(hipGetLastError());
}

int launchScanU64(const uint64_t* in, uint64_t n, uint64_t* out, uint64_t* tileSums, hipStream_t s) {
    return scan3(ArrIn{in}, n, WriteArr{out}, tileSums, out + n, s);
}

int finalOccupancy(const FinalArgs& a) {
    int n = 0;
    if (a.oEntry != nullptr) {
        if (a.hs.n == 1) (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_final<true, true>, WG, 0);
        else (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_final<false, true>, WG, 0);
    } else {
        if (a.hs.n == 1) (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_final<true, false>, WG, 0);
        else (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_final<false, false>, WG, 0);
    }
    return n > 0 ? n : 1;
}

int launchFinal(const FinalArgs& a, hipStream_t s, unsigned g) {
    if (a.E == 0) return 0;
    dim3 grid(g ? g : static_cast<unsigned>((a.E + CE - 1) / CE));
    if (a.fin != nullptr) {
        if (a.hs.n == 1) hipLaunchKernelGGL((k_final_in<true>), grid, dim3(WG), 0, s, a);
        else hipLaunchKernelGGL((k_final_in<false>), grid, dim3(WG), 0, s, a);
    } else if (a.oEntry != nullptr) {
        if (a.hs.n == 1) hipLaunchKernelGGL((k_final<true, true>), grid, dim3(WG), 0, s, a);
        else hipLaunchKernelGGL((k_final<false, true>), grid, dim3(WG), 0, s, a);
    } else {
        if (a.hs.n == 1) hipLaunchKernelGGL((k_final<true, false>), grid, dim3(WG), 0, s, a);
        else hipLaunchKernelGGL((k_final<false, false>), grid, dim3(WG), 0, s, a);
    }
    return static_cast<int>(hipGetLastError());
}

int launchFinalClose(const FinalArgs& a, hipStream_t s) {
    // the moved arrays, one launch row each: row arrays, per-row type / entry / flags, the YIELD
    // columns (values, lengths, types) that are not aliases of a row array, the string arena's words
    CloseCols cc{};
    bool fits = a.nY <= kInlineCols;
    auto add = [&](void* p, int32_t w, int32_t kind) {
        if (!p) return;
        if (cc.n >= kCloseMaxCols) { fits = false; return; }
        cc.c[cc.n++] = CloseCol{p, w, kind};
    };
    add(a.oSrc, a.oSrcW, 0);
    add(a.oDst, a.oDstW, 0);
    add(a.oRank, a.oRankW, 0);
    add(a.oType, 4, 0);
    add(a.oEntry, 4, 0);
    add(a.oFlags, 1, 0);
    for (int y = 0; fits && y < a.nY; y++) {
        const OutCol& oc = a.oColsIn[y];
        if (oc.x && oc.x != a.oSrc && oc.x != a.oDst && oc.x != a.oRank)
            add(oc.x, oc.w, (oc.len && a.strOut && oc.w == 8) ? 1 : 0);
        add(oc.len, 4, 0);
        add(oc.t, 1, 0);
    }
    if (a.strOut) {
        const uint64_t words = static_cast<uint64_t>(a.nStrOut) * kStrBuildBytes / 8;
        for (uint64_t w = 0; fits && w < words; w++) add(a.strOut, static_cast<int32_t>(w), 2);
    }
    if (fits && cc.n > 0) {
        CloseArgs ca{};
        ca.resvCtl = a.resvCtl;
        ca.resvTab = a.resvTab;
        ca.resvNext = a.resvNext;
        ca.err = a.err;
        ca.rowsPub = a.rowsPub;
        ca.rowsSeq = a.rowsSeq;
        ca.strOut = a.strOut;
        ca.oBase = a.oBase;
        ca.dynTotal = a.dynTotal;
        ca.dynTiles = a.dynTiles;
        ca.nDynTiles = a.nDynTiles;
        ca.resvTB = a.resvTB;
        ca.resvSeq = a.resvSeq;
        ca.resvG = a.resvG;
        ca.resvShift = a.resvShift;
        ca.resvStride = a.resvStride;
        ca.nStrOut = a.nStrOut;
        // 8 rows per thread over the rows that may move
        const unsigned gx = static_cast<unsigned>((resvSlack(a) + WG * kCloseBatch - 1) / (WG * kCloseBatch));
        hipLaunchKernelGGL(k_final_close_cols, dim3(gx, static_cast<unsigned>(cc.n)), dim3(WG), 0, s, ca, cc);
    } else {
        const unsigned grid = static_cast<unsigned>((resvSlack(a) + WG - 1) / WG);   // a thread per row that may move
        hipLaunchKernelGGL(k_final_close, dim3(grid), dim3(WG), 0, s, a);
    }
    return static_cast<int>(hipGetLastError());
}

int launchPull(const PullArgs& a, hipStream_t s) {
    if (a.V == 0) return 0;
    if (a.n < 1 || a.n > kPullMaxSlots || a.V >= (1ULL << 31)) return 1;
    const uint64_t slices = a.sliceEnd[a.n - 1];
    if (slices == 0) return 0;
    // a wave per slice; the grid padded to a multiple of 8 for the XCD-aware slice mapping (extra waves exit)
    dim3 grid(static_cast<unsigned>(((slices + NW - 1) / NW + 7) & ~static_cast<uint64_t>(7)));
    if (a.n == 1) hipLaunchKernelGGL((k_pull_head<true>), grid, dim3(WG), 0, s, a);
    else hipLaunchKernelGGL((k_pull_head<false>), grid, dim3(WG), 0, s, a);
    // long unresolved in-lists: at most a.segCap segments, 2 workgroups per CU striding over them
    hipLaunchKernelGGL(k_pull_segments, dim3(256), dim3(WG), 0, s, a);
    return static_cast<int>(hipGetLastError());
}

int launchCopyBatch(const CopyBatch& b, hipStream_t s) {
    if (b.n <= 0 || b.start[b.n] == 0) return 0;
    const uint64_t units = b.start[b.n];
    const unsigned grid = static_cast<unsigned>(std::min<uint64_t>((units + 255) / 256, 4096));
    hipLaunchKernelGGL(k_copy_batch, dim3(grid), dim3(256), 0, s, b);
    return static_cast<int>(hipGetLastError());
}

int launchDistinctMark(const DistinctArgs& a, hipStream_t s) {
    if (a.n == 0) return 0;
    if (a.n >= (1ULL << 32) || a.nY > kMaxDistinctCols) return 1;
    hipLaunchKernelGGL(k_distinct_mark, dim3(static_cast<unsigned>((a.n + 255) / 256)), dim3(256), 0, s, a);
    return static_cast<int>(hipGetLastError());
}

int launchScatterKept(const ScatterArgs& a, hipStream_t s) {
    if (a.n == 0 || a.k == 0) return 0;
    hipLaunchKernelGGL(k_scatter_kept, dim3(static_cast<unsigned>((a.n + 255) / 256)), dim3(256), 0, s, a);
    return static_cast<int>(hipGetLastError());
}

int launchMarkRows(const uint32_t* F, uint64_t n, uint8_t* marks, uint8_t ep, hipStream_t s) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_mark_rows, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, s, F, n, marks, ep);
    return static_cast<int>(hipGetLastError());
}

int launchPublishTail(const uint32_t* err, const uint64_t* extra, int nExtra, uint64_t* slot, uint64_t seq, hipStream_t s) {
    hipLaunchKernelGGL(k_publish_tail, dim3(1), dim3(64), 0, s, err, extra, nExtra, slot, seq);
    return static_cast<int>(hipGetLastError());
}

int launchMarkBits(const uint32_t* F, uint64_t n, uint64_t* bits, hipStream_t s) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_mark_bits, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, s, F, n, bits);
    return static_cast<int>(hipGetLastError());
}

int launchRepackBits(const RepackArgs& a, hipStream_t s) {
    if (a.outWords == 0) return 0;
    if (a.world < 1 || a.world > kMaxWorld) return static_cast<int>(hipErrorInvalidValue);
    hipLaunchKernelGGL(k_repack_bits, dim3(static_cast<unsigned>((a.outWords + 255) / 256)), dim3(256), 0, s, a);
    return static_cast<int>(hipGetLastError());
}

int launchExpandRoots(const uint32_t* F, uint64_t nF, const HopSlots& hs, const uint64_t* rootsCur, uint64_t* rootsNext,
                      uint8_t* visited, uint8_t epoch, hipStream_t s) {
    const uint64_t nEnt = nF * static_cast<uint64_t>(hs.n);
    if (nEnt == 0) return 0;
    dim3 grid(static_cast<unsigned>(std::min<uint64_t>((nEnt + NW - 1) / NW, kDynGrid)));
    hipLaunchKernelGGL(k_expand_roots, grid, dim3(WG), 0, s, F, nEnt, hs, rootsCur,
                       reinterpret_cast<unsigned long long*>(rootsNext), visited, epoch);
    return static_cast<int>(hipGetLastError());
}

int launchScatterRoots(const uint32_t* F, uint64_t n, const uint64_t* bits, uint64_t* roots, hipStream_t s) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_scatter_roots, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, s, F, n, bits,
                       reinterpret_cast<unsigned long long*>(roots));
    return static_cast<int>(hipGetLastError());
}

int launchGatherRoots(const uint32_t* F, uint64_t n, const uint64_t* roots, uint64_t* out, hipStream_t s) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_gather_roots, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, s, F, n, roots, out);
    return static_cast<int>(hipGetLastError());
}

int launchMergeRoots(const uint64_t* own, const uint64_t* recv, uint64_t stride, uint64_t n, int world, int rank,
                     uint64_t* out, hipStream_t s) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_merge_roots, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, s, own, recv, stride, n,
                       world, rank, out);
    return static_cast<int>(hipGetLastError());
}

int launchVertexCells(const VertexCellArgs& a, hipStream_t s) {
    if (a.n == 0) return 0;
    hipLaunchKernelGGL(k_vertex_cells, dim3(static_cast<unsigned>((a.n + 255) / 256)), dim3(256), 0, s, a);
    return static_cast<int>(hipGetLastError());
}

// list pack: 1024 threads x 4 rows per workgroup (row = tile + k * 1024 + thread: coalesced mark loads),
// blockIdx.y = peer
__global__ __launch_bounds__(1024) void k_pack_list(ListXchgArgs a) {
    __shared__ uint64_t sm[1024 / 64 + 1];
    __shared__ uint64_t sBase;
    const int q = blockIdx.y;
    if (q == a.rank && !a.includeSelf) return;
    const uint64_t n = a.sb[q + 1] - a.sb[q];
    const uint64_t tile = static_cast<uint64_t>(blockIdx.x) * 4096;
    if (tile >= n) return;
    const uint8_t* mk = a.visited + a.sb[q];
    uint32_t flags = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint64_t r = tile + k * 1024 + threadIdx.x;
        const uint8_t m = mk[r < n ? r : n - 1];
        flags |= (r < n && m == a.epoch ? 1u : 0u) << k;
    }
    const uint64_t mine = static_cast<uint64_t>(__popc(flags));
    // block exclusive scan of the per-thread counts
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint64_t x = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) sm[wid] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t acc = 0;
        for (int w = 0; w < 16; w++) { const uint64_t t = sm[w]; sm[w] = acc; acc += t; }
        sBase = acc ? static_cast<uint64_t>(atomicAdd(a.counts + q, static_cast<unsigned long long>(acc))) : 0;
    }
    __syncthreads();
    uint64_t at = sBase + sm[wid] + x - mine;
    uint32_t* out = a.list + static_cast<uint64_t>(q) * a.cap;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        if (!((flags >> k) & 1u)) continue;
        if (at < a.cap) out[at] = static_cast<uint32_t>(tile + k * 1024 + threadIdx.x);
        at++;
    }
}

__global__ void k_merge_list(const uint32_t* rows, uint64_t n, uint8_t* own, uint8_t epoch) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n) own[rows[i]] = epoch;
}

__global__ void k_scatter_index(const uint32_t* rows, uint64_t n, uint32_t* map) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n) map[rows[i]] = static_cast<uint32_t>(i);
}

int launchScatterIndex(const uint32_t* rows, uint64_t n, uint32_t* map, hipStream_t s) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_scatter_index, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, s, rows, n, map);
    return static_cast<int>(hipGetLastError());
}

int launchPackLists(const ListXchgArgs& a, hipStream_t s) {
    uint64_t maxRows = 0;
    for (int q = 0; q < a.world; q++)
        if (q != a.rank || a.includeSelf) maxRows = std::max(maxRows, a.sb[q + 1] - a.sb[q]);
    if (maxRows == 0 || a.world < 2 || a.world > kMaxWorld) return 0;
    hipLaunchKernelGGL(k_pack_list, dim3(static_cast<unsigned>((maxRows + 4095) / 4096), a.world), dim3(1024), 0, s, a);
    return static_cast<int>(hipGetLastError());
}

int launchMergeList(const uint32_t* rows, uint64_t n, uint8_t* own, uint8_t epoch, hipStream_t s) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_merge_list, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, s, rows, n, own, epoch);
    return static_cast<int>(hipGetLastError());
}

int launchPackPeers(const ExchangeArgs& a, hipStream_t s) {
    uint64_t maxRows = 0;
    for (int q = 0; q < a.world; q++)
        if (q != a.rank) maxRows = std::max(maxRows, a.sb[q + 1] - a.sb[q]);
    if (maxRows == 0 || a.world < 2 || a.world > kMaxWorld) return 0;
    hipLaunchKernelGGL(k_pack, dim3(static_cast<unsigned>((maxRows + 255) / 256), a.world), dim3(256), 0, s, a);
    return static_cast<int>(hipGetLastError());
}

int launchMergePeers(const ExchangeArgs& a, hipStream_t s) {
    const uint64_t n = a.sb[a.rank + 1] - a.sb[a.rank];
    if (n == 0 || a.world < 2 || a.world > kMaxWorld) return 0;
    hipLaunchKernelGGL(k_merge, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, s, a);
    return static_cast<int>(hipGetLastError());
}

}  // namespace ngx
