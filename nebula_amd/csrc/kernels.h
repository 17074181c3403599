// Host-visible launchers and argument blocks of kernels.hip.
#pragma once

#include <hip/hip_runtime.h>

#include "kargs.h"

namespace ngx {

// host-mapped publication slot of a scan total: slot[0] = value, slot[2] = an extra word (the final
// hop's error bits), slot[1] = pubTag(seq, value, extra). The three are relaxed system-scope stores: a
// release would make the kernel write back every dirty L2 line first (buffer_wbl2, measured on the
// critical path of the seed / compaction / close kernels), and the host needs no device data ordered
// before the value, only the value itself, which it accepts when slot[1] matches the tag of what it
// read (a slot caught between stores mismatches and is polled again).
struct Publish {
    uint64_t* slot;
    uint64_t seq;
};
__host__ __device__ inline uint64_t pubMix(uint64_t x) {
    x ^= x >> 31;
    x *= 0x7fb5d329728ea185ULL;
    x ^= x >> 27;
    x *= 0x81dadef4bc2dd44dULL;
    return x ^ (x >> 33);
}
__host__ __device__ inline uint64_t pubTag(uint64_t seq, uint64_t value, uint64_t extra, uint64_t extra2) {
    return pubMix(seq ^ pubMix(value + 0x9e3779b97f4a7c15ULL) ^ pubMix(extra ^ 0x2545f4914f6cdd1dULL) * 3 ^
                  pubMix(extra2 + 0x632be59bd9b4e019ULL) * 5);
}
// slot[3]: a second extra word (the final hop's packed (|F|, E) when its grid came from the device)
__device__ inline void publishWords(uint64_t* slot, uint64_t seq, uint64_t value, uint64_t extra, uint64_t extra2 = 0) {
    __hip_atomic_store(slot, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(slot + 2, extra, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(slot + 3, extra2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(slot + 1, pubTag(seq, value, extra, extra2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// (part, vid) -> shard vertex row: open-addressing table (linear probing, power-of-two capacity
// >= 2V, built at commit) so a seed lookup is ~1 probe instead of a binary search over V rows
struct VIndexSlot {
    int64_t vid;
    int32_t part;
    uint32_t row;                       // kNoRow: empty
};
struct VIndex {
    const VIndexSlot* slots;
    uint64_t mask;                      // capacity - 1
};
__host__ __device__ inline uint64_t vindexHash(int32_t part, int64_t vid) {
    uint64_t h = static_cast<uint64_t>(vid) * 0x9E3779B97F4A7C15ULL ^ static_cast<uint64_t>(static_cast<uint32_t>(part)) * 0xC2B2AE3D27D4EB4FULL;
    h ^= h >> 29;
    h *= 0xBF58476D1CE4E5B9ULL;
    return h ^ (h >> 32);
}

// seed hop (n seeds, n * hs.n <= kSeedFuseMax entries): launchSeedFrontierCf below
constexpr uint64_t kSeedFuseMax = 4096;

int launchIndexLookup(const int32_t* qpart, const int64_t* qvid, uint64_t n, VIndex idx, uint32_t* out, hipStream_t s);
int launchLookup(const int32_t* qpart, const int64_t* qvid, uint64_t n, const int32_t* vpart, const int64_t* vid,
                 uint64_t V, uint32_t* out, hipStream_t s);
// estart must hold nEnt + 1 entries; estart[nEnt] receives E
int launchDegreeScan(const uint32_t* F, uint64_t nEnt, const HopSlots& hs, uint64_t* estart, uint64_t* tileSums,
                     hipStream_t s, Publish pub = Publish{nullptr, 0});
// chunkFirst must hold ceil(E / kChunk) entries (estart[nEnt] = E)
int launchChunkFirst(const uint64_t* estart, uint64_t nEnt, uint64_t* chunkFirst, hipStream_t s, uint64_t* zero = nullptr,
                     uint64_t nzero = 0);
// mask (nullptr: every edge): only hop edges e with mask[e] != 0 are expanded
// dyn != nullptr (device-driven hop): E / nEnt are upper bounds, the real ones are read from *dyn; the
// kernel does nothing when the real E >= pullMinE (the pull kernels take that hop)
constexpr uint64_t kDynGrid = 2048;                // workgroups of a device-driven (grid-stride) launch
int launchExpandMark(const uint32_t* F, const uint64_t* estart, const uint64_t* chunkFirst, uint64_t nEnt, uint64_t E,
                     const HopSlots& hs, uint8_t* visited, uint8_t epoch, bool pos32, hipStream_t s,
                     const uint8_t* mask = nullptr, const uint64_t* dyn = nullptr, uint64_t pullMinE = ~0ULL,
                     const uint64_t* ebase = nullptr);   // ebase: FinalArgs::ebase
// storage outcome per hop edge (a.E entries of out: 1 = emitted) for the max-edges / TTL mask path;
// a's F / estart / chunkFirst / hs / env / P / propsMask / ttl fields are read
int launchStoragePass(const FinalArgs& a, uint8_t* out, hipStream_t s);
// keep the first `cap` set flags of every frontier entry's hop edges, clear the others
int launchCap(const uint64_t* estart, uint64_t nEnt, uint8_t* mask, int64_t cap, hipStream_t s);
int launchCompact(const uint8_t* visited, uint64_t gbase, uint64_t V, uint8_t epoch, uint32_t* outF,
                  uint64_t* tileSums, uint64_t* count, hipStream_t s);
// fused compaction + next-hop degree scan (kernels.hip FlagDegIn): outF gets the next frontier,
// estart its entries' edge offsets (|F| * hs.n + 1 entries, the last = E), *packedTotal = |F| << kFdShift | E.
// Requires V < 2^(64 - kFdShift) and the slots' total edges < 2^kFdShift.
constexpr int kFdShift = kDynShift;
constexpr uint64_t kFdMask = kDynMask;
int launchCompactDegrees(const uint8_t* visited, uint64_t gbase, uint64_t V, uint8_t epoch, const HopSlots& hs,
                         uint32_t* outF, uint64_t* estart, uint64_t* tileSums, uint64_t* packedTotal, hipStream_t s,
                         Publish pub = Publish{nullptr, 0});
// Compaction of an intermediate hop (kernels.hip k_compact_count + k_compact_write): visited[row] ==
// epoch -> next frontier outF (row order), its entries' estart (|F| * hs.n + 1 entries, the last = E)
// and the next hop's chunk heads chunkFirst (what k_chunk_first computes). Two launches over tiles of
// kCompactTile rows: the first writes each tile's and each wave's packed (count << kFdShift | degree)
// total, the second sums the totals before its tile (no inter-workgroup waiting: the r02 single-pass
// look-back spent most of its 20-38 us on tickets and polling) and writes the rows. Wave w of a tile
// owns rows w * 1024 + k * 64 + lane (k < 16): every mark / offset load of a wave is one coalesced
// access. bits != nullptr: also the frontier bitmap (one 64-bit word per 64 rows, every word of the
// shard written) for the next hop's pull.
struct CompactArgs {
    const uint8_t* visited;             // this shard's rows (visited + gbase)
    uint64_t V;
    HopSlots hs;
    uint32_t* outF;
    uint64_t* estart;
    uint64_t* ebase;                    // optional: the entries' CSR positions (FinalArgs::ebase)
    uint64_t* chunkFirst;
    uint64_t cfCap;                     // entries of chunkFirst (overflow sets err[3])
    uint64_t* tileSum;                  // one word per tile (written by the count launch)
    uint64_t* waveSum;                  // NW words per tile
    uint64_t* total;                    // device copy of the packed total
    Publish pub;
    uint64_t* zero;                     // words the next final kernel needs cleared (zero[k * kDoneOff], k < nzero)
    uint32_t nzero;
    uint32_t* clear32;                  // optional word cleared by the count launch (the pull's segment counter)
    uint32_t* err;
    uint8_t epoch;
    uint64_t* bits;                     // optional frontier bitmap of this shard's rows (V / 64 words, rounded up)
    int32_t laneRows;                   // rows per lane, 4 / 8 / 16; 0: the launcher picks by V (kernels.hip)
    int32_t wgThreads;                  // 1024 (0) or 256 threads per workgroup (256: 16 rows per lane, the same
                                        // 4096-row tile; a workgroup that fits beside another query's final hop)
    int32_t bitsZero;                   // write every word of `bits` as 0 (no hop reads this frontier's bitmap:
                                        // the next hop is the final one), leaving it clean for a sparse hop
    int32_t countOnly;                  // dense final hop next (FinalArgs::denseMark): the count launch, then
                                        // one workgroup summing its tile totals into *total; no rows written
    int32_t totalByClose;               // countOnly, the total read on the device only: no summing launch, the
                                        // final hop's close sums the tile words (FinalArgs::dynTiles)
};
// Sparse intermediate hop (world 1, push, E far below the shard's rows): the expansion builds the next
// frontier itself instead of a compaction sweeping every row (kernels.hip k_expand_sparse). Per edge one
// 64-bit atomicOr on the frontier bitmap (all zero before the launch) dedups the destination and sets the
// pull's bitmap; the rows whose bit an edge set are the next frontier. Each workgroup reserves its new
// rows' places and edge offsets with one packed atomicAdd, so every entry gets estart / ebase / chunk
// heads without a scan; the last workgroup writes the tail estart[|F| ns] = E, the packed total and its
// publication, and clears the counters. Frontier order = reservation order (a set: GoExecutor keeps the
// dsts of a hop in an unordered set too, GoExecutor.cpp:675-718).
struct SparseArgs {
    const uint32_t* F;
    const uint64_t* estart;
    const uint64_t* chunkFirst;
    const uint64_t* ebase;              // optional (FinalArgs::ebase)
    uint64_t nEnt;
    uint64_t E;
    const uint64_t* dynIn;              // or null: packed (|F| << kDynShift | E) of this hop on the device (the
                                        // launch is then a fixed grid striding over the hop's slices)
    HopSlots hs;
    uint64_t* bits;                     // the shard's frontier bitmap, zero before the launch
    uint64_t bitWords;                  // its words
    uint32_t* outF;
    uint64_t* outEst;                   // next hop: estart, |F| * ns + 1 entries
    uint64_t* outEbase;                 // next hop: the entries' CSR positions, or null
    uint64_t* outCf;                    // next hop: chunk heads
    uint64_t cfCap;
    uint64_t* ctl;                      // [0] packed (rows << kFdShift | edges) reserved, [1] finished workgroups
    uint64_t* total;                    // device copy of the packed total
    Publish pub;
    uint32_t* err;
};
int launchExpandSparse(const SparseArgs& a, bool pos32, hipStream_t s);
constexpr uint64_t kCompactLbMaxV = 1ULL << (62 - kFdShift);
constexpr uint64_t kCompactTile = 4096;     // the smallest compaction tile (1024 threads x 4 rows; 8 or 16 per lane on larger shards): sizes the per-tile words
// GO final kernel words: kargs.h (kResv*, kDoneOff). The seed / compaction kernels clear zero[k * kDoneOff]
// for k < nzero.
int launchCompactLb(const CompactArgs& a, hipStream_t s);
// tile words the count launch of launchCompactLb(a) writes (a.tileSum[0 .. n))
uint64_t compactLbTiles(const CompactArgs& a);
// seed hop variant that also writes chunkFirst (cfCap entries) and clears zero[0 .. nzero)
int launchSeedFrontierCf(const int32_t* qpart, const int64_t* qvid, uint64_t n, VIndex idx, const HopSlots& hs,
                         uint32_t* F, uint64_t* estart, Publish pub, uint64_t* chunkFirst, uint64_t cfCap,
                         uint64_t* zero, uint32_t nzero, uint32_t* err, hipStream_t s, uint64_t* packedOut = nullptr,
                         uint64_t* zero8 = nullptr,      // zero8: 8 words cleared first (the query's counters)
                         uint64_t* ebase = nullptr);     // ebase: the entries' CSR positions (FinalArgs::ebase)
// QueryResponse rows of GetNeighbors (storage.thrift IdAndProp.props): per returned edge, the RowWriter
// row of its type's response edge schema (QueryBoundProcessor.cpp:38-43 with collectProps,
// QueryBaseProcessor.inl:325-399). Two launches: write == false stores each row's length in rowLen,
// write == true writes the bytes at rowOff (the exclusive scan of rowLen).
constexpr int32_t kRcSrc = -1, kRcRank = -2, kRcType = -3;    // key props of a response column
constexpr int kMaxRespCols = 128;                             // response columns per edge type
struct RowEncArgs {
    uint64_t n;
    const int32_t* oType;               // signed type per row
    const int64_t* oSrc;
    const int64_t* oRank;
    const uint8_t* oFlags;              // EF_* per row (EF_EMPTY_VALUE: no RowReader), nullptr: none
    const OutCol* cols;                 // the request's return columns (device array)
    int32_t nslots;
    int32_t etype[kMaxSlots];
    int32_t cbeg[kMaxSlots + 1];        // response columns of slot s: [cbeg[s], cbeg[s + 1])
    const int32_t* rcSrc;               // request column index, or kRcSrc / kRcRank / kRcType
    const int32_t* rcType;              // response field type (NGX_T_*)
    uint64_t* rowLen;
    const uint64_t* rowOff;
    uint8_t* out;
};
int launchEncodeRows(const RowEncArgs& a, bool write, hipStream_t s);
// out[0 .. n) = exclusive prefix of in, out[n] = total (3-phase scan, tileSums as launchDegreeScan)
int launchScanU64(const uint64_t* in, uint64_t n, uint64_t* out, uint64_t* tileSums, hipStream_t s);
// v[0 .. n) -> exclusive prefix in place, v[n] = total (one 1024-thread workgroup: n up to ~1e6)
int launchScanInPlace(uint64_t* v, uint64_t n, hipStream_t s);

// ngx_go_result_digest: per row h = mix64(... mix64(mix64(kDigestSeed ^ key) ^ col0) ...) over the row's
// src vid and each listed column's value bits (integers sign-extended from their width w, or the constant
// c when w == 0); out[0] += h (mod 2^64), out[1] ^= h, out[2] += rows. Order-independent, so two result
// multisets compare without a sort (oracle/orc_digest.cpp restates it on the host).
constexpr int kDigestMaxCols = 16;
constexpr uint64_t kDigestSeed = 0x9E3779B97F4A7C15ULL;
struct DigestArgs {
    uint64_t n;
    int32_t ncols;                      // columns after the key
    const void* x[kDigestMaxCols + 1];  // [0] the src vids, then the columns
    int32_t w[kDigestMaxCols + 1];      // bytes per element, 0: constant
    int64_t c[kDigestMaxCols + 1];
    uint64_t* out;                      // 3 words, zeroed by the launcher
};
int launchRowDigest(const DigestArgs& a, hipStream_t s);

// k_final_close_cols: the arrays a close moves (kind 0: plain, w bytes; 1: 8-byte string values
// rebased with their arena slots; 2: 8-byte word w of each row's string-arena block)
struct CloseCol {
    void* p;
    int32_t w;
    int32_t kind;
};
constexpr int kCloseMaxCols = 32;
// the FinalArgs fields k_final_close_cols reads (same names and meaning)
struct CloseArgs {
    uint64_t* resvCtl;
    uint64_t* resvTab;
    uint64_t* resvNext;
    uint32_t* err;
    uint64_t* rowsPub;
    uint64_t rowsSeq;
    char* strOut;
    uint64_t oBase;
    const uint64_t* dynTotal;           // the final hop's packed (|F|, E) on the device, published beside R
    const uint64_t* dynTiles;           // when set: *dynTotal = the sum of these words, written by the close
    uint64_t nDynTiles;
    uint32_t resvTB, resvSeq, resvG, resvShift, resvStride, nStrOut;
};
struct CloseCols {
    CloseCol c[kCloseMaxCols];
    int32_t n;
};

// final hop, one pass (interpreter kernel). a.oEntry set (GetNeighbors): a.lbStatus zeroed, ceil(E /
// kChunk) + 1 words; outputs sized for a.oBase + a.E rows; rows in edge order, rows written = the
// inclusive status of the last chunk. Else (GO): the kResv words of a.lbStatus zeroed, outputs sized for
// a.oBase + a.E + resvSlack() rows, chunks' rows in per-group blocks; launchFinalClose must follow.
int launchFinal(const FinalArgs& a, hipStream_t s, unsigned grid = 0);   // grid 0: one workgroup per chunk of a.E
// GO final hop, after the final kernel (generated or interpreter) on the same stream: the rows past the
// row count moved into the holes of the groups' last blocks, then rows = lbStatus[0] and the row count
// and the query's error bits (bit k = a.err[k] != 0) published to a.rowsPub when set
int launchFinalClose(const FinalArgs& a, hipStream_t s);
// resident workgroups per CU of the interpreter final kernel launchFinal would run for `a`
int finalOccupancy(const FinalArgs& a);

// Direction-optimizing ("pull", Beamer et al. SC'12) intermediate hop, one shard holding every row:
// row r joins the next frontier iff one of its in-neighbours over a hop slot's MIRROR slot (-t for t,
// verified at commit to be the exact transpose of t) is in the current frontier (cur[g] == curEp).
// Same set as the push expansion (getDstIdsFromResp, GoExecutor.cpp:675-718), fewer random accesses
// when the frontier's edges outnumber the shard's rows.
//
// Row pass over a per-slot "head" image built at commit (sliced ELLPACK, SELL-64-sigma): rows are
// taken in slices of 64 (one wave each); inside windows of kPullWindow rows the rows are ordered by
// min(in-degree, kPullK) descending (perm), and the first kPullK in-neighbours of every row are stored
// column-major per slice (head[slice][k][lane]), largest source out-degree first, so one probe round
// of a wave is ONE coalesced 256-byte load and most reached rows hit on their first probe (a frontier
// reached by expansion is hub-heavy). The old row-per-thread pass loaded 8 in-neighbours of its own
// in-list per lane: ~54 distinct cache lines per wave load, address-unit bound (r02: 60 us at C2).
// Rows still open after their kPullK head entries (in-degree > kPullK) reserve segment words; the
// segment pass probes their whole in-list in the mirror CSR (kPullSeg in-edges per workgroup, so a
// supernode spreads over many workgroups). Reached rows get out[r] = ep. ctl[0..3) is zero between
// launches (the segment pass's last workgroup leaves it so).
constexpr int kPullMaxSlots = 4;
constexpr int kPullK = 16;                  // head entries per row (a multiple of 4)
constexpr uint64_t kPullWindow = 2048;      // rows sorted by head length inside windows of this size
constexpr uint32_t kPullLong = 0x80000000u; // perm word flag: in-degree > kPullK (row = word & ~flag)
constexpr uint64_t kPullSeg = 1024;
struct PullArgs {
    int32_t n;
    const uint64_t* ioff[kPullMaxSlots];   // mirror slot CSR offsets (V + 1)
    const uint32_t* isrc[kPullMaxSlots];   // mirror slot dgid: global row of each in-neighbour
    const uint32_t* perm[kPullMaxSlots];   // [slice * 64 + lane]: row | kPullLong, kNoRow past the rows
    const uint32_t* head[kPullMaxSlots];   // [(slice * kPullK + k) * 64 + lane]: k-th in-neighbour or kNoRow
    const uint8_t* nk[kPullMaxSlots];      // per slice: max over its rows of min(in-degree, kPullK)
    uint64_t sliceEnd[kPullMaxSlots];      // inclusive prefix of the slots' slice counts
    const uint64_t* curBits;               // frontier bitmap over global rows (bit g of word g / 64)
    uint8_t* out;                          // this shard's marks (marks + gbase)
    uint64_t V;
    uint64_t* seg;
    uint64_t segCap;
    uint32_t* ctl;                         // [0] segments reserved (zero between hops: CompactArgs::clear32)
    uint32_t* err;                         // [3] queue overflow / spin limit (device fault)
    uint8_t curEp, ep;
    const uint64_t* dyn;                   // device-driven hop: packed totals; the row pass does nothing when
    uint64_t minE;                         // the hop's E < minE (the push expansion takes it)
};
// worst-case queue words: (rows with in-degree > kPullK) * n + in-edges / kPullSeg + 1
int launchPull(const PullArgs& a, hipStream_t s);
// marks[F[i]] = ep for the rows of a frontier list (kNoRow entries skipped)
int launchMarkRows(const uint32_t* F, uint64_t n, uint8_t* marks, uint8_t ep, hipStream_t s);
// end of a query: err[0..4) as bits and extra[0 .. nExtra) to host-mapped slot[1 ..], then slot[0] = seq
int launchPublishTail(const uint32_t* err, const uint64_t* extra, int nExtra, uint64_t* slot, uint64_t seq, hipStream_t s);
// bits of a frontier list's rows set in a bitmap (zeroed by the caller)
int launchMarkBits(const uint32_t* F, uint64_t n, uint64_t* bits, hipStream_t s);
// world > 1 pull: the all-gathered shard bitmaps (segWords words each, local row order) -> one bitmap
// over global rows (shard q's rows start at sb[q])
constexpr int kMaxWorld = 64;
struct RepackArgs {
    const uint64_t* seg;
    uint64_t segWords;
    uint64_t sb[kMaxWorld + 1];
    int world;
    uint64_t* out;
    uint64_t outWords;
};
int launchRepackBits(const RepackArgs& a, hipStream_t s);
// multi-root walk (pipes): every destination of a frontier row ORs in the row's root set (64-bit
// masks over rows) and is marked `epoch`; roots[F[i]] |= bits[i]; out[i] = roots[F[i]]
int launchExpandRoots(const uint32_t* F, uint64_t nF, const HopSlots& hs, const uint64_t* rootsCur, uint64_t* rootsNext,
                      uint8_t* visited, uint8_t epoch, hipStream_t s);
int launchScatterRoots(const uint32_t* F, uint64_t n, const uint64_t* bits, uint64_t* roots, hipStream_t s);
int launchGatherRoots(const uint32_t* F, uint64_t n, const uint64_t* roots, uint64_t* out, hipStream_t s);
// world > 1 multi-root walk: out[i] = own[i] | recv[q * stride + i] over the peers q != rank (the root
// sets the peers' expansions gave this shard's rows), i < n
int launchMergeRoots(const uint64_t* own, const uint64_t* recv, uint64_t stride, uint64_t n, int world, int rank,
                     uint64_t* out, hipStream_t s);
// YIELD DISTINCT on the device (GoExecutor::processFinalResult, GoExecutor.cpp:1298-1305): one row of
// every group of rows with equal YIELD values is kept. Values are equal when their value types are
// equal and their bits are, doubles by value (0.0 == -0.0, NaN == NaN: what the reference's
// boost::hash_range key makes equal), strings by bytes. An open-addressing table (capacity a power of
// two >= 2n, zeroed) holds (hash high 32 bits << 32 | row + 1); a row either claims an empty slot
// (keep[r] = 1) or meets an equal row's slot (keep[r] = 0). Which of equal rows is kept is not fixed
// (GO rows have no fixed order; only the values are returned).
constexpr int kMaxDistinctCols = 64;
struct DistinctArgs {
    uint64_t n;
    int32_t nY;
    const OutCol* cols;                 // nY result columns (device array)
    uint8_t vt[kMaxDistinctCols];       // V_* of column y's rows when cols[y].t is null
    uint64_t* table;
    uint64_t mask;
    uint64_t* keep;                     // n entries
};
int launchDistinctMark(const DistinctArgs& a, hipStream_t s);
// rows r with keep[r] move to pre[r] (exclusive scan of keep) in every array: k arrays of esz-byte
// elements, src -> dst
constexpr int kMaxScatter = 48;
struct ScatterArgs {
    uint64_t n;
    const uint64_t* keep;
    const uint64_t* pre;
    int32_t k;
    const uint8_t* src[kMaxScatter];
    uint8_t* dst[kMaxScatter];
    uint8_t esz[kMaxScatter];
};
int launchScatterKept(const ScatterArgs& a, hipStream_t s);
// Batched device -> host copy by a kernel: every array is streamed with 16-byte loads and stores into
// page-locked host memory mapped into the device address space (dst = hipHostGetDevicePointer), so
// the copy runs at the PCIe write rate on all CUs instead of on one DMA engine.
constexpr int kMaxCopies = 32;
struct CopyBatch {
    int32_t n;
    const uint8_t* src[kMaxCopies];
    uint8_t* dst[kMaxCopies];
    uint64_t bytes[kMaxCopies];
    uint64_t start[kMaxCopies + 1];     // exclusive prefix of 16-byte units per array
};
int launchCopyBatch(const CopyBatch& b, hipStream_t s);
int launchVertexCells(const VertexCellArgs& a, hipStream_t s);
// frontier exchange, one launch each side: pack every peer q's marked rows into bits + q * words;
// merge ORs the world - 1 received bitmaps (bits + q * words, over this shard's rows) into the marks
struct ExchangeArgs {
    uint8_t* visited;
    uint8_t epoch;
    uint64_t sb[kMaxWorld + 1];                      // shard q's rows are [sb[q], sb[q + 1])
    int world, rank;
    uint64_t words;                                  // bitmap stride per peer
    uint64_t* bits;
};
int launchPackPeers(const ExchangeArgs& a, hipStream_t s);
int launchMergePeers(const ExchangeArgs& a, hipStream_t s);
// The list form of the same exchange, for hops whose frontier is far smaller than the peers' rows
// (counts, then the vids): per peer q != rank the marked rows of q's range as u32 offsets
// from sb[q], appended to list[q * cap ..] (one atomic per workgroup and peer; counts[q] zeroed by the
// host first), then each owner marks the rows it received (k_merge_list).
struct ListXchgArgs {
    const uint8_t* visited;
    uint8_t epoch;
    uint64_t sb[kMaxWorld + 1];
    int world, rank;
    uint32_t* list;
    uint64_t cap;                                    // entries per peer in `list`
    unsigned long long* counts;                      // world words
    int includeSelf;                                 // also list this rank's own rows (the $$ owner fetch)
};
int launchPackLists(const ListXchgArgs& a, hipStream_t s);
// map[rows[i]] = i for i < n (the $$ owner fetch: global row -> index of its fetched tag values)
int launchScatterIndex(const uint32_t* rows, uint64_t n, uint32_t* map, hipStream_t s);
// own[rows[i]] = epoch for i < n
int launchMergeList(const uint32_t* rows, uint64_t n, uint8_t* own, uint8_t epoch, hipStream_t s);


}  // namespace ngx
