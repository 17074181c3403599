// libnebula_gn engine: context, schema registry, snapshot upload, the GO multi-hop driver and the
// GetNeighbors processor, behind the C ABI of include/nebula_gn.h.
//
// The hop loop restates GoExecutor (src/graph/GoExecutor.cpp:92-131 execute, :520-606 stepOut /
// onStepOutResponse, :840-914 getStepOutProps, :1082-1335 processFinalResult) on device:
// non-record hops only expand and dedup (storage returns `_dst` only and graphd keeps the set of
// dsts), record hops run the storage filter (pushed only on the last forward hop, :528-533), the
// graphd WHERE and the YIELD columns. With world > 1 every shard expands its own parts and the
// per-hop frontier is exchanged as bitmaps over RCCL (ncclSend/ncclRecv all-to-all).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <random>
#include <cstdio>
#include <cstdlib>
#include <ctime>
#include <functional>
#include <set>
#include <unordered_map>
#include <thread>
#include <unordered_set>

#include <sys/mman.h>
#include <ucontext.h>

#include "exprc.h"
#include "jit.h"
#include "kernels.h"
#include "rowcodec.h"

using namespace ngx;

#define HIP_OK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { throw Error{NGX_E_DEVICE, std::string("HIP: ") + hipGetErrorString(e_) + " at " #x}; } } while (0)
#define NCCL_OK(x) do { ncclResult_t r_ = (x); if (r_ != ncclSuccess) { throw Error{NGX_E_DEVICE, std::string("RCCL: ") + ncclGetErrorString(r_)}; } } while (0)

namespace ngx {

struct DeviceGraph {
    uint64_t V = 0, vglobal = 0, gbase = 0;
    std::vector<uint64_t> shardBase;
    int32_t* vpart = nullptr;
    int64_t* vid = nullptr;
    int32_t vidW = 8;                                   // narrowest signed width holding every vid of vid[]
    VIndex vindex{nullptr, 0};                          // (part, vid) -> row hash index (seed lookup)
    std::vector<DSlot> slots;
    // per slot: the row holding CSR position c * kChunk, for every chunk c of the slot (+ a last row): the
    // chunk map of a final hop over the whole slot (FinalArgs::denseMark)
    std::vector<const uint64_t*> chunkRow;
    std::vector<int32_t> mirror;                        // per slot: the slot holding its exact transpose, or -1
    // per slot with a mirror: the pull hop's head image of the in-lists (kernels.h PullArgs)
    struct PullHead { const uint32_t* perm = nullptr; const uint32_t* head = nullptr; const uint8_t* nk = nullptr;
                      uint64_t slices = 0, longRows = 0; };
    std::vector<PullHead> pullHead;
    // $$ props across shards: every tag table over ALL global rows (replicas of the other shards'
    // rows), gathered on the first query that reads a $$ prop, kept until the next commit
    bool replicas = false;
    std::vector<HostColumn> repHost;                    // host copies (string bytes back result cells)
    DTag* rtags = nullptr;
    DCol* rcols = nullptr;
    std::vector<DTag> tags;
    std::vector<DCol> cols;
    DSlot* dslots = nullptr;
    DTag* dtags = nullptr;
    DCol* dcols = nullptr;
    std::vector<void*> allocs;
    uint64_t bytes = 0;
    struct Range { uint64_t dev; const char* host; uint64_t len; };
    std::vector<Range> strRanges;                       // device string bytes -> host copy
    ~DeviceGraph() { for (void* p : allocs) (void)hipFree(p); }

    template <typename T>
    T* upload(const T* src, uint64_t n) {
        if (n == 0) return nullptr;
        void* p = nullptr;
        HIP_OK(hipMalloc(&p, n * sizeof(T)));
        HIP_OK(hipMemcpy(p, src, n * sizeof(T), hipMemcpyHostToDevice));
        allocs.push_back(p);
        bytes += n * sizeof(T);
        return static_cast<T*>(p);
    }
};

}  // namespace ngx

namespace {

// Debugging aid (flag "poison_buffers", process-wide; NGX_POISON=1 sets it at load, for a whole test
// suite): every device scratch buffer allocated from then on starts as kPoisonByte bytes, so a kernel
// that reads a word no kernel of the query wrote sees garbage instead of whatever an earlier query left
// there (tests/test_gpu_poison.py). The fill is ordered before any use: the engine's stream is
// non-blocking, so a fill on the null stream left running could land after the first copy or kernel
// that writes the buffer; hence the device synchronisation.
std::atomic<bool> gPoison{std::getenv("NGX_POISON") != nullptr && std::getenv("NGX_POISON")[0] == '1'};
constexpr int kPoisonByte = 0xA5;

// Frees deferred while a pipelined batch runs on this thread: hipFree / hipHostFree wait for the whole
// device to go idle, so a scratch buffer that grows in the middle of a batch (a lane meeting a larger
// frontier than its earlier queries) would drain the pipeline (r05 trace: the host stalled 560 us on one
// growth, both final hops behind it running alone). The batch frees them once at its end.
thread_local bool tDeferFree = false;
thread_local std::vector<std::pair<void*, bool>> tGraveyard;   // (pointer, page-locked host memory)
void freeDevice(void* p) {
    if (!p) return;
    if (tDeferFree) tGraveyard.emplace_back(p, false);
    else (void)hipFree(p);
}
void freeHost(void* p) {
    if (!p) return;
    if (tDeferFree) tGraveyard.emplace_back(p, true);
    else (void)hipHostFree(p);
}
void drainGraveyard() {
    for (auto& g : tGraveyard) (void)(g.second ? hipHostFree(g.first) : hipFree(g.first));
    tGraveyard.clear();
}

// growable device buffer
std::atomic<uint64_t> gDBufGen{0};
std::atomic<uint64_t> gDBufBytes{0};                    // bytes allocated by DBuf growth (flag dbuf_alloc_bytes)
const bool gDBufTrace = std::getenv("NGX_DBUF_TRACE") != nullptr;
struct DBuf {
    void* p = nullptr;
    size_t cap = 0;
    uint64_t gen = 0;                                   // unique per allocation (hipMalloc may hand back a freed address)
    template <typename T>
    T* get(size_t n) {
        size_t bytes = std::max<size_t>(n * sizeof(T), 64);
        if (bytes > cap) {
            const size_t cap0 = cap;
            freeDevice(p);
            p = nullptr;
            size_t c = std::max(bytes, cap * 3 / 2);
            HIP_OK(hipMalloc(&p, c));
            cap = c;
            gen = gDBufGen.fetch_add(1, std::memory_order_relaxed) + 1;
            gDBufBytes.fetch_add(c, std::memory_order_relaxed);
            if (gDBufTrace) std::fprintf(stderr, "[ngx dbuf] alloc %zu bytes (asked %zu, had %zu)\n", c, bytes, cap0);
            if (gPoison.load(std::memory_order_relaxed)) {
                HIP_OK(hipMemset(p, kPoisonByte, c));
                HIP_OK(hipDeviceSynchronize());
            }
        }
        return static_cast<T*>(p);
    }
    void release() { if (p) (void)hipFree(p); p = nullptr; cap = 0; gen = 0; }
};

struct Timer {
    hipEvent_t a = nullptr, b = nullptr;
};

// the $$ owner fetch of one lane (fetchDstProps): request lists, exchange blocks, the global row ->
// fetched-row map, and per record hop of the running query the fetched tag tables (device) with the host
// copy of their string bytes (result cells read strings back through it)
struct DstLane {
    DBuf req, counts, recv, blobS, blobR, rows, map;
    uint64_t mapRows = 0;
    std::vector<DBuf> data;                             // per record hop: present / values / strings
    std::vector<std::string> hostStr;                   // per record hop: its string bytes (host copy)
    std::vector<const char*> devStr;                    // ... and where they live on the device
    uint64_t bytes() const {
        uint64_t b = req.cap + counts.cap + recv.cap + blobS.cap + blobR.cap + rows.cap + map.cap;
        for (const DBuf& d : data) b += d.cap;
        return b;
    }
    void release() {
        for (DBuf* b : {&req, &counts, &recv, &blobS, &blobR, &rows, &map}) b->release();
        for (DBuf& d : data) d.release();
        data.clear();
        hostStr.clear();
        devStr.clear();
        mapRows = 0;
    }
};

// ROCTX range on the host timeline of rocprofv3 (--marker-trace): a query, each hop, each kernel class
// launch (the reference's FLAGS_trace_go step log, GoExecutor.cpp:559-569). Without a
// tool attached a push / pop is a check of a registration flag.
struct RoctxRange {
    explicit RoctxRange(const char* name) { roctxRangePushA(name); }
    ~RoctxRange() { roctxRangePop(); }
    RoctxRange(const RoctxRange&) = delete;
    RoctxRange& operator=(const RoctxRange&) = delete;
};

}  // namespace

struct ngx_ctx {
    int32_t device = 0, rank = 0, world = 1;
    hipStream_t stream = nullptr;
    ncclComm_t comm = nullptr;
    ngx_exchange_fn xchg = nullptr;                    // host collective instead of RCCL (tests)
    uint64_t* pin = nullptr;                           // host-mapped [value, seq]: scan totals published by
    uint64_t* pinDev = nullptr;                        // k_scan_tiles (kernels.h Publish)
    uint64_t pinSeq = 0;                               // words [0, 2): scan totals; [kTailOff ..): query tail
    static constexpr size_t kPinBytes = 16384;          // up to eight lanes of 256 words (ngx_ctx::Lane)
    static constexpr size_t kTailOff = 8;               // k_publish_tail: seq, error bits, extra words
    static constexpr uint32_t kSeedSlot = 80;           // the seed hop's publication (nextPub)
    static constexpr uint32_t kRowsSlot = 88;           // a record hop's row count (k_final_close)
    // ngx_go_batch: the next query's host preparation and first hops enqueued while this one's final hop
    // runs (flag "batch_pipeline"; read-only "batch_overlaps" counts the queries that overlapped)
    bool batchPipeline = true;
    struct GoPipe* pipe = nullptr;
    uint64_t pipeOverlaps = 0;
    void* xchgUser = nullptr;
    std::map<int32_t, std::unique_ptr<Space>> spaces;
    std::string lastError;
    std::mutex mu;
    // scratch
    DBuf visited, F0, F1, estart, ebase, chunkFirst, tileSums, counters, lbStatus, seedPart, seedVid;
    DBuf cmpStatus[2];                                  // compaction tile / wave totals (kernels.h CompactArgs)
    DBuf frontierBits;                                  // the pull's frontier bitmap over global rows
    DBuf oSrc, oDst, oRank, oType, oEntry, progBuf, sendBits, recvBits, vcells, misc, oColDesc, edgeMask;
    DBuf resvTab, resvCtl;                              // GO final hop: block tables, counters (kargs.h resv*)
    uint64_t resvTabWords = 0;
    uint32_t resvSeq = 0, resvLastG = 0, resvLastStride = 0, resvParity = 0;
    const uint64_t* resvRows = nullptr;                 // this query's last GO final launch's row count (device word)
    uint64_t strArenaMax = uint64_t(8) << 30;           // bytes of one record hop's result string arena (flag str_arena_max)
    bool resvClosePending = false;                      // counters handed out, their k_final_close not enqueued
    DstLane dst;                                        // the $$ owner fetch's buffers (per lane)
    DBuf oFlags, rowCols, rowLen, rowOff, rowBytes;     // GetNeighbors response rows (encode_rows)
    DBuf dkTable, dkKeep, dkPre, dSrc, dDst, dRank, dType;   // YIELD DISTINCT (table, marks, compacted rows)
    std::vector<DBuf> strArena;                         // result string arenas, one per record hop (FinalArgs::strOut)
    DBuf roots[2], rootBits;                            // multi-root walk: root sets over rows, per-entry bits
    DBuf rootSend, rootRecv;                            // world > 1: root sets of peer rows, both ways
    DBuf pwF, pwIn, pwEst, pwCf;                        // ... reading $-: (row, input row) entries, their estart / heads
    DBuf inX, inLen, inT, inStr, inDesc;                // ... the pipe's input table
    uint64_t pipeWalks = 0;                             // walks run for FROM $- / $var sentences (flag pipe_walks)
    DBuf localBits, pullGather;                         // world > 1 pull: this shard's frontier bitmap, all shards' 
    struct { int64_t qps = 0, errorQps = 0, latencySum = 0, latencyCount = 0, latencyMax = 0; } gbStats;
    std::vector<ngx_stat> statList;                     // ngx_stats view
    int64_t maxEdgesPerVertex = INT32_MAX;             // storaged FLAGS_max_edge_returned_per_vertex (GO hops)
    struct ColBuf { DBuf x, len, t; };
    struct PinBuf {                                     // page-locked host staging for result D2H
        void* p = nullptr;
        size_t cap = 0;
        char* get(size_t bytes) {
            if (bytes > cap) {
                freeHost(p);
                p = nullptr;
                // 25 % headroom: result sizes vary from query to query, and re-pinning a GB-sized
                // staging block costs more than the copy itself
                size_t c = std::max(bytes + bytes / 4, cap * 3 / 2);
                // coherent (fine-grained): kernels read the seeds / inputs the host just wrote, and the copy
                // kernel stores results the host reads after the stream synchronises; neither may meet a
                // stale line the GPU kept cached from an earlier query (hipHostMallocDefault is non-coherent)
                HIP_OK(hipHostMalloc(&p, c, hipHostMallocMapped | hipHostMallocCoherent));
                cap = c;
            }
            return static_cast<char*>(p);
        }
        // grow keeping the first `keep` bytes (the caller has synchronised with copies out of the old block)
        char* getKeep(size_t bytes, size_t keep) {
            if (bytes <= cap) return static_cast<char*>(p);
            std::vector<char> save(static_cast<char*>(p), static_cast<char*>(p) + std::min(keep, cap));
            char* n = get(bytes);
            std::memcpy(n, save.data(), save.size());
            return n;
        }
        void release() { if (p) (void)hipHostFree(p); p = nullptr; cap = 0; }
    } hostStage, inStage, seedStage;
    std::string progLast;                               // the bytes of the last program upload ...
    const char* progLastPtr = nullptr;                  // ... and where they went (uploadPrograms skips a repeat)
    std::string progImg;                                // this call's program bytes (compared before staging)
    std::vector<ColBuf> oCols;                          // result columns (columnar, HBM)
    std::vector<ColBuf> dCols;                          // DISTINCT: the other half of each column's double buffer
    std::vector<OutCol> oColView;                       // their device pointers, as uploaded to oColDesc
    uint64_t visitedSize = 0;
    uint8_t epoch = 0;
    // pull expansion (kernels.h launchPull): segment queue + its counters, kept zero between launches
    DBuf pullSeg, pullCtl;
    uint64_t pullSegWords = 0;
    int32_t compactLaneRows = 0;                        // compaction rows per lane: 0 = by shard size, else 4 / 8 / 16
    int32_t compactWg = 0;                              // compaction workgroup threads: 0 = auto, 256 or 1024
    // generated GO final hops store result rows / load columns non-temporally (flags final_nt_stores /
    // final_nt_loads). r06, both on: the batch 0.2796 vs 0.2833 ms/step on one box (8 rounds), 0.2898 vs
    // 0.2901 on another (6); the final hop alone ~1% slower; either alone slower than neither. Kept off.
    bool finalNtStores = false;
    bool finalNtLoads = false;
    uint32_t resvGroups = kResvGroups;                  // GO final hop row-reservation groups (flag resv_groups, 1 .. kResvMaxGroups)
    int64_t pullFactor = 200;                           // pull when 100 x hop edges >= pullFactor x shard rows (0: never)
    uint64_t pullHops = 0;
    // sparse intermediate hops (kernels.h SparseArgs): a push hop with E * sparseFactor <= V builds the next
    // frontier in the expansion itself (flag "sparse_factor", 0 = never, < 0 = every push hop; read-only
    // "sparse_hops")
    int64_t sparseFactor = 16;
    uint64_t sparseHops = 0;
    bool pullPredict = false;                           // hop 2 of the last query pulled (world 1): launch it early
    DBuf sparseCtl;                                     // the sparse kernel's counters, kept zero between launches
    DBuf estart2, ebase2, chunkFirst2;                  // the next hop's entry arrays while the sparse kernel reads this hop's
    // world > 1 push hops: frontier exchanged as vid lists instead of bitmaps (flag "xchg_lists": -1 by the
    // hop's size, 0 bitmaps, 1 lists; read-only "xchg_list_hops")
    int64_t xchgLists = -1;
    uint64_t xchgListHops = 0;
    DBuf xListSend, xListRecv, xCounts;
    // the frontier bitmap is known to be all zero (a sparse hop's dedup set starts from it): set by a
    // compaction that wrote zeros, cleared by every other writer. Keyed on the allocation (pointer and
    // DBuf::gen) and the words zeroed: a query in a space with more rows needs more zero words
    bool bitsClean = false;
    const void* bitsCleanPtr = nullptr;
    uint64_t bitsCleanGen = 0, bitsCleanWords = 0;
    // device-driven hops (no host round trip per hop). Off by default: on MI355X the upper-bound grids
    // and the idle launch of the expansion not taken cost what the round trips saved (C2 step: device
    // 680 vs 656 us, profiles/r02_dyn_*); kept as an option ("dyn_hops", NGX_DYN_HOPS=1)
    bool dynHops = false;
    bool deviceLibm = false;                            // inexact libm of row values on the device (exprc.cpp)
    bool reservoirSampling = false;                     // storaged FLAGS_enable_reservoir_sampling: refused
    bool narrowColumns = true;                          // integer columns at their narrowest width (at commit)
    bool traceGo = false;                               // graphd FLAGS_trace_go: per-step log on stderr
    DBuf dynStats;                                      // per hop: packed (|F|, E) written by seed / compaction
    int cus = 256;                                      // compute units of the device
    // RCCL watchdog: collective work must finish within this; else the communicator is aborted
    int64_t rcclTimeoutMs = 120000;
    bool broken = false;                                // communicator aborted: every later call fails
    uint64_t lastXchgBytes = 0;                         // bytes this shard sent in the last exchange
    // per-query kernels (hipRTC)
    bool jitOn = true;
    JitCache jit;
    std::string jitNote;
    // profiling
    bool prof = false;
    struct Stat { std::string name; uint32_t launches = 0; double ms = 0; uint64_t bytes = 0; };
    std::vector<Stat> stats;
    std::vector<ngx_kernel_stat> statView;
    std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> pending;
    std::vector<hipEvent_t> eventPool;
    size_t eventNext = 0;

    // A query lane: the per-query scratch of the hop loop and its publication slots (words [pinLane,
    // pinLane + kLaneWords) of the host-mapped block). ngx_go_batch runs consecutive queries on rotating
    // lanes, so that one query's hops run on the device beside the earlier queries' final hops (GoPipe).
    // The active lane's fields are the members above; lane k's are parked in parked[k] while it is not
    // active (parked[activeLane] holds an empty set); useLane swaps sets.
    uint32_t pinLane = 0;
    static constexpr uint32_t kLaneWords = 256;
    static constexpr int kMaxLanes = 8;                 // kPinBytes / (8 * kLaneWords)
    struct Lane {
        DBuf visited, F0, F1, estart, ebase, chunkFirst, estart2, ebase2, chunkFirst2, tileSums, counters, lbStatus,
            seedPart, seedVid, cmpStatus[2], frontierBits, localBits, edgeMask, pullSeg, pullCtl, sparseCtl, dynStats, progBuf;
        uint64_t visitedSize = 0, pullSegWords = 0;
        uint8_t epoch = 0;
        bool bitsClean = false;
        const void* bitsCleanPtr = nullptr;
        uint64_t bitsCleanGen = 0, bitsCleanWords = 0;
        std::string progLast;
        const char* progLastPtr = nullptr;
        PinBuf inStage, seedStage;
        uint32_t pinLane = 0;
        // the lane's result rows and their reservation state (a query's final hop writes its lane's arrays,
        // so its k_final_close may run beside the next query's final hop)
        DBuf oSrc, oDst, oRank, oType, oColDesc, resvTab, resvCtl;
        std::vector<ColBuf> oCols;
        std::vector<OutCol> oColView;
        uint64_t resvTabWords = 0;
        uint32_t resvLastG = 0, resvLastStride = 0, resvParity = 0;
        bool resvClosePending = false;
        DstLane dst;
    } parked[kMaxLanes];
    int activeLane = 0;
    // lanes of a pipelined batch (flag "batch_lanes", 2 .. kMaxLanes): up to lanes - 1 queries wait at their
    // deferral point while the next one runs its hops
    int32_t batchLanes = 4;                            // r06, two final streams: 4 lanes 0.299 vs 3 lanes 0.303 ms per step
    // ngx_go_batch's streams (GoPipe, created with the context at world 1): the queries' hops on the front
    // stream, the last final hop of each overlapped query on the final stream; finalStream is set while a
    // pipelined batch runs. The coroutine stacks of the batch's queries (one per lane).
    // [0] front (hops), [1] final (final hops), [2] the second front stream (flag batch_fronts 2: consecutive
    // queries' hops on alternate front streams, so two queries' hop chains run at once beside a final hop)
    // or the close stream (k_final_close of an overlapped final hop beside the next query's final hop: the
    // close reads and moves its own lane's rows only)
    hipStream_t pipeStreams[4] = {nullptr, nullptr, nullptr, nullptr};   // + [3] the close stream
    hipEvent_t pipeEv[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    // a ring of events for the batch's cross-stream waits: each wait gets an event no later record re-arms
    // while the wait may be pending (flag batch_event_ring; 0: the fixed pipeEv per role)
    static constexpr int kPipeRing = 64;
    hipEvent_t pipeRing[kPipeRing] = {};
    uint32_t pipeRingNext = 0;
    bool batchEventRing = true;
    hipEvent_t pipeEvent(int role) {
        if (!batchEventRing || !pipeRing[0]) return pipeEv[role];
        return pipeRing[pipeRingNext++ % kPipeRing];
    }
    // set while a pipelined batch runs with flag batch_close_stream (default on since the second front
    // stream: C2 0.310 vs 0.317 ms per step; with one front stream it measured 0.330 vs 0.324, the next final
    // hop waiting for its front-stream dependency anyway)
    hipStream_t closeStream = nullptr;
    bool batchCloseStream = true;
    int32_t batchFronts = 2;                           // front streams of a pipelined batch (1 or 2)
    // flag batch_cu_split N > 0: the batch's front streams on N CUs (every CU i with (i / 8) % (256 / N / 8)
    // == 0, spread over the XCDs), its final stream on the others, so the hops' waves do not take slots
    // from the final hop (streams created on first use with that split)
    int32_t batchCuSplit = 0, cuSplitMade = 0;
    hipStream_t splitStreams[4] = {nullptr, nullptr, nullptr, nullptr};
    int32_t pipeFronts = 1;                            // ... of the batch that runs
    hipStream_t finalStream = nullptr;
    // flag batch_finals 2: consecutive queries' final hops on two final streams (the close after its final
    // hop on the same stream, no close stream), so one final hop starts while the other drains its tail;
    // finalCur is the running query's
    int32_t batchFinals = 2;
    // per lane: the event after its last overlapped final hop's close. The lane's next final hop waits for it:
    // that close still moves the earlier query's rows inside the lane's result arrays and reads its block
    // table after the earlier query has read its row count (published by the close's first workgroup), and
    // with two final streams nothing else orders the two (r06: a C2 batch at 4 groups failed on it)
    hipEvent_t laneCloseEv[kMaxLanes] = {};
    bool laneClosePending[kMaxLanes] = {};                           // C2: 0.302 vs 0.309 ms per step (tools/ab_batch.py, 10 rounds)
    hipStream_t finalStream2 = nullptr, finalCur = nullptr;
    void* coStack[kMaxLanes] = {};
    static constexpr size_t kCoStackBytes = size_t(16) << 20;   // + a guard page below each
    void swapLane(Lane& L) {
#define NGX_LANE_SWAP(f) std::swap(f, L.f);
        NGX_LANE_SWAP(visited) NGX_LANE_SWAP(F0) NGX_LANE_SWAP(F1) NGX_LANE_SWAP(estart)
        NGX_LANE_SWAP(ebase) NGX_LANE_SWAP(chunkFirst) NGX_LANE_SWAP(estart2) NGX_LANE_SWAP(ebase2) NGX_LANE_SWAP(chunkFirst2)
        NGX_LANE_SWAP(tileSums) NGX_LANE_SWAP(counters) NGX_LANE_SWAP(lbStatus) NGX_LANE_SWAP(seedPart) NGX_LANE_SWAP(seedVid)
        NGX_LANE_SWAP(cmpStatus[0]) NGX_LANE_SWAP(cmpStatus[1]) NGX_LANE_SWAP(frontierBits) NGX_LANE_SWAP(localBits)
        NGX_LANE_SWAP(edgeMask) NGX_LANE_SWAP(pullSeg) NGX_LANE_SWAP(pullCtl) NGX_LANE_SWAP(sparseCtl) NGX_LANE_SWAP(dynStats)
        NGX_LANE_SWAP(progBuf) NGX_LANE_SWAP(visitedSize) NGX_LANE_SWAP(pullSegWords) NGX_LANE_SWAP(epoch)
        NGX_LANE_SWAP(bitsClean) NGX_LANE_SWAP(bitsCleanPtr) NGX_LANE_SWAP(bitsCleanGen) NGX_LANE_SWAP(bitsCleanWords) NGX_LANE_SWAP(progLast) NGX_LANE_SWAP(progLastPtr)
        NGX_LANE_SWAP(inStage) NGX_LANE_SWAP(seedStage) NGX_LANE_SWAP(pinLane)
        NGX_LANE_SWAP(oSrc) NGX_LANE_SWAP(oDst) NGX_LANE_SWAP(oRank) NGX_LANE_SWAP(oType) NGX_LANE_SWAP(oColDesc)
        NGX_LANE_SWAP(resvTab) NGX_LANE_SWAP(resvCtl) NGX_LANE_SWAP(oCols) NGX_LANE_SWAP(oColView)
        NGX_LANE_SWAP(resvTabWords) NGX_LANE_SWAP(resvLastG) NGX_LANE_SWAP(resvLastStride) NGX_LANE_SWAP(resvParity)
        NGX_LANE_SWAP(resvClosePending) NGX_LANE_SWAP(dst)
#undef NGX_LANE_SWAP
    }
    void initLanes() {
        for (int k = 1; k < kMaxLanes; k++) parked[k].pinLane = k * kLaneWords;
    }
    void useLane(int k) {
        if (k == activeLane) return;
        swapLane(parked[activeLane]);                  // park the active lane (the empty set comes in) ...
        swapLane(parked[k]);                           // ... and bring lane k in (the empty set goes to its slot)
        activeLane = k;
    }

    void releaseLane() {
        for (DBuf* b : {&visited, &F0, &F1, &estart, &ebase, &chunkFirst, &estart2, &ebase2, &chunkFirst2, &tileSums, &counters,
                        &lbStatus, &seedPart, &seedVid, &cmpStatus[0], &cmpStatus[1], &frontierBits, &localBits, &edgeMask,
                        &pullSeg, &pullCtl, &sparseCtl, &dynStats, &progBuf, &oSrc, &oDst, &oRank, &oType, &oColDesc,
                        &resvTab, &resvCtl}) b->release();
        for (auto& cb : oCols) { cb.x.release(); cb.len.release(); cb.t.release(); }
        inStage.release();
        seedStage.release();
        dst.release();
    }
    // the parked lanes' scratch and result rows freed (flag batch_release_lanes, or release_lanes = 1 once):
    // a pipelined batch leaves lanes 1 .. kMaxLanes - 1 holding buffers as large as lane 0's. Called with no
    // batch running; hipFree waits for the work that still reads them.
    uint64_t releaseParked() {
        uint64_t freed = 0;
        const int was = activeLane;
        for (int k = 0; k < kMaxLanes; k++) {
            if (k == was) continue;
            useLane(k);
            for (DBuf* b : {&visited, &F0, &F1, &estart, &ebase, &chunkFirst, &estart2, &ebase2, &chunkFirst2, &tileSums,
                            &counters, &lbStatus, &seedPart, &seedVid, &cmpStatus[0], &cmpStatus[1], &frontierBits,
                            &localBits, &edgeMask, &pullSeg, &pullCtl, &sparseCtl, &dynStats, &progBuf, &oSrc, &oDst, &oRank,
                            &oType, &oColDesc, &resvTab, &resvCtl})
                freed += b->cap;
            for (auto& cb : oCols) freed += cb.x.cap + cb.len.cap + cb.t.cap;
            freed += dst.bytes();
            releaseLane();
            oCols.clear();
            oColView.clear();
            visitedSize = pullSegWords = 0;
            epoch = 0;
            bitsClean = false;
            bitsCleanPtr = nullptr;
            bitsCleanGen = bitsCleanWords = 0;
            progLast.clear();
            progLastPtr = nullptr;
            resvTabWords = 0;
            resvLastG = resvLastStride = resvParity = 0;
            resvClosePending = false;
        }
        useLane(was);
        return freed;
    }
    uint64_t releasedBytes = 0;
    bool batchReleaseLanes = false;
    // $$ props at world > 1 (flag dst_props): -1 by size (replicas while every shard's tag data fits
    // dstReplicaMax bytes), 0 replicas of every tag table over the global rows (gathered once per snapshot),
    // 1 the owner fetch per record hop (GoExecutor::fetchVertexProps -> QueryVertexPropsProcessor)
    int32_t dstProps = -1;
    // the final hop over every CSR position of its slot, reading the frontier from the marks (no next-frontier
    // list, no entry arrays): after a pulled hop at world 1 with one OVER type (flag dense_final)
    bool denseFinal = true;
    bool denseCloseTotal = true;                        // its frontier total summed by the close (flag dense_close_total)
    bool denseWorldDev = true;                          // world > 1: its totals kept on the device (flag dense_world_dev)
    uint64_t denseFinals = 0;
    uint64_t dstReplicaMax = uint64_t(1) << 30;
    uint64_t dstFetches = 0, dstFetchRows = 0;
    ~ngx_ctx() {                                       // also the cleanup of ngx_open's error paths
        (void)hipSetDevice(device);
        if (stream) (void)hipStreamSynchronize(stream);
        for (auto st : pipeStreams) if (st) (void)hipStreamSynchronize(st);
        for (auto st : splitStreams) if (st) (void)hipStreamSynchronize(st);
        spaces.clear();
        for (DBuf* b : {&oEntry, &sendBits, &recvBits,
                        &vcells, &misc, &oFlags, &rowCols, &rowLen, &rowOff, &rowBytes, &dkTable, &dkKeep, &dkPre, &dSrc, &dDst,
                        &dRank, &dType, &xListSend, &xListRecv, &xCounts}) b->release();
        for (auto& cb : dCols) { cb.x.release(); cb.len.release(); cb.t.release(); }
        hostStage.release();
        for (auto e : eventPool) (void)hipEventDestroy(e);
        for (auto e : pipeEv) if (e) (void)hipEventDestroy(e);
        for (auto e : laneCloseEv) if (e) (void)hipEventDestroy(e);
        for (auto e : pipeRing) if (e) (void)hipEventDestroy(e);
        for (auto st : pipeStreams) if (st) (void)hipStreamDestroy(st);
        for (auto st : splitStreams) if (st) (void)hipStreamDestroy(st);
        for (void* st : coStack) if (st) munmap(st, kCoStackBytes + 4096);
        if (comm) (void)ncclCommDestroy(comm);
        if (pin) (void)hipHostFree(pin);
        releaseLane();
        for (auto& L : parked) {
            swapLane(L);
            releaseLane();
        }
        if (stream) (void)hipStreamDestroy(stream);
    }

    hipEvent_t ev() {
        if (eventNext == eventPool.size()) {
            hipEvent_t e;
            HIP_OK(hipEventCreate(&e));
            eventPool.push_back(e);
        }
        return eventPool[eventNext++];
    }
    int statIndex(const char* name) {
        for (size_t i = 0; i < stats.size(); i++) if (stats[i].name == name) return static_cast<int>(i);
        stats.push_back(Stat{name});
        return static_cast<int>(stats.size()) - 1;
    }
    // host timeline of a query (NGX_HOST_TRACE=1): launches and publication waits, printed per query
    bool htrace = false;
    // pipelined batch host timeline (NGX_PIPE_TRACE=1): the same marks, tagged with the running query and
    // kept with absolute CLOCK_MONOTONIC times until the batch ends (the pipeline stays on)
    bool ptrace = false;
    int32_t ptraceQuery = -1;
    std::vector<std::pair<std::string, int64_t>> pmarks;
    void pmark(const std::string& what) {
        timespec ts;
        clock_gettime(CLOCK_MONOTONIC, &ts);
        pmarks.emplace_back("q" + std::to_string(ptraceQuery) + " " + what,
                            static_cast<int64_t>(ts.tv_sec) * 1000000000LL + ts.tv_nsec);
    }
    std::vector<std::pair<std::string, std::chrono::steady_clock::time_point>> hmarks;
    void hmark(const std::string& what) {
        if (htrace) hmarks.emplace_back(what, std::chrono::steady_clock::now());
        if (ptrace) pmark(what);
    }
    void hflush() {
        if (!htrace || hmarks.empty()) return;
        std::string line = "[ngx host]";
        for (auto& m : hmarks)
            line += " " + m.first + "@" + std::to_string(std::chrono::duration<double, std::micro>(m.second - hmarks[0].second).count()).substr(0, 7);
        std::fprintf(stderr, "%s\n", line.c_str());
        hmarks.clear();
    }
    // bracket a launch group with events when profiling
    template <typename F>
    void timed(const char* name, uint64_t algoBytes, F&& f) {
        RoctxRange range(name);                        // a ROCTX range per kernel class launch (rocprofv3 --marker-trace)
        if (htrace || ptrace) hmark(std::string("L:") + name);
        if (!prof) { f(); if (htrace || ptrace) hmark(std::string("l:") + name); return; }
        int k = statIndex(name);
        hipEvent_t a = ev(), b = ev();
        HIP_OK(hipEventRecord(a, stream));
        f();
        HIP_OK(hipEventRecord(b, stream));
        pending.push_back({k, {a, b}});
        stats[k].launches++;
        stats[k].bytes += algoBytes;
    }
    void addBytes(const char* name, uint64_t b) {
        if (prof) stats[statIndex(name)].bytes += b;
    }
    void collectTimings() {
        if (!prof) return;
        for (auto& p : pending) {
            HIP_OK(hipEventSynchronize(p.second.second));
            float ms = 0;
            HIP_OK(hipEventElapsedTime(&ms, p.second.first, p.second.second));
            stats[p.first].ms += ms;
        }
        pending.clear();
        eventNext = 0;
    }
};

// ngx_go_batch's pipeline. The batch's queries run as coroutines (ucontext) on the calling thread, one
// at a time, each on a stack of its own, consecutive queries on alternate lanes (ngx_ctx::Lane: scratch
// and publication slots). A query's hops run on the front stream and its last final hop (with its close)
// on the final stream, each stream on its own share of the CUs. A query whose final hop is enqueued
// yields before it waits for its row count (it is "deferred"); the next query then runs its hops on its
// lane — on the device beside the deferred query's final hop — and enqueues its own final hop behind the
// deferred one's on the final stream (the result arrays and reservation counters are shared); then it
// defers in turn, the first query finishes (row count, result) and the one after starts. On the device
// one query's intermediate hops hide under the other's final hop; on the host the result tail,
// preparation and launch calls overlap the device work. Only one coroutine runs at any time, so the
// context needs no lock between them.
struct GoJob {
    ucontext_t uc;
    int32_t idx = 0;
    int state = 0;
    int32_t rc = NGX_OK;
    uint64_t nrows = 0, edges = 0, digest[3] = {0, 0, 0};
};
struct GoPipe {
    enum { kRunning = 0, kDeferred = 1, kPreFinal = 2, kDone = 3 };
    ucontext_t main;
    GoJob* cur = nullptr;
    int ndeferred = 0;                                 // queries waiting at goDeferPoint
    bool holdFinals = false;                           // digests: a final hop waits for the deferred query
    const ngx_go_plan* const* plans = nullptr;
    int32_t n = 0;
};

namespace {

int32_t fail(ngx_ctx* c, int32_t code, const std::string& msg) {
    c->lastError = msg;
    return code;
}

Space* findSpace(ngx_ctx* c, int32_t id) {
    auto it = c->spaces.find(id);
    return it == c->spaces.end() ? nullptr : it->second.get();
}

// ------------------------------------------------------------------------ upload
// Integer columns can be stored at the narrowest signed width that holds every value (HBM bytes per
// edge for a filter/YIELD column: 8 -> 1 for a 0..99 property); loads sign-extend (vm.h:loadI64).
template <class T>
const void* uploadAs(DeviceGraph& d, const std::vector<int64_t>& v, uint64_t n) {
    std::vector<T> t(n);
    for (uint64_t i = 0; i < n; i++) t[i] = static_cast<T>(v[i]);
    return d.upload(t.data(), n);
}
const void* uploadNarrow(DeviceGraph& d, const std::vector<int64_t>& v, uint64_t n, int32_t& width, bool narrow) {
    // Default on (flag "narrow_columns" 0 keeps 8 bytes): fewer HBM bytes per scanned edge. A strided-load
    // microbenchmark of the final hop's access pattern (tools/mb_final.hip) runs 607 -> 468 us with dst
    // int32, rank / filter column int8 (profiles/r02_mb_final.txt).
    if (!narrow) { width = 8; return d.upload(v.data(), n); }
    int64_t lo = 0, hi = 0;
    for (uint64_t i = 0; i < n; i++) { lo = std::min(lo, v[i]); hi = std::max(hi, v[i]); }
    if (lo >= INT8_MIN && hi <= INT8_MAX) { width = 1; return uploadAs<int8_t>(d, v, n); }
    if (lo >= INT16_MIN && hi <= INT16_MAX) { width = 2; return uploadAs<int16_t>(d, v, n); }
    if (lo >= INT32_MIN && hi <= INT32_MAX) { width = 4; return uploadAs<int32_t>(d, v, n); }
    width = 8;
    return d.upload(v.data(), n);
}

// narrowest signed width (1, 2, 4 or 8 bytes) that holds every value of v[0 .. n)
int32_t narrowWidth(const int64_t* v, uint64_t n) {
    int64_t lo = 0, hi = 0;
    for (uint64_t i = 0; i < n; i++) { lo = std::min(lo, v[i]); hi = std::max(hi, v[i]); }
    if (lo >= INT8_MIN && hi <= INT8_MAX) return 1;
    if (lo >= INT16_MIN && hi <= INT16_MAX) return 2;
    if (lo >= INT32_MIN && hi <= INT32_MAX) return 4;
    return 8;
}

void uploadColumns(DeviceGraph& d, std::vector<HostColumn>& hc, uint64_t n, bool narrow) {
    for (auto& c : hc) {
        DCol dc{};
        dc.type = c.type;
        switch (c.type) {
            case T_INT: case T_TIMESTAMP: case T_VID: dc.data = uploadNarrow(d, c.i64, n, dc.width, narrow); break;
            case T_FLOAT: case T_DOUBLE: dc.data = d.upload(c.f64.data(), n); break;
            case T_BOOL: dc.data = d.upload(c.b.data(), n); break;
            case T_STRING: {
                dc.soff = d.upload(c.soff.data(), n + 1);
                dc.sbytes = c.sbytes.empty() ? nullptr : d.upload(c.sbytes.data(), c.sbytes.size());
                if (dc.sbytes) d.strRanges.push_back({reinterpret_cast<uint64_t>(dc.sbytes), c.sbytes.data(), c.sbytes.size()});
                break;
            }
            default: break;
        }
        if (!c.allValid) dc.valid = d.upload(c.valid.data(), n);
        if (dc.width) c.width = dc.width;
        d.cols.push_back(dc);
    }
}

// TTL info of a schema (buildTTLInfoAndRespSchema, QueryBaseProcessor.inl:670-797): present when
// ttl_col is set and ttl_duration > 0 (rows are then read, bad rows skipped); the column is checked
// only when the latest schema types it INT / TIMESTAMP / VID (checkDataExpiredForTTL), else -1
bool ttlInfo(const SchemaSet* ss, int32_t& col, int64_t& dur) {
    col = -1;
    dur = 0;
    if (!ss) return false;
    const SchemaDef& l = ss->latest();
    if (l.ttlCol.empty() || l.ttlDur <= 0) return false;
    int32_t t = l.typeOf(l.ttlCol);
    if (t == T_INT || t == T_TIMESTAMP || t == T_VID) col = l.index(l.ttlCol);
    dur = l.ttlDur;
    return true;
}

std::unique_ptr<DeviceGraph> upload(HostGraph& g, const Space& sp) {
    auto d = std::make_unique<DeviceGraph>();
    d->V = g.vid.size();
    d->gbase = g.gbase;
    d->vglobal = g.vglobal ? g.vglobal : d->V;
    d->shardBase = g.shardBase;
    d->vpart = d->upload(g.vpart.data(), d->V);
    d->vid = d->upload(g.vid.data(), d->V);
    d->vidW = narrowWidth(g.vid.data(), d->V);
    {
        uint64_t cap = 1024;
        while (cap < 2 * d->V) cap <<= 1;
        std::vector<VIndexSlot> t(cap, VIndexSlot{0, 0, kNoRow});
        for (uint64_t r = 0; r < d->V; r++) {
            uint64_t h = vindexHash(g.vpart[r], g.vid[r]) & (cap - 1);
            while (t[h].row != kNoRow) h = (h + 1) & (cap - 1);
            t[h] = VIndexSlot{g.vid[r], g.vpart[r], static_cast<uint32_t>(r)};
        }
        d->vindex = VIndex{d->upload(t.data(), cap), cap - 1};
    }
    for (auto& s : g.slots) {
        DSlot ds{};
        ds.etype = s.etype;
        ds.colBase = static_cast<int32_t>(d->cols.size());
        ds.ncols = static_cast<int32_t>(s.cols.size());
        ds.off = d->upload(s.off.data(), s.off.size());
        ds.dst = uploadNarrow(*d, s.dst, s.dst.size(), ds.dstW, sp.narrow);
        ds.dgid = d->upload(s.dgid.data(), s.dgid.size());
        // one rank for every edge (RMAT: rank 0 everywhere): no column, the value travels in HopSlots
        const bool rankConst = sp.narrow && !s.rank.empty() &&
                               std::all_of(s.rank.begin(), s.rank.end(), [&](int64_t r) { return r == s.rank[0]; });
        ds.rankConst = rankConst ? s.rank[0] : 0;
        if (rankConst) {
            ds.rank = nullptr;
            ds.rankW = narrowWidth(&s.rank[0], 1);
        } else {
            ds.rank = uploadNarrow(*d, s.rank, s.rank.size(), ds.rankW, sp.narrow);
        }
        ds.hasFlags = s.anyFlags ? 1 : 0;
        ds.eflags = s.anyFlags ? d->upload(s.eflags.data(), s.eflags.size()) : nullptr;
        uploadColumns(*d, s.cols, s.dst.size(), sp.narrow);
        d->slots.push_back(ds);
        {
            const uint64_t E = s.off.empty() ? 0 : s.off.back();
            const uint64_t nCh = (E + kChunk - 1) / kChunk;
            std::vector<uint64_t> cr(nCh + 1, 0);
            uint64_t r = 0;
            for (uint64_t ch = 0; ch < nCh; ch++) {
                const uint64_t pos = ch * kChunk;
                while (r + 1 < s.off.size() && s.off[r + 1] <= pos) r++;
                cr[ch] = r;
            }
            cr[nCh] = s.off.size() >= 2 ? s.off.size() - 2 : 0;
            d->chunkRow.push_back(d->upload(cr.data(), cr.size()));
        }
    }
    for (auto& t : g.tags) {
        DTag dt{};
        dt.tag = t.tag;
        dt.colBase = static_cast<int32_t>(d->cols.size());
        dt.ncols = static_cast<int32_t>(t.cols.size());
        dt.present = d->upload(t.present.data(), t.present.size());
        if (!ttlInfo(sp.tag(t.tag), dt.ttlCol, dt.ttlDur)) dt.ttlCol = -1;
        uploadColumns(*d, t.cols, d->V, sp.narrow);
        d->tags.push_back(dt);
    }
    d->dslots = d->upload(d->slots.data(), d->slots.size());
    d->dtags = d->upload(d->tags.data(), d->tags.size());
    d->dcols = d->upload(d->cols.data(), d->cols.size());
    std::sort(d->strRanges.begin(), d->strRanges.end(), [](const DeviceGraph::Range& a, const DeviceGraph::Range& b) { return a.dev < b.dev; });
    return d;
}

// ------------------------------------------------------------------------ compiled programs on device
struct Programs {
    std::vector<Insn> code;
    std::string pool;
    int32_t P = -1, W = -1;
    std::vector<int32_t> yOff;
    bool usesDst = false;
    int32_t add(const Program& p) {
        int32_t off = static_cast<int32_t>(code.size());
        int64_t poolBase = static_cast<int64_t>(pool.size());
        pool += p.pool;
        for (auto in : p.code) {
            if (in.op == OP_PUSH && in.t1 == V_STR) in.imm += poolBase;
            code.push_back(in);
        }
        usesDst = usesDst || p.usesDstTag;
        return off;
    }
};

struct DevPrograms {
    const Insn* code = nullptr;
    const char* pool = nullptr;
    const int32_t* yOff = nullptr;
    const int32_t* ySlotType = nullptr;
    const int32_t* yColType = nullptr;
};

DevPrograms uploadPrograms(ngx_ctx* c, const Programs& pr, const std::vector<int32_t>& ySlotType,
                           const std::vector<int32_t>& yColType = {}) {
    size_t codeBytes = pr.code.size() * sizeof(Insn);
    size_t yBytes = pr.yOff.size() * 4;
    size_t tBytes = ySlotType.size() * 4;
    size_t cBytes = yColType.size() * 4;
    size_t poolOff = (codeBytes + yBytes + tBytes + cBytes + 63) & ~size_t(63);
    size_t total = poolOff + pr.pool.size() + 64;
    const size_t capBefore = c->progBuf.cap;
    char* base = c->progBuf.get<char>(total);
    if (c->progBuf.cap != capBefore) c->progLastPtr = nullptr;   // a new allocation (maybe at the old address)
    std::string& img = c->progImg;
    img.assign(total, '\0');
    std::memcpy(&img[0], pr.code.data(), codeBytes);
    std::memcpy(&img[codeBytes], pr.yOff.data(), yBytes);
    std::memcpy(&img[codeBytes + yBytes], ySlotType.data(), tBytes);
    std::memcpy(&img[codeBytes + yBytes + tBytes], yColType.data(), cBytes);
    std::memcpy(&img[poolOff], pr.pool.data(), pr.pool.size());
    // the same bytes as the last upload into the same buffer (a prepared query run again): nothing to copy
    // (a copy launch and its dispatch gap, ~7 us of the C2 step on the device timeline)
    if (base != c->progLastPtr || c->progLast != img) {
        // staged in page-locked memory: the copy is asynchronous (the lane's stage is reused only by its
        // next query, after this one has synchronised with its kernels)
        char* host = c->inStage.get(total);
        std::memcpy(host, img.data(), total);
        HIP_OK(hipMemcpyAsync(base, host, total, hipMemcpyHostToDevice, c->stream));
        c->progLast = img;
        c->progLastPtr = base;
    }
    DevPrograms d;
    d.code = reinterpret_cast<const Insn*>(base);
    d.yOff = reinterpret_cast<const int32_t*>(base + codeBytes);
    d.ySlotType = reinterpret_cast<const int32_t*>(base + codeBytes + yBytes);
    d.yColType = cBytes ? reinterpret_cast<const int32_t*>(base + codeBytes + yBytes + tBytes) : nullptr;
    d.pool = base + poolOff;
    return d;
}

// seeds (part, vid) to the device through the page-locked input stage, after the programs in it
// largest number of times one vid appears among the seeds (open addressing; a std::unordered_map
// took ~30 us for 1000 seeds, on the query's critical path)
uint64_t maxMultiplicity(const std::vector<int64_t>& v) {
    size_t cap = 16;
    while (cap < 2 * v.size()) cap <<= 1;
    std::vector<int64_t> key(cap);
    std::vector<uint32_t> cnt(cap, 0);
    uint64_t best = v.empty() ? 0 : 1;
    for (int64_t x : v) {
        uint64_t h = (static_cast<uint64_t>(x) * 0x9E3779B97F4A7C15ULL) >> 20;
        for (;; h++) {
            const size_t i = h & (cap - 1);
            if (cnt[i] == 0) { key[i] = x; cnt[i] = 1; break; }
            if (key[i] == x) { best = std::max<uint64_t>(best, ++cnt[i]); break; }
        }
    }
    return best;
}

// seeds (vids then parts) into one device block with one copy; dvid holds n * 12 bytes. The seeds
// have their own page-locked stage: the seed hop is launched before the programs are staged
// (runGo), so the two must not share a block that may move when it grows.
void stageSeeds(ngx_ctx* c, const std::vector<int32_t>& parts, const std::vector<int64_t>& vids, int32_t* dpart,
                int64_t* dvid) {
    const size_t n = vids.size();
    char* hp = c->seedStage.get(n * 12 + 64);             // the previous call has synchronised with its copies
    std::memcpy(hp, vids.data(), n * 8);
    std::memcpy(hp + n * 8, parts.data(), n * 4);
    if (reinterpret_cast<char*>(dpart) == reinterpret_cast<char*>(dvid) + n * 8) {
        HIP_OK(hipMemcpyAsync(dvid, hp, n * 12, hipMemcpyHostToDevice, c->stream));
    } else {
        HIP_OK(hipMemcpyAsync(dvid, hp, n * 8, hipMemcpyHostToDevice, c->stream));
        HIP_OK(hipMemcpyAsync(dpart, hp + n * 8, n * 4, hipMemcpyHostToDevice, c->stream));
    }
}

// seeds (vids then parts) into the page-locked seed stage, returned as device-visible pointers into it
// (mapped): the seed kernel reads them over the bus, no copy launch. False when the stage cannot be
// mapped (the caller copies instead).
bool stageSeedsMapped(ngx_ctx* c, const std::vector<int32_t>& parts, const std::vector<int64_t>& vids, const int32_t*& hpart,
                      const int64_t*& hvid) {
    const size_t n = vids.size();
    char* host = c->seedStage.get(n * 12 + 64);
    char* dev = nullptr;
    if (hipHostGetDevicePointer(reinterpret_cast<void**>(&dev), c->seedStage.p, 0) != hipSuccess || dev == nullptr) return false;
    std::memcpy(host, vids.data(), n * 8);
    std::memcpy(host + n * 8, parts.data(), n * 4);
    hvid = reinterpret_cast<const int64_t*>(dev);
    hpart = reinterpret_cast<const int32_t*>(dev + n * 8);
    return true;
}

// VM string pointer -> host bytes
std::string hostString(const DeviceGraph& d, const DevPrograms& dp, const std::string& pool, uint64_t ptr, uint32_t len) {
    if (len == 0) return std::string();
    uint64_t pb = reinterpret_cast<uint64_t>(dp.pool);
    if (ptr >= pb && ptr + len <= pb + pool.size()) return pool.substr(ptr - pb, len);
    auto it = std::upper_bound(d.strRanges.begin(), d.strRanges.end(), ptr,
                               [](uint64_t v, const DeviceGraph::Range& r) { return v < r.dev; });
    if (it == d.strRanges.begin()) return std::string();
    --it;
    if (ptr + len > it->dev + it->len) return std::string();
    return std::string(it->host + (ptr - it->dev), len);
}

// device string pointer -> host bytes: the query's literal pool (copied to `pool`) or a snapshot
// string column (DeviceGraph::strRanges)
struct StrMap {
    struct Range { uint64_t dev, len; const char* host; };
    const DeviceGraph* d;
    uint64_t poolDev;
    const std::string* pool;
    const std::vector<Range>* built = nullptr;                  // result string arenas (host copies)
    const char* host(uint64_t ptr, uint32_t len) const {
        if (len == 0) return "";
        if (ptr >= poolDev && ptr + len <= poolDev + pool->size()) return pool->data() + (ptr - poolDev);
        if (built) {
            for (const Range& r : *built)
                if (ptr >= r.dev && ptr + len <= r.dev + r.len) return r.host + (ptr - r.dev);
        }
        auto it = std::upper_bound(d->strRanges.begin(), d->strRanges.end(), ptr,
                                   [](uint64_t v, const DeviceGraph::Range& r) { return v < r.dev; });
        if (it == d->strRanges.begin()) return "";
        --it;
        if (ptr + len > it->dev + it->len) return "";
        return it->host + (ptr - it->dev);
    }
};

// one result column staged on the host: value bits, string lengths, per-row types (UNKNOWN columns)
struct ColView {
    int32_t colType = T_UNKNOWN;
    int64_t* x = nullptr;
    uint32_t* len = nullptr;
    uint8_t* t = nullptr;
    uint8_t typeAt(uint64_t r) const {
        if (t) return t[r];
        switch (colType) {
            case T_BOOL: return V_BOOL;
            case T_INT: case T_VID: case T_TIMESTAMP: return V_INT;
            case T_FLOAT: case T_DOUBLE: return V_DBL;
            case T_STRING: return V_STR;
            default: return V_ERR;
        }
    }
};

int hostThreads() { return hostThreadBudget(); }

// f(lo, hi, t) over T contiguous row ranges on T threads (T = 0: hostThreads(), small n: one)
template <typename F>
void parallelRows(uint64_t n, F&& f, int T = 0) {
    if (T <= 0) T = n < (1u << 16) ? 1 : hostThreads();
    if (T == 1) { f(0, n, 0); return; }
    std::vector<std::thread> ts;
    for (int t = 0; t < T; t++) ts.emplace_back([&f, n, t, T] { f(n * t / T, n * (t + 1) / T, t); });
    for (auto& th : ts) th.join();
}

// Mirror slots for the pull expansion (kernels.h launchPull): slot j is the mirror of slot i when
// etype[j] == -etype[i] and the multiset of (src row, dst row) pairs of i equals that of (dst row,
// src row) of j -- every out-edge was also written as its in-edge with the same rank, as
// InsertEdgeExecutor does, and nothing else. One shard holding every row (world == 1). Compared by
// edge count and two independent 64-bit sums of mixed pairs (a commutative digest of the multiset).
uint64_t mixPair(uint64_t a, uint64_t b, uint64_t seed) {
    uint64_t z = (a << 32 | b) + seed;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

struct PairDigest {
    uint64_t n = 0, h1 = 0, h2 = 0;
    bool ok = true;
    bool operator==(const PairDigest& o) const { return ok && o.ok && n == o.n && h1 == o.h1 && h2 == o.h2; }
};

// gbase: the shard's first global row (dgid values are global rows), so digests of every shard add up
PairDigest slotDigest(const HostSlot& s, bool transpose, uint64_t gbase = 0) {
    const uint64_t V = s.off.empty() ? 0 : s.off.size() - 1;
    const int T = V < (1u << 16) ? 1 : hostThreads();
    std::vector<PairDigest> part(T);
    parallelRows(V, [&](uint64_t lo, uint64_t hi, int t) {
        PairDigest d;
        for (uint64_t r = lo; r < hi; r++) {
            for (uint64_t e = s.off[r]; e < s.off[r + 1]; e++) {
                const uint64_t g = s.dgid[e];
                if (g == kNoRow) { d.ok = false; continue; }
                const uint64_t a = transpose ? g : gbase + r, b = transpose ? gbase + r : g;
                d.h1 += mixPair(a, b, 0x9E3779B97F4A7C15ULL);
                d.h2 += mixPair(b, a, 0xD1B54A32D192ED03ULL);
                d.n++;
            }
        }
        part[t] = d;
    }, T);
    PairDigest out;
    for (auto& d : part) { out.n += d.n; out.h1 += d.h1; out.h2 += d.h2; out.ok = out.ok && d.ok; }
    return out;
}

// The pull hop's head image of hop slot `s` whose mirror is `m` (kernels.h PullArgs): the in-list of
// row r over s is r's adjacency in m (dgid = the in-neighbour's row). Rows are ordered inside windows
// of kPullWindow rows by min(in-degree, kPullK) descending, so the lanes of a slice need similar
// numbers of rounds; each row's first kPullK in-neighbours are the ones with the largest out-degree
// over s (a frontier reached by expansion holds the hubs first, so most reached rows hit on their
// first probe). Which in-neighbours are probed first changes nothing but the probe count: the pull
// computes set membership.
// Rows without in-edges can never be reached by a pull: they are left out of the image (16 % of C2's
// rows, 15 % of its slices), so the windows run over the rows that have in-edges, in row order.
void buildPullHead(const HostGraph& g, int32_t s, int32_t m, DeviceGraph& d, const std::vector<uint32_t>* globalDeg = nullptr) {
    const HostSlot& out = g.slots[s];
    const HostSlot& in = g.slots[m];
    const uint64_t Vall = g.vid.size();
    std::vector<uint32_t> live;
    live.reserve(Vall);
    for (uint64_t r = 0; r < Vall; r++) if (in.off[r + 1] != in.off[r]) live.push_back(static_cast<uint32_t>(r));
    const uint64_t V = live.size();
    const uint64_t slices = (V + 63) / 64;
    std::vector<uint32_t> perm(slices * 64, kNoRow), head(slices * 64 * kPullK, kNoRow);
    std::vector<uint8_t> nk(slices, 0);
    const uint64_t windows = (V + kPullWindow - 1) / kPullWindow;
    std::vector<uint64_t> longRows(hostThreads() + 1, 0);
    // in-neighbours are global rows: world 1 reads the out-degree here, world > 1 the gathered one
    auto outDeg = [&](uint32_t u) -> uint64_t {
        if (globalDeg) return u < globalDeg->size() ? (*globalDeg)[u] : 0;
        return u < Vall ? out.off[u + 1] - out.off[u] : 0;
    };
    parallelRows(windows, [&](uint64_t lo, uint64_t hi, int t) {
        std::vector<std::pair<uint32_t, uint32_t>> rows;        // (head length, row)
        std::vector<uint64_t> nb;
        for (uint64_t w = lo; w < hi; w++) {
            const uint64_t r0 = w * kPullWindow, r1 = std::min<uint64_t>(V, r0 + kPullWindow);
            rows.clear();
            for (uint64_t i = r0; i < r1; i++) {
                const uint32_t r = live[i];
                const uint64_t deg = in.off[r + 1] - in.off[r];
                rows.emplace_back(static_cast<uint32_t>(std::min<uint64_t>(deg, kPullK)), r);
            }
            std::stable_sort(rows.begin(), rows.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
            for (uint64_t i = 0; i < rows.size(); i++) {
                const uint64_t at = r0 + i, slice = at / 64, lane = at % 64;
                const uint32_t r = rows[i].second;
                const uint64_t deg = in.off[r + 1] - in.off[r];
                // (out-degree, row) of every in-neighbour, read once each (the comparator of a sort over
                // rows would re-read the degrees at random on every comparison)
                nb.clear();
                for (uint64_t e = in.off[r]; e < in.off[r + 1]; e++) {
                    const uint32_t u = in.dgid[e];
                    if (u == kNoRow) continue;
                    nb.push_back(std::min<uint64_t>(outDeg(u), UINT32_MAX) << 32 | (~static_cast<uint64_t>(u) & 0xFFFFFFFFULL));
                }
                const size_t keep = std::min<size_t>(nb.size(), kPullK);
                // largest degree first, then the smaller row: the largest (degree, ~row) keys
                std::partial_sort(nb.begin(), nb.begin() + keep, nb.end(), std::greater<uint64_t>());
                for (size_t k = 0; k < keep; k++) head[(slice * kPullK + k) * 64 + lane] = static_cast<uint32_t>(~nb[k]);
                const bool isLong = deg > static_cast<uint64_t>(kPullK);
                perm[at] = r | (isLong ? kPullLong : 0u);
                longRows[t] += isLong;
                nk[slice] = std::max<uint8_t>(nk[slice], static_cast<uint8_t>(keep));
            }
        }
    }, windows < 64 ? 1 : hostThreads());
    DeviceGraph::PullHead ph;
    ph.perm = d.upload(perm.data(), perm.size());
    ph.head = d.upload(head.data(), head.size());
    ph.nk = d.upload(nk.data(), nk.size());
    ph.slices = slices;
    for (uint64_t x : longRows) ph.longRows += x;
    d.pullHead[s] = ph;
}

std::vector<int32_t> findMirrors(const HostGraph& g) {
    std::vector<int32_t> m(g.slots.size(), -1);
    if (g.vid.size() >= (1ULL << 31)) return m;
    for (size_t i = 0; i < g.slots.size(); i++) {
        if (m[i] >= 0 || g.slots[i].etype <= 0) continue;
        for (size_t j = 0; j < g.slots.size(); j++) {
            if (g.slots[j].etype != -g.slots[i].etype) continue;
            if (g.slots[i].dst.size() == g.slots[j].dst.size() && slotDigest(g.slots[i], false) == slotDigest(g.slots[j], true)) {
                m[i] = static_cast<int32_t>(j);
                m[j] = static_cast<int32_t>(i);
            }
        }
    }
    return m;
}

std::vector<uint8_t> gatherHost(ngx_ctx* c, const void* host, uint64_t bytes);
template <typename T>
std::vector<T> gatherRows(ngx_ctx* c, const HostGraph& g, const std::vector<T>& local);

// world > 1: type t's in-edge slots mirror its out-edge slots over the whole graph when every shard
// holds both slots and the digests of every shard's (src row, dst row) pairs, over global rows, add up
// to the same multiset both ways. One all-gather of a fixed record per edge type of the schema, so
// every shard takes the same decision (the pull's collectives run in lockstep).
std::vector<int32_t> findMirrorsGlobal(ngx_ctx* c, const Space& sp, const HostGraph& g) {
    std::vector<int32_t> m(g.slots.size(), -1);
    std::vector<int32_t> types;
    for (auto& e : sp.edges) types.push_back(e.first);
    if (types.empty()) return m;
    struct Rec { uint64_t have, ok, n1, a1, b1, n2, a2, b2; };
    std::vector<Rec> mine(types.size(), Rec{0, 0, 0, 0, 0, 0, 0, 0});
    std::vector<std::pair<int32_t, int32_t>> slotOf(types.size(), {-1, -1});
    for (size_t i = 0; i < types.size(); i++) {
        for (size_t k = 0; k < g.slots.size(); k++) {
            if (g.slots[k].etype == types[i]) slotOf[i].first = static_cast<int32_t>(k);
            if (g.slots[k].etype == -types[i]) slotOf[i].second = static_cast<int32_t>(k);
        }
        const auto [so, si] = slotOf[i];
        if (so < 0 || si < 0 || g.vglobal >= (1ULL << 31)) continue;
        const PairDigest o = slotDigest(g.slots[so], false, g.gbase), t = slotDigest(g.slots[si], true, g.gbase);
        mine[i] = Rec{1, o.ok && t.ok ? 1u : 0u, o.n, o.h1, o.h2, t.n, t.h1, t.h2};
    }
    const std::vector<uint8_t> all = gatherHost(c, mine.data(), mine.size() * sizeof(Rec));
    for (size_t i = 0; i < types.size(); i++) {
        Rec sum{1, 1, 0, 0, 0, 0, 0, 0};
        for (int w = 0; w < c->world; w++) {
            Rec r;
            std::memcpy(&r, all.data() + (static_cast<size_t>(w) * types.size() + i) * sizeof(Rec), sizeof(Rec));
            sum.have &= r.have; sum.ok &= r.ok;
            sum.n1 += r.n1; sum.a1 += r.a1; sum.b1 += r.b1; sum.n2 += r.n2; sum.a2 += r.a2; sum.b2 += r.b2;
        }
        if (sum.have && sum.ok && sum.n1 == sum.n2 && sum.a1 == sum.a2 && sum.b1 == sum.b2) {
            m[slotOf[i].first] = slotOf[i].second;
            m[slotOf[i].second] = slotOf[i].first;
        }
    }
    return m;
}

// mirror slots and, for every slot with one, its pull head image; world > 1 orders the head by the
// out-degrees of every shard's rows (gathered once per mirrored slot)
void attachMirrors(ngx_ctx* c, const Space& sp, const HostGraph& g, DeviceGraph& d) {
    d.mirror = c->world == 1 ? findMirrors(g) : findMirrorsGlobal(c, sp, g);
    d.pullHead.assign(g.slots.size(), DeviceGraph::PullHead());
    for (size_t s = 0; s < g.slots.size(); s++) {
        if (d.mirror[s] < 0) continue;
        if (c->world == 1) {
            buildPullHead(g, static_cast<int32_t>(s), d.mirror[s], d);
            continue;
        }
        const HostSlot& out = g.slots[s];
        std::vector<uint32_t> deg(g.vid.size());
        for (size_t r = 0; r < deg.size(); r++)
            deg[r] = static_cast<uint32_t>(std::min<uint64_t>(out.off[r + 1] - out.off[r], UINT32_MAX));
        const std::vector<uint32_t> globalDeg = gatherRows(c, g, deg);
        buildPullHead(g, static_cast<int32_t>(s), d.mirror[s], d, &globalDeg);
    }
}

// ColumnValue per calculateExprType (GoExecutor::toThriftResponse, GoExecutor.cpp:775-829); string
// bytes are appended to `strings` (str_off relative to it)
bool toCell(const OutCell& v, int32_t colType, ngx_cell& out, std::string& strings, const StrMap& sm) {
    out.str_len = 0;
    out.v.i = 0;
    auto str = [&]() {
        out.kind = NGX_CELL_STR;
        out.str_len = static_cast<int32_t>(v.len);
        out.v.str_off = strings.size();
        strings.append(sm.host(static_cast<uint64_t>(v.x), v.len), v.len);
    };
    switch (colType) {
        case T_BOOL: if (v.t != V_BOOL) return false; out.kind = NGX_CELL_BOOL; out.v.i = v.x; return true;
        case T_INT: if (v.t != V_INT) return false; out.kind = NGX_CELL_INT; out.v.i = v.x; return true;
        case T_VID: if (v.t != V_INT) return false; out.kind = NGX_CELL_ID; out.v.i = v.x; return true;
        case T_TIMESTAMP: if (v.t != V_INT) return false; out.kind = NGX_CELL_TIMESTAMP; out.v.i = v.x; return true;
        case T_FLOAT: if (v.t != V_DBL) return false; out.kind = NGX_CELL_FLOAT; out.v.i = v.x; return true;
        case T_DOUBLE: if (v.t != V_DBL) return false; out.kind = NGX_CELL_DOUBLE; out.v.i = v.x; return true;
        case T_STRING: if (v.t != V_STR) return false; str(); return true;
        default:
            switch (v.t) {
                case V_INT: out.kind = NGX_CELL_INT; out.v.i = v.x; return true;
                case V_DBL: out.kind = NGX_CELL_DOUBLE; out.v.i = v.x; return true;
                // left unset by toThriftResponse; the value stays in v.i (str_len 1 marks it) for an
                // interim result and for DISTINCT over pipe walks
                case V_BOOL: out.kind = NGX_CELL_EMPTY; out.v.i = v.x; out.str_len = 1; return true;
                case V_STR: str(); return true;
                default: out.kind = NGX_CELL_EMPTY; return true;
            }
    }
}

// raw value cell (GetNeighbors columns): kind from the VM type
void rawCell(const OutCell& v, ngx_cell& out, std::string& strings, const DeviceGraph& d, const DevPrograms& dp,
             const std::string& pool) {
    out.str_len = 0;
    out.v.i = v.x;
    switch (v.t) {
        case V_INT: out.kind = NGX_CELL_INT; break;
        case V_DBL: out.kind = NGX_CELL_DOUBLE; break;
        case V_BOOL: out.kind = NGX_CELL_BOOL; break;
        case V_STR: {
            std::string s = hostString(d, dp, pool, static_cast<uint64_t>(v.x), v.len);
            out.kind = NGX_CELL_STR;
            out.str_len = static_cast<int32_t>(s.size());
            out.v.str_off = strings.size();
            strings += s;
            break;
        }
        default: out.kind = NGX_CELL_EMPTY; out.v.i = 0; break;
    }
}

uint8_t nextEpoch(ngx_ctx* c) {
    if (c->epoch == 255) {
        HIP_OK(hipMemsetAsync(c->visited.p, 0, c->visitedSize, c->stream));
        c->epoch = 0;
    }
    return ++c->epoch;
}

void ensureVisited(ngx_ctx* c, uint64_t n) {
    if (c->visitedSize < n || c->visited.p == nullptr) {
        c->visited.get<uint8_t>(n);
        HIP_OK(hipMemsetAsync(c->visited.p, 0, n, c->stream));
        c->visitedSize = n;
        c->epoch = 0;
    }
}

template <typename T>
T readScalar(ngx_ctx* c, const T* dev) {
    T v;
    HIP_OK(hipMemcpyAsync(&v, dev, sizeof(T), hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    return v;
}

// next publication slot for a scan total (none when the mapped buffer is unavailable)
// slot 0 (words 0..3) for every publication but the seed hop's, which has slot kSeedSlot of its own: a
// hop sized on the device publishes while the seed total is still unread (spec1)
Publish nextPub(ngx_ctx* c, uint32_t slotWord = 0) {
    if (!c->pinDev) return Publish{nullptr, 0};
    return Publish{c->pinDev + c->pinLane + slotWord, ++c->pinSeq};   // (the active lane's slots)
}

// a plan whose host work may overlap another query's final hop (and whose own final hop may be overlapped):
// device-resident rows without DISTINCT, no input table
bool pipelinable(const ngx_go_plan& p) {
    return p.result_on_device && !p.distinct && !p.input_vid_col && p.record_to > 0;
}

void pipeSwitch(ngx_ctx* c, int state) {
    GoJob* j = c->pipe->cur;
    j->state = state;
    swapcontext(&j->uc, &c->pipe->main);
    j->state = GoPipe::kRunning;
}

// the last final hop's close is enqueued: defer the wait for its row count while the next query runs its
// hops on the other lane
void goDeferPoint(ngx_ctx* c) {
    GoPipe* P = c->pipe;
    GoJob* j = P ? P->cur : nullptr;
    if (!j || j->idx + 1 >= P->n || !pipelinable(*P->plans[j->idx + 1])) return;
    c->pipeOverlaps++;
    pipeSwitch(c, GoPipe::kDeferred);
}

// a record hop is about to write the shared result arrays while the previous query is deferred: with
// digests asked for (GoPipe::holdFinals), wait until that query has finished (its digest reads its rows)
void goPreFinalPoint(ngx_ctx* c) {
    GoPipe* P = c->pipe;
    GoJob* j = P ? P->cur : nullptr;
    if (j && P->holdFinals && P->ndeferred) pipeSwitch(c, GoPipe::kPreFinal);
}

// `to` waits for the work enqueued on `from` so far
void streamAfter(hipStream_t to, hipStream_t from, hipEvent_t ev) {
    HIP_OK(hipEventRecord(ev, from));
    HIP_OK(hipStreamWaitEvent(to, ev, 0));
}

// A record hop during a pipelined batch: the deferrable last final hop runs on the final stream, after
// this query's hops on the front stream, and its k_final_close on the close stream after it; any other
// record hop stays on the front stream, after every final hop and close enqueued so far
struct FinalStreamScope {
    ngx_ctx* c;
    hipStream_t saved = nullptr;
    FinalStreamScope(ngx_ctx* c_, bool onFinal) : c(c_) {
        if (!c->finalStream) return;
        if (onFinal) {
            hipStream_t fs = c->finalCur ? c->finalCur : c->finalStream;
            streamAfter(fs, c->stream, c->pipeEvent(0));
            if (c->laneClosePending[c->activeLane]) HIP_OK(hipStreamWaitEvent(fs, c->laneCloseEv[c->activeLane], 0));
            saved = c->stream;
            c->stream = fs;
        } else {
            streamAfter(c->stream, c->finalStream, c->pipeEvent(1));
            if (c->finalStream2) streamAfter(c->stream, c->finalStream2, c->pipeEvent(1));
            if (c->closeStream) streamAfter(c->stream, c->closeStream, c->pipeEvent(3));
        }
    }
    void restore() {
        if (saved) c->stream = saved;
        saved = nullptr;
    }
    ~FinalStreamScope() { restore(); }
};

// the front stream after every final hop enqueued so far (a batch query's rows read on the front stream)
void joinFinal(ngx_ctx* c) {
    if (c->finalStream) streamAfter(c->stream, c->finalStream, c->pipeEvent(1));
    if (c->finalStream2) streamAfter(c->stream, c->finalStream2, c->pipeEvent(1));
    if (c->closeStream) streamAfter(c->stream, c->closeStream, c->pipeEvent(3));
}

// the published scan total: poll the host-mapped slot (no stream round trip); after ~50 ms block on
// the stream, and read the device copy if the slot still disagrees. extra (final-hop publications):
// the word published beside the value (the query's error bits), or read from errDev on the fallback.
uint64_t awaitPub(ngx_ctx* c, const Publish& p, const uint64_t* devCopy, uint64_t* extra = nullptr,
                  const uint32_t* errDev = nullptr, uint64_t* extra2 = nullptr, const uint64_t* extra2Dev = nullptr) {
    auto errBits = [&] {
        if (!extra) return;
        uint32_t f[4];
        HIP_OK(hipMemcpy(f, errDev, 16, hipMemcpyDeviceToHost));
        *extra = 0;
        for (int k = 0; k < 4; k++) *extra |= static_cast<uint64_t>(f[k] != 0) << k;
    };
    if (!p.slot) { errBits(); return readScalar(c, devCopy); }
    auto t0 = std::chrono::steady_clock::now();
    // kernels.h Publish: the words are taken once the tag matches them
    uint64_t* const w = c->pin + (p.slot - c->pinDev);            // the slot's host view
    c->hmark("await");
    auto take = [&](uint64_t& v) {
        const uint64_t tag = __atomic_load_n(&w[1], __ATOMIC_ACQUIRE);
        v = __atomic_load_n(&w[0], __ATOMIC_ACQUIRE);
        const uint64_t x = __atomic_load_n(&w[2], __ATOMIC_ACQUIRE);
        const uint64_t x2 = __atomic_load_n(&w[3], __ATOMIC_ACQUIRE);
        if (tag != pubTag(p.seq, v, x, x2)) return false;
        if (extra) *extra = x;
        if (extra2) *extra2 = x2;
        return true;
    };
    uint64_t v = 0;
    for (uint32_t i = 0;; i++) {
        if (take(v)) {
            c->hmark("pub");
            return v;
        }
        __builtin_ia32_pause();
        if ((i & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(50)) break;
    }
    HIP_OK(hipStreamSynchronize(c->stream));
    if (c->finalStream) HIP_OK(hipStreamSynchronize(c->finalStream));   // (a batch's final hop runs there)
    if (c->finalStream2) HIP_OK(hipStreamSynchronize(c->finalStream2));
    if (c->closeStream) HIP_OK(hipStreamSynchronize(c->closeStream));
    if (take(v)) return v;
    errBits();
    if (extra2) *extra2 = extra2Dev ? readScalar(c, extra2Dev) : 0;
    return readScalar(c, devCopy);
}

// the query tail published by k_publish_tail: out[0] = error bits, out[1 ..] the extra words; false
// if it did not arrive within ~50 ms of polling (the caller synchronises and copies instead)
bool awaitTail(ngx_ctx* c, uint64_t seq, uint64_t* out, int n) {
    volatile uint64_t* slot = c->pin + c->pinLane + ngx_ctx::kTailOff;
    auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 0;; i++) {
        if (__atomic_load_n(const_cast<uint64_t*>(slot), __ATOMIC_ACQUIRE) == seq) {
            for (int k = 0; k < n; k++) out[k] = __atomic_load_n(const_cast<uint64_t*>(slot + 1 + k), __ATOMIC_RELAXED);
            return true;
        }
        __builtin_ia32_pause();
        if ((i & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(50)) return false;
    }
}

struct ColSpec { bool len, t; };

// Result holders: the C structs point into these vectors
struct GoResultHolder {
    ngx_go_result r{};
    std::vector<ngx_dev_column> devCols;
    std::vector<ngx_dev_column> hostCols;
    std::vector<int32_t> colTypes;
    std::vector<ngx_cell> cells;
    std::vector<int64_t> src, dst, rank;
    std::vector<int32_t> type;
    std::string strings;
    std::vector<std::string> built;                             // host copies of the result string arenas
    std::vector<uint64_t> hopFrontier, hopEdges, hopNext, hopXchg;
    // host-side timing of the call (steady clock): entry, first launch, device done
    std::chrono::steady_clock::time_point tIn, tLaunch, tDone;
    // host_columnar: the row arrays live in the context's page-locked staging
    const int64_t *rowSrcView = nullptr, *rowDstView = nullptr, *rowRankView = nullptr;
    const int32_t* rowTypeView = nullptr;
    std::vector<int32_t> devColW;                               // result_on_device: bytes per dev_cols[c].x
    std::vector<int64_t> devColConst;                           // ... and the value of a constant one (width 0)
};
struct GnResultHolder {
    ngx_gn_result r{};
    std::vector<int32_t> failed;
    std::vector<uint32_t> edgeVertex;
    std::vector<int32_t> edgeType;
    std::vector<int64_t> edgeDst;
    std::vector<ngx_cell> edgeCells, vertexCells;
    std::vector<uint8_t> vertexHasTag;
    std::string strings;
    // encode_rows: QueryResponse payload
    std::vector<uint8_t> edgeProps, tagProps;
    std::vector<uint64_t> edgePropsOff, tagPropsOff;
    std::vector<uint32_t> tagRowVertex;
    std::vector<int32_t> tagRowTag;
    struct Schema { int32_t isEdge, id; std::vector<std::string> names; std::vector<const char*> cnames; std::vector<int32_t> types; };
    std::vector<Schema> schemas;
    std::vector<ngx_schema_def> schemaView;
};

HopSlots makeHopSlots(const Space& sp, const DeviceGraph& d, const std::vector<int32_t>& types,
                      std::vector<int32_t>& hopTypes) {
    HopSlots hs{};
    hs.n = 0;
    hopTypes.clear();
    for (int32_t t : types) {
        int32_t si = sp.slotOf(t);
        if (si < 0) continue;                                  // no edges of this type here
        if (hs.n >= kMaxSlots) throw Error{NGX_E_UNSUPPORTED, "too many edge types in one hop"};
        const DSlot& ds = d.slots[si];
        hs.slotIdx[hs.n] = si;
        hs.etype[hs.n] = t;
        hs.off[hs.n] = ds.off;
        hs.dgid[hs.n] = ds.dgid;
        hs.dst[hs.n] = ds.dst;
        hs.rank[hs.n] = ds.rank;
        hs.rankC[hs.n] = ds.rankConst;
        hs.dstW[hs.n] = static_cast<int8_t>(ds.dstW);
        hs.rankW[hs.n] = static_cast<int8_t>(ds.rankW);
        hs.eflags[hs.n] = ds.hasFlags ? ds.eflags : nullptr;
        hs.colBase[hs.n] = ds.colBase;
        hs.n++;
        hopTypes.push_back(t);
    }
    return hs;
}

// host collective (ngx_config.exchange): device blocks staged through host memory
void hostExchange(ngx_ctx* c, int32_t op, const void* dsend, void* drecv, uint64_t bytes) {
    uint64_t sendBytes = op == NGX_XCHG_ALLGATHER ? bytes : bytes * c->world;
    std::vector<uint8_t> hs(sendBytes), hr(bytes * c->world);
    HIP_OK(hipMemcpyAsync(hs.data(), dsend, sendBytes, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    if (c->xchg(c->xchgUser, op, hs.data(), hr.data(), bytes) != 0) throw Error{NGX_E_DEVICE, "host exchange failed"};
    HIP_OK(hipMemcpyAsync(drecv, hr.data(), hr.size(), hipMemcpyHostToDevice, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
}

// RCCL watchdog: wait for the stream (which holds collective work) with a deadline, polling the
// communicator's asynchronous error. A peer that died or hangs must not hang this rank: on an error
// or after rcclTimeoutMs the communicator is aborted (ncclCommAbort ends its kernels) and the call
// fails; the context is then unusable (every later call returns NGX_E_DEVICE).
void rcclWait(ngx_ctx* c, const char* what) {
    if (!c->comm) return;
    auto t0 = std::chrono::steady_clock::now();
    auto abortWith = [&](const std::string& why) {
        (void)ncclCommAbort(c->comm);
        c->comm = nullptr;
        c->broken = true;
        throw Error{NGX_E_DEVICE, std::string("RCCL ") + what + ": " + why + "; communicator aborted"};
    };
    for (uint32_t i = 0;; i++) {
        hipError_t q = hipStreamQuery(c->stream);
        if (q == hipSuccess) return;
        if (q != hipErrorNotReady) abortWith(std::string("stream error ") + hipGetErrorString(q));
        ncclResult_t ae = ncclSuccess;
        if (ncclCommGetAsyncError(c->comm, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress)
            abortWith(std::string("async error ") + ncclGetErrorString(ae));
        if ((i & 255) == 255 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(c->rcclTimeoutMs))
            abortWith("timed out after " + std::to_string(c->rcclTimeoutMs) + " ms");
        if (i > 4096) std::this_thread::sleep_for(std::chrono::microseconds(50));
        else __builtin_ia32_pause();
    }
}

// all-gather of `bytes` per rank (rank order) over RCCL or the host exchange
void allGather(ngx_ctx* c, const void* dsend, void* drecv, uint64_t bytes) {
    if (c->xchg) {
        hostExchange(c, NGX_XCHG_ALLGATHER, dsend, drecv, bytes);
    } else {
        NCCL_OK(ncclAllGather(dsend, drecv, bytes, ncclUint8, c->comm, c->stream));
        rcclWait(c, "all-gather");
    }
}

// all-gather of host data: `bytes` per rank -> world blocks in rank order (host memory)
std::vector<uint8_t> gatherHost(ngx_ctx* c, const void* host, uint64_t bytes) {
    std::vector<uint8_t> out(bytes * c->world);
    if (bytes == 0) return out;
    uint8_t* ds = c->sendBits.get<uint8_t>(bytes);
    uint8_t* dr = c->recvBits.get<uint8_t>(bytes * c->world);
    HIP_OK(hipMemcpyAsync(ds, host, bytes, hipMemcpyHostToDevice, c->stream));
    allGather(c, ds, dr, bytes);
    HIP_OK(hipMemcpyAsync(out.data(), dr, out.size(), hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    return out;
}

// rows of every shard in global row order: each shard contributes its rows' `elem`-byte values
template <typename T>
std::vector<T> gatherRows(ngx_ctx* c, const HostGraph& g, const std::vector<T>& local) {
    uint64_t maxV = 0;
    for (int r = 0; r < c->world; r++) maxV = std::max(maxV, g.shardBase[r + 1] - g.shardBase[r]);
    std::vector<T> send(std::max<uint64_t>(maxV, 1));
    std::copy(local.begin(), local.end(), send.begin());
    std::vector<uint8_t> all = gatherHost(c, send.data(), maxV * sizeof(T));
    std::vector<T> out(g.vglobal);
    for (int r = 0; r < c->world; r++) {
        const uint64_t n = g.shardBase[r + 1] - g.shardBase[r];
        if (n) std::memcpy(out.data() + g.shardBase[r], all.data() + r * maxV * sizeof(T), n * sizeof(T));
    }
    return out;
}

// $$ props across shards (GoExecutor::fetchVertexProps -> QueryVertexPropsProcessor,
// src/graph/GoExecutor.cpp:937-973, src/storage/query/QueryVertexPropsProcessor.cpp:16-58): instead of
// a per-query fetch of the destinations' tag rows, every shard keeps replicas of all tag tables over
// the global rows (288 GB of HBM per GPU holds them), gathered once per snapshot on the first query
// that reads a $$ prop. Collective: every rank runs the same queries (GO is SPMD over the shards).
void ensureDstReplicas(ngx_ctx* c, Space& sp) {
    DeviceGraph& d = *sp.dev;
    const HostGraph& g = *sp.host;
    if (d.replicas) return;
    const uint64_t VG = g.vglobal;
    std::vector<DTag> rt;
    std::vector<DCol> rc;
    d.repHost.clear();
    std::vector<std::vector<HostColumn>> repCols(g.tags.size());
    for (size_t k = 0; k < g.tags.size(); k++) {
        const HostTag& t = g.tags[k];
        DTag dt = d.tags[k];
        dt.present = d.upload(gatherRows(c, g, t.present).data(), VG);
        dt.colBase = static_cast<int32_t>(rc.size());
        for (const HostColumn& lc : t.cols) {
            HostColumn h;
            h.type = lc.type;
            h.width = 8;
            switch (lc.type) {
                case T_INT: case T_TIMESTAMP: case T_VID: h.i64 = gatherRows(c, g, lc.i64); break;
                case T_FLOAT: case T_DOUBLE: h.f64 = gatherRows(c, g, lc.f64); break;
                case T_BOOL: h.b = gatherRows(c, g, lc.b); break;
                case T_STRING: {
                    std::vector<uint32_t> len(lc.soff.empty() ? 0 : lc.soff.size() - 1);
                    for (size_t i = 0; i < len.size(); i++) len[i] = static_cast<uint32_t>(lc.soff[i + 1] - lc.soff[i]);
                    std::vector<uint32_t> glen = gatherRows(c, g, len);
                    uint64_t mine = lc.sbytes.size();
                    std::vector<uint8_t> tot = gatherHost(c, &mine, 8);
                    uint64_t maxB = 0;
                    std::vector<uint64_t> per(c->world);
                    for (int r = 0; r < c->world; r++) { std::memcpy(&per[r], tot.data() + 8 * r, 8); maxB = std::max(maxB, per[r]); }
                    std::string sendB(lc.sbytes);
                    sendB.resize(std::max<uint64_t>(maxB, 1));
                    std::vector<uint8_t> allB = gatherHost(c, sendB.data(), maxB);
                    for (int r = 0; r < c->world; r++) h.sbytes.append(reinterpret_cast<const char*>(allB.data()) + r * maxB, per[r]);
                    h.soff.assign(VG + 1, 0);
                    for (uint64_t i = 0; i < VG; i++) h.soff[i + 1] = h.soff[i] + glen[i];
                    if (h.soff[VG] != h.sbytes.size()) throw Error{NGX_E_DEVICE, "tag replica string bytes disagree"};
                    break;
                }
                default: break;
            }
            // validity: replicated when any shard's column lacks values for some rows
            uint8_t allValid = lc.allValid ? 1 : 0;
            std::vector<uint8_t> flags = gatherHost(c, &allValid, 1);
            h.allValid = std::all_of(flags.begin(), flags.end(), [](uint8_t f) { return f != 0; });
            if (!h.allValid) {
                std::vector<uint8_t> lv = lc.allValid ? std::vector<uint8_t>(g.vid.size(), 1) : lc.valid;
                h.valid = gatherRows(c, g, lv);
            }
            repCols[k].push_back(std::move(h));
        }
        rt.push_back(dt);
    }
    // upload at 8 bytes per integer (the generated kernels read replicas at that width); repHost is
    // sized once: strRanges point into its strings
    size_t ncols = 0;
    for (auto& v : repCols) ncols += v.size();
    d.repHost.reserve(ncols);
    for (size_t k = 0; k < repCols.size(); k++) {
        for (HostColumn& h : repCols[k]) {
            DCol dc{};
            dc.type = h.type;
            switch (h.type) {
                case T_INT: case T_TIMESTAMP: case T_VID: dc.width = 8; dc.data = d.upload(h.i64.data(), VG); break;
                case T_FLOAT: case T_DOUBLE: dc.data = d.upload(h.f64.data(), VG); break;
                case T_BOOL: dc.data = d.upload(h.b.data(), VG); break;
                case T_STRING:
                    dc.soff = d.upload(h.soff.data(), VG + 1);
                    dc.sbytes = h.sbytes.empty() ? nullptr : d.upload(h.sbytes.data(), h.sbytes.size());
                    break;
                default: break;
            }
            if (!h.allValid) dc.valid = d.upload(h.valid.data(), VG);
            d.repHost.push_back(std::move(h));
            if (dc.sbytes) {
                const HostColumn& kept = d.repHost.back();
                d.strRanges.push_back({reinterpret_cast<uint64_t>(dc.sbytes), kept.sbytes.data(), kept.sbytes.size()});
            }
            rc.push_back(dc);
        }
    }
    std::sort(d.strRanges.begin(), d.strRanges.end(), [](const DeviceGraph::Range& a, const DeviceGraph::Range& b) { return a.dev < b.dev; });
    d.rtags = d.upload(rt.data(), rt.size());
    d.rcols = d.upload(rc.data(), rc.size());
    d.replicas = true;
}

}  // namespace

// ============================================================================ C ABI
extern "C" {

int32_t ngx_get_unique_id(void* out128) {
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return NGX_E_DEVICE;
    std::memcpy(out128, &id, sizeof(id));
    return NGX_OK;
}

int32_t ngx_open(const ngx_config* cfg, ngx_ctx** out) {
    if (!cfg || !out) return NGX_E_BAD_ARGUMENT;
    auto c = std::make_unique<ngx_ctx>();
    c->initLanes();
    c->device = cfg->device;
    c->rank = cfg->rank;
    c->world = cfg->world < 1 ? 1 : cfg->world;
    if (c->rank < 0 || c->rank >= c->world || c->device < 0 || c->world > kMaxWorld) return NGX_E_BAD_ARGUMENT;
    if (const char* j = std::getenv("NGX_JIT")) c->jitOn = std::string(j) != "0";
    if (const char* t = std::getenv("NGX_RCCL_TIMEOUT_MS")) c->rcclTimeoutMs = std::max<int64_t>(1, std::atoll(t));
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return NGX_E_DEVICE;
    if (hipSetDevice(c->device) != hipSuccess) return NGX_E_DEVICE;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) return NGX_E_DEVICE;
    {                                                 // ngx_go_batch's pipeline (without them: one at a time)
        // the hops (latency-bound, streams 0 and 2) at the higher priority, the final hops (bandwidth-bound,
        // streams 1 and 3: the two final streams, or the final and the close stream) at the lower: 0.365 /
        // 0.371 vs 0.374 / 0.412 ms per C2 step with both at the default, same box (r05); r06, stream 3 at
        // the lower too once it carries every second final hop: 0.2612 / 0.2648 vs 0.2753 / 0.2806 (two
        // process pairs, 4 rounds each)
        int prLo = 0, prHi = 0;
        (void)hipDeviceGetStreamPriorityRange(&prLo, &prHi);
        // (r06, priorities front / final / front / final, in-process medians: -1 / 1 / -1 / 1 0.2608 and 0.2574,
        // 0 / 1 / -1 / 1 0.2580, -1 / 1 / 0 / 1 0.2585; either final stream at the normal 0: 0.277 - 0.280)
        for (int k = 0; k < 4; k++)
            if (hipStreamCreateWithPriority(&c->pipeStreams[k], hipStreamNonBlocking, (k & 1) ? prLo : prHi) != hipSuccess)
                c->pipeStreams[k] = nullptr;
        for (auto& e : c->pipeEv)
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) e = nullptr;
        for (auto& e : c->pipeRing)
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) { c->pipeRing[0] = nullptr; break; }
        for (auto& e : c->laneCloseEv)
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) e = nullptr;
        // every event recorded once now: an event's first record costs far more than a later one (r06: a
        // process's first C2 batch, which reached ring events the 5-query warm-up had not, ran 0.31-0.32 vs
        // 0.29 ms per step; tools/ab_batch.py --prewarm-warm)
        for (auto e : c->pipeEv) if (e) (void)hipEventRecord(e, c->stream);
        for (auto e : c->pipeRing) if (e) (void)hipEventRecord(e, c->stream);
        for (auto e : c->laneCloseEv) if (e) (void)hipEventRecord(e, c->stream);
        (void)hipStreamSynchronize(c->stream);
    }
    if (hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess || c->cus < 1) c->cus = 256;
    if (const char* ht = std::getenv("NGX_HOST_TRACE")) c->htrace = std::string(ht) == "1";
    if (const char* pt = std::getenv("NGX_PIPE_TRACE")) c->ptrace = std::string(pt) == "1";
    if (hipHostMalloc(reinterpret_cast<void**>(&c->pin), ngx_ctx::kPinBytes, hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess) {
        std::memset(c->pin, 0, ngx_ctx::kPinBytes);
        if (hipHostGetDevicePointer(reinterpret_cast<void**>(&c->pinDev), c->pin, 0) != hipSuccess) c->pinDev = nullptr;
    } else {
        c->pin = nullptr;
    }
    c->xchg = cfg->exchange;
    c->xchgUser = cfg->exchange_user;
    if (c->world > 1 && !c->xchg) {
        if (!cfg->nccl_unique_id) return NGX_E_BAD_ARGUMENT;
        ncclUniqueId id;
        std::memcpy(&id, cfg->nccl_unique_id, sizeof(id));
        if (ncclCommInitRank(&c->comm, c->world, id, c->rank) != ncclSuccess) return NGX_E_DEVICE;
    }
    *out = c.release();
    return NGX_OK;
}

void ngx_close(ngx_ctx* c) {
    if (!c) return;
    {
        std::lock_guard<std::mutex> g(c->mu);          // waits for an in-flight call
        (void)hipSetDevice(c->device);
        (void)hipStreamSynchronize(c->stream);
    }
    delete c;                                          // ~ngx_ctx releases everything
}

const char* ngx_last_error(ngx_ctx* c) { return c ? c->lastError.c_str() : "no context"; }

#ifndef NGX_SRC_SHA
#define NGX_SRC_SHA "unknown"
#endif
const char* ngx_build_info(void) {
    return "src_sha=" NGX_SRC_SHA " arch=gfx950 built=" __DATE__ " " __TIME__;
}

int32_t ngx_add_space(ngx_ctx* c, int32_t space, int32_t numParts) {
    std::lock_guard<std::mutex> g(c->mu);
    auto& sp = c->spaces[space];
    if (!sp) sp = std::make_unique<Space>();
    sp->id = space;
    sp->numParts = numParts;
    return NGX_OK;
}

int32_t ngx_add_schema(ngx_ctx* c, int32_t space, int32_t isEdge, int32_t id, const char* name, int64_t ver,
                       int32_t nfields, const char* const* names, const int32_t* types, const char* ttlCol,
                       int64_t ttlDur) {
    std::lock_guard<std::mutex> g(c->mu);
    Space* sp = findSpace(c, space);
    if (!sp) return fail(c, NGX_E_SPACE_NOT_FOUND, "space not found");
    SchemaDef s;
    s.ver = ver;
    for (int32_t i = 0; i < nfields; i++) s.fields.push_back(FieldDef{names[i], types[i]});
    s.ttlCol = ttlCol ? ttlCol : "";
    s.ttlDur = ttlDur;
    auto& set = isEdge ? sp->edges[id] : sp->tags[id];
    set.id = id;
    set.name = name;
    set.versions[ver] = s;
    if (isEdge) {
        sp->edgeByName[name] = id;
        if (std::find(sp->edgeOrder.begin(), sp->edgeOrder.end(), name) == sp->edgeOrder.end()) sp->edgeOrder.push_back(name);
    } else {
        sp->tagByName[name] = id;
    }
    return NGX_OK;
}

}  // extern "C"

namespace {
// one KV row into the space's staging (rows of parts another shard owns are dropped)
void stageRow(ngx_ctx* c, StagedRows& st, const uint8_t* k, uint64_t kl, const uint8_t* v, uint64_t vl) {
    if (kl < 4) return;
    int32_t item;
    std::memcpy(&item, k, 4);
    int32_t part = item >> 8;
    if (c->world > 1 && ((part % c->world) + c->world) % c->world != c->rank) return;   // not ours
    st.koff.push_back(st.keys.size());
    st.klen.push_back(static_cast<uint32_t>(kl));
    st.keys.insert(st.keys.end(), k, k + kl);
    st.vals.insert(st.vals.end(), v, v + vl);
    st.voff.push_back(st.vals.size());
}

// snapshot generation: bumped by every commit / snapshot open (keys the JIT cache)
uint64_t nextGeneration() {
    static std::atomic<uint64_t> generations{0};
    return ++generations;
}
}  // namespace

extern "C" {

int32_t ngx_load_kv(ngx_ctx* c, int32_t space, const ngx_kv_batch* b) {
    std::lock_guard<std::mutex> g(c->mu);
    Space* sp = findSpace(c, space);
    if (!sp) return fail(c, NGX_E_SPACE_NOT_FOUND, "space not found");
    auto& st = sp->staged;
    if (st.voff.empty()) st.voff.push_back(0);
    for (uint64_t i = 0; i < b->n; i++) {
        stageRow(c, st, b->keys + b->key_off[i], b->key_off[i + 1] - b->key_off[i], b->vals + b->val_off[i],
                 b->val_off[i + 1] - b->val_off[i]);
    }
    return NGX_OK;
}

// encodeKV records (LogEncoder.cpp:16-27) of a part's snapshot stream; decodeKV as Part::commitSnapshot
int32_t ngx_load_snapshot_rows(ngx_ctx* c, int32_t space, const uint8_t* rows, uint64_t len) {
    if (!c || (len && !rows)) return NGX_E_BAD_ARGUMENT;
    std::lock_guard<std::mutex> g(c->mu);
    Space* sp = findSpace(c, space);
    if (!sp) return fail(c, NGX_E_SPACE_NOT_FOUND, "space not found");
    // validate the whole stream first: a truncated record stages nothing
    for (uint64_t p = 0; p < len;) {
        if (len - p < 8) return fail(c, NGX_E_BAD_ARGUMENT, "truncated snapshot record header");
        uint32_t ks, vs;
        std::memcpy(&ks, rows + p, 4);
        std::memcpy(&vs, rows + p + 4, 4);
        if (len - p - 8 < static_cast<uint64_t>(ks) + vs) return fail(c, NGX_E_BAD_ARGUMENT, "truncated snapshot record");
        p += 8 + static_cast<uint64_t>(ks) + vs;
    }
    auto& st = sp->staged;
    if (st.voff.empty()) st.voff.push_back(0);
    for (uint64_t p = 0; p < len;) {
        uint32_t ks, vs;
        std::memcpy(&ks, rows + p, 4);
        std::memcpy(&vs, rows + p + 4, 4);
        stageRow(c, st, rows + p + 8, ks, rows + p + 8 + ks, vs);
        p += 8 + static_cast<uint64_t>(ks) + vs;
    }
    return NGX_OK;
}

int32_t ngx_save_snapshot(ngx_ctx* c, int32_t space, const char* path, const char* tag) {
    if (!c || !path) return NGX_E_BAD_ARGUMENT;
    std::lock_guard<std::mutex> g(c->mu);
    Space* sp = findSpace(c, space);
    if (!sp) return fail(c, NGX_E_SPACE_NOT_FOUND, "space not found");
    if (!sp->host) return fail(c, NGX_E_NOT_LOADED, "space not committed");
    Error e = writeSnapshotFile(*sp, *sp->host, c->rank, c->world, path, tag ? tag : "");
    return e.code ? fail(c, e.code, e.msg) : NGX_OK;
}

int32_t ngx_open_snapshot(ngx_ctx* c, int32_t space, const char* path, char* tagOut) {
    if (!c || !path) return NGX_E_BAD_ARGUMENT;
    std::lock_guard<std::mutex> g(c->mu);
    Space* sp = findSpace(c, space);
    if (!sp) return fail(c, NGX_E_SPACE_NOT_FOUND, "space not found");
    try {
        HIP_OK(hipSetDevice(c->device));
        auto hg = std::make_unique<HostGraph>();
        std::string tag;
        Error e = readSnapshotFile(*sp, path, c->rank, c->world, *hg, tag);
        if (c->world > 1) {
            // collective: every rank's file must come from the same commit (the shards' global rows and
            // destination rows encode each other's vertex tables); a rank whose file failed still takes
            // part, so every rank reaches the same verdict and none waits in a later collective alone
            uint64_t mine[2] = {e.code ? 0ULL : 1ULL, e.code ? 0ULL : hg->commitDigest};
            std::vector<uint8_t> all = gatherHost(c, mine, sizeof(mine));
            for (int w = 0; w < c->world && !e.code; w++) {
                uint64_t other[2];
                std::memcpy(other, all.data() + w * sizeof(mine), sizeof(mine));
                if (!other[0]) e = Error{NGX_E_SNAPSHOT, std::string(path) + ": the snapshot of shard " + std::to_string(w) + " failed to open"};
                else if (other[1] != mine[1]) e = Error{NGX_E_SNAPSHOT, std::string(path) + ": snapshots of different commits across shards"};
            }
        }
        if (e.code) return fail(c, e.code, e.msg);
        sp->narrow = c->narrowColumns;
        auto dev = upload(*hg, *sp);
        attachMirrors(c, *sp, *hg, *dev);
        HIP_OK(hipDeviceSynchronize());
        sp->dev = std::move(dev);
        sp->gen = nextGeneration();
        sp->host = std::move(hg);
        sp->staged = StagedRows();
        if (tagOut) {
            std::memset(tagOut, 0, 64);
            std::memcpy(tagOut, tag.data(), std::min<size_t>(tag.size(), 63));
        }
        return NGX_OK;
    } catch (const Error& e) {
        return fail(c, e.code, e.msg);
    }
}

int32_t ngx_load_csr(ngx_ctx* c, int32_t space, const ngx_csr_shard* shard) {
    if (!c || !shard) return NGX_E_BAD_ARGUMENT;
    std::lock_guard<std::mutex> g(c->mu);
    Space* sp = findSpace(c, space);
    if (!sp) return fail(c, NGX_E_SPACE_NOT_FOUND, "space not found");
    auto hg = std::make_unique<HostGraph>();
    Error e = loadCsrShard(*sp, c->rank, c->world, *shard, *hg);
    if (e.code != NGX_OK) return fail(c, e.code, e.msg);
    sp->loaded = std::move(hg);
    sp->staged = StagedRows();
    return NGX_OK;
}

int32_t ngx_commit(ngx_ctx* c, int32_t space) {
    std::lock_guard<std::mutex> g(c->mu);
    Space* sp = findSpace(c, space);
    if (!sp) return fail(c, NGX_E_SPACE_NOT_FOUND, "space not found");
    try {
        HIP_OK(hipSetDevice(c->device));
        // NGX_HOST_TRACE=1: the commit's phases on stderr (export, tables, destinations, upload, mirrors)
        auto tc = std::chrono::steady_clock::now();
        auto phase = [&](const char* what) {
            if (!c->htrace) return;
            const auto now = std::chrono::steady_clock::now();
            std::fprintf(stderr, "[ngx commit r%d] %s %.2f s\n", c->rank, what, std::chrono::duration<double>(now - tc).count());
            tc = now;
        };
        std::unique_ptr<HostGraph> hg;
        if (sp->loaded) {                                        // ngx_load_csr: the shard is built
            hg = std::move(sp->loaded);
        } else {
            hg = std::make_unique<HostGraph>();
            if (sp->staged.voff.empty()) sp->staged.voff.push_back(0);
            Error e = exportSnapshot(*sp, c->rank, c->world, *hg);
            if (e.code != NGX_OK) return fail(c, e.code, e.msg);
        }
        phase("export");
        // vertex tables of every shard -> destination rows
        std::vector<std::vector<std::pair<int32_t, int64_t>>> tables(c->world);
        std::vector<std::pair<int32_t, int64_t>> mine(hg->vid.size());
        for (size_t i = 0; i < mine.size(); i++) mine[i] = {hg->vpart[i], hg->vid[i]};
        std::vector<uint64_t> nonces(c->world);
        const uint64_t nonce = std::random_device{}() ^ (static_cast<uint64_t>(std::random_device{}()) << 32) ^
                               static_cast<uint64_t>(std::chrono::steady_clock::now().time_since_epoch().count());
        if (c->world == 1) {
            tables[0] = mine;
            nonces[0] = nonce;
        } else {
            // allgather (count, commit nonce) pairs, then the (part, vid) tables, through RCCL
            uint64_t* dcnt = c->misc.get<uint64_t>(c->world * 2 + 2);
            uint64_t myCount[2] = {mine.size(), nonce};
            HIP_OK(hipMemcpyAsync(dcnt + 2 * c->world, myCount, 16, hipMemcpyHostToDevice, c->stream));
            allGather(c, dcnt + 2 * c->world, dcnt, 16);
            std::vector<uint64_t> cn(2 * c->world), counts(c->world);
            HIP_OK(hipMemcpyAsync(cn.data(), dcnt, 16 * c->world, hipMemcpyDeviceToHost, c->stream));
            HIP_OK(hipStreamSynchronize(c->stream));
            for (int w = 0; w < c->world; w++) { counts[w] = cn[2 * w]; nonces[w] = cn[2 * w + 1]; }
            uint64_t maxc = *std::max_element(counts.begin(), counts.end());
            std::vector<int64_t> packed(maxc * 2, 0);
            for (size_t i = 0; i < mine.size(); i++) { packed[2 * i] = mine[i].first; packed[2 * i + 1] = mine[i].second; }
            int64_t* sendb = c->sendBits.get<int64_t>(std::max<uint64_t>(maxc * 2, 2));
            int64_t* recvb = c->recvBits.get<int64_t>(std::max<uint64_t>(maxc * 2 * c->world, 2));
            HIP_OK(hipMemcpyAsync(sendb, packed.data(), maxc * 16, hipMemcpyHostToDevice, c->stream));
            allGather(c, sendb, recvb, maxc * 16);
            std::vector<int64_t> all(maxc * 2 * c->world);
            HIP_OK(hipMemcpyAsync(all.data(), recvb, all.size() * 8, hipMemcpyDeviceToHost, c->stream));
            HIP_OK(hipStreamSynchronize(c->stream));
            for (int w = 0; w < c->world; w++) {
                tables[w].resize(counts[w]);
                for (uint64_t i = 0; i < counts[w]; i++) {
                    tables[w][i] = {static_cast<int32_t>(all[(w * maxc + i) * 2]), all[(w * maxc + i) * 2 + 1]};
                }
            }
        }
        phase("vertex tables");
        resolveDstRows(*sp, *hg, tables, c->world);
        hg->commitDigest = tablesDigest(tables, nonces);
        if (hg->shardBase.empty()) { hg->shardBase = {0, hg->vid.size()}; hg->vglobal = hg->vid.size(); }
        hg->gbase = hg->shardBase[c->rank];
        phase("destination rows");
        sp->narrow = c->narrowColumns;
        sp->dev = upload(*hg, *sp);
        phase("upload");
        attachMirrors(c, *sp, *hg, *sp->dev);
        phase("mirrors + pull heads");
        sp->gen = nextGeneration();
        sp->host = std::move(hg);
        sp->staged = StagedRows();
        return NGX_OK;
    } catch (const Error& e) {
        return fail(c, e.code, e.msg);
    }
}

int32_t ngx_graph_info_get(ngx_ctx* c, int32_t space, ngx_graph_info* out) {
    std::lock_guard<std::mutex> g(c->mu);
    Space* sp = findSpace(c, space);
    if (!sp || !sp->dev) return fail(c, NGX_E_NOT_LOADED, "space not committed");
    out->vertices = sp->dev->V;
    out->edges = sp->host->edges;
    out->device_bytes = sp->dev->bytes;
    out->slots = static_cast<int32_t>(sp->dev->slots.size());
    out->tags = static_cast<int32_t>(sp->dev->tags.size());
    return NGX_OK;
}

int32_t ngx_device_to_host(ngx_ctx* c, void* dst, const void* src, uint64_t bytes) {
    if (!c || (bytes && (!dst || !src))) return NGX_E_BAD_ARGUMENT;
    std::lock_guard<std::mutex> g(c->mu);
    try {
        HIP_OK(hipSetDevice(c->device));
        if (bytes) {
            HIP_OK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
            HIP_OK(hipStreamSynchronize(c->stream));
        }
    } catch (const Error& e) {
        return fail(c, e.code, e.msg);
    }
    return NGX_OK;
}

int32_t ngx_synchronize(ngx_ctx* c) {
    if (!c) return NGX_E_BAD_ARGUMENT;
    std::lock_guard<std::mutex> g(c->mu);
    try {
        HIP_OK(hipSetDevice(c->device));
        HIP_OK(hipStreamSynchronize(c->stream));
    } catch (const Error& e) {
        return fail(c, e.code, e.msg);
    }
    return NGX_OK;
}

static int32_t resultDigest(ngx_ctx* c, const ngx_go_result* r, uint64_t out[3]);
int32_t ngx_go_result_digest(ngx_ctx* c, const ngx_go_result* r, uint64_t out[3]) {
    if (!c || !r || !out) return NGX_E_BAD_ARGUMENT;
    std::lock_guard<std::mutex> g(c->mu);
    return resultDigest(c, r, out);
}

// ngx_go_result_digest under the caller's lock
static int32_t resultDigest(ngx_ctx* c, const ngx_go_result* r, uint64_t out[3]) {
    try {
        HIP_OK(hipSetDevice(c->device));
        if (r->code != NGX_OK || (r->nrows && !r->dev_cols && r->ncols)) return fail(c, NGX_E_BAD_ARGUMENT, "digest: not a device-resident result");
        if (r->ncols > kDigestMaxCols) return fail(c, NGX_E_UNSUPPORTED, "digest: more than 16 YIELD columns");
        DigestArgs a{};
        a.n = r->nrows;
        a.ncols = r->ncols;
        a.x[0] = r->dev_src;
        a.w[0] = r->dev_key_w[0];
        a.c[0] = r->dev_key_const[0];
        if (!a.x[0]) a.w[0] = 0, a.c[0] = 0;          // yield_only (no src row array): the key hashes as 0
        for (int32_t k = 0; k < r->ncols; k++) {
            const ngx_dev_column& dc = r->dev_cols[k];
            if (dc.len || dc.type) return fail(c, NGX_E_UNSUPPORTED, "digest: string or untyped YIELD column");
            a.x[k + 1] = dc.x;
            a.w[k + 1] = r->dev_col_w ? r->dev_col_w[k] : 8;
            a.c[k + 1] = r->dev_col_const ? r->dev_col_const[k] : 0;
            if (a.n && a.w[k + 1] != 0 && !dc.x) return fail(c, NGX_E_BAD_ARGUMENT, "digest: column without values");
        }
        uint64_t* dev = c->misc.get<uint64_t>(3);
        a.out = dev;
        if (launchRowDigest(a, c->stream)) throw Error{NGX_E_DEVICE, "row digest"};
        HIP_OK(hipMemcpyAsync(out, dev, 24, hipMemcpyDeviceToHost, c->stream));
        HIP_OK(hipStreamSynchronize(c->stream));
    } catch (const Error& e) {
        return fail(c, e.code, e.msg);
    }
    return NGX_OK;
}

int32_t ngx_set_profiling(ngx_ctx* c, int32_t on) {
    std::lock_guard<std::mutex> g(c->mu);
    c->prof = on != 0;
    c->stats.clear();
    return NGX_OK;
}

int32_t ngx_kernel_stats(ngx_ctx* c, const ngx_kernel_stat** out, int32_t* n) {
    std::lock_guard<std::mutex> g(c->mu);
    c->statView.clear();
    for (auto& s : c->stats) c->statView.push_back(ngx_kernel_stat{s.name.c_str(), s.launches, s.ms, s.bytes});
    *out = c->statView.data();
    *n = static_cast<int32_t>(c->statView.size());
    return NGX_OK;
}

int32_t ngx_set_flag(ngx_ctx* c, const char* name, int64_t value) {
    std::lock_guard<std::mutex> g(c->mu);
    std::string n = name ? name : "";
    if (n == "jit") { c->jitOn = value != 0; return NGX_OK; }
    if (n == "poison_buffers") { gPoison.store(value != 0); return NGX_OK; }
    if (n == "str_arena_max") { c->strArenaMax = value > 0 ? static_cast<uint64_t>(value) : (uint64_t(8) << 30); return NGX_OK; }
    if (n == "rccl_timeout_ms") { c->rcclTimeoutMs = value < 1 ? 1 : value; return NGX_OK; }
    if (n == "max_edge_returned_per_vertex") { c->maxEdgesPerVertex = value <= 0 ? INT32_MAX : value; return NGX_OK; }
    if (n == "jit_cache_capacity") { c->jit.capacity = value < 1 ? 1 : static_cast<size_t>(value); return NGX_OK; }
    if (n == "pull_factor") { c->pullFactor = value < 0 ? 0 : value; return NGX_OK; }
    if (n == "jit_async") { c->jit.async = value != 0; c->jit.device = c->device; return NGX_OK; }
    if (n == "dyn_hops") { c->dynHops = value != 0; return NGX_OK; }
    if (n == "sparse_factor") { c->sparseFactor = value < 0 ? -1 : value; return NGX_OK; }
    if (n == "xchg_lists") { c->xchgLists = value < 0 ? -1 : (value ? 1 : 0); return NGX_OK; }
    if (n == "device_libm") { c->deviceLibm = value != 0; return NGX_OK; }
    if (n == "enable_reservoir_sampling") { c->reservoirSampling = value != 0; return NGX_OK; }
    if (n == "narrow_columns") { c->narrowColumns = value != 0; return NGX_OK; }
    if (n == "trace_go") { c->traceGo = value != 0; return NGX_OK; }
    if (n == "batch_pipeline") { c->batchPipeline = value != 0; return NGX_OK; }
    if (n == "batch_close_stream") { c->batchCloseStream = value != 0; return NGX_OK; }
    if (n == "batch_cu_split") {
        if (value != 0 && value != 32 && value != 64 && value != 128) return fail(c, NGX_E_BAD_ARGUMENT, "batch_cu_split: 0, 32, 64 or 128");
        c->batchCuSplit = static_cast<int32_t>(value);
        return NGX_OK;
    }
    if (n == "batch_fronts") {
        if (value != 1 && value != 2) return fail(c, NGX_E_BAD_ARGUMENT, "batch_fronts: 1 or 2");
        c->batchFronts = static_cast<int32_t>(value);
        return NGX_OK;
    }
    if (n == "batch_event_ring") { c->batchEventRing = value != 0; return NGX_OK; }
    if (n == "batch_finals") {
        if (value != 1 && value != 2) return fail(c, NGX_E_BAD_ARGUMENT, "batch_finals: 1 or 2");
        c->batchFinals = static_cast<int32_t>(value);
        return NGX_OK;
    }
    if (n == "batch_release_lanes") { c->batchReleaseLanes = value != 0; return NGX_OK; }
    if (n == "dst_props") {
        if (value < -1 || value > 1) return fail(c, NGX_E_BAD_ARGUMENT, "dst_props: -1 (by size), 0 (replicas) or 1 (owner fetch)");
        c->dstProps = static_cast<int32_t>(value);
        return NGX_OK;
    }
    if (n == "dense_final") { c->denseFinal = value != 0; return NGX_OK; }
    if (n == "dense_close_total") { c->denseCloseTotal = value != 0; return NGX_OK; }
    if (n == "dense_world_dev") { c->denseWorldDev = value != 0; return NGX_OK; }
    if (n == "dst_replica_max") { c->dstReplicaMax = static_cast<uint64_t>(std::max<int64_t>(value, 0)); return NGX_OK; }
    if (n == "release_lanes") {                       // action: free the parked lanes' buffers now
        if (value) c->releasedBytes += c->releaseParked();
        return NGX_OK;
    }
    if (n == "batch_lanes") {
        if (value < 2 || value > ngx_ctx::kMaxLanes) return fail(c, NGX_E_BAD_ARGUMENT, "batch_lanes: 2 .. 8");
        c->batchLanes = static_cast<int32_t>(value);
        return NGX_OK;
    }
    if (n == "final_nt_stores") { c->finalNtStores = value != 0; return NGX_OK; }
    if (n == "final_nt_loads") { c->finalNtLoads = value != 0; return NGX_OK; }
    if (n == "resv_groups") {
        if (value < 1 || value > static_cast<int64_t>(kResvMaxGroups))
            return fail(c, NGX_E_BAD_ARGUMENT, "resv_groups: 1 .. " + std::to_string(kResvMaxGroups));
        c->resvGroups = static_cast<uint32_t>(value);
        return NGX_OK;
    }
    if (n == "compact_wg") {
        if (value != 0 && value != 256 && value != 1024) return fail(c, NGX_E_BAD_ARGUMENT, "compact_wg: 0, 256 or 1024");
        c->compactWg = static_cast<int32_t>(value);
        return NGX_OK;
    }
    if (n == "compact_lane_rows") {
        if (value != 0 && value != 4 && value != 8 && value != 16) return fail(c, NGX_E_BAD_ARGUMENT, "compact_lane_rows: 0, 4, 8 or 16");
        c->compactLaneRows = static_cast<int32_t>(value);
        return NGX_OK;
    }
    if (n == "jit_wait") { c->jit.drain(); return NGX_OK; }
    return fail(c, NGX_E_BAD_ARGUMENT, "unknown flag " + n);
}

int32_t ngx_get_flag(ngx_ctx* c, const char* name, int64_t* value) {
    std::lock_guard<std::mutex> g(c->mu);
    std::string n = name ? name : "";
    if (n == "jit") *value = c->jitOn ? 1 : 0;
    else if (n == "poison_buffers") *value = gPoison.load() ? 1 : 0;
    else if (n == "str_arena_max") *value = static_cast<int64_t>(c->strArenaMax);
    else if (n == "rccl_timeout_ms") *value = c->rcclTimeoutMs;
    else if (n == "max_edge_returned_per_vertex") *value = c->maxEdgesPerVertex;
    else if (n == "pull_factor") *value = c->pullFactor;
    else if (n == "jit_async") *value = c->jit.async ? 1 : 0;
    else if (n == "dyn_hops") *value = c->dynHops ? 1 : 0;
    else if (n == "device_libm") *value = c->deviceLibm ? 1 : 0;
    else if (n == "enable_reservoir_sampling") *value = c->reservoirSampling ? 1 : 0;
    else if (n == "narrow_columns") *value = c->narrowColumns ? 1 : 0;
    else if (n == "trace_go") *value = c->traceGo ? 1 : 0;
    else if (n == "batch_pipeline") *value = c->batchPipeline ? 1 : 0;
    else if (n == "batch_lanes") *value = c->batchLanes;
    else if (n == "batch_finals") *value = c->batchFinals;
    else if (n == "dbuf_allocs") *value = static_cast<int64_t>(gDBufGen.load());
    else if (n == "dbuf_alloc_bytes") *value = static_cast<int64_t>(gDBufBytes.load());
    else if (n == "dst_props") *value = c->dstProps;
    else if (n == "dense_final") *value = c->denseFinal ? 1 : 0;
    else if (n == "dense_close_total") *value = c->denseCloseTotal ? 1 : 0;
    else if (n == "dense_world_dev") *value = c->denseWorldDev ? 1 : 0;
    else if (n == "dense_finals") *value = static_cast<int64_t>(c->denseFinals);
    else if (n == "dst_replica_max") *value = static_cast<int64_t>(c->dstReplicaMax);
    else if (n == "dst_fetches") *value = static_cast<int64_t>(c->dstFetches);
    else if (n == "dst_fetch_rows") *value = static_cast<int64_t>(c->dstFetchRows);
    else if (n == "batch_release_lanes") *value = c->batchReleaseLanes ? 1 : 0;
    else if (n == "released_lane_bytes") *value = static_cast<int64_t>(c->releasedBytes);
    else if (n == "batch_close_stream") *value = c->batchCloseStream ? 1 : 0;
    else if (n == "batch_fronts") *value = c->batchFronts;
    else if (n == "batch_cu_split") *value = c->batchCuSplit;
    else if (n == "batch_event_ring") *value = c->batchEventRing ? 1 : 0;
    else if (n == "batch_overlaps") *value = static_cast<int64_t>(c->pipeOverlaps);
    else if (n == "compact_lane_rows") *value = c->compactLaneRows;
    else if (n == "compact_wg") *value = c->compactWg;
    else if (n == "final_nt_stores") *value = c->finalNtStores ? 1 : 0;
    else if (n == "final_nt_loads") *value = c->finalNtLoads ? 1 : 0;
    else if (n == "resv_groups") *value = c->resvGroups;
    else if (n == "pull_hops") *value = static_cast<int64_t>(c->pullHops);
    else if (n == "sparse_hops") *value = static_cast<int64_t>(c->sparseHops);
    else if (n == "xchg_lists") *value = c->xchgLists;
    else if (n == "xchg_list_hops") *value = static_cast<int64_t>(c->xchgListHops);
    else if (n == "sparse_factor") *value = c->sparseFactor;
    else if (n == "pipe_walks") *value = static_cast<int64_t>(c->pipeWalks);
    else if (n == "jit_compiled") *value = static_cast<int64_t>(c->jit.compiled);
    else if (n == "jit_hits") *value = static_cast<int64_t>(c->jit.hits);
    else if (n == "jit_cached") *value = static_cast<int64_t>(c->jit.size());
    else if (n == "jit_evicted") *value = static_cast<int64_t>(c->jit.evicted);
    else if (n == "jit_failed") *value = static_cast<int64_t>(c->jit.failed);
    else if (n == "jit_compile_us") *value = static_cast<int64_t>(c->jit.compileSeconds * 1e6);
    else if (n == "jit_vgprs") *value = c->jit.lastRegs;          // registers / scratch of the last compiled
    else if (n == "jit_scratch") *value = c->jit.lastScratch;     // final-hop kernel (occupancy check)
    else return fail(c, NGX_E_BAD_ARGUMENT, "unknown flag " + n);
    return NGX_OK;
}

const char* ngx_jit_note(ngx_ctx* c) { return c ? c->jitNote.c_str() : ""; }

int64_t ngx_hash_string(const char* s, uint64_t n) {
    return static_cast<int64_t>(std::hash<std::string>()(std::string(s, n)));
}

void ngx_go_result_free(ngx_go_result* r) {
    if (r) delete reinterpret_cast<GoResultHolder*>(r);
}
void ngx_gn_result_free(ngx_gn_result* r) {
    if (r) delete reinterpret_cast<GnResultHolder*>(r);
}

}  // extern "C"

// ============================================================================ GO
namespace {

struct GoPlan {
    std::vector<int32_t> edgeTypes;                          // signed, GoExecutor::addToEdgeTypes order
    std::map<std::string, int32_t> aliasType;
    std::vector<std::string> aliasOrder;
    std::unique_ptr<ExprNode> where, pushed;
    std::vector<std::unique_ptr<ExprNode>> yields;
    PropRefs refs;
    std::vector<int32_t> colTypes;
};

// FROM $-.col / $var.col: the interim result the sentence reads and, during one sub-run, the input
// row whose values `$-.x' / `$var.x' take (InterimResultIndex::getColumnWithRow,
// src/graph/InterimResult.cpp:282-297)
struct InputBind {
    bool isVar = false;
    std::string var;
    std::map<std::string, int32_t> colIdx;                  // columnToIndex_: the last column of a name
    const ngx_go_plan* p = nullptr;
    const ngx_cell* row = nullptr;                          // bound row, or none (prepare only)
    // calculateExprType of kInputProp / kVariableProp (TraverseExecutor.cpp:141-158): the column's
    // type, UNKNOWN without data or for a column the schema lacks
    int32_t typeOf(const std::string& col) const {
        if (!p || p->input_nrows == 0) return T_UNKNOWN;
        auto it = colIdx.find(col);
        return it == colIdx.end() ? T_UNKNOWN : p->input_types[it->second];
    }
};

// `$-.x' / `$var.x' -> the bound row's value as a constant of its variant type; graphd evaluates them
// per input row, never at storage (they are not pushable: TraverseExecutor.cpp:512-516)
int32_t bindRow(ExprNode& n, const InputBind& b, std::string& err) {
    if (n.kind == K_INPUT_PROP || n.kind == K_VAR_PROP) {
        auto it = b.colIdx.find(n.prop);
        if (it == b.colIdx.end()) { err = "Prop `" + n.prop + "' not found"; return NGX_E_QUERY; }
        const ngx_cell& v = b.row[it->second];
        n.kind = K_PRIMARY;
        n.ref.clear(); n.alias.clear(); n.prop.clear();
        switch (v.kind) {
            case NGX_CELL_BOOL: n.vtype = 2; n.i = v.v.i != 0; break;
            case NGX_CELL_INT: case NGX_CELL_ID: case NGX_CELL_TIMESTAMP: n.vtype = 0; n.i = v.v.i; break;
            case NGX_CELL_FLOAT: case NGX_CELL_DOUBLE: n.vtype = 1; n.d = v.v.d; break;
            case NGX_CELL_STR:
                n.vtype = 3;
                n.s.assign(b.p->input_strings + v.v.str_off, static_cast<size_t>(v.str_len));
                break;
            default: err = "Unknown VariantType in the input row"; return NGX_E_BAD_ARGUMENT;
        }
        return NGX_OK;
    }
    for (auto& k : n.kids) {
        int32_t rc = bindRow(*k, b, err);
        if (rc) return rc;
    }
    return NGX_OK;
}

int32_t prepareGo(ngx_ctx* c, const Space& sp, const ngx_go_plan& p, GoPlan& gp, const InputBind* in = nullptr) {
    auto addTypes = [&](int32_t t) {                         // GoExecutor.cpp:297-319
        if (p.direction == NGX_DIR_FORWARD) gp.edgeTypes.push_back(t);
        else if (p.direction == NGX_DIR_REVERSELY) gp.edgeTypes.push_back(-t);
        else { gp.edgeTypes.push_back(t); gp.edgeTypes.push_back(-t); }
    };
    if (p.over_all) {
        for (auto& name : sp.edgeOrder) {
            int32_t t = sp.edgeByName.at(name);
            addTypes(t);
            if (gp.aliasType.count(name)) return fail(c, NGX_E_QUERY, "edge alias(" + name + ") was dup");
            gp.aliasType[name] = std::abs(t);
            gp.aliasOrder.push_back(name);
        }
    } else {
        for (int32_t i = 0; i < p.nover; i++) {
            std::string name = p.over_names[i];
            auto it = sp.edgeByName.find(name);
            if (it == sp.edgeByName.end()) return fail(c, NGX_E_QUERY, "Edge `" + name + "' not found");
            addTypes(it->second);
            std::string alias = (p.over_aliases && p.over_aliases[i] && p.over_aliases[i][0]) ? p.over_aliases[i] : name;
            if (gp.aliasType.count(alias)) return fail(c, NGX_E_QUERY, "edge alias(" + alias + ") was dup");
            gp.aliasType[alias] = std::abs(it->second);
            gp.aliasOrder.push_back(alias);
        }
    }
    std::string err;
    if (p.where && p.where_len) {
        gp.where = decodeExpr(p.where, p.where_len, err);
        if (!gp.where) return fail(c, NGX_E_QUERY, err);
        collectRefs(*gp.where, gp.refs);
        if (p.filter_pushdown) {
            auto copy = cloneExpr(*gp.where);
            if (rewritePushdown(*copy)) gp.pushed = std::move(copy);
        }
    }
    for (int32_t i = 0; i < p.nyields; i++) {
        auto y = decodeExpr(p.yields[i], p.yield_lens[i], err);
        if (!y) return fail(c, NGX_E_QUERY, err);
        collectRefs(*y, gp.refs);
        gp.yields.push_back(std::move(y));
    }
    if (p.over_all && gp.yields.empty()) {                    // GoExecutor.cpp:723-732
        for (auto& a : gp.aliasOrder) {
            auto n = std::make_unique<ExprNode>();
            n->kind = K_EDGE_DST; n->alias = a; n->prop = "_dst";
            gp.yields.push_back(std::move(n));
        }
    }
    // prepareNeededProps (GoExecutor.cpp:367-392)
    if (gp.refs.variable) {
        if (!in || !in->isVar) return fail(c, NGX_E_QUERY, "A variable must be referred in FROM before used in WHERE or YIELD");
        if (gp.refs.vars.size() > 1) return fail(c, NGX_E_QUERY, "Only one variable allowed to use");
        if (*gp.refs.vars.begin() != in->var)
            return fail(c, NGX_E_QUERY, "Variable name not match: `" + *gp.refs.vars.begin() + "' vs. `" + in->var + "'");
    }
    if (gp.refs.input && (!in || in->isVar)) return fail(c, NGX_E_QUERY, "`$-' must be referred in FROM before used in WHERE or YIELD");
    for (auto& tp : gp.refs.srcTag) if (!sp.tagByName.count(tp.first)) return fail(c, NGX_E_QUERY, "Tag `" + tp.first + "' not found.");
    for (auto& tp : gp.refs.dstTag) if (!sp.tagByName.count(tp.first)) return fail(c, NGX_E_QUERY, "Tag `" + tp.first + "' not found.");
    // checkNeededProps (GoExecutor.cpp:422-468)
    for (auto* set : {&gp.refs.srcTag, &gp.refs.dstTag}) {
        for (auto& tp : *set) {
            const SchemaSet* ss = sp.tag(sp.tagByName.at(tp.first));
            if (!ss) return fail(c, NGX_E_QUERY, "No tag schema for " + tp.first);
            if (ss->latest().index(tp.second) < 0) return fail(c, NGX_E_QUERY, "`" + tp.second + "' is not a prop of `" + tp.first + "'");
        }
    }
    for (auto& ap : gp.refs.alias) {
        auto at = gp.aliasType.find(ap.first);
        if (at == gp.aliasType.end()) return fail(c, NGX_E_QUERY, "Edge `" + ap.first + "' not found.");
        if (ap.second == "_src" || ap.second == "_dst" || ap.second == "_rank" || ap.second == "_type") continue;
        const SchemaSet* es = sp.edge(at->second);
        if (!es) return fail(c, NGX_E_QUERY, "No edge schema for " + ap.first);
        if (es->latest().index(ap.second) < 0) return fail(c, NGX_E_QUERY, "`" + ap.second + "' is not a prop of `" + ap.first + "'");
    }
    for (auto& f : gp.refs.funcs) (void)f;
    for (auto& y : gp.yields) {
        bool inputCol = in && (y->kind == K_INPUT_PROP || y->kind == K_VAR_PROP);
        gp.colTypes.push_back(inputCol ? in->typeOf(y->prop) : exprType(*y, sp));
    }
    if (in && in->row && (gp.refs.input || gp.refs.variable)) {
        // the pushed copy was rewritten before binding: input props never reach storage
        if (gp.where) {
            int32_t rc = bindRow(*gp.where, *in, err);
            if (rc) return fail(c, rc, err);
        }
        for (auto& y : gp.yields) {
            int32_t rc = bindRow(*y, *in, err);
            if (rc) return fail(c, rc, err);
        }
    }
    return NGX_OK;
}

// exchange the hop's marks: every shard sends peer q the bitmap of q's rows it marked
void exchangeFrontier(ngx_ctx* c, const DeviceGraph& d, uint8_t epoch) {
    int W = c->world;
    const auto& sb = d.shardBase;
    uint64_t maxWords = 0;
    for (int q = 0; q < W; q++) maxWords = std::max(maxWords, (sb[q + 1] - sb[q] + 63) / 64);
    uint64_t* send = c->sendBits.get<uint64_t>(std::max<uint64_t>(maxWords * W, 1));
    uint64_t* recv = c->recvBits.get<uint64_t>(std::max<uint64_t>(maxWords * W, 1));
    uint64_t myRows = sb[c->rank + 1] - sb[c->rank];
    uint64_t myWords = (myRows + 63) / 64;
    ExchangeArgs xa{};
    xa.visited = c->visited.get<uint8_t>(d.vglobal);
    xa.epoch = epoch;
    for (int q = 0; q <= W; q++) xa.sb[q] = sb[q];
    xa.world = W;
    xa.rank = c->rank;
    xa.words = maxWords;
    xa.bits = send;
    if (launchPackPeers(xa, c->stream)) throw Error{NGX_E_DEVICE, "pack"};
    c->lastXchgBytes = 0;
    for (int q = 0; q < W; q++) if (q != c->rank) c->lastXchgBytes += (sb[q + 1] - sb[q] + 63) / 64 * 8;
    if (c->xchg) {
        hostExchange(c, NGX_XCHG_ALLTOALL, send, recv, maxWords * 8);
    } else {
        NCCL_OK(ncclGroupStart());
        for (int q = 0; q < W; q++) {
            if (q == c->rank) continue;
            uint64_t nq = (sb[q + 1] - sb[q] + 63) / 64;
            if (nq) NCCL_OK(ncclSend(send + q * maxWords, nq * 8, ncclUint8, q, c->comm, c->stream));
            if (myWords) NCCL_OK(ncclRecv(recv + q * maxWords, myWords * 8, ncclUint8, q, c->comm, c->stream));
        }
        NCCL_OK(ncclGroupEnd());
        rcclWait(c, "frontier all-to-all");
    }
    xa.bits = recv;
    if (launchMergePeers(xa, c->stream)) throw Error{NGX_E_DEVICE, "merge"};
}

// The list form (for hops whose frontier is small next to the peers' rows; StorageClient
// groups a request's vids per host the same way, StorageClient.h:260-290): every shard lists the rows
// it marked in each peer's range, the shards all-gather their per-peer counts (W words each, so every
// rank knows what it sends and receives), then send exactly those vids (4 B each) and each owner marks
// the rows it received. Bytes per hop: 4 x the marked peer rows + the counts, against V / 8 per peer
// for the bitmaps.
void exchangeFrontierList(ngx_ctx* c, const DeviceGraph& d, uint8_t epoch) {
    const int W = c->world;
    const auto& sb = d.shardBase;
    uint64_t cap = 1;
    for (int q = 0; q < W; q++) cap = std::max<uint64_t>(cap, sb[q + 1] - sb[q]);
    uint32_t* send = c->xListSend.get<uint32_t>(cap * W);
    unsigned long long* counts = c->xCounts.get<unsigned long long>(static_cast<size_t>(W) * (W + 1));
    unsigned long long* all = counts + W;
    HIP_OK(hipMemsetAsync(counts, 0, W * 8, c->stream));
    ListXchgArgs la{};
    la.visited = c->visited.get<uint8_t>(d.vglobal);
    la.epoch = epoch;
    for (int q = 0; q <= W; q++) la.sb[q] = sb[q];
    la.world = W;
    la.rank = c->rank;
    la.list = send;
    la.cap = cap;
    la.counts = counts;
    if (launchPackLists(la, c->stream)) throw Error{NGX_E_DEVICE, "pack lists"};
    allGather(c, counts, all, static_cast<uint64_t>(W) * 8);         // all[p * W + q]: p sends q
    std::vector<uint64_t> m(static_cast<size_t>(W) * W);
    HIP_OK(hipMemcpyAsync(m.data(), all, m.size() * 8, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    std::vector<uint64_t> roff(W + 1, 0);                              // received list q at roff[q]
    uint64_t block = 0;
    for (int q = 0; q < W; q++) {
        roff[q + 1] = roff[q] + (q == c->rank ? 0 : m[static_cast<size_t>(q) * W + c->rank]);
        for (int p = 0; p < W; p++) if (p != q) block = std::max<uint64_t>(block, m[static_cast<size_t>(p) * W + q]);
    }
    uint32_t* recv = c->xListRecv.get<uint32_t>(std::max<uint64_t>(roff[W], 1));
    c->lastXchgBytes = static_cast<uint64_t>(W - 1) * W * 8;
    for (int q = 0; q < W; q++) if (q != c->rank) c->lastXchgBytes += m[static_cast<size_t>(c->rank) * W + q] * 4;
    if (c->xchg) {
        // the host collective moves equal blocks: every list padded to the largest count of any pair
        if (block) {
            std::vector<uint32_t> hs(block * W, 0), hr(block * W, 0);
            for (int q = 0; q < W; q++) {
                const uint64_t n = q == c->rank ? 0 : m[static_cast<size_t>(c->rank) * W + q];
                if (n) HIP_OK(hipMemcpyAsync(hs.data() + q * block, send + q * cap, n * 4, hipMemcpyDeviceToHost, c->stream));
            }
            HIP_OK(hipStreamSynchronize(c->stream));
            if (c->xchg(c->xchgUser, NGX_XCHG_ALLTOALL, hs.data(), hr.data(), block * 4) != 0)
                throw Error{NGX_E_DEVICE, "host exchange failed"};
            std::vector<uint32_t> packed(std::max<uint64_t>(roff[W], 1));
            for (int q = 0; q < W; q++)
                std::copy(hr.begin() + q * block, hr.begin() + q * block + (roff[q + 1] - roff[q]), packed.begin() + roff[q]);
            if (roff[W]) HIP_OK(hipMemcpyAsync(recv, packed.data(), roff[W] * 4, hipMemcpyHostToDevice, c->stream));
            HIP_OK(hipStreamSynchronize(c->stream));
        }
    } else {
        NCCL_OK(ncclGroupStart());
        for (int q = 0; q < W; q++) {
            if (q == c->rank) continue;
            const uint64_t ns = m[static_cast<size_t>(c->rank) * W + q], nr = roff[q + 1] - roff[q];
            if (ns) NCCL_OK(ncclSend(send + q * cap, ns * 4, ncclUint8, q, c->comm, c->stream));
            if (nr) NCCL_OK(ncclRecv(recv + roff[q], nr * 4, ncclUint8, q, c->comm, c->stream));
        }
        NCCL_OK(ncclGroupEnd());
        rcclWait(c, "frontier vid lists");
    }
    if (launchMergeList(recv, roff[W], c->visited.get<uint8_t>(d.vglobal) + d.gbase, epoch, c->stream))
        throw Error{NGX_E_DEVICE, "merge lists"};
    c->xchgListHops++;
}

// Variable-size all-to-all of device blocks: this rank sends block q (sendDev + soff[q], mat[me * W + q]
// bytes) to rank q and receives rank p's block at recvDev + roff[p] (mat[p * W + me] bytes). Every rank
// passes the same byte matrix mat[p * W + q]. Its own block is a device copy; the host collective moves
// equal blocks of the largest count of any pair; RCCL sends and receives exactly.
void allToAllV(ngx_ctx* c, const uint8_t* sendDev, const std::vector<uint64_t>& soff, uint8_t* recvDev,
               const std::vector<uint64_t>& roff, const std::vector<uint64_t>& mat) {
    const int W = c->world, me = c->rank;
    const uint64_t self = mat[static_cast<size_t>(me) * W + me];
    if (self) HIP_OK(hipMemcpyAsync(recvDev + roff[me], sendDev + soff[me], self, hipMemcpyDeviceToDevice, c->stream));
    uint64_t block = 0;
    for (int p = 0; p < W; p++)
        for (int q = 0; q < W; q++) if (p != q) block = std::max<uint64_t>(block, mat[static_cast<size_t>(p) * W + q]);
    if (block == 0) return;
    if (c->xchg) {
        std::vector<uint8_t> hs(block * W, 0), hr(block * W, 0);
        for (int q = 0; q < W; q++) {
            const uint64_t n = q == me ? 0 : mat[static_cast<size_t>(me) * W + q];
            if (n) HIP_OK(hipMemcpyAsync(hs.data() + q * block, sendDev + soff[q], n, hipMemcpyDeviceToHost, c->stream));
        }
        HIP_OK(hipStreamSynchronize(c->stream));
        if (c->xchg(c->xchgUser, NGX_XCHG_ALLTOALL, hs.data(), hr.data(), block) != 0) throw Error{NGX_E_DEVICE, "host exchange failed"};
        for (int p = 0; p < W; p++) {
            const uint64_t n = p == me ? 0 : mat[static_cast<size_t>(p) * W + me];
            if (n) HIP_OK(hipMemcpyAsync(recvDev + roff[p], hr.data() + p * block, n, hipMemcpyHostToDevice, c->stream));
        }
        HIP_OK(hipStreamSynchronize(c->stream));
    } else {
        NCCL_OK(ncclGroupStart());
        for (int q = 0; q < W; q++) {
            if (q == me) continue;
            const uint64_t ns = mat[static_cast<size_t>(me) * W + q], nr = mat[static_cast<size_t>(q) * W + me];
            if (ns) NCCL_OK(ncclSend(sendDev + soff[q], ns, ncclUint8, q, c->comm, c->stream));
            if (nr) NCCL_OK(ncclRecv(recvDev + roff[q], nr, ncclUint8, q, c->comm, c->stream));
        }
        NCCL_OK(ncclGroupEnd());
        rcclWait(c, "dst props all-to-all");
    }
}

// the byte matrix of an exchange: this rank's row (bytes to each rank) all-gathered
std::vector<uint64_t> gatherMatrix(ngx_ctx* c, const std::vector<uint64_t>& row) {
    const int W = c->world;
    const std::vector<uint8_t> all = gatherHost(c, row.data(), static_cast<uint64_t>(W) * 8);
    std::vector<uint64_t> m(static_cast<size_t>(W) * W);
    std::memcpy(m.data(), all.data(), m.size() * 8);
    return m;
}

// bytes of one fetched row's fixed record: per tag its present byte; per column its 8-byte value (int /
// double bits / bool), its valid byte and, for strings, a 4-byte length (the bytes follow the records)
uint64_t dstRecordBytes(const HostGraph& g) {
    uint64_t b = 0;
    for (const HostTag& t : g.tags) {
        b += 1;
        for (const HostColumn& col : t.cols) b += 9 + (col.type == T_STRING ? 4 : 0);
    }
    return b;
}

// $$ props at world > 1, fetched from their owners for one record hop (GoExecutor::fetchVertexProps,
// GoExecutor.cpp:937-973, answered by QueryVertexPropsProcessor, src/storage/query/
// QueryVertexPropsProcessor.cpp:16-58): every shard
//   1. marks the global rows its record hop's edges lead to (the push expansion's kernel, a fresh epoch),
//   2. lists them per owner (its own rows too) and sends each owner its list (counts all-gathered first),
//   3. as an owner, reads the requested rows' tag values from its host tables and sends them back,
//   4. stores what it receives as tag tables over the fetched rows only, and a global row -> fetched row
//      map (FinalArgs::dstMap) that the final hop's $$ reads go through.
// Collective: every shard calls it for every record hop (E = 0 too: it still answers its peers). Memory is
// O(fetched rows) per query, not O(global rows) of every tag column per shard as the replicas are.
struct DstFetch { const DTag* tags = nullptr; const DCol* cols = nullptr; const uint32_t* map = nullptr; };
DstFetch fetchDstProps(ngx_ctx* c, Space& sp, size_t recIdx, const uint32_t* F, const uint64_t* estart,
                       const uint64_t* chunkFirst, uint64_t nEnt, uint64_t E, const HopSlots& hs, bool pos32,
                       const uint64_t* ebase) {
    DeviceGraph& d = *sp.dev;
    const HostGraph& g = *sp.host;
    const int W = c->world, me = c->rank;
    const auto& sb = d.shardBase;
    DstLane& L = c->dst;
    // 1. destination rows
    ensureVisited(c, d.vglobal);
    const uint8_t ep = nextEpoch(c);
    if (E && launchExpandMark(F, estart, chunkFirst, nEnt, E, hs, static_cast<uint8_t*>(c->visited.p), ep, pos32, c->stream,
                              nullptr, nullptr, ~0ULL, ebase))
        throw Error{NGX_E_DEVICE, "dst marks"};
    // 2. per owner lists (local offsets in the owner's range), counts all-gathered
    uint64_t cap = 1;
    for (int q = 0; q < W; q++) cap = std::max<uint64_t>(cap, sb[q + 1] - sb[q]);
    uint32_t* lists = L.req.get<uint32_t>(cap * W);
    unsigned long long* counts = L.counts.get<unsigned long long>(W);
    HIP_OK(hipMemsetAsync(counts, 0, W * 8, c->stream));
    ListXchgArgs la{};
    la.visited = static_cast<const uint8_t*>(c->visited.p);
    la.epoch = ep;
    for (int q = 0; q <= W; q++) la.sb[q] = sb[q];
    la.world = W;
    la.rank = me;
    la.list = lists;
    la.cap = cap;
    la.counts = counts;
    la.includeSelf = 1;
    if (launchPackLists(la, c->stream)) throw Error{NGX_E_DEVICE, "dst lists"};
    std::vector<uint64_t> mine(W);
    HIP_OK(hipMemcpyAsync(mine.data(), counts, W * 8, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    const std::vector<uint64_t> m = gatherMatrix(c, mine);         // m[p * W + q]: rows p asks of q
    std::vector<uint64_t> soff(W), roff(W + 1, 0), mat4(static_cast<size_t>(W) * W);
    for (int q = 0; q < W; q++) soff[q] = static_cast<uint64_t>(q) * cap * 4;
    for (int p = 0; p < W; p++) roff[p + 1] = roff[p] + m[static_cast<size_t>(p) * W + me] * 4;
    for (size_t k = 0; k < mat4.size(); k++) mat4[k] = m[k] * 4;
    uint8_t* recv = L.recv.get<uint8_t>(std::max<uint64_t>(roff[W], 4));
    allToAllV(c, reinterpret_cast<const uint8_t*>(lists), soff, recv, roff, mat4);
    // 3. as the owner: the requested rows' values from the host tables, one blob per requester
    std::vector<uint32_t> asked(roff[W] / 4);
    if (!asked.empty()) HIP_OK(hipMemcpyAsync(asked.data(), recv, roff[W], hipMemcpyDeviceToHost, c->stream));
    std::vector<uint32_t> myReq;                                   // my lists, owner by owner (the row order)
    uint64_t nReq = 0;
    for (int q = 0; q < W; q++) nReq += m[static_cast<size_t>(me) * W + q];
    myReq.resize(nReq);
    {
        uint64_t at = 0;
        for (int q = 0; q < W; q++) {
            const uint64_t n = m[static_cast<size_t>(me) * W + q];
            if (n) HIP_OK(hipMemcpyAsync(myReq.data() + at, lists + q * cap, n * 4, hipMemcpyDeviceToHost, c->stream));
            at += n;
        }
    }
    HIP_OK(hipStreamSynchronize(c->stream));
    const uint64_t rec = dstRecordBytes(g);
    std::vector<uint64_t> boff(W + 1, 0);                          // blob of requester p at boff[p]
    std::vector<uint8_t> blobs;
    for (int p = 0; p < W; p++) {
        const uint32_t* rows = asked.data() + roff[p] / 4;
        const uint64_t n = (roff[p + 1] - roff[p]) / 4;
        const uint64_t base = blobs.size();
        blobs.resize(base + n * rec);
        std::string bytes;
        for (uint64_t i = 0; i < n; i++) {
            const uint32_t r = rows[i];
            if (r >= g.vid.size()) throw Error{NGX_E_DEVICE, "dst fetch: row outside the shard"};
            uint8_t* o = blobs.data() + base + i * rec;
            for (const HostTag& t : g.tags) {
                *o++ = t.present[r];
                for (const HostColumn& col : t.cols) {
                    uint64_t v = 0;
                    switch (col.type) {
                        case T_INT: case T_TIMESTAMP: case T_VID: v = static_cast<uint64_t>(col.i64[r]); break;
                        case T_FLOAT: case T_DOUBLE: std::memcpy(&v, &col.f64[r], 8); break;
                        case T_BOOL: v = col.b[r]; break;
                        default: break;
                    }
                    std::memcpy(o, &v, 8);
                    o[8] = col.allValid ? 1 : col.valid[r];
                    o += 9;
                    if (col.type == T_STRING) {
                        const uint32_t len = static_cast<uint32_t>(col.soff[r + 1] - col.soff[r]);
                        std::memcpy(o, &len, 4);
                        o += 4;
                        bytes.append(col.sbytes, col.soff[r], len);
                    }
                }
            }
        }
        blobs.insert(blobs.end(), bytes.begin(), bytes.end());
        boff[p + 1] = blobs.size();
    }
    std::vector<uint64_t> brow(W);
    for (int p = 0; p < W; p++) brow[p] = boff[p + 1] - boff[p];
    const std::vector<uint64_t> bm = gatherMatrix(c, brow);       // bm[q * W + p]: bytes owner q sends p
    uint8_t* bs = L.blobS.get<uint8_t>(std::max<uint64_t>(blobs.size(), 8));
    if (!blobs.empty()) HIP_OK(hipMemcpyAsync(bs, blobs.data(), blobs.size(), hipMemcpyHostToDevice, c->stream));
    std::vector<uint64_t> bro(W + 1, 0);
    for (int q = 0; q < W; q++) bro[q + 1] = bro[q] + bm[static_cast<size_t>(q) * W + me];
    uint8_t* br = L.blobR.get<uint8_t>(std::max<uint64_t>(bro[W], 8));
    allToAllV(c, bs, boff, br, bro, bm);
    std::vector<uint8_t> got(bro[W]);
    if (!got.empty()) HIP_OK(hipMemcpyAsync(got.data(), br, got.size(), hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    // 4. tables over the fetched rows (owner order, each owner's list order) + the row map
    struct ColOut { std::vector<uint8_t> val8, valid; std::vector<uint8_t> b; std::vector<uint64_t> soff; bool anyInvalid = false; };
    std::vector<std::vector<ColOut>> cols(g.tags.size());
    std::vector<std::vector<uint8_t>> present(g.tags.size(), std::vector<uint8_t>(nReq));
    for (size_t k = 0; k < g.tags.size(); k++) {
        cols[k].resize(g.tags[k].cols.size());
        for (size_t j = 0; j < g.tags[k].cols.size(); j++) {
            ColOut& co = cols[k][j];
            const int32_t ty = g.tags[k].cols[j].type;
            if (ty == T_BOOL) co.b.resize(nReq);
            else if (ty != T_STRING) co.val8.resize(nReq * 8);
            co.valid.resize(nReq);
            if (ty == T_STRING) co.soff.assign(nReq + 1, 0);
        }
    }
    std::string strBytes;
    uint64_t at = 0;
    for (int q = 0; q < W; q++) {
        const uint64_t n = m[static_cast<size_t>(me) * W + q];
        const uint8_t* blob = got.data() + bro[q];
        if (bro[q + 1] - bro[q] < n * rec) throw Error{NGX_E_DEVICE, "dst fetch: short reply"};
        const char* sbytes = reinterpret_cast<const char*>(blob + n * rec);
        uint64_t scur = 0;
        for (uint64_t i = 0; i < n; i++, at++) {
            const uint8_t* o = blob + i * rec;
            for (size_t k = 0; k < g.tags.size(); k++) {
                present[k][at] = *o++;
                for (size_t j = 0; j < g.tags[k].cols.size(); j++) {
                    ColOut& co = cols[k][j];
                    const int32_t ty = g.tags[k].cols[j].type;
                    if (ty == T_BOOL) co.b[at] = o[0];
                    else if (ty != T_STRING) std::memcpy(co.val8.data() + at * 8, o, 8);
                    co.valid[at] = o[8];
                    co.anyInvalid = co.anyInvalid || o[8] == 0;
                    o += 9;
                    if (ty == T_STRING) {
                        uint32_t len;
                        std::memcpy(&len, o, 4);
                        o += 4;
                        co.soff[at + 1] = len;                 // lengths now, offsets below
                        (void)scur;
                    }
                }
            }
        }
        // the owner appended each row's strings in (tag, column) order: re-cut them per column
        for (uint64_t i = 0, r0 = at - n; i < n; i++) {
            for (size_t k = 0; k < g.tags.size(); k++)
                for (size_t j = 0; j < g.tags[k].cols.size(); j++) {
                    ColOut& co = cols[k][j];
                    if (g.tags[k].cols[j].type != T_STRING) continue;
                    const uint64_t len = co.soff[r0 + i + 1];
                    if (sbytes + scur + len > reinterpret_cast<const char*>(blob) + (bro[q + 1] - bro[q]))
                        throw Error{NGX_E_DEVICE, "dst fetch: short string reply"};
                    co.b.insert(co.b.end(), sbytes + scur, sbytes + scur + len);     // (per column, row order)
                    scur += len;
                }
        }
    }
    // device layout: one allocation per record hop of the query; strings of every column in one block
    if (L.data.size() <= recIdx) {
        L.data.resize(recIdx + 1);
        L.hostStr.resize(recIdx + 1);
        L.devStr.resize(recIdx + 1, nullptr);
    }
    std::vector<uint8_t> img;
    auto put = [&](const void* src, uint64_t n) {
        const uint64_t o = (img.size() + 15) & ~uint64_t(15);
        img.resize(o + n);
        if (n) std::memcpy(img.data() + o, src, n);
        return o;
    };
    struct Pend { uint64_t present; std::vector<uint64_t> data, valid, soff; };
    std::vector<Pend> pend(g.tags.size());
    std::string& hs8 = L.hostStr[recIdx];
    hs8.clear();
    std::vector<std::vector<uint64_t>> strBase(g.tags.size());
    for (size_t k = 0; k < g.tags.size(); k++) {
        pend[k].present = put(present[k].data(), nReq);
        strBase[k].resize(g.tags[k].cols.size(), 0);
        for (size_t j = 0; j < g.tags[k].cols.size(); j++) {
            ColOut& co = cols[k][j];
            const int32_t ty = g.tags[k].cols[j].type;
            uint64_t dOff = ~0ULL, sOff = ~0ULL;
            if (ty == T_STRING) {
                for (uint64_t i = 0; i < nReq; i++) co.soff[i + 1] += co.soff[i];
                strBase[k][j] = hs8.size();
                hs8.append(reinterpret_cast<const char*>(co.b.data()), co.b.size());
                for (uint64_t i = 0; i <= nReq; i++) co.soff[i] += strBase[k][j];   // offsets into the block
                sOff = put(co.soff.data(), (nReq + 1) * 8);
            } else if (ty == T_BOOL) {
                dOff = put(co.b.data(), nReq);
            } else {
                dOff = put(co.val8.data(), nReq * 8);
            }
            pend[k].data.push_back(dOff);
            pend[k].soff.push_back(sOff);
            pend[k].valid.push_back(co.anyInvalid ? put(co.valid.data(), nReq) : ~0ULL);
        }
    }
    const uint64_t strOff = put(hs8.data(), hs8.size());
    // descriptors after the data
    std::vector<DTag> tagsOut;
    std::vector<DCol> colsOut;
    uint8_t* dev = L.data[recIdx].get<uint8_t>(img.size() + (g.tags.size() + 1) * sizeof(DTag) + (d.cols.size() + 64) * sizeof(DCol) + 64);
    for (size_t k = 0; k < g.tags.size(); k++) {
        DTag t = d.tags[k];
        t.present = dev + pend[k].present;
        t.colBase = static_cast<int32_t>(colsOut.size());
        tagsOut.push_back(t);
        for (size_t j = 0; j < g.tags[k].cols.size(); j++) {
            DCol dc{};
            dc.type = g.tags[k].cols[j].type;
            dc.width = 8;
            if (pend[k].data[j] != ~0ULL) dc.data = dev + pend[k].data[j];
            if (pend[k].soff[j] != ~0ULL) {
                dc.soff = reinterpret_cast<const uint64_t*>(dev + pend[k].soff[j]);
                dc.sbytes = reinterpret_cast<const char*>(dev + strOff);
            }
            if (pend[k].valid[j] != ~0ULL) dc.valid = dev + pend[k].valid[j];
            colsOut.push_back(dc);
        }
    }
    const uint64_t tOff = put(tagsOut.data(), tagsOut.size() * sizeof(DTag));
    const uint64_t cOff = put(colsOut.data(), colsOut.size() * sizeof(DCol));
    if (img.size() > L.data[recIdx].cap) throw Error{NGX_E_DEVICE, "dst fetch: table image larger than sized"};
    HIP_OK(hipMemcpyAsync(dev, img.data(), img.size(), hipMemcpyHostToDevice, c->stream));
    L.devStr[recIdx] = reinterpret_cast<const char*>(dev + strOff);
    // the map: global row of fetched row i = sb[q] + list offset
    std::vector<uint32_t> grow(nReq);
    {
        uint64_t i = 0;
        for (int q = 0; q < W; q++)
            for (uint64_t j = 0; j < m[static_cast<size_t>(me) * W + q]; j++, i++) grow[i] = static_cast<uint32_t>(sb[q] + myReq[i]);
    }
    uint32_t* drows = L.rows.get<uint32_t>(std::max<uint64_t>(nReq, 1));
    if (nReq) HIP_OK(hipMemcpyAsync(drows, grow.data(), nReq * 4, hipMemcpyHostToDevice, c->stream));
    uint32_t* map = L.map.get<uint32_t>(std::max<uint64_t>(d.vglobal, 1));
    if (launchScatterIndex(drows, nReq, map, c->stream)) throw Error{NGX_E_DEVICE, "dst map"};
    HIP_OK(hipStreamSynchronize(c->stream));                       // the host staging leaves scope
    c->dstFetches++;
    c->dstFetchRows += nReq;
    return DstFetch{reinterpret_cast<const DTag*>(dev + tOff), reinterpret_cast<const DCol*>(dev + cOff), map};
}

// multi-root walk at world > 1: the expansion OR-ed root sets into next[] over global rows; every
// shard sends peer q the sets of q's rows (next + sb[q], dense) and ORs what it receives into its own
// rows: out[i] = next[gbase + i] | the peers' sets of row i. Dense like the frontier bitmaps, 8 B per
// peer row: root walks serve pipes, whose frontiers are small next to a full GO's.
void exchangeRoots(ngx_ctx* c, const DeviceGraph& d, const uint64_t* next, uint64_t* out) {
    const int W = c->world;
    const auto& sb = d.shardBase;
    uint64_t maxRows = 1;
    for (int q = 0; q < W; q++) maxRows = std::max<uint64_t>(maxRows, sb[q + 1] - sb[q]);
    const uint64_t myRows = sb[c->rank + 1] - sb[c->rank];
    uint64_t* recv = c->rootRecv.get<uint64_t>(maxRows * W);
    uint64_t sent = 0;
    for (int q = 0; q < W; q++) if (q != c->rank) sent += (sb[q + 1] - sb[q]) * 8;
    c->lastXchgBytes += sent;
    if (c->xchg) {
        uint64_t* send = c->rootSend.get<uint64_t>(maxRows * W);      // equal blocks for the host collective
        for (int q = 0; q < W; q++) {
            const uint64_t nq = sb[q + 1] - sb[q];
            if (q != c->rank && nq)
                HIP_OK(hipMemcpyAsync(send + q * maxRows, next + sb[q], nq * 8, hipMemcpyDeviceToDevice, c->stream));
        }
        hostExchange(c, NGX_XCHG_ALLTOALL, send, recv, maxRows * 8);
    } else {
        NCCL_OK(ncclGroupStart());
        for (int q = 0; q < W; q++) {
            if (q == c->rank) continue;
            const uint64_t nq = sb[q + 1] - sb[q];
            if (nq) NCCL_OK(ncclSend(next + sb[q], nq * 8, ncclUint8, q, c->comm, c->stream));
            if (myRows) NCCL_OK(ncclRecv(recv + q * maxRows, myRows * 8, ncclUint8, q, c->comm, c->stream));
        }
        NCCL_OK(ncclGroupEnd());
        rcclWait(c, "root set all-to-all");
    }
    if (launchMergeRoots(next + d.gbase, recv, maxRows, myRows, W, c->rank, out, c->stream))
        throw Error{NGX_E_DEVICE, "merge roots"};
}

// grow a device buffer to `bytes`, keeping its first `keep` bytes
void growKeep(ngx_ctx* c, DBuf& b, size_t bytes, size_t keep) {
    bytes = std::max<size_t>(bytes, 64);
    if (b.cap >= bytes) return;
    if (keep == 0 || b.p == nullptr) { b.get<char>(bytes); return; }
    DBuf nb;
    nb.get<char>(bytes);
    HIP_OK(hipMemcpyAsync(nb.p, b.p, keep, hipMemcpyDeviceToDevice, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    b.release();
    b = nb;
}

// the final kernel's look-back words: ticket / row counter, one status per chunk, the done counter
// (chunks + 2 words); zeroed by the hop's k_chunk_first launch
uint64_t lookBackWords(uint64_t chunks) { return chunks + 2; }
uint64_t* lookBack(ngx_ctx* c, uint64_t chunks) { return c->lbStatus.get<uint64_t>(lookBackWords(chunks)); }
// the GO final hop's block tables (kargs.h kResv*): entries carry the launch's tag, so the table is
// cleared only when it is (re)allocated
// reservation geometry (kargs.h resv*) and the counters, cleared once here and then by every k_final_close.
// Measured at C2 (final hop / close, us): 8 groups x 8 K-row blocks 765 / 34 (chunks wait on block
// allocations), 8 x 32 K 346 / 15, 8 x 64 K 325 / 15, 8 x 128 K 320 / 18, 16 x 32 K 326 / 24, 32 x 8 K
// 347 / 83, 64 x 4 K 339 / 193 (the close kernel moves up to G blocks of rows)
void resvGeometry(ngx_ctx* c, FinalArgs& a) {
    a.resvG = c->resvGroups;
    a.resvShift = kResvShift;
    a.resvStride = 32;                                          // counters 256 B apart
    // two sets of counters: a launch uses one and its k_final_close clears the other for the next
    const uint64_t words = (a.resvG + 2) * static_cast<uint64_t>(a.resvStride);
    if (c->resvCtl.cap < 2 * words * 8 || c->resvCtl.p == nullptr || c->resvLastG != a.resvG ||
        c->resvLastStride != a.resvStride) {
        c->resvCtl.get<uint64_t>(2 * words);
        HIP_OK(hipMemsetAsync(c->resvCtl.p, 0, c->resvCtl.cap, c->stream));
        c->resvParity = 0;
    }
    uint64_t* base = static_cast<uint64_t*>(c->resvCtl.p);
    a.resvCtl = base + c->resvParity * words;
    a.resvNext = base + (1 - c->resvParity) * words;
    // a query that bailed out between the last hand-out and its k_final_close (string-arena limit, a
    // throw) left this set uncleared: clear it here instead
    if (c->resvClosePending) HIP_OK(hipMemsetAsync(a.resvCtl, 0, words * 8, c->stream));
    c->resvClosePending = true;                                 // until launchFinalClose is enqueued
    c->resvParity ^= 1;
    c->resvLastG = a.resvG;
    c->resvLastStride = a.resvStride;
}
// the frontier bitmap's zero state (ngx_ctx::bitsClean): `bits` is one of the context's bitmaps
static uint64_t bitsGen(const ngx_ctx* c, const void* bits) {
    return bits == c->frontierBits.p ? c->frontierBits.gen : bits == c->localBits.p ? c->localBits.gen : 0;
}
bool bitsKnownZero(const ngx_ctx* c, const void* bits, uint64_t words) {
    return c->bitsClean && bits != nullptr && c->bitsCleanPtr == bits && c->bitsCleanGen == bitsGen(c, bits) &&
           c->bitsCleanGen != 0 && c->bitsCleanWords >= words;
}
void markBitsZero(ngx_ctx* c, const void* bits, uint64_t words) {
    c->bitsClean = true;
    c->bitsCleanPtr = bits;
    c->bitsCleanGen = bitsGen(c, bits);
    c->bitsCleanWords = words;
}
uint64_t* resvTable(ngx_ctx* c, uint64_t words) {
    if (c->resvTabWords < words || c->resvTab.p == nullptr) {
        c->resvTab.get<uint64_t>(words);
        HIP_OK(hipMemsetAsync(c->resvTab.p, 0, c->resvTab.cap, c->stream));
        c->resvTabWords = c->resvTab.cap / 8;
    }
    return static_cast<uint64_t*>(c->resvTab.p);
}

// YIELD columns that are exactly an edge key prop of every edge the hop expands (`e._dst`,
// `e._src`, `e._rank` of the only OVER type, typed INT/VID): their cells equal the oSrc/oDst/oRank
// row, so the column aliases that array instead of storing the same 8 B per row again.
std::vector<int32_t> keyAliases(const Programs& progs, const std::vector<int32_t>& colTypes, const HopSlots& hs) {
    std::vector<int32_t> k(progs.yOff.size(), -1);
    for (size_t y = 0; y < progs.yOff.size(); y++) {
        const Insn* code = progs.code.data() + progs.yOff[y];
        int32_t ct = y < colTypes.size() ? colTypes[y] : T_UNKNOWN;
        if (code[1].op != OP_END || !(ct == T_INT || ct == T_VID || ct == T_TIMESTAMP)) continue;
        int32_t key = code[0].op == OP_EDST ? 1 : (code[0].op == OP_EKEY && code[0].a >= 0 && code[0].a <= 2) ? code[0].a : -1;
        if (key < 0) continue;
        bool all = true;
        for (int s = 0; s < hs.n; s++) all = all && (code[0].b == 0 || std::abs(hs.etype[s]) == code[0].b);
        if (all) k[y] = key;
    }
    return k;
}

// size the result columns for `cap` rows (keeping `keep`) and upload their descriptors; aliased
// key columns (keyAliases) point at oSrc/oDst/oRank, which must already be sized
void prepareCols(ngx_ctx* c, FinalArgs& a, const std::vector<ColSpec>& spec, uint64_t cap, uint64_t keep,
                 const std::vector<int32_t>& alias = {}, const std::vector<int32_t>* widths = nullptr,
                 bool rankConst = false) {
    if (c->oCols.size() < spec.size()) c->oCols.resize(spec.size());
    c->oColView.assign(spec.size(), OutCol{nullptr, nullptr, nullptr, 8, 0});
    for (size_t y = 0; widths && y < spec.size() && y < widths->size(); y++) c->oColView[y].w = (*widths)[y];
    for (size_t y = 0; y < spec.size(); y++) {
        auto& cb = c->oCols[y];
        if (y < alias.size() && alias[y] >= 0) {
            DBuf& kb = alias[y] == 0 ? c->oSrc : alias[y] == 1 ? c->oDst : c->oRank;
            // a constant rank is stored nowhere (the kernels skip a column without an array)
            c->oColView[y].x = (alias[y] == 2 && rankConst) ? nullptr : static_cast<int64_t*>(kb.p);
            continue;
        }
        growKeep(c, cb.x, cap * 8, keep * 8);
        c->oColView[y].x = static_cast<int64_t*>(cb.x.p);
        if (spec[y].len) { growKeep(c, cb.len, cap * 4, keep * 4); c->oColView[y].len = static_cast<uint32_t*>(cb.len.p); }
        if (spec[y].t) { growKeep(c, cb.t, cap, keep); c->oColView[y].t = static_cast<uint8_t*>(cb.t.p); }
    }
    // the first kInlineCols descriptors travel in the kernel arguments; only wider results upload a table
    for (size_t y = 0; y < spec.size() && y < static_cast<size_t>(kInlineCols); y++) a.oColsIn[y] = c->oColView[y];
    a.oCols = nullptr;
    if (spec.size() > static_cast<size_t>(kInlineCols)) {
        OutCol* dev = c->oColDesc.get<OutCol>(spec.size());
        HIP_OK(hipMemcpyAsync(dev, c->oColView.data(), spec.size() * sizeof(OutCol), hipMemcpyHostToDevice, c->stream));
        a.oCols = dev;
    }
}

// result columns rows [first, first + n) -> host OutCells (row-major); a typed column's rows carry its static type
// device arrays -> the context's page-locked staging, one synchronisation. Small batches go through one
// copy kernel storing into the mapped staging: each DMA copy costs ~8 us of latency, which made a
// GetNeighbors response's dozen arrays take 166 us (tools/gn_trace.py). Large batches use the DMA
// engine (57 GB/s vs 55 GB/s for the kernel, tools/mb_d2h.hip, and the CUs stay free);
struct HostArr { const void* dev; size_t bytes; char* host; };
void stageArrays(ngx_ctx* c, std::vector<HostArr>& arrs) {
    constexpr size_t kKernelCopyMax = size_t(32) << 20;
    size_t total = 0;
    for (auto& a : arrs) total += (a.bytes + 63) & ~size_t(63);
    char* stage = c->hostStage.get(std::max<size_t>(total, 64));
    const bool useKernel = total <= kKernelCopyMax;
    char* stageDev = nullptr;
    if (useKernel && hipHostGetDevicePointer(reinterpret_cast<void**>(&stageDev), c->hostStage.p, 0) != hipSuccess)
        stageDev = nullptr;
    CopyBatch cb{};
    for (auto& a : arrs) {
        const size_t at = stage - static_cast<char*>(c->hostStage.p);
        a.host = stage;
        stage += (a.bytes + 63) & ~size_t(63);
        if (!a.bytes) continue;
        if (stageDev == nullptr) {
            HIP_OK(hipMemcpyAsync(a.host, a.dev, a.bytes, hipMemcpyDeviceToHost, c->stream));
            continue;
        }
        if (cb.n == kMaxCopies) {
            if (launchCopyBatch(cb, c->stream)) throw Error{NGX_E_DEVICE, "copy to host"};
            cb = CopyBatch{};
        }
        cb.src[cb.n] = static_cast<const uint8_t*>(a.dev);
        cb.dst[cb.n] = reinterpret_cast<uint8_t*>(stageDev + at);
        cb.bytes[cb.n] = a.bytes;
        cb.start[cb.n + 1] = cb.start[cb.n] + (a.bytes + 15) / 16;
        cb.n++;
    }
    if (cb.n && launchCopyBatch(cb, c->stream)) throw Error{NGX_E_DEVICE, "copy to host"};
    HIP_OK(hipStreamSynchronize(c->stream));
}

// the result columns (and `extra` device arrays, staged alongside: their host copies come back in
// extra[i].host), read in place from the page-locked staging as raw typed cells
struct StagedCells {
    std::vector<const int64_t*> x;
    std::vector<const uint32_t*> len;
    std::vector<const uint8_t*> t;
    std::vector<uint8_t> st;                                     // value type of a column without types
    OutCell at(uint64_t r, size_t y) const {
        OutCell o;
        o.x = x[y][r];
        o.len = len[y] ? len[y][r] : 0;
        o.t = t[y] ? t[y][r] : st[y];
        return o;
    }
};
StagedCells stageCells(ngx_ctx* c, const std::vector<ColSpec>& spec, const std::vector<int32_t>& colTypes,
                       uint64_t n, uint64_t first, std::vector<HostArr>& extra) {
    size_t nY = spec.size();
    std::vector<HostArr> arrs(extra);
    std::vector<size_t> iX(nY, SIZE_MAX), iLen(nY, SIZE_MAX), iT(nY, SIZE_MAX);
    for (size_t y = 0; y < nY && n; y++) {
        const OutCol& v = c->oColView[y];
        iX[y] = arrs.size(); arrs.push_back(HostArr{v.x + first, n * 8, nullptr});
        if (v.len) { iLen[y] = arrs.size(); arrs.push_back(HostArr{v.len + first, n * 4, nullptr}); }
        if (v.t) { iT[y] = arrs.size(); arrs.push_back(HostArr{v.t + first, n, nullptr}); }
    }
    stageArrays(c, arrs);
    for (size_t i = 0; i < extra.size(); i++) extra[i].host = arrs[i].host;
    StagedCells sc;
    for (size_t y = 0; y < nY && n; y++) {
        sc.x.push_back(reinterpret_cast<const int64_t*>(arrs[iX[y]].host));
        sc.len.push_back(iLen[y] == SIZE_MAX ? nullptr : reinterpret_cast<const uint32_t*>(arrs[iLen[y]].host));
        sc.t.push_back(iT[y] == SIZE_MAX ? nullptr : reinterpret_cast<const uint8_t*>(arrs[iT[y]].host));
        uint8_t st = V_ERR;
        switch (y < colTypes.size() ? colTypes[y] : T_UNKNOWN) {
            case T_BOOL: st = V_BOOL; break;
            case T_INT: case T_VID: case T_TIMESTAMP: st = V_INT; break;
            case T_FLOAT: case T_DOUBLE: st = V_DBL; break;
            case T_STRING: st = V_STR; break;
            default: break;
        }
        sc.st.push_back(st);
    }
    return sc;
}

// the hop's side of a generated final-hop kernel's shape: slots, widths, TTL, programs
JitQuery jitHopQuery(const Space& sp, const HopSlots& hs, const Programs& progs) {
    JitQuery jq;
    jq.oneSlot = hs.n == 1;
    jq.pos32 = true;
    for (int s = 0; s < hs.n; s++) jq.pos32 = jq.pos32 && sp.host->slots[hs.slotIdx[s]].dst.size() < (1ULL << 32);
    jq.P = JitProgram{progs.P >= 0 ? progs.code.data() + progs.P : nullptr, progs.P >= 0};
    jq.W = JitProgram{progs.W >= 0 ? progs.code.data() + progs.W : nullptr, progs.W >= 0};
    for (int32_t off : progs.yOff) jq.Y.push_back(JitProgram{progs.code.data() + off, true});
    for (int s = 0; s < hs.n; s++) {
        jq.slots.push_back(hs.slotIdx[s]);
        int32_t tc;
        int64_t td;
        jq.ttl = jq.ttl || ttlInfo(sp.edge(std::abs(hs.etype[s])), tc, td);
    }
    jq.etype0 = hs.n == 1 ? hs.etype[0] : 0;
    jq.dstW = hs.n ? hs.dstW[0] : 0;
    jq.rankW = hs.n ? hs.rankW[0] : 0;
    jq.rankConst = hs.n > 0;
    for (int s = 0; s < hs.n; s++) {
        if (hs.dstW[s] != jq.dstW) jq.dstW = 0;
        if (hs.rankW[s] != jq.rankW) jq.rankW = 0;
        jq.rankConst = jq.rankConst && hs.rank[s] == nullptr;
    }
    if (!jq.rankConst) {                                      // a rank column somewhere: widths per slot
        for (int s = 0; s < hs.n; s++) if (hs.rank[s] == nullptr) jq.rankW = 0;
    }
    return jq;
}

// literals -> launch-time constant slots (one kernel per query shape)
void jitSlotConsts(JitQuery& jq, std::vector<int64_t>& kc, std::vector<uint32_t>& kl) {
    auto slotConsts = [&](const Insn* code) {
        for (const Insn* in = code; in && in->op != OP_END; in++) {
            if (in->op != OP_PUSH || static_cast<int>(kc.size()) >= kJitConsts) continue;
            jq.constSlot[in] = static_cast<int32_t>(kc.size());
            kc.push_back(in->imm);
            kl.push_back(static_cast<uint32_t>(in->a));
        }
    };
    if (jq.P.present) slotConsts(jq.P.code);
    if (jq.W.present) slotConsts(jq.W.code);
    for (auto& y : jq.Y) slotConsts(y.code);
}

// A multi-root walk (runPipe): the sentence from every start at once, each frontier row carrying the
// bitmask of the starts (roots, at most 64) that reach it — GoExecutor's VertexBackTracker
// (GoExecutor.h:189-207) — so that every record hop's rows can be attributed to their roots
// (getRoots, GoExecutor.cpp:1317-1330). World 1, push hops, no storage mask (the caller walks per
// root otherwise: runGo fails such a walk with NGX_E_UNSUPPORTED before any row).
struct RootWalk {
    std::unordered_map<int64_t, uint64_t> bitsOf;              // start vid -> its root bit
    // WHERE / YIELD read $-.x: every record hop's entries are (frontier row, input row) pairs, one per
    // input row of each root reaching the row, and the programs read the row's columns (OP_INPUT)
    bool perRow = false;
    const std::vector<std::vector<uint32_t>>* rowsOfBit = nullptr;   // root bit -> its input rows
    const DInputCol* input = nullptr;                          // the input table on the device
    uint64_t inStrDev = 0, inStrBytes = 0;                     // its string pool (device) ...
    const char* inStrHost = nullptr;                           // ... and the same bytes on the host
    struct Hop { uint64_t rowBase = 0, rows = 0; std::unordered_map<int64_t, uint64_t> rootsOf; };
    std::vector<Hop> record;                                   // per record hop: src vid -> roots
};

// FLAGS_enable_reservoir_sampling: storage keeps a random sample of each vertex's edges
// (QueryBoundProcessor::processEdgeSampling, QueryBoundProcessor.cpp:83-164, chosen at :213; the cap
// stops applying in collectEdgeProps, QueryBaseProcessor.inl:502). A random sample has no bit-exact
// device counterpart, so requests under the flag go to the reference's CPU path.
const char* const kSamplingRefused =
    "enable_reservoir_sampling: edges are sampled at random by the CPU path (QueryBoundProcessor::processEdgeSampling)";

int32_t runGo(ngx_ctx* c, Space& sp, const ngx_go_plan& p, GoResultHolder& R, const InputBind* in = nullptr,
              RootWalk* rw = nullptr) {
    c->hmark("in");
    RoctxRange queryRange("ngx_go");
    DeviceGraph& d = *sp.dev;
    c->resvRows = nullptr;                                       // set by this query's final launches only
    const int64_t now = p.now_sec > 0 ? p.now_sec : static_cast<int64_t>(std::time(nullptr));   // WallClock
    GoPlan gp;
    int32_t rc = prepareGo(c, sp, p, gp, in);
    if (rc) return rc;
    c->hmark("prep");
    R.colTypes = gp.colTypes;
    uint32_t recordFrom = p.record_from, steps = p.record_to;
    if (steps == 0) return NGX_OK;                               // GoExecutor.cpp:99-104
    if (recordFrom == 0) recordFrom = 1;

    // ---- final-hop request (getStepOutProps for record hops)
    GraphdCtx gctx;
    gctx.sp = &sp;
    gctx.deviceLibm = c->deviceLibm;
    if (rw && rw->perRow && in) gctx.inputCols = &in->colIdx;
    gctx.aliasType = gp.aliasType;
    gctx.direction = p.direction;
    gctx.nEdgeTypes = gp.edgeTypes.size();
    for (auto& ap : gp.refs.alias) {
        if (ap.second == "_dst") continue;
        int32_t t = gp.aliasType.at(ap.first);
        int32_t ptype = (ap.second == "_src") ? T_VID : (ap.second == "_rank" || ap.second == "_type") ? T_INT
                      : sp.edge(t)->latest().typeOf(ap.second);
        std::vector<int32_t> signedTypes;
        if (p.direction == NGX_DIR_FORWARD) signedTypes = {t};
        else if (p.direction == NGX_DIR_REVERSELY) signedTypes = {-t};
        else signedTypes = {t, -t};
        for (int32_t st : signedTypes) gctx.respSchema[st][ap.second] = ptype;
    }
    StorageCtx sctx;
    sctx.sp = &sp;
    sctx.deviceLibm = c->deviceLibm;
    sctx.haveEdgeContexts = true;
    for (int32_t t : gp.edgeTypes) {
        const SchemaSet* es = sp.edge(std::abs(t));
        if (es) sctx.edgeMap[es->name] = std::abs(t);
    }
    Programs progs;
    std::string err;
    bool pushHere = p.filter_pushdown && p.direction == NGX_DIR_FORWARD && gp.pushed;
    bool pushInvalid = false;
    if (pushHere) {
        Program pp;
        int32_t crc = compileStorage(*gp.pushed, sctx, pp, err);
        if (crc == NGX_E_INVALID_FILTER) {
            // every part of the final-hop request fails (E_INVALID_FILTER), but only if that request is
            // issued: a frontier that empties earlier ends the query with no rows (GoExecutor.cpp:580-606)
            pushInvalid = true;
            pushHere = false;
        } else if (crc) {
            return fail(c, crc, err);
        } else {
            // a $^ tag referenced only by the filter: every src tag prop of WHERE/YIELD is requested too
            progs.P = progs.add(pp);
        }
    }
    if (gp.where) {
        Program wp;
        int32_t crc = compileGraphd(*gp.where, gctx, wp, err);
        if (crc) return fail(c, crc, err);
        progs.W = progs.add(wp);
    }
    for (auto& y : gp.yields) {
        Program yp;
        int32_t crc = compileGraphd(*y, gctx, yp, err);
        if (crc) return fail(c, crc, err);
        progs.yOff.push_back(progs.add(yp));
    }
    // YIELD columns that build strings keep them in the result string arena (one slot per row)
    uint32_t strOutMask = 0;
    for (size_t y = 0; y < progs.yOff.size(); y++) {
        if (!strBuffersOf(progs.code.data() + progs.yOff[y])) continue;
        if (y >= 32) return fail(c, NGX_E_UNSUPPORTED, "a YIELD column past the 32nd that builds strings");
        strOutMask |= 1u << y;
    }
    const uint32_t nStrOut = static_cast<uint32_t>(__builtin_popcount(strOutMask));
    struct Arena { const char* dev; uint64_t rows; };
    std::vector<Arena> arenas;                                   // this query's, in record-hop order
    // $$ props: tag tables over every global row (world > 1: replicas of the other shards' rows)
    const bool dstReplica = progs.usesDst && c->world > 1;
    // owner fetch per record hop, or replicas over every global row (flag dst_props; by size: the replicas
    // while every shard's tag data would take at most dstReplicaMax bytes on each shard)
    bool ownerDst = false;
    if (dstReplica) {
        uint64_t local = 0;
        for (const HostTag& t : sp.host->tags) {
            local += t.present.size();
            for (const HostColumn& col : t.cols) local += t.present.size() * 9 + col.sbytes.size();
        }
        ownerDst = c->dstProps == 1 ||
                   (c->dstProps < 0 && !d.replicas && local * static_cast<uint64_t>(c->world) > c->dstReplicaMax);
    }
    if (dstReplica && !ownerDst) ensureDstReplicas(c, sp);
    size_t dstRec = 0;                                           // record hops fetched so far (owner fetch)
    const DTag* dstTags = dstReplica ? d.rtags : d.dtags;
    const DCol* dstCols = dstReplica ? d.rcols : d.dcols;
    std::vector<int32_t> ySlotType(progs.yOff.size(), 0);
    c->hmark("compile");
    // WHERE fully pushed: for edges whose storage filter ran, graphd's re-evaluation is implied
    bool wIsP = pushHere && gp.where && encodeExpr(*gp.pushed) == encodeExpr(*gp.where);
    std::vector<int32_t> hopTypes;
    HopSlots hs = makeHopSlots(sp, d, gp.edgeTypes, hopTypes);
    // one OVER type: every row's type is hs.etype[0], so the final hop writes no per-row type column
    const bool constType = hs.n == 1;
    const std::vector<int32_t> yAlias = keyAliases(progs, gp.colTypes, hs);
    // yield_only: the row arrays no YIELD column aliases are not written (bit k: src, dst, rank)
    int32_t rowMask = 7;
    if (p.yield_only && p.result_on_device && !p.distinct) {
        rowMask = 0;
        for (int32_t al : yAlias) if (al >= 0) rowMask |= 1 << al;
    }
    // compact results (plan.compact_results): the row arrays at the width of the stored key columns
    // (src: of the shard's vid table), and a YIELD column that copies one stored integer column of the
    // only OVER type, present in every row, at that column's width; every other column at 8 bytes
    const bool compact = p.compact_results && p.result_on_device && !p.distinct && rw == nullptr;
    // compact results over slots whose every rank is one value (no rank column in HBM, HopSlots::rankC):
    // the rank is a constant column of the result (width 0), no byte per row
    bool rankConst = compact && hs.n > 0;
    for (int s = 0; rankConst && s < hs.n; s++)
        rankConst = hs.rank[s] == nullptr && hs.rankC[s] == hs.rankC[0];
    if (rankConst) rowMask &= ~4;
    int32_t outW[3] = {8, 8, 8};
    std::vector<int32_t> yW(progs.yOff.size(), 8);
    if (compact) {
        outW[0] = d.vidW;
        outW[1] = outW[2] = 1;
        for (int s = 0; s < hs.n; s++) {
            outW[1] = std::max<int32_t>(outW[1], hs.dstW[s]);
            outW[2] = std::max<int32_t>(outW[2], hs.rankW[s]);
        }
        for (size_t y = 0; y < progs.yOff.size(); y++) {
            const Insn* code = progs.code.data() + progs.yOff[y];
            const int32_t ct = y < gp.colTypes.size() ? gp.colTypes[y] : T_UNKNOWN;
            // an aliased key column is the row array itself, at its width, whatever the slots
            if (y < yAlias.size() && yAlias[y] >= 0) { yW[y] = outW[yAlias[y]]; continue; }
            if (hs.n != 1) continue;
            if (code[0].op != OP_ECOL || code[1].op != OP_END || code[0].b != std::abs(hs.etype[0])) continue;
            if (!(ct == T_INT || ct == T_VID || ct == T_TIMESTAMP)) continue;
            const HostSlot& hsl = sp.host->slots[hs.slotIdx[0]];
            if (code[0].a < 0 || code[0].a >= static_cast<int32_t>(hsl.cols.size())) continue;
            const auto& col = hsl.cols[code[0].a];
            if (!col.allValid || !(col.type == T_INT || col.type == T_VID || col.type == T_TIMESTAMP)) continue;
            if (col.width == 1 || col.width == 2 || col.width == 4) yW[y] = col.width;
        }
    }
    // algorithmic-byte model inputs: k_f prop columns read by the filter, k_y yielded
    uint64_t ky = 0, kfBytes = 0;
    {
        PropRefs wr, yr;
        if (gp.where) collectRefs(*gp.where, wr);
        for (auto& y : gp.yields) collectRefs(*y, yr);
        auto count = [](const PropRefs& r) {
            uint64_t n = 0;
            for (auto& ap : r.alias) n += (ap.second != "_src" && ap.second != "_dst" && ap.second != "_rank" && ap.second != "_type");
            return n + r.srcTag.size() + r.dstTag.size();
        };
        ky = count(yr);
        // 8 logical bytes per edge for each filter edge prop (§8d), whatever width it is stored at;
        // compact results count every integer column at its stored width (the bytes this layout reads)
        auto storedWidth = [&](const std::string& alias, const std::string& prop) -> uint64_t {
            auto at = gp.aliasType.find(alias);
            const SchemaSet* es = at == gp.aliasType.end() ? nullptr : sp.edge(at->second);
            const int32_t col = es ? es->latest().index(prop) : -1;
            int32_t w = 0;
            for (int s = 0; col >= 0 && s < hs.n; s++) {
                if (std::abs(hs.etype[s]) != at->second) continue;
                const auto& cols = sp.host->slots[hs.slotIdx[s]].cols;
                const int32_t t = col < static_cast<int32_t>(cols.size()) ? cols[col].type : T_UNKNOWN;
                w = std::max<int32_t>(w, (t == T_INT || t == T_VID || t == T_TIMESTAMP) ? cols[col].width
                                         : t == T_BOOL ? 1 : 8);
            }
            return w > 0 ? static_cast<uint64_t>(w) : 8u;
        };
        for (auto& ap : wr.alias) {
            if (ap.second == "_src" || ap.second == "_dst" || ap.second == "_rank" || ap.second == "_type") continue;
            kfBytes += compact ? storedWidth(ap.first, ap.second) : 8;
        }
        kfBytes += 8 * (wr.srcTag.size() + wr.dstTag.size());
    }
    // per scanned edge: dst + rank (8 B each in §8d; compact: their stored widths) + the filter props
    const uint64_t keyReadBytes = compact ? static_cast<uint64_t>(outW[1] + (rankConst ? 0 : outW[2])) : 16u;
    // bytes written per passing edge: the row arrays and the k_y yielded props, 8 B each (§8d); compact
    // results count each at the width it is written at
    uint64_t rowBytes = 0;
    for (int k = 0; k < 3; k++) rowBytes += (rowMask >> k & 1) ? (compact ? outW[k] : 8) : 0;
    if (compact) {
        uint64_t stored = 0, storedBytes = 0;
        for (size_t y = 0; y < yW.size(); y++) {
            if (y < yAlias.size() && yAlias[y] >= 0) continue;
            stored++;
            storedBytes += yW[y];
        }
        rowBytes += storedBytes + 8 * (ky > stored ? ky - stored : 0);
    } else {
        rowBytes += 8 * ky;
    }

    // ---- seeds (starts_), routed by ID_HASH; duplicates kept unless DISTINCT (:123-129)
    std::vector<int64_t> starts(p.starts, p.starts + p.nstarts);
    if (p.distinct) {
        std::unordered_set<int64_t> u(starts.begin(), starts.end());
        starts.assign(u.begin(), u.end());
    }
    std::vector<int32_t> sparts;
    std::vector<int64_t> svids;
    for (int64_t v : starts) {
        int32_t part = idHash(v, sp.numParts);
        if (c->world > 1 && part % c->world != c->rank) continue;
        sparts.push_back(part);
        svids.push_back(v);
    }
    // marks over global rows: [0, vAl) the push expansion's (and the exchange's), [vAl, 2 vAl) a pull
    // hop's output, so a pull never overwrites the frontier marks it reads; one epoch counter for both
    const uint64_t vAl = (d.vglobal + 15) & ~15ULL;
    ensureVisited(c, 2 * vAl);
    uint8_t* const marksA = c->visited.get<uint8_t>(2 * vAl);
    PullArgs pa{};                                              // pull expansion (kernels.h launchPull)
    // world > 1: every shard pulls its own rows against the all-gathered frontier bitmap; the mirrors
    // and the decision are global (findMirrorsGlobal, one all-gather per intermediate hop). pullGather:
    // whether the shards hold that per-hop all-gather, from values every shard has alike (the query,
    // the world), so all of them enter it; what a shard itself can do (its rows, limits, flags) travels
    // inside it
    const bool pullGather = c->world > 1 && !rw && hs.n >= 1 && hs.n <= kPullMaxSlots && d.vglobal < (1ULL << 31) &&
                            c->world <= kMaxWorld;
    bool pullable = !rw && c->pullFactor > 0 && (c->world == 1 || (d.vglobal < (1ULL << 31) && c->world <= kMaxWorld)) &&
                    hs.n >= 1 && hs.n <= kPullMaxSlots && d.V < (1ULL << 32) && d.mirror.size() == d.slots.size();
    if (pullable) {
        uint64_t inEdges = 0, longRows = 0, slices = 0;
        pa.n = hs.n;
        for (int s = 0; s < hs.n && pullable; s++) {
            const int32_t m = d.mirror[hs.slotIdx[s]];
            if (m < 0 || d.pullHead.size() != d.slots.size() || !d.pullHead[hs.slotIdx[s]].perm) { pullable = false; break; }
            const DeviceGraph::PullHead& ph = d.pullHead[hs.slotIdx[s]];
            pa.ioff[s] = d.slots[m].off;
            pa.isrc[s] = d.slots[m].dgid;
            pa.perm[s] = ph.perm;
            pa.head[s] = ph.head;
            pa.nk[s] = ph.nk;
            slices += ph.slices;
            pa.sliceEnd[s] = slices;
            longRows += ph.longRows;
            inEdges += sp.host->slots[m].dst.size();
        }
        if (pullable) {
            pa.segCap = longRows + inEdges / kPullSeg + 1;
            if (c->pullSegWords < pa.segCap) {
                c->pullSeg.get<uint64_t>(pa.segCap);
                HIP_OK(hipMemsetAsync(c->pullSeg.p, 0, c->pullSeg.cap, c->stream));
                c->pullSegWords = c->pullSeg.cap / 8;
            }
            if (!c->pullCtl.p) {
                c->pullCtl.get<uint32_t>(16);
                HIP_OK(hipMemsetAsync(c->pullCtl.p, 0, c->pullCtl.cap, c->stream));
            }
            pa.seg = static_cast<uint64_t*>(c->pullSeg.p);
            pa.ctl = static_cast<uint32_t*>(c->pullCtl.p);
            pa.V = d.V;
        }
    }
    // the compaction after an intermediate hop also writes the next hop's estart[] and E (fused
    // scan) when the packed (|F|, E) total fits; the slot totals bound E
    uint64_t slotEdges = 0;
    bool pos32 = true;                                         // every CSR position fits 32 bits
    for (int s = 0; s < hs.n; s++) {
        uint64_t es = sp.host->slots[hs.slotIdx[s]].dst.size();
        slotEdges += es;
        pos32 = pos32 && es < (1ULL << 32);
    }
    const bool fuseDeg = d.V < (1ULL << (64 - kFdShift)) && slotEdges <= kFdMask && hs.n > 0;
    // single-pass compaction (k_compact_lb): the next hop's chunk heads come with its estart; every
    // hop after the seed hop has unique frontier rows, so E <= slotEdges bounds chunkFirst
    const bool lbCompact = fuseDeg && d.V < kCompactLbMaxV;
    const uint64_t cfCap = slotEdges / kChunk + 2;
    c->chunkFirst.get<uint64_t>(cfCap);
    // compaction tile / wave totals (kernels.h CompactArgs)
    uint64_t* cmpTile = nullptr;
    uint64_t* cmpWave = nullptr;
    if (lbCompact) {
        const uint64_t tiles = (d.V + kCompactTile - 1) / kCompactTile + 1;
        cmpTile = c->cmpStatus[0].get<uint64_t>(tiles);
        cmpWave = c->cmpStatus[1].get<uint64_t>(tiles * (kCompactTile / 256));   // a word per wave (up to 16 per tile)
    }
    // the pull reads the frontier as a bitmap over global rows, written by the compaction that built it
    // (or from the frontier list for the seed frontier); the pull's segment counter is cleared by the
    // compaction after it
    if (!lbCompact) pullable = false;
    // sparse hops: one shard (its rows are the global rows), the frontier bitmap as the dedup set
    const bool sparseOk = c->world == 1 && lbCompact && !rw && c->sparseFactor != 0 && hs.n > 0 && d.gbase == 0 &&
                          d.vglobal == d.V && d.V < (1ULL << 32);
    uint64_t* fbits = (pullable || sparseOk) ? c->frontierBits.get<uint64_t>(vAl / 64 + 1) : nullptr;
    if (sparseOk) {
        // both sets of entry arrays at full size now: no buffer a kernel of this query reads is regrown later
        const uint64_t n = d.V * static_cast<uint64_t>(hs.n) + 1;
        c->estart.get<uint64_t>(n);
        c->estart2.get<uint64_t>(n);
        c->ebase.get<uint64_t>(n);
        c->ebase2.get<uint64_t>(n);
        c->chunkFirst2.get<uint64_t>(cfCap);
    }
    // world > 1: the compaction writes this shard's bitmap (local rows), gathered into fbits when a hop
    // pulls; segWords = the largest shard's words (the all-gather block)
    uint64_t segWords = 0;
    for (int q = 0; q + 1 < static_cast<int>(d.shardBase.size()); q++)
        segWords = std::max<uint64_t>(segWords, (d.shardBase[q + 1] - d.shardBase[q] + 63) / 64);
    uint64_t* lbits = (pullable && c->world > 1) ? c->localBits.get<uint64_t>(std::max<uint64_t>(segWords, 1)) : fbits;
    bool haveBits = false;
    pa.curBits = fbits;
    // storage-side request of each hop (getStepOutProps): props only on record hops, TTL info always
    uint32_t recordPropsMask = 0, ttlMask = 0;
    int32_t ttlCol[kMaxSlots];
    int64_t ttlDur[kMaxSlots];
    for (int s = 0; s < hs.n; s++) {
        if (gctx.respSchema.count(hs.etype[s]) && !gctx.respSchema[hs.etype[s]].empty()) recordPropsMask |= 1u << s;
        if (ttlInfo(sp.edge(std::abs(hs.etype[s])), ttlCol[s], ttlDur[s])) ttlMask |= 1u << s;
    }
    const int64_t edgeCap = c->maxEdgesPerVertex;              // FLAGS_max_edge_returned_per_vertex
    const bool capped = edgeCap < INT32_MAX;
    // Device-driven hops: every kernel reads the frontier size and E that the previous kernel wrote
    // (dynStats), grids are upper bounds striding over the real work, pull-or-push is decided on the
    // device; the host enqueues the whole query without waiting (no round trip per hop) and reads the
    // hop totals once at the end. Single shard, fused seed hop, one record hop, no storage mask.
    bool intermediateChecks = false;
    for (int s = 0; s < hs.n; s++) {
        if ((ttlMask >> s & 1u) && (hs.eflags[s] != nullptr || ttlCol[s] >= 0)) intermediateChecks = true;
    }
    if (rw && c->world > 1) {
        // a root walk cannot run over a storage mask (below); at world > 1 the shards agree on that
        // before the first exchange, so all of them fall back together (a shard's rows decide whether
        // its slots carry flags)
        bool maskPossible = capped;
        const uint32_t checked = ttlMask | (recordFrom < steps ? recordPropsMask : 0u);
        for (int s = 0; s < hs.n; s++)
            if ((checked >> s & 1u) && (hs.eflags[s] != nullptr || ttlCol[s] >= 0)) maskPossible = true;
        const uint64_t mine = maskPossible ? 1 : 0;
        const std::vector<uint8_t> all = gatherHost(c, &mine, sizeof(mine));
        for (int w = 0; w < c->world; w++) {
            uint64_t x;
            std::memcpy(&x, all.data() + w * sizeof(x), sizeof(x));
            if (x) return fail(c, NGX_E_UNSUPPORTED, "multi-root walk over a storage mask (TTL / max-edges cap)");
        }
    }
    const bool dyn = !rw && c->dynHops && c->world == 1 && lbCompact && hs.n > 0 && !capped && recordFrom == steps && !pushInvalid &&
                     !intermediateChecks && !svids.empty() && svids.size() <= kSeedFuseMax &&
                     svids.size() * static_cast<uint64_t>(hs.n) <= kSeedFuseMax && d.vindex.slots != nullptr;
    // The final hop's grid and E from the device (finalDev): the compaction before it keeps its packed
    // (|F|, E) in dynStats and publishes nothing, the final kernel strides an upper-bound grid over the
    // real chunks (a device-driven hop measured as fast as a host-sized one), and k_final_close publishes
    // that hop's totals beside the row count: one host round trip fewer. One shard, one record hop (the
    // last), outputs sized for every edge of the slots, no string arena, no storage mask on it.
    const bool finalDev = !dyn && !rw && c->world == 1 && lbCompact && hs.n > 0 && steps >= 2 && recordFrom == steps &&
                          !pushInvalid && !capped && nStrOut == 0;
    // Hop 1 as a sparse hop sized on the device (spec1): the fused seed kernel's packed (|F|, E) feeds the
    // sparse kernel, which strides a fixed grid over the hop's slices, so the host launches hop 1 without
    // waiting for the seed hop's total (one host round trip fewer). Chosen before E1 is known, from the
    // seeds x the OVER types' average degree: a wrong guess costs time, never rows (the sparse kernel is
    // exact for any E).
    const double e1est = d.V ? static_cast<double>(svids.size()) * static_cast<double>(slotEdges) / static_cast<double>(d.V) : 0.0;
    const bool spec1 = sparseOk && !dyn && steps >= 2 && recordFrom > 1 && !capped && !intermediateChecks &&
                       !svids.empty() && svids.size() <= kSeedFuseMax && svids.size() * static_cast<uint64_t>(hs.n) <= kSeedFuseMax &&
                       d.vindex.slots != nullptr &&
                       (c->sparseFactor < 0 || e1est * static_cast<double>(c->sparseFactor) <= static_cast<double>(d.V)) &&
                       !(pullable && e1est * 100.0 >= static_cast<double>(c->pullFactor) * static_cast<double>(d.V)) &&
                       // a pull factor set below 1 (pull on any hop of E >= V / 100: tests, pull-heavy tuning)
                       // wants hop 1's direction from its real E, which only the seed hop knows
                       !(pullable && c->pullFactor < 100);
    uint64_t* dynStats = (dyn || finalDev || spec1 || c->world > 1) ? c->dynStats.get<uint64_t>(steps + 2) : nullptr;
    const uint64_t pullMinE = pullable ? (static_cast<uint64_t>(c->pullFactor) * d.V + 99) / 100 : ~0ULL;
    if (dyn && c->epoch + 2 * static_cast<uint64_t>(steps) + 4 > 255) {   // no epoch wrap inside the query
        HIP_OK(hipMemsetAsync(c->visited.p, 0, c->visitedSize, c->stream));
        c->epoch = 0;
    }
    if (dyn || c->pipe) {
        // every buffer a hop's kernels use is sized for the whole query before the first launch: a
        // DBuf that grew later would free memory still read by kernels already enqueued. In a pipelined
        // batch too (r06): a lane growing mid-batch as a later query's frontier outgrows the earlier ones'
        // paid a hipMalloc inside the timed loop (a process's first C2 batch after a 5-query warm-up ran
        // 0.31-0.32 vs 0.29-0.30 ms per step, tools/ab_batch.py)
        const uint64_t mult = std::max<uint64_t>(maxMultiplicity(svids), 1);
        const uint64_t rowsCap = std::max<uint64_t>(d.V, svids.size());
        c->F0.get<uint32_t>(rowsCap);
        c->F1.get<uint32_t>(rowsCap);
        c->estart.get<uint64_t>(rowsCap * static_cast<uint64_t>(hs.n) + 1);
        c->ebase.get<uint64_t>(rowsCap * static_cast<uint64_t>(hs.n) + 1);
        c->tileSums.get<uint64_t>((rowsCap * static_cast<uint64_t>(hs.n) + kTile - 1) / kTile + 1);
        // (at least twice the slots' chunks: a later query whose seeds repeat a vid must not grow it inside
        // a batch — r06, the one allocation left in a C2 batch, a hipMalloc plus a device-wide free)
        const uint64_t cfBig = std::max<uint64_t>((slotEdges * std::max<uint64_t>(mult, 2) + kChunk - 1) / kChunk + 1, cfCap);
        c->chunkFirst.get<uint64_t>(cfBig);
        c->chunkFirst2.get<uint64_t>(cfBig);                // (a sparse hop swaps the two)
    }
    bool haveHeads = false;                                    // chunkFirst of the next hop already built
    bool denseNextFinal = false;                               // the final hop reads the marks of epoch denseEpoch
    uint8_t denseEpoch = 0;
    bool denseDevFinal = false;                                // world > 1: its totals from the device (close)
    const uint64_t* denseTiles = nullptr;                      // its frontier total: the close sums these
    uint64_t denseTileN = 0;
    uint64_t finalErrBits = 0;                                 // error bits published by the last final kernel
    bool haveFinalErrs = false;
    // device time of the query (HIP events) only while profiling: an event query costs ~10 us of host
    // time per call (ngx_set_profiling; bench.py reads device time from its profiled pass)
    hipEvent_t t0 = c->prof ? c->ev() : nullptr, t1 = c->prof ? c->ev() : nullptr;
    R.tLaunch = std::chrono::steady_clock::now();
    c->hmark("start");
    if (t0) HIP_OK(hipEventRecord(t0, c->stream));
    uint64_t* counters = c->counters.get<uint64_t>(8);
    uint32_t* errFlag = reinterpret_cast<uint32_t*>(counters + 4);
    uint64_t nF = svids.size();
    // the fused seed hop clears the counters itself (no memset launch); every other start clears them here
    const bool fusedSeed = nF && hs.n > 0 && nF <= kSeedFuseMax && nF * static_cast<uint64_t>(hs.n) <= kSeedFuseMax &&
                           d.vindex.slots != nullptr;
    if (!fusedSeed) HIP_OK(hipMemsetAsync(counters, 0, 64, c->stream));
    uint32_t* F = c->F0.get<uint32_t>(std::max<uint64_t>(nF, 1));
    bool haveEstart = false;                                   // estart[] / E of the next hop already built
    bool haveEbase = false;                                    // ... and its entries' CSR positions (ebase[])
    uint64_t fusedE = 0;
    Publish pendingPub{nullptr, 0};                            // a device-sized hop's total not yet read (spec1)
    Publish seedPub{nullptr, 0};                               // the fused seed hop's E, awaited after the host prep
    const uint64_t* seedE = nullptr;
    if (nF) {
        // the fused seed kernel reads the seeds from the mapped page-locked stage; else a device copy
        const int64_t* dv = nullptr;
        const int32_t* dp_ = nullptr;
        if (!fusedSeed || !stageSeedsMapped(c, sparts, svids, dp_, dv)) {
            int64_t* cv = reinterpret_cast<int64_t*>(c->seedVid.get<uint8_t>(nF * 12));   // vids, then parts
            int32_t* cp = reinterpret_cast<int32_t*>(cv + nF);
            stageSeeds(c, sparts, svids, cp, cv);
            dv = cv;
            dp_ = cp;
        }
        const uint64_t nEnt0 = nF * static_cast<uint64_t>(hs.n);
        if (fusedSeed) {
            // lookup + degrees + scan + chunk heads of the seed hop in one workgroup; E published (no
            // stream round trip); the first hop's final-kernel words cleared on the way
            uint64_t* est0 = c->estart.get<uint64_t>(nEnt0 + 1);
            uint64_t* eb0 = c->ebase.get<uint64_t>(nEnt0 + 1);
            Publish pub = nextPub(c, ngx_ctx::kSeedSlot);
            // seeds may repeat (no DISTINCT): E <= slot edges x the largest multiplicity
            const uint64_t mult = std::max<uint64_t>(maxMultiplicity(svids), 1);
            const uint64_t cf0 = (slotEdges * mult + kChunk - 1) / kChunk + 1;
            uint64_t* cf = c->chunkFirst.get<uint64_t>(std::max(cf0, cfCap));
            c->timed("seed", nF * 12 + nEnt0 * 24, [&] {
                if (launchSeedFrontierCf(dp_, dv, nF, d.vindex, hs, F, est0, pub, cf, std::max(cf0, cfCap), nullptr, 0, errFlag,
                                         c->stream, dynStats, counters, eb0))
                    throw Error{NGX_E_DEVICE, "seed"};
            });
            if (dyn) {
                fusedE = slotEdges * mult;                     // an upper bound: the device has the real E
            } else {
                seedPub = pub;
                seedE = est0 + nEnt0;
            }
            haveEstart = true;
            haveEbase = true;
            haveHeads = true;
        } else {
            c->timed("lookup", nF * 12, [&] {
                if (launchLookup(dp_, dv, nF, d.vpart, d.vid, d.V, F, c->stream)) throw Error{NGX_E_DEVICE, "lookup"};
            });
        }
    }
    // spec1: hop 1's sparse kernel enqueued right behind the seed hop, before the host prepares the
    // programs below (the GPU idled ~4 us between the two while the host did that first)
    SparseArgs sa1{};
    uint32_t* F1spec = nullptr;
    const bool devNext1 = spec1 && finalDev && steps == 2;
    if (spec1) {
        if (!bitsKnownZero(c, lbits, (d.V + 63) / 64)) HIP_OK(hipMemsetAsync(lbits, 0, (d.V + 63) / 64 * 8, c->stream));
        c->bitsClean = false;
        if (!c->sparseCtl.p) {
            c->sparseCtl.get<uint64_t>(2);
            HIP_OK(hipMemsetAsync(c->sparseCtl.p, 0, c->sparseCtl.cap, c->stream));
        }
        F1spec = (F == c->F0.p) ? c->F1.get<uint32_t>(std::max<uint64_t>(d.V, 1)) : c->F0.get<uint32_t>(std::max<uint64_t>(d.V, 1));
        sa1.F = F; sa1.estart = static_cast<const uint64_t*>(c->estart.p); sa1.chunkFirst = static_cast<const uint64_t*>(c->chunkFirst.p);
        sa1.ebase = static_cast<const uint64_t*>(c->ebase.p);
        sa1.dynIn = dynStats;                                      // the seed kernel's packed (|F|, E)
        sa1.hs = hs;
        sa1.bits = lbits;
        sa1.bitWords = (d.V + 63) / 64;
        sa1.outF = F1spec;
        sa1.outEst = c->estart2.get<uint64_t>(d.V * static_cast<uint64_t>(hs.n) + 1);
        sa1.outEbase = c->ebase2.get<uint64_t>(d.V * static_cast<uint64_t>(hs.n) + 1);
        sa1.outCf = c->chunkFirst2.get<uint64_t>(cfCap);
        sa1.cfCap = cfCap;
        sa1.ctl = static_cast<uint64_t*>(c->sparseCtl.p);
        sa1.total = devNext1 ? dynStats + 1 : counters + 2;
        sa1.pub = devNext1 ? Publish{nullptr, 0} : nextPub(c);
        sa1.err = errFlag;
        c->timed("expand_sparse", 0, [&] {
            if (launchExpandSparse(sa1, pos32, c->stream)) throw Error{NGX_E_DEVICE, "sparse expand"};
        });
        std::swap(c->estart, c->estart2);
        std::swap(c->ebase, c->ebase2);
        std::swap(c->chunkFirst, c->chunkFirst2);
    }
    // the programs and the generated kernels, prepared while the seed hop runs (only the record hops
    // read them)
    DevPrograms dp = uploadPrograms(c, progs, ySlotType, gp.colTypes);
    c->hmark("upload");
    // per-query straight-line kernels (jit.cpp); the interpreter kernels otherwise
    std::shared_ptr<const JitKernels> jk, jkNoP;             // jkNoP: record hops before the last (no pushdown)
    std::vector<int64_t> jitKc;                              // their literal table (FinalArgs::kc/kl)
    std::vector<uint32_t> jitKl;
    c->jitNote.clear();
    c->jit.releaseRetired(c->stream, c->finalStream, c->finalStream2);        // modules evicted by earlier queries (either stream)
    if (c->jitOn) {
        JitQuery jq = jitHopQuery(sp, hs, progs);
        jq.yColType = gp.colTypes;
        jq.yKey = yAlias;
        jq.dstReplica = dstReplica;
        jq.rowMask = rowMask;
        jq.ntStore = c->finalNtStores ? 1 : 0;
        jq.ntLoad = c->finalNtLoads ? 1 : 0;
        for (int k = 0; k < 3; k++) jq.outW[k] = outW[k];
        if (compact) jq.yW = yW;
        jq.input = rw && rw->perRow;
        jitSlotConsts(jq, jitKc, jitKl);
        std::string jerr;
        // kernels cached by query shape: the source is generated only on a miss
        jk = c->jit.get(jitShapeKey(sp, jq), [&] { return jitSource(sp, jq); }, jerr);
        if (jk && jq.P.present && recordFrom < steps) {
            jq.P = JitProgram{};
            jkNoP = c->jit.get(jitShapeKey(sp, jq), [&] { return jitSource(sp, jq); }, jerr);
            if (!jkNoP) jk = nullptr;
        } else {
            jkNoP = jk;
        }
        if (!jk) c->jitNote = jerr.empty() ? "jit: unsupported program" : jerr;
        c->hmark("jit");
    }
    if (seedE && !spec1) fusedE = awaitPub(c, seedPub, seedE); // the seed hop ran under the host prep above
    // multi-root walk: root sets over rows, the seed frontier's from the starts' bits
    uint64_t* rootsCur = nullptr;
    uint64_t* rootsNext = nullptr;
    if (rw) {
        // cur: this shard's rows; next: global rows (world > 1: peers' rows exchanged after each hop)
        rootsCur = c->roots[0].get<uint64_t>(std::max<uint64_t>(d.V, 1));
        rootsNext = c->roots[1].get<uint64_t>(std::max<uint64_t>(d.vglobal, 1));
        HIP_OK(hipMemsetAsync(rootsCur, 0, std::max<uint64_t>(d.V, 1) * 8, c->stream));
        if (nF) {
            std::vector<uint64_t> bits(nF, 0);
            for (uint64_t i = 0; i < nF; i++) {
                auto it = rw->bitsOf.find(svids[i]);
                bits[i] = it == rw->bitsOf.end() ? 0 : it->second;
            }
            uint64_t* db = c->rootBits.get<uint64_t>(nF);
            HIP_OK(hipMemcpyAsync(db, bits.data(), nF * 8, hipMemcpyHostToDevice, c->stream));
            if (launchScatterRoots(F, nF, db, rootsCur, c->stream)) throw Error{NGX_E_DEVICE, "scatter roots"};
            HIP_OK(hipStreamSynchronize(c->stream));           // `bits` leaves scope
        }
    }
    uint64_t totalRows = 0;
    // result columns: value bits always; lengths when strings can appear; per-row types when the
    // column's static type is unknown
    std::vector<ColSpec> colSpec;
    for (int32_t ct : gp.colTypes) colSpec.push_back(ColSpec{ct == T_UNKNOWN || ct == T_STRING, ct == T_UNKNOWN});

    std::vector<std::chrono::steady_clock::time_point> hopT;   // trace_go: host time at each hop's start
    for (uint32_t h = 1; h <= steps; h++) {
        const std::string hopName = "ngx_go hop " + std::to_string(h);
        RoctxRange hopRange(hopName.c_str());
        if (c->traceGo) hopT.push_back(std::chrono::steady_clock::now());
        bool isRecord = h >= recordFrom;
        bool isFinal = h == steps;
        if (spec1 && h == 1) {
            // the seed hop's frontier expanded by the sparse kernel (launched above), its size read on the device
            const bool devNext = devNext1;
            uint32_t* Fn = F1spec;
            const SparseArgs& sa = sa1;
            const uint64_t E1 = awaitPub(c, seedPub, seedE);     // published before the sparse kernel ran
            R.hopFrontier.push_back(nF);
            R.hopEdges.push_back(E1);
            c->addBytes("expand_sparse", E1 * 12);
            haveEstart = haveEbase = haveHeads = haveBits = true;
            c->sparseHops++;
            F = Fn;
            if (devNext) {
                nF = d.V;
                fusedE = slotEdges;
                R.hopNext.push_back(nF);
            } else {
                pendingPub = sa.pub;                               // read at the next hop's start
            }
            continue;
        }
        // the previous hop (sparse, sized on the device) published its total and the host has not read it:
        // if this hop is predicted to pull (the last query's hop 2 did), its pull is launched first, reading
        // E on the device (it does nothing when E is below the threshold), so the host's wait for the total
        // overlaps the pull instead of idling the GPU (r05: 12-15 us per C2 step)
        bool specPull = false;
        uint8_t specEp = 0;
        if (pendingPub.slot) {
            const bool tryPull = !isFinal && pullable && c->world == 1 && c->pullPredict && !capped && !intermediateChecks;
            if (tryPull) {
                specEp = nextEpoch(c);
                pa.out = marksA + d.gbase;
                pa.ep = specEp;
                pa.err = errFlag;
                pa.dyn = counters + 2;                             // the sparse hop's packed (|F|, E)
                pa.minE = pullMinE;
                c->timed("pull", d.V * 9 * static_cast<uint64_t>(hs.n), [&] {
                    if (launchPull(pa, c->stream)) throw Error{NGX_E_DEVICE, "pull"};
                });
            }
            const uint64_t packed = awaitPub(c, pendingPub, counters + 2);
            pendingPub = Publish{nullptr, 0};
            nF = packed >> kFdShift;
            fusedE = packed & kFdMask;
            c->addBytes("expand_sparse", nF * (4 + 24 * static_cast<uint64_t>(hs.n)));
            R.hopNext.push_back(nF);
            if (nF == 0) break;                                    // GO_EXIT: empty frontier
            specPull = tryPull && fusedE >= pullMinE;
        }
        const bool devE = (finalDev || denseDevFinal) && isFinal;   // E below is an upper bound; the device has it
        uint64_t nEnt = nF * static_cast<uint64_t>(hs.n);
        uint64_t* estart = c->estart.get<uint64_t>(nEnt + 1);
        const uint64_t* ebase = haveEbase ? c->ebase.get<uint64_t>(nEnt + 1) : nullptr;
        uint64_t* tiles = c->tileSums.get<uint64_t>((std::max<uint64_t>(nEnt, 1) + kTile - 1) / kTile + 1);
        uint64_t E = 0;
        if (haveEstart) {
            E = nEnt ? fusedE : 0;
        } else if (nEnt) {
            Publish pub = nextPub(c);
            c->timed("degree_scan", nEnt * 24, [&] {
                if (launchDegreeScan(F, nEnt, hs, estart, tiles, c->stream, pub)) throw Error{NGX_E_DEVICE, "degree scan"};
            });
            E = awaitPub(c, pub, estart + nEnt);
        }
        haveEstart = false;
        haveEbase = false;
        if (isFinal && pushInvalid && nF) return fail(c, NGX_E_QUERY, "Get neighbors failed");
        if (!dyn) {                                              // dyn: read back after the last hop
            R.hopFrontier.push_back(nF);
            R.hopEdges.push_back(E);
        }
        const uint64_t* dynTotal = (dyn || devE) ? dynStats + (h - 1) : nullptr;   // this hop's (|F|, E), device side
        uint64_t chunks = (E + kChunk - 1) / kChunk;
        uint64_t* chunkFirst = c->chunkFirst.get<uint64_t>(std::max<uint64_t>(chunks, 1));
        if (E && !haveHeads) {
            c->timed("chunk_first", nEnt * 16, [&] {
                if (launchChunkFirst(estart, nEnt, chunkFirst, c->stream, nullptr, 0))
                    throw Error{NGX_E_DEVICE, "chunk first"};
            });
        }
        haveHeads = false;
        // the hop's storage request: which edges the processor emits (collectEdgeProps, .inl:501-608)
        FinalArgs a{};
        a.F = F; a.estart = estart; a.chunkFirst = chunkFirst; a.nEnt = nEnt; a.E = E; a.hs = hs;
        a.ebase = ebase;
        a.vid = d.vid; a.V = d.V; a.gbase = d.gbase;
        a.env = VmEnv{d.dslots, d.dtags, d.dcols, dp.pool, errFlag + 1, now, dstTags, dstCols};
        a.P = (isFinal && progs.P >= 0) ? dp.code + progs.P : nullptr;
        a.propsMask = isRecord ? recordPropsMask : 0;
        a.ttlMask = ttlMask;
        for (int s = 0; s < hs.n; s++) { a.ttlCol[s] = ttlCol[s]; a.ttlDur[s] = ttlDur[s]; }
        a.now = now;
        a.err = errFlag;
        // Edges the expansion must skip (rows read with TTL / bad rows, intermediate hops) or a per-vertex
        // cap: the storage outcome is materialised per hop edge (k_storage_pass + k_cap) and both the
        // final kernel and the expansion read it; otherwise the final kernel checks storage in place.
        bool checks = false;
        for (int s = 0; s < hs.n; s++) {
            if (((a.propsMask | a.ttlMask) >> s & 1u) && (hs.eflags[s] != nullptr || ttlCol[s] >= 0)) checks = true;
        }
        const uint8_t* mask = nullptr;
        if (E && (capped || (!isFinal && checks))) {
            uint8_t* m = c->edgeMask.get<uint8_t>(E);
            c->timed("storage_mask", E, [&] {
                if (launchStoragePass(a, m, c->stream)) throw Error{NGX_E_DEVICE, "storage pass"};
                if (capped && launchCap(estart, nEnt, m, edgeCap, c->stream)) throw Error{NGX_E_DEVICE, "cap"};
            });
            mask = m;
        }
        a.mask = mask;
        if (isRecord && ownerDst) {                              // every shard, E = 0 too (it answers its peers)
            const DstFetch f = fetchDstProps(c, sp, dstRec++, F, estart, chunkFirst, nEnt, E, hs, pos32, ebase);
            a.env.dtags = f.tags;
            a.env.dcols = f.cols;
            a.dstMap = f.map;
        }
        if (isRecord && E) {
            // ngx_go_batch: this query's last final hop may overlap the next query (goDeferPoint): not with a
            // device read-back left (multi-root walks), string arenas, profiling or host traces. World > 1 too
            // (r06): the final hop is the shard's own work, no collective follows it; the next query's hops and
            // collectives run on the one front stream beside it
            const bool deferrable = c->pipe && isFinal && c->pinDev && !dyn && !rw && nStrOut == 0 &&
                                    !c->prof && !c->htrace && !c->traceGo && pipelinable(p);
            if (c->pipe) goPreFinalPoint(c);
            FinalStreamScope fss(c, deferrable);
            a.W = progs.W >= 0 ? dp.code + progs.W : nullptr;
            a.nY = static_cast<int32_t>(progs.yOff.size());
            a.yCode = dp.code;
            a.yOff = dp.yOff;
            a.ySlotType = nullptr;
            a.yColType = dp.yColType;
            a.wIsP = (isFinal && wIsP) ? 1u : 0u;
            for (size_t k = 0; k < jitKc.size(); k++) { a.kc[k] = jitKc[k]; a.kl[k] = jitKl[k]; }
            // a masked hop (max-edges cap) runs on the interpreter kernel: the generated ones skip the mask
            const JitKernels* kj = mask ? nullptr : (isFinal ? jk.get() : jkNoP.get());
            uint64_t Ef = E;                                    // edges the final launch evaluates
            uint64_t gridf = chunks;
            a.fin = nullptr;
            a.denseMark = nullptr;
            a.denseEp = 0;
            if (isFinal && denseNextFinal) {
                // every CSR position of the slot; entries = the shard's rows, the frontier = the marks
                a.estart = hs.off[0];
                a.ebase = hs.off[0];
                a.chunkFirst = d.chunkRow[hs.slotIdx[0]];
                a.nEnt = d.V;
                a.E = slotEdges;
                a.denseMark = marksA + d.gbase;
                a.denseEp = denseEpoch;
                Ef = slotEdges;
                gridf = (slotEdges + kChunk - 1) / kChunk;
                c->denseFinals++;
            }
            if (rw && rw->perRow) {
                // the hop's entries as (frontier row, input row) pairs: a frontier row once per input row
                // of every root that reaches it, the input row travelling with the entry (FinalArgs::fin)
                if (mask) return fail(c, NGX_E_UNSUPPORTED, "multi-root walk over a storage mask (TTL / max-edges cap)");
                std::vector<uint64_t> m(nF);
                std::vector<uint32_t> rows(nF);
                uint64_t* dm = c->rootBits.get<uint64_t>(std::max<uint64_t>(nF, 1));
                if (launchGatherRoots(F, nF, rootsCur, dm, c->stream)) throw Error{NGX_E_DEVICE, "gather roots"};
                HIP_OK(hipMemcpyAsync(m.data(), dm, nF * 8, hipMemcpyDeviceToHost, c->stream));
                HIP_OK(hipMemcpyAsync(rows.data(), F, nF * 4, hipMemcpyDeviceToHost, c->stream));
                HIP_OK(hipStreamSynchronize(c->stream));
                std::vector<uint32_t> f2, in2;
                for (uint64_t i = 0; i < nF; i++) {
                    if (rows[i] == kNoRow) continue;
                    for (uint64_t r = m[i]; r; r &= r - 1) {
                        for (uint32_t ir : (*rw->rowsOfBit)[__builtin_ctzll(r)]) { f2.push_back(rows[i]); in2.push_back(ir); }
                    }
                }
                const uint64_t n2 = f2.size(), nEnt2 = n2 * static_cast<uint64_t>(hs.n);
                uint32_t* dF2 = c->pwF.get<uint32_t>(std::max<uint64_t>(n2, 1));
                uint32_t* dIn2 = c->pwIn.get<uint32_t>(std::max<uint64_t>(n2, 1));
                uint64_t* est2 = c->pwEst.get<uint64_t>(nEnt2 + 1);
                uint64_t* tiles2 = c->tileSums.get<uint64_t>((std::max<uint64_t>(nEnt2, 1) + kTile - 1) / kTile + 1);
                HIP_OK(hipMemcpyAsync(dF2, f2.data(), n2 * 4, hipMemcpyHostToDevice, c->stream));
                HIP_OK(hipMemcpyAsync(dIn2, in2.data(), n2 * 4, hipMemcpyHostToDevice, c->stream));
                Ef = 0;
                if (nEnt2) {
                    Publish pub = nextPub(c);
                    if (launchDegreeScan(dF2, nEnt2, hs, est2, tiles2, c->stream, pub)) throw Error{NGX_E_DEVICE, "degree scan"};
                    Ef = awaitPub(c, pub, est2 + nEnt2);
                }
                gridf = (Ef + kChunk - 1) / kChunk;
                uint64_t* cf2 = c->pwCf.get<uint64_t>(std::max<uint64_t>(gridf, 1));
                if (launchChunkFirst(est2, nEnt2, cf2, c->stream, nullptr, 0)) throw Error{NGX_E_DEVICE, "chunk first"};
                HIP_OK(hipStreamSynchronize(c->stream));       // f2 / in2 leave scope
                a.F = dF2; a.fin = dIn2; a.estart = est2; a.chunkFirst = cf2; a.nEnt = nEnt2; a.E = Ef;
                a.ebase = nullptr;
                a.env.input = rw->input;
            }
            // outputs sized for every edge passing (rows are written in the same launch), plus the groups'
            // partly filled last blocks (kargs.h resv*)
            resvGeometry(c, a);
            uint64_t cap = totalRows + Ef + resvSlack(a);
            growKeep(c, c->oSrc, cap * 8, totalRows * 8);
            growKeep(c, c->oDst, cap * 8, totalRows * 8);
            growKeep(c, c->oRank, cap * 8, totalRows * 8);
            growKeep(c, c->oType, cap * 4, totalRows * 4);
            prepareCols(c, a, colSpec, cap, totalRows, yAlias, compact ? &yW : nullptr, rankConst);
            a.oBase = totalRows;
            a.oSrcW = static_cast<int8_t>(outW[0]);
            a.oDstW = static_cast<int8_t>(outW[1]);
            a.oRankW = static_cast<int8_t>(outW[2]);
            a.oSrc = (rowMask & 1) ? static_cast<int64_t*>(c->oSrc.p) : nullptr;
            a.oDst = (rowMask & 2) ? static_cast<int64_t*>(c->oDst.p) : nullptr;
            a.oRank = (rowMask & 4) ? static_cast<int64_t*>(c->oRank.p) : nullptr;
            a.oType = constType ? nullptr : static_cast<int32_t*>(c->oType.p);
            a.oEntry = nullptr;
            a.lbStatus = nullptr;
            // k_final_close publishes the row count, in a slot of its own (a batch's next query publishes its
            // first hops' totals while this one is deferred: goDeferPoint)
            Publish rowsPub = dyn ? Publish{nullptr, 0} : nextPub(c, ngx_ctx::kRowsSlot);
            a.rowsPub = rowsPub.slot;
            a.rowsSeq = rowsPub.seq;
            a.dynTotal = dynTotal;
            if (isFinal && denseNextFinal && denseTiles != nullptr) {
                if (dynTotal == nullptr) throw Error{NGX_E_DEVICE, "dense final hop without a device total"};
                a.dynTiles = denseTiles;
                a.nDynTiles = denseTileN;
            }
            a.strOut = nullptr;
            a.nStrOut = nStrOut;
            a.strOutMask = strOutMask;
            if (nStrOut) {
                // one 64-byte slot per (edge, building column): past str_arena_max the caller's CPU path
                // runs the query instead of a device allocation failure
                const uint64_t arenaBytes = (Ef + resvSlack(a)) * nStrOut * static_cast<uint64_t>(kStrBuildBytes);
                if (arenaBytes > c->strArenaMax)
                    return fail(c, NGX_E_UNSUPPORTED, "built strings of " + std::to_string(Ef) + " edges exceed the device string arena");
                if (c->strArena.size() <= arenas.size()) c->strArena.resize(arenas.size() + 1);
                a.strOut = c->strArena[arenas.size()].get<char>((Ef + resvSlack(a)) * nStrOut * static_cast<uint64_t>(kStrBuildBytes));
                arenas.push_back(Arena{a.strOut, 0});
            }
            // dyn: chunks of the upper bound E; the workgroups past the real chunks return at once
            // a 512-thread generated kernel covers two CE chunks per workgroup (dyn: an upper bound anyway)
            const unsigned nt = 256u;
            const unsigned grid = static_cast<unsigned>(gridf);
            // each group's block table: virtual rows of the group's chunks / block, + 1 partial block
            const uint64_t perGroup = (grid + a.resvG - 1) / a.resvG * kChunk;
            a.resvTB = static_cast<uint32_t>(((perGroup + (1ULL << a.resvShift) - 1) >> a.resvShift) + 1);
            a.resvTab = resvTable(c, static_cast<uint64_t>(a.resvTB) * a.resvG);
            if (++c->resvSeq == 0) c->resvSeq = 1;
            a.resvSeq = c->resvSeq;
            c->timed("final", (dyn || devE) ? 0 : Ef * (keyReadBytes + kfBytes), [&] {
                if (grid == 0) return;
                if (kj) {
                    void* args[] = {&a};
                    HIP_OK(hipModuleLaunchKernel(kj->final, grid, 1, 1, nt, 1, 1, 0, c->stream, args, nullptr));
                } else if (launchFinal(a, c->stream, grid)) {
                    throw Error{NGX_E_DEVICE, "final"};
                }
            });
            // the holes of the groups' last blocks closed, the row count published (also for grid 0). An
            // overlapped final hop's close runs on the close stream: the next query's final hop (another
            // lane's rows and counters) starts on the final stream without waiting for it
            {
                hipStream_t fs = c->stream;
                if (deferrable && c->closeStream) {
                    streamAfter(c->closeStream, fs, c->pipeEvent(4));
                    c->stream = c->closeStream;
                }
                try {
                    c->timed("final_close", 0, [&] {
                        if (launchFinalClose(a, c->stream)) throw Error{NGX_E_DEVICE, "final close"};
                    });
                    if (deferrable) {                          // the lane's next final hop waits for this close
                        hipEvent_t& ev = c->laneCloseEv[c->activeLane];
                        if (!ev) HIP_OK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
                        HIP_OK(hipEventRecord(ev, c->stream));
                        c->laneClosePending[c->activeLane] = true;
                    }
                } catch (...) {
                    c->stream = fs;
                    throw;
                }
                c->stream = fs;
            }
            c->resvClosePending = false;
            c->resvRows = a.resvCtl + (a.resvG + 1) * static_cast<uint64_t>(a.resvStride);
            fss.restore();                                      // (the front stream again)
            if (!dyn) {
                // GO: the row count and the query's error bits so far, published by k_final_close
                uint64_t fin = 0;                               // devE: this hop's packed (|F|, E)
                const uint64_t* rowsDev = c->resvRows;          // (the next query resets c->resvRows)
                if (deferrable) goDeferPoint(c);                // ngx_go_batch: the next query runs here
                uint64_t nrows = awaitPub(c, rowsPub, rowsDev, &finalErrBits, errFlag, devE ? &fin : nullptr,
                                          devE ? dynTotal : nullptr);
                haveFinalErrs = true;
                if (devE) {                                     // the hop's statistics, known now
                    const uint64_t fF = fin >> kDynShift, fE = fin & kDynMask;
                    R.hopFrontier.back() = fF;
                    R.hopEdges.back() = fE;
                    if (!R.hopNext.empty()) R.hopNext.back() = fF;
                    c->addBytes("final", fE * (keyReadBytes + kfBytes));
                    c->addBytes("compact_degrees", fF * 8 + fF * static_cast<uint64_t>(hs.n) * 24);
                }
                c->addBytes("final", nrows * rowBytes);
                if (rw && !rw->perRow) {                        // the rows' src vids -> their roots
                    RootWalk::Hop hop;
                    hop.rowBase = totalRows;
                    hop.rows = nrows;
                    std::vector<uint64_t> m(nF);
                    std::vector<uint32_t> rows(nF);
                    if (nF) {
                        uint64_t* dm = c->rootBits.get<uint64_t>(nF);
                        if (launchGatherRoots(F, nF, rootsCur, dm, c->stream)) throw Error{NGX_E_DEVICE, "gather roots"};
                        HIP_OK(hipMemcpyAsync(m.data(), dm, nF * 8, hipMemcpyDeviceToHost, c->stream));
                        HIP_OK(hipMemcpyAsync(rows.data(), F, nF * 4, hipMemcpyDeviceToHost, c->stream));
                        HIP_OK(hipStreamSynchronize(c->stream));
                    }
                    for (uint64_t i = 0; i < nF; i++)
                        if (rows[i] != kNoRow) hop.rootsOf[sp.host->vid[rows[i]]] |= m[i];
                    rw->record.push_back(std::move(hop));
                }
                totalRows += nrows;
                if (nStrOut) arenas.back().rows = nrows;
            }
        }
        if (isFinal) break;
        // ---- expand to the next frontier (set of distinct dsts)
        // pull when the hop's edges outnumber the shard's rows pullFactor/100 times (every row's in-list is
        // probed instead of every frontier edge storing a mark); push otherwise, or when a storage mask
        // (TTL / max-edges) decides which edges count
        // dyn: both expansions are enqueued and the device takes the one its E selects (pullMinE)
        bool pull = dyn ? pullable : pullable && !mask && E && E * 100 >= static_cast<uint64_t>(c->pullFactor) * d.V;
        pull = pull || specPull;                                   // (the same threshold: pullMinE)
        if (h == 2 && c->world == 1 && !dyn) c->pullPredict = pull;
        uint64_t eMaxShard = 0;                                  // the largest shard's E (from the pull gather)
        bool eMaxKnown = false;
        if (!dyn && pullGather) {
            // the hop's edges over every shard, whether every shard can pull (its pull state built, no
            // storage mask) and rank 0's pull_factor (one threshold for all)
            const uint64_t rec[3] = {E, (pullable && !mask) ? 1u : 0u, static_cast<uint64_t>(std::max<int64_t>(c->pullFactor, 0))};
            const std::vector<uint8_t> all = gatherHost(c, rec, sizeof(rec));
            uint64_t eAll = 0, can = 1, pf = 0;
            for (int w = 0; w < c->world; w++) {
                uint64_t r[3];
                std::memcpy(r, all.data() + w * sizeof(rec), sizeof(rec));
                eAll += r[0];
                eMaxShard = std::max(eMaxShard, r[0]);
                can &= r[1];
                if (w == 0) pf = r[2];
            }
            pull = can && pf > 0 && eAll && eAll * 100 >= pf * d.vglobal;
            eMaxKnown = true;
        }
        // the hop's output marks (pull and push alike; the pull reads the frontier from the bitmap)
        uint8_t* const marks = marksA;
        // sparse: this push hop's expansion builds the next frontier itself (no compaction sweep)
        const bool sparse = sparseOk && !dyn && !pull && !mask && E > 0 &&
                            (c->sparseFactor < 0 || static_cast<unsigned __int128>(E) * static_cast<uint64_t>(c->sparseFactor) <= d.V);
        if (pull && !haveBits) {                                // the seed frontier: bitmap from its list
            c->bitsClean = false;
            HIP_OK(hipMemsetAsync(lbits, 0, (d.V + 63) / 64 * 8, c->stream));
            if (launchMarkBits(F, nF, lbits, c->stream)) throw Error{NGX_E_DEVICE, "mark bits"};
        }
        if (pull && c->world > 1) {
            // every shard's frontier bitmap -> one bitmap over global rows
            uint64_t* seg = c->pullGather.get<uint64_t>(segWords * c->world);
            c->timed("frontier_allgather", 0, [&] { allGather(c, lbits, seg, segWords * 8); });
            RepackArgs ra{};
            ra.seg = seg;
            ra.segWords = segWords;
            for (int q = 0; q <= c->world; q++) ra.sb[q] = d.shardBase[q];
            ra.world = c->world;
            ra.out = fbits;
            ra.outWords = (d.vglobal + 63) / 64;
            if (launchRepackBits(ra, c->stream)) throw Error{NGX_E_DEVICE, "repack bits"};
            c->lastXchgBytes = segWords * 8 * static_cast<uint64_t>(c->world - 1);
            c->addBytes("exchange", c->lastXchgBytes);
            R.hopXchg.push_back(c->lastXchgBytes);
        }
        uint8_t ep = specPull ? specEp : nextEpoch(c);
        if (specPull) c->pullHops++;                               // launched above
        if (pull && !specPull) {
            pa.out = marks + d.gbase;
            pa.ep = ep;
            pa.err = errFlag;
            pa.dyn = dynTotal;
            pa.minE = pullMinE;
            c->timed("pull", dyn ? 0 : d.V * 9 * static_cast<uint64_t>(hs.n), [&] {
                if (launchPull(pa, c->stream)) throw Error{NGX_E_DEVICE, "pull"};
            });
            if (!dyn) c->pullHops++;
        }
        if (rw && E) {
            // multi-root walk: destinations take the union of their sources' roots
            if (mask) return fail(c, NGX_E_UNSUPPORTED, "multi-root walk over a storage mask (TTL / max-edges cap)");
            HIP_OK(hipMemsetAsync(rootsNext, 0, std::max<uint64_t>(d.vglobal, 1) * 8, c->stream));
            c->timed("expand_roots", E * 16, [&] {
                if (launchExpandRoots(F, nF, hs, rootsCur, rootsNext, marks, ep, c->stream))
                    throw Error{NGX_E_DEVICE, "expand roots"};
            });
        } else if ((!pull || dyn) && E && !sparse) {
            c->timed("expand", dyn ? 0 : E * 8, [&] {
                if (launchExpandMark(F, estart, chunkFirst, nEnt, E, hs, marks, ep, pos32, c->stream, mask,
                                     dynTotal, dyn ? pullMinE : ~0ULL, ebase))
                    throw Error{NGX_E_DEVICE, "expand"};
            });
        }
        if (c->world > 1 && !pull) {                            // a pull computed every local row already
            // vid lists when they are sure to be smaller than the bitmaps: a shard marks at most E rows,
            // 4 B each, against (peer rows) / 8 B per peer. Every shard decides alike (the gathered E).
            uint64_t minPeer = ~0ULL;
            for (int q = 0; q < c->world; q++) minPeer = std::min<uint64_t>(minPeer, d.shardBase[q + 1] - d.shardBase[q]);
            const bool lists = c->xchgLists > 0 || (c->xchgLists < 0 && eMaxKnown && 32 * eMaxShard < minPeer);
            c->timed("exchange", 0, [&] {
                if (lists) exchangeFrontierList(c, d, ep);
                else exchangeFrontier(c, d, ep);
                if (rw) {                                       // E == 0: no expansion wrote next[]
                    if (!E) HIP_OK(hipMemsetAsync(rootsNext, 0, std::max<uint64_t>(d.vglobal, 1) * 8, c->stream));
                    exchangeRoots(c, d, rootsNext, rootsCur);   // cur is dead after the expansion
                }
            });
            c->addBytes("exchange", c->lastXchgBytes);
            R.hopXchg.push_back(c->lastXchgBytes);
        }
        uint32_t* Fn = (F == c->F0.p) ? c->F1.get<uint32_t>(std::max<uint64_t>(d.V, 1)) : c->F0.get<uint32_t>(std::max<uint64_t>(d.V, 1));
        uint64_t* tiles2 = c->tileSums.get<uint64_t>((std::max<uint64_t>(d.V, 1) + kTile - 1) / kTile + 1);
        if (sparse) {
            // the bitmap must start all zero: it is the hop's dedup set and then the next frontier's bits
            if (!bitsKnownZero(c, lbits, (d.V + 63) / 64)) HIP_OK(hipMemsetAsync(lbits, 0, (d.V + 63) / 64 * 8, c->stream));
            c->bitsClean = false;
            if (!c->sparseCtl.p) {
                c->sparseCtl.get<uint64_t>(2);
                HIP_OK(hipMemsetAsync(c->sparseCtl.p, 0, c->sparseCtl.cap, c->stream));
            }
            const bool devNext = finalDev && h + 1 == steps;      // the next hop is the device-sized final one
            SparseArgs sa{};
            sa.F = F; sa.estart = estart; sa.chunkFirst = chunkFirst; sa.ebase = ebase;
            sa.nEnt = nEnt; sa.E = E; sa.hs = hs;
            sa.bits = lbits;
            sa.bitWords = (d.V + 63) / 64;
            sa.outF = Fn;
            sa.outEst = c->estart2.get<uint64_t>(d.V * static_cast<uint64_t>(hs.n) + 1);
            sa.outEbase = c->ebase2.get<uint64_t>(d.V * static_cast<uint64_t>(hs.n) + 1);
            sa.outCf = c->chunkFirst2.get<uint64_t>(cfCap);
            sa.cfCap = cfCap;
            sa.ctl = static_cast<uint64_t*>(c->sparseCtl.p);
            sa.total = devNext ? dynStats + h : counters + 2;
            sa.pub = devNext ? Publish{nullptr, 0} : nextPub(c);
            sa.err = errFlag;
            c->timed("expand_sparse", E * 12, [&] {
                if (launchExpandSparse(sa, pos32, c->stream)) throw Error{NGX_E_DEVICE, "sparse expand"};
            });
            // the next hop reads the arrays just written; this hop's become the spares
            std::swap(c->estart, c->estart2);
            std::swap(c->ebase, c->ebase2);
            std::swap(c->chunkFirst, c->chunkFirst2);
            haveEstart = true;
            haveEbase = true;
            haveHeads = true;
            haveBits = true;                                    // the bitmap holds exactly the next frontier
            c->sparseHops++;
            if (devNext) {
                nF = d.V;
                fusedE = slotEdges;
            } else {
                uint64_t packed = awaitPub(c, sa.pub, counters + 2);
                nF = packed >> kFdShift;
                fusedE = packed & kFdMask;
                c->addBytes("expand_sparse", nF * (4 + 24 * static_cast<uint64_t>(hs.n)));
            }
        } else if (lbCompact) {
            // one launch: next frontier + estart + chunk heads; the look-back words of the next
            // compaction cleared on the way
            CompactArgs ca{};
            ca.visited = marks + d.gbase;
            ca.V = d.V;
            ca.hs = hs;
            ca.outF = Fn;
            ca.estart = c->estart.get<uint64_t>(d.V * static_cast<uint64_t>(hs.n) + 1);
            ca.ebase = c->ebase.get<uint64_t>(d.V * static_cast<uint64_t>(hs.n) + 1);
            ca.chunkFirst = c->chunkFirst.get<uint64_t>(cfCap);
            ca.cfCap = cfCap;
            ca.tileSum = cmpTile;
            ca.waveSum = cmpWave;
            ca.clear32 = pullable ? pa.ctl : nullptr;
            ca.bits = lbits;
            // a bitmap no hop will read (the next hop is the final one, or no hop pulls) is written as
            // zeros: a later sparse hop then finds it clean without a memset
            ca.bitsZero = (h + 1 == steps || !pullable) ? 1 : 0;
            haveBits = lbits != nullptr && !ca.bitsZero;
            c->bitsClean = false;
            const bool devNext = finalDev && h + 1 == steps;      // the next hop is the device-sized final one
            // dense final hop next: after a pull (its frontier is most of the shard's edges), one OVER type; at
            // world > 1 too (the pull marked this shard's own rows, no exchange follows it), but not with the
            // $$ owner fetch (it expands the frontier list)
            const bool denseNext = (devNext || (c->world > 1 && !dyn && h + 1 == steps && !ownerDst)) && c->denseFinal &&
                                   pull && !mask && !capped && !rw && hs.n == 1 && recordFrom == steps &&
                                   hs.slotIdx[0] >= 0 && hs.slotIdx[0] < static_cast<int32_t>(d.chunkRow.size());
            ca.countOnly = denseNext ? 1 : 0;
            // world > 1: the dense final hop's grid is static, so its totals (the statistics) can stay on the
            // device too, published by its close: no host wait after this launch (flag dense_world_dev)
            const bool denseWorld = denseNext && !devNext && c->denseWorldDev;
            const bool devTotal = devNext || denseWorld;
            // device-sized dense final hop: its close sums the count launch's tiles (no launch here)
            ca.totalByClose = denseNext && devTotal && !dyn && c->denseCloseTotal ? 1 : 0;
            denseNextFinal = denseNext;
            denseDevFinal = denseWorld;
            denseEpoch = ep;
            ca.total = (dyn || devTotal) ? dynStats + h : counters + 2;
            ca.pub = (dyn || devTotal) ? Publish{nullptr, 0} : nextPub(c);
            ca.zero = nullptr;
            ca.nzero = 0;
            ca.err = errFlag;
            ca.epoch = ep;
            ca.laneRows = c->compactLaneRows;
            // auto: 256-thread workgroups while a pipelined batch may run another query's final hop beside
            // this compaction (ngx_go_batch's front stream), 1024 alone (2 us faster there)
            ca.wgThreads = c->compactWg != 0 ? c->compactWg : (c->finalStream ? 256 : 1024);
            c->timed("compact_degrees", 0, [&] {
                if (launchCompactLb(ca, c->stream)) throw Error{NGX_E_DEVICE, "compact"};
            });
            denseTiles = ca.totalByClose ? cmpTile : nullptr;
            denseTileN = ca.totalByClose ? compactLbTiles(ca) : 0;
            if (ca.bits && ca.bitsZero) markBitsZero(c, ca.bits, (d.V + 63) / 64);
            haveEstart = true;
            haveEbase = true;
            haveHeads = true;
            if (dyn || devTotal) {                              // upper bounds; the device has the real ones
                nF = d.V;
                fusedE = slotEdges;
            } else {
                uint64_t packed = awaitPub(c, ca.pub, counters + 2);
                nF = packed >> kFdShift;
                fusedE = packed & kFdMask;
                c->addBytes("compact_degrees", nF * 8 + nF * static_cast<uint64_t>(hs.n) * 24);
            }
        } else if (fuseDeg) {
            // estart sized for any next frontier (every row of the shard) so the next hop's get() keeps it
            uint64_t* est = c->estart.get<uint64_t>(d.V * static_cast<uint64_t>(hs.n) + 1);
            Publish pub = nextPub(c);
            c->timed("compact_degrees", 0, [&] {
                if (launchCompactDegrees(marks, d.gbase, d.V, ep, hs, Fn, est, tiles2,
                                         counters + 2, c->stream, pub))
                    throw Error{NGX_E_DEVICE, "compact"};
            });
            uint64_t packed = awaitPub(c, pub, counters + 2);
            nF = packed >> kFdShift;
            fusedE = packed & kFdMask;
            haveEstart = true;
            c->addBytes("compact_degrees", nF * 8 + nF * static_cast<uint64_t>(hs.n) * 24);
        } else {
            c->timed("compact", 0, [&] {
                if (launchCompact(marks, d.gbase, d.V, ep, Fn, tiles2, counters + 2, c->stream))
                    throw Error{NGX_E_DEVICE, "compact"};
            });
            nF = readScalar(c, counters + 2);
            c->addBytes("compact", nF * 8);
        }
        if (!dyn) R.hopNext.push_back(nF);
        F = Fn;
        if (rw && c->world == 1) std::swap(rootsCur, rootsNext);
        if (!dyn && nF == 0 && c->world == 1) break;            // GO_EXIT: empty frontier
    }
    if (t1) HIP_OK(hipEventRecord(t1, c->stream));
    // the outcome (error words; dyn: the hop totals and the row count) published to host-mapped memory
    // by one last kernel and polled; the event / copy route is the fallback
    uint64_t tail[1 + 64];
    const int nExtra = dyn ? static_cast<int>(steps) + 1 : 0;
    bool tailOk = false;
    if (dyn) {                                                   // the row count next to the hop totals
        if (c->resvRows) HIP_OK(hipMemcpyAsync(dynStats + steps, c->resvRows, 8, hipMemcpyDeviceToDevice, c->stream));
        else HIP_OK(hipMemsetAsync(dynStats + steps, 0, 8, c->stream));
    }
    if (!dyn && haveFinalErrs) {                                 // the last final kernel published them
        tail[0] = finalErrBits;
        tailOk = true;
    } else if (c->pinDev && nExtra <= 64) {
        const uint64_t seq = ++c->pinSeq;
        if (launchPublishTail(errFlag, dynStats, nExtra, c->pinDev + c->pinLane + ngx_ctx::kTailOff, seq, c->stream))
            throw Error{NGX_E_DEVICE, "publish tail"};
        tailOk = awaitTail(c, seq, tail, 1 + nExtra);
    }
    if (!tailOk) {
        HIP_OK(hipStreamSynchronize(c->stream));
        uint32_t f[4];
        HIP_OK(hipMemcpy(f, errFlag, 16, hipMemcpyDeviceToHost));
        tail[0] = 0;
        for (int k = 0; k < 4; k++) tail[0] |= static_cast<uint64_t>(f[k] != 0) << k;
        if (nExtra) HIP_OK(hipMemcpy(tail + 1, dynStats, nExtra * 8, hipMemcpyDeviceToHost));
    }
    c->hmark("sync");
    if (dyn) {
        // the hop totals the kernels passed along, and the final kernel's row count
        std::vector<uint64_t> st(tail + 1, tail + 1 + steps);
        uint64_t rows = tail[1 + steps];
        for (uint32_t h = 1; h <= steps; h++) {
            const uint64_t nf = st[h - 1] >> kFdShift, e = st[h - 1] & kFdMask;
            if (h > 1 && nf == 0) break;                        // GO_EXIT: empty frontier (the kernels idled)
            R.hopFrontier.push_back(nf);
            R.hopEdges.push_back(e);
            if (h < steps) {
                R.hopNext.push_back(st[h] >> kFdShift);
                if (pullable && e >= pullMinE) c->pullHops++;
                c->addBytes(pullable && e >= pullMinE ? "pull" : "expand",
                            pullable && e >= pullMinE ? d.V * 9 * static_cast<uint64_t>(hs.n) : e * 8);
                c->addBytes("compact_degrees", (st[h] >> kFdShift) * (8 + 24 * static_cast<uint64_t>(hs.n)));
            } else {
                c->addBytes("final", e * (keyReadBytes + kfBytes) + rows * rowBytes);
            }
        }
        totalRows = rows;
        if (nStrOut && !arenas.empty()) arenas.back().rows = rows;
    }
    float ms = 0;
    if (t1) {
        HIP_OK(hipEventSynchronize(t1));
        HIP_OK(hipEventElapsedTime(&ms, t0, t1));
    }
    c->collectTimings();
    R.r.device_ms = ms;
    R.tDone = std::chrono::steady_clock::now();
    if (c->traceGo) {
        // GoExecutor's FLAGS_trace_go log (GoExecutor.cpp:559-569, 748-751, 834-836), one line per step of
        // this shard: its frontier, scanned edges, the next frontier and the host time from the step's
        // start to the next one's (or to the result)
        hopT.push_back(R.tDone);
        for (size_t h = 0; h + 1 < hopT.size() && h < R.hopEdges.size(); h++) {
            std::fprintf(stderr, "[ngx trace_go r%d] Step:%zu finished, total request vertices %llu, scanned edges %llu, "
                         "next frontier %llu, time cost %.0fus\n", c->rank, h + 1,
                         static_cast<unsigned long long>(h < R.hopFrontier.size() ? R.hopFrontier[h] : 0),
                         static_cast<unsigned long long>(R.hopEdges[h]),
                         static_cast<unsigned long long>(h < R.hopNext.size() ? R.hopNext[h] : 0),
                         std::chrono::duration<double, std::micro>(hopT[h + 1] - hopT[h]).count());
        }
        std::fprintf(stderr, "[ngx trace_go r%d] Total rows:%llu, total time %.0fus\n", c->rank,
                     static_cast<unsigned long long>(totalRows), std::chrono::duration<double, std::micro>(R.tDone - R.tIn).count());
    }
    c->hmark("done");
    c->hflush();
    const uint64_t flags = tail[0];
    if (flags & 8u) return fail(c, NGX_E_DEVICE, "final-hop row reservation did not complete (device fault)");
    if (flags & 2u) return fail(c, NGX_E_UNSUPPORTED, "an expression needs a host-only construct (string building or parsing)");
    if (flags & 1u) return fail(c, NGX_E_QUERY, "an expression of WHERE / YIELD failed to evaluate");
    if (flags & 4u) return fail(c, NGX_E_QUERY, "YIELD value does not match its column type (boost::get)");

    int32_t nY = static_cast<int32_t>(progs.yOff.size());
    if (p.distinct && totalRows) {
        // YIELD DISTINCT (processFinalResult, GoExecutor.cpp:1298-1305) on the device: mark one row of
        // every group of equal YIELD rows, then move the kept rows of every result array together
        if (nY > kMaxDistinctCols || totalRows >= (1ULL << 32)) return fail(c, NGX_E_UNSUPPORTED, "DISTINCT over this result");
        const uint64_t n = totalRows;
        uint64_t cap = 1024;
        while (cap < 2 * n) cap <<= 1;
        DistinctArgs da{};
        da.n = n;
        da.nY = nY;
        OutCol* colsDev = c->oColDesc.get<OutCol>(std::max<int32_t>(nY, 1));
        HIP_OK(hipMemcpyAsync(colsDev, c->oColView.data(), nY * sizeof(OutCol), hipMemcpyHostToDevice, c->stream));
        da.cols = colsDev;
        for (int32_t y = 0; y < nY; y++) {
            ColView cv;
            cv.colType = gp.colTypes[y];
            da.vt[y] = cv.typeAt(0);
        }
        da.table = c->dkTable.get<uint64_t>(cap);
        HIP_OK(hipMemsetAsync(da.table, 0, cap * 8, c->stream));
        da.mask = cap - 1;
        da.keep = c->dkKeep.get<uint64_t>(n + 1);
        uint64_t* pre = c->dkPre.get<uint64_t>(n + 1);
        uint64_t* tiles = c->tileSums.get<uint64_t>((n + kTile - 1) / kTile + 1);
        c->timed("distinct", n * 8 * static_cast<uint64_t>(nY), [&] {
            if (launchDistinctMark(da, c->stream)) throw Error{NGX_E_DEVICE, "distinct"};
            if (launchScanU64(da.keep, n, pre, tiles, c->stream)) throw Error{NGX_E_DEVICE, "distinct scan"};
        });
        const uint64_t kept = readScalar(c, pre + n);
        ScatterArgs sa{};
        sa.n = n;
        sa.keep = da.keep;
        sa.pre = pre;
        auto move = [&](DBuf& from, DBuf& to, uint8_t esz) {
            if (!from.p) return;
            sa.src[sa.k] = static_cast<const uint8_t*>(from.p);
            sa.dst[sa.k] = to.get<uint8_t>(std::max<uint64_t>(kept, 1) * esz);
            sa.esz[sa.k] = esz;
            sa.k++;
        };
        move(c->oSrc, c->dSrc, 8);
        move(c->oDst, c->dDst, 8);
        move(c->oRank, c->dRank, 8);
        if (!constType) move(c->oType, c->dType, 4);
        if (c->dCols.size() < static_cast<size_t>(nY)) c->dCols.resize(nY);
        for (int32_t y = 0; y < nY; y++) {
            if (y < static_cast<int32_t>(yAlias.size()) && yAlias[y] >= 0) continue;
            if (sa.k + 3 > kMaxScatter) {
                if (launchScatterKept(sa, c->stream)) throw Error{NGX_E_DEVICE, "distinct scatter"};
                sa.k = 0;
            }
            move(c->oCols[y].x, c->dCols[y].x, 8);
            if (c->oColView[y].len) move(c->oCols[y].len, c->dCols[y].len, 4);
            if (c->oColView[y].t) move(c->oCols[y].t, c->dCols[y].t, 1);
        }
        if (launchScatterKept(sa, c->stream)) throw Error{NGX_E_DEVICE, "distinct scatter"};
        // the compacted arrays become the result arrays (the old ones are scratch for the next DISTINCT)
        std::swap(c->oSrc, c->dSrc);
        std::swap(c->oDst, c->dDst);
        std::swap(c->oRank, c->dRank);
        if (!constType) std::swap(c->oType, c->dType);
        for (int32_t y = 0; y < nY; y++) {
            OutCol& v = c->oColView[y];
            if (y < static_cast<int32_t>(yAlias.size()) && yAlias[y] >= 0) {
                v.x = static_cast<int64_t*>((yAlias[y] == 0 ? c->oSrc : yAlias[y] == 1 ? c->oDst : c->oRank).p);
                continue;
            }
            const bool hasLen = v.len != nullptr, hasT = v.t != nullptr;
            std::swap(c->oCols[y].x, c->dCols[y].x);
            if (hasLen) std::swap(c->oCols[y].len, c->dCols[y].len);
            if (hasT) std::swap(c->oCols[y].t, c->dCols[y].t);
            v.x = static_cast<int64_t*>(c->oCols[y].x.p);
            v.len = hasLen ? static_cast<uint32_t*>(c->oCols[y].len.p) : nullptr;
            v.t = hasT ? static_cast<uint8_t*>(c->oCols[y].t.p) : nullptr;
        }
        totalRows = kept;
    }
    if (p.result_on_device) {                                 // rows stay in HBM (valid until the next call)
        R.r.nrows = totalRows;
        R.r.dev_src = (rowMask & 1) ? static_cast<const int64_t*>(c->oSrc.p) : nullptr;
        R.r.dev_dst = (rowMask & 2) ? static_cast<const int64_t*>(c->oDst.p) : nullptr;
        R.r.dev_rank = (rowMask & 4) ? static_cast<const int64_t*>(c->oRank.p) : nullptr;
        R.r.dev_type = constType ? nullptr : static_cast<const int32_t*>(c->oType.p);
        R.r.dev_type_const = constType ? hs.etype[0] : 0;
        R.devCols.clear();
        for (int32_t y = 0; y < nY; y++) {
            bool have = y < static_cast<int32_t>(c->oColView.size()) && totalRows;
            R.devCols.push_back(ngx_dev_column{have ? c->oColView[y].x : nullptr, have ? c->oColView[y].len : nullptr,
                                               have ? c->oColView[y].t : nullptr});
        }
        R.r.dev_cols = R.devCols.data();
        R.devColW.assign(nY, 8);
        for (int k = 0; k < 3; k++) R.r.dev_key_w[k] = compact ? outW[k] : 8;
        for (int32_t y = 0; compact && y < nY; y++) R.devColW[y] = yW[y];
        R.devColConst.assign(nY, 0);
        if (rankConst) {                                      // the rank and the YIELD columns that alias it
            R.r.dev_key_w[2] = 0;
            R.r.dev_key_const[2] = hs.rankC[0];
            for (int32_t y = 0; y < nY; y++) {
                if (y >= static_cast<int32_t>(yAlias.size()) || yAlias[y] != 2) continue;
                R.devColW[y] = 0;
                R.devColConst[y] = hs.rankC[0];
                R.devCols[y].x = nullptr;
            }
        }
        R.r.dev_col_w = R.devColW.data();
        R.r.dev_col_const = R.devColConst.data();
        return NGX_OK;
    }
    // ---- results to the host: every array in one batch of D2H copies into page-locked staging
    const uint64_t n = totalRows;
    std::vector<HostArr> arrs;
    auto want = [&](const void* dev, size_t bytes) { arrs.push_back(HostArr{dev, bytes, nullptr}); return arrs.size() - 1; };
    size_t iSrc = want(c->oSrc.p, n * 8), iDst = want(c->oDst.p, n * 8), iRank = want(c->oRank.p, n * 8);
    size_t iType = constType ? SIZE_MAX : want(c->oType.p, n * 4);
    std::vector<size_t> iX(nY, SIZE_MAX), iLen(nY, SIZE_MAX), iT(nY, SIZE_MAX);
    for (int32_t y = 0; y < nY && n; y++) {
        if (y < static_cast<int32_t>(yAlias.size()) && yAlias[y] >= 0) continue;       // = a key array
        const OutCol& v = c->oColView[y];
        iX[y] = want(v.x, n * 8);
        if (v.len) iLen[y] = want(v.len, n * 4);
        if (v.t) iT[y] = want(v.t, n);
    }
    stageArrays(c, arrs);
    int64_t* hSrc = reinterpret_cast<int64_t*>(arrs[iSrc].host);
    int64_t* hDst = reinterpret_cast<int64_t*>(arrs[iDst].host);
    int64_t* hRank = reinterpret_cast<int64_t*>(arrs[iRank].host);
    int32_t* hType = iType == SIZE_MAX ? nullptr : reinterpret_cast<int32_t*>(arrs[iType].host);
    std::vector<ColView> cols(nY);
    for (int32_t y = 0; y < nY; y++) {
        ColView& cv = cols[y];
        cv.colType = gp.colTypes[y];
        if (y < static_cast<int32_t>(yAlias.size()) && yAlias[y] >= 0) {
            cv.x = yAlias[y] == 0 ? hSrc : yAlias[y] == 1 ? hDst : hRank;
        } else if (n) {
            cv.x = reinterpret_cast<int64_t*>(arrs[iX[y]].host);
            cv.len = iLen[y] == SIZE_MAX ? nullptr : reinterpret_cast<uint32_t*>(arrs[iLen[y]].host);
            cv.t = iT[y] == SIZE_MAX ? nullptr : reinterpret_cast<uint8_t*>(arrs[iT[y]].host);
        }
    }
    R.strings = progs.pool;                                    // string literals of YIELD, kept with the result
    // the strings YIELD columns built: each record hop's arena rows, copied next to the result
    R.built.clear();
    std::vector<StrMap::Range> builtRanges;
    for (const Arena& ar : arenas) {
        const uint64_t bytes = ar.rows * nStrOut * static_cast<uint64_t>(kStrBuildBytes);
        if (!bytes) continue;
        R.built.emplace_back(bytes, '\0');
        HIP_OK(hipMemcpyAsync(&R.built.back()[0], ar.dev, bytes, hipMemcpyDeviceToHost, c->stream));
        builtRanges.push_back(StrMap::Range{reinterpret_cast<uint64_t>(ar.dev), bytes, R.built.back().data()});
    }
    if (!builtRanges.empty()) HIP_OK(hipStreamSynchronize(c->stream));
    if (rw && rw->perRow && rw->inStrBytes)                      // YIELD $-.s: strings of the input table
        builtRanges.push_back(StrMap::Range{rw->inStrDev, rw->inStrBytes, rw->inStrHost});
    for (size_t k = 0; k < dstRec && k < c->dst.hostStr.size(); k++)   // $$ strings of the owner fetches
        if (!c->dst.hostStr[k].empty())
            builtRanges.push_back(StrMap::Range{reinterpret_cast<uint64_t>(c->dst.devStr[k]), c->dst.hostStr[k].size(),
                                                c->dst.hostStr[k].data()});
    StrMap sm{&d, reinterpret_cast<uint64_t>(dp.pool), &R.strings, &builtRanges};
    uint64_t nOut = n;
    R.r.nrows = nOut;
    R.r.dev_type_const = constType ? hs.etype[0] : 0;
    if (p.host_columnar) {
        // columnar host result, no per-cell conversion: string values become host pointers
        parallelRows(nOut, [&](uint64_t lo, uint64_t hi, int) {
            for (int32_t y = 0; y < nY; y++) {
                ColView& cv = cols[y];
                if (!cv.len) continue;
                for (uint64_t r = lo; r < hi; r++) {
                    if (cv.typeAt(r) == V_STR) cv.x[r] = reinterpret_cast<int64_t>(sm.host(static_cast<uint64_t>(cv.x[r]), cv.len[r]));
                }
            }
        });
        R.rowSrcView = hSrc; R.rowDstView = hDst; R.rowRankView = hRank; R.rowTypeView = hType;
        for (int32_t y = 0; y < nY; y++) R.hostCols.push_back(ngx_dev_column{cols[y].x, cols[y].len, cols[y].t});
        return NGX_OK;
    }
    R.src.assign(hSrc, hSrc + nOut);
    R.dst.assign(hDst, hDst + nOut);
    R.rank.assign(hRank, hRank + nOut);
    if (hType) R.type.assign(hType, hType + nOut);
    else R.type.assign(nOut, hs.etype[0]);
    // typed cells (ColumnValue, toThriftResponse) in parallel; per-thread string arenas, then appended
    R.cells.resize(nOut * nY);
    const int T = static_cast<int>(std::max<uint64_t>(1, std::min<uint64_t>(hostThreads(), (nOut + 65535) / 65536)));
    std::vector<std::string> arena(T);
    std::vector<uint8_t> bad(T, 0);
    parallelRows(nOut, [&](uint64_t lo, uint64_t hi, int t) {
        std::string& out = arena[t];
        for (uint64_t r = lo; r < hi && !bad[t]; r++) {
            for (int32_t y = 0; y < nY; y++) {
                OutCell v{cols[y].x[r], cols[y].len ? cols[y].len[r] : 0u, cols[y].typeAt(r), {0, 0, 0}};
                if (!toCell(v, gp.colTypes[y], R.cells[r * nY + y], out, sm)) { bad[t] = 1; break; }
            }
        }
    }, T);
    for (int t = 0; t < T; t++) if (bad[t]) return fail(c, NGX_E_QUERY, "YIELD value does not match its column type (boost::get)");
    {
        // arena t's offsets are relative to it: rebase onto R.strings
        std::vector<uint64_t> base(T);
        uint64_t b = R.strings.size();
        for (int t = 0; t < T; t++) { base[t] = b; b += arena[t].size(); }
        parallelRows(nOut, [&](uint64_t lo, uint64_t hi, int t) {
            for (uint64_t i = lo * nY; i < hi * nY; i++) if (R.cells[i].kind == NGX_CELL_STR) R.cells[i].v.str_off += base[t];
        }, T);
        R.strings.reserve(b);
        for (int t = 0; t < T; t++) R.strings += arena[t];
    }
    return NGX_OK;
}

// One YIELD row as a DISTINCT key: boost::hash_range over the record (GoExecutor.cpp:1298-1305), which
// treats 0.0 and -0.0 as one value; every NaN alike, as the device DISTINCT (kernels.hip dBits)
void rowKey(const GoResultHolder& S, uint64_t r, int32_t nY, std::string& key) {
    key.clear();
    for (int32_t y = 0; y < nY; y++) {
        const ngx_cell& v = S.cells[r * nY + y];
        key.push_back(static_cast<char>(v.kind));
        if (v.kind == NGX_CELL_STR) {
            uint32_t n = static_cast<uint32_t>(v.str_len);
            key.append(reinterpret_cast<const char*>(&n), 4);
            key.append(S.strings.data() + v.v.str_off, n);
            continue;
        }
        uint64_t bits = static_cast<uint64_t>(v.v.i);
        if (v.kind == NGX_CELL_DOUBLE || v.kind == NGX_CELL_FLOAT) {
            if (v.v.d == 0.0) bits = 0;
            else if (v.v.d != v.v.d) bits = 0x7FF8000000000000ULL;
        }
        key.append(reinterpret_cast<const char*>(&bits), 8);
    }
}

// GO FROM $-.col / $var.col (GoExecutor fromType_ kPipe / kVariable). The reference walks once from the
// distinct input vids, records per hop which roots reach each vertex (VertexBackTracker,
// GoExecutor.h:189-207, getDstIdsFromRespWithBackTrack :675-718) and emits each edge row once per input
// row whose vid is one of the edge's roots (getRoots + rowsOfVids, :1317-1330), evaluating `$-.x' with
// that row. Per root that is exactly a GO from the root alone: the hop-k frontier of root r is the set
// of vertices r reaches in k hops, so the rows of root r are the rows of `GO ... FROM r'. The device
// runs:
//   - one walk from all distinct vids when no expression reads the input and the sentence has one
//     step: the root of an edge row is its src, and each row is repeated once per input row of that
//     vid (the multimap order of rowsOfVid is irrelevant: results are sets of rows);
//   - one walk per distinct vid when no expression reads the input (rows repeated per input row);
//   - one walk per input row otherwise, `$-.x' bound to that row's values as constants (device
//     kernels for the query shape are reused across rows: literals travel in launch slots).
// DISTINCT (one uniqResult over the whole result, :1298-1305) is the device DISTINCT of every walk,
// then the union deduplicated here.
int32_t runPipe(ngx_ctx* c, Space& sp, const ngx_go_plan& p, GoResultHolder& R) {
    if (p.result_on_device || p.host_columnar)
        return fail(c, NGX_E_BAD_ARGUMENT, "FROM $-/$var: the result comes back as host cells (no result_on_device / host_columnar)");
    if (p.input_nrows && (p.input_ncols <= 0 || !p.input_names || !p.input_types || !p.input_cells))
        return fail(c, NGX_E_BAD_ARGUMENT, "input rows without columns");
    if (std::string(p.input_vid_col) == "*")                     // prepareFrom (GoExecutor.cpp:175-178)
        return fail(c, NGX_E_QUERY, "Can not use `*' to reference a vertex id column.");
    InputBind b;
    b.p = &p;
    b.isVar = p.input_var && p.input_var[0];
    if (b.isVar) b.var = p.input_var;
    for (int32_t i = 0; i < p.input_ncols; i++) b.colIdx[p.input_names[i] ? p.input_names[i] : ""] = i;
    // prepareClauses first: its errors come before any about the input (GoExecutor.cpp:92-97)
    GoPlan probe;
    int32_t rc = prepareGo(c, sp, p, probe, &b);
    if (rc) return rc;
    R.colTypes = probe.colTypes;
    if (p.input_nrows == 0 || p.record_to == 0) return NGX_OK;      // no data: onEmptyInputs (:119-122)
    // setupStarts (:471-509): checkIfDuplicateColumn, getDistinctVIDs (a VID or INT column,
    // RowReader::getVid), buildIndex
    if (!b.isVar && static_cast<int32_t>(b.colIdx.size()) != p.input_ncols) {    // inputs_ only
        std::set<std::string> seen;
        for (int32_t i = 0; i < p.input_ncols; i++)
            if (!seen.insert(p.input_names[i]).second) return fail(c, NGX_E_QUERY, std::string("Duplicate column `") + p.input_names[i] + "'");
    }
    const std::string col = p.input_vid_col;
    auto ci = b.colIdx.find(col);
    if (ci == b.colIdx.end() || (p.input_types[ci->second] != T_INT && p.input_types[ci->second] != T_VID))
        return fail(c, NGX_E_QUERY, "Column `" + col + "' not found");
    const int32_t vc = ci->second, nc = p.input_ncols;
    std::vector<int64_t> vids;                                   // distinct, first-seen order
    std::vector<std::vector<uint64_t>> rowsOf;
    std::unordered_map<int64_t, uint32_t> group;
    for (uint64_t r = 0; r < p.input_nrows; r++) {
        int64_t v = p.input_cells[r * nc + vc].v.i;
        auto [it, fresh] = group.emplace(v, static_cast<uint32_t>(vids.size()));
        if (fresh) { vids.push_back(v); rowsOf.emplace_back(); }
        rowsOf[it->second].push_back(r);
    }
    const bool perRow = probe.refs.input || probe.refs.variable;
    const bool oneWalk = !perRow && p.record_to == 1;
    const int32_t nY = static_cast<int32_t>(R.colTypes.size());
    std::unordered_set<std::string> seen;
    std::string key;
    bool first = true;
    // append a walk's rows, each `times(r)' times (DISTINCT: once, and only if new)
    auto absorb = [&](GoResultHolder& S, const std::function<uint64_t(uint64_t)>& times) {
        if (first) { R.tLaunch = S.tLaunch; first = false; }
        R.tDone = S.tDone;
        R.r.device_ms += S.r.device_ms;
        auto addv = [](std::vector<uint64_t>& a, const std::vector<uint64_t>& x) {
            if (a.size() < x.size()) a.resize(x.size(), 0);
            for (size_t i = 0; i < x.size(); i++) a[i] += x[i];
        };
        addv(R.hopFrontier, S.hopFrontier); addv(R.hopEdges, S.hopEdges); addv(R.hopNext, S.hopNext);
        const uint64_t base = R.strings.size();
        R.strings += S.strings;
        for (uint64_t r = 0; r < S.r.nrows; r++) {
            uint64_t k = times(r);
            if (p.distinct) {
                rowKey(S, r, nY, key);
                k = (k && seen.insert(key).second) ? 1 : 0;
            }
            for (uint64_t j = 0; j < k; j++) {
                for (int32_t y = 0; y < nY; y++) {
                    ngx_cell cl = S.cells[r * nY + y];
                    if (cl.kind == NGX_CELL_STR) cl.v.str_off += base;
                    R.cells.push_back(cl);
                }
                R.src.push_back(S.src[r]); R.dst.push_back(S.dst[r]);
                R.rank.push_back(S.rank[r]); R.type.push_back(S.type[r]);
            }
        }
    };
    ngx_go_plan sub = p;
    sub.input_vid_col = nullptr;
    sub.input_nrows = 0;
    auto walk = [&](const int64_t* starts, uint64_t n, const ngx_cell* row, GoResultHolder& S) {
        sub.starts = starts;
        sub.nstarts = n;
        b.row = row;
        S.tIn = std::chrono::steady_clock::now();
        S.tLaunch = S.tDone = S.tIn;
        return runGo(c, sp, sub, S, &b);
    };
    if (oneWalk) {
        GoResultHolder S;
        if ((rc = walk(vids.data(), vids.size(), nullptr, S))) return rc;
        c->pipeWalks++;
        absorb(S, [&](uint64_t r) { return rowsOf[group.at(S.src[r])].size(); });
    } else if (!perRow) {
        // multi-step, nothing reads the input: one multi-root walk per 64 distinct vids (root sets over
        // the frontier rows); a row from a src reached by roots R repeats once per input row of every
        // root in R. A walk the device cannot key by root (a storage mask; at world > 1 decided by all
        // shards together) falls back to a walk per vid, before any row is kept.
        bool batched = true;
        std::vector<std::pair<std::unique_ptr<GoResultHolder>, std::unique_ptr<RootWalk>>> walks;
        for (size_t b0 = 0; batched && b0 < vids.size(); b0 += 64) {
            const size_t n = std::min<size_t>(64, vids.size() - b0);
            auto rw = std::make_unique<RootWalk>();
            for (size_t j = 0; j < n; j++) rw->bitsOf[vids[b0 + j]] = 1ULL << j;
            auto S = std::make_unique<GoResultHolder>();
            sub.starts = &vids[b0];
            sub.nstarts = n;
            b.row = nullptr;
            S->tIn = std::chrono::steady_clock::now();
            S->tLaunch = S->tDone = S->tIn;
            rc = runGo(c, sp, sub, *S, &b, rw.get());
            if (rc == NGX_E_UNSUPPORTED) { batched = false; break; }
            if (rc) return rc;
            walks.emplace_back(std::move(S), std::move(rw));
        }
        if (batched) {
            c->pipeWalks += walks.size();
            for (size_t w = 0; w < walks.size(); w++) {
                GoResultHolder& S = *walks[w].first;
                const RootWalk& rw = *walks[w].second;
                const size_t b0 = w * 64;
                absorb(S, [&](uint64_t r) {
                    for (const RootWalk::Hop& hop : rw.record) {
                        if (r < hop.rowBase || r >= hop.rowBase + hop.rows) continue;
                        auto it = hop.rootsOf.find(S.src[r]);
                        uint64_t roots = it == hop.rootsOf.end() ? 0 : it->second, k = 0;
                        for (; roots; roots &= roots - 1) k += rowsOf[b0 + __builtin_ctzll(roots)].size();
                        return k;
                    }
                    return uint64_t(0);
                });
            }
        } else {
            for (size_t g = 0; g < vids.size(); g++) {
                GoResultHolder S;
                if ((rc = walk(&vids[g], 1, nullptr, S))) return rc;
                c->pipeWalks++;
                const uint64_t m = rowsOf[g].size();
                absorb(S, [&](uint64_t) { return m; });
            }
        }
    } else {
        // WHERE / YIELD read $-.x: one multi-root walk per 64 distinct vids, the input table on the
        // device and every record hop's entries keyed by (frontier row, input row) (RootWalk::perRow);
        // a walk per input row, values bound as constants, where the device cannot key a walk by root
        bool batched = true;
        for (uint64_t i = 0; batched && i < p.input_nrows * static_cast<uint64_t>(nc); i++) {
            const int32_t k = p.input_cells[i].kind;
            batched = k == NGX_CELL_BOOL || k == NGX_CELL_INT || k == NGX_CELL_ID || k == NGX_CELL_TIMESTAMP ||
                      k == NGX_CELL_FLOAT || k == NGX_CELL_DOUBLE || k == NGX_CELL_STR;
        }
        std::vector<std::pair<std::unique_ptr<GoResultHolder>, std::unique_ptr<RootWalk>>> walks;
        std::vector<std::vector<std::vector<uint32_t>>> rowsOfBit;
        const DInputCol* inputDev = nullptr;
        uint64_t inStrBytes = 0;
        if (batched) {
            // the input table: per column value bits / lengths / VM types, strings in one device pool
            const uint64_t n = p.input_nrows;
            uint64_t strBytes = 0;
            for (uint64_t i = 0; i < n * static_cast<uint64_t>(nc); i++)
                if (p.input_cells[i].kind == NGX_CELL_STR)
                    strBytes = std::max<uint64_t>(strBytes, p.input_cells[i].v.str_off + static_cast<uint64_t>(p.input_cells[i].str_len));
            inStrBytes = strBytes;
            char* dStr = c->inStr.get<char>(std::max<uint64_t>(strBytes, 1));
            int64_t* dX = c->inX.get<int64_t>(n * nc);
            uint32_t* dLen = c->inLen.get<uint32_t>(n * nc);
            uint8_t* dT = c->inT.get<uint8_t>(n * nc);
            std::vector<int64_t> hx(n * nc);
            std::vector<uint32_t> hl(n * nc, 0);
            std::vector<uint8_t> ht(n * nc);
            std::vector<DInputCol> desc(nc);
            for (int32_t col = 0; col < nc; col++) {
                desc[col] = DInputCol{dX + col * n, dLen + col * n, dT + col * n};
                for (uint64_t r = 0; r < n; r++) {
                    const ngx_cell& v = p.input_cells[r * nc + col];
                    const uint64_t at = col * n + r;
                    switch (v.kind) {
                        case NGX_CELL_BOOL: ht[at] = V_BOOL; hx[at] = v.v.i != 0; break;
                        case NGX_CELL_FLOAT: case NGX_CELL_DOUBLE: ht[at] = V_DBL; std::memcpy(&hx[at], &v.v.d, 8); break;
                        case NGX_CELL_STR:
                            ht[at] = V_STR; hl[at] = static_cast<uint32_t>(v.str_len);
                            hx[at] = reinterpret_cast<int64_t>(dStr + v.v.str_off);
                            break;
                        default: ht[at] = V_INT; hx[at] = v.v.i; break;
                    }
                }
            }
            DInputCol* dDesc = c->inDesc.get<DInputCol>(std::max<int32_t>(nc, 1));
            if (strBytes) HIP_OK(hipMemcpyAsync(dStr, p.input_strings, strBytes, hipMemcpyHostToDevice, c->stream));
            HIP_OK(hipMemcpyAsync(dX, hx.data(), hx.size() * 8, hipMemcpyHostToDevice, c->stream));
            HIP_OK(hipMemcpyAsync(dLen, hl.data(), hl.size() * 4, hipMemcpyHostToDevice, c->stream));
            HIP_OK(hipMemcpyAsync(dT, ht.data(), ht.size(), hipMemcpyHostToDevice, c->stream));
            HIP_OK(hipMemcpyAsync(dDesc, desc.data(), nc * sizeof(DInputCol), hipMemcpyHostToDevice, c->stream));
            HIP_OK(hipStreamSynchronize(c->stream));
            inputDev = dDesc;
            rowsOfBit.resize((vids.size() + 63) / 64);
        }
        for (size_t b0 = 0; batched && b0 < vids.size(); b0 += 64) {
            const size_t n = std::min<size_t>(64, vids.size() - b0);
            auto& rob = rowsOfBit[b0 / 64];
            rob.resize(n);
            auto rwk = std::make_unique<RootWalk>();
            for (size_t j = 0; j < n; j++) {
                rwk->bitsOf[vids[b0 + j]] = 1ULL << j;
                for (uint64_t r : rowsOf[b0 + j]) rob[j].push_back(static_cast<uint32_t>(r));
            }
            rwk->perRow = true;
            rwk->rowsOfBit = &rob;
            rwk->input = inputDev;
            rwk->inStrDev = reinterpret_cast<uint64_t>(c->inStr.p);
            rwk->inStrBytes = inStrBytes;
            rwk->inStrHost = p.input_strings;
            auto S = std::make_unique<GoResultHolder>();
            sub.starts = &vids[b0];
            sub.nstarts = n;
            b.row = nullptr;
            S->tIn = std::chrono::steady_clock::now();
            S->tLaunch = S->tDone = S->tIn;
            rc = runGo(c, sp, sub, *S, &b, rwk.get());
            if (rc == NGX_E_UNSUPPORTED) { batched = false; break; }
            if (rc) return rc;
            walks.emplace_back(std::move(S), std::move(rwk));
        }
        if (batched) {
            c->pipeWalks += walks.size();
            for (auto& w : walks) absorb(*w.first, [](uint64_t) { return uint64_t(1); });
        } else {
            for (size_t g = 0; g < vids.size(); g++) {
                for (uint64_t r : rowsOf[g]) {
                    GoResultHolder S;
                    if ((rc = walk(&vids[g], 1, p.input_cells + r * nc, S))) return rc;
                    c->pipeWalks++;
                    absorb(S, [](uint64_t) { return uint64_t(1); });
                }
            }
        }
    }
    R.r.nrows = R.src.size();
    return NGX_OK;
}

}  // namespace

namespace {

// ngx_go under the caller's lock of c->mu
int32_t goCall(ngx_ctx* c, const ngx_go_plan* p, ngx_go_result** out) {
    auto R = std::make_unique<GoResultHolder>();
    R->tIn = std::chrono::steady_clock::now();
    R->tLaunch = R->tDone = R->tIn;
    int32_t rc;
    try {
        if (c->broken) throw Error{NGX_E_DEVICE, "context unusable: its RCCL communicator was aborted"};
        HIP_OK(hipSetDevice(c->device));
        Space* sp = findSpace(c, p->space);
        if (!sp || !sp->dev) rc = fail(c, NGX_E_NOT_LOADED, "space not committed");
        else if (c->reservoirSampling) rc = fail(c, NGX_E_UNSUPPORTED, kSamplingRefused);
        else if (p->input_vid_col) rc = runPipe(c, *sp, *p, *R);
        else rc = runGo(c, *sp, *p, *R);
    } catch (const Error& e) {
        rc = fail(c, e.code, e.msg);
    }
    // a failed query may leave kernels enqueued that still read the page-locked seed / program stages
    // the next call rewrites: drain them first
    if (rc != NGX_OK) {
        (void)hipStreamSynchronize(c->stream);
        if (c->finalStream) (void)hipStreamSynchronize(c->finalStream);
        if (c->finalStream2) (void)hipStreamSynchronize(c->finalStream2);
    }
    R->r.code = rc;
    R->r.ncols = static_cast<int32_t>(R->colTypes.size());
    R->r.col_types = R->colTypes.data();
    R->r.cells = R->cells.data();
    R->r.row_src = R->rowSrcView ? R->rowSrcView : R->src.data();
    R->r.row_dst = R->rowDstView ? R->rowDstView : R->dst.data();
    R->r.row_rank = R->rowRankView ? R->rowRankView : R->rank.data();
    R->r.row_type = R->rowSrcView ? R->rowTypeView : R->type.data();
    R->r.host_cols = R->hostCols.empty() ? nullptr : R->hostCols.data();
    auto msBetween = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
        return std::chrono::duration<double, std::milli>(b - a).count();
    };
    R->r.host_prep_ms = msBetween(R->tIn, R->tLaunch);
    R->r.host_tail_ms = msBetween(R->tDone, std::chrono::steady_clock::now());
    R->r.strings = R->strings.data();
    R->r.strings_len = R->strings.size();
    R->r.nhops = static_cast<int32_t>(R->hopEdges.size());
    R->hopNext.resize(R->hopEdges.size(), 0);
    R->hopXchg.resize(R->hopEdges.size(), 0);
    R->r.hop_exchange_bytes = R->hopXchg.data();
    R->r.hop_frontier = R->hopFrontier.data();
    R->r.hop_edges = R->hopEdges.data();
    R->r.hop_next = R->hopNext.data();
    if (rc != NGX_OK) { R->r.nrows = 0; }
    *out = &R.release()->r;
    return rc;
}

// one query of a batch: exactly one ngx_go, its counts (and digest) kept, its result freed at once
void batchQuery(ngx_ctx* c, const ngx_go_plan* p, GoJob& j, bool digest) {
    ngx_go_result* r = nullptr;
    try {
        j.rc = goCall(c, p, &r);
        j.nrows = r ? r->nrows : 0;
        j.edges = 0;
        if (r) for (int32_t h = 0; h < r->nhops; h++) j.edges += r->hop_edges[h];
        // a result the digest does not cover (host rows, string columns) keeps zeros
        if (digest && r && j.rc == NGX_OK && p->result_on_device) {
            joinFinal(c);                               // the rows were written on the final stream
            if (resultDigest(c, r, j.digest) != NGX_OK) j.digest[0] = j.digest[1] = j.digest[2] = 0;
        }
    } catch (...) {                                     // nothing unwinds past a coroutine's entry
        j.rc = NGX_E_DEVICE;
        (void)hipStreamSynchronize(c->stream);
    }
    if (r) ngx_go_result_free(r);
}

struct BatchCo {
    ngx_ctx* c;
    GoPipe* P;
    bool digest;
};
thread_local BatchCo* tBatch = nullptr;

void batchEntry() {
    BatchCo* b = tBatch;
    GoJob* j = b->P->cur;
    batchQuery(b->c, b->P->plans[j->idx], *j, b->digest);
    j->state = GoPipe::kDone;                           // uc_link: back to the batch loop
}

// the batch's coroutine stacks (once per context): 16 MB reserved each (pages committed on first touch),
// a guard page below
bool coStacks(ngx_ctx* c) {
    for (auto& st : c->coStack) {
        if (st) continue;
        void* m = mmap(nullptr, ngx_ctx::kCoStackBytes + 4096, PROT_READ | PROT_WRITE,
                       MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE | MAP_STACK, -1, 0);
        if (m == MAP_FAILED) return false;
        (void)mprotect(m, 4096, PROT_NONE);
        st = m;
    }
    return true;
}

}  // namespace

extern "C" int32_t ngx_go(ngx_ctx* c, const ngx_go_plan* p, ngx_go_result** out) {
    std::lock_guard<std::mutex> g(c->mu);
    return goCall(c, p, out);
}

// A native host loop over prepared plans: each is exactly one ngx_go (its result freed at once), so a
// caller that drives many queries (a graphd, the bench) pays no interpreter between them. Consecutive
// pipelinable plans overlap (GoPipe above): the next query's host work and first hops are enqueued while
// this one's final hop runs. Every query's rows, counts and errors are those it has alone.
extern "C" int32_t ngx_go_batch(ngx_ctx* c, const ngx_go_plan* const* plans, int32_t n, int32_t* codes, uint64_t* nrows,
                                uint64_t* edges, uint64_t* digests) {
    // a call that fails before a query runs reports its code for every query (never zero-filled success)
    auto failAll = [&](int32_t rc) {
        for (int32_t i = 0; codes && i < n; i++) codes[i] = rc;
        for (int32_t i = 0; nrows && i < n; i++) nrows[i] = 0;
        for (int32_t i = 0; edges && i < n; i++) edges[i] = 0;
        return rc;
    };
    if (!c || (n > 0 && !plans)) return failAll(NGX_E_BAD_ARGUMENT);
    for (int32_t i = 0; i < n; i++) if (!plans[i]) return failAll(fail(c, NGX_E_BAD_ARGUMENT, "go_batch: null plan"));
    std::lock_guard<std::mutex> g(c->mu);
    int32_t first = NGX_OK;
    auto record = [&](const GoJob& j) {
        if (codes) codes[j.idx] = j.rc;
        if (nrows) nrows[j.idx] = j.nrows;
        if (edges) edges[j.idx] = j.edges;
        if (digests) for (int k = 0; k < 3; k++) digests[3 * static_cast<size_t>(j.idx) + k] = j.digest[k];
        if (j.rc != NGX_OK && first == NGX_OK) first = j.rc;
    };
    const bool pipe = c->batchPipeline && n > 1 && !c->prof && !c->htrace && !c->traceGo &&
                      c->pipeStreams[0] && c->pipeStreams[1] && c->pipeStreams[2] && c->pipeStreams[3] && c->pipeEv[0] && c->pipeEv[1] &&
                      c->pipeEv[2] && c->pipeEv[3] && c->pipeEv[4] && coStacks(c);
    if (!pipe) {
        for (int32_t i = 0; i < n; i++) {
            GoJob j;
            j.idx = i;
            batchQuery(c, plans[i], j, digests != nullptr);
            record(j);
        }
        return first;
    }
    // CU split: masked copies of the role streams (front A, final, front B), made once per split
    if (c->batchCuSplit > 0 && c->cuSplitMade != c->batchCuSplit && c->cus >= 256) {
        for (auto& st : c->splitStreams) {
            if (st) { (void)hipStreamSynchronize(st); (void)hipStreamDestroy(st); }
            st = nullptr;
        }
        const int nw = (c->cus + 31) / 32;
        std::vector<uint32_t> front(nw, 0), fin(nw, 0);
        const int period = c->cus / c->batchCuSplit;       // one group of 8 CUs of every `period` to the fronts
        for (int i = 0; i < c->cus; i++) {
            const bool toFront = (i / 8) % period == 0;
            (toFront ? front : fin)[i / 32] |= 1u << (i % 32);
        }
        bool ok = true;
        for (int k = 0; k < 4 && ok; k++)
            ok = hipExtStreamCreateWithCUMask(&c->splitStreams[k], static_cast<uint32_t>(nw), k == 1 ? fin.data() : front.data()) == hipSuccess;
        c->cuSplitMade = ok ? c->batchCuSplit : 0;
    }
    hipStream_t* roles = (c->batchCuSplit > 0 && c->cuSplitMade == c->batchCuSplit) ? c->splitStreams : c->pipeStreams;
    GoPipe P;
    P.plans = plans;
    P.n = n;
    // digests need no hold since each lane has its own result rows: a deferred query hashes its rows when it
    // resumes, and no later final hop writes them (the next query on its lane starts after it finished)
    P.holdFinals = false;
    hipStream_t ctxStream = c->stream;
    try {
        if (c->activeLane != 0) c->useLane(0);
        // both streams after the context's earlier work
        // every stream after the context's earlier work
        for (int k = 0; k < 4; k++) streamAfter(roles[k], ctxStream, c->pipeEv[2]);
    } catch (const Error& e) {
        return failAll(fail(c, e.code, e.msg));
    }
    c->stream = roles[0];
    c->finalStream = roles[1];
    // the third stream: a second front stream, or (one front stream) the close stream
    // world > 1: one front stream, so every query's collectives and the kernels around them (exchange
    // buffers, host collectives, the RCCL watchdog's stream query) stay in one order on every rank
    c->pipeFronts = c->batchFronts == 2 && c->world == 1 ? 2 : 1;
    c->closeStream = c->batchCloseStream ? roles[3] : nullptr;
    // two final streams: the fourth role stream is the second final stream; each close follows its final
    // hop on that hop's stream
    c->finalStream2 = c->batchFinals == 2 ? roles[3] : nullptr;
    if (c->finalStream2) c->closeStream = nullptr;
    BatchCo co{c, &P, digests != nullptr};
    // query i runs on lane i % lanes with the coroutine stack of that lane; up to lanes - 1 queries wait at
    // their deferral point (holding finals: one)
    const int lanes = P.holdFinals ? 2 : std::max(2, std::min<int>(c->batchLanes, ngx_ctx::kMaxLanes));
    GoJob jobs[ngx_ctx::kMaxLanes];
    auto start = [&](int32_t i) -> GoJob* {
        GoJob& j = jobs[i % lanes];
        j = GoJob{};
        j.idx = i;
        getcontext(&j.uc);
        j.uc.uc_stack.ss_sp = static_cast<char*>(c->coStack[i % lanes]) + 4096;
        j.uc.uc_stack.ss_size = ngx_ctx::kCoStackBytes;
        j.uc.uc_link = &P.main;
        makecontext(&j.uc, batchEntry, 0);
        return &j;
    };
    auto resume = [&](GoJob* j) {
        c->ptraceQuery = j->idx;
        if (c->ptrace) c->pmark("resume");
        c->useLane(j->idx % lanes);
        c->stream = roles[c->pipeFronts == 2 && (j->idx & 1) ? 2 : 0];   // query i's hops: front i % fronts
        c->finalCur = (c->finalStream2 && (j->idx & 1)) ? c->finalStream2 : c->finalStream;   // its final hop
        P.cur = j;
        tBatch = &co;
        swapcontext(&P.main, &j->uc);
        P.cur = nullptr;
        if (c->ptrace) c->pmark("yield " + std::to_string(j->state));
        return j->state;
    };
    c->pipe = &P;
    tDeferFree = true;                                  // no device-wide wait inside the batch (freeDevice)
    GoJob* waiting[ngx_ctx::kMaxLanes];                 // deferred queries, oldest first
    int nw = 0;
    auto finishOldest = [&] {
        GoJob* d = waiting[0];
        for (int k = 1; k < nw; k++) waiting[k - 1] = waiting[k];
        P.ndeferred = --nw;
        while (resume(d) != GoPipe::kDone) {}             // a query defers once; nothing else yields it
        record(*d);
    };
    GoJob* a = start(0);
    int st = resume(a);
    for (;;) {
        if (st == GoPipe::kPreFinal) {                   // a's final hop waits for the deferred queries' digests
            while (nw) finishOldest();
            st = resume(a);
            continue;
        }
        if (st == GoPipe::kDeferred) {
            // a waits for its row count while the next query runs its hops on its own lane and enqueues its
            // final hop behind a's; the oldest waiting query finishes first when every other lane is taken
            waiting[nw] = a;
            P.ndeferred = ++nw;
        } else {
            record(*a);                                   // kDone
        }
        const int32_t next = a->idx + 1;
        if (next >= n) break;
        // the query that last used the next one's lane (and coroutine) has finished
        while (nw && waiting[0]->idx + lanes <= next) finishOldest();
        a = start(next);
        st = resume(a);
    }
    while (nw) finishOldest();
    c->pipe = nullptr;
    tDeferFree = false;
    c->finalStream = nullptr;
    c->finalStream2 = nullptr;
    c->finalCur = nullptr;
    c->closeStream = nullptr;
    if (c->ptrace && !c->pmarks.empty()) {
        timespec tm, tb;
        clock_gettime(CLOCK_MONOTONIC, &tm);
        clock_gettime(CLOCK_BOOTTIME, &tb);
        std::fprintf(stderr, "[ngx pipe] clocks monotonic %lld boottime %lld\n",
                     static_cast<long long>(tm.tv_sec) * 1000000000LL + tm.tv_nsec,
                     static_cast<long long>(tb.tv_sec) * 1000000000LL + tb.tv_nsec);
        for (auto& m : c->pmarks) std::fprintf(stderr, "[ngx pipe] %lld %s\n", static_cast<long long>(m.second), m.first.c_str());
        c->pmarks.clear();
    }
    c->stream = ctxStream;
    // later calls use lane 0 and the context's stream, ordered after everything the batch enqueued
    c->useLane(0);
    try {
        streamAfter(ctxStream, roles[0], c->pipeEv[0]);
        streamAfter(ctxStream, roles[1], c->pipeEv[1]);
        streamAfter(ctxStream, roles[2], c->pipeEv[3]);
        streamAfter(ctxStream, roles[3], c->pipeEv[4]);
    } catch (const Error& e) {
        if (first == NGX_OK) first = fail(c, e.code, e.msg);
    }
    drainGraveyard();                                   // buffers replaced during the batch (one device wait)
    if (c->batchReleaseLanes) c->releasedBytes += c->releaseParked();
    return first;
}

// ============================================================================ GetNeighbors
namespace {

const std::map<std::string, int> kKeyProps = {{"_src", 0}, {"_dst", 1}, {"_rank", 2}, {"_type", 3}};

struct HostSchemaView {
    int32_t isEdge, id;
    std::vector<std::string> names;
    std::vector<int32_t> types;
};
void addSchema(GnResultHolder& R, const HostSchemaView& hv) {
    GnResultHolder::Schema s{hv.isEdge, hv.id, hv.names, {}, hv.types};
    R.schemas.push_back(std::move(s));
}

// poison_buffers: every word k_encode_rows is about to read, checked on the host first — the row's
// type and flags, and per prop column of its type the value type, and for a string its length and
// that the pointer lies in a snapshot string column or the query's literal pool. A word no kernel
// wrote still holds kPoisonByte bytes and fails here (NGX_E_DEVICE) instead of faulting the encoder.
void checkEncodeInputs(ngx_ctx* c, const RowEncArgs& e, const std::vector<int32_t>& srcs, uint64_t nrows,
                       const DeviceGraph& d, const DevPrograms& dp, const std::string& pool) {
    HIP_OK(hipStreamSynchronize(c->stream));
    auto fetch = [&](const void* dev, size_t bytes) {
        std::vector<uint8_t> h(bytes);
        if (bytes && dev) HIP_OK(hipMemcpy(h.data(), dev, bytes, hipMemcpyDeviceToHost));
        return h;
    };
    auto bad = [&](uint64_t i, const std::string& what) {
        throw Error{NGX_E_DEVICE, "encode_rows: row " + std::to_string(i) + ": " + what + " (unwritten word)"};
    };
    std::vector<uint8_t> ty = fetch(e.oType, nrows * 4), fl = fetch(e.oFlags, e.oFlags ? nrows : 0);
    const int32_t* type = reinterpret_cast<const int32_t*>(ty.data());
    struct HostCol { std::vector<uint8_t> x, len, t; };
    std::map<int32_t, HostCol> cols;
    for (int32_t s : srcs) {
        if (s < 0 || cols.count(s)) continue;
        const OutCol& oc = c->oColView.at(static_cast<size_t>(s));
        cols[s] = HostCol{fetch(oc.x, nrows * 8), fetch(oc.len, oc.len ? nrows * 4 : 0), fetch(oc.t, oc.t ? nrows : 0)};
    }
    const uint64_t pb = reinterpret_cast<uint64_t>(dp.pool);
    auto knownString = [&](uint64_t p, uint32_t len) {
        if (len == 0) return true;
        if (p >= pb && p + len <= pb + pool.size()) return true;
        for (const auto& r : d.strRanges) if (p >= r.dev && p + len <= r.dev + r.len) return true;
        return false;
    };
    for (uint64_t i = 0; i < nrows; i++) {
        int sl = -1;
        for (int s = 0; s < e.nslots; s++) if (e.etype[s] == type[i]) sl = s;
        if (sl < 0) bad(i, "edge type " + std::to_string(type[i]) + " not requested");
        const uint8_t f = fl.empty() ? 0 : fl[i];
        if (f & ~(EF_EMPTY_VALUE | EF_BAD_ROW)) bad(i, "flags " + std::to_string(f));
        if (f & EF_EMPTY_VALUE) continue;
        for (int32_t j = e.cbeg[sl]; j < e.cbeg[sl + 1]; j++) {
            const int32_t s = srcs[static_cast<size_t>(j)];
            if (s < 0) continue;
            const HostCol& hc = cols[s];
            int64_t x;
            std::memcpy(&x, hc.x.data() + i * 8, 8);
            const uint8_t t = hc.t.empty() ? V_INT : hc.t[i];
            uint32_t len = 0;
            if (!hc.len.empty()) std::memcpy(&len, hc.len.data() + i * 4, 4);
            const std::string col = "column " + std::to_string(s);
            if (t != V_INT && t != V_DBL && t != V_BOOL && t != V_STR && t != 0xFF) bad(i, col + " value type " + std::to_string(t));
            if (t == V_STR && !knownString(static_cast<uint64_t>(x), len))
                bad(i, col + " string pointer / length " + std::to_string(len));
        }
    }
}

// IdAndProp.props of every returned edge, encoded on the device (kernels.hip k_encode_rows): row
// lengths, their scan, then the bytes; copied to the result on the context's stream
void encodeEdgeRows(ngx_ctx* c, const FinalArgs& a, uint64_t nrows,
                    const std::map<int32_t, std::vector<std::pair<int32_t, int32_t>>>& respCols, GnResultHolder& R,
                    const DeviceGraph& d, const DevPrograms& dp, const std::string& pool) {
    RowEncArgs e{};
    e.n = nrows;
    e.oType = a.oType;
    e.oSrc = a.oSrc;
    e.oRank = a.oRank;
    e.oFlags = a.oFlags;
    // every column descriptor in one device table (the final kernel took the first kInlineCols by value)
    OutCol* dcols = c->oColDesc.get<OutCol>(std::max<size_t>(c->oColView.size(), 1));
    HIP_OK(hipMemcpyAsync(dcols, c->oColView.data(), c->oColView.size() * sizeof(OutCol), hipMemcpyHostToDevice, c->stream));
    e.cols = dcols;
    std::vector<int32_t> srcs, types;                     // rcSrc then rcType, slot after slot
    e.nslots = 0;
    e.cbeg[0] = 0;
    for (auto& kv : respCols) {
        if (e.nslots >= kMaxSlots) throw Error{NGX_E_UNSUPPORTED, "too many edge types in one request"};
        e.etype[e.nslots] = kv.first;
        for (auto& p : kv.second) { srcs.push_back(p.first); types.push_back(p.second); }
        e.cbeg[e.nslots + 1] = static_cast<int32_t>(srcs.size());
        e.nslots++;
    }
    srcs.insert(srcs.end(), types.begin(), types.end());
    int32_t* drc = c->rowCols.get<int32_t>(std::max<size_t>(srcs.size(), 1));
    HIP_OK(hipMemcpyAsync(drc, srcs.data(), srcs.size() * 4, hipMemcpyHostToDevice, c->stream));
    e.rcSrc = drc;
    e.rcType = drc + types.size();
    if (gPoison.load(std::memory_order_relaxed)) {
        checkEncodeInputs(c, e, std::vector<int32_t>(srcs.begin(), srcs.begin() + static_cast<std::ptrdiff_t>(types.size())),
                          nrows, d, dp, pool);
    }
    uint64_t* len = c->rowLen.get<uint64_t>(nrows + 1);
    uint64_t* off = c->rowOff.get<uint64_t>(nrows + 1);
    uint64_t* tiles = c->tileSums.get<uint64_t>((nrows + kTile - 1) / kTile + 1);
    e.rowLen = len;
    if (launchEncodeRows(e, false, c->stream)) throw Error{NGX_E_DEVICE, "row sizes"};
    if (launchScanU64(len, nrows, off, tiles, c->stream)) throw Error{NGX_E_DEVICE, "row offsets"};
    uint64_t total = readScalar(c, off + nrows);
    e.rowOff = off;
    e.out = c->rowBytes.get<uint8_t>(std::max<uint64_t>(total, 1));
    if (launchEncodeRows(e, true, c->stream)) throw Error{NGX_E_DEVICE, "rows"};
    R.edgePropsOff.resize(nrows + 1);
    R.edgeProps.resize(total);
    // the rows into pageable vectors: wait for the encode launch, then plain synchronous copies (an
    // asynchronous copy into pageable memory is staged by the runtime; keep the order explicit)
    HIP_OK(hipStreamSynchronize(c->stream));
    HIP_OK(hipMemcpy(R.edgePropsOff.data(), off, (nrows + 1) * 8, hipMemcpyDeviceToHost));
    if (total) HIP_OK(hipMemcpy(R.edgeProps.data(), e.out, total, hipMemcpyDeviceToHost));
}

// TagData rows (QueryBoundProcessor.cpp:175-204): per request vid, per tag of the response in order, the
// RowWriter row of its return columns when the vertex has a live row of the tag (collectVertexProps
// collected something: writer.size() > 1)
void encodeTagRows(const ngx_gn_request& q, const std::vector<int32_t>& tagOrder, uint64_t nF, GnResultHolder& R) {
    const int32_t nY = q.ncols;
    R.tagPropsOff.assign(1, 0);
    for (uint64_t v = 0; v < nF; v++) {
        for (int32_t t : tagOrder) {
            std::vector<int32_t> cols;
            for (int32_t i = 0; i < nY; i++) {
                if ((q.cols[i].owner == 1 || q.cols[i].owner == 2) && q.cols[i].id == t) cols.push_back(i);
            }
            if (cols.empty() || !R.vertexHasTag[v * nY + cols[0]]) continue;
            const GnResultHolder::Schema* sch = nullptr;
            for (auto& s : R.schemas) if (!s.isEdge && s.id == t) sch = &s;
            // the cord, recording a block offset after every 16 fields (RW_CLEAN_UP_WRITE)
            std::vector<uint64_t> offs;
            auto cord = [&](RowSink& s) {
                offs.clear();
                for (size_t k = 0; k < cols.size(); k++) {
                    const ngx_cell& cell = R.vertexCells[v * nY + cols[k]];
                    uint8_t vt = cell.kind == NGX_CELL_BOOL ? V_BOOL : cell.kind == NGX_CELL_DOUBLE ? V_DBL
                               : cell.kind == NGX_CELL_STR ? V_STR : V_INT;
                    int64_t x = vt == V_STR ? reinterpret_cast<int64_t>(R.strings.data() + cell.v.str_off) : cell.v.i;
                    rowField(s, vt, x, static_cast<uint32_t>(cell.str_len), sch->types[k]);
                    if (((k + 1) & 15) == 0) offs.push_back(s.n);
                }
            };
            RowSink cs{nullptr, 0};
            cord(cs);
            const int ob = rowOffsetBytes(cs.n);
            const size_t at = R.tagProps.size();
            R.tagProps.resize(at + 1 + offs.size() * ob + cs.n);
            RowSink hs{R.tagProps.data() + at, 0};
            hs.put(static_cast<uint8_t>(ob - 1));
            for (uint64_t o : offs) hs.le(o, ob);
            RowSink ws{R.tagProps.data() + at + hs.n, 0};
            cord(ws);
            R.tagPropsOff.push_back(R.tagProps.size());
            R.tagRowVertex.push_back(static_cast<uint32_t>(v));
            R.tagRowTag.push_back(t);
        }
    }
}

int32_t runGetNeighbors(ngx_ctx* c, Space& sp, const ngx_gn_request& q, GnResultHolder& R) {
    c->hmark("gn");
    DeviceGraph& d = *sp.dev;
    auto failAll = [&](int32_t code) {
        R.r.code = code;
        for (int32_t i = 0; i < q.nparts; i++) { R.failed.push_back(code); R.failed.push_back(q.parts[i]); }
        return NGX_OK;
    };
    // checkAndBuildContexts (QueryBaseProcessor.inl:66-170)
    std::map<int32_t, std::vector<int32_t>> edgeCols;            // signed type -> return column indices
    std::set<int32_t> tagCols;
    StorageCtx sctx;
    sctx.sp = &sp;
    sctx.deviceLibm = c->deviceLibm;
    for (int32_t i = 0; i < q.nedge_types; i++) edgeCols[q.edge_types[i]];
    for (int32_t i = 0; i < q.ncols; i++) {
        const ngx_prop_def& col = q.cols[i];
        std::string name = col.name ? col.name : "";
        if (col.owner == 1 || col.owner == 2) {
            const SchemaSet* ts = sp.tag(col.id);
            if (!ts) return failAll(NGX_E_TAG_PROP_NOT_FOUND);
            if (ts->latest().typeOf(name) == T_UNKNOWN) return failAll(NGX_E_IMPROPER_DATA_TYPE);
            tagCols.insert(col.id);
        } else {
            const SchemaSet* es = sp.edge(std::abs(col.id));
            if (!es) return failAll(NGX_E_EDGE_NOT_FOUND);
            sctx.edgeMap[es->name] = std::abs(col.id);
            if (!kKeyProps.count(name) && es->latest().typeOf(name) == T_UNKNOWN) return failAll(NGX_E_IMPROPER_DATA_TYPE);
            edgeCols[col.id].push_back(i);
        }
    }
    sctx.haveEdgeContexts = !edgeCols.empty();
    Programs progs;
    std::string err;
    if (q.filter && q.filter_len) {
        auto f = decodeExpr(q.filter, q.filter_len, err);
        if (!f) return failAll(NGX_E_INVALID_FILTER);
        Program pp;
        int32_t crc = compileStorage(*f, sctx, pp, err);
        if (crc == NGX_E_INVALID_FILTER) return failAll(NGX_E_INVALID_FILTER);
        if (crc) return fail(c, crc, err);
        progs.P = progs.add(pp);
        for (int32_t t : sctx.filterTags) {
            if (!tagCols.count(t)) {                              // processVertex: no response schema
                for (int32_t i = 0; i < q.nparts; i++) {
                    if (q.part_nvids[i]) { R.failed.push_back(-25); R.failed.push_back(q.parts[i]); }
                }
                return NGX_OK;
            }
        }
    }
    const int64_t edgeCap = (q.max_edges_per_vertex > 0 && q.max_edges_per_vertex < INT32_MAX) ? q.max_edges_per_vertex
                                                                                               : INT32_MAX;
    // response schemas (buildTTLInfoAndRespSchema, QueryBaseProcessor.inl:670-797): per edge type its
    // return columns but _dst, in request order; per tag its return columns, tags in first-appearance order
    std::map<int32_t, std::vector<std::pair<int32_t, int32_t>>> respCols;    // type -> (source, field type)
    std::vector<int32_t> tagOrder;
    if (q.encode_rows) {
        for (auto& kv : edgeCols) {
            std::vector<std::pair<int32_t, int32_t>> rc;
            HostSchemaView hv{1, kv.first};
            for (int32_t ci : kv.second) {
                std::string name = q.cols[ci].name;
                if (name == "_dst") continue;
                int32_t src = name == "_src" ? kRcSrc : name == "_rank" ? kRcRank : name == "_type" ? kRcType : ci;
                int32_t ft = name == "_src" ? T_VID : (name == "_rank" || name == "_type") ? T_INT
                                                     : sp.edge(std::abs(kv.first))->latest().typeOf(name);
                rc.push_back({src, ft});
                hv.names.push_back(name);
                hv.types.push_back(ft);
            }
            if (rc.empty()) continue;
            if (rc.size() > static_cast<size_t>(kMaxRespCols)) return fail(c, NGX_E_UNSUPPORTED, "too many return columns of one edge type");
            respCols[kv.first] = rc;
            addSchema(R, hv);
        }
        for (int32_t i = 0; i < q.ncols; i++) {
            if (q.cols[i].owner != 1 && q.cols[i].owner != 2) continue;
            if (std::find(tagOrder.begin(), tagOrder.end(), q.cols[i].id) == tagOrder.end()) tagOrder.push_back(q.cols[i].id);
        }
        for (int32_t t : tagOrder) {
            HostSchemaView hv{0, t};
            for (int32_t i = 0; i < q.ncols; i++) {
                if ((q.cols[i].owner != 1 && q.cols[i].owner != 2) || q.cols[i].id != t) continue;
                hv.names.push_back(q.cols[i].name);
                hv.types.push_back(sp.tag(t)->latest().typeOf(q.cols[i].name));
            }
            addSchema(R, hv);
        }
    }
    const int64_t now = q.now_sec > 0 ? q.now_sec : static_cast<int64_t>(std::time(nullptr));    // WallClock
    // processed types: edge contexts with props (QueryBoundProcessor.cpp:65-81)
    std::vector<int32_t> types;
    for (auto& kv : edgeCols) if (!kv.second.empty()) types.push_back(kv.first);
    // column programs: collectProps semantics (key props from the key, others value-or-default)
    std::vector<int32_t> ySlotType;
    for (int32_t i = 0; i < q.ncols; i++) {
        const ngx_prop_def& col = q.cols[i];
        Program yp;
        Insn in{};
        std::string name = col.name ? col.name : "";
        if (col.owner == 3) {
            auto kp = kKeyProps.find(name);
            if (kp != kKeyProps.end()) { in.op = OP_EKEY; in.a = kp->second; in.b = 0; }
            else {
                in.op = OP_ECOL;
                in.a = sp.edge(std::abs(col.id))->latest().index(name);
                in.b = std::abs(col.id);
                in.mode = 2;
            }
            ySlotType.push_back(col.id);
        } else {
            in.op = OP_ERR;                                       // per-vertex columns: k_vertex_cells
            ySlotType.push_back(INT32_MIN);
        }
        yp.code.push_back(in);
        Insn end{};
        yp.code.push_back(end);
        progs.yOff.push_back(progs.add(yp));
    }
    DevPrograms dp = uploadPrograms(c, progs, ySlotType);
    c->hmark("progs");
    // seeds in request order; a part this shard does not hold fails with E_PART_NOT_FOUND (NebulaStore::
    // prefix -> ERR_PART_NOT_FOUND, BaseProcessor::to; QueryBaseProcessor.inl:835-851) and its vids match
    // no vertex row
    std::vector<int32_t> sparts;
    std::vector<int64_t> svids;
    uint64_t k = 0;
    for (int32_t i = 0; i < q.nparts; i++) {
        int32_t part = q.parts[i];
        bool held = sp.numParts <= 0 ||                                   // test-only layouts: every part
                    (part >= 1 && part <= sp.numParts && part % c->world == c->rank);
        if (!held && q.part_nvids[i]) { R.failed.push_back(NGX_E_PART_NOT_FOUND); R.failed.push_back(part); }
        for (uint32_t j = 0; j < q.part_nvids[i]; j++) {
            sparts.push_back(held ? part : INT32_MIN);
            svids.push_back(q.vids[k++]);
        }
    }
    uint64_t nF = svids.size();
    uint32_t* F = c->F0.get<uint32_t>(std::max<uint64_t>(nF, 1));
    if (nF) {
        int32_t* dpart = c->seedPart.get<int32_t>(nF);
        int64_t* dv = c->seedVid.get<int64_t>(nF);
        stageSeeds(c, sparts, svids, dpart, dv);
        if (launchIndexLookup(dpart, dv, nF, d.vindex, F, c->stream)) throw Error{NGX_E_DEVICE, "lookup"};
    }
    std::vector<int32_t> hopTypes;
    HopSlots hs = makeHopSlots(sp, d, types, hopTypes);
    uint64_t* counters = c->counters.get<uint64_t>(8);
    uint32_t* errFlag = reinterpret_cast<uint32_t*>(counters + 4);
    HIP_OK(hipMemsetAsync(counters, 0, 64, c->stream));
    // per-vertex tag columns (k_vertex_cells), launched now; their cells come back with the edge arrays
    const int32_t nY = q.ncols;
    OutCell* vcellsDev = nullptr;
    if (nF && nY) {
        std::vector<int32_t> tslot(nY, -1), tcol(nY, 0);
        for (int32_t i = 0; i < nY; i++) {
            if (q.cols[i].owner == 1 || q.cols[i].owner == 2) {
                tslot[i] = sp.tagSlotOf(q.cols[i].id);
                tcol[i] = sp.tag(q.cols[i].id)->latest().index(q.cols[i].name);
            }
        }
        int32_t* dts = c->misc.get<int32_t>(2 * nY);
        std::vector<int32_t> both(tslot);
        both.insert(both.end(), tcol.begin(), tcol.end());
        HIP_OK(hipMemcpyAsync(dts, both.data(), both.size() * 4, hipMemcpyHostToDevice, c->stream));
        VertexCellArgs va{};
        va.rows = F; va.n = nF; va.ncols = nY; va.tagSlot = dts; va.col = dts + nY;
        va.env = VmEnv{d.dslots, d.dtags, d.dcols, dp.pool, errFlag + 1, now, d.dtags, d.dcols};
        va.out = vcellsDev = c->vcells.get<OutCell>(nF * nY);
        if (launchVertexCells(va, c->stream)) throw Error{NGX_E_DEVICE, "vertex cells"};
    }

    uint64_t nEnt = nF * static_cast<uint64_t>(hs.n);
    uint64_t E = 0;
    uint64_t* estart = c->estart.get<uint64_t>(nEnt + 1);
    if (nEnt) {
        uint64_t* tiles = c->tileSums.get<uint64_t>((nEnt + kTile - 1) / kTile + 1);
        Publish pub = nextPub(c);                                 // E published to host-mapped memory
        if (launchDegreeScan(F, nEnt, hs, estart, tiles, c->stream, pub)) throw Error{NGX_E_DEVICE, "degree"};
        E = awaitPub(c, pub, estart + nEnt);
    }
    c->hmark("E");
    uint64_t nrows = 0;
    StagedCells staged;
    std::vector<char*> vhost;                                     // staged flags / vertex cells, if rows came back
    uint32_t flagsHost[4];
    if (E) {
        uint64_t chunks = (E + kChunk - 1) / kChunk;
        uint64_t* chunkFirst = c->chunkFirst.get<uint64_t>(chunks);
        uint64_t* lb = lookBack(c, chunks);
        if (launchChunkFirst(estart, nEnt, chunkFirst, c->stream, lb, lookBackWords(chunks))) throw Error{NGX_E_DEVICE, "chunk first"};
        FinalArgs a{};
        a.F = F; a.estart = estart; a.chunkFirst = chunkFirst; a.nEnt = nEnt; a.E = E; a.hs = hs;
        a.vid = d.vid; a.V = d.V; a.gbase = d.gbase;
        a.env = VmEnv{d.dslots, d.dtags, d.dcols, dp.pool, errFlag + 1, now, d.dtags, d.dcols};
        a.P = progs.P >= 0 ? dp.code + progs.P : nullptr;
        a.W = nullptr;
        for (int s = 0; s < hs.n; s++) {
            bool onlyStructure = true;
            for (int32_t ci : edgeCols[hs.etype[s]]) if (std::string(q.cols[ci].name) != "_dst") onlyStructure = false;
            if (!onlyStructure) a.propsMask |= 1u << s;
            if (ttlInfo(sp.edge(std::abs(hs.etype[s])), a.ttlCol[s], a.ttlDur[s])) a.ttlMask |= 1u << s;
        }
        a.now = now;
        a.err = errFlag;
        if (edgeCap < INT32_MAX) {                                // max_edge_returned_per_vertex (.inl:501-505)
            uint8_t* m = c->edgeMask.get<uint8_t>(E);
            if (launchStoragePass(a, m, c->stream)) throw Error{NGX_E_DEVICE, "storage pass"};
            if (launchCap(estart, nEnt, m, edgeCap, c->stream)) throw Error{NGX_E_DEVICE, "cap"};
            a.mask = m;
        }
        a.nY = nY;
        a.yCode = dp.code;
        a.yOff = dp.yOff;
        a.ySlotType = dp.ySlotType;
        a.oBase = 0;
        a.oSrc = c->oSrc.get<int64_t>(E);
        a.oDst = c->oDst.get<int64_t>(E);
        a.oRank = c->oRank.get<int64_t>(E);
        a.oType = c->oType.get<int32_t>(E);
        a.oEntry = c->oEntry.get<uint32_t>(E);
        a.oFlags = q.encode_rows ? c->oFlags.get<uint8_t>(E) : nullptr;
        std::vector<ColSpec> spec(nY, ColSpec{true, true});   // raw value cells: every column typed per row
        prepareCols(c, a, spec, E, 0);
        a.lbStatus = lb;
        // a generated kernel for the request shape (the interpreter's per-instruction loads serialize a
        // chunk's edges: 170 us for 25 K edges); a masked request (max-edges cap) stays on the interpreter
        std::shared_ptr<const JitKernels> jk;
        if (c->jitOn && !a.mask) {
            JitQuery jq = jitHopQuery(sp, hs, progs);
            jq.fidx = true;
            jq.yColType.assign(nY, 0);
            jq.yKey.assign(nY, -1);
            for (int32_t y = 0; y < nY; y++) {
                int32_t st = ySlotType[y];
                if (hs.n == 1 && st == hs.etype[0]) st = 0;   // every edge is of the column's type
                if (st != INT32_MIN && hs.n == 1 && st != 0) st = INT32_MIN;   // a type this request skips
                jq.ySlot.push_back(st);
            }
            std::vector<int64_t> kc;
            std::vector<uint32_t> kl;
            jitSlotConsts(jq, kc, kl);
            for (size_t k = 0; k < kc.size(); k++) { a.kc[k] = kc[k]; a.kl[k] = kl[k]; }
            std::string jerr;
            c->jit.releaseRetired(c->stream, c->finalStream, c->finalStream2);
            jk = c->jit.get(jitShapeKey(sp, jq), [&] { return jitSource(sp, jq); }, jerr);
        }
        if (jk) {
            void* args[] = {&a};
            HIP_OK(hipModuleLaunchKernel(jk->final, static_cast<unsigned>(chunks), 1, 1, 256, 1, 1, 0, c->stream, args, nullptr));
        } else if (launchFinal(a, c->stream)) {
            throw Error{NGX_E_DEVICE, "final"};
        }
        nrows = readScalar(c, a.lbStatus + chunks) & ((1ULL << 62) - 1);
        c->hmark("rows");
        R.edgeVertex.resize(nrows);
        R.edgeType.resize(nrows);
        R.edgeDst.resize(nrows);
        if (nrows) {
            // the per-edge arrays staged with the cells (a pageable destination makes each copy a
            // synchronous staged transfer)
            std::vector<HostArr> ex{{a.oEntry, nrows * 4, nullptr}, {a.oType, nrows * 4, nullptr}, {a.oDst, nrows * 8, nullptr},
                                    {errFlag, 16, nullptr}};
            if (vcellsDev) ex.push_back(HostArr{vcellsDev, nF * nY * sizeof(OutCell), nullptr});
            staged = stageCells(c, spec, std::vector<int32_t>(nY, T_UNKNOWN), nrows, 0, ex);
            for (size_t i = 3; i < ex.size(); i++) vhost.push_back(ex[i].host);
            std::memcpy(R.edgeVertex.data(), ex[0].host, nrows * 4);
            std::memcpy(R.edgeType.data(), ex[1].host, nrows * 4);
            std::memcpy(R.edgeDst.data(), ex[2].host, nrows * 8);
            if (q.encode_rows) encodeEdgeRows(c, a, nrows, respCols, R, d, dp, progs.pool);
            HIP_OK(hipStreamSynchronize(c->stream));
            c->hmark("d2h");
            // IdAndProp.dst is set only by a `_dst` return column of the edge type (PropsCollector::
            // collectDstId, Collector.h:77-82); without one the reference leaves it 0
            std::set<int32_t> withDst;
            for (auto& kv : edgeCols)
                for (int32_t ci : kv.second) if (std::string(q.cols[ci].name) == "_dst") withDst.insert(kv.first);
            for (uint64_t i = 0; i < nrows; i++) if (!withDst.count(R.edgeType[i])) R.edgeDst[i] = 0;
        }
    }
    // per-vertex tag cells and the error flags: staged with the edge arrays when there are rows,
    // otherwise on their own (one synchronisation either way)
    std::vector<OutCell> vraw(nF * std::max(nY, 1));
    {
        std::vector<HostArr> tail{{errFlag, 16, nullptr}};
        if (vcellsDev) tail.push_back(HostArr{vcellsDev, nF * nY * sizeof(OutCell), nullptr});
        if (!vhost.empty()) {
            for (size_t i = 0; i < tail.size(); i++) tail[i].host = vhost[i];
        } else {
            stageArrays(c, tail);
        }
        std::memcpy(flagsHost, tail[0].host, 16);
        if (vcellsDev) std::memcpy(vraw.data(), tail[1].host, nF * nY * sizeof(OutCell));
    }
    c->hmark("vcells");
    uint32_t flags[4];
    std::memcpy(flags, flagsHost, 16);
    if (flags[3]) throw Error{NGX_E_DEVICE, "final-hop look-back did not complete (device fault)"};
    if (flags[1]) throw Error{NGX_E_UNSUPPORTED, "a return column needs a host-only construct"};
    R.edgeCells.resize(nrows * nY);
    {
        // typed cells on host threads, per-thread string arenas appended in order afterwards
        const int T = static_cast<int>(std::max<uint64_t>(1, std::min<uint64_t>(hostThreads(), (nrows * nY) / 65536 + 1)));
        std::vector<std::string> arena(T);
        parallelRows(nrows, [&](uint64_t lo, uint64_t hi, int t) {
            // column by column: each staged array is read front to back
            for (int32_t y = 0; y < nY; y++) {
                const int64_t* x = staged.x[y];
                const uint32_t* ln = staged.len[y];
                const uint8_t* ty = staged.t[y];
                const uint8_t st = staged.st[y];
                for (uint64_t r = lo; r < hi; r++) {
                    OutCell v;
                    v.x = x[r];
                    v.len = ln ? ln[r] : 0;
                    v.t = ty ? ty[r] : st;
                    rawCell(v, R.edgeCells[r * nY + y], arena[t], d, dp, progs.pool);
                }
            }
        }, T);
        std::vector<uint64_t> base(T);
        for (int t = 0; t < T; t++) { base[t] = R.strings.size(); R.strings += arena[t]; }
        parallelRows(nrows, [&](uint64_t lo, uint64_t hi, int t) {
            for (uint64_t i = lo * nY; i < hi * nY; i++) if (R.edgeCells[i].kind == NGX_CELL_STR) R.edgeCells[i].v.str_off += base[t];
        }, T);
    }
    R.vertexCells.resize(nF * nY);
    R.vertexHasTag.assign(nF * nY, 0);
    for (uint64_t i = 0; i < nF * static_cast<uint64_t>(nY); i++) {
        rawCell(vraw[i], R.vertexCells[i], R.strings, d, dp, progs.pool);
        R.vertexHasTag[i] = vraw[i].t != 0xFF ? 1 : 0;
    }
    c->hmark("cells");
    R.r.nvertices = static_cast<uint32_t>(nF);
    R.r.nedges = nrows;
    if (q.encode_rows) {
        if (R.edgePropsOff.empty()) R.edgePropsOff.assign(nrows + 1, 0);
        encodeTagRows(q, tagOrder, nF, R);
    }
    return NGX_OK;
}

}  // namespace

extern "C" int32_t ngx_get_neighbors(ngx_ctx* c, const ngx_gn_request* q, ngx_gn_result** out) {
    const auto tIn = std::chrono::steady_clock::now();
    std::lock_guard<std::mutex> g(c->mu);
    auto R = std::make_unique<GnResultHolder>();
    int32_t rc;
    try {
        HIP_OK(hipSetDevice(c->device));
        Space* sp = findSpace(c, q->space);
        if (!sp || !sp->dev) rc = fail(c, NGX_E_NOT_LOADED, "space not committed");
        else if (c->reservoirSampling) rc = fail(c, NGX_E_UNSUPPORTED, kSamplingRefused);
        else rc = runGetNeighbors(c, *sp, *q, *R);
    } catch (const Error& e) {
        rc = fail(c, e.code, e.msg);
    }
    if (rc != NGX_OK) (void)hipStreamSynchronize(c->stream);     // as ngx_go: no kernel left reading the stages
    c->hmark("end");
    c->hflush();
    if (rc != NGX_OK) R->r.code = rc;
    R->r.nfailed = static_cast<int32_t>(R->failed.size() / 2);
    R->r.failed_codes = R->failed.data();
    R->r.edge_vertex = R->edgeVertex.data();
    R->r.edge_type = R->edgeType.data();
    R->r.edge_dst = R->edgeDst.data();
    R->r.ncols = q->ncols;
    R->r.edge_cells = R->edgeCells.data();
    R->r.vertex_cells = R->vertexCells.data();
    R->r.vertex_has_tag = R->vertexHasTag.data();
    R->r.strings = R->strings.data();
    R->r.strings_len = R->strings.size();
    if (q->encode_rows) {
        R->r.edge_props = R->edgeProps.data();
        R->r.edge_props_off = R->edgePropsOff.data();
        for (auto& sc : R->schemas) {
            sc.cnames.clear();
            for (auto& n : sc.names) sc.cnames.push_back(n.c_str());
            R->schemaView.push_back(ngx_schema_def{sc.isEdge, sc.id, static_cast<int32_t>(sc.names.size()),
                                                   sc.cnames.data(), sc.types.data()});
        }
        R->r.nschemas = static_cast<int32_t>(R->schemaView.size());
        R->r.schemas = R->schemaView.data();
        R->r.ntag_rows = static_cast<uint32_t>(R->tagRowVertex.size());
        R->r.tag_row_vertex = R->tagRowVertex.data();
        R->r.tag_row_tag = R->tagRowTag.data();
        R->r.tag_props = R->tagProps.data();
        R->r.tag_props_off = R->tagPropsOff.data();
    }
    // onFinished (BaseProcessor.h:51-60): latency_in_us, and the get_bound stats (ok = no failed part)
    const int64_t us = std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - tIn).count();
    R->r.latency_in_us = us;
    if (rc == NGX_OK && R->failed.empty()) c->gbStats.qps++;
    else c->gbStats.errorQps++;
    c->gbStats.latencySum += us;
    c->gbStats.latencyCount++;
    c->gbStats.latencyMax = std::max(c->gbStats.latencyMax, us);
    *out = &R.release()->r;
    return rc;
}

extern "C" int32_t ngx_stats(ngx_ctx* c, const ngx_stat** out, int32_t* n) {
    if (!c || !out || !n) return NGX_E_BAD_ARGUMENT;
    std::lock_guard<std::mutex> g(c->mu);
    c->statList = {{"storage_get_bound_qps", c->gbStats.qps},
                   {"storage_get_bound_error_qps", c->gbStats.errorQps},
                   {"storage_get_bound_latency_us_sum", c->gbStats.latencySum},
                   {"storage_get_bound_latency_us_count", c->gbStats.latencyCount},
                   {"storage_get_bound_latency_us_max", c->gbStats.latencyMax}};
    *out = c->statList.data();
    *n = static_cast<int32_t>(c->statList.size());
    return NGX_OK;
}
