// Per-query final-hop kernels: WHERE / YIELD bytecode -> straight-line HIP C++ -> hipRTC -> module.
//
// The generated evaluator calls the same op helpers as the interpreter (vm.h) with the opcodes,
// column types and constants as literals, so the type dispatch and the operand stack fold away and
// the evaluation stays in registers. Kernels are cached per generated source; a compile failure
// falls back to the precompiled interpreter kernels (still on the device).
#pragma once

#include <hip/hip_runtime.h>

#include <condition_variable>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "ngx_internal.h"

namespace ngx {

struct JitKernels {
    hipModule_t mod = nullptr;
    hipFunction_t final = nullptr;      // the fused final-hop kernel (final_kernels.h finalBody)
};

// one compiled program segment of a query: code[off ...] up to OP_END
struct JitProgram {
    const Insn* code = nullptr;     // host copy
    bool present = false;
};

struct JitQuery {
    JitProgram P, W;
    // PUSH literals passed at launch (FinalArgs::kc/kl) instead of being compiled in, so queries that
    // differ only in literals share one kernel: instruction -> slot (< kJitConsts); others are inlined
    std::map<const Insn*, int32_t> constSlot;
    std::vector<JitProgram> Y;
    std::vector<int32_t> yColType;  // calculateExprType per column
    std::vector<int32_t> yKey;      // >= 0: column is the edge's key prop (0 src, 1 dst, 2 rank), written
                                    // once as oSrc/oDst/oRank and aliased, not stored again (engine.cpp keyAliases)
    bool oneSlot = false;           // the hop expands a single edge-type slot (ONE kernels)
    bool pos32 = false;             // every CSR position of the hop's slots fits 32 bits (ChunkMap P32)
    int dstW = 0, rankW = 0;        // key column widths shared by every slot of the hop (0: per slot)
    bool rankConst = false;         // no slot of the hop has a rank column (HopSlots::rankC)
    std::vector<int32_t> slots;     // the hop's slots (HostGraph::slots indices)
    bool ttl = false;               // some slot's edge type has TTL info
    int32_t etype0 = 0;             // the only slot's signed type (0: several slots)
    bool dstReplica = false;        // $$ props read the cross-shard replicas (8-byte, may lack values)
    int32_t rowMask = 7;            // row arrays written: 1 src, 2 dst, 4 rank (ngx_go_plan::yield_only)
    int32_t ntStore = 0;            // result stores non-temporal (flag final_nt_stores)
    int32_t ntLoad = 0;             // global loads non-temporal, vm.h gld (flag final_nt_loads)
    bool fidx = false;              // GetNeighbors kernel: request-ordered rows with their frontier index
    bool input = false;             // GO over frontier entries that carry input rows (OP_INPUT, FinalArgs::fin)
    std::vector<int32_t> ySlot;     // per column: 0 any edge, else the signed type whose edges it reads
                                    // (others get an empty cell); INT32_MIN: never an edge column
    int32_t outW[3] = {8, 8, 8};    // bytes per row of the src / dst / rank arrays (compact results)
    std::vector<int32_t> yW;        // bytes per value of each stored column (empty or 8: int64 bits)
};

class JitCache {
public:
    ~JitCache();
    // nullptr when compilation failed (err set). Kernels are cached by query shape (jitShapeKey), at most
    // `capacity` modules, least recently used evicted first. An evicted module is retired, not unloaded:
    // a query may still hold it (a later get() of the same query can evict an entry an earlier one
    // returned), and releaseRetired() unloads the retired modules at the start of the next query, after
    // the context's stream has drained; the returned handle keeps its descriptor alive meanwhile.
    // `source` generates the hipRTC source on a miss. With `async` set, a miss queues the compile on a
    // background thread and returns nullptr at once (err "jit: compiling"): the query runs on the
    // interpreter kernels and a later query of the same shape finds the module (hipRTC's ~170 ms stays
    // off the query's critical path). Finished modules enter the cache only inside get(), on the
    // caller's thread, so a module in use by the calling query is never evicted under it.
    std::shared_ptr<const JitKernels> get(const std::string& shape, const std::function<std::string()>& source,
                                          std::string& err);
    // unload the modules evicted since the last call (synchronises `s` first when there are any)
    void releaseRetired(hipStream_t s, hipStream_t s2 = nullptr, hipStream_t s3 = nullptr);   // s2, s3: other streams that may run them
    // block until every queued compile has finished (tests, warm-up)
    void drain();
    uint64_t compiled = 0, hits = 0, failed = 0, evicted = 0;
    double compileSeconds = 0;
    int64_t lastRegs = -1, lastScratch = -1;    // hipFuncGetAttribute of the last compiled kernel
    size_t capacity = 64;
    bool async = false;
    int device = 0;                             // HIP device the background thread loads modules on
    size_t size() const { return cache_.size(); }

private:
    struct Entry { std::shared_ptr<JitKernels> k; uint64_t used = 0; };
    std::vector<hipModule_t> retired_;
    struct Done { std::string shape; JitKernels k; std::string err; double seconds; int64_t regs, scratch; };
    void admit();                               // finished background compiles -> cache_ / failures_
    void insert(const std::string& shape, const JitKernels& k);
    uint64_t tick_ = 0;
    std::map<std::string, Entry> cache_;
    std::map<std::string, std::string> failures_;
    // background compiler
    std::mutex mu_;
    std::condition_variable cv_;
    std::thread worker_;
    bool stop_ = false;
    size_t busy_ = 0;                           // jobs queued or compiling
    std::vector<std::pair<std::string, std::string>> jobs_;   // (shape, full source)
    std::vector<Done> done_;
    std::map<std::string, bool> pending_;
};

// C++ source of the evaluator struct + kernels for one query on one space snapshot (without the
// common device headers, which JitCache::get prepends when it compiles)
std::string jitSource(const Space& sp, const JitQuery& q);
// everything jitSource depends on, compactly: snapshot generation, programs (slotted literals as slot
// numbers), column types, key aliases, hop flags
std::string jitShapeKey(const Space& sp, const JitQuery& q);

}  // namespace ngx
