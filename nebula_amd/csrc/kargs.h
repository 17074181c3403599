// Kernel argument blocks shared by the precompiled kernels (kernels.hip) and the per-query
// kernels generated at run time (jit.cpp, hipRTC). Plain structs passed by value.
#pragma once

#include "vm.h"

namespace ngx {

// the edge-type slots one hop expands (by value in kernel arguments)
struct HopSlots {
    int32_t n;
    int32_t slotIdx[kMaxSlots];         // index into the DSlot table
    int32_t etype[kMaxSlots];
    const uint64_t* off[kMaxSlots];
    const uint32_t* dgid[kMaxSlots];
    const void* dst[kMaxSlots];         // at dstW / rankW bytes per element (DSlot)
    const void* rank[kMaxSlots];
    int8_t dstW[kMaxSlots];
    int8_t rankW[kMaxSlots];
    int64_t rankC[kMaxSlots];           // the slot's one rank when rank[s] == nullptr (no rank column in HBM)
    const uint8_t* eflags[kMaxSlots];   // per-edge EF_* flags, nullptr when the slot has none
    int32_t colBase[kMaxSlots];         // first DCol of the slot in the column table
};

struct OutCell {                        // raw VM value of one YIELD / return column
    int64_t x;
    uint32_t len;
    uint8_t t;                          // V_*; 0xFF: no value (column of another edge type / no tag row)
    uint8_t pad[3];
};

// One YIELD / return column of the result, columnar in HBM (row o at index oBase + o).
struct OutCol {
    int64_t* x;                         // value bits: int, double bits, bool 0/1, string device pointer
    uint32_t* len;                      // string lengths; nullptr when the column holds no strings
    uint8_t* t;                         // V_* (0xFF none) per row; nullptr when every row has the column's static type
    int32_t w;                          // bytes per x element: 1, 2 or 4 (compact integer results, signed), else 8
    int32_t pad;
};

constexpr int kJitConsts = 24;          // PUSH literals a generated kernel reads from its arguments
constexpr int kInlineCols = 12;         // result column descriptors passed in the arguments themselves

struct FinalArgs {
    const uint32_t* F;                  // frontier rows
    const uint64_t* estart;             // exclusive prefix of entry degrees, [nEnt] = E
    const uint64_t* chunkFirst;         // entry holding the first edge of each CE-edge chunk
    const uint64_t* ebase;              // optional: per entry, its CSR position (hs.off[s][F[i]]); null: read off[]
    uint64_t nEnt;
    uint64_t E;
    HopSlots hs;
    const int64_t* vid;                 // vertex table (src vid of an edge)
    uint64_t V;
    uint64_t gbase;
    VmEnv env;
    const Insn* P;                      // pushed storage filter, nullptr if none
    const Insn* W;                      // graphd WHERE, nullptr if none
    uint32_t propsMask;                 // hop slot s reads rows (not onlyStructure)
    uint32_t ttlMask;                   // hop slot s has TTL info: rows are read even without props
    int32_t ttlCol[kMaxSlots];          // TTL column of hop slot s (INT / TIMESTAMP / VID), -1 if none
    int64_t ttlDur[kMaxSlots];
    int64_t now;
    uint64_t* lbStatus;                 // GetNeighbors: [0] chunk ticket, [1 + c] look-back status of chunk c
    uint32_t* err;                      // [0] graphd evaluation error, [1] host-only construct, [2] YIELD type
                                        // mismatch, [3] look-back spin limit (device fault)
    int32_t nY;
    const Insn* yCode;
    const int32_t* yOff;
    const int32_t* ySlotType;           // 0 = any type; else the column belongs to this signed type
    const int32_t* yColType;            // calculateExprType per column (0 UNKNOWN: any value type), may be null
    uint32_t wIsP;                      // WHERE == pushed filter: W is implied by P where P was evaluated
    uint64_t oBase;                     // first output row of this launch (earlier record hops before it)
    int64_t* oSrc;                      // row arrays at oSrcW / oDstW / oRankW bytes per row (1, 2, 4; else 8)
    int64_t* oDst;
    int64_t* oRank;
    int8_t oSrcW, oDstW, oRankW;
    int32_t* oType;
    uint32_t* oEntry;                   // frontier index of each row (GetNeighbors), may be null
    uint8_t* oFlags;                    // EF_* flags of each row's edge (GetNeighbors row encoding), may be null
    const OutCol* oCols;                // nY columns (device array; columns >= kInlineCols read it)
    OutCol oColsIn[kInlineCols];        // the first columns' descriptors, by value (no upload)
    uint64_t* rowsPub;                  // host-mapped [rows, seq, error bits] published by k_final_close (GO), or null
    uint64_t rowsSeq;
    uint64_t* resvTab;                  // GO: per group, the physical block of each virtual row block (resv*)
    uint64_t* resvCtl;                  // GO: this launch's reservation counters (below)
    uint64_t* resvNext;                 // GO: the next launch's (cleared by k_final_close)
    uint32_t resvTB;                    // blocks per group in resvTab
    uint32_t resvSeq;                   // tag of this launch's resvTab entries (never 0; no clearing)
    uint32_t resvG;                     // groups (<= kResvMaxGroups)
    uint32_t resvShift;                 // log2 of the block's rows (block >= rows of one chunk)
    uint32_t resvStride;                // words between two counters of resvCtl
    const uint8_t* mask;                // per hop edge: storage emitted it (max_edge_returned_per_vertex
                                        // path); when set, replaces the storage checks. nullptr: none
    int64_t kc[kJitConsts];             // generated kernels: literal bits (string: pool offset)
    uint32_t kl[kJitConsts];            // string literal lengths
    const uint64_t* dynTotal;           // device-driven hop: packed (frontier rows << kDynShift | E) written by
                                        // the kernel that built the frontier; nullptr: E / nEnt above
    const uint64_t* dynTiles;           // dense final hop: the compaction count launch's tile words; the close
    uint64_t nDynTiles;                 // sums them into *dynTotal before publishing it (no launch of its own)
    const uint32_t* fin;                // per frontier entry: its input row (multi-root pipe walks), or null
    char* strOut;                       // result string arena: kStrBuildBytes per (row - oBase, string column),
                                        // for the strings YIELD columns build; nullptr when none does
    uint32_t nStrOut;                   // columns that build strings (bits of strOutMask, y < 32)
    uint32_t strOutMask;
    const uint32_t* dstMap;             // $$ owner fetch (world > 1): global row -> row of env.dtags' tables, or null
    // dense final hop (one slot, world 1): the launch covers every CSR position of the slot; entries are the
    // shard's rows (estart = ebase = the slot's off[], chunkFirst = the slot's chunkRow), and an edge counts
    // only when its row's mark is denseEp (the frontier the compaction would have listed). null: off
    const uint8_t* denseMark;
    uint32_t denseEp;
};

// rows a GO final launch may leave past its row count before k_final_close (outputs are sized for them)
__host__ __device__ inline uint64_t resvSlack(const FinalArgs& a) { return static_cast<uint64_t>(a.resvG) << a.resvShift; }

// the row's slot of the result string arena for the j-th column that builds strings
__device__ __forceinline__ char* strSlot(const FinalArgs& a, uint64_t o, uint32_t j) {
    return a.strOut == nullptr ? nullptr : a.strOut + ((o - a.oBase) * a.nStrOut + j) * kStrBuildBytes;
}

// packed (frontier rows, hop edges) totals of the compaction / seed kernels
constexpr int kDynShift = 36;
constexpr uint64_t kDynMask = (1ULL << kDynShift) - 1;

struct VertexCellArgs {
    const uint32_t* rows;
    uint64_t n;
    int32_t ncols;
    const int32_t* tagSlot;             // per column: tag slot, -1 for non-tag columns
    const int32_t* col;
    VmEnv env;
    OutCell* out;
};

constexpr uint64_t kTile = 4096;        // items per scan tile
constexpr uint64_t kChunk = 2048;       // edges per edge-balanced workgroup (expansion, final hop)

// GO final hop: where a chunk's passing rows go (engine.cpp resvGeometry). One counter per group of chunks (chunk % resvG:
// dispatch puts consecutive workgroups on different XCDs, so with 8 groups a group is one XCD's
// chunks) hands out virtual rows; each group's virtual rows live in blocks of 2^resvShift physical
// rows taken from one global counter (one atomic per block). Same-address atomics serialise at the
// memory side (~12 ns each, tools/mb_atomic.hip): one counter for every chunk made C2's 31 K chunks a
// 380 us chain. The last block of each group is partly empty: k_final_close moves the rows that lie
// past the row count into those holes (at most resvG blocks of rows), publishes the count and the
// query's error bits, and clears the counters for the next launch.
// Words of FinalArgs::resvCtl, one of two sets used by alternate launches (stride resvStride words;
// cleared at allocation, then k_final_close of each launch clears the other set, resvNext):
//   [0] physical rows handed out (a multiple of the block)
//   [(1 + g) * stride] virtual rows of group g
//   [(1 + G) * stride] the row count (written by k_final_close)
constexpr uint64_t kDoneOff = 1024;
constexpr uint32_t kResvMaxGroups = 64;
constexpr uint32_t kResvGroups = 8;                   // a group per XCD
constexpr uint32_t kResvShift = 16;                   // 64 K rows per block

}  // namespace ngx
