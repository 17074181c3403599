// Internal host-side structures of libnebula_gn: schema registry, the exported per-shard graph
// snapshot (CSR + columnar props, built by exporter.cpp from reference-format KV rows), and the
// device mirror descriptors shared with the HIP kernels (kernels.hip).
#pragma once

#include <sched.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/nebula_gn.h"
#include "ngx_device.h"

namespace ngx {

enum SType : int32_t {
    T_UNKNOWN = 0, T_BOOL = 1, T_INT = 2, T_VID = 3, T_FLOAT = 4, T_DOUBLE = 5, T_STRING = 6, T_TIMESTAMP = 21,
};

struct Error {
    int32_t code;
    std::string msg;
};

struct FieldDef {
    std::string name;
    int32_t type;
};

struct SchemaDef {
    int64_t ver = 0;
    std::vector<FieldDef> fields;
    std::string ttlCol;
    int64_t ttlDur = 0;
    int32_t index(const std::string& n) const {
        for (size_t i = 0; i < fields.size(); i++) if (fields[i].name == n) return static_cast<int32_t>(i);
        return -1;
    }
    int32_t typeOf(const std::string& n) const {
        int32_t i = index(n);
        return i < 0 ? T_UNKNOWN : fields[i].type;
    }
};

struct SchemaSet {
    int32_t id = 0;
    std::string name;
    std::map<int64_t, SchemaDef> versions;
    const SchemaDef& latest() const { return versions.rbegin()->second; }
    const SchemaDef* version(int64_t v) const {
        auto it = versions.find(v);
        return it == versions.end() ? nullptr : &it->second;
    }
};

// ------------------------------------------------------------------ exported snapshot (host)
struct HostColumn {
    int32_t type = T_UNKNOWN;           // latest schema type
    std::vector<int64_t> i64;           // INT / TIMESTAMP / VID
    std::vector<double> f64;            // FLOAT (widened) / DOUBLE
    std::vector<uint8_t> b;             // BOOL
    std::vector<uint64_t> soff;         // STRING offsets (n + 1)
    std::string sbytes;                 // STRING bytes
    std::vector<uint8_t> valid;         // 0 where the row's schema version lacks the field
    bool allValid = true;
    int32_t width = 8;                  // INT/TIMESTAMP/VID bytes per value on the device (set at upload)
};

struct HostSlot {                       // one signed edge type: CSR over the shard's vertex rows
    int32_t etype = 0;
    std::vector<uint64_t> off;          // V + 1
    std::vector<int64_t> dst;
    std::vector<int64_t> rank;
    std::vector<uint32_t> dgid;         // global row of (ID_HASH(dst), dst); kNoRow if absent
    std::vector<uint8_t> eflags;        // EF_* per edge
    bool anyFlags = false;
    std::vector<HostColumn> cols;       // fields of the latest schema of |etype|
};

struct HostTag {
    int32_t tag = 0;
    std::vector<uint8_t> present;       // V: the vertex has a row of this tag
    std::vector<HostColumn> cols;
};

struct HostGraph {
    std::vector<int32_t> vpart;         // vertex table sorted by (part, vid)
    std::vector<int64_t> vid;
    std::vector<HostSlot> slots;
    std::vector<HostTag> tags;
    uint64_t gbase = 0;                 // first global row of this shard
    uint64_t vglobal = 0;               // rows over all shards
    std::vector<uint64_t> shardBase;    // world + 1
    uint64_t edges = 0;
    uint64_t commitDigest = 0;          // digest of every shard's vertex table at commit (the commit set)
};

struct StagedRows {
    std::vector<uint8_t> keys;          // concatenated 24/40-byte keys
    std::vector<uint32_t> klen;
    std::vector<uint64_t> koff;
    std::vector<uint8_t> vals;
    std::vector<uint64_t> voff;         // n + 1
};

struct DeviceGraph;                     // engine.cpp

struct Space {
    int32_t id = 0;
    int32_t numParts = 0;
    uint64_t gen = 0;                   // snapshot generation (bumped by every commit; keys cached kernels)
    std::map<int32_t, SchemaSet> tags, edges;
    std::map<std::string, int32_t> tagByName, edgeByName;
    std::vector<std::string> edgeOrder;
    StagedRows staged;
    std::unique_ptr<HostGraph> loaded;  // ngx_load_csr: the next commit's shard (instead of the staged rows)
    bool narrow = true;                 // device integer columns at their narrowest width (flag narrow_columns)
    std::unique_ptr<HostGraph> host;
    std::unique_ptr<DeviceGraph> dev;
    const SchemaSet* edge(int32_t absType) const {
        auto it = edges.find(absType);
        return it == edges.end() ? nullptr : &it->second;
    }
    const SchemaSet* tag(int32_t id) const {
        auto it = tags.find(id);
        return it == tags.end() ? nullptr : &it->second;
    }
    int32_t slotOf(int32_t signedType) const;   // index into host->slots, -1 if none
    int32_t tagSlotOf(int32_t tagId) const;
};

// host threads for the exporter, the head-image build and result decoding: NGX_HOST_THREADS, else the
// launcher's per-process share (OMP_NUM_THREADS: 16 per GPU on the MI355X boxes), else every CPU this
// process may run on (sched_getaffinity)
inline int hostThreadBudget() {
    static const int n = [] {
        for (const char* v : {"NGX_HOST_THREADS", "OMP_NUM_THREADS"}) {
            const char* s = std::getenv(v);
            if (s && std::atoi(s) > 0) return std::atoi(s);
        }
        cpu_set_t set;
        if (sched_getaffinity(0, sizeof(set), &set) == 0 && CPU_COUNT(&set) > 0) return CPU_COUNT(&set);
        const unsigned h = std::thread::hardware_concurrency();
        return h ? static_cast<int>(h) : 1;
    }();
    return n;
}

inline int32_t idHash(int64_t vid, int32_t numParts) {        // ID_HASH (src/common/base/Base.h:166-167)
    return static_cast<int32_t>(static_cast<uint64_t>(vid) % static_cast<uint64_t>(numParts) + 1);
}

// exporter.cpp: build the shard snapshot from staged rows
Error exportSnapshot(Space& sp, int32_t rank, int32_t world, HostGraph& out);
// exporter.cpp: the same snapshot from a caller's CSR (ngx_load_csr), validated
Error loadCsrShard(const Space& sp, int32_t rank, int32_t world, const ngx_csr_shard& in, HostGraph& out);
// snapshot.cpp: device snapshot files of a committed shard
uint64_t schemaDigest(const Space& sp);
// digest of the vertex tables of every shard, in rank order: equal on all ranks of one commit (the
// global rows dgid / shardBase encode), different for tables of different commits
// the commit's identity: every shard's vertex table plus one random nonce per shard drawn at that
// commit (two commits of identical data are still different commits)
uint64_t tablesDigest(const std::vector<std::vector<std::pair<int32_t, int64_t>>>& tables,
                      const std::vector<uint64_t>& nonces);
Error writeSnapshotFile(const Space& sp, const HostGraph& g, int32_t rank, int32_t world, const std::string& path,
                        const std::string& tag);
Error readSnapshotFile(const Space& sp, const std::string& path, int32_t rank, int32_t world, HostGraph& out,
                       std::string& tag);
// resolve dst -> global row with the vertex tables of every shard (world == 1: local only)
void resolveDstRows(const Space& sp, HostGraph& g,
                    const std::vector<std::vector<std::pair<int32_t, int64_t>>>& shardTables, int32_t world);

}  // namespace ngx
