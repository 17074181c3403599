// ORACLE — TEST INFRASTRUCTURE ONLY (see orc_core.h header).
// Stand-ins for the reference's meta SchemaManager (src/meta/SchemaManager.h:18-56) and the
// kvstore prefix scan (KVStore::prefix -> RocksEngine::prefix, src/kvstore/RocksEngine.cpp:205-214):
// an in-memory array of reference-format keys kept in RocksDB bytewise order.
#pragma once

#include <mutex>
#include <set>
#include <thread>
#include "orc_core.h"

namespace orc {

class SchemaManager {
 public:
    void addSpace(GraphSpaceID space, int32_t numParts) { parts_[space] = numParts; }
    int32_t partsNum(GraphSpaceID space) const {
        auto it = parts_.find(space);
        return it == parts_.end() ? 0 : it->second;
    }
    void addTagSchema(GraphSpaceID s, TagID id, const std::string& name, std::shared_ptr<Schema> sc) {
        tags_[{s, id}][sc->ver] = sc; tagNames_[{s, name}] = id; tagIdNames_[{s, id}] = name;
    }
    void addEdgeSchema(GraphSpaceID s, EdgeType id, const std::string& name, std::shared_ptr<Schema> sc) {
        edges_[{s, id}][sc->ver] = sc; edgeNames_[{s, name}] = id; edgeIdNames_[{s, id}] = name;
        if (std::find(edgeOrder_[s].begin(), edgeOrder_[s].end(), name) == edgeOrder_[s].end()) {
            edgeOrder_[s].push_back(name);
        }
    }
    // ver < 0 => latest (AdHocSchemaManager.cpp:51-93 / MetaClient semantics); else exact version.
    // references into the registry (schemas are added before any query and never removed): the per-edge
    // lookups of collectEdgeProps copy no shared_ptr, whose reference count every reader thread would
    // otherwise increment on one cache line (the baseline's threads then serialise on it)
    const SchemaPtr& getTagSchema(GraphSpaceID s, TagID id, SchemaVer ver = -1) const { return find(tags_, s, id, ver); }
    const SchemaPtr& getEdgeSchema(GraphSpaceID s, EdgeType id, SchemaVer ver = -1) const { return find(edges_, s, id, ver); }
    StatusOr<TagID> toTagID(GraphSpaceID s, const std::string& name) const {
        auto it = tagNames_.find({s, name});
        if (it == tagNames_.end()) return Status::Error("Tag not found");
        return it->second;
    }
    StatusOr<EdgeType> toEdgeType(GraphSpaceID s, const std::string& name) const {
        auto it = edgeNames_.find({s, name});
        if (it == edgeNames_.end()) return Status::Error("Edge not found");
        return it->second;
    }
    StatusOr<std::string> toEdgeName(GraphSpaceID s, EdgeType t) const {
        auto it = edgeIdNames_.find({s, t});
        if (it == edgeIdNames_.end()) return Status::Error("Edge not found");
        return it->second;
    }
    std::vector<std::string> getAllEdge(GraphSpaceID s) const {
        auto it = edgeOrder_.find(s);
        return it == edgeOrder_.end() ? std::vector<std::string>{} : it->second;
    }

 private:
    using Versions = std::map<SchemaVer, SchemaPtr>;
    static const SchemaPtr& find(const std::map<std::pair<GraphSpaceID, int32_t>, Versions>& m,
                                 GraphSpaceID s, int32_t id, SchemaVer ver) {
        static const SchemaPtr none;
        auto it = m.find({s, id});
        if (it == m.end() || it->second.empty()) return none;
        if (ver < 0) return it->second.rbegin()->second;
        auto v = it->second.find(ver);
        return v == it->second.end() ? none : v->second;
    }
    std::map<GraphSpaceID, int32_t> parts_;
    std::map<std::pair<GraphSpaceID, int32_t>, Versions> tags_, edges_;
    std::map<std::pair<GraphSpaceID, std::string>, int32_t> tagNames_, edgeNames_;
    std::map<std::pair<GraphSpaceID, int32_t>, std::string> tagIdNames_, edgeIdNames_;
    std::map<GraphSpaceID, std::vector<std::string>> edgeOrder_;
};

// One space's KV data: a flat blob + an index sorted bytewise by key (RocksDB's default
// comparator). Multiple puts of one key keep the last one, as RocksDB does.
class KVStore {
 public:
    struct Ent {
        uint64_t off;      // key bytes at blob[off], value right after
        uint32_t klen;
        uint32_t vlen;
    };
    void reserve(size_t n, size_t moreBytes) { ents_.reserve(n); blob_.reserve(blob_.size() + moreBytes); }
    void put(const char* k, size_t kl, const char* v, size_t vl) {
        Ent e{blob_.size(), static_cast<uint32_t>(kl), static_cast<uint32_t>(vl)};
        blob_.insert(blob_.end(), k, k + kl);
        blob_.insert(blob_.end(), v, v + vl);
        ents_.push_back(e);
        sorted_ = false;
    }
    void finalize(int threads = 1);
    size_t size() const { return ents_.size(); }
    const char* key(size_t i) const { return blob_.data() + ents_[i].off; }
    size_t klen(size_t i) const { return ents_[i].klen; }
    std::string keyStr(size_t i) const { return std::string(key(i), klen(i)); }
    std::string val(size_t i) const { return std::string(key(i) + ents_[i].klen, ents_[i].vlen); }
    // [lo, hi) of keys starting with prefix
    std::pair<size_t, size_t> prefix(const std::string& p) const;
    void addPart(PartitionID p) { parts_.insert(p); }
    bool hasPart(PartitionID p) const { return parts_.count(p) != 0; }

 private:
    std::vector<char> blob_;
    std::vector<Ent> ents_;
    std::set<PartitionID> parts_;
    bool sorted_ = true;
    bool less(const Ent& a, const Ent& b) const {
        int c = std::memcmp(blob_.data() + a.off, blob_.data() + b.off, std::min(a.klen, b.klen));
        if (c != 0) return c < 0;
        return a.klen < b.klen;
    }
};

}  // namespace orc
