// ORACLE — TEST INFRASTRUCTURE ONLY (see orc_core.h header).
// Restates QueryBaseProcessor<GetNeighborsRequest, QueryResponse> (src/storage/query/
// QueryBaseProcessor.inl:25-855), QueryBoundProcessor (src/storage/query/QueryBoundProcessor.cpp:
// 18-261), the PropsCollector (src/storage/Collector.h:38-84) and checkDataExpiredForTTL
// (src/storage/CommonUtils.cpp:13-49). Buckets run on std::threads like the reader pool.
#include "orc_query.h"

#include <atomic>
#include <functional>
#include <thread>
#include <numeric>

namespace orc {

// ---------------------------------------------------------------- KVStore
void KVStore::finalize(int threads) {
    if (sorted_) return;
    // RocksDB's bytewise order, the later put of a key kept (a stable order for equal keys: the put index
    // breaks ties). Each entry carries its first 16 key bytes as two big-endian words, so most comparisons
    // never touch the blob; the entries are bucketed by their first two key bytes (the key type and the
    // part's low byte) and the buckets sorted in parallel, independently, and concatenated. (32 bytes: an
    // edge key's part, src, type, rank and dst.)
    struct SK {
        uint64_t p[4];
        uint64_t i;
    };
    const size_t n = ents_.size();
    std::vector<SK> keys(n);
    auto be = [](const char* k, size_t len) {
        uint64_t v = 0;
        for (size_t b = 0; b < 8; b++) v = (v << 8) | (b < len ? static_cast<uint8_t>(k[b]) : 0u);
        return v;
    };
    threads = std::max(1, threads);
    auto parallel = [&](size_t count, const std::function<void(size_t, size_t)>& f) {
        const int t = count < (1u << 16) ? 1 : threads;
        std::vector<std::thread> ts;
        for (int k = 0; k < t; k++) ts.emplace_back([&, k] { f(count * k / t, count * (k + 1) / t); });
        for (auto& th : ts) th.join();
    };
    parallel(n, [&](size_t lo, size_t hi) {
        for (size_t i = lo; i < hi; i++) {
            const char* k = blob_.data() + ents_[i].off;
            const size_t kl = ents_[i].klen;
            SK x;
            for (size_t w = 0; w < 4; w++) x.p[w] = kl > 8 * w ? be(k + 8 * w, kl - 8 * w) : 0;
            x.i = i;
            keys[i] = x;
        }
    });
    auto cmp = [this](const SK& a, const SK& b) {
        for (int w = 0; w < 4; w++)
            if (a.p[w] != b.p[w]) return a.p[w] < b.p[w];
        const Ent& ea = ents_[a.i];
        const Ent& eb = ents_[b.i];
        const uint32_t la = ea.klen > 32 ? ea.klen - 32 : 0, lb = eb.klen > 32 ? eb.klen - 32 : 0;
        if (la && lb) {
            const int c = std::memcmp(blob_.data() + ea.off + 32, blob_.data() + eb.off + 32, std::min(la, lb));
            if (c != 0) return c < 0;
        }
        if (ea.klen != eb.klen) return ea.klen < eb.klen;      // (zero padding above: the shorter key first)
        return a.i < b.i;
    };
    // buckets by the first two key bytes
    std::vector<size_t> cnt(65537, 0);
    for (const SK& k : keys) cnt[(k.p[0] >> 48) + 1]++;
    for (size_t b = 1; b <= 65536; b++) cnt[b] += cnt[b - 1];
    std::vector<SK> sorted(n);
    {
        std::vector<size_t> at(cnt.begin(), cnt.end() - 1);
        for (const SK& k : keys) sorted[at[k.p[0] >> 48]++] = k;
    }
    keys.clear();
    keys.shrink_to_fit();
    std::vector<size_t> nonEmpty;
    for (size_t b = 0; b < 65536; b++) if (cnt[b + 1] > cnt[b]) nonEmpty.push_back(b);
    std::atomic<size_t> next{0};
    {
        std::vector<std::thread> ts;
        for (int t = 0; t < (n < (1u << 16) ? 1 : threads); t++) {
            ts.emplace_back([&] {
                for (size_t j; (j = next.fetch_add(1)) < nonEmpty.size();) {
                    const size_t b = nonEmpty[j];
                    std::sort(sorted.begin() + cnt[b], sorted.begin() + cnt[b + 1], cmp);
                }
            });
        }
        for (auto& th : ts) th.join();
    }
    std::vector<Ent> out;
    out.reserve(n);
    for (size_t i = 0; i < n; i++) {
        const Ent& e = ents_[sorted[i].i];
        // the same key as the previous one: equal prefix words first (the blob only for longer keys)
        const bool samePrefix = i > 0 && sorted[i].p[0] == sorted[i - 1].p[0] && sorted[i].p[1] == sorted[i - 1].p[1] &&
                                sorted[i].p[2] == sorted[i - 1].p[2] && sorted[i].p[3] == sorted[i - 1].p[3];
        if (samePrefix && out.back().klen == e.klen &&
            (e.klen <= 32 || std::memcmp(blob_.data() + out.back().off + 32, blob_.data() + e.off + 32, e.klen - 32) == 0)) {
            out.back() = e;                       // same key: the later write wins
        } else {
            out.push_back(e);
        }
    }
    ents_.swap(out);
    sorted_ = true;
}

std::pair<size_t, size_t> KVStore::prefix(const std::string& p) const {
    auto lessKeyPrefix = [&](const Ent& e, const std::string& pre) {
        int c = std::memcmp(blob_.data() + e.off, pre.data(), std::min<size_t>(e.klen, pre.size()));
        if (c != 0) return c < 0;
        return e.klen < pre.size();
    };
    auto lo = std::lower_bound(ents_.begin(), ents_.end(), p, lessKeyPrefix);
    auto hi = lo;
    while (hi != ents_.end() && hi->klen >= p.size() &&
           std::memcmp(blob_.data() + hi->off, p.data(), p.size()) == 0) {
        ++hi;
    }
    return {static_cast<size_t>(lo - ents_.begin()), static_cast<size_t>(hi - ents_.begin())};
}

namespace {

enum class KVCode { SUCCEEDED = 0, ERR_PART_NOT_FOUND = -2, ERR_KEY_NOT_FOUND = -3,
                    ERR_TAG_NOT_FOUND = -11, ERR_EDGE_NOT_FOUND = -12, ERR_CORRUPT_DATA = -14 };

int32_t toErrorCode(KVCode c) {        // BaseProcessor::to
    switch (c) {
        case KVCode::SUCCEEDED: return SUCCEEDED;
        case KVCode::ERR_PART_NOT_FOUND: return E_PART_NOT_FOUND;
        case KVCode::ERR_KEY_NOT_FOUND: return E_KEY_NOT_FOUND;
        case KVCode::ERR_TAG_NOT_FOUND: return E_TAG_NOT_FOUND;
        case KVCode::ERR_EDGE_NOT_FOUND: return E_EDGE_NOT_FOUND;
        default: return E_UNKNOWN;
    }
}

// PropContext (src/storage/CommonUtils.h:27-98)
struct PropContext {
    enum PropInKeyType { NONE = 0, SRC = 1, DST = 2, TYPE = 3, RANK = 4 };
    PropDef prop{EDGE, 0, ""};
    SupportedType type = UNKNOWN;
    PropInKeyType pik = NONE;
    int32_t retIndex = -1;
    bool returned = false;
    bool filtered = false;
    std::string tagOrEdgeName;
    bool fromTagFilter() const { return (prop.owner == DEST || prop.owner == SOURCE) && filtered; }
};
struct TagContext {
    TagID tagId = 0;
    std::vector<PropContext> props;
    std::map<std::string, int32_t> propNameIndex;      // only filled by pushFilterProp
    PropContext* findProp(const std::string& n) {
        auto it = propNameIndex.find(n);
        return it == propNameIndex.end() ? nullptr : &props[it->second];
    }
    void pushFilterProp(const std::string& tagName, const std::string& propName, SupportedType t) {
        PropContext pc;
        pc.prop.name = propName; pc.type = t; pc.prop.owner = SOURCE;
        pc.retIndex = static_cast<int32_t>(props.size());
        pc.filtered = true; pc.tagOrEdgeName = tagName;
        props.push_back(pc);
        propNameIndex[propName] = static_cast<int32_t>(props.size()) - 1;
    }
};
using FilterContext = std::map<std::pair<std::string, std::string>, Variant>;

// PropsCollector (Collector.h:38-84)
struct Collector {
    RowWriter* w = nullptr;
    VertexID dstId = 0;
    void vid(int64_t v) { if (w) (*w) << v; }
    void value(const Variant& v) {
        if (!w) return;
        switch (which(v)) {
            case VAR_INT64: (*w) << std::get<int64_t>(v); break;
            case VAR_DOUBLE: (*w) << std::get<double>(v); break;
            case VAR_BOOL: (*w) << std::get<bool>(v); break;
            default: (*w) << std::get<std::string>(v); break;
        }
    }
};

const std::map<std::string, PropContext::PropInKeyType> kPropsInKey = {    // QueryBaseProcessor.h:22-27
    {"_src", PropContext::SRC}, {"_dst", PropContext::DST},
    {"_type", PropContext::TYPE}, {"_rank", PropContext::RANK}};

class Processor {
 public:
    Processor(const StorageEngine* eng, GraphSpaceID space, bool onlyVertexProps)
        : eng_(eng), sm_(eng->schemas), space_(space), onlyVertexProps_(onlyVertexProps) {
        auto it = eng->stores.find(space);
        kv_ = it == eng->stores.end() ? nullptr : &it->second;
    }

    QueryResponse process(const GetNeighborsRequest& req) {             // .inl:800-855
        QueryResponse resp;
        if (req.has_edge_types) {
            for (auto t : req.edge_types) edgeContexts_.emplace(t, std::vector<PropContext>{});
        }
        int32_t code = checkAndBuildContexts(req);
        if (code != SUCCEEDED) {
            for (auto& p : req.parts) resp.failed_codes.emplace_back(code, p.first);
            return resp;
        }
        auto buckets = StorageEngine::genBuckets(req, eng_->flags.min_vertices_per_bucket,
                                                 std::max(eng_->flags.max_handlers_per_req, 1));
        std::vector<std::vector<VertexData>> bucketVertices(buckets.size());
        std::vector<std::vector<std::pair<PartitionID, KVCode>>> codes(buckets.size());
        std::atomic<int64_t> totalEdges{0}, scanned{0};
        auto runBucket = [&](size_t b) {
            int64_t sc = 0;
            for (auto& pv : buckets[b]) {
                int64_t n = 0;
                auto rc = processVertex(pv.first, pv.second, bucketVertices[b], n, sc);
                totalEdges += n;
                codes[b].emplace_back(pv.first, rc);
            }
            scanned += sc;
        };
        int threads = std::max(1, eng_->flags.threads);
        if (threads == 1 || buckets.size() == 1) {
            for (size_t b = 0; b < buckets.size(); b++) runBucket(b);
        } else {
            std::atomic<size_t> next{0};
            std::vector<std::thread> ts;
            for (int t = 0; t < threads; t++) {
                ts.emplace_back([&] { for (size_t b; (b = next++) < buckets.size();) runBucket(b); });
            }
            for (auto& t : ts) t.join();
        }
        std::set<PartitionID> failedParts;
        for (auto& bc : codes) {
            for (auto& r : bc) {
                if (r.second != KVCode::SUCCEEDED && !failedParts.count(r.first)) {
                    failedParts.insert(r.first);
                    resp.failed_codes.emplace_back(toErrorCode(r.second), r.first);
                }
            }
        }
        for (auto& bv : bucketVertices) for (auto& v : bv) resp.vertices.push_back(std::move(v));
        resp.total_edges = static_cast<int32_t>(totalEdges.load());
        resp.scanned = scanned.load();
        for (auto& kv : vertexSchema_) resp.vertex_schema[kv.first] = kv.second;
        for (auto& kv : edgeSchema_) resp.edge_schema[kv.first] = kv.second;
        return resp;
    }

 private:
    const StorageEngine* eng_;
    const SchemaManager& sm_;
    GraphSpaceID space_;
    bool onlyVertexProps_;
    const KVStore* kv_;
    std::shared_ptr<Expression> exp_;
    std::vector<TagContext> tagContexts_;
    std::map<EdgeType, std::vector<PropContext>> edgeContexts_;
    std::map<TagID, std::shared_ptr<Schema>> vertexSchema_;
    std::map<EdgeType, std::shared_ptr<Schema>> edgeSchema_;
    std::map<EdgeType, bool> onlyStructures_;
    std::map<std::string, EdgeType> edgeMap_;
    std::map<EdgeType, std::pair<std::string, int64_t>> edgeTTL_;
    std::map<TagID, std::pair<std::string, int64_t>> tagTTL_;

    int32_t checkAndBuildContexts(const GetNeighborsRequest& req) {     // .inl:66-170
        std::map<TagID, int32_t> tagIndex;
        int32_t index = 0;
        for (auto& col : req.return_columns) {
            PropContext prop;
            if (col.owner == SOURCE || col.owner == DEST) {
                TagID tagId = col.id;
                auto schema = sm_.getTagSchema(space_, tagId);
                if (!schema) return E_TAG_PROP_NOT_FOUND;
                auto ftype = schema->getFieldType(col.name);
                if (ftype == UNKNOWN) return E_IMPROPER_DATA_TYPE;
                prop.type = ftype;
                prop.retIndex = index++;
                prop.prop = col;
                prop.returned = true;
                auto it = tagIndex.find(tagId);
                if (it == tagIndex.end()) {
                    TagContext tc; tc.tagId = tagId; tc.props.push_back(prop);
                    tagContexts_.push_back(tc);
                    tagIndex[tagId] = static_cast<int32_t>(tagContexts_.size()) - 1;
                } else {
                    tagContexts_[it->second].props.push_back(prop);
                }
            } else {
                EdgeType edgeType = col.id;
                auto edgeName = sm_.toEdgeName(space_, std::abs(edgeType));
                if (!edgeName.ok()) return E_EDGE_NOT_FOUND;
                edgeMap_.emplace(edgeName.value(), std::abs(edgeType));
                auto it = kPropsInKey.find(col.name);
                if (it != kPropsInKey.end()) {
                    prop.pik = it->second;
                    prop.type = (prop.pik == PropContext::SRC || prop.pik == PropContext::DST) ? VID : INT;
                } else {
                    auto schema = sm_.getEdgeSchema(space_, std::abs(edgeType));
                    if (!schema) return E_EDGE_PROP_NOT_FOUND;
                    auto ftype = schema->getFieldType(col.name);
                    if (ftype == UNKNOWN) return E_IMPROPER_DATA_TYPE;
                    prop.type = ftype;
                }
                prop.retIndex = index++;
                prop.prop = col;
                prop.returned = true;
                edgeContexts_[edgeType].push_back(prop);
            }
        }
        if (!req.filter.empty()) {
            auto e = Expression::decode(req.filter);
            if (!e.ok()) return E_INVALID_FILTER;
            exp_ = e.value();
            if (!checkExp(exp_.get())) return E_INVALID_FILTER;
        }
        buildTTLInfoAndRespSchema();
        return SUCCEEDED;
    }

    bool checkExp(const Expression* exp) {                               // .inl:195-322
        switch (exp->kind()) {
            case Expression::kPrimary: return true;
            case Expression::kFunctionCall: {
                auto* f = const_cast<FunctionCallExpression*>(static_cast<const FunctionCallExpression*>(exp));
                auto func = getFunction(f->name(), f->args().size());
                if (!func.ok()) return false;
                for (auto& a : f->args()) if (!checkExp(a.get())) return false;
                f->setFunc(func.value());
                return true;
            }
            case Expression::kUnary: return checkExp(static_cast<const UnaryExpression*>(exp)->operand_.get());
            case Expression::kTypeCasting: return checkExp(static_cast<const TypeCastingExpression*>(exp)->operand_.get());
            case Expression::kArithmetic: case Expression::kRelational: case Expression::kLogical: {
                auto* b = static_cast<const BinaryExpression*>(exp);
                return checkExp(b->left_.get()) && checkExp(b->right_.get());
            }
            case Expression::kSourceProp: {
                auto* s = static_cast<const AliasPropertyExpression*>(exp);
                auto tagRet = sm_.toTagID(space_, s->alias());
                if (!tagRet.ok()) return false;
                auto tagId = tagRet.value();
                auto schema = sm_.getTagSchema(space_, tagId);
                if (!schema) return false;
                if (schema->getFieldIndex(s->prop()) < 0) return false;
                auto ftype = schema->getFieldType(s->prop());
                for (auto& tc : tagContexts_) {
                    if (tc.tagId == tagId) {
                        auto* prop = tc.findProp(s->prop());
                        if (prop == nullptr) {
                            tc.pushFilterProp(s->alias(), s->prop(), ftype);
                        } else if (!prop->filtered) {
                            prop->filtered = true; prop->tagOrEdgeName = s->alias();
                        }
                        return true;
                    }
                }
                TagContext tc; tc.tagId = tagId;
                tc.pushFilterProp(s->alias(), s->prop(), ftype);
                tagContexts_.push_back(tc);
                return true;
            }
            case Expression::kEdgeRank: case Expression::kEdgeDstId:
            case Expression::kEdgeSrcId: case Expression::kEdgeType:
                return true;
            case Expression::kAliasProp: {
                if (edgeContexts_.empty()) return false;
                auto* a = static_cast<const AliasPropertyExpression*>(exp);
                auto et = sm_.toEdgeType(space_, a->alias());
                if (!et.ok()) return false;
                auto schema = sm_.getEdgeSchema(space_, std::abs(et.value()));
                if (!schema) return false;
                return schema->getFieldIndex(a->prop()) >= 0;
            }
            default: return false;          // $-, $var, $$ and unknown kinds
        }
    }

    void buildTTLInfoAndRespSchema() {                                   // .inl:669-797
        for (auto& tc : tagContexts_) {
            auto resp = std::make_shared<Schema>();
            for (auto& p : tc.props) if (p.returned) resp->fields.push_back(Field{p.prop.name, p.type});
            if (!resp->fields.empty() && !vertexSchema_.count(tc.tagId)) vertexSchema_[tc.tagId] = resp;
            if (tagTTL_.count(tc.tagId)) continue;
            auto s = sm_.getTagSchema(space_, tc.tagId);
            if (!s) continue;
            if (s->ttlCol.empty() || s->ttlDuration <= 0) continue;
            tagTTL_[tc.tagId] = {s->ttlCol, s->ttlDuration};
        }
        for (auto& ec : edgeContexts_) {
            auto resp = std::make_shared<Schema>();
            for (auto& p : ec.second) {
                if (p.prop.name == "_dst") continue;
                resp->fields.push_back(Field{p.prop.name, p.type});
            }
            onlyStructures_.emplace(ec.first, resp->fields.empty());
            if (!resp->fields.empty() && !edgeSchema_.count(ec.first)) edgeSchema_[ec.first] = resp;
            if (edgeTTL_.count(ec.first)) continue;
            auto s = sm_.getEdgeSchema(space_, std::abs(ec.first));
            if (!s) continue;
            if (s->ttlCol.empty() || s->ttlDuration <= 0) continue;
            edgeTTL_[ec.first] = {s->ttlCol, s->ttlDuration};
        }
    }

    bool expiredTTL(const Schema* schema, const RowReader* r, const std::string& col, int64_t dur) const {
        int64_t v = 0;                                                  // CommonUtils.cpp:13-49
        switch (schema->getFieldType(col)) {
            case TIMESTAMP: case INT:
                if (r->getInt(r->getSchema()->getFieldIndex(col), v) != ResultType::SUCCEEDED) return false;
                break;
            case VID:
                if (r->getVid(r->getSchema()->getFieldIndex(col), v) != ResultType::SUCCEEDED) return false;
                break;
            default: return false;
        }
        return eng_->flags.now_sec > v + dur;
    }

    void collectProps(const RowReader* reader, const char* key, size_t klen,
                      const std::vector<PropContext>& props, FilterContext* fctx, Collector* col) {
        for (auto& prop : props) {                                       // .inl:324-399
            if (klen != 0) {
                switch (prop.pik) {
                    case PropContext::NONE: break;
                    case PropContext::SRC: col->vid(keys::getSrcId(key)); continue;
                    case PropContext::DST: col->dstId = keys::getDstId(key); continue;
                    case PropContext::TYPE: col->value(Variant(static_cast<int64_t>(keys::getEdgeType(key)))); continue;
                    case PropContext::RANK: col->value(Variant(keys::getRank(key))); continue;
                }
            }
            if (reader != nullptr) {
                Variant v;
                auto res = RowReader::getPropByName(reader, prop.prop.name);
                if (!res.ok()) {
                    auto d = RowReader::getDefaultProp(prop.type);
                    if (!d.ok()) continue;
                    v = d.value();
                } else {
                    v = res.v;
                }
                if (prop.fromTagFilter()) (*fctx)[{prop.tagOrEdgeName, prop.prop.name}] = v;
                if (prop.returned) col->value(v);
            }
        }
    }

    KVCode collectVertexProps(PartitionID part, VertexID vid, TagID tagId,
                              const std::vector<PropContext>& props, FilterContext* fctx, Collector* col) {
        auto schema = sm_.getTagSchema(space_, tagId);                   // .inl:401-476
        if (!kv_ || !kv_->hasPart(part)) return KVCode::ERR_PART_NOT_FOUND;
        auto range = kv_->prefix(keys::vertexPrefix(part, vid, tagId));
        if (range.first == range.second) return KVCode::ERR_KEY_NOT_FOUND;
        std::string val = kv_->val(range.first);
        int32_t ver = RowReader::getSchemaVer(val);
        auto reader = ver >= 0 ? RowReader::make(val, sm_.getTagSchema(space_, tagId, ver)) : nullptr;
        if (!reader) return KVCode::ERR_CORRUPT_DATA;
        auto ttl = tagTTL_.find(tagId);
        if (ttl != tagTTL_.end() && schema &&
            expiredTTL(schema.get(), reader.get(), ttl->second.first, ttl->second.second)) {
            return KVCode::SUCCEEDED;
        }
        collectProps(reader.get(), kv_->key(range.first), kv_->klen(range.first), props, fctx, col);
        return KVCode::SUCCEEDED;
    }

    // collectEdgeProps (.inl:478-610) with processEdgeImpl's proc (QueryBoundProcessor.cpp:18-63)
    KVCode processEdgeImpl(PartitionID part, VertexID vid, EdgeType edgeType,
                           const std::vector<PropContext>& props, FilterContext& fctx, VertexData& vdata,
                           int64_t& scanned) {
        bool onlyStructure = onlyStructures_[edgeType];
        const Schema* currEdgeSchema = nullptr;
        if (!onlyStructure) {
            auto it = edgeSchema_.find(edgeType);
            if (it == edgeSchema_.end()) return KVCode::ERR_EDGE_NOT_FOUND;
            currEdgeSchema = it->second.get();
        }
        if (!kv_ || !kv_->hasPart(part)) return KVCode::ERR_PART_NOT_FOUND;
        auto range = kv_->prefix(keys::edgePrefix(part, vid, edgeType));
        scanned += static_cast<int64_t>(range.second - range.first);   // harness count, not reference logic
        std::vector<IdAndProp> edges;
        EdgeRanking lastRank = -1;
        VertexID lastDst = 0;
        bool firstLoop = true;
        int cnt = 0;
        const auto& schema = sm_.getEdgeSchema(space_, std::abs(edgeType));
        auto ttl = edgeTTL_.find(edgeType);
        bool hasTTL = ttl != edgeTTL_.end();
        for (size_t i = range.first; i < range.second; i++) {
            if (!(cnt < eng_->flags.max_edge_returned_per_vertex)) break;
            const char* key = kv_->key(i);
            size_t klen = kv_->klen(i);
            if (klen != keys::kEdgeLen) continue;          // RocksDB prefix iter never yields others here
            std::string val = kv_->val(i);
            auto rank = keys::getRank(key);
            auto dst = keys::getDstId(key);
            if (!firstLoop && rank == lastRank && lastDst == dst) continue;
            firstLoop = false;
            lastRank = rank;
            lastDst = dst;
            std::unique_ptr<RowReader> reader;
            if ((!onlyStructure || hasTTL) && !val.empty()) {
                int32_t ver = RowReader::getSchemaVer(val);
                reader = ver >= 0 ? RowReader::make(val, sm_.getEdgeSchema(space_, std::abs(edgeType), ver)) : nullptr;
                if (!reader) continue;                                  // "Skip the bad format row!"
                if (hasTTL && schema &&
                    expiredTTL(schema.get(), reader.get(), ttl->second.first, ttl->second.second)) {
                    continue;
                }
                if (exp_ != nullptr) {
                    Getters g;
                    const RowReader* rd = reader.get();
                    g.getAliasProp = [&](const std::string& edgeName, const std::string& prop) -> OptVariant {
                        auto f = edgeMap_.find(edgeName);
                        if (f == edgeMap_.end()) return Status::Error("Edge not found when call getters.");
                        if (std::abs(edgeType) != f->second) return Status::Error("Ignore this edge");
                        if (prop == "_src") return OptVariant(keys::getSrcId(key));
                        if (prop == "_dst") return OptVariant(keys::getDstId(key));
                        if (prop == "_rank") return OptVariant(keys::getRank(key));
                        if (prop == "_type") return OptVariant(static_cast<int64_t>(keys::getEdgeType(key)));
                        auto res = RowReader::getPropByName(rd, prop);
                        if (!res.ok()) return Status::Error("Invalid Prop");
                        return OptVariant(res.v);
                    };
                    g.getEdgeRank = [&]() -> OptVariant { return OptVariant(rank); };
                    g.getEdgeDstId = [&](const std::string& edgeName) -> OptVariant {
                        auto f = edgeMap_.find(edgeName);
                        if (f == edgeMap_.end()) return Status::Error("Edge not found when call getters.");
                        if (std::abs(edgeType) != f->second) return Status::Error("Ignore this edge");
                        return OptVariant(dst);
                    };
                    g.getSrcTagProp = [&](const std::string& tag, const std::string& prop) -> OptVariant {
                        auto it = fctx.find({tag, prop});
                        if (it == fctx.end()) return Status::Error("Invalid Tag Filter");
                        return OptVariant(it->second);
                    };
                    auto value = exp_->eval(g);
                    if (!value.ok()) continue;
                    if (!Expression::asBool(value.value())) continue;
                }
            }
            IdAndProp edge;
            if (!onlyStructure) {
                RowWriter writer(currEdgeSchema);
                Collector c; c.w = &writer;
                collectProps(reader.get(), key, klen, props, &fctx, &c);
                edge.dst = c.dstId;
                edge.props = writer.encode();
                edge.has_props = true;
            } else {
                Collector c;
                collectProps(reader.get(), key, klen, props, &fctx, &c);
                edge.dst = c.dstId;
            }
            edges.push_back(std::move(edge));
            ++cnt;
        }
        if (!edges.empty()) vdata.edge_data.push_back(EdgeData{edgeType, std::move(edges)});
        return KVCode::SUCCEEDED;
    }

    KVCode processVertex(PartitionID part, VertexID vid, std::vector<VertexData>& out, int64_t& nEdges, int64_t& scanned) {
        VertexData v;                                                    // QueryBoundProcessor.cpp:173-234
        v.vertex_id = vid;
        FilterContext fctx;
        for (auto& tc : tagContexts_) {
            auto s = vertexSchema_.find(tc.tagId);
            if (s == vertexSchema_.end()) return KVCode::ERR_TAG_NOT_FOUND;
            RowWriter writer(s->second);
            Collector c; c.w = &writer;
            auto ret = collectVertexProps(part, vid, tc.tagId, tc.props, &fctx, &c);
            if (ret == KVCode::ERR_KEY_NOT_FOUND) continue;
            if (ret != KVCode::SUCCEEDED) return ret;
            if (writer.size() > 1) v.tag_data.push_back(TagData{tc.tagId, writer.encode()});
        }
        if (onlyVertexProps_) { out.push_back(std::move(v)); return KVCode::SUCCEEDED; }
        for (auto& ec : edgeContexts_) {
            if (ec.second.empty()) continue;
            auto ret = processEdgeImpl(part, vid, ec.first, ec.second, fctx, v, scanned);
            if (ret != KVCode::SUCCEEDED) return ret;
        }
        if (!v.edge_data.empty()) {
            for (auto& ed : v.edge_data) nEdges += static_cast<int64_t>(ed.edges.size());
            out.push_back(std::move(v));
        }
        return KVCode::SUCCEEDED;
    }
};

}  // namespace

std::vector<std::vector<std::pair<PartitionID, VertexID>>> StorageEngine::genBuckets(
    const GetNeighborsRequest& req, int32_t minVerticesPerBucket, int32_t maxHandlers) {
    int32_t verticesNum = 0;                                             // .inl:639-667
    for (auto& pv : req.parts) verticesNum += static_cast<int32_t>(pv.second.size());
    int32_t bucketsNum = std::min(std::max(1, verticesNum / minVerticesPerBucket), maxHandlers);
    std::vector<std::vector<std::pair<PartitionID, VertexID>>> buckets(bucketsNum);
    int32_t vNumPerBucket = verticesNum / bucketsNum;
    int32_t leftVertices = verticesNum % bucketsNum;
    int32_t bucketIndex = -1;
    size_t threshold = vNumPerBucket;
    for (auto& pv : req.parts) {
        for (auto vid : pv.second) {
            if (bucketIndex < 0 || buckets[bucketIndex].size() >= threshold) {
                ++bucketIndex;
                threshold = bucketIndex < leftVertices ? vNumPerBucket + 1 : vNumPerBucket;
            }
            buckets[bucketIndex].emplace_back(pv.first, vid);
        }
    }
    return buckets;
}

QueryResponse StorageEngine::getBound(const GetNeighborsRequest& req, bool onlyVertexProps) const {
    Processor p(this, req.space, onlyVertexProps);
    return p.process(req);
}

}  // namespace orc
