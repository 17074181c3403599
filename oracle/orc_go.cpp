// ORACLE — TEST INFRASTRUCTURE ONLY (see orc_core.h header).
// Restates the graphd GoExecutor (src/graph/GoExecutor.cpp:33-1419) for `GO [M TO] N STEPS FROM
// <literal vids> OVER ... [REVERSELY|BIDIRECT] [WHERE ...] YIELD [DISTINCT] ...`, the WhereWrapper
// pushdown rewrite (src/graph/TraverseExecutor.cpp:426-538), calculateExprType (:88-165) and the
// StorageClient routing (vid -> part by ID_HASH, src/storage/client/StorageClient.cpp:439-449) for
// a single storaged host (completeness is 0 as soon as any part fails, StorageClient.inl:134-151).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <unordered_set>

#include "orc_query.h"

namespace orc {

namespace {

bool canPushdown(Expression* expr) {                                  // TraverseExecutor.cpp:525-538
    ExpressionContext ctx;
    if (!expr->prepare(&ctx).ok()) return false;
    if (ctx.hasInputProp() || ctx.hasVariableProp() || ctx.hasDstTagProp()) return false;
    return true;
}

SupportedType columnTypeToSupportedType(ColumnType t) {
    switch (t) {
        case ColumnType::INT: return INT;
        case ColumnType::STRING: return STRING;
        case ColumnType::DOUBLE: return DOUBLE;
        case ColumnType::BOOL: return BOOL;
        case ColumnType::TIMESTAMP: return TIMESTAMP;
    }
    return UNKNOWN;
}

}  // namespace

bool rewriteForPushdown(Expression* expr) {                           // TraverseExecutor.cpp:461-523
    switch (expr->kind()) {
        case Expression::kLogical: {
            auto* l = static_cast<LogicalExpression*>(expr);
            if (l->op_ == LogicalExpression::XOR) return canPushdown(l);
            bool lp = rewriteForPushdown(l->left_.get());
            bool rp = rewriteForPushdown(l->right_.get());
            switch (l->op_) {
                case LogicalExpression::OR: return lp && rp;
                case LogicalExpression::AND:
                    if (!lp && !rp) return false;
                    if (!lp) l->left_ = std::make_unique<PrimaryExpression>(Variant(true));
                    else if (!rp) l->right_ = std::make_unique<PrimaryExpression>(Variant(true));
                    return true;
                default: return false;
            }
        }
        case Expression::kUnary: case Expression::kTypeCasting: case Expression::kArithmetic:
        case Expression::kRelational: case Expression::kFunctionCall:
            return canPushdown(expr);
        case Expression::kPrimary: case Expression::kSourceProp: case Expression::kEdgeRank:
        case Expression::kEdgeDstId: case Expression::kEdgeSrcId: case Expression::kEdgeType:
        case Expression::kAliasProp:
            return true;
        default:
            return false;
    }
}

namespace {

struct GoExec {
    const StorageEngine& eng;
    const SchemaManager& sm;
    GraphSpaceID space;
    const GoSentence& s;
    GoFlags flags;
    GoResult res;
    ExpressionContext ctx;
    uint32_t recordFrom = 1, steps = 1, curStep = 1;
    std::vector<EdgeType> edgeTypes;
    std::shared_ptr<Expression> filter;
    std::string filterPushdown;
    std::vector<std::shared_ptr<Expression>> yields;
    std::vector<std::string> yieldAliases;
    std::vector<VertexID> starts;
    std::vector<QueryResponse> records;
    // VertexHolder (GoExecutor.cpp:1337-1412): (vid, tag) -> (row, schema)
    std::map<std::pair<VertexID, TagID>, std::pair<std::string, std::shared_ptr<Schema>>> vertexHolder;
    std::map<TagID, std::shared_ptr<Schema>> vertexHolderSchemas;
    // VertexBackTracker (GoExecutor.h:189-207): (step, dst) -> root
    std::multimap<std::pair<uint32_t, VertexID>, VertexID> backTracker;
    // InterimResultIndex (InterimResult.h:80-114): column index, rows, vid -> row multimap
    std::map<std::string, uint32_t> columnToIndex;
    std::multimap<VertexID, uint32_t> vidToRowIndex;

    std::vector<VertexID> getRoots(VertexID srcId, size_t record) const {      // GoExecutor.h:218-230
        std::vector<VertexID> ids;
        if (record == 1) { ids.push_back(srcId); return ids; }
        auto range = backTracker.equal_range({static_cast<uint32_t>(record - 1), srcId});
        for (auto i = range.first; i != range.second; ++i) ids.push_back(i->second);
        return ids;
    }
    std::vector<uint32_t> rowsOfVids(const std::vector<VertexID>& ids) const {  // InterimResult.h:95-104
        std::vector<uint32_t> rows;
        for (auto v : ids) {
            auto range = vidToRowIndex.equal_range(v);
            for (auto i = range.first; i != range.second; ++i) rows.push_back(i->second);
        }
        return rows;
    }
    OptVariant getColumnWithRow(size_t row, const std::string& col) const {   // InterimResult.cpp:282-297
        if (row >= s.inputRows.size()) return Status::Error("Out of range");
        auto it = columnToIndex.find(col);
        if (it == columnToIndex.end()) return Status::Error("Prop `" + col + "' not found");
        return OptVariant(s.inputRows[row][it->second]);
    }

    // setupStarts (GoExecutor.cpp:471-509): checkIfDuplicateColumn (TraverseExecutor.cpp:167-181),
    // getDistinctVIDs (InterimResult.cpp:51-72, RowReader::getVid: INT or VID columns), buildIndex
    // (:178-280)
    bool setupStarts() {
        if (s.inputRows.empty()) return true;
        std::unordered_set<std::string> uniq;
        // checkIfDuplicateColumn reads inputs_: the pipe input, not a variable
        if (s.fromType == 1)
            for (auto& n : s.inputNames)
                if (!uniq.insert(n).second) return fail("Duplicate column `" + n + "'");
        int vidCol = -1;
        for (size_t i = 0; i < s.inputNames.size(); i++) if (s.inputNames[i] == s.fromCol) vidCol = static_cast<int>(i);
        // RowReader::getVid by name reads the first field of that name; names are unique here
        if (vidCol < 0 || (s.inputTypes[vidCol] != INT && s.inputTypes[vidCol] != VID))
            return fail("Column `" + s.fromCol + "' not found");
        std::unordered_set<VertexID> u;
        for (auto& r : s.inputRows) u.insert(std::get<int64_t>(r[vidCol]));
        starts.assign(u.begin(), u.end());
        for (size_t i = 0; i < s.inputNames.size(); i++) columnToIndex[s.inputNames[i]] = static_cast<uint32_t>(i);
        for (uint32_t r = 0; r < s.inputRows.size(); r++) vidToRowIndex.emplace(std::get<int64_t>(s.inputRows[r][vidCol]), r);
        return true;
    }

    GoExec(const StorageEngine& e, GraphSpaceID sp, const GoSentence& sent, GoFlags f)
        : eng(e), sm(e.schemas), space(sp), s(sent), flags(f) {}
    ~GoExec() {
        auto t = std::chrono::steady_clock::now();
        records.clear();
        trace("teardown", t);
    }

    bool fail(const std::string& msg) {
        res.ok = false; res.error = msg; res.rows.clear(); res.digests.clear(); res.rowCount = 0;
        return false;
    }
    bool isFinalStep() const { return curStep == steps; }
    // ORC_TRACE=1: phase times on stderr (test harness diagnostics)
    void trace(const char* what, std::chrono::steady_clock::time_point t0) const {
        static const bool on = std::getenv("ORC_TRACE") != nullptr;
        if (!on) return;
        std::fprintf(stderr, "[orc] step %u %s %.3fs\n", curStep, what,
                     std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    }
    bool isRecord() const { return curStep >= recordFrom && curStep <= steps; }

    bool addToEdgeTypes(EdgeType t) {                                  // GoExecutor.cpp:297-319
        if (s.direction == 0) edgeTypes.push_back(t);
        else if (s.direction == 1) edgeTypes.push_back(-t);
        else { edgeTypes.push_back(t); edgeTypes.push_back(-t); }
        return true;
    }

    bool prepareClauses() {                                            // :38-89
        recordFrom = s.recordFrom;
        steps = s.recordTo;
        if (s.fromType != 0 && s.fromCol == "*") return fail("Can not use `*' to reference a vertex id column.");   // :175-178
        // prepareOver (:254-295) / prepareOverAll (:225-252)
        if (s.overAll) {
            ctx.overAll = true;
            for (auto& name : sm.getAllEdge(space)) {
                auto t = sm.toEdgeType(space, name);
                if (!t.ok()) return fail(t.status().msg_);
                addToEdgeTypes(t.value());
                if (!ctx.addEdge(name, std::abs(t.value()))) return fail("edge alias(" + name + ") was dup");
            }
        } else {
            for (auto& e : s.over) {
                auto t = sm.toEdgeType(space, e.first);
                if (!t.ok()) return fail(t.status().msg_);
                addToEdgeTypes(t.value());
                const std::string& alias = e.second.empty() ? e.first : e.second;
                if (!ctx.addEdge(alias, std::abs(t.value()))) return fail("edge alias(" + alias + ") was dup");
            }
        }
        // prepareWhere (:321-326) -> WhereWrapper::prepare (TraverseExecutor.cpp:426-459)
        if (s.hasWhere) {
            auto d = Expression::decode(s.where);
            if (!d.ok()) return fail(d.status().msg_);
            filter = d.value();
            auto st = filter->prepare(&ctx);
            if (!st.ok()) return fail(st.msg_);
            if (flags.filter_pushdown) {
                auto copy = Expression::decode(Expression::encode(filter.get()));
                if (!copy.ok()) return fail(copy.status().msg_);
                if (rewriteForPushdown(copy.value().get())) filterPushdown = Expression::encode(copy.value().get());
            }
        }
        // prepareYield / prepareNeededProps (:329-407)
        for (auto& y : s.yields) {
            auto d = Expression::decode(y.expr);
            if (!d.ok()) return fail(d.status().msg_);
            yields.push_back(d.value());
            yieldAliases.push_back(y.alias);
        }
        for (auto& y : yields) {
            auto st = y->prepare(&ctx);
            if (!st.ok()) return fail(st.msg_);
        }
        if (ctx.hasVariableProp()) {                                   // :367-384
            if (s.fromType != 2) return fail("A variable must be referred in FROM before used in WHERE or YIELD");
            if (ctx.variables.size() > 1) return fail("Only one variable allowed to use");
            if (*ctx.variables.begin() != s.fromVar)
                return fail("Variable name not match: `" + *ctx.variables.begin() + "' vs. `" + s.fromVar + "'");
        }
        if (ctx.hasInputProp() && s.fromType != 1)                    // :386-392
            return fail("`$-' must be referred in FROM before used in WHERE or YIELD");
        for (auto& e : ctx.tagMap) {
            auto id = sm.toTagID(space, e.first);
            if (!id.ok()) return fail("Tag `" + e.first + "' not found.");
            e.second = id.value();
        }
        // checkNeededProps (:422-468)
        auto tagProps = ctx.srcTagProps;
        tagProps.insert(ctx.dstTagProps.begin(), ctx.dstTagProps.end());
        for (auto& p : tagProps) {
            TagID tagId;
            if (!ctx.getTagId(p.first, tagId)) return fail("Tag `" + p.first + "' not found.");
            auto ts = sm.getTagSchema(space, tagId);
            if (!ts) return fail("No tag schema for " + p.first);
            if (ts->getFieldIndex(p.second) == -1) return fail("`" + p.second + "' is not a prop of `" + p.first + "'");
        }
        for (auto& p : ctx.aliasProps) {
            EdgeType et;
            if (!ctx.getEdgeType(p.first, et)) return fail("Edge `" + p.first + "' not found.");
            if (p.second == "_src" || p.second == "_dst" || p.second == "_rank" || p.second == "_type") continue;
            auto es = sm.getEdgeSchema(space, std::abs(et));
            if (!es) return fail("No edge schema for " + p.first);
            if (es->getFieldIndex(p.second) == -1) return fail("`" + p.second + "' is not a prop of `" + p.first + "'");
        }
        return true;
    }

    // getStepOutProps (:840-914)
    std::vector<PropDef> getStepOutProps() {
        std::vector<PropDef> props;
        for (auto e : edgeTypes) props.push_back(PropDef{EDGE, e, "_dst"});
        if (!isRecord()) return props;
        for (auto& tp : ctx.srcTagProps) {
            auto id = sm.toTagID(space, tp.first);
            props.push_back(PropDef{SOURCE, id.ok() ? id.value() : 0, tp.second});
        }
        for (auto& ap : ctx.aliasProps) {
            if (ap.second == "_dst") continue;
            EdgeType et = 0;
            ctx.getEdgeType(ap.first, et);
            if (s.direction == 0) props.push_back(PropDef{EDGE, et, ap.second});
            else if (s.direction == 1) props.push_back(PropDef{EDGE, -et, ap.second});
            else { props.push_back(PropDef{EDGE, et, ap.second}); props.push_back(PropDef{EDGE, -et, ap.second}); }
        }
        return props;
    }

    // StorageClient::clusterIdsToHosts + getNeighbors for one host.
    GetNeighborsRequest makeRequest(const std::vector<VertexID>& vids) {
        GetNeighborsRequest req;
        req.space = space;
        int32_t numParts = sm.partsNum(space);
        std::map<PartitionID, size_t> slot;
        for (auto v : vids) {
            PartitionID p = idHash(v, numParts);
            auto it = slot.find(p);
            if (it == slot.end()) {
                slot[p] = req.parts.size();
                req.parts.push_back({p, {v}});
            } else {
                req.parts[it->second].second.push_back(v);
            }
        }
        return req;
    }

    bool stepOutLoop() {                                               // :520-606
        while (true) {
            auto returns = getStepOutProps();
            std::string pushed;
            if (flags.filter_pushdown && isFinalStep() && s.direction == 0) pushed = filterPushdown;
            auto tr = std::chrono::steady_clock::now();
            auto req = makeRequest(starts);
            trace("request", tr);
            req.edge_types = edgeTypes;
            req.filter = pushed;
            req.return_columns = returns;
            res.hopFrontier.push_back(static_cast<int64_t>(starts.size()));
            auto tq = std::chrono::steady_clock::now();
            auto resp = eng.getBound(req);
            trace("getBound", tq);
            // edges the storage scan iterated (the TEPS numerator): counted by the buckets themselves
            res.hopScanned.push_back(resp.scanned);
            if (!resp.failed_codes.empty()) return fail("Get neighbors failed");
            records.push_back(std::move(resp));
            tq = std::chrono::steady_clock::now();
            // getDstIdsFromRespWithBackTrack (:675-718) — the frontier is the set of distinct dsts;
            // for steps > 1 the back tracker records (step, dst) -> root for non-final steps, all
            // pairs of the step read before any is inserted
            // (the roots are read only by a sentence whose FROM is $- / $var (getRoots, :1317-1330): with
            // literal vids the tracker changes no result, and this harness skips building it)
            const bool track = !isFinalStep() && steps != 1 && s.fromType != 0;
            std::unordered_set<VertexID> set;
            std::set<std::pair<VertexID, VertexID>> curBackTrace;
            const int T = flags.threads;
            if (!track && T > 1 && records.back().vertices.size() >= 1024) {
                // the same set on every thread: thread t inserts the dsts whose hash falls in its
                // partition (each reads every edge, inserts 1/T of them); the union is the frontier
                std::vector<std::unordered_set<VertexID>> sets(T);
                std::vector<std::thread> ts;
                for (int t = 0; t < T; t++) {
                    ts.emplace_back([&, t] {
                        for (auto& vd : records.back().vertices)
                            for (auto& ed : vd.edge_data)
                                for (auto& e : ed.edges)
                                    if (std::hash<VertexID>()(e.dst) % T == static_cast<size_t>(t)) sets[t].insert(e.dst);
                    });
                }
                for (auto& th : ts) th.join();
                trace("frontier", tq);
                if (isFinalStep()) return true;
                starts.clear();
                for (auto& st : sets) starts.insert(starts.end(), st.begin(), st.end());
                if (starts.empty()) {
                    if (!isRecord()) { records.clear(); return true; }
                    return true;
                }
                curStep++;
                continue;
            }
            for (auto& vd : records.back().vertices)
                for (auto& ed : vd.edge_data)
                    for (auto& e : ed.edges) {
                        if (track) {
                            if (curStep == 1) {
                                curBackTrace.emplace(e.dst, vd.vertex_id);
                            } else {
                                auto pre = backTracker.equal_range({curStep - 1, vd.vertex_id});
                                for (auto t = pre.first; t != pre.second; ++t) curBackTrace.emplace(e.dst, t->second);
                            }
                        }
                        set.insert(e.dst);
                    }
            if (track)
                for (auto& t : curBackTrace) backTracker.emplace(std::make_pair(curStep, t.first), t.second);
            trace("frontier", tq);
            if (isFinalStep()) return true;
            starts.assign(set.begin(), set.end());
            if (starts.empty()) {
                if (!isRecord()) { records.clear(); return true; }   // onEmptyInputs
                return true;
            }
            curStep++;
        }
    }

    bool fetchVertexProps() {                                          // :610-635, :937-973
        if (!ctx.hasDstTagProp()) return true;
        std::unordered_set<VertexID> set;
        for (size_t i = recordFrom - 1; i < records.size(); i++)
            for (auto& vd : records[i].vertices)
                for (auto& ed : vd.edge_data)
                    for (auto& e : ed.edges) set.insert(e.dst);
        if (set.empty()) { records.clear(); return true; }
        std::vector<VertexID> ids(set.begin(), set.end());
        auto req = makeRequest(ids);
        req.has_edge_types = false;
        for (auto& tp : ctx.dstTagProps) {
            auto id = sm.toTagID(space, tp.first);
            if (!id.ok()) return fail("No schema found for '" + tp.first + "'");
            req.return_columns.push_back(PropDef{DEST, id.value(), tp.second});
        }
        auto resp = eng.getBound(req, /*onlyVertexProps=*/true);
        if (!resp.failed_codes.empty()) return fail("Get dest props failed");
        for (auto& kv : resp.vertex_schema) vertexHolderSchemas.emplace(kv.first, kv.second);
        for (auto& vd : resp.vertices) {
            for (auto& td : vd.tag_data) {
                vertexHolder.emplace(std::make_pair(vd.vertex_id, td.tag_id),
                                     std::make_pair(td.data, vertexHolderSchemas[td.tag_id]));
            }
        }
        return true;
    }

    SupportedType calculateExprType(const Expression* e) {             // TraverseExecutor.cpp:88-165
        switch (e->kind()) {
            case Expression::kPrimary: case Expression::kFunctionCall:
            case Expression::kUnary: case Expression::kArithmetic: return UNKNOWN;
            case Expression::kTypeCasting:
                return columnTypeToSupportedType(static_cast<const TypeCastingExpression*>(e)->type_);
            case Expression::kRelational: case Expression::kLogical: return BOOL;
            case Expression::kDestProp: case Expression::kSourceProp: {
                auto* a = static_cast<const AliasPropertyExpression*>(e);
                auto id = sm.toTagID(space, a->alias());
                if (id.ok()) {
                    auto ts = sm.getTagSchema(space, id.value());
                    if (ts) return ts->getFieldType(a->prop());
                }
                return UNKNOWN;
            }
            case Expression::kEdgeDstId: case Expression::kEdgeSrcId: return VID;
            case Expression::kEdgeRank: case Expression::kEdgeType: return INT;
            case Expression::kVariableProp: case Expression::kInputProp: {
                // the interim result's column type; UNKNOWN without data (:141-158)
                if (s.inputRows.empty()) return UNKNOWN;
                auto* a = static_cast<const AliasPropertyExpression*>(e);
                for (size_t i = 0; i < s.inputNames.size(); i++)
                    if (s.inputNames[i] == a->prop()) return s.inputTypes[i];
                return UNKNOWN;
            }
            case Expression::kAliasProp: {
                auto* a = static_cast<const AliasPropertyExpression*>(e);
                auto et = sm.toEdgeType(space, a->alias());
                if (et.ok()) {
                    auto es = sm.getEdgeSchema(space, et.value());
                    if (es) return es->getFieldType(a->prop());
                }
                return UNKNOWN;
            }
            default: return UNKNOWN;
        }
    }

    // Evaluation state of processFinalResult (:1082-1335): the getters read the edge being evaluated.
    // One per thread when the rows are split over threads (GoFlags::threads).
    struct FinalEval {
        GoExec& x;
        const std::map<TagID, std::shared_ptr<Schema>>& tagSchema;
        const std::map<EdgeType, std::shared_ptr<Schema>>& edgeSchema;
        VertexID srcId = 0, dstId = 0;
        EdgeType edgeType = 0;
        const std::vector<TagData>* tagData = nullptr;
        RowReader rd;                                  // the edge's row (reset per edge, no allocation)
        bool reader = false;
        size_t inputRow = 0;
        Getters g;
        FinalEval(GoExec& ex, const std::map<TagID, std::shared_ptr<Schema>>& ts,
                  const std::map<EdgeType, std::shared_ptr<Schema>>& es)
            : x(ex), tagSchema(ts), edgeSchema(es) {
            g.getEdgeDstId = [this](const std::string& edgeName) -> OptVariant {
                if (x.edgeTypes.size() > 1) {
                    EdgeType t;
                    if (!x.ctx.getEdgeType(edgeName, t)) return Status::Error("Get edge type failed in getters.");
                    if (t != std::abs(edgeType)) return OptVariant(int64_t(0));
                }
                return OptVariant(dstId);
            };
            g.getSrcTagProp = [this](const std::string& tag, const std::string& prop) -> OptVariant {
                TagID tagId;
                if (!x.ctx.getTagId(tag, tagId)) return Status::Error("Get tag id failed in getters.");
                const TagData* found = nullptr;
                for (auto& td : *tagData) if (td.tag_id == tagId) { found = &td; break; }
                if (!found) {
                    auto ts = x.sm.getTagSchema(x.space, tagId);
                    if (!ts) return Status::Error("No tag schema");
                    auto d = RowReader::getDefaultProp(ts.get(), prop);
                    if (!d.ok()) return d.status();
                    return OptVariant(d.value());
                }
                auto sit = tagSchema.find(tagId);
                auto vr = RowReader::make(found->data, sit == tagSchema.end() ? nullptr : sit->second);
                if (!vr) return Status::Error("bad tag row");
                auto r = RowReader::getPropByName(vr.get(), prop);
                if (!r.ok()) return Status::Error("get prop failed");
                return OptVariant(r.v);
            };
            g.getDstTagProp = [this](const std::string& tag, const std::string& prop) -> OptVariant {
                TagID tagId;
                if (!x.ctx.getTagId(tag, tagId)) return Status::Error("Get tag id failed in getters.");
                auto it = x.vertexHolder.find({dstId, tagId});
                bool ok = false;
                Variant v;
                if (it != x.vertexHolder.end()) {
                    auto vr = RowReader::make(it->second.first, it->second.second);
                    if (vr) {
                        auto r = RowReader::getPropByName(vr.get(), prop);
                        if (r.ok()) { ok = true; v = r.v; }
                    }
                } else {
                    // VertexHolder::getDefaultProp: the holder's response schema, else the latest one
                    auto hs = x.vertexHolderSchemas.find(tagId);
                    StatusOr<Variant> d = hs != x.vertexHolderSchemas.end()
                        ? RowReader::getDefaultProp(hs->second.get(), prop)
                        : (x.sm.getTagSchema(x.space, tagId) ? RowReader::getDefaultProp(x.sm.getTagSchema(x.space, tagId).get(), prop)
                                                             : StatusOr<Variant>(Status::Error("No tag schema")));
                    if (d.ok()) { ok = true; v = d.value(); }
                }
                if (!ok) {
                    auto ts = x.sm.getTagSchema(x.space, tagId);
                    if (!ts) return Status::Error("No tag schema");
                    auto d = RowReader::getDefaultProp(ts.get(), prop);
                    if (!d.ok()) return d.status();
                    return OptVariant(d.value());
                }
                return OptVariant(v);
            };
            g.getAliasProp = [this](const std::string& edgeName, const std::string& prop) -> OptVariant {
                EdgeType type;
                if (!x.ctx.getEdgeType(edgeName, type)) return Status::Error("Get edge type failed in getters.");
                if (std::abs(edgeType) != type) {
                    auto sit = edgeSchema.find(x.s.direction == 1 ? -type : type);
                    if (sit == edgeSchema.end()) return Status::Error("Can't find schema when get default.");
                    auto d = RowReader::getDefaultProp(sit->second.get(), prop);
                    if (!d.ok()) return d.status();
                    return OptVariant(d.value());
                }
                if (prop == "_src") return OptVariant(srcId);
                if (!reader) return Status::Error("null reader");
                auto r = RowReader::getPropByName(&rd, prop);
                if (!r.ok()) return Status::Error("get prop failed");
                return OptVariant(r.v);
            };
            g.getInputProp = [this](const std::string& prop) { return x.getColumnWithRow(inputRow, prop); };
            g.getVariableProp = [this](const std::string& prop) { return x.getColumnWithRow(inputRow, prop); };
        }
    };

    // rows (or their digests) of one thread's vertex range, and the first evaluation error in it
    struct FinalOut {
        std::vector<std::vector<Variant>> rows;
        std::string digests;
        uint64_t count = 0;
        bool ok = true;
        std::string error;
    };

    bool processFinalResult() {                                        // :1082-1335
        std::vector<SupportedType> colTypes;
        for (auto& y : yields) colTypes.push_back(calculateExprType(y.get()));
        res.colTypes = colTypes;
        std::map<TagID, std::shared_ptr<Schema>> tagSchema;
        std::map<EdgeType, std::shared_ptr<Schema>> edgeSchema;
        std::set<std::vector<Variant>> uniq;
        const bool par = flags.threads > 1 && s.fromType == 0 && !s.distinct;
        // one vertex's edges (with the input row bound for pipes); false on an evaluation error
        auto vertexRows = [&](FinalEval& ev, const VertexData& vd, FinalOut& out) -> bool {
            for (auto& ed : vd.edge_data) {
                ev.edgeType = ed.type;
                auto sit = edgeSchema.find(ev.edgeType);
                for (auto& e : ed.edges) {
                    ev.dstId = e.dst;
                    ev.reader = sit != edgeSchema.end() && RowReader::reset(ev.rd, e.props, sit->second.get());
                    if (filter) {
                        auto v = filter->eval(ev.g);
                        if (!v.ok()) { out.ok = false; out.error = v.status().msg_; return false; }
                        if (!Expression::asBool(v.value())) continue;
                    }
                    std::vector<Variant> record;
                    record.reserve(yields.size());
                    for (auto& y : yields) {
                        auto v = y->eval(ev.g);
                        if (!v.ok()) { out.ok = false; out.error = v.status().msg_; return false; }
                        record.push_back(v.value());
                    }
                    if (s.distinct && !uniq.insert(record).second) continue;
                    out.count++;
                    if (flags.digest) {
                        const size_t at = out.digests.size();
                        out.digests.resize(at + 16);
                        flags.digest(colTypes, record, reinterpret_cast<uint8_t*>(&out.digests[at]));
                    } else {
                        out.rows.push_back(std::move(record));
                    }
                }
            }
            return true;
        };
        auto range = [&](FinalEval& ev, const QueryResponse& resp, size_t recordIn, size_t lo, size_t hi, FinalOut& out) {
            for (size_t vi = lo; vi < hi; vi++) {
                const VertexData& vd = resp.vertices[vi];
                ev.tagData = &vd.tag_data;
                ev.srcId = vd.vertex_id;
                if (s.fromType == 0) {
                    if (!vertexRows(ev, vd, out)) return;
                } else {                                               // :1321-1330
                    for (auto row : rowsOfVids(getRoots(ev.srcId, recordIn))) {
                        ev.inputRow = row;
                        if (!vertexRows(ev, vd, out)) return;
                    }
                }
            }
        };
        auto absorb = [&](FinalOut& out) -> bool {
            res.rowCount += out.count;
            res.digests += out.digests;
            for (auto& r : out.rows) res.rows.push_back(std::move(r));
            if (!out.ok) return fail(out.error);
            return true;
        };
        size_t recordIn = recordFrom;                                   // :1089
        for (size_t ri = recordFrom - 1; ri < records.size(); ri++, recordIn++) {
            auto& resp = records[ri];
            for (auto& kv : resp.vertex_schema) tagSchema.emplace(kv.first, kv.second);
            for (auto& kv : resp.edge_schema) edgeSchema.emplace(kv.first, kv.second);
            const size_t nv = resp.vertices.size();
            const int T = par && nv >= 1024 ? flags.threads : 1;
            std::vector<FinalOut> outs(T);
            if (T == 1) {
                FinalEval ev(*this, tagSchema, edgeSchema);
                range(ev, resp, recordIn, 0, nv, outs[0]);
            } else {
                std::vector<std::thread> ts;
                for (int t = 0; t < T; t++) {
                    ts.emplace_back([&, t] {
                        FinalEval ev(*this, tagSchema, edgeSchema);
                        range(ev, resp, recordIn, nv * t / T, nv * (t + 1) / T, outs[t]);
                    });
                }
                for (auto& th : ts) th.join();
            }
            // in sequential order: the first failing range's error is the first error of the record
            for (auto& out : outs) if (!absorb(out)) return false;
        }
        return true;
    }

    GoResult run() {
        if (!prepareClauses()) return res;
        for (size_t i = 0; i < yields.size(); i++) {
            res.columnNames.push_back(yieldAliases[i].empty() ? yields[i]->toString() : yieldAliases[i]);
        }
        if (steps == 0) return res;                                    // :99-104
        if (recordFrom == 0) recordFrom = 1;
        if (s.fromType == 0) starts = s.vids;
        else if (!setupStarts()) return res;
        if (starts.empty()) return res;
        if (s.distinct) {
            std::unordered_set<VertexID> u(starts.begin(), starts.end());
            starts.assign(u.begin(), u.end());
        }
        if (!stepOutLoop()) return res;
        if (records.empty()) return res;
        if (!fetchVertexProps()) return res;
        if (records.empty()) return res;
        if (ctx.overAll && yields.empty()) {                           // :723-732
            for (auto& a : ctx.edgeAlias) {
                auto e = std::make_shared<AliasPropertyExpression>("", a, "_dst");
                e->setKind(Expression::kEdgeDstId);
                yields.push_back(e);
                res.columnNames.push_back(e->toString());             // getResultColumnNames
            }
        }
        auto tf = std::chrono::steady_clock::now();
        processFinalResult();
        trace("final", tf);
        return std::move(res);                                         // a member: not copied (7 M rows at C2)
    }
};

}  // namespace

GoResult runGo(const StorageEngine& eng, GraphSpaceID space, const GoSentence& s, const GoFlags& f) {
    GoExec e(eng, space, s, f);
    return e.run();
}

}  // namespace orc
