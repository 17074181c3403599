#include <thread>
#include <chrono>
// ORACLE — TEST INFRASTRUCTURE ONLY (see orc_core.h header).
// extern "C" surface used by oracle/oracle.py (ctypes). Requests arrive as little-endian blobs
// built by the Python side; responses are returned as blobs the Python side decodes. Response
// rows are returned both as raw RowWriter bytes and decoded with their response schema.
#include <cstdio>

#include "orc_query.h"

using namespace orc;

namespace {

struct Reader {
    const uint8_t* p;
    const uint8_t* e;
    template <typename T> T get() { T v; std::memcpy(&v, p, sizeof(T)); p += sizeof(T); return v; }
    std::string str() { auto n = get<uint32_t>(); std::string s(reinterpret_cast<const char*>(p), n); p += n; return s; }
};
struct Writer {
    std::string b;
    template <typename T> void put(T v) { b.append(reinterpret_cast<const char*>(&v), sizeof(T)); }
    void str(const std::string& s) { put<uint32_t>(static_cast<uint32_t>(s.size())); b.append(s); }
    void variant(const Variant& v) {
        put<uint8_t>(static_cast<uint8_t>(which(v)));
        switch (which(v)) {
            case VAR_INT64: put<int64_t>(std::get<int64_t>(v)); break;
            case VAR_DOUBLE: put<double>(std::get<double>(v)); break;
            case VAR_BOOL: put<uint8_t>(std::get<bool>(v) ? 1 : 0); break;
            default: str(std::get<std::string>(v)); break;
        }
    }
    void schema(const Schema& s) {
        put<int32_t>(static_cast<int32_t>(s.fields.size()));
        for (auto& f : s.fields) { str(f.name); put<int32_t>(f.type); }
    }
    void row(const std::string& bytes, const std::shared_ptr<Schema>& schema) {
        str(bytes);
        if (!schema) { put<int32_t>(-1); return; }
        auto r = RowReader::make(bytes, schema);
        if (!r) { put<int32_t>(-1); return; }
        put<int32_t>(static_cast<int32_t>(schema->fields.size()));
        for (auto& f : schema->fields) {
            auto v = RowReader::getPropByName(r.get(), f.name);
            if (!v.ok()) { put<uint8_t>(0xFF); continue; }
            variant(v.v);
        }
    }
};

char* toHeap(const std::string& s, uint64_t* len) {
    char* out = static_cast<char*>(std::malloc(s.size() ? s.size() : 1));
    std::memcpy(out, s.data(), s.size());
    *len = s.size();
    return out;
}

// ColumnValue per GoExecutor::toThriftResponse (GoExecutor.cpp:775-829)
void cell(Writer& w, SupportedType t, const Variant& v) {
    auto typeErr = [&] { w.put<uint8_t>(0xFE); };
    switch (t) {
        case BOOL: if (which(v) != VAR_BOOL) return typeErr(); w.put<uint8_t>(1); w.put<uint8_t>(std::get<bool>(v)); return;
        case INT: if (which(v) != VAR_INT64) return typeErr(); w.put<uint8_t>(2); w.put<int64_t>(std::get<int64_t>(v)); return;
        case VID: if (which(v) != VAR_INT64) return typeErr(); w.put<uint8_t>(3); w.put<int64_t>(std::get<int64_t>(v)); return;
        case FLOAT: if (which(v) != VAR_DOUBLE) return typeErr(); w.put<uint8_t>(4); w.put<double>(std::get<double>(v)); return;
        case DOUBLE: if (which(v) != VAR_DOUBLE) return typeErr(); w.put<uint8_t>(5); w.put<double>(std::get<double>(v)); return;
        case STRING: if (which(v) != VAR_STR) return typeErr(); w.put<uint8_t>(6); w.str(std::get<std::string>(v)); return;
        case TIMESTAMP: if (which(v) != VAR_INT64) return typeErr(); w.put<uint8_t>(21); w.put<int64_t>(std::get<int64_t>(v)); return;
        default:
            switch (which(v)) {
                case VAR_INT64: w.put<uint8_t>(2); w.put<int64_t>(std::get<int64_t>(v)); return;
                case VAR_DOUBLE: w.put<uint8_t>(5); w.put<double>(std::get<double>(v)); return;
                // left unset by toThriftResponse; the value travels on for an interim result (pipe)
                case VAR_BOOL: w.put<uint8_t>(0xFD); w.put<uint8_t>(std::get<bool>(v)); return;
                default: w.put<uint8_t>(6); w.str(std::get<std::string>(v)); return;
            }
    }
}

template <typename F>
void parallelChunks(uint64_t n, F&& f) {
    unsigned T = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (n < (1u << 15) || T == 1) { f(0, n); return; }
    std::vector<std::thread> ts;
    for (unsigned t = 0; t < T; t++) ts.emplace_back([&f, n, t, T] { f(n * t / T, n * (t + 1) / T); });
    for (auto& th : ts) th.join();
}

// 128-bit digest of one serialized row (test comparison of large results: sorted digests of the
// device's rows against the oracle's, instead of Python tuples)
void rowDigest(const std::string& b, uint8_t* out16) {
    uint64_t h1 = 1469598103934665603ULL, h2 = 0x9E3779B97F4A7C15ULL ^ b.size();
    for (unsigned char ch : b) { h1 ^= ch; h1 *= 1099511628211ULL; }
    size_t i = 0;
    for (; i + 8 <= b.size(); i += 8) {
        uint64_t k;
        std::memcpy(&k, b.data() + i, 8);
        k *= 0x87c37b91114253d5ULL; k = (k << 31) | (k >> 33); k *= 0x4cf5ad432745937fULL;
        h2 ^= k; h2 = ((h2 << 27) | (h2 >> 37)) * 5 + 0x52dce729;
    }
    uint64_t k = 0;
    for (size_t j = 0; i + j < b.size(); j++) k |= static_cast<uint64_t>(static_cast<unsigned char>(b[i + j])) << (8 * j);
    h2 ^= k * 0x87c37b91114253d5ULL;
    h2 ^= h2 >> 33; h2 *= 0xff51afd7ed558ccdULL; h2 ^= h2 >> 33;
    std::memcpy(out16, &h1, 8);
    std::memcpy(out16 + 8, &h2, 8);
}

// GoFlags::digest: a result row serialized as its ColumnValue cells, then digested
void digestRow(const std::vector<SupportedType>& colTypes, const std::vector<Variant>& row, uint8_t* out16) {
    thread_local Writer w;
    w.b.clear();
    for (size_t c = 0; c < row.size(); c++) cell(w, c < colTypes.size() ? colTypes[c] : UNKNOWN, row[c]);
    rowDigest(w.b, out16);
}

}  // namespace

extern "C" {

// Digest rows given column-wise as the device path's host_columnar result (include/nebula_gn.h):
// x = value bits (string: host pointer to bytes), len = string lengths or NULL, t = per-row V_* type
// (1 int, 2 double, 3 bool, 4 string) or NULL for rows of the column's static type. Each row is
// serialized exactly as orc_go serializes the oracle's cells (ColumnValue typing of
// toThriftResponse), then digested.
void orc_digest_columns(int32_t ncols, const int32_t* colTypes, uint64_t nrows, const int64_t* const* x,
                        const uint32_t* const* len, const uint8_t* const* t, uint8_t* out16) {
    parallelChunks(nrows, [&](uint64_t lo, uint64_t hi) {
    Writer w;
    for (uint64_t r = lo; r < hi; r++) {
        w.b.clear();
        for (int32_t c = 0; c < ncols; c++) {
            int32_t ct = colTypes[c];
            uint8_t vt;
            if (t[c]) vt = t[c][r];
            else vt = ct == BOOL ? 3 : (ct == FLOAT || ct == DOUBLE) ? 2 : ct == STRING ? 4 : 1;
            int64_t v = x[c][r];
            double d;
            std::memcpy(&d, &v, 8);
            auto str = [&] {
                uint32_t n = len[c] ? len[c][r] : 0;
                w.put<uint8_t>(6);
                w.str(n ? std::string(reinterpret_cast<const char*>(v), n) : std::string());
            };
            switch (ct) {
                case BOOL: w.put<uint8_t>(1); w.put<uint8_t>(v != 0); break;
                case INT: w.put<uint8_t>(2); w.put<int64_t>(v); break;
                case VID: w.put<uint8_t>(3); w.put<int64_t>(v); break;
                case FLOAT: w.put<uint8_t>(4); w.put<double>(d); break;
                case DOUBLE: w.put<uint8_t>(5); w.put<double>(d); break;
                case STRING: str(); break;
                case TIMESTAMP: w.put<uint8_t>(21); w.put<int64_t>(v); break;
                default:
                    if (vt == 1) { w.put<uint8_t>(2); w.put<int64_t>(v); }
                    else if (vt == 2) { w.put<uint8_t>(5); w.put<double>(d); }
                    else if (vt == 3) { w.put<uint8_t>(0xFD); w.put<uint8_t>(v != 0); }
                    else str();
            }
        }
        rowDigest(w.b, out16 + 16 * r);
    }
    });
}

void* orc_engine_new() { return new StorageEngine(); }
void orc_engine_free(void* e) { delete static_cast<StorageEngine*>(e); }
void orc_buf_free(void* p) { std::free(p); }

void orc_set_flags(void* e, int32_t maxHandlers, int32_t minVertices, int32_t maxEdges, int64_t nowSec,
                   int32_t threads) {
    auto& f = static_cast<StorageEngine*>(e)->flags;
    f.max_handlers_per_req = maxHandlers;
    f.min_vertices_per_bucket = minVertices;
    f.max_edge_returned_per_vertex = maxEdges;
    f.now_sec = nowSec;
    f.threads = threads;
}
void orc_set_graph_threads(void* e, int32_t threads) {
    static_cast<StorageEngine*>(e)->flags.graph_threads = threads < 1 ? 1 : threads;
}

void orc_add_space(void* e, int32_t space, int32_t numParts) {
    auto* eng = static_cast<StorageEngine*>(e);
    eng->schemas.addSpace(space, numParts);
    auto& kv = eng->stores[space];
    for (int32_t p = 1; p <= numParts; p++) kv.addPart(p);
}
void orc_add_part(void* e, int32_t space, int32_t part) {
    static_cast<StorageEngine*>(e)->stores[space].addPart(part);
}

int32_t orc_add_schema(void* e, int32_t space, int32_t isEdge, int32_t id, const char* name, int64_t ver,
                       int32_t nfields, const char** names, const int32_t* types, const char* ttlCol,
                       int64_t ttlDur) {
    auto s = std::make_shared<Schema>();
    s->ver = ver;
    for (int32_t i = 0; i < nfields; i++) s->fields.push_back(Field{names[i], static_cast<SupportedType>(types[i])});
    s->ttlCol = ttlCol ? ttlCol : "";
    s->ttlDuration = ttlDur;
    auto& sm = static_cast<StorageEngine*>(e)->schemas;
    if (isEdge) sm.addEdgeSchema(space, id, name, s); else sm.addTagSchema(space, id, name, s);
    return 0;
}

void orc_put_kv(void* e, int32_t space, uint64_t n, const uint8_t* keys, const uint64_t* koff,
                const uint8_t* vals, const uint64_t* voff) {
    auto& kv = static_cast<StorageEngine*>(e)->stores[space];
    kv.reserve(kv.size() + n, (koff[n] - koff[0]) + (voff[n] - voff[0]));   // (added to what the store holds)
    for (uint64_t i = 0; i < n; i++) {
        kv.put(reinterpret_cast<const char*>(keys + koff[i]), koff[i + 1] - koff[i],
               reinterpret_cast<const char*>(vals + voff[i]), voff[i + 1] - voff[i]);
    }
}
void orc_finalize(void* e, int32_t threads) {
    for (auto& kv : static_cast<StorageEngine*>(e)->stores) kv.second.finalize(threads);
}
uint64_t orc_kv_size(void* e, int32_t space) { return static_cast<StorageEngine*>(e)->stores[space].size(); }

// request blob: i32 space; i32 nparts {i32 part, i32 n, i64 vids[n]}; u8 hasTypes; i32 ntypes i32[];
//               str filter; i32 ncols {i32 owner, i32 id, str name}; u8 onlyVertexProps
char* orc_get_neighbors(void* e, const uint8_t* req, uint64_t len, uint64_t* outLen) {
    auto* eng = static_cast<StorageEngine*>(e);
    Reader r{req, req + len};
    GetNeighborsRequest q;
    q.space = r.get<int32_t>();
    int32_t np = r.get<int32_t>();
    for (int32_t i = 0; i < np; i++) {
        PartitionID p = r.get<int32_t>();
        int32_t n = r.get<int32_t>();
        std::vector<VertexID> v(n);
        for (int32_t j = 0; j < n; j++) v[j] = r.get<int64_t>();
        q.parts.push_back({p, v});
    }
    q.has_edge_types = r.get<uint8_t>() != 0;
    int32_t nt = r.get<int32_t>();
    for (int32_t i = 0; i < nt; i++) q.edge_types.push_back(r.get<int32_t>());
    q.filter = r.str();
    int32_t nc = r.get<int32_t>();
    for (int32_t i = 0; i < nc; i++) {
        PropDef d;
        d.owner = static_cast<PropOwner>(r.get<int32_t>());
        d.id = r.get<int32_t>();
        d.name = r.str();
        q.return_columns.push_back(d);
    }
    bool onlyVertexProps = r.get<uint8_t>() != 0;
    auto resp = eng->getBound(q, onlyVertexProps);
    Writer w;
    w.put<int32_t>(static_cast<int32_t>(resp.failed_codes.size()));
    for (auto& fc : resp.failed_codes) { w.put<int32_t>(fc.first); w.put<int32_t>(fc.second); }
    w.put<int32_t>(static_cast<int32_t>(resp.vertex_schema.size()));
    for (auto& kv : resp.vertex_schema) { w.put<int32_t>(kv.first); w.schema(*kv.second); }
    w.put<int32_t>(static_cast<int32_t>(resp.edge_schema.size()));
    for (auto& kv : resp.edge_schema) { w.put<int32_t>(kv.first); w.schema(*kv.second); }
    w.put<int32_t>(static_cast<int32_t>(resp.vertices.size()));
    for (auto& v : resp.vertices) {
        w.put<int64_t>(v.vertex_id);
        w.put<int32_t>(static_cast<int32_t>(v.tag_data.size()));
        for (auto& td : v.tag_data) {
            w.put<int32_t>(td.tag_id);
            auto s = resp.vertex_schema.find(td.tag_id);
            w.row(td.data, s == resp.vertex_schema.end() ? nullptr : s->second);
        }
        w.put<int32_t>(static_cast<int32_t>(v.edge_data.size()));
        for (auto& ed : v.edge_data) {
            w.put<int32_t>(ed.type);
            w.put<int32_t>(static_cast<int32_t>(ed.edges.size()));
            auto s = resp.edge_schema.find(ed.type);
            for (auto& edge : ed.edges) {
                w.put<int64_t>(edge.dst);
                w.put<uint8_t>(edge.has_props ? 1 : 0);
                if (edge.has_props) w.row(edge.props, s == resp.edge_schema.end() ? nullptr : s->second);
            }
        }
    }
    w.put<int32_t>(resp.total_edges);
    return toHeap(w.b, outLen);
}

// sentence blob: u32 from, to; i32 nvids i64[]; i32 nover {str name, str alias}; u8 overAll;
//                i32 direction; u8 hasWhere; str where; u8 distinct; i32 nyields {str expr, str alias};
//                u8 filterPushdown
char* orc_go(void* e, int32_t space, const uint8_t* blob, uint64_t len, uint64_t* outLen) {
    auto* eng = static_cast<StorageEngine*>(e);
    Reader r{blob, blob + len};
    GoSentence s;
    s.recordFrom = r.get<uint32_t>();
    s.recordTo = r.get<uint32_t>();
    int32_t nv = r.get<int32_t>();
    for (int32_t i = 0; i < nv; i++) s.vids.push_back(r.get<int64_t>());
    int32_t no = r.get<int32_t>();
    for (int32_t i = 0; i < no; i++) { auto n = r.str(); auto a = r.str(); s.over.push_back({n, a}); }
    s.overAll = r.get<uint8_t>() != 0;
    s.direction = r.get<int32_t>();
    s.hasWhere = r.get<uint8_t>() != 0;
    s.where = r.str();
    s.distinct = r.get<uint8_t>() != 0;
    int32_t ny = r.get<int32_t>();
    for (int32_t i = 0; i < ny; i++) { auto x = r.str(); auto a = r.str(); s.yields.push_back({x, a}); }
    GoFlags f;
    f.filter_pushdown = r.get<uint8_t>() != 0;
    uint8_t mode = r.p < r.e ? r.get<uint8_t>() : 0;        // 0 cells, 1 count only, 2 row digests
    bool countOnly = mode != 0;
    f.threads = eng->flags.graph_threads;
    if (mode == 2) f.digest = digestRow;
    if (r.p < r.e) {                                        // FROM $-.col / $var.col and the input
        s.fromType = r.get<uint8_t>();
        s.fromVar = r.str();
        s.fromCol = r.str();
        int32_t nc = r.get<int32_t>();
        for (int32_t i = 0; i < nc; i++) {
            s.inputNames.push_back(r.str());
            s.inputTypes.push_back(static_cast<SupportedType>(r.get<int32_t>()));
        }
        int64_t nr = r.get<int64_t>();
        for (int64_t i = 0; i < nr; i++) {
            std::vector<Variant> row;
            for (int32_t j = 0; j < nc; j++) {
                switch (r.get<uint8_t>()) {
                    case VAR_INT64: row.emplace_back(r.get<int64_t>()); break;
                    case VAR_DOUBLE: row.emplace_back(r.get<double>()); break;
                    case VAR_BOOL: row.emplace_back(r.get<uint8_t>() != 0); break;
                    default: row.emplace_back(r.str()); break;
                }
            }
            s.inputRows.push_back(std::move(row));
        }
    }
    auto t0 = std::chrono::steady_clock::now();
    auto res = runGo(*eng, space, s, f);
    double seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    Writer w;
    w.put<uint8_t>(res.ok ? 1 : 0);
    w.str(res.error);
    w.put<int32_t>(static_cast<int32_t>(res.colTypes.size()));
    for (auto t : res.colTypes) w.put<int32_t>(t);
    w.put<int64_t>(static_cast<int64_t>(mode == 2 ? res.rowCount : res.rows.size()));
    if (mode == 2) w.b += res.digests;
    if (countOnly) res.rows.clear();
    for (auto& row : res.rows) {
        for (size_t c = 0; c < row.size(); c++) {
            cell(w, c < res.colTypes.size() ? res.colTypes[c] : UNKNOWN, row[c]);
        }
    }
    w.put<int32_t>(static_cast<int32_t>(res.hopScanned.size()));
    for (size_t i = 0; i < res.hopScanned.size(); i++) {
        w.put<int64_t>(res.hopFrontier[i]);
        w.put<int64_t>(res.hopScanned[i]);
    }
    w.put<double>(seconds);
    w.put<int32_t>(static_cast<int32_t>(res.columnNames.size()));
    for (auto& n : res.columnNames) w.str(n);
    return toHeap(w.b, outLen);
}

// ---- small utilities for tests: expression round trip, eval of constant expressions, row codec
char* orc_expr_eval(const uint8_t* buf, uint64_t len, uint64_t* outLen) {
    Writer w;
    auto d = Expression::decode(std::string(reinterpret_cast<const char*>(buf), len));
    if (!d.ok()) { w.put<uint8_t>(2); w.str(d.status().msg_); return toHeap(w.b, outLen); }
    ExpressionContext ctx;
    auto st = d.value()->prepare(&ctx);
    if (!st.ok()) { w.put<uint8_t>(2); w.str(st.msg_); return toHeap(w.b, outLen); }
    Getters g;
    auto v = d.value()->eval(g);
    if (!v.ok()) { w.put<uint8_t>(0); w.str(v.status().msg_); return toHeap(w.b, outLen); }
    w.put<uint8_t>(1);
    w.variant(v.value());
    return toHeap(w.b, outLen);
}

char* orc_expr_roundtrip(const uint8_t* buf, uint64_t len, uint64_t* outLen) {
    auto d = Expression::decode(std::string(reinterpret_cast<const char*>(buf), len));
    if (!d.ok()) { *outLen = 0; return nullptr; }
    return toHeap(Expression::encode(d.value().get()), outLen);
}

// pushdown rewrite of an encoded filter: returns the encoded rewritten filter or empty
char* orc_expr_pushdown(const uint8_t* buf, uint64_t len, uint64_t* outLen) {
    auto d = Expression::decode(std::string(reinterpret_cast<const char*>(buf), len));
    if (!d.ok() || !rewriteForPushdown(d.value().get())) { *outLen = 0; return toHeap("", outLen); }
    return toHeap(Expression::encode(d.value().get()), outLen);
}

char* orc_expr_to_string(const uint8_t* buf, uint64_t len, uint64_t* outLen) {
    auto d = Expression::decode(std::string(reinterpret_cast<const char*>(buf), len));
    if (!d.ok()) { *outLen = 0; return toHeap("", outLen); }
    return toHeap(d.value()->toString(), outLen);
}

int64_t orc_std_hash_string(const char* s, uint64_t n) {
    return static_cast<int64_t>(std::hash<std::string>()(std::string(s, n)));
}

// Write a row with a schema (types[]) from a values blob (variant list); returns row bytes.
char* orc_row_write(int64_t ver, int32_t nfields, const int32_t* types, const uint8_t* vals, uint64_t vlen,
                    int32_t withSchema, uint64_t* outLen) {
    auto s = std::make_shared<Schema>();
    s->ver = ver;
    for (int32_t i = 0; i < nfields; i++) s->fields.push_back(Field{"c" + std::to_string(i), static_cast<SupportedType>(types[i])});
    RowWriter w(withSchema ? s : nullptr);
    Reader r{vals, vals + vlen};
    while (r.p < r.e) {
        auto t = r.get<uint8_t>();
        switch (t) {
            case 0: w << r.get<int64_t>(); break;
            case 1: w << r.get<double>(); break;
            case 2: w << (r.get<uint8_t>() != 0); break;
            case 3: w << r.str(); break;
            case 4: w << r.get<float>(); break;
            case 5: w << r.get<uint64_t>(); break;
            case 6: w.skip(r.get<int64_t>()); break;
            default: break;
        }
    }
    return toHeap(w.encode(), outLen);
}

// Decode a row with a schema: per field u8 tag + value (0xFF on error)
char* orc_row_read(int64_t ver, int32_t nfields, const int32_t* types, const uint8_t* row, uint64_t rlen,
                   uint64_t* outLen) {
    auto s = std::make_shared<Schema>();
    s->ver = ver;
    for (int32_t i = 0; i < nfields; i++) s->fields.push_back(Field{"c" + std::to_string(i), static_cast<SupportedType>(types[i])});
    Writer w;
    w.row(std::string(reinterpret_cast<const char*>(row), rlen), s);
    return toHeap(w.b, outLen);
}

int32_t orc_row_schema_ver(const uint8_t* row, uint64_t rlen) {
    return RowReader::getSchemaVer(std::string(reinterpret_cast<const char*>(row), rlen));
}

// genBuckets arithmetic: writes bucket sizes, returns count
int32_t orc_gen_buckets(int32_t nvertices, int32_t minPerBucket, int32_t maxHandlers, int32_t* sizes) {
    GetNeighborsRequest q;
    q.parts.push_back({1, std::vector<VertexID>(nvertices, 0)});
    auto b = StorageEngine::genBuckets(q, minPerBucket, maxHandlers);
    for (size_t i = 0; i < b.size(); i++) sizes[i] = static_cast<int32_t>(b[i].size());
    return static_cast<int32_t>(b.size());
}

}  // extern "C"
