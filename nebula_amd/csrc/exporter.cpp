// Part -> CSR snapshot exporter (the north star's src/kvstore + src/dataman changes).
//
// Input: reference-format KV rows of the parts this shard owns (NebulaKeyUtils keys,
// src/common/utils/NebulaKeyUtils.cpp:12-45; RowWriter values, src/dataman/RowWriter.cpp:39-263).
// Output (HostGraph): a vertex table sorted by (part, vid), one CSR per signed edge type with
// adjacency in RocksDB bytewise key order (what KVStore::prefix(edgePrefix(part, vid, type)) walks,
// src/storage/query/QueryBaseProcessor.inl:485-518), latest-version dedup applied, and every prop
// of the latest schema decoded into a typed column the way RowReader::getPropByName reads it
// (src/dataman/RowReader.h:136-193, RowReader.cpp:171-365) — including block offsets every 16
// fields. Tag rows become per-vertex tag columns (first key of vertexPrefix = latest version,
// QueryBaseProcessor.inl:440-476).
#include <algorithm>
#include <atomic>
#include <numeric>
#include <thread>

#include "ngx_internal.h"

namespace ngx {

namespace {

inline uint64_t be64(const uint8_t* p) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    return __builtin_bswap64(v);
}
template <typename T>
inline T rd(const uint8_t* p) { T v; std::memcpy(&v, p, sizeof(T)); return v; }

int hwThreads() { return hostThreadBudget(); }

template <typename F>
void parallelFor(uint64_t n, F&& f) {
    int T = hwThreads();
    if (n < 4096 || T == 1) { f(0, n); return; }
    std::vector<std::thread> ts;
    for (int t = 0; t < T; t++) {
        uint64_t lo = n * t / T, hi = n * (t + 1) / T;
        ts.emplace_back([&f, lo, hi] { f(lo, hi); });
    }
    for (auto& th : ts) th.join();
}

template <typename It, typename Cmp>
void parallelSort(It begin, It end, Cmp cmp) {
    uint64_t n = static_cast<uint64_t>(end - begin);
    int T = hwThreads();
    if (n < (1u << 16) || T == 1) { std::sort(begin, end, cmp); return; }
    std::vector<uint64_t> cuts;
    for (int t = 0; t <= T; t++) cuts.push_back(n * t / T);
    std::vector<std::thread> ts;
    for (int t = 0; t < T; t++) ts.emplace_back([&, t] { std::sort(begin + cuts[t], begin + cuts[t + 1], cmp); });
    for (auto& th : ts) th.join();
    for (int w = 1; w < T; w <<= 1) {
        std::vector<std::thread> ms;
        for (int t = 0; t + w < T; t += 2 * w) {
            uint64_t lo = cuts[t], mid = cuts[t + w], hi = cuts[std::min(t + 2 * w, T)];
            ms.emplace_back([&, lo, mid, hi] { std::inplace_merge(begin + lo, begin + mid, begin + hi, cmp); });
        }
        for (auto& th : ms) th.join();
    }
}

// ---------------------------------------------------------------- row decoding
// Decodes one field of a row with its own (version) schema, following RowReader: the header
// (low 3 bits + 1 = offset width, top 3 bits = version bytes), block offsets for fields 16, 32, ...,
// and a sequential walk inside the field's block.
struct RowView {
    const uint8_t* data = nullptr;     // after the header
    uint64_t size = 0;
    std::vector<uint64_t> blockStart;  // block k starts at blockStart[k]
    bool ok = false;
};

bool parseHeader(const uint8_t* row, uint64_t len, uint32_t numFields, RowView& rv) {
    if (len == 0) return false;
    uint32_t offBytes = (row[0] & 0x07) + 1;
    uint32_t verBytes = row[0] >> 5;
    uint32_t numOffsets = numFields >> 4;
    if (static_cast<uint64_t>(offBytes) * numOffsets + verBytes + 1 > len) return false;
    const uint8_t* it = row + 1 + verBytes;
    rv.blockStart.assign(numOffsets + 1, 0);
    for (uint32_t i = 0; i < numOffsets; i++) {
        uint64_t o = 0;
        for (uint32_t j = 0; j < offBytes; j++) o |= static_cast<uint64_t>(*it++) << (8 * j);
        rv.blockStart[i + 1] = o;
    }
    uint64_t hdr = static_cast<uint64_t>(it - row);
    rv.data = it;
    rv.size = len - hdr;
    rv.ok = true;
    return true;
}

int32_t varint(const uint8_t* p, uint64_t avail, uint64_t& out) {
    uint64_t v = 0;
    for (int i = 0; i < 10; i++) {
        if (static_cast<uint64_t>(i) >= avail) return -1;
        uint8_t b = p[i];
        v |= static_cast<uint64_t>(b & 0x7f) << (7 * i);
        if (!(b & 0x80)) { out = v; return i + 1; }
    }
    return -1;
}

// byte length of field `t` at offset `off`, or -1
int64_t fieldLen(const RowView& rv, int32_t t, uint64_t off) {
    switch (t) {
        case T_BOOL: return 1;
        case T_INT: case T_TIMESTAMP: {
            uint64_t v;
            if (off > rv.size) return -1;
            int32_t n = varint(rv.data + off, rv.size - off, v);
            return n <= 0 ? -1 : n;
        }
        case T_FLOAT: return 4;
        case T_DOUBLE: return 8;
        case T_VID: return 8;
        case T_STRING: {
            uint64_t l;
            if (off > rv.size) return -1;
            int32_t n = varint(rv.data + off, rv.size - off, l);
            if (n <= 0) return -1;
            return static_cast<int64_t>(n + l);
        }
        default: return -1;
    }
}

// offset of field i (RowReader::skipToField)
int64_t fieldOffset(const RowView& rv, const SchemaDef& s, uint32_t i) {
    uint32_t k = i >> 4;
    uint64_t off = rv.blockStart[k];
    for (uint32_t j = k << 4; j < i; j++) {
        int64_t l = fieldLen(rv, s.fields[j].type, off);
        if (l < 0) return -1;
        off += static_cast<uint64_t>(l);
        if (off > rv.size) return -1;
    }
    return static_cast<int64_t>(off);
}

struct Cell {
    bool ok = false;
    int64_t i = 0;
    double d = 0;
    const uint8_t* s = nullptr;
    uint64_t slen = 0;
};

// RowReader::getPropByName for field i of the version schema (RowReader.h:136-193)
Cell readField(const RowView& rv, const SchemaDef& s, uint32_t i) {
    Cell c;
    int64_t off = fieldOffset(rv, s, i);
    if (off < 0) return c;
    uint64_t o = static_cast<uint64_t>(off);
    switch (s.fields[i].type) {
        case T_BOOL:
            if (o >= rv.size) return c;
            c.i = rv.data[o] != 0; c.ok = true; return c;
        case T_INT: case T_TIMESTAMP: {
            uint64_t v;
            if (o > rv.size || varint(rv.data + o, rv.size - o, v) < 0) return c;
            c.i = static_cast<int64_t>(v); c.ok = true; return c;
        }
        case T_VID:
            if (o + 8 > rv.size) return c;
            c.i = rd<int64_t>(rv.data + o); c.ok = true; return c;
        case T_FLOAT:
            if (o + 4 > rv.size) return c;
            c.d = static_cast<double>(rd<float>(rv.data + o)); c.ok = true; return c;
        case T_DOUBLE:
            if (o + 8 > rv.size) return c;
            c.d = rd<double>(rv.data + o); c.ok = true; return c;
        case T_STRING: {
            uint64_t l;
            if (o > rv.size) return c;
            int32_t n = varint(rv.data + o, rv.size - o, l);
            if (n <= 0 || o + n + l > rv.size) return c;
            c.s = rv.data + o + n; c.slen = l; c.ok = true; return c;
        }
        default: return c;
    }
}

int32_t rowSchemaVer(const uint8_t* row, uint64_t len) {     // RowReader::getSchemaVer
    if (len == 0) return -1;
    uint32_t verBytes = row[0] >> 5;
    if (verBytes == 0) return 0;
    if (verBytes + 1 > len) return -1;
    int32_t v = 0;
    for (uint32_t i = 0; i < verBytes; i++) v |= static_cast<int32_t>(static_cast<uint32_t>(row[1 + i]) << (8 * i));
    return v;
}

// A version schema mapped onto the latest schema's columns.
struct VersionMap {
    const SchemaDef* schema = nullptr;
    std::vector<int32_t> colToField;   // latest column -> field index in this version, -1 if absent
};

Error buildVersionMaps(const SchemaSet& ss, std::map<int64_t, VersionMap>& out) {
    const SchemaDef& latest = ss.latest();
    for (auto& kv : ss.versions) {
        VersionMap vm;
        vm.schema = &kv.second;
        for (auto& f : latest.fields) {
            int32_t i = kv.second.index(f.name);
            if (i >= 0 && kv.second.fields[i].type != f.type) {
                return Error{NGX_E_UNSUPPORTED, "schema `" + ss.name + "' changes the type of `" + f.name +
                             "' across versions; not supported by the columnar export"};
            }
            vm.colToField.push_back(i);
        }
        out[kv.first] = std::move(vm);
    }
    return Error{NGX_OK, ""};
}

void initColumns(std::vector<HostColumn>& cols, const SchemaDef& latest, uint64_t n) {
    cols.resize(latest.fields.size());
    for (size_t c = 0; c < cols.size(); c++) {
        auto& col = cols[c];
        col.type = latest.fields[c].type;
        switch (col.type) {
            case T_INT: case T_TIMESTAMP: case T_VID: col.i64.assign(n, 0); break;
            case T_FLOAT: case T_DOUBLE: col.f64.assign(n, 0.0); break;
            case T_BOOL: col.b.assign(n, 0); break;
            case T_STRING: col.soff.assign(n + 1, 0); break;
            default: break;
        }
        col.valid.assign(n, 1);
    }
}

// Decodes `row` into element `e` of `cols`. String bytes are collected per element in `strs`
// and packed afterwards (strings are the only variable-size column).
// Returns EF_* flags for the row.
uint8_t decodeInto(const uint8_t* row, uint64_t len, const std::map<int64_t, VersionMap>& vmaps,
                   std::vector<HostColumn>& cols, uint64_t e, std::vector<std::vector<std::string>>& strs) {
    auto invalidAll = [&]() {
        for (auto& col : cols) { col.valid[e] = 0; }
    };
    if (len == 0) { invalidAll(); return EF_EMPTY_VALUE; }
    int32_t ver = rowSchemaVer(row, len);
    auto it = ver < 0 ? vmaps.end() : vmaps.find(ver);
    if (it == vmaps.end()) { invalidAll(); return EF_BAD_ROW; }
    const VersionMap& vm = it->second;
    RowView rv;
    if (!parseHeader(row, len, static_cast<uint32_t>(vm.schema->fields.size()), rv)) { invalidAll(); return EF_BAD_ROW; }
    for (size_t c = 0; c < cols.size(); c++) {
        auto& col = cols[c];
        int32_t fi = vm.colToField[c];
        Cell v;
        if (fi >= 0) v = readField(rv, *vm.schema, static_cast<uint32_t>(fi));
        if (!v.ok) { col.valid[e] = 0; continue; }
        switch (col.type) {
            case T_INT: case T_TIMESTAMP: case T_VID: col.i64[e] = v.i; break;
            case T_FLOAT: case T_DOUBLE: col.f64[e] = v.d; break;
            case T_BOOL: col.b[e] = static_cast<uint8_t>(v.i); break;
            case T_STRING: strs[c][e].assign(reinterpret_cast<const char*>(v.s), v.slen); break;
            default: break;
        }
    }
    return 0;
}

void packStrings(std::vector<HostColumn>& cols, std::vector<std::vector<std::string>>& strs) {
    for (size_t c = 0; c < cols.size(); c++) {
        auto& col = cols[c];
        col.allValid = std::all_of(col.valid.begin(), col.valid.end(), [](uint8_t v) { return v != 0; });
        if (col.allValid) { col.valid.clear(); col.valid.shrink_to_fit(); }
        if (col.type != T_STRING) continue;
        uint64_t total = 0;
        for (size_t e = 0; e < strs[c].size(); e++) { col.soff[e] = total; total += strs[c][e].size(); }
        col.soff[strs[c].size()] = total;
        col.sbytes.reserve(total);
        for (auto& s : strs[c]) col.sbytes += s;
        strs[c].clear();
        strs[c].shrink_to_fit();
    }
}

struct EdgeRec {
    uint64_t w[5];     // key bytes as big-endian words: memcmp order
    uint64_t row;
};
// the key fields of an edge record, from its words (no second read of the staged key)
inline int32_t recPart(const EdgeRec& r) { return static_cast<int32_t>(__builtin_bswap32(static_cast<uint32_t>(r.w[0] >> 32))) >> 8; }
inline int64_t recSrc(const EdgeRec& r) { return static_cast<int64_t>(__builtin_bswap64((r.w[0] << 32) | (r.w[1] >> 32))); }
inline int32_t recType(const EdgeRec& r) { return static_cast<int32_t>(__builtin_bswap32(static_cast<uint32_t>(r.w[1]))); }
inline int64_t recRank(const EdgeRec& r) { return static_cast<int64_t>(__builtin_bswap64(r.w[2])); }
inline int64_t recDst(const EdgeRec& r) { return static_cast<int64_t>(__builtin_bswap64(r.w[3])); }

// Sort by the records' order: bucketed by the key's first 4 bytes (the part and key type: ~100 values in a
// space), buckets scattered in parallel and each sorted on its own thread, so no serial merge pass over the
// whole array (r06: the commit of C2's 134 M rows spent 34.6 s in the export, most of it in serial passes)
template <class Cmp>
void bucketSort(std::vector<EdgeRec>& v, Cmp cmp) {
    const uint64_t n = v.size();
    const int T = hwThreads();
    if (n < (1u << 16) || T == 1) { std::sort(v.begin(), v.end(), cmp); return; }
    std::vector<uint32_t> keys;
    {
        std::vector<std::vector<uint32_t>> seen(T);
        bool many = false;
        std::vector<std::thread> ts;
        for (int t = 0; t < T; t++)
            ts.emplace_back([&, t] {
                auto& sv = seen[t];
                for (uint64_t i = n * t / T; i < n * (t + 1) / T && sv.size() <= 4096; i++) {
                    const uint32_t k = static_cast<uint32_t>(v[i].w[0] >> 32);
                    if (!sv.empty() && sv.back() == k) continue;
                    if (std::find(sv.begin(), sv.end(), k) == sv.end()) sv.push_back(k);
                }
            });
        for (auto& th : ts) th.join();
        for (auto& sv : seen) {
            many = many || sv.size() > 4096;
            keys.insert(keys.end(), sv.begin(), sv.end());
        }
        std::sort(keys.begin(), keys.end());
        keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
        if (many || keys.size() > 4096) { parallelSort(v.begin(), v.end(), cmp); return; }
    }
    const size_t B = keys.size();
    auto bucketOf = [&](const EdgeRec& r) {
        return static_cast<size_t>(std::lower_bound(keys.begin(), keys.end(), static_cast<uint32_t>(r.w[0] >> 32)) - keys.begin());
    };
    std::vector<uint64_t> cnt(static_cast<size_t>(T) * B, 0);
    {
        std::vector<std::thread> ts;
        for (int t = 0; t < T; t++)
            ts.emplace_back([&, t] {
                for (uint64_t i = n * t / T; i < n * (t + 1) / T; i++) cnt[static_cast<size_t>(t) * B + bucketOf(v[i])]++;
            });
        for (auto& th : ts) th.join();
    }
    std::vector<uint64_t> start(B + 1, 0), at(static_cast<size_t>(T) * B);
    for (size_t b = 0; b < B; b++) {
        uint64_t s = start[b];
        for (int t = 0; t < T; t++) { at[static_cast<size_t>(t) * B + b] = s; s += cnt[static_cast<size_t>(t) * B + b]; }
        start[b + 1] = s;
    }
    std::vector<EdgeRec> out(n);
    {
        std::vector<std::thread> ts;
        for (int t = 0; t < T; t++)
            ts.emplace_back([&, t] {
                for (uint64_t i = n * t / T; i < n * (t + 1) / T; i++) out[at[static_cast<size_t>(t) * B + bucketOf(v[i])]++] = v[i];
            });
        for (auto& th : ts) th.join();
    }
    std::atomic<size_t> next{0};
    {
        std::vector<std::thread> ts;
        for (int t = 0; t < T; t++)
            ts.emplace_back([&] {
                for (size_t b; (b = next.fetch_add(1)) < B;) std::sort(out.begin() + start[b], out.begin() + start[b + 1], cmp);
            });
        for (auto& th : ts) th.join();
    }
    v.swap(out);
}

}  // namespace

int32_t Space::slotOf(int32_t signedType) const {
    if (!host) return -1;
    for (size_t i = 0; i < host->slots.size(); i++) if (host->slots[i].etype == signedType) return static_cast<int32_t>(i);
    return -1;
}
int32_t Space::tagSlotOf(int32_t tagId) const {
    if (!host) return -1;
    for (size_t i = 0; i < host->tags.size(); i++) if (host->tags[i].tag == tagId) return static_cast<int32_t>(i);
    return -1;
}

Error exportSnapshot(Space& sp, int32_t rank, int32_t world, HostGraph& g) {
    (void)rank; (void)world;
    auto& st = sp.staged;
    uint64_t n = st.klen.size();
    // ---- classify rows (in parallel: per-thread counts, then every thread fills its range in row order)
    auto kindOf = [&](uint64_t i) -> int {                       // 1 edge, 2 vertex, 0 neither
        const uint8_t* k = st.keys.data() + st.koff[i];
        const uint32_t kl = st.klen[i];
        if (kl != 40 && kl != 24) return 0;
        if ((rd<uint32_t>(k) & 0xFF) != 1) return 0;          // NebulaKeyType::kData
        const bool isEdge = (rd<int32_t>(k + 12) & 0x40000000) != 0;
        return (kl == 40 && isEdge) ? 1 : (kl == 24 && !isEdge) ? 2 : 0;
    };
    const int CT = n < 65536 ? 1 : hwThreads();
    std::vector<uint64_t> ce(CT + 1, 0), cv(CT + 1, 0);
    {
        std::vector<std::thread> ts;
        for (int t = 0; t < CT; t++)
            ts.emplace_back([&, t] {
                for (uint64_t i = n * t / CT; i < n * (t + 1) / CT; i++) {
                    const int kd = kindOf(i);
                    ce[t + 1] += kd == 1;
                    cv[t + 1] += kd == 2;
                }
            });
        for (auto& th : ts) th.join();
    }
    for (int t = 0; t < CT; t++) { ce[t + 1] += ce[t]; cv[t + 1] += cv[t]; }
    std::vector<EdgeRec> edges(ce[CT]);
    std::vector<EdgeRec> verts(cv[CT]);
    {
        std::vector<std::thread> ts;
        for (int t = 0; t < CT; t++)
            ts.emplace_back([&, t] {
                uint64_t ei = ce[t], vi = cv[t];
                for (uint64_t i = n * t / CT; i < n * (t + 1) / CT; i++) {
                    const int kd = kindOf(i);
                    if (!kd) continue;
                    const uint8_t* k = st.keys.data() + st.koff[i];
                    EdgeRec r{};
                    if (kd == 1) {
                        for (int j = 0; j < 5; j++) r.w[j] = be64(k + 8 * j);
                        r.row = i;
                        edges[ei++] = r;
                    } else {
                        r.w[0] = be64(k); r.w[1] = be64(k + 8); r.w[2] = be64(k + 16); r.row = i;
                        verts[vi++] = r;
                    }
                }
            });
        for (auto& th : ts) th.join();
    }
    auto lessRec = [](const EdgeRec& a, const EdgeRec& b) {
        for (int j = 0; j < 5; j++) if (a.w[j] != b.w[j]) return a.w[j] < b.w[j];
        return a.row > b.row;      // duplicates: the later put first (RocksDB overwrite keeps it)
    };
    bool sorted = true;
    for (uint64_t i = 1; i < edges.size() && sorted; i++) if (lessRec(edges[i], edges[i - 1])) sorted = false;
    if (!sorted) bucketSort(edges, lessRec);
    parallelSort(verts.begin(), verts.end(), lessRec);
    auto keyOf = [&](const EdgeRec& r) { return st.keys.data() + st.koff[r.row]; };

    // ---- dedup: identical keys (keep the latest write) and latest version per (rank, dst): the first 32
    // key bytes (part, src, type, rank, dst) equal => an older version of one edge (the words, no key reads)
    {
        uint64_t m = 0;
        for (uint64_t i = 0; i < edges.size(); i++) {
            const EdgeRec& r = edges[i];
            if (m) {
                const EdgeRec& p = edges[m - 1];
                if (r.w[0] == p.w[0] && r.w[1] == p.w[1] && r.w[2] == p.w[2] && r.w[3] == p.w[3]) continue;
            }
            edges[m++] = r;
        }
        edges.resize(m);
    }

    // ---- vertex table: (part, vid) of every edge source and tag row
    std::vector<std::pair<int32_t, int64_t>> vt;
    vt.reserve(edges.size() / 4 + verts.size());
    for (auto& r : edges) {
        std::pair<int32_t, int64_t> pv{recPart(r), recSrc(r)};
        if (vt.empty() || vt.back() != pv) vt.push_back(pv);
    }
    for (auto& r : verts) vt.emplace_back(recPart(r), recSrc(r));
    parallelSort(vt.begin(), vt.end(), std::less<std::pair<int32_t, int64_t>>());
    vt.erase(std::unique(vt.begin(), vt.end()), vt.end());
    uint64_t V = vt.size();
    g.vpart.resize(V);
    g.vid.resize(V);
    for (uint64_t i = 0; i < V; i++) { g.vpart[i] = vt[i].first; g.vid[i] = vt[i].second; }
    auto rowOf = [&](int32_t part, int64_t vid) -> uint64_t {
        auto it = std::lower_bound(vt.begin(), vt.end(), std::make_pair(part, vid));
        return static_cast<uint64_t>(it - vt.begin());
    };

    // ---- slots (signed edge types present)
    std::map<int32_t, int32_t> slotIdx;
    {
        int32_t last = 0;
        bool any = false;
        for (auto& r : edges) {
            const int32_t t = recType(r);
            if (any && t == last) continue;
            last = t;
            any = true;
            const int32_t et = t > 0 ? (t & ~0x40000000) : t;   // NebulaKeyUtils::getEdgeType
            if (!slotIdx.count(et)) slotIdx[et] = 0;
        }
    }
    int32_t si = 0;
    for (auto& kv : slotIdx) kv.second = si++;
    g.slots.assign(slotIdx.size(), HostSlot());
    for (auto& kv : slotIdx) {
        auto& s = g.slots[kv.second];
        s.etype = kv.first;
        s.off.assign(V + 1, 0);
    }
    std::vector<uint64_t> eRow(edges.size());
    std::vector<int32_t> eSlot(edges.size());
    parallelFor(edges.size(), [&](uint64_t lo, uint64_t hi) {
        uint64_t cachedRow = 0;
        int32_t cp = INT32_MIN;
        int64_t cv = 0;
        int32_t lt = 0, ls = -1;
        for (uint64_t i = lo; i < hi; i++) {
            const int32_t part = recPart(edges[i]);
            const int64_t src = recSrc(edges[i]);
            if (part != cp || src != cv) { cachedRow = rowOf(part, src); cp = part; cv = src; }
            eRow[i] = cachedRow;
            const int32_t t = recType(edges[i]);
            if (ls < 0 || t != lt) { lt = t; ls = slotIdx.at(t > 0 ? (t & ~0x40000000) : t); }
            eSlot[i] = ls;
        }
    });
    for (uint64_t i = 0; i < edges.size(); i++) g.slots[eSlot[i]].off[eRow[i] + 1]++;
    for (auto& s : g.slots) {
        for (uint64_t v = 0; v < V; v++) s.off[v + 1] += s.off[v];
        uint64_t ne = s.off[V];
        s.dst.resize(ne);
        s.rank.resize(ne);
        s.dgid.assign(ne, kNoRow);
        s.eflags.assign(ne, 0);
    }
    // position of each edge in its slot: edges are sorted by (part, src, type, rank, dst) so
    // within one (row, slot) they are consecutive and already in key order
    std::vector<uint64_t> ePos(edges.size());
    {
        std::vector<uint64_t> cursor;
        for (uint64_t i = 0; i < edges.size(); i++) {
            auto& s = g.slots[eSlot[i]];
            if (i == 0 || eRow[i] != eRow[i - 1] || eSlot[i] != eSlot[i - 1]) ePos[i] = s.off[eRow[i]];
            else ePos[i] = ePos[i - 1] + 1;
        }
    }
    // ---- key fields + props
    std::map<int32_t, std::map<int64_t, VersionMap>> vmapsByType;
    for (auto& s : g.slots) {
        const SchemaSet* ss = sp.edge(std::abs(s.etype));
        if (!ss) continue;                                   // no schema: structure only
        if (!vmapsByType.count(std::abs(s.etype))) {
            auto err = buildVersionMaps(*ss, vmapsByType[std::abs(s.etype)]);
            if (err.code != NGX_OK) return err;
        }
        initColumns(s.cols, ss->latest(), s.dst.size());
    }
    std::vector<std::vector<std::vector<std::string>>> strs(g.slots.size());
    for (size_t k = 0; k < g.slots.size(); k++) {
        strs[k].resize(g.slots[k].cols.size());
        for (size_t c = 0; c < g.slots[k].cols.size(); c++) {
            if (g.slots[k].cols[c].type == T_STRING) strs[k][c].resize(g.slots[k].dst.size());
        }
    }
    parallelFor(edges.size(), [&](uint64_t lo, uint64_t hi) {
        for (uint64_t i = lo; i < hi; i++) {
            auto& s = g.slots[eSlot[i]];
            uint64_t p = ePos[i];
            s.rank[p] = recRank(edges[i]);
            s.dst[p] = recDst(edges[i]);
            auto vm = vmapsByType.find(std::abs(s.etype));
            uint64_t row = edges[i].row;
            const uint8_t* val = st.vals.data() + st.voff[row];
            uint64_t vlen = st.voff[row + 1] - st.voff[row];
            if (vm == vmapsByType.end()) {
                s.eflags[p] = vlen == 0 ? EF_EMPTY_VALUE : EF_BAD_ROW;
                continue;
            }
            s.eflags[p] = decodeInto(val, vlen, vm->second, s.cols, p, strs[eSlot[i]]);
        }
    });
    for (size_t k = 0; k < g.slots.size(); k++) {
        auto& s = g.slots[k];
        s.anyFlags = std::any_of(s.eflags.begin(), s.eflags.end(), [](uint8_t f) { return f != 0; });
        if (!s.anyFlags) { s.eflags.clear(); s.eflags.shrink_to_fit(); }
        packStrings(s.cols, strs[k]);
        g.edges += s.dst.size();
    }

    // ---- tags: first row under vertexPrefix(part, vid, tag) is the latest version
    std::map<int32_t, int32_t> tagIdx;
    for (auto& kv : sp.tags) { tagIdx[kv.first] = static_cast<int32_t>(g.tags.size()); g.tags.emplace_back(); g.tags.back().tag = kv.first; }
    std::map<int32_t, std::map<int64_t, VersionMap>> tvmaps;
    for (auto& t : g.tags) {
        const SchemaSet& ss = sp.tags.at(t.tag);
        auto err = buildVersionMaps(ss, tvmaps[t.tag]);
        if (err.code != NGX_OK) return err;
        initColumns(t.cols, ss.latest(), V);
        t.present.assign(V, 0);
    }
    std::vector<std::vector<std::vector<std::string>>> tstrs(g.tags.size());
    for (size_t k = 0; k < g.tags.size(); k++) {
        tstrs[k].resize(g.tags[k].cols.size());
        for (size_t c = 0; c < g.tags[k].cols.size(); c++) if (g.tags[k].cols[c].type == T_STRING) tstrs[k][c].resize(V);
    }
    for (uint64_t i = 0; i < verts.size(); i++) {
        const uint8_t* k = keyOf(verts[i]);
        if (i > 0 && std::memcmp(k, keyOf(verts[i - 1]), 16) == 0) continue;   // older version
        int32_t tag = rd<int32_t>(k + 12);
        auto ti = tagIdx.find(tag);
        if (ti == tagIdx.end()) continue;
        auto& t = g.tags[ti->second];
        uint64_t v = rowOf(rd<int32_t>(k) >> 8, rd<int64_t>(k + 4));
        uint64_t row = verts[i].row;
        const uint8_t* val = st.vals.data() + st.voff[row];
        uint64_t vlen = st.voff[row + 1] - st.voff[row];
        uint8_t f = decodeInto(val, vlen, tvmaps[tag], t.cols, v, tstrs[ti->second]);
        // collectVertexProps: an unreadable tag row is ERR_CORRUPT_DATA; treated as absent here
        t.present[v] = (f == 0) ? 1 : 0;
    }
    for (size_t k = 0; k < g.tags.size(); k++) packStrings(g.tags[k].cols, tstrs[k]);
    return Error{NGX_OK, ""};
}

// Columnar bulk load (ngx_load_csr): the caller's CSR becomes the shard snapshot exportSnapshot would
// build from the same edges' KV rows. Everything the exporter guarantees is checked instead of built:
// the vertex table sorted by (part, vid) with part = ID_HASH(vid) owned by this shard, CSR offsets,
// every row's adjacency strictly in RocksDB key order (rank LE bytes, then dst LE bytes: no two versions
// of one edge), one slot per signed type with a schema whose latest version has no STRING field.
Error loadCsrShard(const Space& sp, int32_t rank, int32_t world, const ngx_csr_shard& in, HostGraph& g) {
    const uint64_t V = in.nvertices;
    if ((V && (!in.vpart || !in.vid)) || in.nslots < 0 || (in.nslots && !in.slots))
        return Error{NGX_E_BAD_ARGUMENT, "csr: missing arrays"};
    std::atomic<bool> bad{false};
    parallelFor(V, [&](uint64_t lo, uint64_t hi) {
        for (uint64_t i = lo; i < hi && !bad; i++) {
            const int32_t p = in.vpart[i];
            if (sp.numParts > 0 && (p != idHash(in.vid[i], sp.numParts) || (world > 1 && p % world != rank))) bad = true;
            if (i && (in.vpart[i - 1] > p || (in.vpart[i - 1] == p && in.vid[i - 1] >= in.vid[i]))) bad = true;
        }
    });
    if (bad) return Error{NGX_E_BAD_ARGUMENT, "csr: vertex table not sorted by (part, vid), duplicated, or of parts this shard does not own"};
    g.vpart.assign(in.vpart, in.vpart + V);
    g.vid.assign(in.vid, in.vid + V);
    std::vector<const ngx_csr_slot*> order;
    for (int32_t k = 0; k < in.nslots; k++) order.push_back(&in.slots[k]);
    std::sort(order.begin(), order.end(), [](const ngx_csr_slot* a, const ngx_csr_slot* b) { return a->etype < b->etype; });
    for (size_t k = 0; k < order.size(); k++) {
        const ngx_csr_slot& cs = *order[k];
        if (cs.etype == 0 || (k && order[k - 1]->etype == cs.etype)) return Error{NGX_E_BAD_ARGUMENT, "csr: slot types must be distinct and nonzero"};
        const SchemaSet* ss = sp.edge(std::abs(cs.etype));
        if (!ss) return Error{NGX_E_EDGE_NOT_FOUND, "csr: no schema for edge type " + std::to_string(cs.etype)};
        const SchemaDef& latest = ss->latest();
        if (cs.ncols != static_cast<int32_t>(latest.fields.size()) || (cs.ncols && !cs.cols))
            return Error{NGX_E_BAD_ARGUMENT, "csr: columns must be the latest schema's fields"};
        for (auto& f : latest.fields)
            if (f.type == T_STRING) return Error{NGX_E_UNSUPPORTED, "csr: STRING columns are loaded from KV rows"};
        if (!cs.off || cs.off[0] != 0) return Error{NGX_E_BAD_ARGUMENT, "csr: offsets must start at 0"};
        const uint64_t ne = cs.off[V];
        if (ne && !cs.dst) return Error{NGX_E_BAD_ARGUMENT, "csr: missing dst"};
        parallelFor(V, [&](uint64_t lo, uint64_t hi) {
            for (uint64_t r = lo; r < hi && !bad; r++) {
                if (cs.off[r] > cs.off[r + 1]) { bad = true; break; }
                for (uint64_t e = cs.off[r] + 1; e < cs.off[r + 1]; e++) {
                    const uint64_t ra = cs.rank ? __builtin_bswap64(static_cast<uint64_t>(cs.rank[e - 1])) : 0;
                    const uint64_t rb = cs.rank ? __builtin_bswap64(static_cast<uint64_t>(cs.rank[e])) : 0;
                    const uint64_t da = __builtin_bswap64(static_cast<uint64_t>(cs.dst[e - 1]));
                    const uint64_t db = __builtin_bswap64(static_cast<uint64_t>(cs.dst[e]));
                    if (ra > rb || (ra == rb && da >= db)) { bad = true; break; }
                }
            }
        });
        if (bad) return Error{NGX_E_BAD_ARGUMENT, "csr: offsets not monotone or a row's edges not in key order (rank, dst LE bytes)"};
        g.slots.emplace_back();
        HostSlot& hs = g.slots.back();
        hs.etype = cs.etype;
        hs.off.assign(cs.off, cs.off + V + 1);
        hs.dst.assign(cs.dst, cs.dst + ne);
        if (cs.rank) hs.rank.assign(cs.rank, cs.rank + ne);
        else hs.rank.assign(ne, 0);
        hs.dgid.assign(ne, kNoRow);
        hs.cols.resize(latest.fields.size());
        for (size_t c = 0; c < hs.cols.size(); c++) {
            HostColumn& col = hs.cols[c];
            col.type = latest.fields[c].type;
            const int64_t* x = cs.cols[c];
            if (ne && !x) return Error{NGX_E_BAD_ARGUMENT, "csr: missing column " + latest.fields[c].name};
            switch (col.type) {
                case T_INT: case T_TIMESTAMP: case T_VID: col.i64.assign(x, x + ne); break;
                case T_FLOAT: case T_DOUBLE:
                    col.f64.resize(ne);
                    if (ne) std::memcpy(col.f64.data(), x, ne * 8);
                    break;
                case T_BOOL:
                    col.b.resize(ne);
                    for (uint64_t e = 0; e < ne; e++) col.b[e] = x[e] != 0;
                    break;
                default: break;
            }
        }
        g.edges += ne;
    }
    // tags of the space: no rows (ngx_load_csr carries edges only)
    for (auto& kv : sp.tags) {
        g.tags.emplace_back();
        HostTag& t = g.tags.back();
        t.tag = kv.first;
        initColumns(t.cols, kv.second.latest(), V);
        t.present.assign(V, 0);
        std::vector<std::vector<std::string>> none(t.cols.size());
        for (size_t c = 0; c < t.cols.size(); c++) if (t.cols[c].type == T_STRING) none[c].resize(V);
        packStrings(t.cols, none);
    }
    return Error{NGX_OK, ""};
}

// Destination rows: the global row of (ID_HASH(dst), dst) in its owner's vertex table. One open-address
// hash of every shard's rows (only (part, vid) with part = ID_HASH(vid) can be found, as a lookup of
// (ID_HASH(dst), dst) in the owner's table would), probed for the edges in blocks with the slots'
// cache lines prefetched: a per-edge binary search over a 3 M-row table cost ~1 us of cache misses
// (C3: 254 M edges per shard, 60 s on 2 threads), a prefetched probe ~30 ns.
void resolveDstRows(const Space& sp, HostGraph& g,
                    const std::vector<std::vector<std::pair<int32_t, int64_t>>>& shardTables, int32_t world) {
    if (sp.numParts <= 0) return;                    // test-only layouts: no ID_HASH routing
    g.shardBase.assign(world + 1, 0);
    for (int32_t w = 0; w < world; w++) g.shardBase[w + 1] = g.shardBase[w] + shardTables[w].size();
    g.vglobal = g.shardBase[world];
    uint64_t cap = 16;
    while (cap < 2 * g.vglobal) cap <<= 1;
    const uint64_t mask = cap - 1;
    std::vector<int64_t> key(cap);
    std::vector<uint32_t> row(cap, kNoRow);
    auto slotOf = [mask](int64_t v) {
        uint64_t z = static_cast<uint64_t>(v) + 0x9E3779B97F4A7C15ULL;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        return (z ^ (z >> 31)) & mask;
    };
    for (int32_t w = 0; w < world; w++) {
        const auto& tab = shardTables[w];
        for (uint64_t i = 0; i < tab.size(); i++) {
            if (tab[i].first != idHash(tab[i].second, sp.numParts)) continue;
            uint64_t h = slotOf(tab[i].second);
            while (row[h] != kNoRow && key[h] != tab[i].second) h = (h + 1) & mask;
            if (row[h] != kNoRow) continue;          // (part, vid) appears once per table: cannot happen
            key[h] = tab[i].second;
            row[h] = static_cast<uint32_t>(g.shardBase[w] + i);
        }
    }
    for (auto& s : g.slots) {
        parallelFor(s.dst.size(), [&](uint64_t lo, uint64_t hi) {
            constexpr uint64_t kBlock = 32;
            uint64_t hs[kBlock];
            for (uint64_t b = lo; b < hi; b += kBlock) {
                const uint64_t n = std::min<uint64_t>(kBlock, hi - b);
                for (uint64_t k = 0; k < n; k++) {
                    hs[k] = slotOf(s.dst[b + k]);
                    __builtin_prefetch(&key[hs[k]]);
                    __builtin_prefetch(&row[hs[k]]);
                }
                for (uint64_t k = 0; k < n; k++) {
                    const int64_t d = s.dst[b + k];
                    uint64_t h = hs[k];
                    while (row[h] != kNoRow && key[h] != d) h = (h + 1) & mask;
                    s.dgid[b + k] = row[h];           // kNoRow: the destination has no edges or tags here
                }
            }
        });
    }
}

}  // namespace ngx
