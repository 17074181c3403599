// Device snapshot files: one committed shard (HostGraph: vertex table, per-slot CSR + dst rows +
// columns, tag columns) written as a single versioned file, so a storaged restart loads its shard
// without re-reading and re-decoding the part's KV rows. It plays the role of the reference's
// RocksDB checkpoint (RocksEngine::createCheckpoint, src/kvstore/RocksEngine.cpp:433-480: a named
// snapshot of the space's data under checkpoints/<name>) for the device-side copy of the data.
//
// Layout (little endian):
//   header   magic "NGXSNAP\0", u32 format version, u32 reserved, i32 space, i32 num_parts, i32 rank,
//            i32 world, u64 schema digest, char tag[64], u64 payload bytes, u64 payload hash,
//            u64 commit digest (HostGraph::commitDigest: all shards' vertex tables; ngx_open_snapshot
//            at world > 1 requires every rank's to agree)
//   payload  the HostGraph fields in a fixed order; every array as [u64 count][count * sizeof(T)]
// The payload hash (64-bit, 8 bytes a step) is checked before anything is replaced; the schema
// digest covers every tag / edge schema version (names, types, TTL) registered for the space, so
// rows are never read back against other schemas.
#include <cstdio>
#include <memory>
#include <type_traits>

#include "ngx_internal.h"

namespace ngx {

namespace {

constexpr char kMagic[8] = {'N', 'G', 'X', 'S', 'N', 'A', 'P', '\0'};
constexpr uint32_t kFormat = 2;

struct Header {
    char magic[8];
    uint32_t format;
    uint32_t reserved;
    int32_t space, numParts, rank, world;
    uint64_t schemaDigest;
    char tag[64];
    uint64_t payloadBytes;
    uint64_t payloadHash;
    uint64_t commitDigest;
};
static_assert(sizeof(Header) == 128, "snapshot header layout");

// running hash over a byte stream, 8 bytes a step (tail bytes zero-padded per call boundary-free)
struct StreamHash {
    uint64_t h = 0x9E3779B97F4A7C15ULL, n = 0;
    uint8_t pend[8];
    int np = 0;
    void word(uint64_t w) {
        h ^= w;
        h *= 0xBF58476D1CE4E5B9ULL;
        h ^= h >> 31;
    }
    void add(const void* p, uint64_t len) {
        const uint8_t* b = static_cast<const uint8_t*>(p);
        n += len;
        while (len && np) { pend[np++] = *b++; len--; if (np == 8) { uint64_t w; std::memcpy(&w, pend, 8); word(w); np = 0; } }
        for (; len >= 8; b += 8, len -= 8) { uint64_t w; std::memcpy(&w, b, 8); word(w); }
        while (len--) pend[np++] = *b++;
    }
    uint64_t done() {
        uint64_t w = 0;
        std::memcpy(&w, pend, np);
        word(w ^ (n << 8));
        return h;
    }
};

class Out {
public:
    explicit Out(FILE* f) : f_(f) {}
    bool ok() const { return ok_; }
    uint64_t bytes() const { return hash_.n; }
    uint64_t hash() { return hash_.done(); }
    void raw(const void* p, uint64_t n) {
        if (!ok_ || n == 0) return;
        hash_.add(p, n);
        ok_ = std::fwrite(p, 1, n, f_) == n;
    }
    template <typename T>
    void pod(T v) { static_assert(std::is_trivially_copyable<T>::value, "pod"); raw(&v, sizeof(T)); }
    template <typename T>
    void vec(const std::vector<T>& v) { pod<uint64_t>(v.size()); raw(v.data(), v.size() * sizeof(T)); }
    void str(const std::string& s) { pod<uint64_t>(s.size()); raw(s.data(), s.size()); }

private:
    FILE* f_;
    bool ok_ = true;
    StreamHash hash_;
};

class In {
public:
    In(FILE* f, uint64_t limit) : f_(f), left_(limit) {}
    bool ok() const { return ok_; }
    uint64_t hash() { return hash_.done(); }
    uint64_t left() const { return left_; }
    void raw(void* p, uint64_t n) {
        if (!ok_ || n == 0) return;
        if (n > left_) { ok_ = false; return; }
        ok_ = std::fread(p, 1, n, f_) == n;
        if (ok_) { hash_.add(p, n); left_ -= n; }
    }
    template <typename T>
    T pod() { T v{}; raw(&v, sizeof(T)); return v; }
    template <typename T>
    void vec(std::vector<T>& v) {
        uint64_t n = pod<uint64_t>();
        if (!ok_ || n > left_ / (sizeof(T) ? sizeof(T) : 1)) { ok_ = false; return; }
        v.resize(n);
        raw(v.data(), n * sizeof(T));
    }
    void str(std::string& s) {
        uint64_t n = pod<uint64_t>();
        if (!ok_ || n > left_) { ok_ = false; return; }
        s.resize(n);
        raw(&s[0], n);
    }

private:
    FILE* f_;
    uint64_t left_;
    bool ok_ = true;
    StreamHash hash_;
};

void putColumn(Out& o, const HostColumn& c) {
    o.pod<int32_t>(c.type);
    o.pod<uint8_t>(c.allValid ? 1 : 0);
    o.vec(c.i64);
    o.vec(c.f64);
    o.vec(c.b);
    o.vec(c.soff);
    o.str(c.sbytes);
    o.vec(c.valid);
}

void getColumn(In& in, HostColumn& c) {
    c.type = in.pod<int32_t>();
    c.allValid = in.pod<uint8_t>() != 0;
    in.vec(c.i64);
    in.vec(c.f64);
    in.vec(c.b);
    in.vec(c.soff);
    in.str(c.sbytes);
    in.vec(c.valid);
    c.width = 8;                        // chosen again at upload
}

void putGraph(Out& o, const HostGraph& g) {
    o.vec(g.vpart);
    o.vec(g.vid);
    o.pod<uint64_t>(g.gbase);
    o.pod<uint64_t>(g.vglobal);
    o.vec(g.shardBase);
    o.pod<uint64_t>(g.edges);
    o.pod<uint64_t>(g.slots.size());
    for (const HostSlot& s : g.slots) {
        o.pod<int32_t>(s.etype);
        o.vec(s.off);
        o.vec(s.dst);
        o.vec(s.rank);
        o.vec(s.dgid);
        o.vec(s.eflags);
        o.pod<uint8_t>(s.anyFlags ? 1 : 0);
        o.pod<uint64_t>(s.cols.size());
        for (const HostColumn& c : s.cols) putColumn(o, c);
    }
    o.pod<uint64_t>(g.tags.size());
    for (const HostTag& t : g.tags) {
        o.pod<int32_t>(t.tag);
        o.vec(t.present);
        o.pod<uint64_t>(t.cols.size());
        for (const HostColumn& c : t.cols) putColumn(o, c);
    }
}

bool getGraph(In& in, HostGraph& g) {
    in.vec(g.vpart);
    in.vec(g.vid);
    g.gbase = in.pod<uint64_t>();
    g.vglobal = in.pod<uint64_t>();
    in.vec(g.shardBase);
    g.edges = in.pod<uint64_t>();
    const uint64_t ns = in.pod<uint64_t>();
    if (!in.ok() || ns > 4096) return false;
    g.slots.resize(ns);
    for (HostSlot& s : g.slots) {
        s.etype = in.pod<int32_t>();
        in.vec(s.off);
        in.vec(s.dst);
        in.vec(s.rank);
        in.vec(s.dgid);
        in.vec(s.eflags);
        s.anyFlags = in.pod<uint8_t>() != 0;
        const uint64_t nc = in.pod<uint64_t>();
        if (!in.ok() || nc > 65536) return false;
        s.cols.resize(nc);
        for (HostColumn& c : s.cols) getColumn(in, c);
    }
    const uint64_t nt = in.pod<uint64_t>();
    if (!in.ok() || nt > 65536) return false;
    g.tags.resize(nt);
    for (HostTag& t : g.tags) {
        t.tag = in.pod<int32_t>();
        in.vec(t.present);
        const uint64_t nc = in.pod<uint64_t>();
        if (!in.ok() || nc > 65536) return false;
        t.cols.resize(nc);
        for (HostColumn& c : t.cols) getColumn(in, c);
    }
    return in.ok();
}

// a column of n values: its arrays sized for n, string offsets 0-based and non-decreasing up to the bytes
bool columnOk(const HostColumn& c, uint64_t n) {
    if (!c.allValid && c.valid.size() != n) return false;
    switch (c.type) {
        case T_BOOL: return c.b.size() == n;
        case T_FLOAT: case T_DOUBLE: return c.f64.size() == n;
        case T_STRING: {
            if (c.soff.size() != n + 1 || c.soff[0] != 0 || c.soff[n] != c.sbytes.size()) return false;
            for (uint64_t i = 0; i < n; i++) if (c.soff[i] > c.soff[i + 1]) return false;
            return true;
        }
        default: return c.i64.size() == n;
    }
}

// structural checks of a decoded graph against itself and the space (a bad file must not reach the
// kernels): array sizes, monotonic offsets, parts in range, the vertex table sorted by (part, vid) (the
// seed lookup's binary search and index), destination rows inside the global table, shard bases
bool consistent(const HostGraph& g, int32_t numParts, int32_t rank, int32_t world) {
    const uint64_t V = g.vid.size();
    if (g.vpart.size() != V || g.vglobal < V || g.gbase + V > g.vglobal) return false;
    for (uint64_t r = 0; r < V; r++) {
        if (numParts > 0 && (g.vpart[r] < 1 || g.vpart[r] > numParts)) return false;
        if (r && !(g.vpart[r - 1] < g.vpart[r] || (g.vpart[r - 1] == g.vpart[r] && g.vid[r - 1] < g.vid[r]))) return false;
    }
    if (!g.shardBase.empty()) {
        if (g.shardBase.size() != static_cast<size_t>(world) + 1 || g.shardBase[0] != 0) return false;
        for (int32_t w = 0; w < world; w++) if (g.shardBase[w] > g.shardBase[w + 1]) return false;
        if (g.gbase != g.shardBase[rank] || g.shardBase[rank + 1] - g.shardBase[rank] != V ||
            g.vglobal != g.shardBase[world]) return false;
    }
    for (const HostSlot& s : g.slots) {
        if (s.off.size() != V + 1 || s.off[0] != 0) return false;
        const uint64_t E = s.off[V];
        for (uint64_t r = 0; r < V; r++) if (s.off[r] > s.off[r + 1]) return false;
        if (s.dst.size() != E || s.rank.size() != E || s.dgid.size() != E) return false;
        if (s.anyFlags ? s.eflags.size() != E : !s.eflags.empty() && s.eflags.size() != E) return false;
        for (uint32_t x : s.dgid) if (x != kNoRow && x >= g.vglobal) return false;
        for (const HostColumn& c : s.cols) if (!columnOk(c, E)) return false;
    }
    for (const HostTag& t : g.tags) {
        if (t.present.size() != V) return false;
        for (const HostColumn& c : t.cols) if (!columnOk(c, V)) return false;
    }
    return true;
}

}  // namespace

uint64_t schemaDigest(const Space& sp) {
    StreamHash h;
    auto s = [&](const std::string& x) { uint64_t n = x.size(); h.add(&n, 8); h.add(x.data(), n); };
    auto sets = [&](const std::map<int32_t, SchemaSet>& m) {
        uint64_t n = m.size();
        h.add(&n, 8);
        for (auto& kv : m) {
            h.add(&kv.first, 4);
            s(kv.second.name);
            for (auto& v : kv.second.versions) {
                h.add(&v.first, 8);
                for (auto& f : v.second.fields) { s(f.name); h.add(&f.type, 4); }
                s(v.second.ttlCol);
                h.add(&v.second.ttlDur, 8);
            }
        }
    };
    sets(sp.tags);
    sets(sp.edges);
    h.add(&sp.numParts, 4);
    return h.done();
}

uint64_t tablesDigest(const std::vector<std::vector<std::pair<int32_t, int64_t>>>& tables,
                      const std::vector<uint64_t>& nonces) {
    StreamHash h;
    for (auto& t : tables) {
        uint64_t n = t.size();
        h.add(&n, 8);
        for (auto& pv : t) { h.add(&pv.first, 4); h.add(&pv.second, 8); }
    }
    for (uint64_t x : nonces) h.add(&x, 8);
    return h.done();
}

Error writeSnapshotFile(const Space& sp, const HostGraph& g, int32_t rank, int32_t world, const std::string& path,
                        const std::string& tag) {
    if (tag.size() > 63) return Error{NGX_E_BAD_ARGUMENT, "snapshot tag longer than 63 bytes"};
    const std::string tmp = path + ".tmp";
    std::unique_ptr<FILE, int (*)(FILE*)> f(std::fopen(tmp.c_str(), "wb"), std::fclose);
    if (!f) return Error{NGX_E_SNAPSHOT, "cannot create " + tmp};
    std::vector<char> buf(8 << 20);
    std::setvbuf(f.get(), buf.data(), _IOFBF, buf.size());
    Header h{};
    std::memcpy(h.magic, kMagic, 8);
    h.format = kFormat;
    h.space = sp.id;
    h.numParts = sp.numParts;
    h.rank = rank;
    h.world = world;
    h.schemaDigest = schemaDigest(sp);
    h.commitDigest = g.commitDigest;
    std::memcpy(h.tag, tag.data(), tag.size());
    bool ok = std::fwrite(&h, sizeof(h), 1, f.get()) == 1;
    Out o(f.get());
    putGraph(o, g);
    ok = ok && o.ok();
    h.payloadBytes = o.bytes();
    h.payloadHash = o.hash();
    ok = ok && std::fseek(f.get(), 0, SEEK_SET) == 0 && std::fwrite(&h, sizeof(h), 1, f.get()) == 1;
    ok = std::fflush(f.get()) == 0 && ok;
    f.reset();
    if (!ok || std::rename(tmp.c_str(), path.c_str()) != 0) {
        std::remove(tmp.c_str());
        return Error{NGX_E_SNAPSHOT, "cannot write " + path};
    }
    return Error{NGX_OK, ""};
}

Error readSnapshotFile(const Space& sp, const std::string& path, int32_t rank, int32_t world, HostGraph& out,
                       std::string& tag) {
    std::unique_ptr<FILE, int (*)(FILE*)> f(std::fopen(path.c_str(), "rb"), std::fclose);
    if (!f) return Error{NGX_E_SNAPSHOT, "cannot open " + path};
    std::vector<char> buf(8 << 20);
    std::setvbuf(f.get(), buf.data(), _IOFBF, buf.size());
    Header h{};
    if (std::fread(&h, sizeof(h), 1, f.get()) != 1 || std::memcmp(h.magic, kMagic, 8) != 0)
        return Error{NGX_E_SNAPSHOT, path + ": not a device snapshot"};
    if (h.format != kFormat) return Error{NGX_E_SNAPSHOT, path + ": snapshot format " + std::to_string(h.format)};
    if (h.space != sp.id || h.numParts != sp.numParts) return Error{NGX_E_SNAPSHOT, path + ": snapshot of another space"};
    if (h.rank != rank || h.world != world) return Error{NGX_E_SNAPSHOT, path + ": snapshot of another shard"};
    if (h.schemaDigest != schemaDigest(sp)) return Error{NGX_E_SNAPSHOT, path + ": schemas differ from the snapshot's"};
    In in(f.get(), h.payloadBytes);
    HostGraph g;
    const bool parsed = getGraph(in, g);
    if (!parsed || !in.ok() || in.left() != 0 || in.hash() != h.payloadHash)
        return Error{NGX_E_SNAPSHOT, path + ": snapshot payload corrupt"};
    if (!consistent(g, sp.numParts, rank, world)) return Error{NGX_E_SNAPSHOT, path + ": snapshot arrays inconsistent"};
    g.commitDigest = h.commitDigest;
    h.tag[63] = '\0';
    tag = h.tag;
    out = std::move(g);
    return Error{NGX_OK, ""};
}

}  // namespace ngx
