// Synthetic graph generators emitting reference-format KV rows (NebulaKeyUtils keys + RowWriter
// values), the form in which a storaged part would be exported (src/common/utils/NebulaKeyUtils.cpp:
// 12-45, src/dataman/RowWriter.cpp:39-263). Used by bench.py and the parity tests for the BASELINE
// configs: RMAT (C2/C3), power-law with supernodes (C4) and an LDBC-SNB-like multi-type schema (C5).
//
// Every random draw is a counter-based hash of (seed, stream, index), so the generated graph is a
// pure function of the parameters, independent of thread count and of (rank, world) filtering:
// with world > 1 only the rows of parts p with p % world == rank are materialised.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

inline uint64_t mix64(uint64_t x) {             // splitmix64 finaliser
    x += 0x9e3779b97f4a7c15ULL;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
    return x ^ (x >> 31);
}
inline uint64_t draw(uint64_t seed, uint64_t stream, uint64_t i) {
    return mix64(seed * 0x100000001b3ULL ^ mix64(stream * 0x9e3779b97f4a7c15ULL + i));
}

// RowWriter with a schema of ints / doubles / strings, schema version 0 and < 16 fields:
// header byte (offset width - 1) then the fields (RowWriter.cpp:49-75, RowWriter.inl).
struct Row {
    std::string cord;
    void i64(int64_t v) {
        uint64_t u = static_cast<uint64_t>(v);
        while (u >= 0x80) { cord.push_back(static_cast<char>((u & 0x7F) | 0x80)); u >>= 7; }
        cord.push_back(static_cast<char>(u));
    }
    void f64(double d) { cord.append(reinterpret_cast<const char*>(&d), 8); }
    void str(const std::string& s) { i64(static_cast<int64_t>(s.size())); cord += s; }
    void encodeTo(std::vector<uint8_t>& out) const {
        uint64_t n = cord.size();
        int ob = 0;
        do { ob++; n >>= 8; } while (n);
        out.push_back(static_cast<uint8_t>(ob - 1));
        out.insert(out.end(), cord.begin(), cord.end());
    }
};

struct Sink {                                    // one thread's output
    std::vector<uint8_t> keys, vals;
    std::vector<uint64_t> klen, vlen;            // per-row lengths; offsets are built in finish()
    uint64_t n = 0;
    void edge(int32_t part, int64_t src, int32_t etype, int64_t rank, int64_t dst, const Row& r) {
        uint8_t k[40];
        int32_t item = (part << 8) | 1;
        uint32_t et = static_cast<uint32_t>(etype) | 0x40000000u;
        int64_t ver = 0;
        std::memcpy(k, &item, 4); std::memcpy(k + 4, &src, 8); std::memcpy(k + 12, &et, 4);
        std::memcpy(k + 16, &rank, 8); std::memcpy(k + 24, &dst, 8); std::memcpy(k + 32, &ver, 8);
        keys.insert(keys.end(), k, k + 40);
        klen.push_back(40);
        size_t before = vals.size();
        r.encodeTo(vals);
        vlen.push_back(vals.size() - before);
        n++;
    }
    void vertex(int32_t part, int64_t vid, int32_t tag, const Row& r) {
        uint8_t k[24];
        int32_t item = (part << 8) | 1;
        int64_t ver = 0;
        std::memcpy(k, &item, 4); std::memcpy(k + 4, &vid, 8); std::memcpy(k + 12, &tag, 4);
        std::memcpy(k + 16, &ver, 8);
        keys.insert(keys.end(), k, k + 24);
        klen.push_back(24);
        size_t before = vals.size();
        r.encodeTo(vals);
        vlen.push_back(vals.size() - before);
        n++;
    }
};

struct Gen {
    int32_t numParts, rank, world;
    int threads;
    std::vector<Sink> sinks;
    int32_t partOf(int64_t vid) const { return static_cast<int32_t>(static_cast<uint64_t>(vid) % numParts + 1); }
    bool owned(int64_t vid) const { return world <= 1 || partOf(vid) % world == rank; }
    template <typename F>
    void run(uint64_t n, F&& f) {                // f(sink, i) for i in [0, n), contiguous chunks per thread
        sinks.assign(threads, Sink());
        std::vector<std::thread> th;
        for (int t = 0; t < threads; t++) {
            th.emplace_back([&, t] {
                uint64_t lo = n * t / threads, hi = n * (t + 1) / threads;
                for (uint64_t i = lo; i < hi; i++) f(sinks[t], i);
            });
        }
        for (auto& x : th) x.join();
        flush();
    }
    std::vector<Sink> done;
    void flush() { for (auto& s : sinks) done.push_back(std::move(s)); sinks.clear(); }
};

}  // namespace

extern "C" {

typedef struct {
    uint64_t n;
    uint8_t* keys;
    uint64_t* key_off;
    uint8_t* vals;
    uint64_t* val_off;
} ngd_rows;

void ngd_free(ngd_rows* r) {
    if (!r) return;
    std::free(r->keys); std::free(r->key_off); std::free(r->vals); std::free(r->val_off);
    std::memset(r, 0, sizeof(*r));
}

}  // extern "C"

namespace {

// concatenate the thread sinks into one ngd_rows (key offsets from the per-row key lengths)
void finish(Gen& g, ngd_rows* out) {
    uint64_t n = 0, kb = 0, vb = 0;
    for (auto& s : g.done) { n += s.n; kb += s.keys.size(); vb += s.vals.size(); }
    out->n = n;
    out->keys = static_cast<uint8_t*>(std::malloc(std::max<uint64_t>(kb, 1)));
    out->vals = static_cast<uint8_t*>(std::malloc(std::max<uint64_t>(vb, 1)));
    out->key_off = static_cast<uint64_t*>(std::malloc((n + 1) * 8));
    out->val_off = static_cast<uint64_t*>(std::malloc((n + 1) * 8));
    out->key_off[0] = out->val_off[0] = 0;
    uint64_t ki = 0, vi = 0, r = 0;
    for (auto& s : g.done) {
        std::memcpy(out->keys + ki, s.keys.data(), s.keys.size());
        std::memcpy(out->vals + vi, s.vals.data(), s.vals.size());
        for (uint64_t j = 0; j < s.n; j++) {
            r++;
            out->key_off[r] = out->key_off[r - 1] + s.klen[j];
            out->val_off[r] = out->val_off[r - 1] + s.vlen[j];
        }
        ki += s.keys.size();
        vi += s.vals.size();
        std::vector<uint8_t>().swap(s.keys);
        std::vector<uint8_t>().swap(s.vals);
    }
    g.done.clear();
}

// RMAT quadrant walk with 16-bit probabilities, four levels per 64-bit draw
inline void rmatEdge(uint64_t seed, uint64_t i, int scale, uint32_t a, uint32_t ab, uint32_t abc, uint64_t& s,
                     uint64_t& d) {
    s = 0; d = 0;
    uint64_t bits = 0;
    for (int l = 0; l < scale; l++) {
        if ((l & 3) == 0) bits = draw(seed, 1 + l / 4, i);
        uint32_t r = static_cast<uint32_t>(bits & 0xFFFF);
        bits >>= 16;
        // quadrants [0, a) (0, 0), [a, ab) (0, 1), [ab, abc) (1, 0), [abc, 2^16) (1, 1), without branches
        // (a branch per level on random bits mispredicts half the time: 5x slower)
        const uint64_t sb = r >= ab;
        const uint64_t db = static_cast<uint64_t>(r >= a) ^ static_cast<uint64_t>(r >= ab) ^ static_cast<uint64_t>(r >= abc);
        s = (s << 1) | sb;
        d = (d << 1) | db;
    }
}

// bijective scramble of [0, 2^scale): hubs are spread over the id space (Graph500 permutes ids)
inline uint64_t scramble(uint64_t v, int scale, uint64_t seed) {
    uint64_t mask = (scale >= 64) ? ~0ULL : ((1ULL << scale) - 1);
    uint64_t k1 = (mix64(seed ^ 0xa5a5) | 1) & mask, k2 = mix64(seed ^ 0x5a5a) & mask;
    for (int r = 0; r < 2; r++) {
        v = (v * k1) & mask;
        v ^= (v >> (scale / 2 + 1));
        v = (v + k2) & mask;
    }
    return v;
}

}  // namespace

extern "C" {

// RMAT (Graph500 A/B/C/D) with `ef * 2^scale` edges of one type `etype` carrying two INT props
// p0 = h(src,dst) % 100 and p1 = h'(src,dst) as a full-range int64 (deterministic per (src,dst), so duplicate
// generated edges write byte-identical rows). rank 0. with_in also writes the in-edge rows
// (dst, -etype, rank, src), as InsertEdgeExecutor does. with_tag writes tag `tag` (v0 INT = vid % 1000,
// name STRING = "v<vid>") for every vertex id.
int32_t ngd_rmat(int32_t scale, int32_t ef, double A, double B, double C, uint64_t seed, int32_t num_parts,
                 int32_t etype, int32_t with_in, int32_t with_tag, int32_t tag, int32_t rank, int32_t world,
                 int32_t threads, ngd_rows* out) {
    if (scale < 1 || scale > 40 || ef < 1 || num_parts < 1 || !out) return -1;
    Gen g{num_parts, rank, world, threads < 1 ? 1 : threads};
    uint32_t a = static_cast<uint32_t>(A * 65536), ab = static_cast<uint32_t>((A + B) * 65536),
             abc = static_cast<uint32_t>((A + B + C) * 65536);
    uint64_t E = static_cast<uint64_t>(ef) << scale;
    g.run(E, [&](Sink& s, uint64_t i) {
        uint64_t su, du;
        rmatEdge(seed, i, scale, a, ab, abc, su, du);
        int64_t src = static_cast<int64_t>(scramble(su, scale, seed));
        int64_t dst = static_cast<int64_t>(scramble(du, scale, seed));
        uint64_t h = mix64((static_cast<uint64_t>(src) << 20) ^ static_cast<uint64_t>(dst) ^ seed);
        Row r;
        r.i64(static_cast<int64_t>(h % 100));
        r.i64(static_cast<int64_t>(mix64(h ^ 0x70f1)));
        if (g.owned(src)) { s.edge(g.partOf(src), src, etype, 0, dst, r); }
        if (with_in && g.owned(dst)) { s.edge(g.partOf(dst), dst, -etype, 0, src, r); }
    });
    if (with_tag) {
        uint64_t V = 1ULL << scale;
        g.run(V, [&](Sink& s, uint64_t v) {
            int64_t vid = static_cast<int64_t>(v);
            if (!g.owned(vid)) return;
            Row r;
            r.i64(vid % 1000);
            r.str("v" + std::to_string(vid));
            s.vertex(g.partOf(vid), vid, tag, r);
        });
    }
    finish(g, out);
    return 0;
}

// Power-law graph with supernodes (C4): n vertices, ef * n background edges whose dst follows a
// Zipf-like law (dst = floor(n * u^alpha)), plus `nsuper` supernodes each receiving `superdeg`
// in-edges from uniform sources. Two edge props (INT w = h % 100, DOUBLE score in [0, 1)).
// Always writes out- and in-edge rows (the config runs REVERSELY).
int32_t ngd_powerlaw(int64_t n, int32_t ef, double alpha, int32_t nsuper, int64_t superdeg, uint64_t seed,
                     int32_t num_parts, int32_t etype, int32_t rank, int32_t world, int32_t threads, ngd_rows* out) {
    if (n < 2 || num_parts < 1 || !out) return -1;
    Gen g{num_parts, rank, world, threads < 1 ? 1 : threads};
    uint64_t E = static_cast<uint64_t>(ef) * static_cast<uint64_t>(n);
    uint64_t S = static_cast<uint64_t>(nsuper) * static_cast<uint64_t>(superdeg);
    g.run(E + S, [&](Sink& s, uint64_t i) {
        int64_t src, dst;
        if (i < E) {
            src = static_cast<int64_t>(draw(seed, 11, i) % static_cast<uint64_t>(n));
            double u = (draw(seed, 12, i) >> 11) * (1.0 / 9007199254740992.0);
            dst = static_cast<int64_t>(std::floor(static_cast<double>(n) * std::pow(u, alpha)));
            if (dst >= n) dst = n - 1;
        } else {
            uint64_t j = i - E;
            dst = static_cast<int64_t>((j / superdeg) * 7919 % static_cast<uint64_t>(n));
            src = static_cast<int64_t>(draw(seed, 13, j) % static_cast<uint64_t>(n));
        }
        uint64_t h = mix64((static_cast<uint64_t>(src) << 24) ^ static_cast<uint64_t>(dst) ^ seed);
        Row r;
        r.i64(static_cast<int64_t>(h % 100));
        r.f64((h >> 11) * (1.0 / 9007199254740992.0));
        if (g.owned(src)) { s.edge(g.partOf(src), src, etype, 0, dst, r); }
        if (g.owned(dst)) { s.edge(g.partOf(dst), dst, -etype, 0, src, r); }
    });
    finish(g, out);
    return 0;
}

// LDBC-SNB-like social graph (C5). Persons 0..np-1 (tag person: firstName STRING, age INT,
// gender STRING), posts np..np+nposts-1 (tag post: content STRING, length INT, lang STRING).
// Edge types (ids from the caller): knows person->person (creationDate INT, weight DOUBLE),
// likes person->post (creationDate INT), hasCreator post->person (creationDate INT).
// Out- and in-edge rows for every edge.
int32_t ngd_snb(int64_t np, int32_t knowsDeg, int64_t nposts, int32_t likesDeg, uint64_t seed, int32_t num_parts,
                int32_t tPerson, int32_t tPost, int32_t eKnows, int32_t eLikes, int32_t eHasCreator, int32_t rank,
                int32_t world, int32_t threads, ngd_rows* out) {
    if (np < 2 || nposts < 1 || num_parts < 1 || !out) return -1;
    Gen g{num_parts, rank, world, threads < 1 ? 1 : threads};
    static const char* kNames[] = {"Ada", "Bo", "Chen", "Dara", "Eli", "Fay", "Gus", "Hana", "Ivo", "Jun",
                                   "Kai", "Lea", "Mo", "Nia", "Oto", "Pia"};
    static const char* kLang[] = {"en", "de", "zh", "es", "fr"};
    auto both = [&](Sink& s, int64_t src, int32_t et, int64_t rank_, int64_t dst, const Row& r) {
        if (g.owned(src)) { s.edge(g.partOf(src), src, et, rank_, dst, r); }
        if (g.owned(dst)) { s.edge(g.partOf(dst), dst, -et, rank_, src, r); }
    };
    // vertices
    g.run(static_cast<uint64_t>(np + nposts), [&](Sink& s, uint64_t i) {
        int64_t vid = static_cast<int64_t>(i);
        if (!g.owned(vid)) return;
        uint64_t h = draw(seed, 21, i);
        Row r;
        if (vid < np) {
            r.str(kNames[h % 16]);
            r.i64(static_cast<int64_t>(18 + (h >> 8) % 60));
            r.str(((h >> 20) & 1) ? "female" : "male");
            s.vertex(g.partOf(vid), vid, tPerson, r);
        } else {
            uint64_t len = 8 + (h >> 8) % 120;
            std::string content;
            for (uint64_t k = 0; k < len; k++) content.push_back(static_cast<char>('a' + (mix64(h + k) % 26)));
            r.str(content);
            r.i64(static_cast<int64_t>(len));
            r.str(kLang[(h >> 30) % 5]);
            s.vertex(g.partOf(vid), vid, tPost, r);
        }
    });
    // knows: Zipf-ish popularity of the target, rank 0
    uint64_t EK = static_cast<uint64_t>(np) * knowsDeg;
    g.run(EK, [&](Sink& s, uint64_t i) {
        int64_t a = static_cast<int64_t>(i / knowsDeg);
        double u = (draw(seed, 22, i) >> 11) * (1.0 / 9007199254740992.0);
        int64_t b = static_cast<int64_t>(std::floor(static_cast<double>(np) * u * u));
        if (b >= np) b = np - 1;
        if (b == a) return;
        Row r;
        uint64_t h = mix64((static_cast<uint64_t>(a) << 24) ^ static_cast<uint64_t>(b) ^ seed);
        r.i64(static_cast<int64_t>(1262304000 + h % 315360000));
        r.f64((h >> 11) * (1.0 / 9007199254740992.0) * 10.0);
        both(s, a, eKnows, 0, b, r);
    });
    uint64_t EL = static_cast<uint64_t>(np) * likesDeg;
    g.run(EL, [&](Sink& s, uint64_t i) {
        int64_t a = static_cast<int64_t>(i / likesDeg);
        int64_t p = np + static_cast<int64_t>(draw(seed, 23, i) % static_cast<uint64_t>(nposts));
        Row r;
        r.i64(static_cast<int64_t>(1262304000 + mix64(i ^ seed) % 315360000));
        both(s, a, eLikes, 0, p, r);
    });
    g.run(static_cast<uint64_t>(nposts), [&](Sink& s, uint64_t i) {
        int64_t p = np + static_cast<int64_t>(i);
        int64_t a = static_cast<int64_t>(draw(seed, 24, i) % static_cast<uint64_t>(np));
        Row r;
        r.i64(static_cast<int64_t>(1262304000 + mix64(i ^ seed ^ 77) % 315360000));
        both(s, p, eHasCreator, 0, a, r);
    });
    finish(g, out);
    return 0;
}

// ---------------------------------------------------------------------------------------------
// The RMAT graph of ngd_rmat (the same edges and props) directly as one shard's CSR, for the
// columnar bulk load (ngx_load_csr): the vertex table sorted by (part, vid), one CSR per slot (+etype
// out-edges, -etype in-edges when with_in) whose adjacency is in RocksDB key order (rank 0, then dst
// LE bytes), duplicates collapsed (identical keys). No KV rows are built, so a C3-size shard (254 M
// edges with in-edges) costs 24 B per edge here and no sort of 40-byte keys. scale <= 31.
typedef struct {
    uint64_t nv;
    int32_t* vpart;
    int64_t* vid;
    int32_t nslots;
    int32_t etype[2];
    uint64_t ne[2];
    uint64_t* off[2];                // nv + 1
    int64_t* dst[2];
    int64_t* p0[2];
    int64_t* p1[2];
} ngd_csr;

void ngd_csr_free(ngd_csr* c) {
    if (!c) return;
    std::free(c->vpart); std::free(c->vid);
    for (int s = 0; s < 2; s++) { std::free(c->off[s]); std::free(c->dst[s]); std::free(c->p0[s]); std::free(c->p1[s]); }
    std::memset(c, 0, sizeof(*c));
}

}  // extern "C"

namespace {

// LSD radix sort of u64 keys (11-bit digits over the bits that vary), then duplicates dropped
void sortUnique(std::vector<uint64_t>& v) {
    if (v.size() < 2) return;
    uint64_t orAll = 0, andAll = ~0ULL;
    for (uint64_t x : v) { orAll |= x; andAll &= x; }
    const uint64_t vary = orAll ^ andAll;
    std::vector<uint64_t> tmp(v.size());
    for (int sh = 0; sh < 64; sh += 11) {
        if (((vary >> sh) & 0x7FF) == 0) continue;
        uint64_t cnt[2048] = {0};
        for (uint64_t x : v) cnt[(x >> sh) & 0x7FF]++;
        uint64_t acc = 0;
        for (int d = 0; d < 2048; d++) { uint64_t c = cnt[d]; cnt[d] = acc; acc += c; }
        for (uint64_t x : v) tmp[cnt[(x >> sh) & 0x7FF]++] = x;
        v.swap(tmp);
    }
    v.erase(std::unique(v.begin(), v.end()), v.end());
}

inline uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

struct RmatParams {
    int32_t scale;
    uint64_t E, seed, np;
    uint32_t a, ab, abc;
    int32_t numParts;
    bool withIn;
    RmatParams(int32_t scale_, int32_t ef, double A, double B, double C, uint64_t seed_, int32_t numParts_, bool withIn_)
        : scale(scale_), E(static_cast<uint64_t>(ef) << scale_), seed(seed_), np(static_cast<uint64_t>(numParts_)),
          a(static_cast<uint32_t>(A * 65536)), ab(static_cast<uint32_t>((A + B) * 65536)),
          abc(static_cast<uint32_t>((A + B + C) * 65536)), numParts(numParts_), withIn(withIn_) {}
};

struct Lap {
    bool on = std::getenv("NGD_TRACE") != nullptr;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    void operator()(const char* what) {
        if (!on) return;
        auto t1 = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[ngd_rmat_csr] %s %.2fs\n", what, std::chrono::duration<double>(t1 - t0).count());
        t0 = t1;
    }
};

// samples [lo, hi) of the RMAT stream on T threads; every edge becomes an out-key under its src and
// (withIn) an in-key under its dst: keys (vid << 32 | bswap32(other)), the order of (vid, the other
// end's LE bytes) = RocksDB's within one (part, vid, type) prefix at rank 0. bucketOf(slot, part)
// picks the output vector (or -1: not kept); returns per-thread vectors, nb of them per thread.
template <typename BucketOf>
std::vector<std::vector<std::vector<uint64_t>>> sampleKeys(const RmatParams& P, uint64_t lo, uint64_t hi, int T, size_t nb,
                                                            BucketOf bucketOf) {
    std::vector<std::vector<std::vector<uint64_t>>> loc(T, std::vector<std::vector<uint64_t>>(nb));
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++) {
        th.emplace_back([&, t] {
            auto& L = loc[t];
            for (uint64_t i = lo + (hi - lo) * t / T; i < lo + (hi - lo) * (t + 1) / T; i++) {
                uint64_t su, du;
                rmatEdge(P.seed, i, P.scale, P.a, P.ab, P.abc, su, du);
                const uint64_t src = scramble(su, P.scale, P.seed), dst = scramble(du, P.scale, P.seed);
                const uint32_t ps = static_cast<uint32_t>(src % P.np) + 1, pd = static_cast<uint32_t>(dst % P.np) + 1;
                const int64_t bo = bucketOf(0, ps);
                if (bo >= 0) L[bo].push_back(src << 32 | bswap32(static_cast<uint32_t>(dst)));
                if (P.withIn) {
                    const int64_t bi = bucketOf(1, pd);
                    if (bi >= 0) L[bi].push_back(dst << 32 | bswap32(static_cast<uint32_t>(src)));
                }
            }
        });
    }
    for (auto& x : th) x.join();
    return loc;
}

// the shard's CSR from its keys per (slot, part) bucket (bk[slot * (numParts + 1) + part], unsorted;
// consumed): sorted and deduplicated per bucket, vertex table = union of the key vids per part
void buildCsr(const RmatParams& P, int32_t etype, int T, std::vector<std::vector<uint64_t>>& bk, ngd_csr* out, Lap& lap) {
    const int NS = P.withIn ? 2 : 1;
    const int32_t num_parts = P.numParts;
    const size_t NB = static_cast<size_t>(NS) * (num_parts + 1);
    {
        std::atomic<size_t> next{0};
        std::vector<std::thread> th;
        for (int t = 0; t < T; t++) th.emplace_back([&] { for (size_t b; (b = next.fetch_add(1)) < NB;) sortUnique(bk[b]); });
        for (auto& x : th) x.join();
    }
    lap("sort");
    // vertex table: per part, the union of the slots' key vids (every key's src is a vertex row)
    std::vector<std::vector<int64_t>> pv(num_parts + 1);
    std::vector<uint64_t> vbase(num_parts + 2, 0);
    for (int32_t p = 1; p <= num_parts; p++) {
        auto& V = pv[p];
        for (int s = 0; s < NS; s++) {
            const auto& K = bk[static_cast<size_t>(s) * (num_parts + 1) + p];
            std::vector<int64_t> m;
            m.reserve(V.size() + K.size() / 4 + 1);
            size_t i = 0;
            for (size_t j = 0; j < K.size();) {
                const int64_t v = static_cast<int64_t>(K[j] >> 32);
                while (i < V.size() && V[i] < v) m.push_back(V[i++]);
                if (i < V.size() && V[i] == v) i++;
                m.push_back(v);
                while (j < K.size() && static_cast<int64_t>(K[j] >> 32) == v) j++;
            }
            while (i < V.size()) m.push_back(V[i++]);
            V.swap(m);
        }
        vbase[p + 1] = vbase[p] + V.size();
    }
    const uint64_t nv = vbase[num_parts + 1];
    out->nv = nv;
    out->nslots = NS;
    out->vpart = static_cast<int32_t*>(std::malloc(std::max<uint64_t>(nv, 1) * 4));
    out->vid = static_cast<int64_t*>(std::malloc(std::max<uint64_t>(nv, 1) * 8));
    for (int32_t p = 1; p <= num_parts; p++)
        for (uint64_t i = 0; i < pv[p].size(); i++) { out->vpart[vbase[p] + i] = p; out->vid[vbase[p] + i] = pv[p][i]; }
    for (int s = 0; s < NS; s++) {
        out->etype[s] = s == 0 ? etype : -etype;
        uint64_t ne = 0;
        for (int32_t p = 1; p <= num_parts; p++) ne += bk[static_cast<size_t>(s) * (num_parts + 1) + p].size();
        out->ne[s] = ne;
        out->off[s] = static_cast<uint64_t*>(std::malloc((nv + 1) * 8));
        out->dst[s] = static_cast<int64_t*>(std::malloc(std::max<uint64_t>(ne, 1) * 8));
        out->p0[s] = static_cast<int64_t*>(std::malloc(std::max<uint64_t>(ne, 1) * 8));
        out->p1[s] = static_cast<int64_t*>(std::malloc(std::max<uint64_t>(ne, 1) * 8));
        std::vector<uint64_t> ebase(num_parts + 2, 0);
        for (int32_t p = 1; p <= num_parts; p++) ebase[p + 1] = ebase[p] + bk[static_cast<size_t>(s) * (num_parts + 1) + p].size();
        std::atomic<int32_t> next{1};
        std::vector<std::thread> th;
        for (int t = 0; t < T; t++) {
            th.emplace_back([&, s] {
                for (int32_t p; (p = next.fetch_add(1)) <= num_parts;) {
                    auto& K = bk[static_cast<size_t>(s) * (num_parts + 1) + p];
                    const auto& V = pv[p];
                    uint64_t e = ebase[p];
                    size_t j = 0;
                    for (size_t r = 0; r < V.size(); r++) {
                        out->off[s][vbase[p] + r] = e;
                        for (; j < K.size() && static_cast<int64_t>(K[j] >> 32) == V[r]; j++, e++) {
                            const int64_t v = V[r];
                            const int64_t o = static_cast<int64_t>(bswap32(static_cast<uint32_t>(K[j])));
                            out->dst[s][e] = o;
                            const int64_t os = s == 0 ? v : o, od = s == 0 ? o : v;   // the edge as generated
                            const uint64_t h = mix64((static_cast<uint64_t>(os) << 20) ^ static_cast<uint64_t>(od) ^ P.seed);
                            out->p0[s][e] = static_cast<int64_t>(h % 100);
                            out->p1[s][e] = static_cast<int64_t>(mix64(h ^ 0x70f1));
                        }
                    }
                    std::vector<uint64_t>().swap(K);
                }
            });
        }
        for (auto& x : th) x.join();
        out->off[s][nv] = ne;
    }
    lap("csr");
}

std::string shardFile(const char* prefix, int32_t producer, int32_t consumer, int s) {
    return std::string(prefix) + "." + std::to_string(producer) + "." + std::to_string(consumer) + "." + std::to_string(s);
}

}  // namespace

extern "C" {

int32_t ngd_rmat_csr(int32_t scale, int32_t ef, double A, double B, double C, uint64_t seed, int32_t num_parts,
                     int32_t etype, int32_t with_in, int32_t rank, int32_t world, int32_t threads, ngd_csr* out) {
    if (scale < 1 || scale > 31 || ef < 1 || num_parts < 1 || num_parts > 4096 || etype <= 0 || !out) return -1;
    std::memset(out, 0, sizeof(*out));
    const int T = threads < 1 ? 1 : threads;
    const RmatParams P(scale, ef, A, B, C, seed, num_parts, with_in != 0);
    const int NS = with_in ? 2 : 1;
    const size_t NB = static_cast<size_t>(NS) * (num_parts + 1);
    std::vector<uint8_t> mine(num_parts + 1, 0);                 // the parts this shard owns
    for (int32_t p = 1; p <= num_parts; p++) mine[p] = world <= 1 || p % world == rank;
    Lap lap;
    auto loc = sampleKeys(P, 0, P.E, T, NB, [&](int s, uint32_t p) -> int64_t {
        return mine[p] ? static_cast<int64_t>(s) * (num_parts + 1) + p : -1;
    });
    lap("sample");
    std::vector<std::vector<uint64_t>> bk(NB);
    for (size_t b = 0; b < NB; b++) {
        size_t n = 0;
        for (int u = 0; u < T; u++) n += loc[u][b].size();
        bk[b].reserve(n);
        for (int u = 0; u < T; u++) {
            bk[b].insert(bk[b].end(), loc[u][b].begin(), loc[u][b].end());
            std::vector<uint64_t>().swap(loc[u][b]);
        }
    }
    buildCsr(P, etype, T, bk, out, lap);
    return 0;
}

// The same shard built by `world` processes that split the sampling: producer q samples its 1/producers
// of the edge stream and writes the keys of every consumer shard r (the owner of the key's part) to
// "<prefix>.<q>.<r>.<slot>" (raw u64); once every producer has written, each shard reads its files
// (ngd_rmat_csr_build, which removes them) and builds exactly what ngd_rmat_csr would.
int32_t ngd_rmat_csr_sample(int32_t scale, int32_t ef, double A, double B, double C, uint64_t seed, int32_t num_parts,
                            int32_t with_in, int32_t world, int32_t producer, int32_t producers, int32_t threads,
                            const char* prefix) {
    if (scale < 1 || scale > 31 || ef < 1 || num_parts < 1 || num_parts > 4096 || world < 1 || producers < 1 ||
        producer < 0 || producer >= producers || !prefix)
        return -1;
    const int T = threads < 1 ? 1 : threads;
    const RmatParams P(scale, ef, A, B, C, seed, num_parts, with_in != 0);
    const int NS = with_in ? 2 : 1;
    const size_t NB = static_cast<size_t>(world) * NS;
    Lap lap;
    const uint64_t lo = P.E * producer / producers, hi = P.E * (producer + 1) / producers;
    auto loc = sampleKeys(P, lo, hi, T, NB, [&](int s, uint32_t p) -> int64_t {
        return static_cast<int64_t>(world > 1 ? p % world : 0) * NS + s;
    });
    lap("sample");
    for (int32_t r = 0; r < world; r++) {
        for (int s = 0; s < NS; s++) {
            const std::string path = shardFile(prefix, producer, r, s);
            FILE* f = std::fopen(path.c_str(), "wb");
            if (!f) return -2;
            bool ok = true;
            for (int u = 0; u < T && ok; u++) {
                auto& v = loc[u][static_cast<size_t>(r) * NS + s];
                ok = v.empty() || std::fwrite(v.data(), 8, v.size(), f) == v.size();
                std::vector<uint64_t>().swap(v);
            }
            if (std::fclose(f) != 0 || !ok) return -2;
        }
    }
    lap("write");
    return 0;
}

int32_t ngd_rmat_csr_build(int32_t scale, uint64_t seed, int32_t num_parts, int32_t etype, int32_t with_in, int32_t rank,
                           int32_t world, int32_t producers, int32_t threads, const char* prefix, ngd_csr* out) {
    if (scale < 1 || scale > 31 || num_parts < 1 || num_parts > 4096 || etype <= 0 || !out || !prefix) return -1;
    std::memset(out, 0, sizeof(*out));
    const int T = threads < 1 ? 1 : threads;
    const RmatParams P(scale, 16, 0, 0, 0, seed, num_parts, with_in != 0);
    const int NS = with_in ? 2 : 1;
    Lap lap;
    std::vector<std::vector<uint64_t>> bk(static_cast<size_t>(NS) * (num_parts + 1));
    for (int s = 0; s < NS; s++) {
        // every producer's keys for this shard and slot, bucketed by part
        std::vector<uint64_t> all;
        for (int32_t q = 0; q < producers; q++) {
            const std::string path = shardFile(prefix, q, rank, s);
            FILE* f = std::fopen(path.c_str(), "rb");
            if (!f) return -2;
            std::fseek(f, 0, SEEK_END);
            const long bytes = std::ftell(f);
            std::fseek(f, 0, SEEK_SET);
            const size_t n = bytes > 0 ? static_cast<size_t>(bytes) / 8 : 0;
            const size_t at = all.size();
            all.resize(at + n);
            const bool ok = n == 0 || std::fread(all.data() + at, 8, n, f) == n;
            std::fclose(f);
            std::remove(path.c_str());
            if (!ok) return -2;
        }
        std::vector<uint64_t> cnt(num_parts + 2, 0);
        for (uint64_t k : all) cnt[(k >> 32) % P.np + 1]++;
        for (int32_t p = 1; p <= num_parts; p++) bk[static_cast<size_t>(s) * (num_parts + 1) + p].reserve(cnt[p]);
        for (uint64_t k : all) bk[static_cast<size_t>(s) * (num_parts + 1) + ((k >> 32) % P.np + 1)].push_back(k);
    }
    lap("read");
    buildCsr(P, etype, T, bk, out, lap);
    return 0;
}

// GO FROM list for the RMAT configs: `k` vids drawn uniformly (with repetition) from the vertices
// with at least one out-edge (SURVEY §8d "sampled uniformly from non-isolated vertices").
int32_t ngd_rmat_seeds(int32_t scale, int32_t ef, double A, double B, double C, uint64_t seed, uint64_t sampleSeed,
                       uint64_t k, int32_t threads, int64_t* out) {
    if (scale < 1 || scale > 40) return -1;
    uint64_t V = 1ULL << scale, E = static_cast<uint64_t>(ef) << scale;
    std::vector<std::atomic<uint8_t>> has(V);
    for (auto& h : has) h.store(0, std::memory_order_relaxed);
    uint32_t a = static_cast<uint32_t>(A * 65536), ab = static_cast<uint32_t>((A + B) * 65536),
             abc = static_cast<uint32_t>((A + B + C) * 65536);
    int T = threads < 1 ? 1 : threads;
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++) {
        th.emplace_back([&, t] {
            for (uint64_t i = E * t / T; i < E * (t + 1) / T; i++) {
                uint64_t su, du;
                rmatEdge(seed, i, scale, a, ab, abc, su, du);
                has[scramble(su, scale, seed)].store(1, std::memory_order_relaxed);
            }
        });
    }
    for (auto& x : th) x.join();
    uint64_t found = 0;
    for (uint64_t i = 0; found < k && i < 64 * k + V; i++) {
        uint64_t v = draw(sampleSeed, 98, i) % V;
        if (has[v].load(std::memory_order_relaxed)) out[found++] = static_cast<int64_t>(v);
    }
    return found == k ? 0 : -2;
}

// deterministic sample of `k` vids in [0, range) (the GO FROM list), with repetitions possible
void ngd_sample_vids(uint64_t seed, uint64_t range, uint64_t k, int64_t* out) {
    for (uint64_t i = 0; i < k; i++) out[i] = static_cast<int64_t>(draw(seed, 99, i) % range);
}

}  // extern "C"
