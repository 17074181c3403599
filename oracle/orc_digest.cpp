// ORACLE — TEST INFRASTRUCTURE ONLY. The expected digest of a GO record hop's rows, computed on the
// host from a shard's generated CSR (tests/c3_rehearsal_worker.py): the result rows of
// `GO … OVER e [WHERE e.p0 < 50 | e.p0 >= 50] YIELD e._dst, e._rank, e.p0, e.p1` are, per frontier row
// of the last hop, every out-edge of the row (GoExecutor::processFinalResult, GoExecutor.cpp:1082-1335,
// one row per edge that passes the filter; rows compared as a multiset, TestBase.h:188-233).
//
// Row hash (restated independently of the device kernel, kernels.hip k_row_digest, and of the header's
// description of ngx_go_result_digest): h = m(...m(m(S ^ src) ^ dst) ^ rank) ^ p0) ^ p1), m = splitmix64's
// finalizer, S = 0x9E3779B97F4A7C15; the digest is (sum of h mod 2^64, XOR of h, rows).
#include <cstdint>
#include <thread>
#include <vector>

namespace {

inline uint64_t mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

inline uint64_t rowHash(const int64_t* v, int n) {
    uint64_t h = 0x9E3779B97F4A7C15ULL;
    for (int k = 0; k < n; k++) h = mix(h ^ static_cast<uint64_t>(v[k]));
    return h;
}

}  // namespace

extern "C" {

// out[3 * m + {0, 1, 2}] = (sum, xor, rows) for m = 0: every edge, 1: p0 < 50, 2: p0 >= 50, over the
// out-edges [off[r], off[r + 1]) of each frontier row r in rows[0 .. nrows); src = vid[r], rank = `rank`.
int orc_hop_digest(uint64_t nrows, const int64_t* rows, const int64_t* vid, const uint64_t* off, const int64_t* dst,
                   const int8_t* p0, const int64_t* p1, int64_t rank, int threads, uint64_t* out) {
    if (threads < 1) threads = 1;
    std::vector<uint64_t> part(static_cast<size_t>(threads) * 9, 0);
    auto work = [&](int t) {
        uint64_t* o = part.data() + static_cast<size_t>(t) * 9;
        for (uint64_t i = t; i < nrows; i += threads) {
            const int64_t r = rows[i];
            const int64_t src = vid[r];
            for (uint64_t e = off[r]; e < off[r + 1]; e++) {
                const int64_t v[5] = {src, dst[e], rank, p0[e], p1[e]};
                const uint64_t h = rowHash(v, 5);
                const int m = p0[e] < 50 ? 1 : 2;
                o[0] += h; o[1] ^= h; o[2]++;
                o[3 * m] += h; o[3 * m + 1] ^= h; o[3 * m + 2]++;
            }
        }
    };
    std::vector<std::thread> ts;
    for (int t = 1; t < threads; t++) ts.emplace_back(work, t);
    work(0);
    for (auto& t : ts) t.join();
    for (int k = 0; k < 9; k++) out[k] = 0;
    for (int t = 0; t < threads; t++) {
        for (int m = 0; m < 3; m++) {
            out[3 * m] += part[t * 9 + 3 * m];
            out[3 * m + 1] ^= part[t * 9 + 3 * m + 1];
            out[3 * m + 2] += part[t * 9 + 3 * m + 2];
        }
    }
    return 0;
}

// the same hash over given row tuples (tests: the device digest of small results against this)
int orc_row_digest(uint64_t n, int ncols, const int64_t* const* cols, uint64_t* out) {
    out[0] = out[1] = out[2] = 0;
    std::vector<int64_t> v(static_cast<size_t>(ncols));
    for (uint64_t i = 0; i < n; i++) {
        for (int k = 0; k < ncols; k++) v[k] = cols[k][i];
        const uint64_t h = rowHash(v.data(), ncols);
        out[0] += h; out[1] ^= h; out[2]++;
    }
    return 0;
}

}  // extern "C"
