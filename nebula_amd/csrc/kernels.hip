// HIP kernels of the GetNeighbors / GO path on gfx950 (MI355X), and their host launchers.
//
//  * k_lookup           seed (part, vid) -> vertex row, binary search of the sorted vertex table
//  * tile scans         3-phase reduce-then-scan (tile = 256 threads x 16 items) used for entry
//                       degrees (CSR offsets of the frontier) and for frontier compaction
//  * k_expand_mark      intermediate hop: edge-balanced expansion. A workgroup owns 4096 consecutive
//                       frontier edges whatever their vertices' degrees (a supernode spreads over
//                       many workgroups, a thread never loops over a whole adjacency); the edge ->
//                       frontier-entry map is built in LDS (atomicMax scatter + max-scan); each
//                       edge reads one 4-byte destination row id (coalesced) and marks the
//                       destination in an epoch byte array = the hop's frontier dedup
//  * k_compact          visited[row] == epoch -> next frontier (ballot-free tile compaction)
//  * k_final_eval       last hop: storage filter (pushdown) + graphd WHERE through the bytecode VM,
//                       wave-ballot pass masks + per-chunk pass counts
//  * k_final_emit       last hop: YIELD columns for passing edges, written densely at
//                       chunk offset + ballot prefix (deterministic order)
//  * k_pack / k_merge   multi-GPU frontier exchange: epoch marks -> per-peer bitmaps and back
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>

#include "kernels.h"

namespace ngx {

constexpr int WG = 256;
constexpr int ITEMS = 16;
constexpr int TILE = WG * ITEMS;      // 4096
constexpr int NW = WG / 64;

// ------------------------------------------------------------------------------ VM
__device__ Val vmEval(const Insn* code, const VmEnv& env, const EdgeCtx& ec) {
    Val st[kMaxStack];
    int sp = 0;
    for (int pc = 0;; pc++) {
        const Insn in = code[pc];
        switch (in.op) {
            case OP_END:
                return sp > 0 ? st[sp - 1] : mkErr();
            case OP_PUSH:
                st[sp++] = constVal(in.t1, in.imm, static_cast<uint32_t>(in.a), env.pool);
                break;
            case OP_ERR:
                st[sp++] = mkErr();
                break;
            case OP_ECOL: {
                int32_t at = ec.etype < 0 ? -ec.etype : ec.etype;
                if (at != in.b) {
                    st[sp++] = (in.mode & 1) ? constVal(in.t2, in.imm, 0, env.pool) : mkErr();
                    break;
                }
                const DSlot& s = env.slots[ec.slot];
                const DCol& c = env.cols[s.colBase + in.a];
                if (c.valid != nullptr && c.valid[ec.pos] == 0) {
                    st[sp++] = (in.mode & 2) ? defaultOfType(c.type) : mkErr();
                    break;
                }
                st[sp++] = loadCol(c, ec.pos);
                break;
            }
            case OP_EKEY: {
                int32_t at = ec.etype < 0 ? -ec.etype : ec.etype;
                if (in.b != 0 && at != in.b) {
                    st[sp++] = (in.mode & 1) ? constVal(in.t2, in.imm, 0, env.pool) : mkErr();
                    break;
                }
                int64_t v = in.a == 0 ? ec.src : in.a == 1 ? ec.dst : in.a == 2 ? ec.rank : static_cast<int64_t>(ec.etype);
                st[sp++] = mkInt(v);
                break;
            }
            case OP_EDST: {
                int32_t at = ec.etype < 0 ? -ec.etype : ec.etype;
                st[sp++] = mkInt((in.b != 0 && at != in.b) ? 0 : ec.dst);
                break;
            }
            case OP_SRCTAG: case OP_DSTTAG: {
                const DTag& t = env.tags[in.b];
                uint32_t row = in.op == OP_SRCTAG ? ec.srow : ec.drow;
                if (row == kNoRow || t.present[row] == 0) {
                    st[sp++] = (in.mode & 1) ? constVal(in.t2, in.imm, 0, env.pool) : mkErr();
                    break;
                }
                const DCol& c = env.cols[t.colBase + in.a];
                if (c.valid != nullptr && c.valid[row] == 0) { st[sp++] = defaultOfType(c.type); break; }
                st[sp++] = loadCol(c, row);
                break;
            }
            case OP_PLUS:
                break;
            case OP_NEG: {
                Val& v = st[sp - 1];
                if (v.t == V_INT) v.x = static_cast<int64_t>(0ULL - static_cast<uint64_t>(v.x));
                else if (v.t == V_DBL) v = mkDbl(-dblOf(v));
                else v = mkErr();
                break;
            }
            case OP_NOT: {
                Val& v = st[sp - 1];
                if (v.t != V_ERR) v = mkBool(!asBool(v));
                break;
            }
            case OP_CAST: {                                  // TypeCastingExpression::eval
                Val& v = st[sp - 1];
                if (v.t == V_ERR) break;
                if (v.t == V_STR) {                          // folly::to<int/double>(string): host only
                    if (in.t1 != 3) { atomicOr(env.unsupported, 1u); v = mkErr(); break; }
                    v = mkBool(asBool(v));
                    break;
                }
                if (in.t1 == 0 || in.t1 == 4) v = mkInt(toInt(v));
                else if (in.t1 == 2) v = mkDbl(toDouble(v));
                else v = mkBool(asBool(v));
                break;
            }
            case OP_ADD: case OP_SUB: case OP_MUL: case OP_DIV: case OP_MOD: case OP_AXOR: {
                Val r = st[--sp];
                Val l = st[sp - 1];
                Val out = mkErr();
                if (l.t == V_ERR) { out = l; }
                else if (r.t == V_ERR) { out = r; }
                else if ((l.t == V_INT || l.t == V_DBL) && (r.t == V_INT || r.t == V_DBL)) {
                    bool dbl = l.t == V_DBL || r.t == V_DBL;
                    if (dbl) {
                        double a = asDouble(l), b = asDouble(r);
                        switch (in.op) {
                            case OP_ADD: out = mkDbl(a + b); break;
                            case OP_SUB: out = mkDbl(a - b); break;
                            case OP_MUL: out = mkDbl(a * b); break;
                            case OP_DIV: out = fabs(b) < 1e-8 ? mkErr() : mkDbl(a / b); break;
                            case OP_MOD: out = fabs(b) < 1e-8 ? mkErr() : mkDbl(fmod(a, b)); break;
                            default: out = mkInt(static_cast<int64_t>(round(a)) ^ static_cast<int64_t>(round(b))); break;
                        }
                    } else {
                        int64_t a = l.x, b = r.x;
                        switch (in.op) {
                            case OP_ADD: {
                                bool of = (a >= 0 && b >= 0) ? (INT64_MAX - a < b) : (a < 0 && b < 0) ? (INT64_MIN - a > b) : false;
                                out = of ? mkErr() : mkInt(a + b);
                                break;
                            }
                            case OP_SUB: {
                                bool of = (a > 0 && b < 0) ? (b == INT64_MIN || INT64_MAX - a < -b)
                                        : (a < 0 && b > 0) ? (INT64_MIN - a > -b) : false;
                                out = of ? mkErr() : mkInt(a - b);
                                break;
                            }
                            case OP_MUL:
                                out = mulOverflow(a, b) ? mkErr()
                                    : mkInt(static_cast<int64_t>(static_cast<uint64_t>(a) * static_cast<uint64_t>(b)));
                                break;
                            case OP_DIV:
                                out = (b == 0 || (a == INT64_MIN && b == -1)) ? mkErr() : mkInt(a / b);
                                break;
                            case OP_MOD:
                                out = b == 0 ? mkErr() : (b == -1 ? mkInt(0) : mkInt(a % b));
                                break;
                            default: out = mkInt(a ^ b); break;
                        }
                    }
                } else if (in.op == OP_ADD && l.t == V_STR && r.t == V_STR) {
                    atomicOr(env.unsupported, 1u);           // string concatenation builds a new string
                }
                st[sp - 1] = out;
                break;
            }
            case OP_LT: case OP_LE: case OP_GT: case OP_GE: case OP_EQ: case OP_NE: case OP_CONTAINS: {
                Val r = st[--sp];
                Val l = st[sp - 1];
                Val out;
                if (l.t == V_ERR) out = l;
                else if (r.t == V_ERR) out = r;
                else if (in.op == OP_CONTAINS) {
                    out = (l.t == V_STR && r.t == V_STR) ? mkBool(strContains(l, r)) : mkErr();
                } else if ((l.t == V_STR) != (r.t == V_STR)) {
                    out = mkErr();                           // string vs non-string
                } else {
                    int c;                                   // -1 / 0 / 1, 2 = unordered (NaN)
                    bool eqOnly = false, eqv = false;
                    if (l.t == V_STR) {
                        c = strCmp(l, r);
                    } else if (l.t == V_DBL || r.t == V_DBL) {
                        double a = toDouble(l), b = toDouble(r);
                        c = a < b ? -1 : (a > b ? 1 : (a == b ? 0 : 2));
                        if (in.op == OP_EQ || in.op == OP_NE) { eqOnly = true; eqv = fabs(a - b) < 1e-8; }
                    } else if (l.t == V_INT || r.t == V_INT) {
                        int64_t a = toInt(l), b = toInt(r);
                        c = a < b ? -1 : (a > b ? 1 : 0);
                    } else {                                 // bool vs bool
                        c = l.x < r.x ? -1 : (l.x > r.x ? 1 : 0);
                    }
                    bool res;
                    switch (in.op) {
                        case OP_LT: res = c == -1; break;
                        case OP_LE: res = c == -1 || c == 0; break;
                        case OP_GT: res = c == 1; break;
                        case OP_GE: res = c == 1 || c == 0; break;
                        case OP_EQ: res = eqOnly ? eqv : c == 0; break;
                        default: res = eqOnly ? !eqv : c != 0; break;
                    }
                    out = mkBool(res);
                }
                st[sp - 1] = out;
                break;
            }
            case OP_AND: case OP_OR: case OP_LXOR: {
                Val r = st[--sp];
                Val l = st[sp - 1];
                if (l.t == V_ERR) { st[sp - 1] = l; break; }
                if (r.t == V_ERR) { st[sp - 1] = r; break; }
                bool a = asBool(l), b = asBool(r);
                st[sp - 1] = mkBool(in.op == OP_AND ? (a && b) : in.op == OP_OR ? (a || b) : (a != b));
                break;
            }
            case OP_FUNC: {
                int argc = in.b;
                Val* args = &st[sp - argc];
                Val out = mkErr();
                bool anyErr = false;
                for (int k = 0; k < argc; k++) if (args[k].t == V_ERR) { out = args[k]; anyErr = true; break; }
                if (!anyErr) {
                    bool num1 = args[0].t == V_INT || args[0].t == V_DBL;
                    switch (in.a) {
                        case F_ABS: if (num1) out = mkDbl(fabs(asDouble(args[0]))); break;
                        case F_FLOOR: if (num1) out = mkDbl(floor(asDouble(args[0]))); break;
                        case F_CEIL: if (num1) out = mkDbl(ceil(asDouble(args[0]))); break;
                        case F_ROUND: if (num1) out = mkDbl(round(asDouble(args[0]))); break;
                        case F_SQRT: if (num1) out = mkDbl(sqrt(asDouble(args[0]))); break;
                        case F_CBRT: if (num1) out = mkDbl(cbrt(asDouble(args[0]))); break;
                        case F_EXP: if (num1) out = mkDbl(exp(asDouble(args[0]))); break;
                        case F_EXP2: if (num1) out = mkDbl(exp2(asDouble(args[0]))); break;
                        case F_LOG: if (num1) out = mkDbl(log(asDouble(args[0]))); break;
                        case F_LOG2: if (num1) out = mkDbl(log2(asDouble(args[0]))); break;
                        case F_LOG10: if (num1) out = mkDbl(log10(asDouble(args[0]))); break;
                        case F_SIN: if (num1) out = mkDbl(sin(asDouble(args[0]))); break;
                        case F_ASIN: if (num1) out = mkDbl(asin(asDouble(args[0]))); break;
                        case F_COS: if (num1) out = mkDbl(cos(asDouble(args[0]))); break;
                        case F_ACOS: if (num1) out = mkDbl(acos(asDouble(args[0]))); break;
                        case F_TAN: if (num1) out = mkDbl(tan(asDouble(args[0]))); break;
                        case F_ATAN: if (num1) out = mkDbl(atan(asDouble(args[0]))); break;
                        case F_HYPOT: case F_POW: {
                            bool num2 = args[1].t == V_INT || args[1].t == V_DBL;
                            if (num1 && num2) {
                                double a = asDouble(args[0]), b = asDouble(args[1]);
                                out = mkDbl(in.a == F_HYPOT ? hypot(a, b) : pow(a, b));
                            }
                            break;
                        }
                        case F_LENGTH: if (args[0].t == V_STR) out = mkInt(args[0].len); break;
                        case F_STRCASECMP: {
                            if (args[0].t == V_STR && args[1].t == V_STR) {      // C strings: stop at NUL
                                const unsigned char* p = reinterpret_cast<const unsigned char*>(args[0].x);
                                const unsigned char* q = reinterpret_cast<const unsigned char*>(args[1].x);
                                int res = 0;
                                for (uint32_t k = 0;; k++) {
                                    int c1 = k < args[0].len ? p[k] : 0;
                                    int c2 = k < args[1].len ? q[k] : 0;
                                    if (c1 >= 'A' && c1 <= 'Z') c1 += 32;
                                    if (c2 >= 'A' && c2 <= 'Z') c2 += 32;
                                    if (c1 != c2 || c1 == 0) { res = c1 - c2; break; }
                                }
                                out = mkInt(res);
                            }
                            break;
                        }
                        case F_HASH: {
                            const Val& a = args[0];
                            if (a.t == V_INT || a.t == V_BOOL) out = mkInt(a.x);
                            else if (a.t == V_DBL) {
                                double d = dblOf(a);
                                out = mkInt(d != 0.0 ? static_cast<int64_t>(hashBytes(reinterpret_cast<const unsigned char*>(&d), 8)) : 0);
                            } else {
                                out = mkInt(static_cast<int64_t>(hashBytes(reinterpret_cast<const unsigned char*>(a.x), a.len)));
                            }
                            break;
                        }
                        case F_UDF_IS_IN: {                  // FunctionManager.cpp:467-513
                            const Val& c = args[0];
                            bool found = false;
                            for (int k = 1; k < argc && !found; k++) {
                                const Val& v = args[k];
                                if (c.t == V_INT) {
                                    if (v.t == V_STR) { atomicOr(env.unsupported, 1u); break; }
                                    found = toInt(v) == c.x;
                                } else if (c.t == V_DBL) {
                                    if (v.t == V_STR) { atomicOr(env.unsupported, 1u); break; }
                                    found = toDouble(v) == dblOf(c);
                                } else if (c.t == V_BOOL) {
                                    found = asBool(v) == (c.x != 0);
                                } else {
                                    if (v.t != V_STR) { atomicOr(env.unsupported, 1u); break; }   // toString
                                    found = strCmp(c, v) == 0;
                                }
                            }
                            out = mkBool(found);
                            break;
                        }
                        default: break;
                    }
                }
                sp -= argc;
                st[sp++] = out;
                break;
            }
            default:
                return mkErr();
        }
    }
}

// ------------------------------------------------------------------------------ block helpers
__device__ __forceinline__ uint64_t blockExScan(uint64_t v, uint64_t& total, uint64_t* sm) {
    int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint64_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint64_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) sm[wid] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t acc = 0;
        for (int w = 0; w < NW; w++) { uint64_t t = sm[w]; sm[w] = acc; acc += t; }
        sm[NW] = acc;
    }
    __syncthreads();
    uint64_t r = sm[wid] + x - v;
    total = sm[NW];
    __syncthreads();
    return r;
}

__device__ __forceinline__ uint64_t blockSum(uint64_t v, uint64_t* sm) {
    uint64_t t;
    blockExScan(v, t, sm);
    return t;
}

// ------------------------------------------------------------------------------ 3-phase scans
struct DegreeIn {                // degree of frontier entry i = (frontier row i / ns, slot i % ns)
    const uint32_t* F;
    HopSlots hs;
    __device__ __forceinline__ uint64_t operator()(uint64_t i) const {
        uint32_t r = F[i / hs.n];
        if (r == kNoRow) return 0;
        const uint64_t* off = hs.off[i % hs.n];
        return off[r + 1] - off[r];
    }
};
struct FlagIn {                  // visited[gbase + r] == epoch
    const uint8_t* visited;
    uint64_t gbase;
    uint8_t epoch;
    __device__ __forceinline__ uint64_t operator()(uint64_t r) const { return visited[gbase + r] == epoch ? 1 : 0; }
};
struct CountIn {                 // plain uint32 counts
    const uint32_t* c;
    __device__ __forceinline__ uint64_t operator()(uint64_t i) const { return c[i]; }
};
struct WriteEstart {
    uint64_t* estart;
    __device__ __forceinline__ void operator()(uint64_t i, uint64_t v, uint64_t pre) const { (void)v; estart[i] = pre; }
};
struct WriteCompact {
    uint32_t* out;
    __device__ __forceinline__ void operator()(uint64_t i, uint64_t v, uint64_t pre) const { if (v) out[pre] = static_cast<uint32_t>(i); }
};

template <class In>
__global__ __launch_bounds__(WG) void k_tile_reduce(In in, uint64_t n, uint64_t* tileSums) {
    __shared__ uint64_t sm[NW + 1];
    uint64_t base = static_cast<uint64_t>(blockIdx.x) * TILE + static_cast<uint64_t>(threadIdx.x) * ITEMS;
    uint64_t s = 0;
#pragma unroll 4
    for (int k = 0; k < ITEMS; k++) if (base + k < n) s += in(base + k);
    uint64_t t = blockSum(s, sm);
    if (threadIdx.x == 0) tileSums[blockIdx.x] = t;
}

__global__ __launch_bounds__(1024) void k_scan_tiles(uint64_t* sums, uint64_t nt, uint64_t* total) {
    __shared__ uint64_t sm[1024 / 64 + 1];
    uint64_t per = (nt + 1023) / 1024;
    uint64_t lo = threadIdx.x * per, hi = lo + per < nt ? lo + per : nt;
    uint64_t s = 0;
    for (uint64_t i = lo; i < hi; i++) s += sums[i];
    // block exclusive scan over 1024 threads
    int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint64_t x = s;
    for (int o = 1; o < 64; o <<= 1) {
        uint64_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) sm[wid] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t acc = 0;
        for (int w = 0; w < 16; w++) { uint64_t t = sm[w]; sm[w] = acc; acc += t; }
        sm[16] = acc;
    }
    __syncthreads();
    uint64_t pre = sm[wid] + x - s;
    for (uint64_t i = lo; i < hi; i++) { uint64_t t = sums[i]; sums[i] = pre; pre += t; }
    if (threadIdx.x == 0) *total = sm[16];
}

template <class In, class Out>
__global__ __launch_bounds__(WG) void k_tile_scan(In in, uint64_t n, const uint64_t* tileOff, Out out) {
    __shared__ uint64_t sm[NW + 1];
    uint64_t base = static_cast<uint64_t>(blockIdx.x) * TILE + static_cast<uint64_t>(threadIdx.x) * ITEMS;
    uint64_t v[ITEMS];
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < ITEMS; k++) { v[k] = base + k < n ? in(base + k) : 0; s += v[k]; }
    uint64_t tot;
    uint64_t pre = blockExScan(s, tot, sm) + tileOff[blockIdx.x];
#pragma unroll
    for (int k = 0; k < ITEMS; k++) {
        if (base + k < n) out(base + k, v[k], pre);
        pre += v[k];
    }
}

template <class In, class Out>
static int scan3(In in, uint64_t n, Out out, uint64_t* tileSums, uint64_t* total, hipStream_t s) {
    uint64_t nt = (n + TILE - 1) / TILE;
    if (nt == 0) { (void)hipMemsetAsync(total, 0, 8, s); return 0; }
    hipLaunchKernelGGL(k_tile_reduce<In>, dim3(static_cast<unsigned>(nt)), dim3(WG), 0, s, in, n, tileSums);
    hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(1024), 0, s, tileSums, nt, total);
    hipLaunchKernelGGL((k_tile_scan<In, Out>), dim3(static_cast<unsigned>(nt)), dim3(WG), 0, s, in, n, tileSums, out);
    return static_cast<int>(hipGetLastError());
}

// ------------------------------------------------------------------------------ seeds
__global__ void k_lookup(const int32_t* qpart, const int64_t* qvid, uint64_t n, const int32_t* vpart,
                         const int64_t* vid, uint64_t V, uint32_t* out) {
    uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int32_t p = qpart[i];
    int64_t v = qvid[i];
    uint64_t lo = 0, hi = V;
    while (lo < hi) {
        uint64_t mid = (lo + hi) >> 1;
        bool less = vpart[mid] < p || (vpart[mid] == p && vid[mid] < v);
        if (less) lo = mid + 1; else hi = mid;
    }
    out[i] = (lo < V && vpart[lo] == p && vid[lo] == v) ? static_cast<uint32_t>(lo) : kNoRow;
}

// ------------------------------------------------------------------------------ edge -> entry map
// Fills smap[p] = (entry - lo) for the edges base .. base + cnt - 1. estart is the exclusive
// prefix of entry degrees (non-decreasing, estart[nEnt] = E).
__device__ __forceinline__ uint64_t mapChunk(const uint64_t* estart, uint64_t nEnt, uint64_t base, uint32_t cnt,
                                             uint32_t* smap, uint64_t* sLo) {
    if (threadIdx.x == 0) {
        uint64_t lo = 0, hi = nEnt;                  // last entry with estart <= base
        while (hi - lo > 1) {
            uint64_t mid = (lo + hi) >> 1;
            if (estart[mid] <= base) lo = mid; else hi = mid;
        }
        *sLo = lo;
    }
    for (int p = threadIdx.x; p < TILE; p += WG) smap[p] = 0;
    __syncthreads();
    uint64_t lo = *sLo;
    for (uint64_t i = lo + 1 + threadIdx.x; i < nEnt; i += WG) {
        uint64_t e = estart[i];
        if (e >= base + cnt) break;
        atomicMax(&smap[e - base], static_cast<uint32_t>(i - lo));
    }
    __syncthreads();
    // inclusive max-scan over smap[0 .. TILE): blocked, 16 per thread
    uint32_t* my = smap + threadIdx.x * ITEMS;
    uint32_t run = 0;
#pragma unroll
    for (int k = 0; k < ITEMS; k++) { run = run > my[k] ? run : my[k]; my[k] = run; }
    __shared__ uint32_t wmax[NW];
    int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t x = run;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x = x > y ? x : y;
    }
    if (lane == 63) wmax[wid] = x;
    uint32_t prevLane = __shfl_up(x, 1, 64);
    __syncthreads();
    uint32_t carry = lane == 0 ? 0 : prevLane;
    for (int w = 0; w < wid; w++) carry = carry > wmax[w] ? carry : wmax[w];
#pragma unroll
    for (int k = 0; k < ITEMS; k++) my[k] = my[k] > carry ? my[k] : carry;
    __syncthreads();
    return lo;
}

// ------------------------------------------------------------------------------ intermediate hop
__global__ __launch_bounds__(WG) void k_expand_mark(const uint32_t* F, const uint64_t* estart, uint64_t nEnt,
                                                    uint64_t E, HopSlots hs, uint8_t* visited, uint8_t epoch) {
    __shared__ uint32_t smap[TILE];
    __shared__ uint64_t sLo;
    uint64_t base = static_cast<uint64_t>(blockIdx.x) * TILE;
    uint32_t cnt = static_cast<uint32_t>(E - base < TILE ? E - base : TILE);
    uint64_t lo = mapChunk(estart, nEnt, base, cnt, smap, &sLo);
#pragma unroll 4
    for (int k = 0; k < ITEMS; k++) {
        uint32_t p = threadIdx.x + k * WG;
        if (p >= cnt) break;
        uint64_t ent = lo + smap[p];
        int s = static_cast<int>(ent % hs.n);
        uint32_t r = F[ent / hs.n];
        uint64_t pos = hs.off[s][r] + (base + p - estart[ent]);
        uint32_t g = hs.dgid[s][pos];
        if (g != kNoRow && visited[g] != epoch) visited[g] = epoch;
    }
}

// ------------------------------------------------------------------------------ final hop
__device__ __forceinline__ void edgeCtxOf(const FinalArgs& a, uint64_t e, uint64_t ent, EdgeCtx& ec) {
    int s = static_cast<int>(ent % a.hs.n);
    uint32_t r = a.F[ent / a.hs.n];
    ec.slot = a.hs.slotIdx[s];
    ec.etype = a.hs.etype[s];
    ec.pos = a.hs.off[s][r] + (e - a.estart[ent]);
    ec.srow = r;
    ec.src = a.vid[r];
    ec.dst = a.hs.dst[s][ec.pos];
    ec.rank = a.hs.rank[s][ec.pos];
    uint32_t g = a.hs.dgid[s][ec.pos];
    ec.drow = (g != kNoRow && g >= a.gbase && g - a.gbase < a.V) ? static_cast<uint32_t>(g - a.gbase) : kNoRow;
}

// storage filter + TTL + graphd WHERE for one edge (QueryBaseProcessor.inl:520-602, GoExecutor.cpp:1277-1287)
__device__ __forceinline__ bool passes(const FinalArgs& a, const EdgeCtx& ec, int s) {
    uint32_t bit = 1u << s;
    bool withReader = (a.propsMask & bit) || a.ttlCol[s] >= 0;
    if (withReader) {
        const DSlot& ds = a.env.slots[ec.slot];
        uint8_t f = ds.hasFlags ? ds.eflags[ec.pos] : 0;
        if (!(f & EF_EMPTY_VALUE)) {
            if (f & EF_BAD_ROW) return false;
            if (a.ttlCol[s] >= 0) {                       // checkDataExpiredForTTL (CommonUtils.cpp:13-49)
                const DCol& c = a.env.cols[ds.colBase + a.ttlCol[s]];
                if (c.valid == nullptr || c.valid[ec.pos]) {
                    int64_t v = static_cast<const int64_t*>(c.data)[ec.pos];
                    if (a.now > v + a.ttlDur[s]) return false;
                }
            }
            if (a.P != nullptr && (a.propsMask & bit)) {
                Val v = vmEval(a.P, a.env, ec);
                if (v.t == V_ERR || !asBool(v)) return false;
            }
        }
    }
    if (a.W != nullptr) {
        Val v = vmEval(a.W, a.env, ec);
        if (v.t == V_ERR) { atomicOr(a.err, 1u); return false; }
        if (!asBool(v)) return false;
    }
    return true;
}

__global__ __launch_bounds__(WG) void k_final_eval(FinalArgs a) {
    __shared__ uint32_t smap[TILE];
    __shared__ uint64_t sLo;
    __shared__ uint64_t sm[NW + 1];
    uint64_t base = static_cast<uint64_t>(blockIdx.x) * TILE;
    uint32_t cnt = static_cast<uint32_t>(a.E - base < TILE ? a.E - base : TILE);
    uint64_t lo = mapChunk(a.estart, a.nEnt, base, cnt, smap, &sLo);
    int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint64_t mine = 0;
    for (int k = 0; k < ITEMS; k++) {
        uint32_t p = threadIdx.x + k * WG;
        bool pass = false;
        if (p < cnt) {
            uint64_t ent = lo + smap[p];
            EdgeCtx ec;
            edgeCtxOf(a, base + p, ent, ec);
            pass = passes(a, ec, static_cast<int>(ent % a.hs.n));
        }
        uint64_t ballot = __ballot(pass);
        if (lane == 0) a.mask[blockIdx.x * (TILE / 64) + k * NW + wid] = ballot;
        mine += pass ? 1 : 0;
    }
    uint64_t t = blockSum(mine, sm);
    if (threadIdx.x == 0) a.chunkCount[blockIdx.x] = static_cast<uint32_t>(t);
}

__global__ __launch_bounds__(WG) void k_final_emit(FinalArgs a, const uint64_t* chunkOff) {
    __shared__ uint32_t smap[TILE];
    __shared__ uint64_t sLo;
    __shared__ uint32_t wordPre[TILE / 64];
    __shared__ uint32_t sNone;
    uint64_t base = static_cast<uint64_t>(blockIdx.x) * TILE;
    uint32_t cnt = static_cast<uint32_t>(a.E - base < TILE ? a.E - base : TILE);
    const uint64_t* mask = a.mask + blockIdx.x * (TILE / 64);
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (int w = 0; w < TILE / 64; w++) { wordPre[w] = acc; acc += __popcll(mask[w]); }
        sNone = acc == 0 ? 1u : 0u;
    }
    __syncthreads();
    if (sNone) return;                                      // nothing passed in this chunk (uniform)
    uint64_t lo = mapChunk(a.estart, a.nEnt, base, cnt, smap, &sLo);
    int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint64_t outBase = chunkOff[blockIdx.x];
    for (int k = 0; k < ITEMS; k++) {
        uint32_t p = threadIdx.x + k * WG;
        int w = k * NW + wid;
        uint64_t word = mask[w];
        if (p >= cnt || !((word >> lane) & 1)) continue;
        uint64_t o = outBase + wordPre[w] + __popcll(word & ((1ULL << lane) - 1));
        uint64_t ent = lo + smap[p];
        EdgeCtx ec;
        edgeCtxOf(a, base + p, ent, ec);
        a.oSrc[o] = ec.src;
        a.oDst[o] = ec.dst;
        a.oRank[o] = ec.rank;
        a.oType[o] = ec.etype;
        if (a.oEntry) a.oEntry[o] = static_cast<uint32_t>(ent / a.hs.n);
        for (int y = 0; y < a.nY; y++) {
            OutCell c;
            const Insn* prog = a.yCode + a.yOff[y];
            if (a.ySlotType != nullptr && a.ySlotType[y] != 0 && a.ySlotType[y] != ec.etype) {
                c.t = 0xFF; c.len = 0; c.x = 0;              // column of another edge type (GetNeighbors)
            } else {
                Val v = vmEval(prog, a.env, ec);
                if (v.t == V_ERR) atomicOr(a.err, 1u);
                c.t = v.t; c.len = v.len; c.x = v.x;
            }
            a.oCells[o * a.nY + y] = c;
        }
    }
}

// ------------------------------------------------------------------------------ vertex cells
__global__ void k_vertex_cells(VertexCellArgs a) {
    uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    uint32_t r = a.rows[i];
    for (int c = 0; c < a.ncols; c++) {
        OutCell out{0, 0, 0xFF};
        int tslot = a.tagSlot[c];
        if (tslot >= 0 && r != kNoRow) {
            const DTag& t = a.env.tags[tslot];
            if (t.present[r]) {
                const DCol& col = a.env.cols[t.colBase + a.col[c]];
                Val v = (col.valid != nullptr && col.valid[r] == 0) ? defaultOfType(col.type) : loadCol(col, r);
                out.t = v.t; out.len = v.len; out.x = v.x;
            }
        }
        a.out[i * a.ncols + c] = out;
    }
}

// ------------------------------------------------------------------------------ multi-GPU exchange
// pack this shard's marks for peer q's rows into a bitmap; merge received bitmaps into visited
__global__ void k_pack(const uint8_t* visited, uint8_t epoch, uint64_t lo, uint64_t n, uint64_t* bits) {
    uint64_t w = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (w * 64 >= n) return;
    uint64_t word = 0;
    for (int b = 0; b < 64; b++) {
        uint64_t i = w * 64 + b;
        if (i < n && visited[lo + i] == epoch) word |= 1ULL << b;
    }
    bits[w] = word;
}
__global__ void k_merge(const uint64_t* bits, uint64_t nwords, uint8_t* visited, uint64_t lo, uint64_t n, uint8_t epoch) {
    uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if ((bits[i >> 6] >> (i & 63)) & 1) visited[lo + i] = epoch;
    (void)nwords;
}

// ------------------------------------------------------------------------------ launchers
int launchLookup(const int32_t* qpart, const int64_t* qvid, uint64_t n, const int32_t* vpart, const int64_t* vid,
                 uint64_t V, uint32_t* out, hipStream_t s) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_lookup, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, s, qpart, qvid, n, vpart, vid, V, out);
    return static_cast<int>(hipGetLastError());
}

int launchDegreeScan(const uint32_t* F, uint64_t nEnt, const HopSlots& hs, uint64_t* estart, uint64_t* tileSums,
                     hipStream_t s) {
    return scan3(DegreeIn{F, hs}, nEnt, WriteEstart{estart}, tileSums, estart + nEnt, s);
}

int launchExpandMark(const uint32_t* F, const uint64_t* estart, uint64_t nEnt, uint64_t E, const HopSlots& hs,
                     uint8_t* visited, uint8_t epoch, hipStream_t s) {
    if (E == 0) return 0;
    uint64_t chunks = (E + TILE - 1) / TILE;
    hipLaunchKernelGGL(k_expand_mark, dim3(static_cast<unsigned>(chunks)), dim3(WG), 0, s, F, estart, nEnt, E, hs, visited, epoch);
    return static_cast<int>(hipGetLastError());
}

int launchCompact(const uint8_t* visited, uint64_t gbase, uint64_t V, uint8_t epoch, uint32_t* outF, uint64_t* tileSums,
                  uint64_t* count, hipStream_t s) {
    return scan3(FlagIn{visited, gbase, epoch}, V, WriteCompact{outF}, tileSums, count, s);
}

int launchFinal(const FinalArgs& a, uint64_t* chunkOff, uint64_t* tileSums, uint64_t* total, hipStream_t s) {
    if (a.E == 0) { (void)hipMemsetAsync(total, 0, 8, s); return 0; }
    uint64_t chunks = (a.E + TILE - 1) / TILE;
    hipLaunchKernelGGL(k_final_eval, dim3(static_cast<unsigned>(chunks)), dim3(WG), 0, s, a);
    int rc = scan3(CountIn{a.chunkCount}, chunks, WriteEstart{chunkOff}, tileSums, total, s);
    if (rc) return rc;
    return static_cast<int>(hipGetLastError());
}

int launchEmit(const FinalArgs& a, const uint64_t* chunkOff, hipStream_t s) {
    if (a.E == 0) return 0;
    uint64_t chunks = (a.E + TILE - 1) / TILE;
    hipLaunchKernelGGL(k_final_emit, dim3(static_cast<unsigned>(chunks)), dim3(WG), 0, s, a, chunkOff);
    return static_cast<int>(hipGetLastError());
}

int launchVertexCells(const VertexCellArgs& a, hipStream_t s) {
    if (a.n == 0) return 0;
    hipLaunchKernelGGL(k_vertex_cells, dim3(static_cast<unsigned>((a.n + 255) / 256)), dim3(256), 0, s, a);
    return static_cast<int>(hipGetLastError());
}

int launchPack(const uint8_t* visited, uint8_t epoch, uint64_t lo, uint64_t n, uint64_t* bits, hipStream_t s) {
    uint64_t words = (n + 63) / 64;
    if (words == 0) return 0;
    hipLaunchKernelGGL(k_pack, dim3(static_cast<unsigned>((words + 255) / 256)), dim3(256), 0, s, visited, epoch, lo, n, bits);
    return static_cast<int>(hipGetLastError());
}

int launchMerge(const uint64_t* bits, uint64_t n, uint8_t* visited, uint64_t lo, uint8_t epoch, hipStream_t s) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_merge, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, s, bits, (n + 63) / 64, visited, lo, n, epoch);
    return static_cast<int>(hipGetLastError());
}

}  // namespace ngx
