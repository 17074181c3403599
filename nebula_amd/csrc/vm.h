// Device bytecode VM: evaluates one compiled WHERE / YIELD program (exprc.cpp) for one edge,
// restating the reference evaluation rules exactly (src/common/filter/Expressions.cpp:662-1228,
// FunctionManager.cpp:20-555): no short circuit, error propagation left-first, implicit casts
// bool < int < double, |l - r| < 1e-8 double equality, int64 overflow and division errors.
//
// Each operation is a __forceinline__ helper with the opcode as an argument, shared by the
// interpreter below (vmEval, kernels.hip) and by the straight-line evaluators jit.cpp generates per
// query (compiled with hipRTC): there the opcodes and column types are literals and the type
// dispatch folds away.
#pragma once

#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#include <cmath>
#endif

#include "ngx_device.h"

namespace ngx {

struct Val {
    int64_t x;      // int / double bits / bool / string pointer
    uint32_t len;   // string length
    uint8_t t;      // V_*
};

struct EdgeCtx {
    int32_t slot;
    int32_t etype;
    const DCol* cols;   // first column of the slot's edge schema
    uint64_t pos;       // edge index inside the slot arrays
    uint32_t srow;      // local row of the source vertex
    uint32_t drow;      // global row of the destination (kNoRow: no vertex row on any shard)
    int64_t src, dst, rank;
};

struct VmEnv {
    const DSlot* slots;
    const DTag* tags;
    const DCol* cols;
    const char* pool;
    uint32_t* unsupported;     // set when a value needs a host-only construct
    int64_t now;               // WallClock::fastNowInSec of the request (TTL)
    const DTag* dtags;         // $$ props: tag tables over GLOBAL rows (world 1: the shard's own tables;
    const DCol* dcols;         // world > 1: replicas of every shard's rows, built on first use)
};

// Loads through the global address space. Column pointers come from device-side tables (DCol, DTag),
// which the compiler cannot prove global, so plain dereferences become flat loads (ordered with LDS
// traffic: every wait on them also waits on lgkmcnt).
template <typename T>
__device__ __forceinline__ T gld(const void* p, uint64_t i) {
    return ((const __attribute__((address_space(1))) T*)p)[i];
}

template <typename T>
__device__ __forceinline__ void gst(void* p, uint64_t i, T v) {
    ((__attribute__((address_space(1))) T*)p)[i] = v;
}

// element i of an integer array stored at its narrowest signed width w (1, 2, 4 or 8 bytes)
__device__ __forceinline__ int64_t loadW(const void* p, int32_t w, uint64_t i) {
    switch (w) {
        case 1: return gld<int8_t>(p, i);
        case 2: return gld<int16_t>(p, i);
        case 4: return gld<int32_t>(p, i);
        default: return gld<int64_t>(p, i);
    }
}
template <int W>                        // width known at compile time (generated kernels); 0: runtime w
__device__ __forceinline__ int64_t loadWT(const void* p, int32_t w, uint64_t i) {
    if constexpr (W == 1) return gld<int8_t>(p, i);
    else if constexpr (W == 2) return gld<int16_t>(p, i);
    else if constexpr (W == 4) return gld<int32_t>(p, i);
    else if constexpr (W == 8) return gld<int64_t>(p, i);
    else return loadW(p, w, i);
}

__device__ __forceinline__ Val mkInt(int64_t v) { return Val{v, 0, V_INT}; }
__device__ __forceinline__ Val mkBool(bool v) { return Val{v ? 1 : 0, 0, V_BOOL}; }
__device__ __forceinline__ Val mkDbl(double d) { return Val{__double_as_longlong(d), 0, V_DBL}; }
__device__ __forceinline__ Val mkErr() { return Val{0, 0, V_ERR}; }
__device__ __forceinline__ double dblOf(const Val& v) { return __longlong_as_double(v.x); }

// Expression::asBool (Expressions.h:284-298): string -> empty()
__device__ __forceinline__ bool asBool(const Val& v) {
    switch (v.t) {
        case V_INT: return v.x != 0;
        case V_DBL: return dblOf(v) != 0.0;
        case V_BOOL: return v.x != 0;
        case V_STR: return v.len == 0;
        default: return false;
    }
}
__device__ __forceinline__ double asDouble(const Val& v) {
    return v.t == V_INT ? static_cast<double>(v.x) : dblOf(v);
}
// Expression::toInt / toDouble for non-string values
__device__ __forceinline__ int64_t toInt(const Val& v) {
    if (v.t == V_INT) return v.x;
    if (v.t == V_BOOL) return v.x ? 1 : 0;
    double d = dblOf(v);
    if (!(d > -9223372036854775809.0 && d < 9223372036854775808.0)) return INT64_MIN;
    return static_cast<int64_t>(d);
}
__device__ __forceinline__ double toDouble(const Val& v) {
    if (v.t == V_INT) return static_cast<double>(v.x);
    if (v.t == V_BOOL) return v.x ? 1.0 : 0.0;
    return dblOf(v);
}

__device__ __forceinline__ int strCmp(const Val& a, const Val& b) {
    const unsigned char* p = reinterpret_cast<const unsigned char*>(a.x);
    const unsigned char* q = reinterpret_cast<const unsigned char*>(b.x);
    uint32_t n = a.len < b.len ? a.len : b.len;
    for (uint32_t i = 0; i < n; i++) {
        if (p[i] != q[i]) return p[i] < q[i] ? -1 : 1;
    }
    return a.len < b.len ? -1 : (a.len > b.len ? 1 : 0);
}
__device__ __forceinline__ bool strContains(const Val& a, const Val& b) {
    const char* p = reinterpret_cast<const char*>(a.x);
    const char* q = reinterpret_cast<const char*>(b.x);
    if (b.len == 0) return true;
    if (b.len > a.len) return false;
    for (uint32_t i = 0; i + b.len <= a.len; i++) {
        uint32_t j = 0;
        while (j < b.len && p[i + j] == q[j]) j++;
        if (j == b.len) return true;
    }
    return false;
}

// libstdc++ std::_Hash_bytes (64-bit), seed 0xc70f6907 (std::hash<std::string>, std::hash<double>)
__device__ __forceinline__ uint64_t hashBytes(const unsigned char* p, uint64_t n) {
    const uint64_t mul = (0xc6a4a793ULL << 32) + 0x5bd1e995ULL;
    uint64_t h = 0xc70f6907ULL ^ (n * mul);
    uint64_t aligned = n & ~7ULL;
    for (uint64_t i = 0; i < aligned; i += 8) {
        uint64_t d = 0;
        for (int k = 7; k >= 0; k--) d = (d << 8) | p[i + k];
        d *= mul;
        d ^= d >> 47;
        d *= mul;
        h ^= d;
        h *= mul;
    }
    if (n & 7) {
        uint64_t d = 0;
        for (int64_t k = static_cast<int64_t>(n & 7) - 1; k >= 0; k--) d = (d << 8) | p[aligned + k];
        h ^= d;
        h *= mul;
    }
    h ^= h >> 47;
    h *= mul;
    h ^= h >> 47;
    return h;
}

// integer column element: the column is stored at the narrowest signed width holding all its values
// (export-time choice, uniform per column, so the branch is scalar)
__device__ __forceinline__ int64_t loadI64(const DCol& c, uint64_t i) {
    switch (c.width) {
        case 1: return gld<int8_t>(c.data, i);
        case 2: return gld<int16_t>(c.data, i);
        case 4: return gld<int32_t>(c.data, i);
        default: return gld<int64_t>(c.data, i);
    }
}
__device__ __forceinline__ Val loadCol(const DCol& c, uint64_t i) {
    switch (c.type) {
        case 2: case 21: case 3: return mkInt(loadI64(c, i));
        case 4: case 5: return mkDbl(gld<double>(c.data, i));
        case 1: return mkBool(gld<uint8_t>(c.data, i) != 0);
        case 6: {
            uint64_t o = gld<uint64_t>(c.soff, i);
            return Val{reinterpret_cast<int64_t>(c.sbytes + o), static_cast<uint32_t>(gld<uint64_t>(c.soff, i + 1) - o), V_STR};
        }
        default: return mkErr();
    }
}
__device__ __forceinline__ Val defaultOfType(int32_t t) {
    switch (t) {
        case 1: return mkBool(false);
        case 4: case 5: return mkDbl(0.0);
        case 6: return Val{0, 0, V_STR};
        default: return mkInt(0);
    }
}
__device__ __forceinline__ Val constVal(uint8_t t, int64_t bits, uint32_t len, const char* pool) {
    if (t == V_STR) return Val{reinterpret_cast<int64_t>(pool + bits), len, V_STR};
    return Val{bits, 0, t};
}

__device__ __forceinline__ bool mulOverflow(int64_t lv, int64_t rv) {    // Expressions.cpp:862-874
    const int64_t maxInt = INT64_MAX, minInt = INT64_MIN;
    if (lv > 0 && rv > 0) return maxInt / lv < rv;
    if (lv < 0 && rv < 0) return maxInt / lv > rv;
    if (lv > 0 && rv < 0) return minInt / lv > rv;
    if (lv < 0 && rv > 0) return minInt / rv > lv;
    return false;
}

// ------------------------------------------------------------------------------ loads
template <int W>                        // integer storage width known at compile time (JIT); 0: read c.width
__device__ __forceinline__ int64_t loadI64T(const DCol& c, uint64_t i) {
    if constexpr (W == 1) return gld<int8_t>(c.data, i);
    else if constexpr (W == 2) return gld<int16_t>(c.data, i);
    else if constexpr (W == 4) return gld<int32_t>(c.data, i);
    else if constexpr (W == 8) return gld<int64_t>(c.data, i);
    else return loadI64(c, i);
}
template <int CT, int W = 0>            // column type (and integer width) known at compile time (JIT)
__device__ __forceinline__ Val loadColT(const DCol& c, uint64_t i) {
    if constexpr (CT == 2 || CT == 21 || CT == 3) return mkInt(loadI64T<W>(c, i));
    else if constexpr (CT == 4 || CT == 5) return mkDbl(gld<double>(c.data, i));
    else if constexpr (CT == 1) return mkBool(gld<uint8_t>(c.data, i) != 0);
    else if constexpr (CT == 6) {
        uint64_t o = gld<uint64_t>(c.soff, i);
        return Val{reinterpret_cast<int64_t>(c.sbytes + o), static_cast<uint32_t>(gld<uint64_t>(c.soff, i + 1) - o), V_STR};
    } else return mkErr();
}
template <int CT>
__device__ __forceinline__ Val defaultOfTypeT() {
    if constexpr (CT == 1) return mkBool(false);
    else if constexpr (CT == 4 || CT == 5) return mkDbl(0.0);
    else if constexpr (CT == 6) return Val{0, 0, V_STR};
    else return mkInt(0);
}

// OP_ECOL: edge column a of |type| b; mode bit0 mismatch -> dflt, bit1 missing field -> type default
// VALID: the column may lack rows (a valid[] bitmap exists); false when the host knows every row of
// every slot has the field, which keeps the value's type a compile-time constant
template <int CT, int W = 0, bool VALID = true>
__device__ __forceinline__ Val opEcolT(const VmEnv& env, const EdgeCtx& ec, int32_t a, int32_t b, uint8_t mode, Val dflt) {
    int32_t at = ec.etype < 0 ? -ec.etype : ec.etype;
    if (at != b) return (mode & 1) ? dflt : mkErr();
    const DCol& c = ec.cols[a];
    if constexpr (VALID) {
        if (c.valid != nullptr && gld<uint8_t>(c.valid, ec.pos) == 0) return (mode & 2) ? defaultOfTypeT<CT>() : mkErr();
    }
    return loadColT<CT, W>(c, ec.pos);
}
__device__ __forceinline__ Val opEcol(const VmEnv& env, const EdgeCtx& ec, int32_t a, int32_t b, uint8_t mode, Val dflt) {
    int32_t at = ec.etype < 0 ? -ec.etype : ec.etype;
    if (at != b) return (mode & 1) ? dflt : mkErr();
    const DCol& c = ec.cols[a];
    if (c.valid != nullptr && gld<uint8_t>(c.valid, ec.pos) == 0) return (mode & 2) ? defaultOfType(c.type) : mkErr();
    return loadCol(c, ec.pos);
}
// OP_EKEY: key prop a (0 src, 1 dst, 2 rank, 3 type) of alias type b (0: any)
__device__ __forceinline__ Val opEkey(const EdgeCtx& ec, int32_t a, int32_t b, uint8_t mode, Val dflt) {
    int32_t at = ec.etype < 0 ? -ec.etype : ec.etype;
    if (b != 0 && at != b) return (mode & 1) ? dflt : mkErr();
    return mkInt(a == 0 ? ec.src : a == 1 ? ec.dst : a == 2 ? ec.rank : static_cast<int64_t>(ec.etype));
}
__device__ __forceinline__ Val opEdst(const EdgeCtx& ec, int32_t b) {
    int32_t at = ec.etype < 0 ? -ec.etype : ec.etype;
    return mkInt((b != 0 && at != b) ? 0 : ec.dst);
}
// no tag row for the vertex, or its TTL expired: collectVertexProps collects nothing for the tag
// (QueryBaseProcessor.inl:440-476; checkDataExpiredForTTL, CommonUtils.cpp:13-49: an unreadable TTL
// field never expires)
__device__ __forceinline__ bool tagAbsentIn(const VmEnv& env, const DCol* cols, const DTag& t, uint32_t row) {
    if (row == kNoRow || gld<uint8_t>(t.present, row) == 0) return true;
    if (t.ttlCol < 0) return false;
    const DCol& c = cols[t.colBase + t.ttlCol];
    if (c.valid != nullptr && gld<uint8_t>(c.valid, row) == 0) return false;
    return env.now > loadI64(c, row) + t.ttlDur;
}

__device__ __forceinline__ bool tagAbsent(const VmEnv& env, const DTag& t, uint32_t row) {
    return tagAbsentIn(env, env.cols, t, row);
}

// OP_SRCTAG / OP_DSTTAG: column a of tag slot b for the src row (the shard's tables, local row) or
// the dst row (DST: env.dtags / dcols, global row)
template <int CT, int W = 0, bool VALID = true, bool DST = false>
__device__ __forceinline__ Val opTagT(const VmEnv& env, uint32_t row, int32_t a, int32_t b, uint8_t mode, Val dflt) {
    const DCol* cols = DST ? env.dcols : env.cols;
    const DTag& t = (DST ? env.dtags : env.tags)[b];
    if (tagAbsentIn(env, cols, t, row)) return (mode & 1) ? dflt : mkErr();
    const DCol& c = cols[t.colBase + a];
    if constexpr (VALID) {
        if (c.valid != nullptr && gld<uint8_t>(c.valid, row) == 0) return defaultOfTypeT<CT>();
    }
    return loadColT<CT, W>(c, row);
}
__device__ __forceinline__ Val opTag(const VmEnv& env, uint32_t row, int32_t a, int32_t b, uint8_t mode, Val dflt,
                                     bool dst = false) {
    const DCol* cols = dst ? env.dcols : env.cols;
    const DTag& t = (dst ? env.dtags : env.tags)[b];
    if (tagAbsentIn(env, cols, t, row)) return (mode & 1) ? dflt : mkErr();
    const DCol& c = cols[t.colBase + a];
    if (c.valid != nullptr && gld<uint8_t>(c.valid, row) == 0) return defaultOfType(c.type);
    return loadCol(c, row);
}

// ------------------------------------------------------------------------------ unary / cast
__device__ __forceinline__ Val opNeg(Val v) {              // UnaryExpression NEGATE
    if (v.t == V_INT) { v.x = static_cast<int64_t>(0ULL - static_cast<uint64_t>(v.x)); return v; }
    if (v.t == V_DBL) return mkDbl(-dblOf(v));
    return mkErr();
}
__device__ __forceinline__ Val opNot(Val v) { return v.t == V_ERR ? v : mkBool(!asBool(v)); }
// TypeCastingExpression::eval; t1 = ColumnType (INT 0, STRING 1, DOUBLE 2, BOOL 3, TIMESTAMP 4)
__device__ __forceinline__ Val opCast(Val v, uint8_t t1, const VmEnv& env) {
    if (v.t == V_ERR) return v;
    if (v.t == V_STR) {                                    // folly::to<int/double>(string): host only
        if (t1 != 3) { atomicOr(env.unsupported, 1u); return mkErr(); }
        return mkBool(asBool(v));
    }
    if (t1 == 0 || t1 == 4) return mkInt(toInt(v));
    if (t1 == 2) return mkDbl(toDouble(v));
    return mkBool(asBool(v));
}

// (string) cast, Expression::toString (Expressions.h:334-348), into a 24-byte buffer of the
// evaluation (the caller's private memory: a WHERE / pushed filter consumes the string before the
// program returns; a YIELD whose value is such a string is refused at compile time). int64 prints as
// folly::to<std::string> (decimal, '-' sign), bool as "true" / "false"; a double needs folly's
// shortest round-trip form: host only.
__device__ __forceinline__ Val castToString(Val v, char* buf, const VmEnv& env) {
    if (v.t == V_ERR || v.t == V_STR) return v;
    uint32_t n = 0;
    if (v.t == V_BOOL) {
        const char* w = v.x ? "true" : "false";
        for (; w[n]; n++) buf[n] = w[n];
    } else if (v.t == V_INT) {
        uint64_t u = v.x < 0 ? 0ULL - static_cast<uint64_t>(v.x) : static_cast<uint64_t>(v.x);
        uint32_t digits = 1;
        for (uint64_t t = u; t >= 10; t /= 10) digits++;
        if (v.x < 0) buf[n++] = '-';
        for (uint32_t k = digits; k > 0; k--) {
            buf[n + k - 1] = static_cast<char>('0' + u % 10);
            u /= 10;
        }
        n += digits;
    } else {
        atomicOr(env.unsupported, 1u);
        return mkErr();
    }
    return Val{reinterpret_cast<int64_t>(buf), n, V_STR};
}

// ------------------------------------------------------------------------------ arithmetic
__device__ __forceinline__ Val opArith(uint8_t op, Val l, Val r, const VmEnv& env) {
    if (l.t == V_ERR) return l;
    if (r.t == V_ERR) return r;
    if ((l.t == V_INT || l.t == V_DBL) && (r.t == V_INT || r.t == V_DBL)) {
        if (l.t == V_DBL || r.t == V_DBL) {
            double a = asDouble(l), b = asDouble(r);
            switch (op) {
                case OP_ADD: return mkDbl(a + b);
                case OP_SUB: return mkDbl(a - b);
                case OP_MUL: return mkDbl(a * b);
                case OP_DIV: return fabs(b) < 1e-8 ? mkErr() : mkDbl(a / b);
                case OP_MOD: return fabs(b) < 1e-8 ? mkErr() : mkDbl(fmod(a, b));
                default: return mkInt(static_cast<int64_t>(round(a)) ^ static_cast<int64_t>(round(b)));
            }
        }
        int64_t a = l.x, b = r.x;
        switch (op) {
            case OP_ADD: {
                bool of = (a >= 0 && b >= 0) ? (INT64_MAX - a < b) : (a < 0 && b < 0) ? (INT64_MIN - a > b) : false;
                return of ? mkErr() : mkInt(a + b);
            }
            case OP_SUB: {
                bool of = (a > 0 && b < 0) ? (b == INT64_MIN || INT64_MAX - a < -b)
                        : (a < 0 && b > 0) ? (INT64_MIN - a > -b) : false;
                return of ? mkErr() : mkInt(a - b);
            }
            case OP_MUL:
                return mulOverflow(a, b) ? mkErr()
                     : mkInt(static_cast<int64_t>(static_cast<uint64_t>(a) * static_cast<uint64_t>(b)));
            case OP_DIV: return (b == 0 || (a == INT64_MIN && b == -1)) ? mkErr() : mkInt(a / b);
            case OP_MOD: return b == 0 ? mkErr() : (b == -1 ? mkInt(0) : mkInt(a % b));
            default: return mkInt(a ^ b);
        }
    }
    if (op == OP_ADD && l.t == V_STR && r.t == V_STR) atomicOr(env.unsupported, 1u);   // builds a string
    return mkErr();
}

// ------------------------------------------------------------------------------ relational / logical
__device__ __forceinline__ Val opRel(uint8_t op, Val l, Val r) {
    if (l.t == V_ERR) return l;
    if (r.t == V_ERR) return r;
    if (op == OP_CONTAINS) return (l.t == V_STR && r.t == V_STR) ? mkBool(strContains(l, r)) : mkErr();
    if ((l.t == V_STR) != (r.t == V_STR)) return mkErr();  // string vs non-string
    int c;                                                 // -1 / 0 / 1, 2 = unordered (NaN)
    bool eqOnly = false, eqv = false;
    if (l.t == V_STR) {
        c = strCmp(l, r);
    } else if (l.t == V_DBL || r.t == V_DBL) {
        double a = toDouble(l), b = toDouble(r);
        c = a < b ? -1 : (a > b ? 1 : (a == b ? 0 : 2));
        if (op == OP_EQ || op == OP_NE) { eqOnly = true; eqv = fabs(a - b) < 1e-8; }
    } else if (l.t == V_INT || r.t == V_INT) {
        int64_t a = toInt(l), b = toInt(r);
        c = a < b ? -1 : (a > b ? 1 : 0);
    } else {                                               // bool vs bool
        c = l.x < r.x ? -1 : (l.x > r.x ? 1 : 0);
    }
    switch (op) {
        case OP_LT: return mkBool(c == -1);
        case OP_LE: return mkBool(c == -1 || c == 0);
        case OP_GT: return mkBool(c == 1);
        case OP_GE: return mkBool(c == 1 || c == 0);
        case OP_EQ: return mkBool(eqOnly ? eqv : c == 0);
        default: return mkBool(eqOnly ? !eqv : c != 0);
    }
}
__device__ __forceinline__ Val opLogic(uint8_t op, Val l, Val r) {
    if (l.t == V_ERR) return l;
    if (r.t == V_ERR) return r;
    bool a = asBool(l), b = asBool(r);
    return mkBool(op == OP_AND ? (a && b) : op == OP_OR ? (a || b) : (a != b));
}

// ------------------------------------------------------------------------------ functions
__device__ __forceinline__ Val opFunc(int32_t fid, const Val* args, int argc, const VmEnv& env) {
    for (int k = 0; k < argc; k++) if (args[k].t == V_ERR) return args[k];
    bool num1 = args[0].t == V_INT || args[0].t == V_DBL;
    switch (fid) {
        case F_ABS: return num1 ? mkDbl(fabs(asDouble(args[0]))) : mkErr();
        case F_FLOOR: return num1 ? mkDbl(floor(asDouble(args[0]))) : mkErr();
        case F_CEIL: return num1 ? mkDbl(ceil(asDouble(args[0]))) : mkErr();
        case F_ROUND: return num1 ? mkDbl(round(asDouble(args[0]))) : mkErr();
        case F_SQRT: return num1 ? mkDbl(sqrt(asDouble(args[0]))) : mkErr();
        case F_CBRT: return num1 ? mkDbl(cbrt(asDouble(args[0]))) : mkErr();
        case F_EXP: return num1 ? mkDbl(exp(asDouble(args[0]))) : mkErr();
        case F_EXP2: return num1 ? mkDbl(exp2(asDouble(args[0]))) : mkErr();
        case F_LOG: return num1 ? mkDbl(log(asDouble(args[0]))) : mkErr();
        case F_LOG2: return num1 ? mkDbl(log2(asDouble(args[0]))) : mkErr();
        case F_LOG10: return num1 ? mkDbl(log10(asDouble(args[0]))) : mkErr();
        case F_SIN: return num1 ? mkDbl(sin(asDouble(args[0]))) : mkErr();
        case F_ASIN: return num1 ? mkDbl(asin(asDouble(args[0]))) : mkErr();
        case F_COS: return num1 ? mkDbl(cos(asDouble(args[0]))) : mkErr();
        case F_ACOS: return num1 ? mkDbl(acos(asDouble(args[0]))) : mkErr();
        case F_TAN: return num1 ? mkDbl(tan(asDouble(args[0]))) : mkErr();
        case F_ATAN: return num1 ? mkDbl(atan(asDouble(args[0]))) : mkErr();
        case F_HYPOT: case F_POW: {
            bool num2 = args[1].t == V_INT || args[1].t == V_DBL;
            if (!(num1 && num2)) return mkErr();
            double a = asDouble(args[0]), b = asDouble(args[1]);
            return mkDbl(fid == F_HYPOT ? hypot(a, b) : pow(a, b));
        }
        case F_LENGTH: return args[0].t == V_STR ? mkInt(args[0].len) : mkErr();
        case F_STRCASECMP: {
            if (!(args[0].t == V_STR && args[1].t == V_STR)) return mkErr();
            const unsigned char* p = reinterpret_cast<const unsigned char*>(args[0].x);     // C strings: stop at NUL
            const unsigned char* q = reinterpret_cast<const unsigned char*>(args[1].x);
            for (uint32_t k = 0;; k++) {
                int c1 = k < args[0].len ? p[k] : 0;
                int c2 = k < args[1].len ? q[k] : 0;
                if (c1 >= 'A' && c1 <= 'Z') c1 += 32;
                if (c2 >= 'A' && c2 <= 'Z') c2 += 32;
                if (c1 != c2 || c1 == 0) return mkInt(c1 - c2);
            }
        }
        case F_HASH: {
            const Val& a = args[0];
            if (a.t == V_INT || a.t == V_BOOL) return mkInt(a.x);
            if (a.t == V_DBL) {
                double d = dblOf(a);
                return mkInt(d != 0.0 ? static_cast<int64_t>(hashBytes(reinterpret_cast<const unsigned char*>(&d), 8)) : 0);
            }
            return mkInt(static_cast<int64_t>(hashBytes(reinterpret_cast<const unsigned char*>(a.x), a.len)));
        }
        case F_UDF_IS_IN: {                                // FunctionManager.cpp:467-513
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
            return mkBool(found);
        }
        default: return mkErr();
    }
}

// ------------------------------------------------------------------------------ interpreter
static __device__ __noinline__ Val vmEval(const Insn* code, const VmEnv& env, const EdgeCtx& ec) {
    Val st[kMaxStack];
    char sbuf[kMaxStrCasts][kStrCastBytes];
    int sp = 0, nsb = 0;
    for (int pc = 0;; pc++) {
        const Insn in = code[pc];
        switch (in.op) {
            case OP_END: return sp > 0 ? st[sp - 1] : mkErr();
            case OP_PUSH: st[sp++] = constVal(in.t1, in.imm, static_cast<uint32_t>(in.a), env.pool); break;
            case OP_ERR: st[sp++] = mkErr(); break;
            case OP_ECOL: st[sp++] = opEcol(env, ec, in.a, in.b, in.mode, constVal(in.t2, in.imm, 0, env.pool)); break;
            case OP_EKEY: st[sp++] = opEkey(ec, in.a, in.b, in.mode, constVal(in.t2, in.imm, 0, env.pool)); break;
            case OP_EDST: st[sp++] = opEdst(ec, in.b); break;
            case OP_SRCTAG: case OP_DSTTAG:
                st[sp++] = opTag(env, in.op == OP_SRCTAG ? ec.srow : ec.drow, in.a, in.b, in.mode,
                                 constVal(in.t2, in.imm, 0, env.pool), in.op == OP_DSTTAG);
                break;
            case OP_PLUS: break;
            case OP_NEG: st[sp - 1] = opNeg(st[sp - 1]); break;
            case OP_NOT: st[sp - 1] = opNot(st[sp - 1]); break;
            case OP_CAST:
                if (in.t1 == 1) st[sp - 1] = nsb < kMaxStrCasts ? castToString(st[sp - 1], sbuf[nsb++], env) : mkErr();
                else st[sp - 1] = opCast(st[sp - 1], in.t1, env);
                break;
            case OP_ADD: case OP_SUB: case OP_MUL: case OP_DIV: case OP_MOD: case OP_AXOR:
                sp--; st[sp - 1] = opArith(in.op, st[sp - 1], st[sp], env); break;
            case OP_LT: case OP_LE: case OP_GT: case OP_GE: case OP_EQ: case OP_NE: case OP_CONTAINS:
                sp--; st[sp - 1] = opRel(in.op, st[sp - 1], st[sp]); break;
            case OP_AND: case OP_OR: case OP_LXOR:
                sp--; st[sp - 1] = opLogic(in.op, st[sp - 1], st[sp]); break;
            case OP_FUNC: {
                int argc = in.b;
                Val out = opFunc(in.a, &st[sp - argc], argc, env);
                sp -= argc;
                st[sp++] = out;
                break;
            }
            default: return mkErr();
        }
    }
}

}  // namespace ngx
