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
#include "dtoa.h"

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
    uint32_t in;        // input row of the edge's frontier entry (multi-root pipe walks; 0 otherwise)
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
    const DInputCol* input;    // the pipe's input columns (OP_INPUT), nullptr when none
};

// Loads through the global address space. Column pointers come from device-side tables (DCol, DTag),
// which the compiler cannot prove global, so plain dereferences become flat loads (ordered with LDS
// traffic: every wait on them also waits on lgkmcnt). NGX_GLD_NT (a generated kernel's own #define, flag
// final_nt_loads): non-temporal loads, each line read once and not kept in L2.
template <typename T>
__device__ __forceinline__ T gld(const void* p, uint64_t i) {
#ifdef NGX_GLD_NT
    return __builtin_nontemporal_load(&((const __attribute__((address_space(1))) T*)p)[i]);
#else
    return ((const __attribute__((address_space(1))) T*)p)[i];
#endif
}

template <typename T>
__device__ __forceinline__ void gst(void* p, uint64_t i, T v) {
    ((__attribute__((address_space(1))) T*)p)[i] = v;
}
// a non-temporal (streaming) store: the line is not kept in L2 for reuse
template <typename T>
__device__ __forceinline__ void gstNT(void* p, uint64_t i, T v) {
    __builtin_nontemporal_store(v, &((__attribute__((address_space(1))) T*)p)[i]);
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

// element i of an integer result array at width w (1, 2 or 4 bytes, two's complement; else 8): compact
// device results (ngx_go_plan::compact_results) hold each integer column at the width of the stored
// column it copies, so the store keeps every bit of the value
__device__ __forceinline__ void storeW(void* p, int32_t w, uint64_t i, int64_t v) {
    switch (w) {
        case 1: gst<int8_t>(p, i, static_cast<int8_t>(v)); break;
        case 2: gst<int16_t>(p, i, static_cast<int16_t>(v)); break;
        case 4: gst<int32_t>(p, i, static_cast<int32_t>(v)); break;
        default: gst<int64_t>(p, i, v); break;
    }
}
template <int W, bool NT = false>      // width known at compile time (generated kernels); 0: runtime w
__device__ __forceinline__ void storeWT(void* p, int32_t w, uint64_t i, int64_t v) {
    if constexpr (NT && W == 1) gstNT<int8_t>(p, i, static_cast<int8_t>(v));
    else if constexpr (NT && W == 2) gstNT<int16_t>(p, i, static_cast<int16_t>(v));
    else if constexpr (NT && W == 4) gstNT<int32_t>(p, i, static_cast<int32_t>(v));
    else if constexpr (NT && W == 8) gstNT<int64_t>(p, i, v);
    else if constexpr (W == 1) gst<int8_t>(p, i, static_cast<int8_t>(v));
    else if constexpr (W == 2) gst<int16_t>(p, i, static_cast<int16_t>(v));
    else if constexpr (W == 4) gst<int32_t>(p, i, static_cast<int32_t>(v));
    else if constexpr (W == 8) gst<int64_t>(p, i, v);
    else storeW(p, w, i, v);
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
// ------------------------------------------------------------------------------ strings
// Strings are (pointer, length) views: into a column's bytes, the program's literal pool, or one
// kStrBuildBytes buffer of the evaluation that a builder (lower, upper, lpad, rpad, string +,
// (string)) wrote (the compiler gives every builder its own buffer, Insn::mode). A result longer
// than a buffer is a host-only construct (env.unsupported: the query returns NGX_E_UNSUPPORTED and
// the caller runs its CPU path), never a truncated string. Bytes are read through flat pointers, so a
// view of a private buffer reads like one of a column.
__device__ __forceinline__ Val mkStr(const char* p, uint32_t n) { return Val{reinterpret_cast<int64_t>(p), n, V_STR}; }
__device__ __forceinline__ const char* strPtr(const Val& v) { return reinterpret_cast<const char*>(v.x); }
__device__ __forceinline__ Val hostOnly(const VmEnv& env) { atomicOr(env.unsupported, 1u); return mkErr(); }
__device__ __forceinline__ bool isSpaceC(char c) { return c == ' ' || (c >= '\t' && c <= '\r'); }
__device__ __forceinline__ bool isDigitC(char c) { return c >= '0' && c <= '9'; }

// folly::to<int64_t>(string) as the oracle restates it (orc_expr.cpp toInt: strtoll base 10, the
// whole C string consumed, no ERANGE): leading white space, one sign, digits, then the end or a NUL
__device__ __forceinline__ Val strToInt(const Val& v) {
    const char* p = strPtr(v);
    const uint32_t n = v.len;
    uint32_t k = 0;
    while (k < n && isSpaceC(p[k])) k++;
    bool neg = false;
    if (k < n && (p[k] == '+' || p[k] == '-')) neg = p[k++] == '-';
    if (k >= n || !isDigitC(p[k])) return mkErr();
    const uint64_t limit = neg ? (1ULL << 63) : (1ULL << 63) - 1;
    uint64_t acc = 0;
    bool range = false;
    for (; k < n && isDigitC(p[k]); k++) {
        const uint64_t d = static_cast<uint64_t>(p[k] - '0');
        if (acc > (limit - d) / 10) range = true;
        else acc = acc * 10 + d;
    }
    if (range || (k < n && p[k] != '\0')) return mkErr();
    return mkInt(neg ? static_cast<int64_t>(0ULL - acc) : static_cast<int64_t>(acc));
}

// folly::to<double>(string) (orc_expr.cpp toDouble: strtod, the whole C string consumed) for the
// decimal forms strtod rounds with one IEEE operation (Clinger's fast path: at most 19 significant
// digits, a mantissa <= 2^53 and a power of ten <= 1e22, all exact as doubles; or an integer mantissa
// of up to 19 digits, converted once). Hex floats, inf / nan,
// longer mantissas and larger exponents need strtod's big-number rounding: host-only constructs.
__device__ __forceinline__ Val strToDouble(const Val& v, const VmEnv& env) {
    const char* p = strPtr(v);
    const uint32_t n = v.len;
    uint32_t k = 0;
    while (k < n && isSpaceC(p[k])) k++;
    bool neg = false;
    if (k < n && (p[k] == '+' || p[k] == '-')) neg = p[k++] == '-';
    if (k < n && !isDigitC(p[k]) && p[k] != '.') {
        const char c = p[k] | 0x20;
        return (c == 'i' || c == 'n') ? hostOnly(env) : mkErr();        // inf / nan: strtod's spellings
    }
    uint64_t m = 0;
    int sig = 0, exp10 = 0;
    bool digits = false;
    if (k + 1 < n && p[k] == '0' && (p[k + 1] | 0x20) == 'x') return hostOnly(env);
    for (; k < n && isDigitC(p[k]); k++) {
        digits = true;
        if (m == 0 && p[k] == '0') continue;
        if (sig < 19) { m = m * 10 + static_cast<uint64_t>(p[k] - '0'); sig++; }
        else { if (p[k] != '0') return hostOnly(env); exp10++; }
    }
    if (k < n && p[k] == '.') {
        k++;
        for (; k < n && isDigitC(p[k]); k++) {
            digits = true;
            if (m == 0 && p[k] == '0') { exp10--; continue; }
            if (sig < 19) { m = m * 10 + static_cast<uint64_t>(p[k] - '0'); sig++; exp10--; }
            else if (p[k] != '0') return hostOnly(env);
        }
    }
    if (!digits) return mkErr();
    if (k < n && (p[k] | 0x20) == 'e') {                 // an exponent only with at least one digit
        uint32_t j = k + 1;
        bool eneg = false;
        if (j < n && (p[j] == '+' || p[j] == '-')) eneg = p[j++] == '-';
        if (j < n && isDigitC(p[j])) {
            int64_t e = 0;
            for (; j < n && isDigitC(p[j]); j++) if (e < 100000) e = e * 10 + (p[j] - '0');
            exp10 += static_cast<int>(eneg ? -e : e);
            k = j;
        }
    }
    if (k < n && p[k] != '\0') return mkErr();
    double d;
    if (m == 0) {
        d = 0.0;
    } else if (exp10 == 0) {
        d = static_cast<double>(m);                     // one correctly rounded conversion
    } else {
        if (m > (1ULL << 53) || exp10 > 22 || exp10 < -22) return hostOnly(env);
        double pw = 1.0;
        for (int i = 0; i < (exp10 < 0 ? -exp10 : exp10); i++) pw *= 10.0;   // 10^k, k <= 22: exact
        d = exp10 < 0 ? static_cast<double>(m) / pw : static_cast<double>(m) * pw;
    }
    return mkDbl(neg ? -d : d);
}

// TypeCastingExpression::eval; t1 = ColumnType (INT 0, STRING 1, DOUBLE 2, BOOL 3, TIMESTAMP 4)
__device__ __forceinline__ Val opCast(Val v, uint8_t t1, const VmEnv& env) {
    if (v.t == V_ERR) return v;
    if (v.t == V_STR) {
        if (t1 == 0 || t1 == 4) return strToInt(v);
        if (t1 == 2) return strToDouble(v, env);
        return mkBool(asBool(v));
    }
    if (t1 == 0 || t1 == 4) return mkInt(toInt(v));
    if (t1 == 2) return mkDbl(toDouble(v));
    return mkBool(asBool(v));
}

// (string) cast, Expression::toString (Expressions.h:334-348), into the cast's builder buffer.
// int64 prints as folly::to<std::string> (decimal, '-' sign), bool as "true" / "false", a double in
// double-conversion's SHORTEST form (dtoa.h: exact shortest round-trip digits, formatted as
// orc_expr.cpp toString does).
__device__ __forceinline__ Val castToString(Val v, char* buf, const VmEnv& env) {
    if (v.t == V_ERR || v.t == V_STR) return v;
    if (buf == nullptr) return hostOnly(env);
    uint32_t n = 0;
    if (v.t == V_BOOL) {
        const char* w = v.x ? "true" : "false";
        for (; w[n]; n++) buf[n] = w[n];
    } else if (v.t == V_INT) {
        const bool neg = v.x < 0;
        uint64_t u = neg ? 0ULL - static_cast<uint64_t>(v.x) : static_cast<uint64_t>(v.x);
        uint32_t digits = 1;
        for (uint64_t t = u; t >= 10; t /= 10) digits++;
        if (neg) buf[n++] = '-';
        for (uint32_t k = digits; k > 0; k--) {
            buf[n + k - 1] = static_cast<char>('0' + u % 10);
            u /= 10;
        }
        n += digits;
    } else if (v.t == V_DBL) {
        n = static_cast<uint32_t>(dtoa::format(dblOf(v), buf));     // at most 25 bytes
    } else {
        return hostOnly(env);
    }
    return mkStr(buf, n);
}

// a YIELD value that is a view of the evaluation's builder buffers [lo, lo + bytes): copied to the
// row's slot of the result string arena (out), which outlives the evaluation
__device__ __forceinline__ Val copyOut(Val v, char* out, const char* lo, uint64_t bytes) {
    if (out == nullptr || v.t != V_STR || v.len == 0) return v;
    const uint64_t x = static_cast<uint64_t>(v.x), b = reinterpret_cast<uint64_t>(lo);
    if (x < b || x >= b + bytes) return v;
    const char* p = strPtr(v);
    for (uint32_t k = 0; k < v.len; k++) out[k] = p[k];
    v.x = reinterpret_cast<int64_t>(out);
    return v;
}

// ------------------------------------------------------------------------------ arithmetic
__device__ __forceinline__ Val opArith(uint8_t op, Val l, Val r, const VmEnv& env, char* buf = nullptr) {
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
    if (op == OP_ADD && l.t == V_STR && r.t == V_STR) {                // concatenation (Expressions.cpp:936)
        if (buf == nullptr || l.len + r.len > static_cast<uint32_t>(kStrBuildBytes)) return hostOnly(env);
        const char* p = strPtr(l);
        const char* q = strPtr(r);
        for (uint32_t k = 0; k < l.len; k++) buf[k] = p[k];
        for (uint32_t k = 0; k < r.len; k++) buf[l.len + k] = q[k];
        return mkStr(buf, l.len + r.len);
    }
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
__device__ __forceinline__ Val opFunc(int32_t fid, const Val* args, int argc, const VmEnv& env, char* buf = nullptr) {
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
        // FunctionManager.cpp:197-301 (std::tolower / toupper in the C locale, trims of ' ' only)
        case F_LOWER: case F_UPPER: {
            if (args[0].t != V_STR) return mkErr();
            const uint32_t n = args[0].len;
            if (buf == nullptr || n > static_cast<uint32_t>(kStrBuildBytes)) return hostOnly(env);
            const char* p = strPtr(args[0]);
            const char lo = fid == F_LOWER ? 'A' : 'a';
            for (uint32_t k = 0; k < n; k++) {
                const char ch = p[k];
                buf[k] = (ch >= lo && ch <= lo + 25) ? static_cast<char>(ch ^ 0x20) : ch;
            }
            return mkStr(buf, n);
        }
        case F_TRIM: case F_LTRIM: case F_RTRIM: {
            if (args[0].t != V_STR) return mkErr();
            const char* p = strPtr(args[0]);
            uint32_t b = 0, e = args[0].len;
            if (fid != F_RTRIM) while (b < e && p[b] == ' ') b++;
            if (fid != F_LTRIM) while (e > b && p[e - 1] == ' ') e--;
            return mkStr(p + b, e - b);
        }
        case F_LEFT: case F_RIGHT: {
            if (args[0].t != V_STR || args[1].t != V_INT) return mkErr();
            const char* p = strPtr(args[0]);
            const uint32_t n = args[0].len;
            const int64_t k = args[1].x;
            if (k <= 0) return mkStr(p, 0);
            const uint32_t m = k < static_cast<int64_t>(n) ? static_cast<uint32_t>(k) : n;
            return fid == F_LEFT ? mkStr(p, m) : mkStr(p + (n - m), m);
        }
        case F_SUBSTR: {
            if (args[0].t != V_STR || args[1].t != V_INT || args[2].t != V_INT) return mkErr();
            const char* p = strPtr(args[0]);
            const uint64_t n = args[0].len;
            const int64_t start = args[1].x, len = args[2].x;
            // |start| > size (llabs(INT64_MIN) stays negative: a huge size_t), len <= 0 or start 0: ""
            const uint64_t mag = start < 0 ? 0ULL - static_cast<uint64_t>(start) : static_cast<uint64_t>(start);
            if (mag > n || len <= 0 || start == 0) return mkStr(p, 0);
            const uint64_t pos = start > 0 ? static_cast<uint64_t>(start - 1) : n - mag;
            const uint64_t cnt = static_cast<uint64_t>(len) < n - pos ? static_cast<uint64_t>(len) : n - pos;
            return mkStr(p + pos, static_cast<uint32_t>(cnt));
        }
        case F_LPAD: case F_RPAD: {
            if (args[0].t != V_STR || args[1].t != V_INT) return mkErr();
            const char* p = strPtr(args[0]);
            const uint64_t n = args[0].len;
            const uint64_t size = static_cast<uint64_t>(args[1].x);         // static_cast<size_t>
            if (size == 0) return mkStr(p, 0);
            if (size < n) return mkStr(p, static_cast<uint32_t>(size));     // substr(0, size)
            if (args[2].t != V_STR) return mkErr();                         // the pad is read only here
            if (size == n) return args[0];
            const uint32_t xl = args[2].len;
            // an empty pad never reaches `size` (the reference loops): host-only like an oversize one
            if (xl == 0 || buf == nullptr || size > static_cast<uint64_t>(kStrBuildBytes)) return hostOnly(env);
            const char* x = strPtr(args[2]);
            const uint32_t pad = static_cast<uint32_t>(size - n);
            char* at = buf;
            if (fid == F_RPAD) { for (uint32_t k = 0; k < n; k++) *at++ = p[k]; }
            for (uint32_t k = 0, j = 0; k < pad; k++, j = (j + 1 == xl ? 0 : j + 1)) *at++ = x[j];
            if (fid == F_LPAD) { for (uint32_t k = 0; k < n; k++) *at++ = p[k]; }
            return mkStr(buf, static_cast<uint32_t>(size));
        }
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

// $-.x / $var.x: the value of input column `col` in the edge's input row
__device__ __forceinline__ Val opInput(const VmEnv& env, const EdgeCtx& ec, int32_t col) {
    const DInputCol& c = env.input[col];
    return Val{gld<int64_t>(c.x, ec.in), gld<uint32_t>(c.len, ec.in), gld<uint8_t>(c.t, ec.in)};
}

// ------------------------------------------------------------------------------ interpreter
static __device__ __noinline__ Val vmEval(const Insn* code, const VmEnv& env, const EdgeCtx& ec, char* sout = nullptr) {
    Val st[kMaxStack];
    char sbuf[kMaxStrBuilds][kStrBuildBytes];
    auto bufOf = [&](uint8_t m) -> char* { return m < kMaxStrBuilds ? sbuf[m] : nullptr; };
    int sp = 0;
    for (int pc = 0;; pc++) {
        const Insn in = code[pc];
        switch (in.op) {
            case OP_END: return copyOut(sp > 0 ? st[sp - 1] : mkErr(), sout, &sbuf[0][0], sizeof(sbuf));
            case OP_PUSH: st[sp++] = constVal(in.t1, in.imm, static_cast<uint32_t>(in.a), env.pool); break;
            case OP_ERR: st[sp++] = mkErr(); break;
            case OP_ECOL: st[sp++] = opEcol(env, ec, in.a, in.b, in.mode, constVal(in.t2, in.imm, 0, env.pool)); break;
            case OP_EKEY: st[sp++] = opEkey(ec, in.a, in.b, in.mode, constVal(in.t2, in.imm, 0, env.pool)); break;
            case OP_EDST: st[sp++] = opEdst(ec, in.b); break;
            case OP_INPUT: st[sp++] = opInput(env, ec, in.a); break;
            case OP_SRCTAG: case OP_DSTTAG:
                st[sp++] = opTag(env, in.op == OP_SRCTAG ? ec.srow : ec.drow, in.a, in.b, in.mode,
                                 constVal(in.t2, in.imm, 0, env.pool), in.op == OP_DSTTAG);
                break;
            case OP_PLUS: break;
            case OP_NEG: st[sp - 1] = opNeg(st[sp - 1]); break;
            case OP_NOT: st[sp - 1] = opNot(st[sp - 1]); break;
            case OP_CAST:
                if (in.t1 == 1) st[sp - 1] = castToString(st[sp - 1], bufOf(in.mode), env);
                else st[sp - 1] = opCast(st[sp - 1], in.t1, env);
                break;
            case OP_ADD:
                sp--; st[sp - 1] = opArith(in.op, st[sp - 1], st[sp], env, bufOf(in.mode)); break;
            case OP_SUB: case OP_MUL: case OP_DIV: case OP_MOD: case OP_AXOR:
                sp--; st[sp - 1] = opArith(in.op, st[sp - 1], st[sp], env); break;
            case OP_LT: case OP_LE: case OP_GT: case OP_GE: case OP_EQ: case OP_NE: case OP_CONTAINS:
                sp--; st[sp - 1] = opRel(in.op, st[sp - 1], st[sp]); break;
            case OP_AND: case OP_OR: case OP_LXOR:
                sp--; st[sp - 1] = opLogic(in.op, st[sp - 1], st[sp]); break;
            case OP_FUNC: {
                int argc = in.b;
                Val out = opFunc(in.a, &st[sp - argc], argc, env, bufOf(in.mode));
                sp -= argc;
                st[sp++] = out;
                break;
            }
            default: return mkErr();
        }
    }
}

}  // namespace ngx
