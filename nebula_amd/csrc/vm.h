// Device bytecode VM: evaluates one compiled WHERE / YIELD program (exprc.cpp) for one edge,
// restating the reference evaluation rules exactly (src/common/filter/Expressions.cpp:662-1228,
// FunctionManager.cpp:20-555): no short circuit, error propagation left-first, implicit casts
// bool < int < double, |l - r| < 1e-8 double equality, int64 overflow and division errors.
#pragma once

#include <hip/hip_runtime.h>

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
    uint64_t pos;       // edge index inside the slot arrays
    uint32_t srow;      // local row of the source vertex
    uint32_t drow;      // local row of the destination (kNoRow when not on this shard)
    int64_t src, dst, rank;
};

struct VmEnv {
    const DSlot* slots;
    const DTag* tags;
    const DCol* cols;
    const char* pool;
    uint32_t* unsupported;     // set when a value needs a host-only construct
};

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

__device__ __forceinline__ Val loadCol(const DCol& c, uint64_t i) {
    switch (c.type) {
        case 2: case 21: case 3: return mkInt(static_cast<const int64_t*>(c.data)[i]);
        case 4: case 5: return mkDbl(static_cast<const double*>(c.data)[i]);
        case 1: return mkBool(static_cast<const uint8_t*>(c.data)[i] != 0);
        case 6: {
            uint64_t o = c.soff[i];
            return Val{reinterpret_cast<int64_t>(c.sbytes + o), static_cast<uint32_t>(c.soff[i + 1] - o), V_STR};
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

__device__ Val vmEval(const Insn* code, const VmEnv& env, const EdgeCtx& ec);

}  // namespace ngx
