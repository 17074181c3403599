// POD types shared by the host engine and the HIP kernels: device column / slot / tag
// descriptors and the flat filter bytecode the host compiles WHERE / YIELD expressions into
// (exprc.cpp) and the device VM executes per edge (kernels.hip).
#pragma once

#ifndef __HIPCC_RTC__
#include <cstdint>
#endif

namespace ngx {

constexpr uint32_t kNoRow = 0xFFFFFFFFu;
constexpr int kMaxSlots = 16;
constexpr int kMaxStack = 12;
constexpr int kStrBuildBytes = 64;          // longest string a builder (lower, upper, lpad, rpad, string +,
                                            // (string)) makes on the device; longer: host-only construct
constexpr int kMaxStrBuilds = 4;            // builder buffers per program (exprc.cpp refuses more)
constexpr uint8_t kNoBuf = 0xFF;            // Insn::mode of an OP_ADD / OP_FUNC / OP_CAST without a buffer

// a column of a pipe's input table on the device (the InterimResult rows a $- / $var sentence reads):
// value bits (string: device pointer), string lengths, VM value types per row
struct DInputCol {
    const int64_t* x;
    const uint32_t* len;
    const uint8_t* t;
};

// per-edge flags (HostSlot::eflags)
enum : uint8_t {
    EF_EMPTY_VALUE = 1,    // the KV value was empty: no RowReader, filter not evaluated (.inl:520)
    EF_BAD_ROW = 2,        // getEdgePropReader returned null: skipped when props are read (.inl:525-528)
};

// device column descriptor
struct DCol {
    int32_t type;          // SType of the latest schema
    int32_t width;         // INT/TIMESTAMP/VID storage bytes: 1, 2, 4 (narrowed at export, sign-extended) or 8
    const void* data;      // int64_t (INT/TIMESTAMP/VID; see width), double (FLOAT/DOUBLE), uint8_t (BOOL)
    const uint64_t* soff;  // STRING: n + 1 offsets
    const char* sbytes;    // STRING bytes
    const uint8_t* valid;  // nullptr when every row had the field
};

struct DSlot {
    int32_t etype;         // signed edge type
    int32_t ncols;
    int32_t colBase;       // first DCol of this slot in the column table
    int32_t hasFlags;
    const uint64_t* off;   // V + 1
    const void* dst;       // dst vids at dstW bytes (1 / 2 / 4 / 8, sign-extended on load)
    const uint32_t* dgid;
    const void* rank;      // ranks at rankW bytes; nullptr when every edge of the slot has rank rankConst
    const uint8_t* eflags;
    int32_t dstW, rankW;
    int64_t rankConst;
};



struct DTag {
    int32_t tag;
    int32_t ncols;
    int32_t colBase;
    int32_t ttlCol;        // TTL column (INT / TIMESTAMP / VID of the latest schema), -1: no TTL check
    const uint8_t* present;
    int64_t ttlDur;        // ttl_duration (> 0 when ttlCol >= 0)
};

// ------------------------------------------------------------------ bytecode
// VM values
enum : uint8_t { V_ERR = 0, V_INT = 1, V_DBL = 2, V_BOOL = 3, V_STR = 4 };

enum Op : uint8_t {
    OP_END = 0,
    OP_PUSH,           // push constant: t1 = value type, imm = bits (string: imm = pool offset, a = len)
    OP_ERR,            // push an error (a getter that always fails)
    OP_ECOL,           // edge column: a = column index in |type| schema, b = |type| required
                       //   mode bit0: mismatch -> default (graphd) instead of error (storage)
                       //   mode bit1: invalid field -> default (graphd) instead of error
                       //   t2/imm: default value type/bits
    OP_EKEY,           // key prop: a = 0 src,1 dst,2 rank,3 type; b = |type| required (0: any)
                       //   mode bit0 as OP_ECOL; t2/imm default
    OP_EDST,           // EdgeDstIdExpression in graphd: b = alias type (0: no check), mismatch -> 0
    OP_SRCTAG,         // src tag column: a = column, b = tag slot; mode bit0: missing -> default
    OP_DSTTAG,         // dst tag column (graphd $$): a = column, b = tag slot; missing -> default
    OP_NEG, OP_PLUS, OP_NOT,
    OP_CAST,           // t1 = ColumnType target (INT=0, STRING=1, DOUBLE=2, BOOL=3, TIMESTAMP=4);
                       // (string): mode = builder buffer
    OP_ADD,            // mode = builder buffer for string + string (kNoBuf: none)
    OP_SUB, OP_MUL, OP_DIV, OP_MOD, OP_AXOR,
    OP_LT, OP_LE, OP_GT, OP_GE, OP_EQ, OP_NE, OP_CONTAINS,
    OP_AND, OP_OR, OP_LXOR,
    OP_FUNC,           // a = function id, b = argc, mode = builder buffer (kNoBuf: none)
    OP_INPUT,          // $-.x / $var.x of the edge's input row (multi-root pipe walks): a = input column
};

enum Func : int32_t {
    F_ABS = 0, F_FLOOR, F_CEIL, F_ROUND, F_SQRT, F_CBRT, F_EXP, F_EXP2, F_LOG, F_LOG2, F_LOG10,
    F_SIN, F_ASIN, F_COS, F_ACOS, F_TAN, F_ATAN, F_HYPOT, F_POW, F_STRCASECMP, F_LENGTH, F_HASH,
    F_UDF_IS_IN,
    // strings (FunctionManager.cpp:197-301): views of their argument
    F_TRIM, F_LTRIM, F_RTRIM, F_LEFT, F_RIGHT, F_SUBSTR,
    // ... and builders (Insn::mode = the evaluation buffer they write)
    F_LOWER, F_UPPER, F_LPAD, F_RPAD,
};

struct Insn {
    uint8_t op;
    uint8_t t1;
    uint8_t t2;
    uint8_t mode;
    int32_t a;
    int32_t b;
    int32_t pad;
    int64_t imm;
};
static_assert(sizeof(Insn) == 24, "Insn layout");

#ifndef __HIPCC_RTC__
// how many builder buffers (Insn::mode) the program's evaluation needs: a YIELD column whose program
// uses any stores its built strings in the result string arena (FinalArgs::strOut)
inline int strBuffersOf(const Insn* code) {
    int n = 0;
    for (const Insn* in = code; in->op != OP_END; in++) {
        const bool builder = (in->op == OP_CAST && in->t1 == 1) || in->op == OP_ADD || in->op == OP_FUNC;
        if (builder && in->mode < kMaxStrBuilds && in->mode + 1 > n) n = in->mode + 1;
    }
    return n;
}
#endif

}  // namespace ngx
