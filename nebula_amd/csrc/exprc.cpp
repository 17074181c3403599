// Expression decode / pushdown rewrite / bytecode compile. See exprc.h.
#include "exprc.h"

#include <functional>
#include <cmath>

namespace ngx {

namespace {

struct Cursor {
    const uint8_t* p;
    const uint8_t* e;
    bool need(size_t n) const { return p + n <= e; }
};

bool rdStr(Cursor& c, std::string& out) {
    if (!c.need(2)) return false;
    uint16_t n;
    std::memcpy(&n, c.p, 2);
    c.p += 2;
    if (!c.need(n)) return false;
    out.assign(reinterpret_cast<const char*>(c.p), n);
    c.p += n;
    return true;
}

std::unique_ptr<ExprNode> decodeOne(Cursor& c, std::string& err, int depth) {
    if (depth > 256) { err = "expression too deep"; return nullptr; }
    if (!c.need(1)) { err = "Not enough space left"; return nullptr; }
    auto n = std::make_unique<ExprNode>();
    n->kind = *c.p++;
    switch (n->kind) {
        case K_PRIMARY: {
            if (!c.need(1)) { err = "Not enough space left"; return nullptr; }
            n->vtype = *c.p++;
            switch (n->vtype) {
                case 0: if (!c.need(8)) { err = "short"; return nullptr; } std::memcpy(&n->i, c.p, 8); c.p += 8; break;
                case 1: if (!c.need(8)) { err = "short"; return nullptr; } std::memcpy(&n->d, c.p, 8); c.p += 8; break;
                case 2: if (!c.need(1)) { err = "short"; return nullptr; } n->i = *c.p++ != 0; break;
                case 3: if (!rdStr(c, n->s)) { err = "short"; return nullptr; } break;
                default: err = "Unknown variant type"; return nullptr;
            }
            return n;
        }
        case K_FUNC: {
            if (!rdStr(c, n->name)) { err = "short"; return nullptr; }
            if (!c.need(2)) { err = "short"; return nullptr; }
            uint16_t argc;
            std::memcpy(&argc, c.p, 2);
            c.p += 2;
            for (uint16_t i = 0; i < argc; i++) {
                auto a = decodeOne(c, err, depth + 1);
                if (!a) return nullptr;
                n->kids.push_back(std::move(a));
            }
            return n;
        }
        case K_UNARY: case K_CAST: {
            if (!c.need(2)) { err = "short"; return nullptr; }
            n->op = *c.p++;
            auto a = decodeOne(c, err, depth + 1);
            if (!a) return nullptr;
            n->kids.push_back(std::move(a));
            return n;
        }
        case K_ARITH: case K_REL: case K_LOGIC: {
            if (!c.need(2)) { err = "short"; return nullptr; }
            n->op = *c.p++;
            auto l = decodeOne(c, err, depth + 1);
            if (!l) return nullptr;
            auto r = decodeOne(c, err, depth + 1);
            if (!r) return nullptr;
            n->kids.push_back(std::move(l));
            n->kids.push_back(std::move(r));
            return n;
        }
        case K_SRC_PROP: case K_EDGE_RANK: case K_EDGE_DST: case K_EDGE_SRC: case K_EDGE_TYPE:
        case K_ALIAS: case K_VAR_PROP: case K_DST_PROP: case K_INPUT_PROP:
            if (!rdStr(c, n->ref) || !rdStr(c, n->alias) || !rdStr(c, n->prop)) { err = "short"; return nullptr; }
            return n;
        default:
            err = "Illegal expression kind";
            return nullptr;
    }
}

template <typename T>
void put(std::string& s, T v) { s.append(reinterpret_cast<const char*>(&v), sizeof(T)); }
void putStr(std::string& s, const std::string& v) { put<uint16_t>(s, static_cast<uint16_t>(v.size())); s += v; }

}  // namespace

std::unique_ptr<ExprNode> decodeExpr(const uint8_t* buf, size_t len, std::string& err) {
    Cursor c{buf, buf + len};
    auto n = decodeOne(c, err, 0);
    if (n && c.p != c.e) { err = "Buffer not consumed up"; return nullptr; }
    return n;
}

std::string encodeExpr(const ExprNode& n) {
    std::string s;
    put<uint8_t>(s, n.kind);
    switch (n.kind) {
        case K_PRIMARY:
            put<uint8_t>(s, n.vtype);
            if (n.vtype == 0) put<int64_t>(s, n.i);
            else if (n.vtype == 1) put<double>(s, n.d);
            else if (n.vtype == 2) put<uint8_t>(s, n.i ? 1 : 0);
            else putStr(s, n.s);
            break;
        case K_FUNC:
            putStr(s, n.name);
            put<uint16_t>(s, static_cast<uint16_t>(n.kids.size()));
            for (auto& k : n.kids) s += encodeExpr(*k);
            break;
        case K_UNARY: case K_CAST:
            put<uint8_t>(s, n.op);
            s += encodeExpr(*n.kids[0]);
            break;
        case K_ARITH: case K_REL: case K_LOGIC:
            put<uint8_t>(s, n.op);
            s += encodeExpr(*n.kids[0]);
            s += encodeExpr(*n.kids[1]);
            break;
        default:
            putStr(s, n.ref); putStr(s, n.alias); putStr(s, n.prop);
            break;
    }
    return s;
}

std::unique_ptr<ExprNode> cloneExpr(const ExprNode& n) {
    auto c = std::make_unique<ExprNode>();
    c->kind = n.kind; c->op = n.op; c->vtype = n.vtype; c->i = n.i; c->d = n.d; c->s = n.s;
    c->ref = n.ref; c->alias = n.alias; c->prop = n.prop; c->name = n.name;
    for (auto& k : n.kids) c->kids.push_back(cloneExpr(*k));
    return c;
}

void collectRefs(const ExprNode& n, PropRefs& r) {
    switch (n.kind) {
        case K_SRC_PROP: r.srcTag.emplace(n.alias, n.prop); break;
        case K_DST_PROP: r.dstTag.emplace(n.alias, n.prop); break;
        case K_INPUT_PROP: r.input = true; break;
        case K_VAR_PROP: r.variable = true; r.vars.insert(n.alias); break;
        case K_ALIAS: case K_EDGE_RANK: case K_EDGE_DST: case K_EDGE_SRC: case K_EDGE_TYPE:
            r.alias.emplace(n.alias, n.prop); break;
        case K_FUNC: r.funcs.insert(n.name); break;
        default: break;
    }
    for (auto& k : n.kids) collectRefs(*k, r);
}

namespace {
struct FuncInfo { int32_t id; size_t minA, maxA; };
const std::map<std::string, FuncInfo>& functions() {          // FunctionManager.cpp:20-555
    static const std::map<std::string, FuncInfo> m = {
        {"abs", {F_ABS, 1, 1}}, {"floor", {F_FLOOR, 1, 1}}, {"ceil", {F_CEIL, 1, 1}},
        {"round", {F_ROUND, 1, 1}}, {"sqrt", {F_SQRT, 1, 1}}, {"cbrt", {F_CBRT, 1, 1}},
        {"exp", {F_EXP, 1, 1}}, {"exp2", {F_EXP2, 1, 1}}, {"log", {F_LOG, 1, 1}},
        {"log2", {F_LOG2, 1, 1}}, {"log10", {F_LOG10, 1, 1}}, {"sin", {F_SIN, 1, 1}},
        {"asin", {F_ASIN, 1, 1}}, {"cos", {F_COS, 1, 1}}, {"acos", {F_ACOS, 1, 1}},
        {"tan", {F_TAN, 1, 1}}, {"atan", {F_ATAN, 1, 1}}, {"hypot", {F_HYPOT, 2, 2}},
        {"pow", {F_POW, 2, 2}}, {"strcasecmp", {F_STRCASECMP, 2, 2}}, {"length", {F_LENGTH, 1, 1}},
        {"hash", {F_HASH, 1, 1}}, {"udf_is_in", {F_UDF_IS_IN, 2, 1u << 20}},
        {"lower", {F_LOWER, 1, 1}}, {"upper", {F_UPPER, 1, 1}}, {"trim", {F_TRIM, 1, 1}},
        {"ltrim", {F_LTRIM, 1, 1}}, {"rtrim", {F_RTRIM, 1, 1}}, {"left", {F_LEFT, 2, 2}},
        {"right", {F_RIGHT, 2, 2}}, {"lpad", {F_LPAD, 3, 3}}, {"rpad", {F_RPAD, 3, 3}},
        {"substr", {F_SUBSTR, 3, 3}},
    };
    return m;
}
// functions the reference has but the device VM does not evaluate (nondeterministic, or geo / vector
// helpers): they compile to NGX_E_UNSUPPORTED rather than to a wrong answer
const std::set<std::string> kHostOnlyFuncs = {"rand32", "rand64", "now", "near", "cos_similarity"};
// functions whose value is a string (views of an argument, or built in a buffer)
bool stringFunc(int32_t fid) { return fid >= F_TRIM && fid <= F_RPAD; }
bool builderFunc(int32_t fid) { return fid >= F_LOWER && fid <= F_RPAD; }
}  // namespace

bool rewritePushdown(ExprNode& n) {                            // TraverseExecutor.cpp:461-538
    auto canPushdown = [](const ExprNode& e) {
        PropRefs r;
        collectRefs(e, r);
        for (auto& f : r.funcs) {
            auto it = functions().find(f);
            if (it == functions().end() && !kHostOnlyFuncs.count(f)) return false;   // prepare fails
        }
        return !(r.input || r.variable || !r.dstTag.empty());
    };
    switch (n.kind) {
        case K_LOGIC: {
            if (n.op == 2) return canPushdown(n);              // XOR
            bool lp = rewritePushdown(*n.kids[0]);
            bool rp = rewritePushdown(*n.kids[1]);
            if (n.op == 1) return lp && rp;                    // OR
            if (n.op == 0) {                                   // AND
                if (!lp && !rp) return false;
                auto t = std::make_unique<ExprNode>();
                t->kind = K_PRIMARY; t->vtype = 2; t->i = 1;
                if (!lp) n.kids[0] = std::move(t);
                else if (!rp) n.kids[1] = std::move(t);
                return true;
            }
            return false;
        }
        case K_UNARY: case K_CAST: case K_ARITH: case K_REL: case K_FUNC:
            return canPushdown(n);
        case K_PRIMARY: case K_SRC_PROP: case K_EDGE_RANK: case K_EDGE_DST: case K_EDGE_SRC:
        case K_EDGE_TYPE: case K_ALIAS:
            return true;
        default:
            return false;
    }
}

namespace {

struct Emitter {
    Program& P;
    bool deviceLibm = false;            // let inexact libm calls of row values run on the device libm
    const Space* sp = nullptr;          // prop types (which string + can concatenate)
    int builds = 0;                     // builder buffers handed out (Insn::mode)
    // the next builder buffer, or kNoBuf when the program has used them all
    uint8_t takeBuf() { return builds < kMaxStrBuilds ? static_cast<uint8_t>(builds++) : kNoBuf; }
    void emit(uint8_t op, int32_t a = 0, int32_t b = 0, uint8_t t1 = 0, uint8_t t2 = 0, uint8_t mode = 0, int64_t imm = 0) {
        Insn in{};
        in.op = op; in.a = a; in.b = b; in.t1 = t1; in.t2 = t2; in.mode = mode; in.imm = imm;
        P.code.push_back(in);
    }
    void pushConst(const ExprNode& n) {
        switch (n.vtype) {
            case 0: emit(OP_PUSH, 0, 0, V_INT, 0, 0, n.i); break;
            case 1: { int64_t bits; std::memcpy(&bits, &n.d, 8); emit(OP_PUSH, 0, 0, V_DBL, 0, 0, bits); break; }
            case 2: emit(OP_PUSH, 0, 0, V_BOOL, 0, 0, n.i ? 1 : 0); break;
            default: {
                int64_t off = static_cast<int64_t>(P.pool.size());
                P.pool += n.s;
                emit(OP_PUSH, static_cast<int32_t>(n.s.size()), 0, V_STR, 0, 0, off);
                break;
            }
        }
    }
    // default value of a schema type (RowReader::getDefaultProp, RowReader.h:111-134) -> (vtype, bits)
    static bool defaultOf(int32_t t, uint8_t& vt, int64_t& bits) {
        switch (t) {
            case T_BOOL: vt = V_BOOL; bits = 0; return true;
            case T_INT: case T_TIMESTAMP: case T_VID: vt = V_INT; bits = 0; return true;
            case T_FLOAT: case T_DOUBLE: vt = V_DBL; bits = 0; return true;
            case T_STRING: vt = V_STR; bits = 0; return true;    // "" (len 0)
            default: return false;
        }
    }
};

// Math functions whose device (ocml) result is the correctly rounded one, so equal to glibc's bit for bit:
// fabs, floor, ceil, round and sqrt (IEEE-754 requires sqrt correctly rounded; the gfx950 f64 sqrt
// lowering refines to it). The rest are within an ulp or two of glibc but not always equal to it.
bool libmExact(int32_t fid) {
    return fid == F_ABS || fid == F_FLOOR || fid == F_CEIL || fid == F_ROUND || fid == F_SQRT;
}
bool libmFunc(int32_t fid) {
    switch (fid) {
        case F_ABS: case F_FLOOR: case F_CEIL: case F_ROUND: case F_SQRT: case F_CBRT: case F_EXP:
        case F_EXP2: case F_LOG: case F_LOG2: case F_LOG10: case F_SIN: case F_ASIN: case F_COS:
        case F_ACOS: case F_TAN: case F_ATAN: case F_HYPOT: case F_POW:
            return true;
        default:
            return false;
    }
}

// A numeric value known at compile time: a literal, its sign flip, or a math function of such values,
// evaluated here with the host libm the reference evaluates it with (FunctionManager.cpp:20-120 calls
// std::sin ... on graphd/storaged hosts). The value is the same for every row, so folding it is exact.
bool constNumber(const ExprNode& n, double& d, bool& isInt, int64_t& i) {
    if (n.kind == K_PRIMARY) {
        if (n.vtype == 0) { isInt = true; i = n.i; d = static_cast<double>(n.i); return true; }
        if (n.vtype == 1) { isInt = false; d = n.d; return true; }
        return false;
    }
    if (n.kind == K_UNARY && (n.op == 0 || n.op == 1)) {           // +x, -x (Expressions.cpp:682-706)
        if (!constNumber(*n.kids[0], d, isInt, i)) return false;
        if (n.op == 0) return true;
        if (isInt) {
            if (i == INT64_MIN) return false;                       // leave the overflow to the evaluator
            i = -i; d = static_cast<double>(i);
        } else {
            d = -d;
        }
        return true;
    }
    if (n.kind != K_FUNC) return false;
    auto it = functions().find(n.name);
    if (it == functions().end() || !libmFunc(it->second.id) || n.kids.size() < it->second.minA ||
        n.kids.size() > it->second.maxA)
        return false;
    double a[2];
    for (size_t k = 0; k < n.kids.size(); k++) {
        bool ki; int64_t kv;
        if (!constNumber(*n.kids[k], a[k], ki, kv)) return false;
    }
    switch (it->second.id) {
        case F_ABS: d = std::fabs(a[0]); break;
        case F_FLOOR: d = std::floor(a[0]); break;
        case F_CEIL: d = std::ceil(a[0]); break;
        case F_ROUND: d = std::round(a[0]); break;
        case F_SQRT: d = std::sqrt(a[0]); break;
        case F_CBRT: d = std::cbrt(a[0]); break;
        case F_EXP: d = std::exp(a[0]); break;
        case F_EXP2: d = std::exp2(a[0]); break;
        case F_LOG: d = std::log(a[0]); break;
        case F_LOG2: d = std::log2(a[0]); break;
        case F_LOG10: d = std::log10(a[0]); break;
        case F_SIN: d = std::sin(a[0]); break;
        case F_ASIN: d = std::asin(a[0]); break;
        case F_COS: d = std::cos(a[0]); break;
        case F_ACOS: d = std::acos(a[0]); break;
        case F_TAN: d = std::tan(a[0]); break;
        case F_ATAN: d = std::atan(a[0]); break;
        case F_HYPOT: d = std::hypot(a[0], a[1]); break;
        case F_POW: d = std::pow(a[0], a[1]); break;
        default: return false;
    }
    isInt = false;
    return true;
}

// whether the expression's value can be a string (string + needs a builder buffer only then)
bool mayBeString(const ExprNode& n, const Space* sp) {
    switch (n.kind) {
        case K_PRIMARY: return n.vtype == 3;
        case K_CAST: return n.op == 1;
        case K_UNARY: return n.op == 0 && mayBeString(*n.kids[0], sp);
        case K_ARITH: return n.op == 0 && mayBeString(*n.kids[0], sp) && mayBeString(*n.kids[1], sp);
        case K_REL: case K_LOGIC: return false;
        case K_FUNC: {
            auto it = functions().find(n.name);
            return it == functions().end() || stringFunc(it->second.id);
        }
        default: {
            if (sp == nullptr) return true;
            const int32_t t = exprType(n, *sp);
            return t == T_STRING || t == T_UNKNOWN;
        }
    }
}

int32_t compileCommon(const ExprNode& n, Emitter& em, std::string& err,
                      const std::function<int32_t(const ExprNode&)>& leaf,
                      const std::function<int32_t(const ExprNode&)>& rec) {
    switch (n.kind) {
        case K_PRIMARY: em.pushConst(n); return NGX_OK;
        case K_UNARY: {
            int32_t rc = rec(*n.kids[0]);
            if (rc) return rc;
            em.emit(n.op == 0 ? OP_PLUS : n.op == 1 ? OP_NEG : OP_NOT);
            return NGX_OK;
        }
        case K_CAST: {
            int32_t rc = rec(*n.kids[0]);
            if (rc) return rc;
            uint8_t buf = kNoBuf;
            if (n.op == 1 && (buf = em.takeBuf()) == kNoBuf) {
                err = "more strings built in one expression than the device evaluator buffers";
                return NGX_E_UNSUPPORTED;
            }
            em.emit(OP_CAST, 0, 0, n.op, 0, buf);
            return NGX_OK;
        }
        case K_ARITH: case K_REL: case K_LOGIC: {
            int32_t rc = rec(*n.kids[0]);
            if (rc) return rc;
            rc = rec(*n.kids[1]);
            if (rc) return rc;
            uint8_t op;
            if (n.kind == K_ARITH) {
                static const uint8_t m[] = {OP_ADD, OP_SUB, OP_MUL, OP_DIV, OP_MOD, OP_AXOR};
                if (n.op > 5) { em.emit(OP_ERR); return NGX_OK; }
                op = m[n.op];
                if (n.op == 0) {
                    // string + string builds a string: a buffer when both sides can be strings; an ADD
                    // without one flags a string operand pair as a host-only construct at run time
                    const uint8_t buf = (mayBeString(*n.kids[0], em.sp) && mayBeString(*n.kids[1], em.sp))
                                            ? em.takeBuf() : kNoBuf;
                    em.emit(op, 0, 0, 0, 0, buf);
                    return NGX_OK;
                }
            } else if (n.kind == K_REL) {
                static const uint8_t m[] = {OP_LT, OP_LE, OP_GT, OP_GE, OP_EQ, OP_NE, OP_CONTAINS};
                if (n.op > 6) { em.emit(OP_ERR); return NGX_OK; }
                op = m[n.op];
            } else {
                op = n.op == 0 ? OP_AND : n.op == 1 ? OP_OR : OP_LXOR;
            }
            em.emit(op);
            return NGX_OK;
        }
        case K_FUNC: {
            auto it = functions().find(n.name);
            if (it == functions().end()) {
                if (kHostOnlyFuncs.count(n.name)) { err = "function `" + n.name + "' is not evaluated on the device"; return NGX_E_UNSUPPORTED; }
                err = "Function `" + n.name + "' not defined";
                return NGX_E_INVALID_FILTER;
            }
            if (n.kids.size() < it->second.minA || n.kids.size() > it->second.maxA) {
                err = "Arity not match for function `" + n.name + "'";
                return NGX_E_INVALID_FILTER;
            }
            if (libmFunc(it->second.id)) {
                double d; bool isInt; int64_t iv;
                if (constNumber(n, d, isInt, iv)) {
                    ExprNode c;
                    c.kind = K_PRIMARY; c.vtype = 1; c.d = d;
                    em.pushConst(c);
                    return NGX_OK;
                }
                // a row-dependent argument: refuse rather than return a double that may differ from
                // glibc's in the last place (the caller evaluates the query on its CPU path instead);
                // constant non-numeric arguments go to the evaluator, which fails them without libm
                bool rowDependent = false;
                for (auto& k : n.kids) {
                    double kd; bool ki; int64_t kv;
                    if (k->kind != K_PRIMARY && !constNumber(*k, kd, ki, kv)) rowDependent = true;
                }
                if (rowDependent && !libmExact(it->second.id) && !em.deviceLibm) {
                    err = "function `" + n.name + "' of a row value is not evaluated on the device (its libm "
                          "is not glibc's bit for bit; set flag device_libm to accept it)";
                    return NGX_E_UNSUPPORTED;
                }
            }
            for (auto& k : n.kids) {
                int32_t rc = rec(*k);
                if (rc) return rc;
            }
            uint8_t buf = kNoBuf;
            if (builderFunc(it->second.id) && (buf = em.takeBuf()) == kNoBuf) {
                err = "more strings built in one expression than the device evaluator buffers";
                return NGX_E_UNSUPPORTED;
            }
            em.emit(OP_FUNC, it->second.id, static_cast<int32_t>(n.kids.size()), 0, 0, buf);
            return NGX_OK;
        }
        default:
            return leaf(n);
    }
}

int32_t keyIndex(const std::string& prop) {
    if (prop == "_src") return 0;
    if (prop == "_dst") return 1;
    if (prop == "_rank") return 2;
    if (prop == "_type") return 3;
    return -1;
}

}  // namespace

int32_t compileStorage(const ExprNode& root, StorageCtx& ctx, Program& out, std::string& err) {
    Emitter em{out};
    em.deviceLibm = ctx.deviceLibm;
    em.sp = ctx.sp;
    std::function<int32_t(const ExprNode&)> rec;
    auto leaf = [&](const ExprNode& n) -> int32_t {
        const Space& sp = *ctx.sp;
        switch (n.kind) {
            case K_ALIAS: {                                        // checkExp .inl:280-310
                if (!ctx.haveEdgeContexts) { err = "No edge requested"; return NGX_E_INVALID_FILTER; }
                auto et = sp.edgeByName.find(n.alias);
                if (et == sp.edgeByName.end()) { err = "Can't find edge " + n.alias; return NGX_E_INVALID_FILTER; }
                const SchemaSet* ss = sp.edge(std::abs(et->second));
                if (!ss) { err = "no edge schema"; return NGX_E_INVALID_FILTER; }
                int32_t col = ss->latest().index(n.prop);
                if (col < 0) { err = "Can't find related prop " + n.prop; return NGX_E_INVALID_FILTER; }
                // getAliasProp (.inl:539-565): edgeMap_ miss => error; type mismatch => error;
                // prop missing in the row's schema version => "Invalid Prop" error
                auto em_ = ctx.edgeMap.find(n.alias);
                if (em_ == ctx.edgeMap.end()) { em.emit(OP_ERR); return NGX_OK; }
                if (em_->second != std::abs(et->second)) { em.emit(OP_ERR); return NGX_OK; }
                em.emit(OP_ECOL, col, em_->second, 0, 0, 0, 0);
                return NGX_OK;
            }
            case K_EDGE_RANK: case K_EDGE_SRC: case K_EDGE_TYPE: case K_EDGE_DST: {
                auto em_ = ctx.edgeMap.find(n.alias);               // no checkExp constraint (:274-279)
                if (em_ == ctx.edgeMap.end()) { em.emit(OP_ERR); return NGX_OK; }
                int32_t k = n.kind == K_EDGE_DST ? 1 : keyIndex(n.prop);
                if (k < 0) { em.emit(OP_ERR); return NGX_OK; }
                em.emit(OP_EKEY, k, em_->second, 0, 0, 0, 0);
                return NGX_OK;
            }
            case K_SRC_PROP: {                                     // checkExp .inl:236-273
                auto tid = sp.tagByName.find(n.alias);
                if (tid == sp.tagByName.end()) { err = "Can't find tag " + n.alias; return NGX_E_INVALID_FILTER; }
                const SchemaSet* ss = sp.tag(tid->second);
                int32_t col = ss ? ss->latest().index(n.prop) : -1;
                if (col < 0) { err = "Can't find related prop " + n.prop; return NGX_E_INVALID_FILTER; }
                int32_t tslot = sp.tagSlotOf(tid->second);
                if (tslot < 0) { em.emit(OP_ERR); return NGX_OK; }
                ctx.filterTags.insert(tid->second);
                out.usesSrcTag = true;
                em.emit(OP_SRCTAG, col, tslot, 0, 0, 0, 0);        // no tag row => "Invalid Tag Filter"
                return NGX_OK;
            }
            default:                                               // $-, $var, $$, unknown
                err = "Unsupport expression type in storage filter";
                return NGX_E_INVALID_FILTER;
        }
    };
    rec = [&](const ExprNode& n) { return compileCommon(n, em, err, leaf, rec); };
    int32_t rc = rec(root);
    if (rc == NGX_OK) em.emit(OP_END);
    return rc;
}

int32_t compileGraphd(const ExprNode& root, GraphdCtx& ctx, Program& out, std::string& err) {
    Emitter em{out};
    em.deviceLibm = ctx.deviceLibm;
    em.sp = ctx.sp;
    std::function<int32_t(const ExprNode&)> rec;
    auto leaf = [&](const ExprNode& n) -> int32_t {
        const Space& sp = *ctx.sp;
        switch (n.kind) {
            case K_ALIAS: case K_EDGE_RANK: case K_EDGE_SRC: case K_EDGE_TYPE: {
                // getAliasProp (GoExecutor.cpp:1183-1220)
                auto at = ctx.aliasType.find(n.alias);
                if (at == ctx.aliasType.end()) { err = "Edge `" + n.alias + "' not found."; return NGX_E_QUERY; }
                int32_t type = at->second;
                int32_t keyed = ctx.direction == NGX_DIR_REVERSELY ? -type : type;
                // the default used when the edge being read is of another type
                uint8_t dvt = 0; int64_t dbits = 0; uint8_t mode = 0;
                auto rs = ctx.respSchema.find(keyed);
                if (rs != ctx.respSchema.end()) {
                    auto f = rs->second.find(n.prop);
                    if (f != rs->second.end() && Emitter::defaultOf(f->second, dvt, dbits)) mode = 1;
                }
                // mode bit0 clear => mismatch is an error ("Can't find schema ... when get default")
                int32_t k = n.kind == K_ALIAS ? keyIndex(n.prop) : keyIndex(n.prop);
                if (n.kind == K_ALIAS && k < 0) {
                    const SchemaSet* ss = sp.edge(type);
                    int32_t col = ss ? ss->latest().index(n.prop) : -1;
                    if (col < 0) { err = "`" + n.prop + "' is not a prop of `" + n.alias + "'"; return NGX_E_QUERY; }
                    em.emit(OP_ECOL, col, type, 0, dvt, static_cast<uint8_t>(mode | 2), dbits);
                    return NGX_OK;
                }
                if (k < 0 || k == 1) {          // `_dst' through getAliasProp reads the row: not requested
                    em.emit(OP_ERR);
                    return NGX_OK;
                }
                em.emit(OP_EKEY, k, type, 0, dvt, mode, dbits);
                return NGX_OK;
            }
            case K_EDGE_DST: {                                     // getEdgeDstId (:1102-1117)
                int32_t type = 0;
                if (ctx.nEdgeTypes > 1) {
                    auto at = ctx.aliasType.find(n.alias);
                    if (at == ctx.aliasType.end()) { em.emit(OP_ERR); return NGX_OK; }
                    type = at->second;
                }
                em.emit(OP_EDST, 0, type);
                return NGX_OK;
            }
            case K_SRC_PROP: case K_DST_PROP: {                    // getSrcTagProp / getDstTagProp
                auto tid = sp.tagByName.find(n.alias);
                if (tid == sp.tagByName.end()) { err = "Tag `" + n.alias + "' not found."; return NGX_E_QUERY; }
                const SchemaSet* ss = sp.tag(tid->second);
                int32_t col = ss ? ss->latest().index(n.prop) : -1;
                if (col < 0) { err = "`" + n.prop + "' is not a prop of `" + n.alias + "'"; return NGX_E_QUERY; }
                uint8_t dvt; int64_t dbits;
                Emitter::defaultOf(ss->latest().fields[col].type, dvt, dbits);
                int32_t tslot = sp.tagSlotOf(tid->second);
                if (tslot < 0) { em.emit(OP_PUSH, 0, 0, dvt, 0, 0, dbits); return NGX_OK; }
                if (n.kind == K_SRC_PROP) { out.usesSrcTag = true; em.emit(OP_SRCTAG, col, tslot, 0, dvt, 1, dbits); }
                else { out.usesDstTag = true; em.emit(OP_DSTTAG, col, tslot, 0, dvt, 1, dbits); }
                return NGX_OK;
            }
            case K_INPUT_PROP: case K_VAR_PROP: {
                if (ctx.inputCols == nullptr) {
                    err = "$- / $var inputs are outside the GO fast path";
                    return NGX_E_UNSUPPORTED;
                }
                auto it = ctx.inputCols->find(n.prop);          // InterimResult::getColumnWithRow
                if (it == ctx.inputCols->end()) { err = "Prop `" + n.prop + "' not found"; return NGX_E_QUERY; }
                em.emit(OP_INPUT, it->second);
                return NGX_OK;
            }
            default:
                err = "$- / $var inputs are outside the GO fast path";
                return NGX_E_UNSUPPORTED;
        }
    };
    rec = [&](const ExprNode& n) { return compileCommon(n, em, err, leaf, rec); };
    int32_t rc = rec(root);
    if (rc == NGX_OK) em.emit(OP_END);
    return rc;
}

int32_t exprType(const ExprNode& n, const Space& sp) {
    switch (n.kind) {
        case K_PRIMARY: case K_FUNC: case K_UNARY: case K_ARITH: return T_UNKNOWN;
        case K_CAST: {
            static const int32_t m[] = {T_INT, T_STRING, T_DOUBLE, T_BOOL, T_TIMESTAMP};
            return n.op < 5 ? m[n.op] : T_UNKNOWN;
        }
        case K_REL: case K_LOGIC: return T_BOOL;
        case K_SRC_PROP: case K_DST_PROP: {
            auto t = sp.tagByName.find(n.alias);
            if (t == sp.tagByName.end()) return T_UNKNOWN;
            const SchemaSet* ss = sp.tag(t->second);
            return ss ? ss->latest().typeOf(n.prop) : T_UNKNOWN;
        }
        case K_EDGE_DST: case K_EDGE_SRC: return T_VID;
        case K_EDGE_RANK: case K_EDGE_TYPE: return T_INT;
        case K_ALIAS: {
            auto e = sp.edgeByName.find(n.alias);
            if (e == sp.edgeByName.end()) return T_UNKNOWN;
            const SchemaSet* ss = sp.edge(e->second);
            return ss ? ss->latest().typeOf(n.prop) : T_UNKNOWN;
        }
        default: return T_UNKNOWN;
    }
}

}  // namespace ngx
