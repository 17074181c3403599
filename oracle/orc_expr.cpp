// ORACLE — TEST INFRASTRUCTURE ONLY (see orc_core.h header).
// Restates src/common/filter/Expressions.cpp and FunctionManager.cpp.
#include "orc_expr.h"

#include <charconv>
#include <cstdlib>
#include <strings.h>
#include <unordered_set>

namespace orc {

namespace {
Status spaceErr() { return Status::Error("Not enough space left"); }
#define ORC_NEED(POS, END, N) do { if ((POS) + (N) > (END)) throw spaceErr(); } while (false)

template <typename T>
T rd(const char*& p) { T v; std::memcpy(&v, p, sizeof(T)); p += sizeof(T); return v; }
template <typename T>
void wr(std::string& s, T v) { s.append(reinterpret_cast<const char*>(&v), sizeof(T)); }
void wrStr16(std::string& s, const std::string& v) { wr<uint16_t>(s, static_cast<uint16_t>(v.size())); s.append(v); }
std::string rdStr16(const char*& pos, const char* end) {
    ORC_NEED(pos, end, 2);
    auto n = rd<uint16_t>(pos);
    ORC_NEED(pos, end, n);
    std::string s(pos, n);
    pos += n;
    return s;
}
Status badGet() { return Status::Error("bad_get: argument type mismatch"); }
}  // namespace

// folly::to<std::string>(double): double-conversion SHORTEST, NO_FLAGS, 'E', low -6, high 21.
std::string Expression::toString(const Variant& v) {
    switch (which(v)) {
        case VAR_INT64: return std::to_string(std::get<int64_t>(v));
        case VAR_DOUBLE: {
            double d = std::get<double>(v);
            if (std::isnan(d)) return "NaN";
            if (std::isinf(d)) return d < 0 ? "-Infinity" : "Infinity";
            if (d == 0) return std::signbit(d) ? "-0" : "0";
            char buf[64];
            auto r = std::to_chars(buf, buf + sizeof(buf), d, std::chars_format::scientific);
            std::string sci(buf, r.ptr);                  // e.g. "-1.2345e+02"
            bool neg = sci[0] == '-';
            if (neg) sci = sci.substr(1);
            auto epos = sci.find('e');
            int exp10 = std::atoi(sci.c_str() + epos + 1);
            std::string digits;
            for (size_t i = 0; i < epos; i++) if (sci[i] != '.') digits.push_back(sci[i]);
            int decimalPoint = exp10 + 1;                 // position of the point after digit[0..]
            std::string out = neg ? "-" : "";
            if (-6 < decimalPoint && decimalPoint <= 21) {
                if (decimalPoint <= 0) {
                    out += "0.";
                    out.append(static_cast<size_t>(-decimalPoint), '0');
                    out += digits;
                } else if (decimalPoint >= static_cast<int>(digits.size())) {
                    out += digits;
                    out.append(static_cast<size_t>(decimalPoint - static_cast<int>(digits.size())), '0');
                } else {
                    out += digits.substr(0, decimalPoint);
                    out += ".";
                    out += digits.substr(decimalPoint);
                }
            } else {
                out += digits.substr(0, 1);
                if (digits.size() > 1) { out += "."; out += digits.substr(1); }
                out += "E";
                out += std::to_string(exp10);
            }
            return out;
        }
        case VAR_BOOL: return std::get<bool>(v) ? "true" : "false";
        case VAR_STR: return std::get<std::string>(v);
    }
    return "";
}

double Expression::toDouble(const Variant& v) {
    switch (which(v)) {
        case VAR_INT64: return static_cast<double>(std::get<int64_t>(v));
        case VAR_DOUBLE: return std::get<double>(v);
        case VAR_BOOL: return std::get<bool>(v) ? 1.0 : 0.0;
        case VAR_STR: {
            const auto& s = std::get<std::string>(v);
            char* end = nullptr;
            double d = std::strtod(s.c_str(), &end);
            if (end == s.c_str() || *end != '\0') throw Status::Error("folly::to<double> failed");
            return d;
        }
    }
    return 0;
}

int64_t Expression::toInt(const Variant& v) {
    switch (which(v)) {
        case VAR_INT64: return std::get<int64_t>(v);
        case VAR_DOUBLE: {
            double d = std::get<double>(v);
            // static_cast<int64_t>(double): x86 cvttsd2si yields INT64_MIN out of range / NaN.
            if (!(d > -9223372036854775809.0 && d < 9223372036854775808.0)) return INT64_MIN;
            return static_cast<int64_t>(d);
        }
        case VAR_BOOL: return std::get<bool>(v) ? 1 : 0;
        case VAR_STR: {
            const auto& s = std::get<std::string>(v);
            char* end = nullptr;
            errno = 0;
            long long x = std::strtoll(s.c_str(), &end, 10);
            if (end == s.c_str() || *end != '\0' || errno) throw Status::Error("folly::to<int64_t> failed");
            return x;
        }
    }
    return 0;
}

// Expression::makeExpr (Expressions.cpp:50-89)
std::unique_ptr<Expression> Expression::makeExpr(uint8_t kind) {
    switch (kind) {
        case kPrimary: return std::make_unique<PrimaryExpression>();
        case kFunctionCall: return std::make_unique<FunctionCallExpression>();
        case kUnary: return std::make_unique<UnaryExpression>();
        case kTypeCasting: return std::make_unique<TypeCastingExpression>();
        case kUUID: throw Status::Error("Not supported yet");
        case kArithmetic: return std::make_unique<ArithmeticExpression>();
        case kRelational: return std::make_unique<RelationalExpression>();
        case kLogical: return std::make_unique<LogicalExpression>();
        case kSourceProp: case kEdgeRank: case kEdgeDstId: case kEdgeSrcId: case kEdgeType:
        case kAliasProp: case kVariableProp: case kDestProp: case kInputProp: {
            auto e = std::make_unique<AliasPropertyExpression>();
            e->setKind(static_cast<Kind>(kind));
            return e;
        }
        default: throw Status::Error("Illegal expression kind");
    }
}

// Expression::decode (Expressions.cpp:100-116)
StatusOr<std::shared_ptr<Expression>> Expression::decode(const std::string& buf) {
    const char* pos = buf.data();
    const char* end = pos + buf.size();
    try {
        ORC_NEED(pos, end, 1);
        auto expr = makeExpr(static_cast<uint8_t>(*pos++));
        pos = expr->decode(pos, end);
        if (pos != end) return Status::Error("Buffer not consumed up");
        return std::shared_ptr<Expression>(std::move(expr));
    } catch (const Status& s) {
        return s;
    }
}

// ---------------------------------------------------------------- alias family
OptVariant AliasPropertyExpression::eval(Getters& g) const {
    switch (kind_) {
        case kInputProp:                                                // :214-219
            if (!g.getInputProp) return Status::Error("`getInputProp' function is not implemented");
            return g.getInputProp(prop_);
        case kDestProp:                                                 // :237-242
            if (!g.getDstTagProp) return Status::Error("`getDstTagProp' function is not implemented");
            return g.getDstTagProp(alias_, prop_);
        case kVariableProp:                                             // :265-270
            if (!g.getVariableProp) return Status::Error("`getVariableProp' function is not implemented");
            return g.getVariableProp(prop_);
        case kEdgeDstId:                                                // :327-332
            if (!g.getEdgeDstId) return Status::Error("`getEdgeDstId' function is not implemented");
            return g.getEdgeDstId(alias_);
        case kSourceProp:                                               // :376-381
            if (!g.getSrcTagProp) return Status::Error("`getSrcTagProp' function is not implemented");
            return g.getSrcTagProp(alias_, prop_);
        default:                                                        // kAliasProp/_type/_src/_rank
            if (!g.getAliasProp) return Status::Error("`getAliasProp' function is not implemented");
            return g.getAliasProp(alias_, prop_);
    }
}
Status AliasPropertyExpression::prepare(ExpressionContext* ctx) {
    switch (kind_) {
        case kInputProp: ctx->addInputProp(prop_); break;
        case kDestProp: ctx->addDstTagProp(alias_, prop_); break;
        case kVariableProp: ctx->addVariableProp(alias_, prop_); break;
        case kSourceProp: ctx->addSrcTagProp(alias_, prop_); break;
        default: ctx->addAliasProp(alias_, prop_); break;
    }
    return Status::OK();
}
void AliasPropertyExpression::encode(std::string& out) const {       // :159-167
    wr<uint8_t>(out, kind_);
    wrStr16(out, ref_); wrStr16(out, alias_); wrStr16(out, prop_);
}
const char* AliasPropertyExpression::decode(const char* pos, const char* end) {   // :169-199
    ref_ = rdStr16(pos, end);
    alias_ = rdStr16(pos, end);
    prop_ = rdStr16(pos, end);
    return pos;
}
ExprPtr AliasPropertyExpression::clone() const {
    auto e = std::make_unique<AliasPropertyExpression>(ref_, alias_, prop_);
    e->setKind(kind_);
    return e;
}
std::string AliasPropertyExpression::toString() const {             // :118-137
    std::string buf = ref_;
    if (ref_ != "" && ref_ != "$") buf += ".";
    buf += alias_;
    if (alias_ != "") buf += ".";
    buf += prop_;
    return buf;
}

// ---------------------------------------------------------------- primary
void PrimaryExpression::encode(std::string& out) const {             // :450-473
    wr<uint8_t>(out, kind_);
    wr<uint8_t>(out, static_cast<uint8_t>(which(v_)));
    switch (which(v_)) {
        case VAR_INT64: wr<int64_t>(out, std::get<int64_t>(v_)); break;
        case VAR_DOUBLE: wr<double>(out, std::get<double>(v_)); break;
        case VAR_BOOL: wr<uint8_t>(out, std::get<bool>(v_) ? 1 : 0); break;
        case VAR_STR: wrStr16(out, std::get<std::string>(v_)); break;
    }
}
const char* PrimaryExpression::decode(const char* pos, const char* end) {  // :476-507
    ORC_NEED(pos, end, 1);
    auto w = static_cast<uint8_t>(*pos++);
    switch (w) {
        case VAR_INT64: ORC_NEED(pos, end, 8); v_ = rd<int64_t>(pos); break;
        case VAR_DOUBLE: ORC_NEED(pos, end, 8); v_ = rd<double>(pos); break;
        case VAR_BOOL: ORC_NEED(pos, end, 1); v_ = (*pos++ != 0); break;
        case VAR_STR: v_ = rdStr16(pos, end); break;
        default: throw Status::Error("Unknown variant type");
    }
    return pos;
}
std::string PrimaryExpression::toString() const {
    switch (which(v_)) {
        case VAR_INT64: return std::to_string(std::get<int64_t>(v_));
        case VAR_DOUBLE: { char b[64]; snprintf(b, sizeof(b), "%.15lf", std::get<double>(v_)); return b; }
        case VAR_BOOL: return std::get<bool>(v_) ? "true" : "false";
        default: return std::get<std::string>(v_);
    }
}

// ---------------------------------------------------------------- function call
OptVariant FunctionCallExpression::eval(Getters& g) const {          // :526-540
    std::vector<Variant> args;
    for (auto& a : args_) {
        auto r = a->eval(g);
        if (!r.ok()) return r;
        args.push_back(r.value());
    }
    if (!func_) return Status::Error("function not bound");
    return func_(args);
}
Status FunctionCallExpression::prepare(ExpressionContext* ctx) {     // :553-569
    auto f = getFunction(name_, args_.size());
    if (!f.ok()) return f.status();
    func_ = f.value();
    for (auto& a : args_) {
        auto s = a->prepare(ctx);
        if (!s.ok()) return s;
    }
    return Status::OK();
}
void FunctionCallExpression::encode(std::string& out) const {        // :572-582
    wr<uint8_t>(out, kind_);
    wrStr16(out, name_);
    wr<uint16_t>(out, static_cast<uint16_t>(args_.size()));
    for (auto& a : args_) a->encode(out);
}
const char* FunctionCallExpression::decode(const char* pos, const char* end) {   // :585-605
    name_ = rdStr16(pos, end);
    ORC_NEED(pos, end, 2);       // the reference reads the count without a space check
    auto count = rd<uint16_t>(pos);
    for (unsigned i = 0; i < count; i++) {
        ORC_NEED(pos, end, 1);
        auto a = makeExpr(static_cast<uint8_t>(*pos++));
        pos = a->decode(pos, end);
        args_.push_back(std::move(a));
    }
    return pos;
}
ExprPtr FunctionCallExpression::clone() const {
    auto e = std::make_unique<FunctionCallExpression>();
    e->name_ = name_;
    for (auto& a : args_) e->args_.push_back(a->clone());
    e->func_ = func_;
    return e;
}
std::string FunctionCallExpression::toString() const {
    std::string b = name_ + "(";
    for (size_t i = 0; i < args_.size(); i++) { if (i) b += ","; b += args_[i]->toString(); }
    return b + ")";
}

// ---------------------------------------------------------------- unary
OptVariant UnaryExpression::eval(Getters& g) const {                 // :662-681
    auto value = operand_->eval(g);
    if (!value.ok()) return value;   // the reference dereferences the failed value here (crash)
    const auto& v = value.value();
    if (op_ == PLUS) return value;
    if (op_ == NEGATE) {
        if (isInt(v)) return OptVariant(static_cast<int64_t>(0ULL - static_cast<uint64_t>(asInt(v))));
        if (isDouble(v)) return OptVariant(-asDouble(v));
        return Status::Error("attempt to perform unary arithmetic");
    }
    return OptVariant(!asBool(v));
}
void UnaryExpression::encode(std::string& out) const {
    wr<uint8_t>(out, kind_); wr<uint8_t>(out, op_); operand_->encode(out);
}
const char* UnaryExpression::decode(const char* pos, const char* end) {   // :704-711
    ORC_NEED(pos, end, 2);
    op_ = static_cast<Operator>(*pos++);
    operand_ = makeExpr(static_cast<uint8_t>(*pos++));
    return operand_->decode(pos, end);
}
ExprPtr UnaryExpression::clone() const {
    auto e = std::make_unique<UnaryExpression>(); e->op_ = op_; e->operand_ = operand_->clone(); return e;
}
std::string UnaryExpression::toString() const {
    const char* o = op_ == PLUS ? "+" : op_ == NEGATE ? "-" : "!";
    return std::string(o) + "(" + operand_->toString() + ")";
}

// ---------------------------------------------------------------- type casting
OptVariant TypeCastingExpression::eval(Getters& g) const {           // :745-763
    auto r = operand_->eval(g);
    if (!r.ok()) return r;
    try {
        switch (type_) {
            case ColumnType::INT: case ColumnType::TIMESTAMP: return OptVariant(toInt(r.value()));
            case ColumnType::STRING: return OptVariant(Expression::toString(r.value()));
            case ColumnType::DOUBLE: return OptVariant(toDouble(r.value()));
            case ColumnType::BOOL: return OptVariant(toBool(r.value()));
        }
    } catch (const Status& s) {
        return s;
    }
    return Status::Error("casting to unknown type");
}
void TypeCastingExpression::encode(std::string& out) const {
    wr<uint8_t>(out, kind_); wr<uint8_t>(out, static_cast<uint8_t>(type_)); operand_->encode(out);
}
const char* TypeCastingExpression::decode(const char* pos, const char* end) {    // :786-792
    ORC_NEED(pos, end, 2);
    type_ = static_cast<ColumnType>(*pos++);
    operand_ = makeExpr(static_cast<uint8_t>(*pos++));
    return operand_->decode(pos, end);
}
ExprPtr TypeCastingExpression::clone() const {
    auto e = std::make_unique<TypeCastingExpression>(); e->type_ = type_; e->operand_ = operand_->clone(); return e;
}
std::string TypeCastingExpression::toString() const {
    static const char* n[] = {"int", "string", "double", "bool", "timestamp"};
    return std::string("(") + n[static_cast<int>(type_) % 5] + ")" + operand_->toString();
}

// ---------------------------------------------------------------- binary
void BinaryExpression::encode(std::string& out) const {              // :1002-1007 etc.
    wr<uint8_t>(out, kind_); wr<uint8_t>(out, op_); left_->encode(out); right_->encode(out);
}
const char* BinaryExpression::decode(const char* pos, const char* end) {    // :1010-1021 etc.
    ORC_NEED(pos, end, 2);
    op_ = static_cast<uint8_t>(*pos++);
    left_ = makeExpr(static_cast<uint8_t>(*pos++));
    pos = left_->decode(pos, end);
    ORC_NEED(pos, end, 1);
    right_ = makeExpr(static_cast<uint8_t>(*pos++));
    return right_->decode(pos, end);
}

template <typename T>
static ExprPtr cloneBinary(const BinaryExpression& b) {
    auto e = std::make_unique<T>();
    e->op_ = b.op_; e->left_ = b.left_->clone(); e->right_ = b.right_->clone();
    return e;
}
ExprPtr ArithmeticExpression::clone() const { return cloneBinary<ArithmeticExpression>(*this); }
ExprPtr RelationalExpression::clone() const { return cloneBinary<RelationalExpression>(*this); }
ExprPtr LogicalExpression::clone() const { return cloneBinary<LogicalExpression>(*this); }
std::string ArithmeticExpression::toString() const {
    static const char* n[] = {"+", "-", "*", "/", "%", "^"};
    return "(" + left_->toString() + (op_ < 6 ? n[op_] : "?") + right_->toString() + ")";
}
std::string RelationalExpression::toString() const {
    static const char* n[] = {"<", "<=", ">", ">=", "==", "!=", " CONTAINS "};
    return "(" + left_->toString() + (op_ < 7 ? n[op_] : "?") + right_->toString() + ")";
}
std::string LogicalExpression::toString() const {
    static const char* n[] = {"&&", "||", "XOR"};
    return "(" + left_->toString() + (op_ < 3 ? n[op_] : "?") + right_->toString() + ")";
}

// ArithmeticExpression::eval (Expressions.cpp:825-977)
OptVariant ArithmeticExpression::eval(Getters& g) const {
    auto left = left_->eval(g);
    auto right = right_->eval(g);
    if (!left.ok()) return left;
    if (!right.ok()) return right;
    const Variant& l = left.value();
    const Variant& r = right.value();
    constexpr int64_t maxInt = INT64_MAX;
    constexpr int64_t minInt = INT64_MIN;
    auto isAddOverflow = [](int64_t lv, int64_t rv) {
        if (lv >= 0 && rv >= 0) return maxInt - lv < rv;
        if (lv < 0 && rv < 0) return minInt - lv > rv;
        return false;
    };
    auto isSubOverflow = [](int64_t lv, int64_t rv) {
        // -rv for rv == INT64_MIN is UB in the reference; it only arises with lv < 0 here.
        if (lv > 0 && rv < 0) return rv == minInt ? true : maxInt - lv < -rv;
        if (lv < 0 && rv > 0) return minInt - lv > -rv;
        return false;
    };
    auto isMulOverflow = [](int64_t lv, int64_t rv) {
        if (lv > 0 && rv > 0) return maxInt / lv < rv;
        if (lv < 0 && rv < 0) return maxInt / lv > rv;
        if (lv > 0 && rv < 0) return minInt / lv > rv;
        if (lv < 0 && rv > 0) return minInt / rv > lv;
        return false;
    };
    switch (op_) {
        case ADD:
            if (isArithmetic(l) && isArithmetic(r)) {
                if (isDouble(l) || isDouble(r)) return OptVariant(asDouble(l) + asDouble(r));
                int64_t a = asInt(l), b = asInt(r);
                if (isAddOverflow(a, b)) return Status::Error("Out of range");
                return OptVariant(a + b);
            }
            if (isString(l) && isString(r)) return OptVariant(asString(l) + asString(r));
            break;
        case SUB:
            if (isArithmetic(l) && isArithmetic(r)) {
                if (isDouble(l) || isDouble(r)) return OptVariant(asDouble(l) - asDouble(r));
                int64_t a = asInt(l), b = asInt(r);
                if (isSubOverflow(a, b)) return Status::Error("Out of range");
                return OptVariant(a - b);
            }
            break;
        case MUL:
            if (isArithmetic(l) && isArithmetic(r)) {
                if (isDouble(l) || isDouble(r)) return OptVariant(asDouble(l) * asDouble(r));
                int64_t a = asInt(l), b = asInt(r);
                if (isMulOverflow(a, b)) return Status::Error("Out of range");
                return OptVariant(static_cast<int64_t>(static_cast<uint64_t>(a) * static_cast<uint64_t>(b)));
            }
            break;
        case DIV:
            if (isArithmetic(l) && isArithmetic(r)) {
                if (isDouble(l) || isDouble(r)) {
                    // unqualified abs() on a double (Expressions.cpp:925): taken as std::abs(double).
                    if (std::abs(asDouble(r)) < 1e-8) return Status::Error("Division by zero");
                    return OptVariant(asDouble(l) / asDouble(r));
                }
                int64_t a = asInt(l), b = asInt(r);
                if (b == 0) return Status::Error("Division by zero");
                if (a == minInt && b == -1) return Status::Error("Out of range");
                return OptVariant(a / b);
            }
            break;
        case MOD:
            if (isArithmetic(l) && isArithmetic(r)) {
                if (isDouble(l) || isDouble(r)) {
                    if (std::abs(asDouble(r)) < 1e-8) return Status::Error("Division by zero");
                    return OptVariant(std::fmod(asDouble(l), asDouble(r)));
                }
                if (asInt(r) == 0) return Status::Error("Division by zero");
                if (asInt(r) == -1) return OptVariant(int64_t(0));   // INT64_MIN % -1 traps in the reference
                return OptVariant(asInt(l) % asInt(r));
            }
            break;
        case XOR:
            if (isArithmetic(l) && isArithmetic(r)) {
                if (isDouble(l) || isDouble(r)) {
                    return OptVariant(static_cast<int64_t>(std::round(asDouble(l))) ^
                                      static_cast<int64_t>(std::round(asDouble(r))));
                }
                return OptVariant(asInt(l) ^ asInt(r));
            }
            break;
        default: break;
    }
    return Status::Error("attempt to perform arithmetic");
}

// RelationalExpression::eval (Expressions.cpp:1057-1110) + implicitCasting (:1122-1140)
OptVariant RelationalExpression::eval(Getters& g) const {
    auto left = left_->eval(g);
    auto right = right_->eval(g);
    if (!left.ok()) return left;
    if (!right.ok()) return right;
    Variant l = left.value();
    Variant r = right.value();
    if (which(l) != which(r)) {
        if (which(l) == VAR_STR || which(r) == VAR_STR) {
            return Status::Error("A string type can not be compared with a non-string type.");
        } else if (which(l) == VAR_DOUBLE || which(r) == VAR_DOUBLE) {
            l = toDouble(l); r = toDouble(r);
        } else if (which(l) == VAR_INT64 || which(r) == VAR_INT64) {
            l = toInt(l); r = toInt(r);
        }
    }
    switch (op_) {
        case LT: return OptVariant(l < r);
        case LE: return OptVariant(l <= r);
        case GT: return OptVariant(l > r);
        case GE: return OptVariant(l >= r);
        case EQ:
            if (isArithmetic(l) && isArithmetic(r) && (isDouble(l) || isDouble(r))) {
                return OptVariant(almostEqual(asDouble(l), asDouble(r)));
            }
            return OptVariant(l == r);
        case NE:
            if (isArithmetic(l) && isArithmetic(r) && (isDouble(l) || isDouble(r))) {
                return OptVariant(!almostEqual(asDouble(l), asDouble(r)));
            }
            return OptVariant(l != r);
        case CONTAINS:
            if (isString(l) && isString(r)) {
                return OptVariant(asString(l).find(asString(r)) != std::string::npos);
            }
            break;
        default: break;
    }
    return Status::Error("Wrong operator");
}

// LogicalExpression::eval (Expressions.cpp:1200-1228) — no short circuit.
OptVariant LogicalExpression::eval(Getters& g) const {
    auto left = left_->eval(g);
    auto right = right_->eval(g);
    if (!left.ok()) return left;
    if (!right.ok()) return right;
    if (op_ == AND) {
        if (!asBool(left.value())) return OptVariant(false);
        return OptVariant(asBool(right.value()));
    } else if (op_ == OR) {
        if (asBool(left.value())) return OptVariant(true);
        return OptVariant(asBool(right.value()));
    }
    return OptVariant(asBool(left.value()) != asBool(right.value()));
}

// ---------------------------------------------------------------- FunctionManager
namespace {
struct FuncAttr { size_t minArity, maxArity; Function body; };

// Each body mirrors FunctionManager.cpp:20-555. boost::get on a mismatched argument type throws in
// the reference; here it becomes an error status.
#define ORC_DBL(i) ([&]() -> double { if (!Expression::isArithmetic(args[i])) throw badGet(); return Expression::asDouble(args[i]); }())
#define ORC_INT(i) ([&]() -> int64_t { if (!Expression::isInt(args[i])) throw badGet(); return Expression::asInt(args[i]); }())
#define ORC_STR(i) ([&]() -> std::string { if (!Expression::isString(args[i])) throw badGet(); return Expression::asString(args[i]); }())

Function wrap(std::function<OptVariant(const std::vector<Variant>&)> f) {
    return [f](const std::vector<Variant>& a) -> OptVariant {
        try { return f(a); } catch (const Status& s) { return s; }
    };
}
#define UNARY_MATH(NAME, FN) \
    m[NAME] = {1, 1, wrap([](const std::vector<Variant>& args) -> OptVariant { return OptVariant(FN(ORC_DBL(0))); })}

std::unordered_map<std::string, FuncAttr> buildFunctions() {
    std::unordered_map<std::string, FuncAttr> m;
    UNARY_MATH("abs", std::fabs);
    UNARY_MATH("floor", std::floor);
    UNARY_MATH("ceil", std::ceil);
    UNARY_MATH("round", std::round);
    UNARY_MATH("sqrt", std::sqrt);
    UNARY_MATH("cbrt", std::cbrt);
    UNARY_MATH("exp", std::exp);
    UNARY_MATH("exp2", std::exp2);
    UNARY_MATH("log", std::log);
    UNARY_MATH("log2", std::log2);
    UNARY_MATH("log10", std::log10);
    UNARY_MATH("sin", std::sin);
    UNARY_MATH("asin", std::asin);
    UNARY_MATH("cos", std::cos);
    UNARY_MATH("acos", std::acos);
    UNARY_MATH("tan", std::tan);
    UNARY_MATH("atan", std::atan);
    m["hypot"] = {2, 2, wrap([](const std::vector<Variant>& args) -> OptVariant { return OptVariant(std::hypot(ORC_DBL(0), ORC_DBL(1))); })};
    m["pow"] = {2, 2, wrap([](const std::vector<Variant>& args) -> OptVariant { return OptVariant(std::pow(ORC_DBL(0), ORC_DBL(1))); })};
    m["strcasecmp"] = {2, 2, wrap([](const std::vector<Variant>& args) -> OptVariant {
        return OptVariant(static_cast<int64_t>(::strcasecmp(ORC_STR(0).c_str(), ORC_STR(1).c_str()))); })};
    m["lower"] = {1, 1, wrap([](const std::vector<Variant>& args) -> OptVariant {
        auto v = ORC_STR(0); for (auto& c : v) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c))); return OptVariant(v); })};
    m["upper"] = {1, 1, wrap([](const std::vector<Variant>& args) -> OptVariant {
        auto v = ORC_STR(0); for (auto& c : v) c = static_cast<char>(std::toupper(static_cast<unsigned char>(c))); return OptVariant(v); })};
    m["length"] = {1, 1, wrap([](const std::vector<Variant>& args) -> OptVariant {
        return OptVariant(static_cast<int64_t>(ORC_STR(0).length())); })};
    m["trim"] = {1, 1, wrap([](const std::vector<Variant>& args) -> OptVariant {
        auto v = ORC_STR(0); v.erase(0, v.find_first_not_of(" ")); v.erase(v.find_last_not_of(" ") + 1); return OptVariant(v); })};
    m["ltrim"] = {1, 1, wrap([](const std::vector<Variant>& args) -> OptVariant {
        auto v = ORC_STR(0); v.erase(0, v.find_first_not_of(" ")); return OptVariant(v); })};
    m["rtrim"] = {1, 1, wrap([](const std::vector<Variant>& args) -> OptVariant {
        auto v = ORC_STR(0); v.erase(v.find_last_not_of(" ") + 1); return OptVariant(v); })};
    m["left"] = {2, 2, wrap([](const std::vector<Variant>& args) -> OptVariant {
        auto v = ORC_STR(0); auto n = ORC_INT(1); if (n <= 0) return OptVariant(std::string());
        return OptVariant(v.substr(0, static_cast<size_t>(n))); })};
    m["right"] = {2, 2, wrap([](const std::vector<Variant>& args) -> OptVariant {
        auto v = ORC_STR(0); auto n = ORC_INT(1); if (n <= 0) return OptVariant(std::string());
        if (n > static_cast<int64_t>(v.size())) n = static_cast<int64_t>(v.size());
        return OptVariant(v.substr(v.size() - static_cast<size_t>(n))); })};
    m["lpad"] = {3, 3, wrap([](const std::vector<Variant>& args) -> OptVariant {
        auto v = ORC_STR(0); size_t size = static_cast<size_t>(ORC_INT(1));
        if (size == 0) return OptVariant(std::string(""));
        if (size < v.size()) return OptVariant(v.substr(0, size));
        auto extra = ORC_STR(2); size -= v.size(); std::string s;
        while (size > extra.size()) { s += extra; size -= extra.size(); }
        s += extra.substr(0, size); s += v; return OptVariant(s); })};
    m["rpad"] = {3, 3, wrap([](const std::vector<Variant>& args) -> OptVariant {
        auto v = ORC_STR(0); size_t size = static_cast<size_t>(ORC_INT(1));
        if (size == 0) return OptVariant(std::string(""));
        if (size < v.size()) return OptVariant(v.substr(0, size));
        auto extra = ORC_STR(2); std::string s = v; size -= v.size();
        while (size > extra.size()) { s += extra; size -= extra.size(); }
        s += extra.substr(0, size); return OptVariant(s); })};
    m["substr"] = {3, 3, wrap([](const std::vector<Variant>& args) -> OptVariant {
        auto v = ORC_STR(0); auto start = ORC_INT(1); auto len = ORC_INT(2);
        if (static_cast<size_t>(std::llabs(start)) > v.size() || len <= 0 || start == 0) return OptVariant(std::string(""));
        if (start > 0) return OptVariant(v.substr(static_cast<size_t>(start - 1), static_cast<size_t>(len)));
        return OptVariant(v.substr(v.size() + start, static_cast<size_t>(len))); })};
    m["hash"] = {1, 1, wrap([](const std::vector<Variant>& args) -> OptVariant {   // :439-465 (libstdc++ std::hash)
        switch (which(args[0])) {
            case VAR_INT64: return OptVariant(static_cast<int64_t>(std::hash<int64_t>()(std::get<int64_t>(args[0]))));
            case VAR_DOUBLE: return OptVariant(static_cast<int64_t>(std::hash<double>()(std::get<double>(args[0]))));
            case VAR_BOOL: return OptVariant(static_cast<int64_t>(std::hash<bool>()(std::get<bool>(args[0]))));
            default: return OptVariant(static_cast<int64_t>(std::hash<std::string>()(std::get<std::string>(args[0]))));
        } })};
    m["udf_is_in"] = {2, static_cast<size_t>(INT64_MAX), wrap([](const std::vector<Variant>& args) -> OptVariant {
        const Variant& cmp = args.front();                                             // :467-513
        switch (which(cmp)) {
            case VAR_INT64: {
                for (size_t i = 1; i < args.size(); i++) if (static_cast<uint64_t>(Expression::toInt(args[i])) == static_cast<uint64_t>(std::get<int64_t>(cmp))) return OptVariant(true);
                return OptVariant(false);
            }
            case VAR_DOUBLE: {
                for (size_t i = 1; i < args.size(); i++) if (Expression::toDouble(args[i]) == std::get<double>(cmp)) return OptVariant(true);
                return OptVariant(false);
            }
            case VAR_BOOL: {
                for (size_t i = 1; i < args.size(); i++) if (Expression::toBool(args[i]) == std::get<bool>(cmp)) return OptVariant(true);
                return OptVariant(false);
            }
            default: {
                for (size_t i = 1; i < args.size(); i++) if (Expression::toString(args[i]) == std::get<std::string>(cmp)) return OptVariant(true);
                return OptVariant(false);
            }
        } })};
    m["cos_similarity"] = {2, static_cast<size_t>(INT64_MAX), wrap([](const std::vector<Variant>& args) -> OptVariant {
        if (args.size() % 2 != 0) return OptVariant(-2.0);                             // :528-555
        auto mid = args.size() / 2;
        double s1 = 0, s2 = 0, s3 = 0;
        for (size_t i = 0; i < mid; i++) {
            auto xi = Expression::toDouble(args[i]); auto yi = Expression::toDouble(args[i + mid]);
            s1 += xi * yi; s2 += xi * xi; s3 += yi * yi;
        }
        if (s2 == 0 || s3 == 0) return OptVariant(-2.0);
        return OptVariant(s1 / (std::sqrt(s2) * std::sqrt(s3))); })};
    // rand32/rand64/now are nondeterministic and `near` needs the geo index: not restated.
    return m;
}
}  // namespace

StatusOr<Function> getFunction(const std::string& name, size_t arity) {
    static const auto table = buildFunctions();
    auto it = table.find(name);
    if (it == table.end()) return Status::Error("Function `" + name + "' not defined");
    if (arity < it->second.minArity || arity > it->second.maxArity) return Status::Error("Arity not match");
    return it->second.body;
}

}  // namespace orc
