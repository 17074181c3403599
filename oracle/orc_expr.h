// ORACLE — TEST INFRASTRUCTURE ONLY (see orc_core.h header).
// Restates src/common/filter/Expressions.{h,cpp} (AST, binary encode/decode, eval) and
// src/common/filter/FunctionManager.cpp (built-in functions).
#pragma once

#include <set>
#include "orc_core.h"

namespace orc {

enum class ColumnType : uint8_t { INT, STRING, DOUBLE, BOOL, TIMESTAMP };   // Expressions.h:22-24

// Getters (Expressions.h:29-37)
struct Getters {
    std::function<OptVariant()> getEdgeRank;
    std::function<OptVariant(const std::string&)> getInputProp;
    std::function<OptVariant(const std::string&)> getVariableProp;
    std::function<OptVariant(const std::string&, const std::string&)> getSrcTagProp;
    std::function<OptVariant(const std::string&, const std::string&)> getDstTagProp;
    std::function<OptVariant(const std::string&, const std::string&)> getAliasProp;
    std::function<OptVariant(const std::string&)> getEdgeDstId;
};

// ExpressionContext (Expressions.h:39-192) — the prop bookkeeping used by GoExecutor/WhereWrapper.
struct ExpressionContext {
    std::set<std::pair<std::string, std::string>> srcTagProps, dstTagProps, aliasProps, variableProps;
    std::set<std::string> variables, inputProps;
    std::map<std::string, EdgeType> edgeMap;
    std::map<std::string, TagID> tagMap;
    std::vector<std::string> edgeAlias;
    bool overAll = false;
    void addSrcTagProp(const std::string& t, const std::string& p) { tagMap.emplace(t, -1); srcTagProps.emplace(t, p); }
    void addDstTagProp(const std::string& t, const std::string& p) { tagMap.emplace(t, -1); dstTagProps.emplace(t, p); }
    void addVariableProp(const std::string& v, const std::string& p) { variableProps.emplace(v, p); variables.emplace(v); }
    void addInputProp(const std::string& p) { inputProps.emplace(p); }
    void addAliasProp(const std::string& a, const std::string& p) { aliasProps.emplace(a, p); }
    bool addEdge(const std::string& alias, EdgeType t) {
        if (edgeMap.count(alias)) return false;
        edgeMap.emplace(alias, t); edgeAlias.push_back(alias); return true;
    }
    bool getEdgeType(const std::string& alias, EdgeType& t) const {
        auto it = edgeMap.find(alias);
        if (it == edgeMap.end()) return false;
        t = it->second; return true;
    }
    bool getTagId(const std::string& tag, TagID& id) const {
        auto it = tagMap.find(tag);
        if (it == tagMap.end() || it->second < 0) return false;
        id = it->second; return true;
    }
    bool hasSrcTagProp() const { return !srcTagProps.empty(); }
    bool hasDstTagProp() const { return !dstTagProps.empty(); }
    bool hasEdgeProp() const { return !aliasProps.empty(); }
    bool hasVariableProp() const { return !variableProps.empty(); }
    bool hasInputProp() const { return !inputProps.empty(); }
};

using Function = std::function<OptVariant(const std::vector<Variant>&)>;
// FunctionManager::get (FunctionManager.cpp:560-589)
StatusOr<Function> getFunction(const std::string& name, size_t arity);

class Expression {
 public:
    enum Kind : uint8_t {                                          // Expressions.h:386-407
        kUnknown = 0, kPrimary, kFunctionCall, kUnary, kTypeCasting, kArithmetic, kRelational,
        kLogical, kSourceProp, kEdgeRank, kEdgeDstId, kEdgeSrcId, kEdgeType, kAliasProp,
        kVariableProp, kDestProp, kInputProp, kUUID, kMax,
    };
    virtual ~Expression() = default;
    Kind kind() const { return kind_; }
    virtual OptVariant eval(Getters& g) const = 0;
    virtual Status prepare(ExpressionContext* ctx) = 0;
    virtual void encode(std::string& out) const = 0;
    virtual const char* decode(const char* pos, const char* end) = 0;   // throws Status
    virtual void traversal(const std::function<void(const Expression*)>& v) const = 0;
    virtual std::unique_ptr<Expression> clone() const = 0;
    virtual std::string toString() const = 0;

    static std::string encode(const Expression* e) { std::string s; e->encode(s); return s; }
    static StatusOr<std::shared_ptr<Expression>> decode(const std::string& buf);
    static std::unique_ptr<Expression> makeExpr(uint8_t kind);

    // Expressions.h:261-382 value helpers
    static int64_t asInt(const Variant& v) { return std::get<int64_t>(v); }
    static double asDouble(const Variant& v) {
        if (which(v) == VAR_INT64) return static_cast<double>(std::get<int64_t>(v));
        return std::get<double>(v);
    }
    static bool asBool(const Variant& v) {
        switch (which(v)) {
            case VAR_INT64: return asInt(v) != 0;
            case VAR_DOUBLE: return asDouble(v) != 0.0;
            case VAR_BOOL: return std::get<bool>(v);
            case VAR_STR: return std::get<std::string>(v).empty();
        }
        return false;
    }
    static const std::string& asString(const Variant& v) { return std::get<std::string>(v); }
    static bool isInt(const Variant& v) { return which(v) == VAR_INT64; }
    static bool isDouble(const Variant& v) { return which(v) == VAR_DOUBLE; }
    static bool isBool(const Variant& v) { return which(v) == VAR_BOOL; }
    static bool isString(const Variant& v) { return which(v) == VAR_STR; }
    static bool isArithmetic(const Variant& v) { return isInt(v) || isDouble(v); }
    static bool almostEqual(double l, double r) { return std::abs(l - r) < 1e-8; }
    static std::string toString(const Variant& v);
    static bool toBool(const Variant& v) { return asBool(v); }
    static double toDouble(const Variant& v);
    static int64_t toInt(const Variant& v);

 protected:
    Kind kind_{kUnknown};
};
using ExprPtr = std::unique_ptr<Expression>;

// Alias.prop and its $-, $$, $var, _type/_src/_dst/_rank, $^ relatives (Expressions.h:459-654)
class AliasPropertyExpression : public Expression {
 public:
    AliasPropertyExpression() { kind_ = kAliasProp; }
    AliasPropertyExpression(std::string ref, std::string alias, std::string prop)
        : ref_(std::move(ref)), alias_(std::move(alias)), prop_(std::move(prop)) { kind_ = kAliasProp; }
    OptVariant eval(Getters& g) const override;
    Status prepare(ExpressionContext* ctx) override;
    void encode(std::string& out) const override;
    const char* decode(const char* pos, const char* end) override;
    void traversal(const std::function<void(const Expression*)>& v) const override { v(this); }
    ExprPtr clone() const override;
    std::string toString() const override;
    const std::string& alias() const { return alias_; }
    const std::string& prop() const { return prop_; }
    const std::string& ref() const { return ref_; }
    void setKind(Kind k) { kind_ = k; }
 protected:
    std::string ref_, alias_, prop_;
};

class PrimaryExpression : public Expression {
 public:
    PrimaryExpression() { kind_ = kPrimary; }
    explicit PrimaryExpression(Variant v) : v_(std::move(v)) { kind_ = kPrimary; }
    OptVariant eval(Getters&) const override { return OptVariant(v_); }
    Status prepare(ExpressionContext*) override { return Status::OK(); }
    void encode(std::string& out) const override;
    const char* decode(const char* pos, const char* end) override;
    void traversal(const std::function<void(const Expression*)>& v) const override { v(this); }
    ExprPtr clone() const override { return std::make_unique<PrimaryExpression>(v_); }
    std::string toString() const override;
    const Variant& value() const { return v_; }
 private:
    Variant v_;
};

class FunctionCallExpression : public Expression {
 public:
    FunctionCallExpression() { kind_ = kFunctionCall; }
    OptVariant eval(Getters& g) const override;
    Status prepare(ExpressionContext* ctx) override;
    void encode(std::string& out) const override;
    const char* decode(const char* pos, const char* end) override;
    void traversal(const std::function<void(const Expression*)>& v) const override {
        for (auto& a : args_) a->traversal(v);
        v(this);
    }
    ExprPtr clone() const override;
    std::string toString() const override;
    const std::string& name() const { return name_; }
    const std::vector<ExprPtr>& args() const { return args_; }
    void setFunc(Function f) { func_ = std::move(f); }
    std::string name_;
    std::vector<ExprPtr> args_;
 private:
    Function func_;
};

class UnaryExpression : public Expression {
 public:
    enum Operator : uint8_t { PLUS, NEGATE, NOT };
    UnaryExpression() { kind_ = kUnary; }
    OptVariant eval(Getters& g) const override;
    Status prepare(ExpressionContext* ctx) override { return operand_->prepare(ctx); }
    void encode(std::string& out) const override;
    const char* decode(const char* pos, const char* end) override;
    void traversal(const std::function<void(const Expression*)>& v) const override { operand_->traversal(v); v(this); }
    ExprPtr clone() const override;
    std::string toString() const override;
    Operator op_ = PLUS;
    ExprPtr operand_;
};

class TypeCastingExpression : public Expression {
 public:
    TypeCastingExpression() { kind_ = kTypeCasting; }
    OptVariant eval(Getters& g) const override;
    Status prepare(ExpressionContext* ctx) override { return operand_->prepare(ctx); }
    void encode(std::string& out) const override;
    const char* decode(const char* pos, const char* end) override;
    void traversal(const std::function<void(const Expression*)>& v) const override { operand_->traversal(v); v(this); }
    ExprPtr clone() const override;
    std::string toString() const override;
    ColumnType type_ = ColumnType::INT;
    ExprPtr operand_;
};

class BinaryExpression : public Expression {
 public:
    Status prepare(ExpressionContext* ctx) override {
        auto s = left_->prepare(ctx);
        if (!s.ok()) return s;
        return right_->prepare(ctx);
    }
    void encode(std::string& out) const override;
    const char* decode(const char* pos, const char* end) override;
    void traversal(const std::function<void(const Expression*)>& v) const override {
        left_->traversal(v); right_->traversal(v); v(this);
    }
    uint8_t op_ = 0;
    ExprPtr left_, right_;
};

class ArithmeticExpression : public BinaryExpression {
 public:
    enum Operator : uint8_t { ADD, SUB, MUL, DIV, MOD, XOR };
    ArithmeticExpression() { kind_ = kArithmetic; }
    OptVariant eval(Getters& g) const override;
    ExprPtr clone() const override;
    std::string toString() const override;
};

class RelationalExpression : public BinaryExpression {
 public:
    enum Operator : uint8_t { LT, LE, GT, GE, EQ, NE, CONTAINS };
    RelationalExpression() { kind_ = kRelational; }
    OptVariant eval(Getters& g) const override;
    ExprPtr clone() const override;
    std::string toString() const override;
};

class LogicalExpression : public BinaryExpression {
 public:
    enum Operator : uint8_t { AND, OR, XOR };
    LogicalExpression() { kind_ = kLogical; }
    OptVariant eval(Getters& g) const override;
    Status prepare(ExpressionContext* ctx) override {       // Expressions.cpp:1240-1247
        auto s = left_->prepare(ctx);
        if (!s.ok()) return s;
        (void)right_->prepare(ctx);                         // result ignored by the reference
        return Status::OK();
    }
    ExprPtr clone() const override;
    std::string toString() const override;
};

}  // namespace orc
