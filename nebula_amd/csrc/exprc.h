// Expression -> flat device bytecode compiler (the north star's src/common/filter change).
//
// Decodes the reference's binary Expression encoding (src/common/filter/Expressions.cpp:93-116)
// and compiles it for one of two evaluation contexts:
//   STORAGE — the pushed-down filter inside GetNeighbors (QueryBaseProcessor.inl:538-602 getters,
//             checkExp :195-322): any getter failure is an error and the edge is skipped;
//   GRAPHD  — GoExecutor::processFinalResult's WHERE / YIELD (GoExecutor.cpp:1101-1220 getters):
//             other-edge-type props read as defaults, missing tag rows read as defaults, an error
//             fails the query.
// Every schema / alias / tag lookup is resolved at compile time; the device only executes loads,
// type checks and arithmetic (kernels.hip, vmEval).
#pragma once

#include <set>

#include "ngx_internal.h"

namespace ngx {

struct ExprNode {
    uint8_t kind = 0;
    uint8_t op = 0;
    // primary
    uint8_t vtype = 0;           // 0 int, 1 double, 2 bool, 3 string (Expressions.cpp:450-507)
    int64_t i = 0;
    double d = 0;
    std::string s;
    // property refs
    std::string ref, alias, prop;
    // function
    std::string name;
    std::vector<std::unique_ptr<ExprNode>> kids;
};
enum Kind : uint8_t {
    K_PRIMARY = 1, K_FUNC = 2, K_UNARY = 3, K_CAST = 4, K_ARITH = 5, K_REL = 6, K_LOGIC = 7,
    K_SRC_PROP = 8, K_EDGE_RANK = 9, K_EDGE_DST = 10, K_EDGE_SRC = 11, K_EDGE_TYPE = 12, K_ALIAS = 13,
    K_VAR_PROP = 14, K_DST_PROP = 15, K_INPUT_PROP = 16, K_UUID = 17,
};

// returns nullptr and sets err on malformed input
std::unique_ptr<ExprNode> decodeExpr(const uint8_t* buf, size_t len, std::string& err);
std::string encodeExpr(const ExprNode& n);
std::unique_ptr<ExprNode> cloneExpr(const ExprNode& n);
// WhereWrapper::rewrite (src/graph/TraverseExecutor.cpp:461-538); mutates n, returns pushable
bool rewritePushdown(ExprNode& n);
// the props an expression references, like ExpressionContext after prepare()
struct PropRefs {
    std::set<std::pair<std::string, std::string>> srcTag, dstTag, alias;
    bool input = false, variable = false;
    std::set<std::string> vars;                  // $var names (ExpressionContext::variables())
    std::set<std::string> funcs;
};
void collectRefs(const ExprNode& n, PropRefs& r);

struct Program {
    std::vector<Insn> code;
    std::string pool;            // constant strings
    bool usesDstTag = false;
    bool usesSrcTag = false;
    bool empty() const { return code.empty(); }
};

// Storage-side (pushed filter) compile context for one GetNeighbors request
struct StorageCtx {
    const Space* sp = nullptr;
    std::map<std::string, int32_t> edgeMap;      // edge NAME -> |type| of EDGE return columns
    bool haveEdgeContexts = false;
    std::set<int32_t> filterTags;                // tag ids referenced by $^ (checkExp adds contexts)
    bool deviceLibm = false;                     // flag device_libm: inexact libm of row values allowed
};

// Graphd-side compile context for one GO
struct GraphdCtx {
    const Space* sp = nullptr;
    std::map<std::string, int32_t> aliasType;    // expCtx edgeMap: alias -> |type|
    int32_t direction = 0;
    size_t nEdgeTypes = 0;
    // final-hop response schema per signed type: prop name -> type
    std::map<int32_t, std::map<std::string, int32_t>> respSchema;
    bool deviceLibm = false;                     // flag device_libm: inexact libm of row values allowed
    // $-.x / $var.x read from the pipe's input table (OP_INPUT: column index); null: outside the fast path
    const std::map<std::string, int32_t>* inputCols = nullptr;
};

// Compile. Returns NGX_OK, NGX_E_INVALID_FILTER (storage checkExp failure), NGX_E_UNSUPPORTED, or
// NGX_E_QUERY (graphd prepare failure).
int32_t compileStorage(const ExprNode& n, StorageCtx& ctx, Program& out, std::string& err);
int32_t compileGraphd(const ExprNode& n, GraphdCtx& ctx, Program& out, std::string& err);


// TraverseExecutor::calculateExprType (src/graph/TraverseExecutor.cpp:88-165)
int32_t exprType(const ExprNode& n, const Space& sp);

}  // namespace ngx
