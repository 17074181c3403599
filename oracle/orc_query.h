// ORACLE — TEST INFRASTRUCTURE ONLY (see orc_core.h header).
// Wire types of the boundary (src/interface/storage.thrift:62-187) and the restated
// QueryBoundProcessor / QueryVertexPropsProcessor / GoExecutor.
#pragma once

#include "orc_expr.h"
#include "orc_store.h"

namespace orc {

enum ErrorCode : int32_t {                // storage.thrift:13-59 (subset used on this path)
    SUCCEEDED = 0, E_LEADER_CHANGED = -11, E_SPACE_NOT_FOUND = -13, E_PART_NOT_FOUND = -14,
    E_KEY_NOT_FOUND = -15, E_EDGE_PROP_NOT_FOUND = -21, E_TAG_PROP_NOT_FOUND = -22,
    E_IMPROPER_DATA_TYPE = -23, E_EDGE_NOT_FOUND = -24, E_TAG_NOT_FOUND = -25,
    E_INVALID_FILTER = -31, E_UNKNOWN = -100,
};
enum PropOwner : int32_t { SOURCE = 1, DEST = 2, EDGE = 3 };

struct PropDef {
    PropOwner owner;
    int32_t id;            // tag id (SOURCE/DEST) or signed edge type (EDGE)
    std::string name;
};
struct GetNeighborsRequest {
    GraphSpaceID space = 0;
    std::vector<std::pair<PartitionID, std::vector<VertexID>>> parts;
    std::vector<EdgeType> edge_types;
    bool has_edge_types = true;
    std::string filter;
    std::vector<PropDef> return_columns;
};
struct IdAndProp { VertexID dst = 0; std::string props; bool has_props = false; };
struct EdgeData { EdgeType type; std::vector<IdAndProp> edges; };
struct TagData { TagID tag_id; std::string data; };
struct VertexData { VertexID vertex_id; std::vector<TagData> tag_data; std::vector<EdgeData> edge_data; };
struct QueryResponse {
    std::vector<std::pair<int32_t, PartitionID>> failed_codes;      // (code, part)
    std::map<TagID, std::shared_ptr<Schema>> vertex_schema;
    std::map<EdgeType, std::shared_ptr<Schema>> edge_schema;
    std::vector<VertexData> vertices;
    int32_t total_edges = 0;
    int64_t scanned = 0;                   // harness: keys under the requested (vertex, type) prefixes (TEPS)
};

struct StorageFlags {                      // QueryBaseProcessor.cpp:9-13 defaults
    int32_t max_handlers_per_req = 10;
    int32_t min_vertices_per_bucket = 3;
    int32_t max_edge_returned_per_vertex = INT32_MAX;
    int64_t now_sec = 0;                   // WallClock::fastNowInSec() — fixed for determinism
    int32_t threads = 1;                   // reader-pool threads used to run buckets
    int32_t graph_threads = 1;             // test harness: threads of processFinalResult (GoFlags::threads)
};

class StorageEngine {
 public:
    SchemaManager schemas;
    std::map<GraphSpaceID, KVStore> stores;
    StorageFlags flags;
    QueryResponse getBound(const GetNeighborsRequest& req, bool onlyVertexProps = false) const;
    // genBuckets arithmetic (QueryBaseProcessor.inl:632-667)
    static std::vector<std::vector<std::pair<PartitionID, VertexID>>> genBuckets(
        const GetNeighborsRequest& req, int32_t minVerticesPerBucket, int32_t maxHandlers);
};

// ------------------------------------------------------------------ GO
struct GoYield { std::string expr; std::string alias; };
struct GoSentence {
    uint32_t recordFrom = 1, recordTo = 1;
    std::vector<VertexID> vids;
    std::vector<std::pair<std::string, std::string>> over;    // (edge name, alias or "")
    bool overAll = false;
    int direction = 0;                                        // 0 forward, 1 REVERSELY, 2 BIDIRECT
    bool hasWhere = false;
    std::string where;                                        // encoded Expression
    bool distinct = false;
    std::vector<GoYield> yields;                              // the parser's default is <edge>._dst
    // FROM $-.col / $var.col (fromType_ kPipe / kVariable, GoExecutor.cpp:149-180): the interim
    // result of the previous sentence (InterimResult: column names, schema types, rows)
    int fromType = 0;                                         // 0 literal vids, 1 $-, 2 $var
    std::string fromVar, fromCol;
    std::vector<std::string> inputNames;
    std::vector<SupportedType> inputTypes;
    std::vector<std::vector<Variant>> inputRows;
};
struct GoResult {
    bool ok = true;
    std::string error;
    std::vector<std::string> columnNames;
    std::vector<SupportedType> colTypes;                      // calculateExprType
    std::vector<std::vector<Variant>> rows;
    std::vector<int64_t> hopScanned;                          // edges scanned per hop (stats)
    std::vector<int64_t> hopFrontier;
    // GoFlags::digest set: one 16-byte digest per result row instead of `rows' (rowCount rows)
    std::string digests;
    uint64_t rowCount = 0;
};
// Test-harness knobs (not reference flags): `threads' > 1 splits processFinalResult's rows over threads
// in contiguous vertex ranges, rows concatenated in the sequential order (no DISTINCT, literal FROM);
// `digest' turns every result row into a 16-byte digest as it is produced (large-result comparison).
using RowDigestFn = void (*)(const std::vector<SupportedType>& colTypes, const std::vector<Variant>& row, uint8_t* out16);
struct GoFlags {
    bool filter_pushdown = true;
    int threads = 1;
    RowDigestFn digest = nullptr;
};

GoResult runGo(const StorageEngine& eng, GraphSpaceID space, const GoSentence& s, const GoFlags& f);

// WhereWrapper::rewrite / canPushdown (src/graph/TraverseExecutor.cpp:461-538)
bool rewriteForPushdown(Expression* expr);

}  // namespace orc
