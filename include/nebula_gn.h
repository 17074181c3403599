/*
 * nebula_gn.h — C ABI of the MI355X GetNeighbors / GO engine (libnebula_gn.so).
 *
 * Drop-in boundary for the storage-side neighbor expansion + property filter of NebulaGraph v1
 * (the reference at /root/reference) and the graphd GoExecutor multi-hop driver. Plain C types
 * only; no exceptions cross it; every call returns an int32 status whose negative values are the
 * reference's storage.thrift ErrorCode numbers (src/interface/storage.thrift:13-59) or the
 * NGX_E_* codes below. One in-flight call per ngx_ctx (calls on one context are serialized by an
 * internal mutex). The context owns one HIP device and one stream; with world > 1 it also owns an
 * RCCL communicator whose ranks are the GPUs of one node (one process per GPU).
 *
 * Reference interfaces replaced (file:line in /root/reference):
 *   ngx_open / ngx_close        StorageServer::start + NebulaStore instance (src/storage/StorageServer.cpp:99-168)
 *   ngx_add_space / _schema     meta::SchemaManager::getTagSchema/getEdgeSchema/toEdgeType/toTagID
 *                               (src/meta/SchemaManager.h:18-56) and partsNum (StorageClient.h:292-295)
 *   ngx_load_kv / ngx_commit    the part -> CSR snapshot export: KVStore::prefix over a part
 *                               (src/kvstore/KVStore.h:108-111, NebulaStore.cpp:451-464) as dumped by
 *                               DumpEdgesTool (src/tools/dump-edges/DumpEdgesTool.cpp:17-50)
 *   ngx_load_csr                a bulk-built shard (spark-sstfile-generator + ingest's role: offline
 *                               tabular data -> the store, src/tools/spark-sstfile-generator)
 *   ngx_load_snapshot_rows      a part's raft snapshot stream: SnapshotManagerImpl::accessAllRowsInSnapshot
 *                               rows (src/kvstore/SnapshotManagerImpl.cpp:15-53) as Part::commitSnapshot
 *                               applies them (src/kvstore/Part.cpp:319-344), encodeKV records
 *   ngx_save/open_snapshot      RocksEngine::createCheckpoint (src/kvstore/RocksEngine.cpp:433-480) for the
 *                               device copy: a named, versioned file of the committed shard
 *   ngx_get_neighbors           QueryBoundProcessor::process (src/storage/query/QueryBaseProcessor.inl:800-855,
 *                               src/storage/query/QueryBoundProcessor.cpp:18-261), invoked from
 *                               StorageServiceHandler::future_getBound (src/storage/StorageServiceHandler.cpp:45-53)
 *   ngx_go                      GoExecutor::execute .. toThriftResponse (src/graph/GoExecutor.cpp:92-838, 1082-1335)
 *   ngx_*_free                  results are library-allocated, host-visible, freed only by the library
 */
#ifndef NEBULA_GN_H_
#define NEBULA_GN_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes: 0 ok, reference ErrorCode values, and these */
#define NGX_OK 0
#define NGX_E_INVALID_FILTER (-31)      /* storage.thrift E_INVALID_FILTER */
#define NGX_E_EDGE_PROP_NOT_FOUND (-21)
#define NGX_E_TAG_PROP_NOT_FOUND (-22)
#define NGX_E_IMPROPER_DATA_TYPE (-23)
#define NGX_E_EDGE_NOT_FOUND (-24)
#define NGX_E_TAG_NOT_FOUND (-25)
#define NGX_E_SPACE_NOT_FOUND (-13)
#define NGX_E_PART_NOT_FOUND (-14)      /* a part this shard does not hold (per-part failed code) */
#define NGX_E_BAD_ARGUMENT (-1001)
#define NGX_E_UNSUPPORTED (-1002)       /* a construct the device path does not implement */
#define NGX_E_QUERY (-1003)             /* graphd-side evaluation error (GoExecutor doError) */
#define NGX_E_DEVICE (-1004)            /* HIP / RCCL failure */
#define NGX_E_NOT_LOADED (-1005)
#define NGX_E_SNAPSHOT (-1006)          /* snapshot file unreadable, corrupt, or of another space / shard / schema */

/* SupportedType (src/interface/common.thrift:30-56) */
#define NGX_T_BOOL 1
#define NGX_T_INT 2
#define NGX_T_VID 3
#define NGX_T_FLOAT 4
#define NGX_T_DOUBLE 5
#define NGX_T_STRING 6
#define NGX_T_TIMESTAMP 21

typedef struct ngx_ctx ngx_ctx;

/* Host-side collective for world > 1 in place of RCCL (rehearsal hook: ranks that share one GPU,
 * e.g. torch.distributed gloo in the multi-shard tests). `bytes` is the block size per rank:
 *   NGX_XCHG_ALLGATHER: send = 1 block, recv = world blocks in rank order;
 *   NGX_XCHG_ALLTOALL:  send = world blocks (block q goes to rank q), recv = world blocks (block q
 *                       came from rank q); the rank's own block is ignored.
 * Returns 0 on success. Every rank calls it the same number of times with the same op and bytes. */
#define NGX_XCHG_ALLGATHER 0
#define NGX_XCHG_ALLTOALL 1
typedef int32_t (*ngx_exchange_fn)(void* user, int32_t op, const void* send, void* recv, uint64_t bytes);

typedef struct {
    int32_t device;               /* HIP device ordinal */
    int32_t rank;                 /* this shard (GPU) 0..world-1 */
    int32_t world;                /* shards on the node (1..64); part p lives on shard p % world */
    const void* nccl_unique_id;   /* 128-byte ncclUniqueId when world > 1 and no host exchange */
    ngx_exchange_fn exchange;     /* optional: host collective instead of RCCL (may be NULL) */
    void* exchange_user;
} ngx_config;

int32_t ngx_open(const ngx_config* cfg, ngx_ctx** out);
void ngx_close(ngx_ctx* ctx);
const char* ngx_last_error(ngx_ctx* ctx);
/* "src_sha=<16 hex> arch=gfx950 built=<date time>": src_sha digests every library source (Makefile
 * SRCS), so a run can check that the library it loaded was built from the sources beside it */
const char* ngx_build_info(void);
/* rank 0 calls this and broadcasts the 128 bytes to the other ranks before ngx_open */
int32_t ngx_get_unique_id(void* out128);

/* ---------------------------------------------------------------- schema registry */
int32_t ngx_add_space(ngx_ctx* ctx, int32_t space, int32_t num_parts);
int32_t ngx_add_schema(ngx_ctx* ctx, int32_t space, int32_t is_edge, int32_t id, const char* name,
                       int64_t version, int32_t nfields, const char* const* field_names,
                       const int32_t* field_types, const char* ttl_col, int64_t ttl_duration);

/* ---------------------------------------------------------------- snapshot export */
typedef struct {
    uint64_t n;                   /* rows */
    const uint8_t* keys;          /* reference NebulaKeyUtils keys, concatenated */
    const uint64_t* key_off;      /* n + 1 offsets into keys */
    const uint8_t* vals;          /* RowWriter values, concatenated */
    const uint64_t* val_off;      /* n + 1 offsets into vals */
} ngx_kv_batch;

/* Stage rows; rows of parts this shard does not own are dropped. May be called repeatedly. */
int32_t ngx_load_kv(ngx_ctx* ctx, int32_t space, const ngx_kv_batch* batch);
/* Build the per-part CSR + columnar props from the staged rows and upload them to HBM.
 * Collective when world > 1 (vertex tables are exchanged to resolve destination rows). */
int32_t ngx_commit(ngx_ctx* ctx, int32_t space);

/* Stage one part's snapshot stream: `rows` holds back-to-back records in the reference's encodeKV
 * layout (src/kvstore/LogEncoder.cpp:16-27): u32 key size, u32 value size, key bytes, value bytes,
 * as SnapshotManagerImpl streams a part (prefix iteration over snapshotPrefix(part)). Keys that are not
 * vertex / edge data (system, uuid keys) are skipped at commit; rows of parts this shard does not own
 * are dropped. NGX_E_BAD_ARGUMENT (nothing staged) if the last record is truncated. */
int32_t ngx_load_snapshot_rows(ngx_ctx* ctx, int32_t space, const uint8_t* rows, uint64_t len);

/* Columnar bulk load of this shard's edges, in place of KV rows: the snapshot an offline bulk tool
 * builds from tabular data (the role of the reference's spark-sstfile-generator + ingest,
 * src/tools/spark-sstfile-generator, src/storage/admin), in the form ngx_commit's export would give
 * the same edges' KV rows. The next ngx_commit uses it and drops any staged rows; the commit is
 * collective as usual. Checked, NGX_E_BAD_ARGUMENT otherwise: the vertex table is sorted by (part, vid)
 * without duplicates, part = ID_HASH(vid) and part % world == rank; offsets start at 0 and never
 * decrease; within a vertex row the edges are in RocksDB key order (rank LE bytes, then dst LE bytes)
 * with no (rank, dst) twice (one version per edge); slots have distinct signed types with a schema.
 * Columns are the latest schema's fields in order (STRING: NGX_E_UNSUPPORTED, load KV rows). Tags
 * of the space get no rows. */
typedef struct {
    int32_t etype;                /* signed edge type (-t: in-edges of t, stored under the dst's part) */
    const uint64_t* off;          /* nvertices + 1: the edges of vertex row r are [off[r], off[r + 1]) */
    const int64_t* dst;           /* off[nvertices] destination vids */
    const int64_t* rank;          /* NULL: rank 0 for every edge */
    int32_t ncols;
    const int64_t* const* cols;   /* per field: INT / TIMESTAMP / VID values, FLOAT / DOUBLE as double
                                   * bits, BOOL 0 / 1 */
} ngx_csr_slot;
typedef struct {
    uint64_t nvertices;
    const int32_t* vpart;
    const int64_t* vid;
    int32_t nslots;
    const ngx_csr_slot* slots;
} ngx_csr_shard;
int32_t ngx_load_csr(ngx_ctx* ctx, int32_t space, const ngx_csr_shard* shard);

/* Device snapshot file of the committed shard (CSR, destination rows, prop and tag columns), so a
 * restart skips the KV decode. `tag` (<= 63 bytes) names the checkpoint. ngx_open_snapshot needs the
 * space added with the same num_parts and identical schemas (digest), the same rank / world, and
 * replaces any committed data of the space; tag_out (64 bytes, may be NULL) receives the tag. A file
 * that fails any check returns NGX_E_SNAPSHOT and leaves the space as it was. */
int32_t ngx_save_snapshot(ngx_ctx* ctx, int32_t space, const char* path, const char* tag);
int32_t ngx_open_snapshot(ngx_ctx* ctx, int32_t space, const char* path, char* tag_out);

typedef struct {
    uint64_t vertices;            /* rows in this shard's vertex table */
    uint64_t edges;               /* CSR edges over all edge-type slots (after version dedup) */
    uint64_t device_bytes;        /* HBM held by the snapshot */
    int32_t slots;                /* signed edge types present */
    int32_t tags;
} ngx_graph_info;
int32_t ngx_graph_info_get(ngx_ctx* ctx, int32_t space, ngx_graph_info* out);

/* ---------------------------------------------------------------- result cells */
/* One typed value, mirroring graph.thrift ColumnValue (src/interface/graph.thrift:80-127) as set
 * by GoExecutor::toThriftResponse (GoExecutor.cpp:775-829). */
#define NGX_CELL_EMPTY 0
#define NGX_CELL_BOOL 1
#define NGX_CELL_INT 2
#define NGX_CELL_ID 3
#define NGX_CELL_FLOAT 4
#define NGX_CELL_DOUBLE 5
#define NGX_CELL_STR 6
#define NGX_CELL_TIMESTAMP 21
typedef struct {
    int32_t kind;                 /* NGX_CELL_* */
    int32_t str_len;              /* for NGX_CELL_STR; 1 on an EMPTY cell that holds a bool in v.i (a bool
                                   * of an UNKNOWN-typed YIELD column: toThriftResponse leaves it unset,
                                   * the interim result of a pipe keeps it) */
    union { int64_t i; double d; uint64_t str_off; } v;   /* str_off indexes the result's strings */
} ngx_cell;

/* ---------------------------------------------------------------- GetNeighbors */
typedef struct {
    int32_t owner;                /* PropOwner: 1 SOURCE, 2 DEST, 3 EDGE (storage.thrift:62-83) */
    int32_t id;                   /* tag id, or signed edge type */
    const char* name;
} ngx_prop_def;

typedef struct {
    int32_t space;
    int32_t nparts;
    const int32_t* parts;         /* part id of each group */
    const uint32_t* part_nvids;   /* vids per group */
    const int64_t* vids;          /* all vids, group after group */
    int32_t nedge_types;
    const int32_t* edge_types;    /* signed: > 0 out-edges, < 0 in-edges */
    const uint8_t* filter;        /* Expression::encode bytes, may be empty */
    uint32_t filter_len;
    int32_t ncols;
    const ngx_prop_def* cols;     /* return_columns */
    int32_t max_edges_per_vertex; /* FLAGS_max_edge_returned_per_vertex, <= 0 or INT32_MAX: unlimited */
    int64_t now_sec;              /* clock for TTL (WallClock::fastNowInSec); <= 0: the current time */
    int32_t encode_rows;          /* 1: also return the QueryResponse payload (RowWriter rows, schemas) */
} ngx_gn_request;

/* One response schema of a QueryResponse (common.thrift Schema): columns in order. */
typedef struct {
    int32_t is_edge;              /* 1: edge_schema[id] (signed edge type), 0: vertex_schema[id] (tag) */
    int32_t id;
    int32_t ncols;
    const char* const* names;
    const int32_t* types;         /* NGX_T_* */
} ngx_schema_def;

typedef struct {
    int32_t code;                 /* NGX_OK, or the code pushed for every part (checkAndBuildContexts) */
    int32_t nfailed;
    const int32_t* failed_codes;  /* (code, part) pairs */
    uint64_t nedges;              /* total_edges */
    const uint32_t* edge_vertex;  /* request vid index of each returned edge */
    const int32_t* edge_type;
    const int64_t* edge_dst;
    int32_t ncols;                /* = request ncols; cells[e * ncols + c]; SOURCE/DEST cols are per vertex */
    const ngx_cell* edge_cells;
    uint32_t nvertices;           /* request vids (duplicates included) */
    const ngx_cell* vertex_cells; /* vertex_cells[v * ncols + c] for SOURCE columns; EMPTY if no tag row */
    const uint8_t* vertex_has_tag;/* [v * ncols + c] 1 if the vertex has that tag row */
    const char* strings;
    uint64_t strings_len;
    /* encode_rows: the wire payload of QueryResponse (storage.thrift:112-151), byte-exact with the
     * reference processor. Edge e's IdAndProp.props is edge_props[edge_props_off[e] ..
     * edge_props_off[e + 1]): a RowWriter row (src/dataman/RowWriter.cpp:48-87) of the response
     * schema of its type, encoded on the device; an empty range for a type returning only _dst
     * (onlyStructure: props unset). TagData rows (QueryBoundProcessor.cpp:175-204): tag_row_vertex[k]
     * (request vid index), tag_row_tag[k], data = tag_props[tag_props_off[k] .. tag_props_off[k + 1]),
     * in request-vid order, tags in response order per vertex. */
    const uint8_t* edge_props;
    const uint64_t* edge_props_off;   /* nedges + 1 */
    int32_t nschemas;                 /* edge_schema entries, then vertex_schema entries */
    const ngx_schema_def* schemas;
    uint32_t ntag_rows;
    const uint32_t* tag_row_vertex;
    const int32_t* tag_row_tag;
    const uint8_t* tag_props;
    const uint64_t* tag_props_off;    /* ntag_rows + 1 */
    int64_t latency_in_us;            /* ResponseCommon.latency_in_us (BaseProcessor.h:51-60): the call's
                                       * wall time on the host, entry to result */
} ngx_gn_result;

int32_t ngx_get_neighbors(ngx_ctx* ctx, const ngx_gn_request* req, ngx_gn_result** out);
void ngx_gn_result_free(ngx_gn_result* r);

/* ---------------------------------------------------------------- GO */
#define NGX_DIR_FORWARD 0
#define NGX_DIR_REVERSELY 1
#define NGX_DIR_BIDIRECT 2

typedef struct {
    int32_t space;
    uint32_t record_from, record_to;   /* StepClause: GO [M TO] N STEPS */
    uint64_t nstarts;
    const int64_t* starts;             /* FROM vids (evaluated) */
    int32_t nover;
    const char* const* over_names;     /* edge names */
    const char* const* over_aliases;   /* alias or NULL/"" */
    int32_t over_all;                  /* OVER * */
    int32_t direction;                 /* NGX_DIR_* */
    const uint8_t* where;              /* encoded WHERE, may be NULL */
    uint32_t where_len;
    int32_t nyields;
    const uint8_t* const* yields;      /* encoded YIELD expressions */
    const uint32_t* yield_lens;
    int32_t distinct;                  /* YIELD DISTINCT */
    int32_t filter_pushdown;           /* FLAGS_filter_pushdown */
    int64_t now_sec;                   /* clock for TTL; <= 0: the current time */
    int32_t result_on_device;          /* 1: leave rows in HBM (dev_* below), no host cells / DISTINCT */
    int32_t host_columnar;             /* 1 (host results): columnar host arrays (host_cols), no cells */
    /* FROM $-.col / $var.col: the interim result of the previous sentence (pipe, GoExecutor fromType_
     * kPipe / kVariable, GoExecutor.cpp:149-180, :471-509). input_vid_col == NULL: FROM takes `starts'.
     * The rows are the InterimResult's rows (InterimResult.cpp:178-280); `$-.x' / `$var.x' in WHERE and
     * YIELD read the input row(s) behind each edge row (getRoots + rowsOfVids, GoExecutor.cpp:1317-1330):
     * one output row per (edge row, input row whose FROM column holds a root of the edge). Results come
     * back as host cells (result_on_device and host_columnar are refused). */
    const char* input_vid_col;         /* the FROM column */
    const char* input_var;             /* variable name for FROM $var.col; NULL / "" for $- */
    int32_t input_ncols;
    const char* const* input_names;    /* column names (YIELD aliases or expression text) */
    const int32_t* input_types;        /* NGX_T_* column types of the interim schema */
    uint64_t input_nrows;
    const ngx_cell* input_cells;       /* [row * input_ncols + col]; NGX_CELL_STR: str_off into input_strings */
    const char* input_strings;
    /* result_on_device without DISTINCT: 1 = write only the row arrays a YIELD column aliases
     * (dev_src / dev_dst / dev_rank NULL otherwise). The reference's response holds the YIELD
     * columns alone (GoExecutor::toThriftResponse); the row arrays are this library's extra. */
    int32_t yield_only;
    /* result_on_device without DISTINCT: 1 = compact integer results. The row arrays and every YIELD
     * column that copies one stored integer column (INT / TIMESTAMP / VID, of the only OVER type, present
     * in every row) are written at the width that column is stored at in HBM (1, 2 or 4 bytes, signed
     * two's complement; the src array at the width that holds every vid of the shard), so each value
     * keeps all its bits in fewer bytes. The widths come back in dev_key_w / dev_col_w. The reference's
     * own response carries integers as RowWriter varints (src/dataman/RowWriter.cpp), not at 8 bytes. */
    int32_t compact_results;
} ngx_go_plan;

/* One YIELD column of a device-resident result (result_on_device), columnar in HBM, nrows entries:
 *   x     value bits per row: int, double bits, bool 0/1, or a device pointer to string bytes
 *         (into the snapshot, the query's constant pool or the result string arena of the strings a
 *         YIELD column builds)
 *   len   string byte lengths; NULL when the column holds no strings (its static type is not STRING
 *         and not UNKNOWN)
 *   type  per-row value type (1 int, 2 double, 3 bool, 4 string); NULL when every row has the
 *         column's static type col_types[c] (a row of another type fails the query, as boost::get
 *         in GoExecutor::toThriftResponse does), i.e. non-NULL only for UNKNOWN-typed columns */
typedef struct {
    const int64_t* x;
    const uint32_t* len;
    const uint8_t* type;
} ngx_dev_column;

typedef struct {
    int32_t code;                      /* NGX_OK or an error (message in ngx_last_error) */
    int32_t ncols;
    const int32_t* col_types;          /* calculateExprType per YIELD column */
    uint64_t nrows;
    const ngx_cell* cells;             /* cells[row * ncols + col] */
    const int64_t* row_src;            /* src vid, dst vid, rank, signed type of the edge behind each row */
    const int64_t* row_dst;
    const int64_t* row_rank;
    const int32_t* row_type;
    const char* strings;
    uint64_t strings_len;
    /* statistics of the run on this shard */
    int32_t nhops;
    const uint64_t* hop_frontier;      /* frontier entries expanded per hop */
    const uint64_t* hop_edges;         /* edges scanned per hop (TEPS numerator) */
    const uint64_t* hop_next;          /* unique next-frontier vertices per hop (this shard) */
    double device_ms;                  /* HIP-event time from the first kernel to the last result write */
    /* result_on_device: HBM arrays valid until the next call on the context (nrows entries). Their
     * last writes are ordered on the context's stream: ngx_device_to_host and every later call on the
     * context see them complete; a reader on another stream or process calls ngx_synchronize first. */
    const int64_t* dev_src;
    const int64_t* dev_dst;
    const int64_t* dev_rank;
    const int32_t* dev_type;           /* NULL when the query has one OVER type: see dev_type_const */
    const ngx_dev_column* dev_cols;    /* ncols columns */
    int32_t dev_type_const;            /* signed type of every row when dev_type / row_type is NULL */
    /* host_columnar: one host column per YIELD column, nrows entries, laid out as ngx_dev_column
     * but in host memory (page-locked staging of the context, valid until the next call on it):
     * x holds int / double bits / bool, or for a string value a `const char*` to its bytes (len[r]
     * bytes, not NUL-terminated); `cells` is NULL and row_type is NULL when every row has
     * dev_type_const. row_src / row_dst / row_rank point into the same staging. */
    const ngx_dev_column* host_cols;
    const uint64_t* hop_exchange_bytes;/* world > 1: frontier bytes this shard sent per hop (0 otherwise) */
    double host_prep_ms;               /* host time from the call to the first launch (plan, programs) */
    double host_tail_ms;               /* host time after the device finished (results, checks) */
    /* result_on_device: bytes per element of dev_src / dev_dst / dev_rank and of each dev_cols[c].x
     * (8 unless plan.compact_results; then 1, 2, 4 or 8, signed integers below 8) */
    int32_t dev_key_w[3];
    const int32_t* dev_col_w;          /* ncols entries */
    /* compact_results: a width of 0 in dev_key_w / dev_col_w marks a constant column — the array is NULL
     * and every row holds dev_key_const[k] / dev_col_const[c] (the rank when every edge of the OVER
     * types has the same rank: nothing is written per row) */
    int64_t dev_key_const[3];
    const int64_t* dev_col_const;      /* ncols entries */
} ngx_go_result;

int32_t ngx_go(ngx_ctx* ctx, const ngx_go_plan* plan, ngx_go_result** out);
void ngx_go_result_free(ngx_go_result* r);
/* n GO plans run back to back, each exactly as one ngx_go call whose result is freed at once (a native
 * host loop: a graphd driving many queries, the bench's timed steps). Per query: its code, result rows
 * and edges scanned over all hops, and with `digests` (3 words per query) ngx_go_result_digest of its
 * device-resident result (codes / nrows / edges / digests may be NULL). Consecutive device-resident
 * plans without DISTINCT or input overlap (flag "batch_pipeline", default 1): the next query's host
 * preparation and first hops are enqueued while this one's final hop runs; every query's outcome is the
 * one it has alone. Every query's ngx_go_result is freed inside the call: only the codes, row counts,
 * scanned edges and digests come back (no result handle). Memory: a pipelined batch runs query i on lane
 * i % batch_lanes, and each lane keeps its own scratch (visited marks, frontiers, entry arrays sized by
 * the shard) and result arrays (sized for every edge of the final hop's slots) after the call, so the
 * context's steady HBM use is up to batch_lanes times ngx_go's; flag "release_lanes" = 1 frees the parked
 * lanes now, "batch_release_lanes" = 1 after every batch ("released_lane_bytes" counts what was freed).
 * A call that fails before any query runs (a NULL plan) writes its code for every query.
 * Returns the first code that is not NGX_OK. */
int32_t ngx_go_batch(ngx_ctx* ctx, const ngx_go_plan* const* plans, int32_t n, int32_t* codes, uint64_t* nrows,
                     uint64_t* edges, uint64_t* digests);

/* Copy `bytes` from device memory of this context (e.g. a result_on_device array) to host memory,
 * ordered after the context's work. */
int32_t ngx_device_to_host(ngx_ctx* ctx, void* dst, const void* src, uint64_t bytes);
/* Wait until all work issued on the context has completed (result_on_device arrays fully written). */
int32_t ngx_synchronize(ngx_ctx* ctx);
/* Order-independent digest of a device-resident GO result (result_on_device), computed on the device
 * without copying the rows: per row h = m(...m(m(S ^ src) ^ v0)... ^ v(ncols-1)), m = splitmix64's
 * finalizer, S = 0x9E3779B97F4A7C15, src the row's src vid and v_c the value bits of YIELD column c
 * (integers sign-extended from their stored width, a constant column's value); out[0] = sum of h mod
 * 2^64, out[1] = XOR of h, out[2] = rows. Integer / double / bool columns only (NGX_E_UNSUPPORTED for
 * string or untyped columns). A verification hook: two result multisets of any size compare by their
 * digests (tests/test_gpu_c3.py checks the 1 G-row C3 results against the generator's edges this way).
 * Call it before any other call on the context (the result arrays are valid until then). */
int32_t ngx_go_result_digest(ngx_ctx* ctx, const ngx_go_result* r, uint64_t out[3]);

/* ---------------------------------------------------------------- measurement hooks */
/* Per-kernel device times of the last ngx_go (HIP events on the engine stream), for bench.py. */
typedef struct {
    const char* name;
    uint32_t launches;
    double total_ms;
    uint64_t algo_bytes;               /* algorithmic bytes attributed to this kernel class */
} ngx_kernel_stat;
/* Service counters, named as the reference's stats::Stats registers them (src/common/stats/Stats.cpp:
 * "<server>_<module>_qps" / "_error_qps" / "_latency", StorageServiceHandler.h:55 get_bound):
 * storage_get_bound_qps (requests without failed parts), storage_get_bound_error_qps (the others),
 * storage_get_bound_latency_us_sum / _count / _max (the latency histogram's inputs, in microseconds).
 * Values since ngx_open; the array is valid until the next call on the context. */
typedef struct {
    const char* name;
    int64_t value;
} ngx_stat;
int32_t ngx_stats(ngx_ctx* ctx, const ngx_stat** out, int32_t* n);
int32_t ngx_set_profiling(ngx_ctx* ctx, int32_t on);
int32_t ngx_kernel_stats(ngx_ctx* ctx, const ngx_kernel_stat** out, int32_t* n);

/* Engine flags (the reference's gflags for this path):
 *   "jit"  1 (default; env NGX_JIT=0 turns it off): compile each query's WHERE / YIELD into
 *          final-hop kernels with hipRTC; 0: run the precompiled bytecode-interpreter kernels.
 *          Literals are launch arguments, so queries that differ only in literals share a kernel.
 *   "jit_cache_capacity"  compiled query shapes kept loaded (LRU, default 64).
 *   "jit_async"  0 (default) / 1: compile a new query shape on a background thread; until its module is
 *          ready the queries of that shape run on the interpreter kernels (no hipRTC time on the query's
 *          critical path). "jit_wait" (any value) blocks until the queued compiles have finished.
 *   "pull_factor"  direction-optimizing hops: an intermediate hop with E scanned edges over a shard of
 *          V rows pulls (probes every row's in-edges) when 100 * E >= pull_factor * V and the hop's
 *          in-edge slots mirror its out-edge slots exactly; default 200, 0 = never. Same results.
 * Read-only "pull_hops": intermediate hops that pulled so far.
 *   "device_libm"  math functions of row values. abs/floor/ceil/round/sqrt are correctly rounded on the
 *          device and always run there; calls of the others (sin, cos, tan, asin, acos, atan, exp, exp2,
 *          log, log2, log10, cbrt, hypot, pow) whose arguments are literals are evaluated at compile
 *          time with the host libm. With a row-dependent argument they compile to NGX_E_UNSUPPORTED
 *          (default 0; the caller runs its CPU path) because the device libm may differ from glibc in
 *          the last place; 1 accepts the device libm (within 2 ulp of glibc).
 *   "max_edge_returned_per_vertex"  storaged's flag for the storage requests of every GO hop: at most
 *          this many edges emitted per (vertex, edge type) in key order, counted after the storage
 *          checks and the pushed filter (QueryBaseProcessor.inl:501-505); <= 0: unlimited (default).
 *   "enable_reservoir_sampling"  storaged's FLAGS_enable_reservoir_sampling (default 0). With 1, storage
 *          keeps a random sample of each vertex's edges (QueryBoundProcessor::processEdgeSampling,
 *          QueryBoundProcessor.cpp:83-164): ngx_get_neighbors and ngx_go return NGX_E_UNSUPPORTED before
 *          any work, so the caller runs the reference's CPU path (set it alike on every rank).
 *   "rccl_timeout_ms"     deadline of every RCCL collective (default 120000; env NGX_RCCL_TIMEOUT_MS).
 *          On a timeout or an asynchronous RCCL error the communicator is aborted, the call returns
 *          NGX_E_DEVICE and every later call on the context fails (the caller exits).
 *   "trace_go"  graphd's FLAGS_trace_go (GoExecutor.cpp:559-569, 834-836): 1 logs each step's frontier,
 *          scanned edges, next frontier and time, and the total row count, to stderr (default 0).
 *   "dyn_hops"  0 (default) / 1: device-driven hops at world 1 (hop totals passed between kernels on the
 *          device, upper-bound grids, no host round trip per hop). Same results; measured slower at C2.
 *   "narrow_columns"  1 (default): integer columns, dst and rank stored at the narrowest width holding
 *          every value (applies at the next commit); 0: 8 bytes each. Same results.
 *   "compact_lane_rows"  rows per lane of the next-frontier compaction: 0 (default) = 4; 8 / 16 fewer,
 *          fatter waves (measured slower at C2). Same results.
 *   "batch_pipeline"  1 (default): ngx_go_batch overlaps consecutive device-resident queries (the next
 *          one's host work and first hops enqueued while this one's final hop runs); 0: strictly one
 *          after the other. Same results.
 *   "batch_lanes"  2 .. 8 (default 4): lanes of scratch and result rows a pipelined batch rotates over; up
 *          to lanes - 1 queries wait for their row counts while the next one runs its hops. Same results.
 *   "batch_fronts"  1 or 2 (default 2): streams the batch's hops run on (consecutive queries alternate;
 *          world > 1 always 1, so every rank issues its collectives in one order).
 *   "batch_finals"  1 or 2 (default 2): final streams of a batch; with 2 consecutive queries' final hops
 *          alternate between them (each close after its final hop on the same stream). Same results.
 *   "batch_close_stream"  1 (default) / 0: with one final stream, an overlapped final hop's close on a
 *          stream of its own (the next final hop does not queue behind it). Same results.
 *   "release_lanes"  1: free the parked lanes' scratch and result arrays now; "batch_release_lanes" 1 (default
 *          0): after every batch. Read-only "released_lane_bytes".
 *   "resv_groups"  1 .. 64 (default 8, a group per XCD): row-reservation counters of the GO final hop
 *          (kargs.h resv*). Same rows; more groups shorten the final hop's reservation stream and lengthen
 *          its close.
 *   "dst_props"  world > 1 $$ props: -1 (default) by size, 0 tag replicas over every global row (gathered
 *          once per snapshot), 1 fetched from their owners per record hop (GoExecutor::fetchVertexProps ->
 *          QueryVertexPropsProcessor). "dst_replica_max" (bytes per shard, default 1 GiB): the size rule.
 *          Collective like every GO: set it alike on every rank. Same results. Read-only "dst_fetches",
 *          "dst_fetch_rows".
 *   "batch_cu_split"  0 (default) / 32, 64, 128: a batch's hops on that many CUs (groups of 8 spread over
 *          the XCDs), its final hops on the rest. Same results.
 *   "batch_event_ring"  1 (default): each cross-stream wait of a batch takes its own event. Same results.
 *   "compact_wg"  0 (default: 256 in a pipelined batch, else 1024), 256 or 1024: threads per workgroup of
 *          the next-frontier compaction. Same results.
 *   "dense_final"  1 (default): after a pulled hop the final hop covers every CSR position of its one
 *          OVER slot and reads the pull's marks (no next-frontier list). Read-only "dense_finals". Same results.
 *          "dense_close_total" 1 (default): its frontier total (the hop statistics) is summed by its close
 *          instead of a launch of its own. Same results.
 *          "dense_world_dev" 1 (default): at world > 1 too, that total stays on the device (published with
 *          the row count) instead of a host wait after the count launch. Same results.
 *   "final_nt_loads" / "final_nt_stores"  0 (default) / 1: the generated GO final hop loads its columns /
 *          stores its rows non-temporally (not kept in L2). Same results.
 * Read-only counters for ngx_get_flag: "jit_compiled", "jit_hits", "jit_failed", "jit_compile_us",
 * "jit_cached", "jit_evicted", "batch_overlaps" (queries of ngx_go_batch that overlapped the next),
 * "dbuf_allocs" / "dbuf_alloc_bytes" (device scratch allocations of the process so far). */
int32_t ngx_set_flag(ngx_ctx* ctx, const char* name, int64_t value);
int32_t ngx_get_flag(ngx_ctx* ctx, const char* name, int64_t* value);
/* why the last query ran on the interpreter kernels instead of a generated one ("" if it did not) */
const char* ngx_jit_note(ngx_ctx* ctx);

/* libstdc++ std::hash<std::string>, the NBA fixture's vid function (TraverseTestBase.h:122-126) */
int64_t ngx_hash_string(const char* s, uint64_t n);

#ifdef __cplusplus
}
#endif

#endif  /* NEBULA_GN_H_ */
