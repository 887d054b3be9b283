/*
 * nbg.h — C ABI of nebula_amd, the MI355X-native multi-hop traversal engine for Nebula Graph's
 * GO N STEPS / FIND PATH hot path.
 *
 * Plain C, no exceptions, no callbacks, no torch types.  Every entry point returns an int32_t
 * status: 0 on success, otherwise a storage::cpp2::ErrorCode / graph::cpp2::ErrorCode value
 * (src/interface/storage.thrift:13-44, graph.thrift:12-35) or one of the NBG_E_* codes below.
 * The caller owns every input; outputs are allocated by the library and released with the
 * matching *_free call.  Engines are immutable after nbg_finalize(); queries on one engine are
 * serialised internally (one HIP stream per engine).
 *
 * Reference interfaces this ABI replaces (paths relative to the reference checkout):
 *   nbg_create/…/nbg_finalize  ≙ the storaged data a kvstore part holds: NebulaStore parts
 *       filled through AddEdgesProcessor / AddVerticesProcessor
 *       (src/storage/AddEdgesProcessor.cpp:15-37, src/kvstore/NebulaStore.cpp:326-336)
 *   nbg_go / nbg_go_device     ≙ GoExecutor result semantics (src/graph/GoExecutor.cpp:83-984)
 *   nbg_go_prepare / _execute  ≙ GoExecutor::prepare() / execute() (GoExecutor.cpp:28-110)
 *   nbg_find_path              ≙ FindPathExecutor result semantics
 *       (src/graph/FindPathExecutor.cpp:145-715)
 *   nbg_get_neighbors          ≙ StorageServiceHandler::future_getBound → QueryBoundProcessor
 *       (src/storage/StorageServiceHandler.cpp:33-40, src/storage/QueryBoundProcessor.cpp:16-220)
 */
#ifndef NEBULA_AMD_NBG_H_
#define NEBULA_AMD_NBG_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes (storage.thrift ErrorCode / graph.thrift ErrorCode values) ---------- */
#define NBG_OK                     0
#define NBG_E_EXECUTION_ERROR     (-8)    /* graph E_EXECUTION_ERROR: eval error in WHERE/YIELD */
#define NBG_E_PART_NOT_FOUND      (-14)
#define NBG_E_EDGE_PROP_NOT_FOUND (-21)
#define NBG_E_TAG_PROP_NOT_FOUND  (-22)
#define NBG_E_IMPROPER_DATA_TYPE  (-23)
#define NBG_E_INVALID_FILTER      (-31)
#define NBG_E_UNKNOWN             (-100)
/* nebula_amd specific */
#define NBG_E_INVALID_ARGUMENT    (-1001)
#define NBG_E_UNSUPPORTED         (-1002) /* valid nGQL, not implemented on the device path */
#define NBG_E_DEVICE              (-1003) /* HIP runtime / kernel failure (message in last_error) */
#define NBG_E_OUT_OF_MEMORY       (-1004)
#define NBG_E_STATE               (-1005) /* e.g. query before nbg_finalize */

/* ---- Device limits ----------------------------------------------------------------------
 * A statement past one of these returns NBG_E_UNSUPPORTED before any row is produced (on every
 * rank of a partitioned engine), so the caller can run the reference's own executor on it
 * (tests/test_gpu_limits.py holds one test per limit):
 *   more than NBG_MAX_YIELDS YIELD columns; more than NBG_MAX_OVER OVER types (OVER * included;
 *   GO, FIND PATH, GetNeighbors); a WHERE + YIELD program over 256 instructions or 16 live
 *   registers per OVER type; GO over 32 STEPS; FIND SHORTEST PATH UPTO over 63, FIND ALL PATH
 *   UPTO over 32; $$ of a tag registered 17th or later; more than 32 $- / $var input columns.
 * (A storage filter with a function call is E_INVALID_FILTER per part, as checkExp answers it,
 * QueryBaseProcessor.inl:172-290.)
 * Not limits: $- / $var input strings absent from the snapshot's dictionary, string functions
 * nested to any depth in GO (both lifted in round 6). */
#define NBG_MAX_YIELDS 32
#define NBG_MAX_OVER   32

/* ---- common.thrift SupportedType ------------------------------------------------------ */
#define NBG_T_BOOL      1
#define NBG_T_INT       2
#define NBG_T_VID       3
#define NBG_T_FLOAT     4
#define NBG_T_DOUBLE    5
#define NBG_T_STRING    6
#define NBG_T_TIMESTAMP 7

/* Value tags of result cells: VariantType alternatives (src/common/base/Base.h:140). */
#define NBG_V_INT    0
#define NBG_V_DOUBLE 1
#define NBG_V_BOOL   2
#define NBG_V_STRING 3

typedef struct nbg_engine nbg_engine;
typedef struct nbg_rows nbg_rows;
typedef struct nbg_paths nbg_paths;

typedef struct {
  int32_t num_parts;     /* partition_num of the space: part = uint64(vid) % num_parts + 1   */
  int32_t num_gpus;      /* G: part p is served by GPU rank p % G (CreateSpaceProcessor:84-95) */
  int32_t rank;          /* this engine's GPU rank in [0, G)                                   */
  int32_t device;        /* HIP device ordinal to use                                          */
  int32_t max_edge_returned_per_vertex; /* FLAGS_max_edge_returned_per_vertex (INT32_MAX)       */
  int32_t min_vertices_per_bucket;      /* accepted for flag parity; no device effect           */
  int32_t max_handlers_per_req;         /* accepted for flag parity; no device effect           */
} nbg_config;

typedef struct {
  const char* name;
  int32_t type;          /* NBG_T_* */
} nbg_column_def;

/* ---- engine lifecycle ------------------------------------------------------------------ */
int32_t nbg_create(const nbg_config* cfg, nbg_engine** out);
void nbg_destroy(nbg_engine* e);
/* Message of the last failing call on this engine (valid until the next call). */
const char* nbg_last_error(const nbg_engine* e);

/* Schemas (meta SchemaManager view, src/meta/SchemaManager.h:20-48). */
int32_t nbg_register_tag(nbg_engine* e, int32_t tag_id, const char* name, int64_t schema_ver,
                         const nbg_column_def* cols, int32_t ncols);
int32_t nbg_register_edge(nbg_engine* e, int32_t edge_type, const char* name, int64_t schema_ver,
                          const nbg_column_def* cols, int32_t ncols);

/* Loader: KV records exactly as a kvstore part holds them — NebulaKeyUtils keys
 * (src/common/base/NebulaKeyUtils.cpp:12-47) and RowWriter values (src/dataman/RowWriter.cpp).
 * Record i is key_data[key_offs[i] .. key_offs[i+1]) / val_data[val_offs[i] .. val_offs[i+1]).
 * Later records with an identical key overwrite earlier ones (write-batch semantics).
 * Records of parts this rank does not serve (part % num_gpus != rank) are ignored. */
int32_t nbg_load_part_kv(nbg_engine* e, int32_t part,
                         const uint8_t* key_data, const uint64_t* key_offs,
                         const uint8_t* val_data, const uint64_t* val_offs, uint64_t n);

/* SST-file ingest: RocksDB BlockBasedTable files as rocksdb::SstFileWriter writes them for the
 * Spark generator (src/tools/spark-sstfile-generator/.../SstFileOutputFormat.scala:150-202),
 * replacing StorageHttpIngestHandler -> NebulaStore::ingest -> RocksEngine::ingest
 * (src/storage/StorageHttpIngestHandler.cpp:94-100, src/kvstore/NebulaStore.cpp:436-466,
 * src/kvstore/RocksEngine.cpp:360-370).  Every Put record is loaded as by nbg_load_part_kv (a key
 * already loaded is overwritten: the ingested file is newer).  Before nbg_finalize.
 *   nbg_ingest_sst: one file into `part`;
 *   nbg_ingest_dir: every "*.sst" under <download_dir>/<part>/ (recursively, in name order) for
 *                   every part this engine serves; a missing part directory is skipped.
 * Block compression none / Snappy; NBG_E_UNSUPPORTED for other codecs, record types other than
 * Put and format_version > 3; NBG_E_INVALID_ARGUMENT for unreadable or corrupt files (checksums
 * are verified). */
int32_t nbg_ingest_sst(nbg_engine* e, int32_t part, const char* path);
int32_t nbg_ingest_dir(nbg_engine* e, const char* download_dir);

/* Bulk loader (SST-ingest analogue): n edges of one positive edge type, inserted the way
 * InsertEdgeExecutor does (out-edge with props + in-edge (dst,-type,rank,src) with no props,
 * src/graph/InsertEdgeExecutor.cpp:180-196), all with one version; a later duplicate
 * (src,dst,rank) overwrites an earlier one.  prop_cols[c] points at n values of schema column c:
 * int64 for INT/TIMESTAMP/VID, double for FLOAT/DOUBLE, uint8 for BOOL; STRING columns are not
 * accepted here (use nbg_load_part_kv).  rank may be NULL (all 0). */
int32_t nbg_load_edges(nbg_engine* e, int32_t edge_type, const int64_t* src, const int64_t* dst,
                       const int64_t* rank, uint64_t n, const void* const* prop_cols, int32_t ncols);

/* Build the device snapshot (version de-dup, CSR/CSC per edge type, SoA prop columns) and upload
 * it to HBM.  Host-side staging is released afterwards. */
int32_t nbg_finalize(nbg_engine* e);

/* Snapshot files (restart without re-ingesting the kvstore): nbg_snapshot_save writes a finalized
 * engine's snapshot (schemas, dictionaries, CSR/CSC, columns, tag columns) to `path`;
 * nbg_snapshot_load replaces registration + loading + nbg_finalize on a fresh engine created with
 * the same num_parts / num_gpus / rank (a partitioned engine attaches its communicator first;
 * the load is then collective).  Schemas come from the file. */
int32_t nbg_snapshot_save(nbg_engine* e, const char* path);
int32_t nbg_snapshot_load(nbg_engine* e, const char* path);

typedef struct {
  uint64_t num_vertices;      /* vertices with at least one record in this rank's parts        */
  uint64_t num_edges;         /* live (latest-version) edge records, all signed types          */
  uint64_t device_bytes;      /* HBM held by the snapshot                                      */
  int32_t num_edge_types;     /* signed edge types present                                     */
  int32_t reserved;
  uint64_t tiny_queries;      /* GO queries run as one single-workgroup launch (tiny path)       */
  uint64_t host_agreements;   /* partitioned GO queries that agreed on rank-local statuses on the
                                 host before their first collective ($- / $var inputs); the others
                                 carry them in band                                              */
  uint64_t host_bytes;        /* host memory the finalized engine keeps beside its snapshot (row
                                 offsets, dictionary, the tiny path's walk bounds)               */
  uint64_t path_batch_contexts;  /* nbg_find_path_batch's contexts (rolling-run slots)          */
  uint64_t path_batch_reruns;    /* batched pairs whose search outgrew a context's lists and ran
                                    again on the engine's full-size one                          */
} nbg_stats;
int32_t nbg_get_stats(const nbg_engine* e, nbg_stats* out);

/* ---- GO N STEPS (GoExecutor semantics) ------------------------------------------------- */
/* Expression wire (WHERE / YIELD bytes here and the storage filter of nbg_gn_request): the bytes
 * of Expression::encode (src/common/filter/Expressions.cpp:93-98 and each class's encode), with
 * ONE extension.  The reference's TypeCastingExpression::encode writes nothing
 * (Expressions.cpp:801-802) and its decode throws (Expressions.h:830-832), so a cast cannot cross
 * the reference's own wire.  Here a cast is encoded as
 *     uint8 kind = 4 (kTypeCasting), uint8 ColumnType (0 INT, 1 STRING, 2 DOUBLE, 3 BIGINT,
 *     4 BOOL, 5 TIMESTAMP; Expressions.h:21-23), then the operand's own encoding,
 * which a graphd emits once its TypeCastingExpression::encode writes those three parts
 * (INTEGRATION.md §2 shows the body).  An UNPATCHED graphd drops the cast and its whole operand
 * from the bytes: the remaining tree is missing a subtree, so decoding runs out of bytes and
 * nbg_go fails with NBG_E_INVALID_ARGUMENT (nbg_get_neighbors: E_INVALID_FILTER for every part,
 * as the reference's processor answers a filter it cannot decode), never with rows.  A
 * cast at the ROOT of a WHERE encodes to zero bytes, which means "no WHERE" (where_len = 0): the
 * binding must reject a non-null filter_ whose encoding is empty.  Any other
 * ColumnType byte, or bytes left over after the tree, is NBG_E_INVALID_ARGUMENT. */
typedef struct {
  const int64_t* starts;          /* FROM vids; duplicates are kept (GoExecutor.cpp:136-195)  */
  uint64_t num_starts;
  const int32_t* edge_types;      /* OVER list, positive types, in order                      */
  int32_t num_edge_types;
  int32_t over_all;               /* OVER *: every registered positive edge type               */
  uint32_t steps;                 /* N >= 1                                                    */
  const uint8_t* where;           /* Expression::encode bytes of WHERE; NULL/0 = none         */
  uint32_t where_len;
  const uint8_t* const* yields;   /* Expression::encode bytes per YIELD column; 0 = default    */
  const uint32_t* yield_lens;     /*   (<edge>._dst per OVER edge, parser.yy:518-531)          */
  int32_t num_yields;
  int32_t distinct;               /* YIELD DISTINCT                                            */
  /* Piped / variable input for $-.col / $var.col in WHERE / YIELD: the rows the FROM $-.col or
   * $var.col came from, as columns.  GoExecutor::setupStarts indexes them by the FROM column
   * (input_vid_col; the last row of a vid wins, InterimResult.cpp:158-250) and a final-step row
   * reads the row of its source's root (VertexBackTracker, GoExecutor.h:169-188).  Column c holds
   * num_input_rows int64 payloads (int, double bits, bool 0/1) or, when input_kinds[c] is
   * NBG_V_STRING, a const char* const* of row strings.  num_input_cols = 0: no input. */
  int32_t num_input_cols;
  const char* const* input_names;
  const uint8_t* input_kinds;
  const void* const* input_cols;
  uint64_t num_input_rows;
  int32_t input_vid_col;
} nbg_go_request;

/* Rows are copied to host memory. */
int32_t nbg_go(nbg_engine* e, const nbg_go_request* req, nbg_rows** out);
/* Rows stay in HBM in the query workspace; nbg_rows_fetch() copies them to the host on demand.
 * They stay valid until nbg_rows_free: a later query that needs the workspace hands it over to
 * the live result (released by nbg_rows_free) and continues on a fresh one.  Every result must
 * be freed before nbg_destroy. */
int32_t nbg_go_device(nbg_engine* e, const nbg_go_request* req, nbg_rows** out);

/* Default YIELD of a GO without YIELD: the edge types whose `<edge>._dst` columns it returns, in
 * column order.  OVER e1, e2: the OVER order (parser.yy:518-531).  OVER * (over_all = 1, `over` =
 * every edge type as graphd requests them): the iteration order of the response's edge_schema map
 * (GoExecutor::getEdgeNamesFromResp, GoExecutor.cpp:481-499,546-561).  Returns the column count
 * (writes up to cap types) or a negative status. */
int32_t nbg_go_default_columns(nbg_engine* e, const int32_t* over, int32_t n, int32_t over_all, int32_t* out,
                               int32_t cap);

/* Prepared GO statement: GoExecutor::prepare() once (OVER / WHERE / YIELD validated and compiled
 * per OVER type, GoExecutor.cpp:136-263), then execute() from any number of start lists — the
 * request's starts are ignored by prepare.  Name-resolution errors stay deferred to the final step
 * as in nbg_go.  A statement belongs to its engine and must be freed before it. */
typedef struct nbg_go_stmt nbg_go_stmt;
int32_t nbg_go_prepare(nbg_engine* e, const nbg_go_request* req, nbg_go_stmt** out);
/* device != 0: rows stay in HBM as with nbg_go_device; otherwise as nbg_go. */
int32_t nbg_go_execute(nbg_go_stmt* stmt, const int64_t* starts, uint64_t num_starts, int32_t device,
                       nbg_rows** out);
void nbg_go_stmt_free(nbg_go_stmt* stmt);

/* Asynchronous execution (the way graphd runs concurrent queries): up to NBG_QUERY_SLOTS
 * (environment, default 6) queries of one engine in flight, each on its own workspace and HIP
 * stream.  nbg_go_submit enqueues the query and returns a ticket (when every slot is busy it first
 * completes the oldest query, whose result stays in its ticket); nbg_go_wait completes the ticket
 * (and every older one), returns its rows with nbg_go_execute's semantics and frees the ticket.
 * Device rows (device != 0) stay valid until nbg_rows_free, as with nbg_go_device (a slot whose
 * workspace still holds live rows gives it to them and takes a fresh one).  A ticket never
 * waited for is reclaimed by nbg_destroy; tickets must be
 * waited for before their statement is freed.  On a partitioned engine every rank must submit
 * the same queries in the same order (they are collectives).  Over RCCL each slot gets its own
 * communicator (split from the engine's, collectively, at the slot's first use; NBG_SLOT_COMMS=0
 * keeps one) and stream, so queries of different slots overlap on the device; the in-process
 * transport's slots share the engine's stream and communicator. */
typedef struct nbg_go_ticket nbg_go_ticket;
int32_t nbg_go_submit(nbg_go_stmt* stmt, const int64_t* starts, uint64_t num_starts, int32_t device,
                      nbg_go_ticket** out);
int32_t nbg_go_wait(nbg_go_ticket* ticket, nbg_rows** out);

int64_t nbg_rows_count(const nbg_rows* r);
int32_t nbg_rows_num_cols(const nbg_rows* r);
/* Σ_s E_s: adjacency entries scanned over all steps (the TEPS numerator); whole query, i.e.
 * summed over ranks on a partitioned engine. */
uint64_t nbg_rows_edges_scanned(const nbg_rows* r);
/* Per-step counters: frontier size |F_s| and edges E_s, s = 1..steps (arrays of length steps). */
int32_t nbg_rows_step_stats(const nbg_rows* r, uint64_t* frontier, uint64_t* edges, int32_t cap);
/* Rows into host memory: the device packs the row segments into contiguous columns and DMAs them
 * into pinned memory the engine reuses across results (returned by nbg_rows_free). */
int32_t nbg_rows_fetch(nbg_rows* r);
/* Host views (after nbg_go, or after nbg_rows_fetch): 8-byte cell payloads (int64, double bits,
 * bool as 0/1, string id) and value tags NBG_V_* per row.  The per-row tags are built on the first
 * nbg_rows_col_tags call; nbg_rows_col_kind gives a column's NBG_V_* kind when it is the same for
 * every row (the usual case: every OVER type yields the same kind), else -1. */
const int64_t* nbg_rows_col_bits(const nbg_rows* r, int32_t col);
const uint8_t* nbg_rows_col_tags(const nbg_rows* r, int32_t col);
int32_t nbg_rows_col_kind(const nbg_rows* r, int32_t col);
const char* nbg_rows_string(const nbg_rows* r, int64_t string_id);
/* Device view of a column's 8-byte payloads (valid for nbg_go_device results).  Rows are not
 * contiguous: each producing workgroup appends to its own region, so the result is the union of
 * the row ranges [begin, end) listed by nbg_rows_segment (host fetches pack them in that order). */
const void* nbg_rows_device_col(const nbg_rows* r, int32_t col);
int64_t nbg_rows_num_segments(const nbg_rows* r);
int32_t nbg_rows_segment(const nbg_rows* r, int64_t i, uint64_t* begin, uint64_t* end);
/* Order-independent digest of a result's rows, computed where the rows are (HBM for device
 * results): per row h = splitmix64(... splitmix64(0 ^ cell_0) ... ^ cell_{k-1}) over its 8-byte
 * cell payloads in column order; out[0] = rows, out[1] = XOR of h, out[2] = sum of h (mod 2^64).
 * Verifies results at sizes too large to fetch.  String cells hash their payload: the snapshot's
 * dictionary code for device rows (a string the query built — a concatenation, a cast to string —
 * is 1 << 62 | a 62-bit hash of its bytes, so equal strings hash alike), the result's string
 * index (nbg_rows_string) for host rows. */
int32_t nbg_rows_digest(const nbg_rows* r, uint64_t* out);
void nbg_rows_free(nbg_rows* r);

/* ---- FIND SHORTEST | ALL PATH (FindPathExecutor semantics) ----------------------------- */
typedef struct {
  const int64_t* from;            /* de-duplicated by the callee (VerticesClause::prepare)    */
  uint64_t num_from;
  const int32_t* edge_types;
  int32_t num_edge_types;
  int32_t over_all;
  const int64_t* to;
  uint64_t num_to;
  uint32_t upto;                  /* UPTO N STEPS, default 5 (parser.yy:858-861)              */
  int32_t shortest;               /* 1 = SHORTEST, 0 = ALL                                     */
} nbg_path_request;

/* Each path is an entry list [v0, t0, r0, v1, t1, r1, ..., vk] (vertex, edge type, ranking …)
 * — the graph.thrift Path entry_list (graph.thrift:58-73) with edge names as types.
 * SHORTEST returns at most one path per target: the minimum hop count, ties broken by the
 * lexicographically smallest entry list (the reference's tie-break is iteration order). */
int32_t nbg_find_path(nbg_engine* e, const nbg_path_request* req, nbg_paths** out);
/* Asynchronous FIND PATH: up to NBG_QUERY_SLOTS (default 6) one-pair SHORTEST queries of a
 * single (non-partitioned) engine in flight, each on its own device workspace and HIP stream;
 * every other request runs inside nbg_find_path_submit.  When every slot is busy the oldest query
 * is completed first (its result stays in its ticket).  nbg_find_path_wait returns the result with
 * nbg_find_path's semantics (and status) and frees the ticket; tickets must be waited for before
 * nbg_destroy (outstanding ones are reclaimed there). */
typedef struct nbg_path_ticket nbg_path_ticket;
int32_t nbg_find_path_submit(nbg_engine* e, const nbg_path_request* req, nbg_path_ticket** out);
int32_t nbg_find_path_wait(nbg_path_ticket* ticket, nbg_paths** out);

/* n independent FIND PATH requests at once (a graphd serving many FindPathExecutor queries,
 * src/graph/FindPathExecutor.cpp:145-411, each with its own result): out[i] / rcs[i] receive
 * request i's paths (free each with nbg_paths_free; NULL when rcs[i] != NBG_OK) and status.
 * One-pair SHORTEST requests on a single engine (UPTO <= 32) run as rolling device runs over
 * NBG_SP_BATCH (default 64, at most 64) contexts: every launch serves every context, and a
 * context takes the next queued pair as soon as its pair is done (UPTO over 32: fixed batches of
 * at most 32).  Each context holds a 16-byte label record per vertex and 5 lists of a quarter of
 * the vertices (NBG_SP_BATCH_LIST; ~1.2 GB at RMAT-26; a pair outgrowing them runs again on the
 * engine's full-size context, nbg_stats.path_batch_reruns); as many are made as HBM allows.  Other
 * requests run as nbg_find_path would.  Results equal nbg_find_path's.  Every request gets its
 * status in rcs[i] (out[i] is NULL exactly when rcs[i] != NBG_OK), also when the batch itself
 * fails part way (the requests that did not run carry that failure's code).  Returns NBG_OK
 * unless the batch itself could not run (arguments, device set-up). */
int32_t nbg_find_path_batch(nbg_engine* e, const nbg_path_request* reqs, uint64_t n, nbg_paths** out,
                            int32_t* rcs);
/* Allocate the one-pair SHORTEST contexts now instead of at their first query (what a server
 * does at start-up): the engine's own, `slots` of nbg_find_path_submit's (at most NBG_QUERY_SLOTS)
 * and `batch` of nbg_find_path_batch's (at most NBG_SP_BATCH; as many as fit in HBM, at least
 * one, else NBG_E_OUT_OF_MEMORY).  A one-pair context holds ~76 B per vertex plus its lists' tile
 * splits, a batch context ~31 B.  No-op on a partitioned engine. */
int32_t nbg_path_reserve(nbg_engine* e, int32_t slots, int32_t batch);
int64_t nbg_paths_count(const nbg_paths* p);
int64_t nbg_path_len(const nbg_paths* p, int64_t i);
const int64_t* nbg_path_entries(const nbg_paths* p, int64_t i);
/* Adjacency entries the search scanned (both directions; TEPS numerator). */
uint64_t nbg_paths_edges_scanned(const nbg_paths* p);
/* Diagnostic: launch batches the device level loop needed for this result (1: the first chain
 * finished it; more: the host continued it; 0: the host-driven loop answered). */
uint32_t nbg_paths_chain_batches(const nbg_paths* p);
void nbg_paths_free(nbg_paths* p);

/* ---- GetNeighbors (storage boundary: StorageServiceHandler::future_getBound) -------------
 * Columnar mirror of GetNeighborsRequest / QueryResponse (src/interface/storage.thrift:47-106,
 * 153-161) served by QueryBoundProcessor (src/storage/QueryBoundProcessor.cpp:16-220,
 * QueryBaseProcessor.inl:60-562): per requested (part, vid), tag rows of the SOURCE columns and,
 * per requested edge type that has return columns, the RowSet of its edges in key order
 * (latest version, storage-side filter with keep-on-error, first max_edge_returned_per_vertex
 * accepted edges).  Rows are the exact RowWriter / RowSetWriter bytes storaged would send
 * (src/dataman/RowWriter.cpp:26-95, RowSetWriter.cpp:21-43), so a thrift adapter copies them
 * into QueryResponse unchanged.  Request-level errors (unknown schema / prop, an invalid filter)
 * are reported as one failed code per requested part, like QueryBaseProcessor.inl:529-535;
 * parts this engine does not serve fail with NBG_E_PART_NOT_FOUND.  The edge walk and filter
 * run on the device (one expansion over the requested vertices per edge type). */
#define NBG_PROP_SOURCE 1
#define NBG_PROP_DEST   2
#define NBG_PROP_EDGE   3
typedef struct {
  int32_t owner;                  /* NBG_PROP_SOURCE / _DEST (tag prop) or _EDGE               */
  int32_t id;                     /* tag id, or signed edge type                               */
  const char* name;               /* prop name; _src / _dst / _type / _rank for edge keys      */
} nbg_prop_def;

typedef struct {
  const int32_t* parts;           /* part of each vid: the map<PartitionID, list<VertexID>>   */
  const int64_t* vids;            /*   flattened (one entry per requested vid)                 */
  uint64_t num_vids;
  const int32_t* edge_types;      /* signed: negative = in-edges                               */
  int32_t num_edge_types;
  const uint8_t* filter;          /* Expression::encode bytes; NULL/0 = none                   */
  uint32_t filter_len;
  const nbg_prop_def* return_columns;
  int32_t num_return_columns;
} nbg_gn_request;

typedef struct nbg_gn_response nbg_gn_response;
int32_t nbg_get_neighbors(nbg_engine* e, const nbg_gn_request* req, nbg_gn_response** out);
/* result.failed_codes: (code, part) pairs; latency_in_us */
int32_t nbg_gn_num_failed(const nbg_gn_response* r);
int32_t nbg_gn_failed(const nbg_gn_response* r, int32_t i, int32_t* code, int32_t* part);
int32_t nbg_gn_latency_us(const nbg_gn_response* r);
/* vertex_schema (is_edge = 0) / edge_schema (is_edge = 1): entries, then columns of entry i */
int32_t nbg_gn_num_schemas(const nbg_gn_response* r, int32_t is_edge);
int32_t nbg_gn_schema(const nbg_gn_response* r, int32_t is_edge, int32_t i, int32_t* id, int32_t* ncols);
int32_t nbg_gn_schema_col(const nbg_gn_response* r, int32_t is_edge, int32_t i, int32_t c, const char** name,
                          int32_t* type);
/* vertices[i]: vid, tag_data[k] = (tag, row bytes), edge_data[k] = (type, RowSet bytes) */
int64_t nbg_gn_num_vertices(const nbg_gn_response* r);
int64_t nbg_gn_vertex_id(const nbg_gn_response* r, int64_t i);
int32_t nbg_gn_vertex_num_tags(const nbg_gn_response* r, int64_t i);
int32_t nbg_gn_vertex_tag(const nbg_gn_response* r, int64_t i, int32_t k, int32_t* tag, const uint8_t** data,
                          uint64_t* len);
int32_t nbg_gn_vertex_num_edges(const nbg_gn_response* r, int64_t i);
int32_t nbg_gn_vertex_edges(const nbg_gn_response* r, int64_t i, int32_t k, int32_t* type, const uint8_t** data,
                            uint64_t* len);
/* Adjacency entries the device walk returned (after the filter and cap). */
uint64_t nbg_gn_edges(const nbg_gn_response* r);
void nbg_gn_free(nbg_gn_response* r);

/* ---- boundStats (StorageServiceHandler::future_boundStats -> QueryStatsProcessor) ---------
 * The GetNeighbors request with a StatType per return column (storage.thrift PropDef.stat):
 * one row of SUM / COUNT / AVG over the collected values (QueryStatsProcessor.cpp:16-130,
 * StatsCollector in Collector.h:76-109): tag props of the requested vertices, edge props of the
 * accepted edges; _src/_dst are not collected, bool/string only count; SUM/AVG need a numeric
 * column (else NBG_E_IMPROPER_DATA_TYPE per part).  `data` is the encoded row. */
#define NBG_STAT_SUM   1
#define NBG_STAT_COUNT 2
#define NBG_STAT_AVG   3
typedef struct nbg_stats_response nbg_stats_response;
int32_t nbg_bound_stats(nbg_engine* e, const nbg_gn_request* req, const int32_t* stats, nbg_stats_response** out);
int32_t nbg_stats_num_failed(const nbg_stats_response* r);
int32_t nbg_stats_failed(const nbg_stats_response* r, int32_t i, int32_t* code, int32_t* part);
int32_t nbg_stats_num_cols(const nbg_stats_response* r);
/* column c: name, NBG_T_INT / NBG_T_DOUBLE, value (int64 or double bits) */
int32_t nbg_stats_col(const nbg_stats_response* r, int32_t c, const char** name, int32_t* type, int64_t* bits);
int32_t nbg_stats_data(const nbg_stats_response* r, const uint8_t** data, uint64_t* len);
void nbg_stats_free(nbg_stats_response* r);

/* ---- in-library kernel timing (HIP events on the engine's stream) ----------------------- */
typedef struct {
  const char* name;           /* kernel name (static string)                                  */
  uint64_t launches;
  double total_ms;            /* sum of event-measured launch durations                        */
  double algo_bytes;          /* algorithmic HBM bytes of those launches */
} nbg_kernel_stat;
/* enable = 1 starts (and resets) timing of every launch; 2 times only the final-step /
 * shortest-path expansion kernels (two events per query: minimal perturbation of the timed
 * region); 0 stops timing. */
/* ---- FIND PATH replica of a partitioned engine (replica.hip) ---------------------------------
 * A partitioned engine (num_gpus > 1) also builds, at nbg_finalize (collectively), a replica of
 * every rank's path CSRs (offsets, neighbour ids and vids, ranks; no property columns) when it fits
 * in free HBM.  While it is in use, nbg_find_path / _submit / _batch / nbg_path_reserve run on it
 * RANK-LOCALLY: no collective, each rank may answer different requests, and the results equal the
 * single engine's over the same records.  Without it they are collectives over the partitioned
 * snapshot (every rank calls them with the same requests).
 * nbg_set_path_replica: before nbg_finalize, whether to build it (default: NBG_PATH_REPLICA, 1);
 * after, whether FIND PATH uses it (1 needs a built replica: else NBG_E_STATE).  It replaces
 * no reference interface (graphd reaches storaged for every FindPathExecutor round). */
int32_t nbg_set_path_replica(nbg_engine* e, int32_t mode);
int32_t nbg_path_replica_active(const nbg_engine* e);   /* 1: FIND PATH runs on the replica */

int32_t nbg_profile(nbg_engine* e, int32_t enable);
/* Copies up to cap kernel records; returns the number of kernels. */
int32_t nbg_profile_read(const nbg_engine* e, nbg_kernel_stat* out, int32_t cap);

/* ---- multi-GPU: partitioned engine ------------------------------------
 * With nbg_config.num_gpus = G > 1 an engine holds only the parts p with p % G == rank
 * (CreateSpaceProcessor.cpp:84-95, GPUs as storaged hosts) and every query is a collective:
 * all G engines must run the same nbg_go calls (same arguments, in the same order), the way
 * StorageClient::getNeighbors fans one request out to every host (StorageClient.cpp:94-124).
 * Per GO hop each rank expands its local frontier, and the per-step dst SET
 * (GoExecutor::getDstIdsFromResp, GoExecutor.cpp:501-541) is formed by one bitmap all-to-all:
 * rank q receives the candidates it owns.  Final-step rows stay on the rank that produced
 * them (the result is the union over ranks); nbg_rows_step_stats / nbg_rows_edges_scanned
 * report the whole query (summed over ranks).  The communicator must be attached before
 * nbg_finalize (the loader exchanges vertex dictionaries to build global neighbour ids).
 * nbg_find_path is collective too: each BFS level exchanges its candidate bitmap and the owner
 * claims (meet / target tests local at the owner, FindPathExecutor.cpp:218-290), sizes are summed
 * over ranks, and every rank returns the same paths. */
#define NBG_UNIQUE_ID_BYTES 128
/* RCCL unique id (ncclGetUniqueId); rank 0 creates it and ships it to the others. */
int32_t nbg_comm_unique_id(uint8_t out[NBG_UNIQUE_ID_BYTES]);
/* One process per GPU: RCCL communicator over xGMI (ncclCommInitRank); collective per rank. */
int32_t nbg_comm_init(nbg_engine* e, const uint8_t id[NBG_UNIQUE_ID_BYTES], int32_t world, int32_t rank);
/* Several engines of ONE process (engine i has rank i, num_gpus == n): an in-process group whose
 * collectives copy between the engines' buffers.  Each engine is then driven by its own host
 * thread (finalize and every query), exactly as the RCCL ranks are. */
int32_t nbg_comm_init_local(nbg_engine* const* engines, int32_t n);
/* Failure semantics of a partitioned engine.  The reference keeps a query alive when some
 * storaged parts fail and reports them (StorageClient.inl:112-136, GoExecutor.cpp:424-442); a
 * collective engine cannot run a hop without one of its ranks, so a query fails on EVERY rank
 * with the same code instead:
 *   - a rank-local failure before the query's first collective (allocation, a start list whose
 *     edges exceed one rank's list limit, ...) reaches every rank: every rank returns the code of
 *     the lowest-ranked rank that failed, and the engines stay usable.  For GO without $- / $var
 *     inputs (YIELD DISTINCT included) the failing rank still takes part in the query's
 *     collectives and its status travels with the query's statistics (no extra round trip):
 *     nbg_go_execute fails on every rank; nbg_go_submit returns a ticket on every rank (so every
 *     rank's query slots stay in step) and nbg_go_wait on it returns the code.  Other statements (and
 *     FIND PATH) agree in one small all-reduce before the query, so every rank's call fails;
 *   - a failure between collectives (a device error on one rank) aborts the communicator; the
 *     peers' pending collectives fail (in-process group at once, RCCL when their bounded wait of
 *     NBG_COMM_TIMEOUT_S seconds, default 120, expires) and every later collective call fails
 *     with NBG_E_DEVICE.
 * nbg_comm_abort aborts the engine's communicator(s) from any thread (ncclCommAbort for RCCL):
 * a host watchdog uses it to release a rank blocked in a collective.  Not under the engine
 * lock.  nbg_comm_aborted: 1 after an abort (the engine must be rebuilt), else 0. */
int32_t nbg_comm_abort(nbg_engine* e);
int32_t nbg_comm_aborted(const nbg_engine* e);
/* Testing hook: the next `count` queries of this engine fail at `site` exactly as a real failure
 * there would (the failure paths above are otherwise hard to reach on purpose). */
#define NBG_FAULT_ALLOC  1   /* the query's workspace / held-result hand-over allocation fails */
#define NBG_FAULT_DEVICE 2   /* partitioned GO: a device error after the query's first collective */
#define NBG_FAULT_STREAM 3   /* nbg_go_submit: the query slot's stream cannot be created */
int32_t nbg_inject_fault(nbg_engine* e, int32_t site, int32_t count);
/* The edge records this engine staged for signed edge type `type` (+t: out-edges keyed at src,
 * -t: in-edges keyed at dst), in load order, before nbg_finalize: a partitioned rank keeps the
 * records of the parts it serves (CreateSpaceProcessor.cpp:84-95 with GPUs as hosts), so the
 * ranks' lists partition the load.  Host only (no device call).  *n = the record count; up to
 * `cap` of them are written to src / dst / rank (any may be NULL).  NBG_E_STATE once finalized. */
int32_t nbg_staged_edges(const nbg_engine* e, int32_t type, int64_t* src, int64_t* dst, int64_t* rank, uint64_t cap,
                         uint64_t* n);

#ifdef __cplusplus
}
#endif
#endif /* NEBULA_AMD_NBG_H_ */
