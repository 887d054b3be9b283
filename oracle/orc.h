// SPDX: test infrastructure — NOT product code.
//
// CPU ORACLE for the nebula_amd hot path (GO N STEPS / FIND PATH over GetNeighbors).
//
// This is a plain C++17 restatement of the reference algorithm, written from the
// behaviour of the reference sources (cited per function, paths relative to the
// reference checkout).  It is used ONLY by tests/, __graft_entry__.smoke() and the
// cpu_baseline leg of bench.py, as the checker / the CPU baseline.  Nothing under
// nebula_amd/ links or calls it.
//
// Parity pins: tests/golden/* (FindPathTest.cpp / GoTest.cpp / QueryBoundTest.cpp
// known answers, nba dataset from TraverseTestBase.h) — see tests/test_oracle_golden.py.
#pragma once
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <string_view>
#include <unordered_map>
#include <unordered_set>
#include <variant>
#include <vector>

namespace orc {

// ---- common.thrift SupportedType (src/interface/common.thrift:23-45)
enum SType : int32_t {
  ST_UNKNOWN = 0, ST_BOOL = 1, ST_INT = 2, ST_VID = 3, ST_FLOAT = 4,
  ST_DOUBLE = 5, ST_STRING = 6, ST_TIMESTAMP = 7,
};

// ---- storage.thrift ErrorCode (src/interface/storage.thrift:13-44)
enum ECode : int32_t {
  E_SUCCEEDED = 0, E_LEADER_CHANGED = -11, E_PART_NOT_FOUND = -14,
  E_KEY_NOT_FOUND = -15, E_EDGE_PROP_NOT_FOUND = -21, E_TAG_PROP_NOT_FOUND = -22,
  E_IMPROPER_DATA_TYPE = -23, E_INVALID_FILTER = -31, E_UNKNOWN = -100,
  // graph.thrift ErrorCode E_EXECUTION_ERROR (src/interface/graph.thrift:29)
  E_EXECUTION_ERROR = -8,
};

// ---- VariantType = boost::variant<int64_t,double,bool,std::string>
//      (src/common/base/Base.h:140).  index(): 0 int, 1 double, 2 bool, 3 string.
using Value = std::variant<int64_t, double, bool, std::string>;

struct Status {
  bool ok = true;
  std::string msg;
  static Status Ok() { return {}; }
  static Status Err(std::string m) { Status s; s.ok = false; s.msg = std::move(m); return s; }
};

struct OptValue {  // OptVariantType = StatusOr<VariantType>
  Status st;
  Value v;
  OptValue() = default;
  OptValue(Value x) : v(std::move(x)) {}                 // NOLINT
  OptValue(Status s) : st(std::move(s)) {}               // NOLINT
  bool ok() const { return st.ok; }
};

// ---------------------------------------------------------------- schema
struct ColumnDef { std::string name; SType type; };
struct Schema {
  int64_t version = 0;
  std::vector<ColumnDef> cols;
  int find(const std::string& n) const {
    for (size_t i = 0; i < cols.size(); ++i) if (cols[i].name == n) return (int)i;
    return -1;
  }
  SType typeOf(const std::string& n) const { int i = find(n); return i < 0 ? ST_UNKNOWN : cols[i].type; }
};

// ---------------------------------------------------------------- K1 key codec
// NebulaKeyUtils (src/common/base/NebulaKeyUtils.cpp:28-47, .h:135-159)
std::string edgeKey(int32_t part, int64_t src, int32_t type, int64_t rank, int64_t dst, int64_t ver);
std::string edgePrefix(int32_t part, int64_t src, int32_t type);
std::string vertexKey(int32_t part, int64_t vid, int32_t tag, int64_t ver);
std::string vertexPrefix(int32_t part, int64_t vid, int32_t tag);
inline bool isEdgeKey(const std::string& k) {
  if (k.size() != 40) return false;
  uint32_t t; memcpy(&t, k.data(), 4);
  if ((t & 0xFF) != 1) return false;
  int32_t et; memcpy(&et, k.data() + 12, 4);
  return (et & 0x40000000) != 0;
}
inline bool isVertexKey(const std::string& k) {
  if (k.size() != 24) return false;
  uint32_t t; memcpy(&t, k.data(), 4);
  if ((t & 0xFF) != 1) return false;
  int32_t tg; memcpy(&tg, k.data() + 12, 4);
  return (tg & 0x40000000) == 0;
}
int64_t keySrc(const char* k);
int64_t keyDst(const char* k);
int64_t keyRank(const char* k);
int32_t keyType(const char* k);
int32_t keyPart(const char* k);
// StorageClient::partId (src/storage/client/StorageClient.cpp:10-11,402-407)
inline int32_t partOf(int64_t vid, int32_t numParts) {
  return static_cast<int32_t>(static_cast<uint64_t>(vid) % static_cast<uint64_t>(numParts) + 1);
}

// ---------------------------------------------------------------- K9 row codec
// RowWriter/RowReader (src/dataman/RowWriter.cpp:26-95, RowWriter.inl:9-43,
// RowReader.cpp:117-258, RowReader.h:91-170)
struct RowWriter {
  const Schema* schema = nullptr;   // null: schema is being written (SchemaWriter mode)
  Schema own;                       // SchemaWriter mode columns
  std::string cord;
  std::vector<int64_t> blockOffsets;
  int64_t colNum = 0;
  explicit RowWriter(const Schema* s) : schema(s) {}
  const Schema& sch() const { return schema ? *schema : own; }
  void afterWrite();
  void writeVarint(int64_t v);
  RowWriter& putInt(int64_t v, const char* name = nullptr);
  RowWriter& putVid(int64_t v, const char* name = nullptr);
  RowWriter& putBool(bool v, const char* name = nullptr);
  RowWriter& putDouble(double v, const char* name = nullptr);
  RowWriter& putString(const std::string& v, const char* name = nullptr);
  RowWriter& putValue(const Value& v, SType t, const char* name = nullptr);
  std::string encode();
};

struct RowReader {
  const Schema* schema;
  const uint8_t* data = nullptr;   // after header
  size_t len = 0;
  bool valid = false;
  std::vector<int64_t> offsets;    // offset of field i (computed lazily, sequential)
  RowReader(std::string_view row, const Schema* s);
  // returns false on invalid data
  bool fieldOffset(int idx, int64_t& off);
  // getPropByName semantics; error -> !ok
  OptValue get(const std::string& name);
  OptValue getIdx(int idx);
};
int32_t rowSchemaVer(std::string_view row);
bool decodeVarint(const uint8_t* p, size_t avail, uint64_t& v, int& len);
// RowReader::getDefaultProp (src/dataman/RowReader.h:91-116)
OptValue defaultProp(const Schema& s, const std::string& prop);

// RowSetWriter/RowSetReader (src/dataman/RowSetWriter.cpp:21-43, RowSetReader.cpp:32-72)
void rowSetAdd(std::string& rs, const std::string& row);
std::vector<std::string> rowSetSplit(const std::string& rs);

// ---------------------------------------------------------------- K10 expressions
enum Kind : uint8_t {
  kUnknown = 0, kPrimary, kFunctionCall, kUnary, kTypeCasting, kArithmetic,
  kRelational, kLogical, kSourceProp, kEdgeRank, kEdgeDstId, kEdgeSrcId, kEdgeType,
  kAliasProp, kVariableProp, kDestProp, kInputProp, kUUID, kMax,
};

struct Getters;

struct Expr {
  Kind kind = kUnknown;
  uint8_t op = 0;                  // unary / arithmetic / relational / logical operator
  Value prim;                      // kPrimary
  std::string alias, prop;         // property expressions
  int32_t castType = 0;            // kTypeCasting: ColumnType (INT=0? see expr.cpp)
  std::unique_ptr<Expr> a, b;
  std::vector<std::unique_ptr<Expr>> args;
  OptValue eval(Getters& g) const;
};

// Getters of ExpressionContext (src/common/filter/Expressions.h:36-60)
struct Getters {
  virtual ~Getters() = default;
  virtual OptValue aliasProp(const std::string& edge, const std::string& prop) = 0;
  virtual OptValue srcTagProp(const std::string& tag, const std::string& prop) = 0;
  virtual OptValue dstTagProp(const std::string& tag, const std::string& prop) = 0;
  virtual OptValue edgeRank() { return Status::Err("no rank getter"); }
  virtual OptValue inputProp(const std::string&) { return Status::Err("no input"); }
};

// Expression::decode / encode (src/common/filter/Expressions.cpp:93-116 and per-class codecs)
// returns nullptr + msg on failure.
std::unique_ptr<Expr> decodeExpr(const uint8_t* buf, size_t len, std::string* err);
bool asBool(const Value& v);

// ---------------------------------------------------------------- store
// One kvstore part: records appended in write order into byte arenas; finalize() sorts them
// bytewise (RocksDB's default comparator) keeping the last write of identical keys.
struct PartKV {
  std::string karena, varena;
  std::vector<uint64_t> koff{0}, voff{0};
  std::vector<uint32_t> order;   // sorted record ids (after finalize)
  void add(std::string_view k, std::string_view v) {
    karena.append(k.data(), k.size()); koff.push_back(karena.size());
    varena.append(v.data(), v.size()); voff.push_back(varena.size());
  }
  std::string_view rkey(uint32_t r) const { return {karena.data() + koff[r], koff[r + 1] - koff[r]}; }
  std::string_view rval(uint32_t r) const { return {varena.data() + voff[r], voff[r + 1] - voff[r]}; }
  size_t size() const { return order.size(); }
  std::string_view key(size_t i) const { return rkey(order[i]); }
  std::string_view val(size_t i) const { return rval(order[i]); }
  void finalize();
};

struct Store {
  int32_t numParts = 1;
  int32_t maxEdgePerVertex = 0x7fffffff;   // FLAGS_max_edge_returned_per_vertex
  int32_t minVerticesPerBucket = 3;        // FLAGS_min_vertices_per_bucket
  int32_t maxHandlersPerReq = 10;          // FLAGS_max_handlers_per_req
  int32_t threads = 1;                     // worker threads for bucket parallelism
  std::map<int32_t, PartKV> parts;                 // part -> sorted KV (memcmp)
  int32_t hosts = 1;                       // storaged hosts (part p -> host p % hosts)
  std::unordered_map<int32_t, std::map<int64_t, Schema>> edgeSchemas, tagSchemas;
  std::unordered_map<int32_t, std::string> edgeNames, tagNames;
  std::unordered_map<std::string, int32_t> edgeByName, tagByName;
  const Schema* edgeSchema(int32_t et, int64_t ver = -1) const;
  const Schema* tagSchema(int32_t tag, int64_t ver = -1) const;
  // RocksEngine::prefix: [first key >= prefix, while starts_with(prefix))
  std::pair<size_t, size_t> prefixRange(int32_t part, const std::string& prefix) const;
};

// ---------------------------------------------------------------- getBound (K3-K8)
struct PropDef {   // owner 1 SRC 2 DST 3 EDGE; stat 0 none, 1 SUM, 2 COUNT, 3 AVG
  int32_t owner; int32_t id; std::string name; int32_t stat = 0;
};
struct GNRequest {
  std::unordered_map<int32_t, std::vector<int64_t>> parts;
  std::vector<int32_t> edgeTypes;
  std::string filter;
  std::vector<PropDef> returns;
};
struct EdgeData { int32_t type; std::string data; };
struct TagData { int32_t tag; std::string data; };
struct VertexData { int64_t vid; std::vector<TagData> tags; std::vector<EdgeData> edges; };
struct QueryResponse {
  std::vector<std::pair<int32_t, int32_t>> failed;   // (code, part)
  std::unordered_map<int32_t, Schema> vertexSchema, edgeSchema;
  bool hasVertexSchema = false, hasEdgeSchema = false;
  std::vector<VertexData> vertices;
};
QueryResponse getBound(const Store& st, const GNRequest& req);
// QueryVertexPropsProcessor (src/storage/QueryVertexPropsProcessor.cpp:14-27)
QueryResponse getVertexProps(const Store& st, const GNRequest& req);
// QueryStatsProcessor (src/storage/QueryStatsProcessor.cpp:16-130): one row of SUM/COUNT/AVG
struct StatsResult {
  std::vector<std::pair<int32_t, int32_t>> failed;
  Schema schema;
  std::vector<Value> values;
  std::string data;
};
StatsResult boundStats(const Store& st, const GNRequest& req);
// StorageClient::getNeighbors: group vids by part and issue one request (one host).
QueryResponse getNeighbors(const Store& st, const std::vector<int64_t>& vids,
                           const std::vector<int32_t>& etypes, const std::string& filter,
                           const std::vector<PropDef>& returns);

// ---------------------------------------------------------------- executors
struct ResultSet {
  int32_t code = 0;
  std::string err;
  std::vector<std::string> colNames;
  std::vector<std::vector<Value>> rows;
  uint64_t scanned = 0;   // Σ_s E_s: adjacency entries returned by getBound over all steps
};

struct GoQuery {
  std::vector<int64_t> starts;
  std::vector<int32_t> etypes;    // OVER list (edge types, in order); empty + overAll
  bool overAll = false;
  uint32_t steps = 1;
  std::string where;              // Expression::encode bytes, empty = none
  std::vector<std::string> yields; // encoded yield expressions; empty = default
  std::vector<std::string> yieldNames;
  bool distinct = false;
  // piped / variable input ($-.col, $var.col): the FROM source's rows (InterimResult)
  std::vector<std::string> inputNames;
  std::vector<uint8_t> inputKinds;   // 0 INT, 1 DOUBLE, 2 BOOL, 3 STRING per input column
  std::vector<std::vector<Value>> inputRows;
  int inputVidCol = -1;
};
ResultSet runGo(const Store& st, const GoQuery& q);
// OVER * without YIELD: edge types of the default `_dst` columns, in column order
std::vector<int32_t> responseEdgeSchemaOrder(const std::vector<int32_t>& reqTypes);

struct PathStep { int64_t id; int32_t type; int64_t rank; };
using Path = std::vector<PathStep>;
struct FindPathQuery {
  std::vector<int64_t> from, to;
  std::vector<int32_t> etypes;
  bool overAll = false;
  uint32_t upto = 5;
  bool shortest = true;
};
// Faithful FindPathExecutor restatement (exponential; small graphs only).  SHORTEST
// applies the canonical tie-break among paths of equal length found in the
// same round.  Output: list of canonical entry lists [v0,t0,r0,v1,...,vk].
int32_t runFindPath(const Store& st, const FindPathQuery& q,
                    std::vector<std::vector<int64_t>>& out);
// Canonical BFS restatement of SHORTEST (scales): per target, min walk length L in [1,N]
// and the lexicographically smallest walk of that length.
int32_t runShortestBfs(const Store& st, const FindPathQuery& q,
                       std::vector<std::vector<int64_t>>& out);

}  // namespace orc
