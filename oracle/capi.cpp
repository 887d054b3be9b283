// Test infrastructure (oracle) — C entry points used by tests/ (ctypes) and bench.py's
// cpu_baseline leg.  Not linked by the product.
#include <algorithm>
#include <chrono>
#include <cstring>
#include "orc.h"

using namespace orc;

namespace {
struct OrcResult {
  ResultSet rs;
  uint64_t edgesScanned = 0;
  std::vector<std::string> strings;
  std::vector<std::vector<int64_t>> paths;
};
}  // namespace

extern "C" {

void* orc_create(int32_t num_parts) {
  auto* s = new Store();
  s->numParts = num_parts;
  for (int32_t p = 1; p <= num_parts; ++p) s->parts[p];
  return s;
}
void orc_destroy(void* h) { delete static_cast<Store*>(h); }

void orc_set_config(void* h, int32_t max_edge_per_vertex, int32_t min_vertices_per_bucket,
                    int32_t max_handlers_per_req, int32_t threads) {
  auto* s = static_cast<Store*>(h);
  s->maxEdgePerVertex = max_edge_per_vertex;
  s->minVerticesPerBucket = min_vertices_per_bucket;
  s->maxHandlersPerReq = max_handlers_per_req;
  s->threads = threads;
}

void orc_set_hosts(void* h, int32_t hosts) { static_cast<Store*>(h)->hosts = hosts < 1 ? 1 : hosts; }

int32_t orc_register_schema(void* h, int32_t is_edge, int32_t id, const char* name, int64_t ver,
                            int32_t ncols, const char* const* names, const int32_t* types) {
  auto* s = static_cast<Store*>(h);
  Schema sc;
  sc.version = ver;
  for (int32_t i = 0; i < ncols; ++i) sc.cols.push_back({names[i], static_cast<SType>(types[i])});
  if (is_edge) {
    s->edgeSchemas[id][ver] = sc;
    s->edgeNames[id] = name;
    s->edgeByName[name] = id;
  } else {
    s->tagSchemas[id][ver] = sc;
    s->tagNames[id] = name;
    s->tagByName[name] = id;
  }
  return 0;
}

// Records are appended in the given order; a later record with an identical key overwrites
// the earlier one (RocksDB write-batch semantics).
int32_t orc_load_part_kv(void* h, int32_t part, const uint8_t* kdata, const uint64_t* koffs,
                         const uint8_t* vdata, const uint64_t* voffs, uint64_t n) {
  auto* s = static_cast<Store*>(h);
  auto& v = s->parts[part];
  for (uint64_t i = 0; i < n; ++i) {
    v.add({reinterpret_cast<const char*>(kdata) + koffs[i], koffs[i + 1] - koffs[i]},
          {reinterpret_cast<const char*>(vdata) + voffs[i], voffs[i + 1] - voffs[i]});
  }
  return 0;
}

// InsertEdgeExecutor restated for bulk fixtures (src/graph/InsertEdgeExecutor.cpp:180-196):
// out-edge (src,+type,rank 0,dst) with RowWriter(schema) << props, in-edge (dst,-type,0,src)
// with an empty value, one version for the batch (AddEdgesProcessor.cpp:17-20).
int32_t orc_load_edges(void* h, int32_t etype, const int64_t* src, const int64_t* dst, uint64_t n,
                       const int64_t* const* int_cols, int32_t ncols) {
  auto* s = static_cast<Store*>(h);
  const Schema* sc = s->edgeSchema(etype);
  if (!sc || (int32_t)sc->cols.size() != ncols) return -1;
  int64_t ver = (int64_t)__builtin_bswap64((uint64_t)(INT64_MAX - 1));
  for (uint64_t i = 0; i < n; ++i) {
    RowWriter w(sc);
    for (int32_t c = 0; c < ncols; ++c) w.putInt(int_cols[c][i]);
    int32_t ps = partOf(src[i], s->numParts), pd = partOf(dst[i], s->numParts);
    s->parts[ps].add(edgeKey(ps, src[i], etype, 0, dst[i], ver), w.encode());
    s->parts[pd].add(edgeKey(pd, dst[i], -etype, 0, src[i], ver), std::string_view());
  }
  return 0;
}

int32_t orc_finalize(void* h) {
  auto* s = static_cast<Store*>(h);
  std::vector<PartKV*> ps;
  for (auto& kv : s->parts) ps.push_back(&kv.second);
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t i = 0; i < (int64_t)ps.size(); ++i) ps[i]->finalize();
  return 0;
}

// The next orc_go's piped / variable input (consumed by that call).
static thread_local GoQuery g_input;
void orc_set_input(int32_t ncols, const char* const* names, const uint8_t* kinds, const void* const* cols,
                   uint64_t nrows, int32_t vid_col) {
  g_input = GoQuery();
  g_input.inputVidCol = vid_col;
  for (int32_t c = 0; c < ncols; ++c) g_input.inputNames.emplace_back(names[c]);
  g_input.inputKinds.assign(kinds, kinds + ncols);
  g_input.inputRows.assign(nrows, std::vector<Value>(ncols));
  for (uint64_t r = 0; r < nrows; ++r)
    for (int32_t c = 0; c < ncols; ++c) {
      switch (kinds[c]) {
        case 1: { double d; memcpy(&d, static_cast<const int64_t*>(cols[c]) + r, 8); g_input.inputRows[r][c] = d; break; }
        case 2: g_input.inputRows[r][c] = static_cast<const int64_t*>(cols[c])[r] != 0; break;
        case 3: g_input.inputRows[r][c] = std::string(static_cast<const char* const*>(cols[c])[r]); break;
        default: g_input.inputRows[r][c] = static_cast<const int64_t*>(cols[c])[r];
      }
    }
}

int32_t orc_go(void* h, const int64_t* starts, uint64_t nstarts, const int32_t* etypes, int32_t ntypes,
               int32_t over_all, uint32_t steps, const uint8_t* where, uint32_t where_len,
               const uint8_t* yields_blob, const uint32_t* yield_lens, int32_t nyields, int32_t distinct,
               void** result) {
  auto* s = static_cast<Store*>(h);
  GoQuery q;
  q.starts.assign(starts, starts + nstarts);
  q.etypes.assign(etypes, etypes + ntypes);
  q.overAll = over_all != 0;
  q.steps = steps;
  if (where_len) q.where.assign(reinterpret_cast<const char*>(where), where_len);
  size_t off = 0;
  for (int32_t i = 0; i < nyields; ++i) {
    q.yields.emplace_back(reinterpret_cast<const char*>(yields_blob) + off, yield_lens[i]);
    off += yield_lens[i];
  }
  q.distinct = distinct != 0;
  q.inputNames = std::move(g_input.inputNames);
  q.inputKinds = std::move(g_input.inputKinds);
  q.inputRows = std::move(g_input.inputRows);
  q.inputVidCol = g_input.inputVidCol;
  g_input = GoQuery();
  auto* r = new OrcResult();
  r->rs = runGo(*s, q);
  *result = r;
  return r->rs.code;
}

int32_t orc_go_default_columns(const int32_t* over, int32_t n, int32_t over_all, int32_t* out, int32_t cap) {
  std::vector<int32_t> t(over, over + n);
  if (over_all) t = responseEdgeSchemaOrder(t);
  for (int32_t i = 0; i < cap && i < (int32_t)t.size(); ++i) out[i] = t[i];
  return (int32_t)t.size();
}

int32_t orc_result_code(void* r) { return static_cast<OrcResult*>(r)->rs.code; }
const char* orc_result_error(void* r) { return static_cast<OrcResult*>(r)->rs.err.c_str(); }
int64_t orc_result_rows(void* r) { return (int64_t) static_cast<OrcResult*>(r)->rs.rows.size(); }
int32_t orc_result_cols(void* r) {
  auto* x = static_cast<OrcResult*>(r);
  return x->rs.rows.empty() ? (int32_t)x->rs.colNames.size() : (int32_t)x->rs.rows[0].size();
}
const char* orc_result_colname(void* r, int32_t c) { return static_cast<OrcResult*>(r)->rs.colNames[c].c_str(); }
// cells: bits (int64 / double bits / bool / string index) + type tag per cell
void orc_result_cells(void* r, int64_t* bits, uint8_t* types) {
  auto* x = static_cast<OrcResult*>(r);
  x->strings.clear();
  size_t k = 0;
  for (auto& row : x->rs.rows) {
    for (auto& v : row) {
      types[k] = static_cast<uint8_t>(v.index());
      switch (v.index()) {
        case 0: bits[k] = std::get<0>(v); break;
        case 1: { double d = std::get<1>(v); memcpy(&bits[k], &d, 8); break; }
        case 2: bits[k] = std::get<2>(v) ? 1 : 0; break;
        default: bits[k] = (int64_t)x->strings.size(); x->strings.push_back(std::get<3>(v)); break;
      }
      ++k;
    }
  }
}
const char* orc_result_string(void* r, int64_t idx) { return static_cast<OrcResult*>(r)->strings[idx].c_str(); }
void orc_result_free(void* r) { delete static_cast<OrcResult*>(r); }

int32_t orc_find_path(void* h, const int64_t* from, uint64_t nf, const int64_t* to, uint64_t nt,
                      const int32_t* etypes, int32_t ntypes, int32_t over_all, uint32_t upto,
                      int32_t shortest, int32_t mode, void** result) {
  auto* s = static_cast<Store*>(h);
  FindPathQuery q;
  q.from.assign(from, from + nf);
  q.to.assign(to, to + nt);
  q.etypes.assign(etypes, etypes + ntypes);
  q.overAll = over_all != 0;
  q.upto = upto;
  q.shortest = shortest != 0;
  auto* r = new OrcResult();
  int32_t rc = mode == 0 ? runFindPath(*s, q, r->paths) : runShortestBfs(*s, q, r->paths);
  *result = r;
  return rc;
}
int64_t orc_paths_count(void* r) { return (int64_t) static_cast<OrcResult*>(r)->paths.size(); }
int64_t orc_path_len(void* r, int64_t i) { return (int64_t) static_cast<OrcResult*>(r)->paths[i].size(); }
void orc_path_get(void* r, int64_t i, int64_t* out) {
  auto& p = static_cast<OrcResult*>(r)->paths[i];
  std::copy(p.begin(), p.end(), out);
}

// CPU baseline helper: GO over the store, returning wall seconds and the number of adjacency
// entries scanned (Σ_s E_s: edges returned by getBound at every step).
double orc_go_timed(void* h, const int64_t* starts, uint64_t nstarts, const int32_t* etypes, int32_t ntypes,
                    uint32_t steps, const uint8_t* where, uint32_t where_len, int64_t* rows_out,
                    uint64_t* scanned_out) {
  auto* s = static_cast<Store*>(h);
  GoQuery q;
  q.starts.assign(starts, starts + nstarts);
  q.etypes.assign(etypes, etypes + ntypes);
  q.steps = steps;
  if (where_len) q.where.assign(reinterpret_cast<const char*>(where), where_len);
  auto t0 = std::chrono::steady_clock::now();
  auto rs = runGo(*s, q);
  auto t1 = std::chrono::steady_clock::now();
  if (rows_out) *rows_out = rs.code ? -1 : (int64_t)rs.rows.size();
  if (scanned_out) *scanned_out = rs.scanned;
  return std::chrono::duration<double>(t1 - t0).count();
}

// ---- getBound (QueryBoundProcessor restated), response accessors mirror nbg_gn_*
struct OrcGN { QueryResponse r; std::vector<std::pair<int32_t, Schema>> vs, es; };

void* orc_get_bound(void* h, const int32_t* parts, const int64_t* vids, uint64_t n, const int32_t* etypes,
                    int32_t ne, const uint8_t* filter, uint32_t flen, const int32_t* owners, const int32_t* ids,
                    const char* const* names, int32_t nret) {
  const Store& st = *static_cast<Store*>(h);
  GNRequest req;
  for (uint64_t i = 0; i < n; ++i) req.parts[parts[i]].push_back(vids[i]);
  req.edgeTypes.assign(etypes, etypes + ne);
  if (filter && flen) req.filter.assign(reinterpret_cast<const char*>(filter), flen);
  for (int32_t i = 0; i < nret; ++i) req.returns.push_back(PropDef{owners[i], ids[i], names[i]});
  auto* g = new OrcGN();
  g->r = getBound(st, req);
  for (auto& kv : g->r.vertexSchema) g->vs.emplace_back(kv.first, kv.second);
  for (auto& kv : g->r.edgeSchema) g->es.emplace_back(kv.first, kv.second);
  return g;
}
int32_t orc_gn_num_failed(void* r) { return (int32_t)static_cast<OrcGN*>(r)->r.failed.size(); }
void orc_gn_failed(void* r, int32_t i, int32_t* code, int32_t* part) {
  auto& f = static_cast<OrcGN*>(r)->r.failed[i];
  *code = f.first;
  *part = f.second;
}
int32_t orc_gn_num_schemas(void* r, int32_t is_edge) {
  auto* g = static_cast<OrcGN*>(r);
  return (int32_t)(is_edge ? g->es : g->vs).size();
}
int32_t orc_gn_schema(void* r, int32_t is_edge, int32_t i, int32_t c, const char** name, int32_t* type) {
  auto* g = static_cast<OrcGN*>(r);
  auto& e = (is_edge ? g->es : g->vs)[i];
  if (c < 0) return (int32_t)e.second.cols.size() * 0 + e.first;   // c < 0: the id
  *name = e.second.cols[c].name.c_str();
  *type = e.second.cols[c].type;
  return (int32_t)e.second.cols.size();
}
int64_t orc_gn_num_vertices(void* r) { return (int64_t)static_cast<OrcGN*>(r)->r.vertices.size(); }
int64_t orc_gn_vertex_id(void* r, int64_t i) { return static_cast<OrcGN*>(r)->r.vertices[i].vid; }
int32_t orc_gn_vertex_count(void* r, int64_t i, int32_t edges) {
  auto& v = static_cast<OrcGN*>(r)->r.vertices[i];
  return (int32_t)(edges ? v.edges.size() : v.tags.size());
}
int32_t orc_gn_vertex_item(void* r, int64_t i, int32_t edges, int32_t k, const uint8_t** data, uint64_t* len) {
  auto& v = static_cast<OrcGN*>(r)->r.vertices[i];
  if (edges) {
    *data = reinterpret_cast<const uint8_t*>(v.edges[k].data.data());
    *len = v.edges[k].data.size();
    return v.edges[k].type;
  }
  *data = reinterpret_cast<const uint8_t*>(v.tags[k].data.data());
  *len = v.tags[k].data.size();
  return v.tags[k].tag;
}
void orc_gn_free(void* r) { delete static_cast<OrcGN*>(r); }

// ---- boundStats (QueryStatsProcessor restated)
void* orc_bound_stats(void* h, const int32_t* parts, const int64_t* vids, uint64_t n, const int32_t* etypes,
                      int32_t ne, const uint8_t* filter, uint32_t flen, const int32_t* owners, const int32_t* ids,
                      const char* const* names, const int32_t* stats, int32_t nret) {
  const Store& st = *static_cast<Store*>(h);
  GNRequest req;
  for (uint64_t i = 0; i < n; ++i) req.parts[parts[i]].push_back(vids[i]);
  req.edgeTypes.assign(etypes, etypes + ne);
  if (filter && flen) req.filter.assign(reinterpret_cast<const char*>(filter), flen);
  for (int32_t i = 0; i < nret; ++i) req.returns.push_back(PropDef{owners[i], ids[i], names[i], stats[i]});
  return new StatsResult(boundStats(st, req));
}
int32_t orc_stats_num_failed(void* r) { return (int32_t)static_cast<StatsResult*>(r)->failed.size(); }
void orc_stats_failed(void* r, int32_t i, int32_t* code, int32_t* part) {
  auto& f = static_cast<StatsResult*>(r)->failed[i];
  *code = f.first;
  *part = f.second;
}
int32_t orc_stats_num_cols(void* r) { return (int32_t)static_cast<StatsResult*>(r)->schema.cols.size(); }
void orc_stats_col(void* r, int32_t c, const char** name, int32_t* type, int64_t* bits) {
  auto* s = static_cast<StatsResult*>(r);
  *name = s->schema.cols[c].name.c_str();
  *type = s->schema.cols[c].type;
  const Value& v = s->values[c];
  if (v.index() == 1) { double d = std::get<1>(v); memcpy(bits, &d, 8); }
  else *bits = std::get<0>(v);
}
void orc_stats_data(void* r, const uint8_t** data, uint64_t* len) {
  auto* s = static_cast<StatsResult*>(r);
  *data = reinterpret_cast<const uint8_t*>(s->data.data());
  *len = s->data.size();
}
void orc_stats_free(void* r) { delete static_cast<StatsResult*>(r); }

}  // extern "C"
