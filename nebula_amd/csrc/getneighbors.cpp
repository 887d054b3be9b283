// GetNeighbors — the storage boundary (StorageServiceHandler::future_getBound,
// src/storage/StorageServiceHandler.cpp:33-40) served from the device snapshot.
//
// QueryBoundProcessor (src/storage/QueryBoundProcessor.cpp:16-220) over QueryBaseProcessor
// (src/storage/QueryBaseProcessor.inl:60-562):
//   * checkAndBuildContexts (:60-169): tag contexts for SOURCE/DEST columns, one edge context per
//     requested type (plus types named only by return columns), key props from the key, in-edge
//     value props skipped; the filter is decoded and checked (checkExp, :172-290).  A request-level
//     error is one failed code per requested part (:529-535).
//   * processVertex (QueryBoundProcessor.cpp:64-111): the tag rows first, then one RowSet per edge
//     context with props; a vertex is returned only if some RowSet is non-empty.
//   * collectEdgeProps (:381-458): key order, latest version, the filter on out-edges with
//     keep-on-error, at most max_edge_returned_per_vertex accepted edges.
// The edge walk and the filter run on the device (k_expand<FINAL> with a keep-on-error WHERE and
// the edge index / source vid / return columns as YIELDs); the host regroups the rows in key order
// and writes the RowWriter / RowSetWriter bytes (RowWriter.cpp:26-95, RowSetWriter.cpp:21-43).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <ctime>
#include <unordered_map>

#include <omp.h>

#include "engine.h"

using namespace nbg;

struct nbg_gn_response {
  struct Sch {
    int32_t id;
    std::vector<std::pair<std::string, int32_t>> cols;
  };
  struct Vertex {
    int64_t vid;
    std::vector<std::pair<int32_t, std::string>> tags, edges;
  };
  std::vector<std::pair<int32_t, int32_t>> failed;   // (code, part)
  int32_t latency_us = 0;
  std::vector<Sch> vschema, eschema;
  std::vector<Vertex> vertices;
  uint64_t edges = 0;
};

namespace {

// ------------------------------------------------------------------ RowWriter (schema-less mode)
// QueryBaseProcessor writes rows with RowWriter(nullptr): a SchemaWriter records the columns, the
// header carries no schema version (RowWriter.cpp:49-75); a block offset every 16 columns.
// The column bytes go into a plain buffer (room() grows it, the writers store with memcpy): the
// std::string push_back/append path cost ~25% more per row in the getBound encode.
struct RowBytes {
  std::vector<char> cord = std::vector<char>(256);
  size_t len = 0;
  std::vector<uint64_t> blocks;
  int64_t cols = 0;
  char* room(size_t n) {
    if (len + n > cord.size()) cord.resize(std::max(cord.size() * 2, len + n));
    return cord.data() + len;
  }
  void bytes(const void* p, size_t n) {
    memcpy(room(n), p, n);
    len += n;
  }
  void varint(uint64_t v) {
    char* p = room(10);
    size_t k = 0;
    while (v >= 0x80) {
      p[k++] = (char)(v | 0x80);
      v >>= 7;
    }
    p[k++] = (char)v;
    len += k;
  }
  void done() {
    ++cols;
    if ((cols & 15) == 0) blocks.push_back(len);
  }
  void put_int(int64_t v) { varint((uint64_t)v); done(); }
  void put_vid(int64_t v) { bytes(&v, 8); done(); }
  void put_double(int64_t bits) { bytes(&bits, 8); done(); }
  void put_bool(int64_t v) { *room(1) = v ? 1 : 0; ++len; done(); }
  void put_string(const std::string& s) { varint(s.size()); bytes(s.data(), s.size()); done(); }
  void clear() {   // (keeps the buffers: one RowBytes serves every row of a response)
    len = 0;
    blocks.clear();
    cols = 0;
  }
  int offset_bytes() const {
    int off = 0;
    uint64_t n = len;
    do { ++off; n >>= 8; } while (n);
    return off;
  }
  std::string encode() const {
    std::string out;
    head(out, false);
    out.append(cord.data(), len);
    return out;
  }
  // RowSetWriter::addRow(encode()) (RowSetWriter.cpp:21-43) without the temporaries: varint
  // length, then the row
  void append_to(std::string& rs) const {
    head(rs, true);
    rs.append(cord.data(), len);
  }
  // [varint row length] offset-width byte, block offsets (RowWriter.cpp:49-75), built in one
  // small buffer
  void head(std::string& out, bool with_len) const {
    const int off = offset_bytes();
    char hdr[16];
    size_t k = 0;
    if (with_len) {
      uint64_t v = 1 + blocks.size() * (uint64_t)off + len;
      while (v >= 0x80) {
        hdr[k++] = (char)(v | 0x80);
        v >>= 7;
      }
      hdr[k++] = (char)v;
    }
    hdr[k++] = (char)(off - 1);
    out.append(hdr, k);
    for (uint64_t b : blocks) out.append(reinterpret_cast<const char*>(&b), off);
  }
};

struct PropCtx {
  std::string name;
  int32_t type = 0;     // NBG_T_* of the response schema column
  int pik = 0;          // key prop: 1 _src, 2 _dst, 3 _type, 4 _rank
  int col = -1;         // value column (edge or tag schema)
  int ret = 0;          // retIndex_: position among the returned columns
  int32_t stat = 0;     // boundStats: NBG_STAT_* (0: none)
};

// QueryStatsProcessor / StatsCollector (src/storage/QueryStatsProcessor.cpp:16-130,
// src/storage/Collector.h:76-109): one SUM / COUNT / AVG per returned column over every collected
// value; vids (_src/_dst) are not collected at all, bool and string only count.
struct StatAcc {
  std::string name;
  int32_t stat = 0;
  bool dbl = false;     // the column's values are doubles (sum kept as double)
  int64_t isum = 0;
  double dsum = 0;
  int32_t count = 0;
};
struct StatsSink {
  std::vector<StatAcc> acc;   // by retIndex_
};
struct TagCtx {
  int32_t tag;
  std::vector<PropCtx> props;   // returned props
};
struct EdgeCtx {
  int32_t type;
  std::vector<PropCtx> props;
};

int32_t key_type(const std::string& n) {
  return (n == "_src" || n == "_dst") ? NBG_T_VID : NBG_T_INT;
}
int key_pik(const std::string& n) {
  return n == "_src" ? 1 : n == "_dst" ? 2 : n == "_type" ? 3 : n == "_rank" ? 4 : 0;
}

// QueryBaseProcessor::checkExp (QueryBaseProcessor.inl:172-290): true if the storage can run it
bool check_exp(const Engine& E, const Node& e, bool have_edges) {
  switch (e.kind) {
    case EK_PRIMARY: return true;
    case EK_FUNC: return false;
    case EK_UNARY: case EK_CAST: return check_exp(E, *e.kids[0], have_edges);
    case EK_ARITH: case EK_REL: case EK_LOGIC:
      return check_exp(E, *e.kids[0], have_edges) && check_exp(E, *e.kids[1], have_edges);
    case EK_SRCPROP: {
      for (auto& kv : E.tags)
        if (kv.second.name == e.alias) {
          const Schema* s = kv.second.latest();
          return s && s->find(e.prop) >= 0;
        }
      return false;
    }
    case EK_RANK: case EK_DST: case EK_SRCID: case EK_TYPE: return true;
    case EK_ALIAS: {
      if (!have_edges) return false;
      for (auto& kv : E.edges)
        if (kv.second.name == e.alias) {
          const Schema* s = kv.second.latest();
          return s && s->find(e.prop) >= 0;
        }
      return false;
    }
    default: return false;
  }
}

bool part_served(const Engine& E, int32_t part) {
  if (part < 1 || part > E.cfg.num_parts) return false;
  return E.cfg.num_gpus <= 1 || part % E.cfg.num_gpus == E.cfg.rank;
}

}  // namespace

// NBG_GN_TRACE=1: mean time per phase (contexts + compile, device walk + fetch, response bytes),
// printed every 500 requests
struct GnTrace {
  bool on = getenv("NBG_GN_TRACE") != nullptr;
  uint64_t n = 0;
  double ms[5] = {};
  std::chrono::steady_clock::time_point t;
  void mark(int phase) {
    const auto now = std::chrono::steady_clock::now();
    if (phase >= 0) ms[phase] += std::chrono::duration<double, std::milli>(now - t).count();
    t = now;
  }
  void done() {
    if (++n % 500) return;
    fprintf(stderr,
            "[gn trace] %llu requests: contexts %.4f ms, device %.4f ms, small-rows read %.4f ms, regroup %.4f ms, "
            "row bytes %.4f ms\n",
            (unsigned long long)n, ms[0] / n, ms[1] / n, ms[2] / n, ms[3] / n, ms[4] / n);
  }
};
static thread_local GnTrace g_gn_trace;   // (per calling thread: engines may serve requests concurrently)

// stats != nullptr: boundStats — accumulate per returned column (stat_types[i] per request column)
static int32_t get_neighbors(Engine& E, const nbg_gn_request* rq, nbg_gn_response* resp,
                             const int32_t* stat_types = nullptr, StatsSink* stats = nullptr) {
  int ret_index = 0;
  GnTrace& tr_ = g_gn_trace;
  if (tr_.on) tr_.mark(-1);
  // QueryBaseProcessor::validOperation (QueryBaseProcessor.inl:18-35)
  auto valid_op = [](int32_t type, int32_t stat) {
    if (stat != NBG_STAT_SUM && stat != NBG_STAT_AVG) return true;
    return type == NBG_T_INT || type == NBG_T_VID || type == NBG_T_TIMESTAMP || type == NBG_T_FLOAT ||
           type == NBG_T_DOUBLE;
  };
  // --- checkAndBuildContexts
  std::vector<TagCtx> tctx;
  std::vector<EdgeCtx> ectx;
  auto edge_ctx = [&](int32_t t) -> EdgeCtx* {
    for (auto& c : ectx)
      if (c.type == t) return &c;
    return nullptr;
  };
  for (int32_t i = 0; i < rq->num_edge_types; ++i)
    if (!edge_ctx(rq->edge_types[i])) ectx.push_back(EdgeCtx{rq->edge_types[i], {}});
  int32_t code = NBG_OK;
  for (int32_t i = 0; i < rq->num_return_columns && !code; ++i) {
    const nbg_prop_def& pd = rq->return_columns[i];
    const std::string name = pd.name ? pd.name : "";
    PropCtx pc;
    pc.name = name;
    if (pd.owner == NBG_PROP_SOURCE || pd.owner == NBG_PROP_DEST) {
      auto it = E.tags.find(pd.id);
      const Schema* s = it == E.tags.end() ? nullptr : it->second.latest();
      if (!s) { code = NBG_E_TAG_PROP_NOT_FOUND; break; }
      pc.col = s->find(name);
      if (pc.col < 0) { code = NBG_E_IMPROPER_DATA_TYPE; break; }
      pc.type = s->cols[pc.col].type;
      pc.stat = stat_types ? stat_types[i] : 0;
      if (!valid_op(pc.type, pc.stat)) { code = NBG_E_IMPROPER_DATA_TYPE; break; }
      pc.ret = ret_index++;
      TagCtx* tc = nullptr;
      for (auto& c : tctx)
        if (c.tag == pd.id) tc = &c;
      if (!tc) { tctx.push_back(TagCtx{pd.id, {}}); tc = &tctx.back(); }
      tc->props.push_back(pc);
    } else {
      if ((pc.pik = key_pik(name))) {
        pc.type = key_type(name);
      } else if (pd.id > 0) {
        auto it = E.edges.find(pd.id);
        const Schema* s = it == E.edges.end() ? nullptr : it->second.latest();
        if (!s) { code = NBG_E_EDGE_PROP_NOT_FOUND; break; }
        pc.col = s->find(name);
        if (pc.col < 0) { code = NBG_E_IMPROPER_DATA_TYPE; break; }
        pc.type = s->cols[pc.col].type;
      } else {
        continue;   // "InBound has none props, skip it!"
      }
      pc.stat = stat_types ? stat_types[i] : 0;
      if (!valid_op(pc.type, pc.stat)) { code = NBG_E_IMPROPER_DATA_TYPE; break; }
      pc.ret = ret_index++;
      EdgeCtx* ec = edge_ctx(pd.id);
      if (!ec) { ectx.push_back(EdgeCtx{pd.id, {}}); ec = &ectx.back(); }
      ec->props.push_back(pc);
    }
  }
  std::unique_ptr<Node> filter;
  if (!code && rq->filter && rq->filter_len) {
    std::string err;
    filter = decode_expr(rq->filter, rq->filter_len, &err);
    if (!filter || !check_exp(E, *filter, !ectx.empty())) code = NBG_E_INVALID_FILTER;
  }
  // requested parts, ascending (the processor's part order)
  std::vector<int32_t> parts(rq->parts, rq->parts + rq->num_vids);
  std::sort(parts.begin(), parts.end());
  parts.erase(std::unique(parts.begin(), parts.end()), parts.end());
  if (code) {
    for (int32_t p : parts) resp->failed.emplace_back(code, p);
    return NBG_OK;
  }
  // --- vertices: dense ids of the requested (part, vid) with rows in that part
  std::vector<uint8_t> part_bad(parts.size(), 0);
  for (size_t k = 0; k < parts.size(); ++k)
    if (!part_served(E, parts[k])) {
      part_bad[k] = 1;
      resp->failed.emplace_back(NBG_E_PART_NOT_FOUND, parts[k]);
    }
  auto part_ok = [&](int32_t p) { return !part_bad[std::lower_bound(parts.begin(), parts.end(), p) - parts.begin()]; };
  std::vector<uint32_t> dense(rq->num_vids, NO_ROW);
  std::vector<uint32_t> starts;
  for (uint64_t i = 0; i < rq->num_vids; ++i) {
    if (!part_ok(rq->parts[i])) continue;
    const uint32_t d = E.dense(rq->vids[i]);
    if (d == NO_ROW || E.snap.h_part[d] != rq->parts[i]) continue;   // prefix scan of another part
    dense[i] = d;
    starts.push_back(d);
  }
  std::sort(starts.begin(), starts.end());
  starts.erase(std::unique(starts.begin(), starts.end()), starts.end());

  // --- device walk: one final-step expansion per edge context with props
  struct TypeRows {
    std::vector<int64_t> vid, eidx;
    std::vector<std::vector<int64_t>> vals;   // [prop][row]
    std::unordered_map<int64_t, std::pair<uint64_t, uint64_t>> range;   // vid -> [lo, hi) in key order
  };
  std::vector<TypeRows> trows(ectx.size());
  // superseded versions of a filtered type: rows of its older versions that pass (vid -> (grp, values))
  struct OldRows {
    std::unordered_map<int64_t, std::vector<std::pair<uint32_t, std::vector<int64_t>>>> by_vid;
  };
  std::vector<OldRows> orows(ectx.size());
  std::vector<size_t> active;   // ectx indices walked on the device
  std::vector<std::vector<int>> yield_of(ectx.size());   // returned prop -> YIELD column
  for (size_t k = 0; k < ectx.size(); ++k)
    if (!ectx[k].props.empty() && E.snap.types.count(ectx[k].type)) active.push_back(k);
  if (!starts.empty() && !active.empty()) {
    if (active.size() > (size_t)MAX_TYPES_Q) return E.fail(NBG_E_UNSUPPORTED, "too many edge types");
    std::vector<TypeProgram> plist;
    std::vector<uint64_t> region, blk_cap, ebound;
    uint64_t cap_rows = 0;
    int ncols = 0;
    std::string err;
    for (size_t k : active) {
      const EdgeCtx& ec = ectx[k];
      const DevEdgeType& dt = E.snap.types.at(ec.type);
      TypeProgram tp;
      tp.etype = ec.type;
      tp.keep_on_error = true;
      ProgramBuilder pb;
      if (filter && ec.type > 0) {   // in-edges carry no value: the filter is not evaluated (inl:410)
        std::vector<int32_t> over{ec.type};
        CompileEnv env{ec.type, &over, &E.edges, &E.snap.strings, dt.valid != nullptr, dt.rank != nullptr};
        env.tags = &E.tags;
        env.dtags = &E.snap.tags;
        env.partitioned = E.partitioned();
        env.storage = true;
        Compiled c;
        int32_t rc = compile_expr(*filter, env, pb, &c, &err);
        if (rc) return E.fail(rc == NBG_E_UNSUPPORTED ? rc : NBG_E_INVALID_FILTER, "filter: " + err);
        if (c.is_const) {
          bool tv;
          switch (c.kind) {
            case VK_STRING: tv = c.const_str.empty(); break;
            case VK_DOUBLE: { double d; memcpy(&d, &c.const_bits, 8); tv = d != 0.0; break; }
            default: tv = c.const_bits != 0;
          }
          pb.code.clear();
          pb.code.push_back(Ins{OP_CONST, 0, 0, 0, 0, tv ? 1 : 0});
          c.reg = 0;
          c.kind = VK_BOOL;
          pb.max_reg = std::max(pb.max_reg, 1);
        }
        const uint8_t r = (uint8_t)c.reg;
        if (c.kind == VK_INT) pb.code.push_back(Ins{OP_TRUTHY_I, r, r, 0, 0, 0});
        else if (c.kind == VK_DOUBLE) pb.code.push_back(Ins{OP_TRUTHY_F, r, r, 0, 0, 0});
        else if (c.kind == VK_STRING) pb.code.push_back(Ins{OP_TRUTHY_S, r, r, 0, 0, string_code(E.snap.strings, "")});
        tp.where_len = (int)pb.code.size();
        tp.where_reg = c.reg;
      }
      // YIELDs: source vid, edge index, then one payload per returned prop
      auto yield_op = [&](uint8_t op, int32_t aux = 0) {
        const int reg = (int)tp.yield_reg.size() % MAX_REGS;
        pb.code.push_back(Ins{op, (uint8_t)reg, 0, 0, aux, 0});
        tp.yield_reg.push_back(reg);
        tp.yield_kind.push_back(VK_INT);
        tp.yield_const.push_back(0);
        tp.yield_const_str.emplace_back();
        pb.max_reg = std::max(pb.max_reg, reg + 1);
      };
      yield_op(OP_SRC);
      yield_op(OP_EIDX);
      // one YIELD per distinct source of the returned props (a prop may be asked for repeatedly)
      std::vector<std::pair<int, int>> srcs;   // (pik, col)
      std::vector<int>& map = yield_of[k];
      for (auto& pc : ec.props) {
        const std::pair<int, int> key{pc.pik, pc.pik ? -1 : pc.col};
        auto f = std::find(srcs.begin(), srcs.end(), key);
        map.push_back(2 + (int)(f - srcs.begin()));
        if (f != srcs.end()) continue;
        srcs.push_back(key);
        if (pc.pik == 1) yield_op(OP_SRC);
        else if (pc.pik == 2) yield_op(OP_DST);
        else if (pc.pik == 4) yield_op(OP_RANK);
        else if (pc.pik == 3) {   // constant: the key's type
          tp.yield_reg.push_back(-1);
          tp.yield_kind.push_back(VK_INT);
          tp.yield_const.push_back(ec.type);
          tp.yield_const_str.emplace_back();
        } else {
          yield_op(OP_COL, pc.col);
        }
      }
      if ((int)tp.yield_reg.size() > MAX_YIELDS) return E.fail(NBG_E_UNSUPPORTED, "too many return columns");
      tp.code = pb.code;
      tp.nregs = std::max(1, pb.max_reg);
      if ((int)tp.code.size() > MAX_PROGRAM) return E.fail(NBG_E_UNSUPPORTED, "program too long");
      if (tp.nregs > interp_max_regs()) return E.fail(NBG_E_UNSUPPORTED, "too many return columns for the device's LDS");
      ncols = std::max(ncols, (int)tp.yield_reg.size());
      uint64_t eb = 0;
      for (uint32_t d : starts) eb += dt.h_row_ptr[d + 1] - dt.h_row_ptr[d];
      ebound.push_back(eb);
      blk_cap.push_back(ws_final_blk_cap(starts.size(), eb));
      region.push_back(cap_rows);
      cap_rows += blk_cap.back() * ws_final_grid(starts.size(), eb);
      plist.push_back(std::move(tp));
    }
    // the older versions of filtered out-edge types: walked with the same program (the filtered
    // walk reads them until an edge is accepted, QueryBaseProcessor.inl:394-456)
    std::vector<size_t> olds;   // positions in `active`
    for (size_t i = 0; filter && i < active.size(); ++i) {
      const DevEdgeType& dt = E.snap.types.at(ectx[active[i]].type);
      if (ectx[active[i]].type < 0 || !dt.old || !dt.old->num_edges) continue;
      uint64_t eb = 0;
      for (uint32_t d : starts) eb += dt.old->h_row_ptr[d + 1] - dt.old->h_row_ptr[d];
      if (!eb) continue;
      olds.push_back(i);
      ebound.push_back(eb);
      blk_cap.push_back(ws_final_blk_cap(starts.size(), eb));
      region.push_back(cap_rows);
      cap_rows += blk_cap.back() * ws_final_grid(starts.size(), eb);
      plist.push_back(plist[i]);
    }
    if (plist.size() > (size_t)MAX_TYPES_Q) return E.fail(NBG_E_UNSUPPORTED, "too many edge types");
    if (int32_t rrc = ws_release(E, &E.ws, E.stream)) return rrc;   // a held device GO result keeps its rows
    if (starts.size() > ws_cap_frontier(E.ws)) return E.fail(NBG_E_UNSUPPORTED, "too many vertices in one request");
    static std::atomic<uint64_t> gn_id{1ull << 62};   // program cache keys disjoint from GO statements
    Workspace* ws = E.ws;
    if (tr_.on) tr_.mark(0);
    hipError_t he = ws_reserve_rows(ws, cap_rows, ncols);
    if (he == hipSuccess) he = ws_begin_query(ws, starts.data(), starts.size(), &plist, gn_id++);
    for (size_t i = 0; he == hipSuccess && i < plist.size(); ++i) {
      const DevEdgeType& top = E.snap.types.at(ectx[active[i < active.size() ? i : olds[i - active.size()]]].type);
      const DevEdgeType& dt = i < active.size() ? top : *top.old;
      ExpandArgs a{};
      a.now_sec = (int64_t)time(nullptr);   // now() in a storage filter: the request's second
      a.rand_seed = (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count() * 0x9e3779b97f4a7c15ull;
      a.row_ptr = dt.row_ptr;
      a.col = dt.col;
      a.dst_vid = dt.dst_vid;
      a.rank = dt.rank;
      a.valid = dt.valid;
      a.visible = nullptr;   // the part check above replaces the visibility test
      a.vids = E.snap.d_vids;
      a.str = E.dev_strings();
      a.props = dt.d_props;
      a.hprops = dt.props.data();
      a.hnarrow = nullptr;
      a.hnarrow_bytes = nullptr;
      a.cap = 0x7fffffff;    // the cap counts ACCEPTED edges: applied on the host below
      a.tcols = E.snap.d_tcols;
      a.tpres = E.snap.d_tpres;
      a.gbase = E.partitioned() ? (uint32_t)((uint64_t)E.cfg.rank * E.npad) : 0u;
      he = ws_expand_final(ws, a, starts.size(), ebound[i], 1, (int)i, plist[i], region[i], blk_cap[i], nullptr);
    }
    // the end of the request packs a small result into mapped host memory with the query's state
    // (k_q_out_small): such a request costs one host round trip, not two
    if (he == hipSuccess) {
      SmallPack sp{};
      sp.ntypes = (int)plist.size();
      sp.ncols = ncols;
      for (size_t i = 0; i < plist.size(); ++i) {
        sp.region[i] = region[i];
        sp.blk_cap[i] = blk_cap[i];
        sp.grid[i] = ws_final_grid_of(ws, (int)i);
      }
      he = ws_end_query_async_small(ws, sp);
    }
    if (he == hipSuccess) he = ws_end_query_wait(ws);
    if (he != hipSuccess) return E.fail(NBG_E_DEVICE, std::string("HIP: ") + hipGetErrorString(he));
    if (tr_.on) tr_.mark(1);
    uint64_t all_rows = 0;
    for (size_t i = 0; i < plist.size(); ++i) {
      const unsigned grid = ws_final_grid_of(ws, (int)i);
      const uint32_t* per = ws_host_blk_rows(ws, (int)i);
      for (unsigned b = 0; b < grid; ++b) all_rows += per[b];
    }
    const int64_t* small = ws_host_small_rows(ws, all_rows);   // (nullptr: too large, fetched below)
    // the packed rows out of the mapped block in one pass (each column below is then walked
    // in key order, a gather the mapped pages would serve a line at a time)
    std::vector<int64_t> small_rows;
    if (small) {
      small_rows.assign(small, small + (size_t)ncols * all_rows);   // (k_q_out_small: ncols columns)
      small = small_rows.data();
    }
    if (tr_.on) tr_.mark(2);
    uint64_t small_off = 0;
    for (size_t i = 0; i < plist.size(); ++i) {
      const int nc = (int)plist[i].yield_reg.size();
      const unsigned grid = ws_final_grid_of(ws, (int)i);
      const uint32_t* per = ws_host_blk_rows(ws, (int)i);
      std::vector<std::pair<uint64_t, uint64_t>> segs;
      uint64_t total = 0;
      for (unsigned b = 0; b < grid; ++b)
        if (per[b]) {
          segs.emplace_back(region[i] + (uint64_t)b * blk_cap[i], per[b]);
          total += per[b];
        }
      std::vector<const int64_t*> cols(nc);
      // the rows: in the mapped small block (column c at c * all_rows, this type's rows after the
      // earlier types'), or into a pinned block of the engine's pool (column c at c * total),
      // packed there by the device (a pageable copy per column cost more than the expansion)
      size_t hbytes = 0;
      int64_t* hb = nullptr;
      if (small) {
        for (int c = 0; c < nc; ++c) cols[c] = small + (size_t)c * all_rows + small_off;
        small_off += total;
      } else {
        hb = total ? static_cast<int64_t*>(E.pinned_get(total * (size_t)nc * 8, &hbytes)) : nullptr;
        if (total && !hb) return E.fail(NBG_E_OUT_OF_MEMORY, "row fetch staging");
        for (int c = 0; c < nc; ++c) cols[c] = hb + (size_t)c * total;
      }
      struct Put {   // (the block goes back to the pool on every path out of this scope)
        Engine& e; int64_t* p; size_t n;
        ~Put() { if (p) e.pinned_put(p, n); }
      } put{E, hb, hbytes};
      if (!small && total && ws_fetch_rows_pinned(ws, segs, nc, total, hb) != hipSuccess)
        return E.fail(NBG_E_DEVICE, "row fetch failed");
      // key order: CSR index order (rows of one source are contiguous and sorted)
      // (edge indices are < 2^32 per type and rows < 2^32: one packed key per row, sorted as
      // plain integers, then unpacked to row numbers)
      std::vector<uint64_t> ord(total);
      for (uint64_t r = 0; r < total; ++r) ord[r] = ((uint64_t)cols[1][r] << 32) | r;
      std::sort(ord.begin(), ord.end());
      for (uint64_t r = 0; r < total; ++r) ord[r] &= 0xFFFFFFFFull;
      if (i >= active.size()) {   // older versions: per vid in key order, tagged with their live edge
        const size_t k = active[olds[i - active.size()]];
        const DevEdgeType& od = *E.snap.types.at(ectx[k].type).old;
        const std::vector<int>& ymap = yield_of[k];
        for (uint64_t r = 0; r < total; ++r) {
          const uint64_t q = ord[r];
          std::vector<int64_t> vals(ymap.size());
          for (size_t p = 0; p < ymap.size(); ++p) vals[p] = cols[ymap[p]][q];
          orows[k].by_vid[cols[0][q]].emplace_back(od.h_grp[(size_t)cols[1][q]], std::move(vals));
        }
        continue;
      }
      TypeRows& tr = trows[active[i]];
      tr.vid.resize(total);
      tr.eidx.resize(total);
      const std::vector<int>& ymap = yield_of[active[i]];
      tr.vals.assign(ymap.size(), std::vector<int64_t>(total));
      for (uint64_t r = 0; r < total; ++r) {
        tr.vid[r] = cols[0][ord[r]];
        tr.eidx[r] = cols[1][ord[r]];
        for (size_t p = 0; p < ymap.size(); ++p) tr.vals[p][r] = cols[ymap[p]][ord[r]];
      }
      tr.range.reserve(starts.size());
      for (uint64_t r = 0; r < total;) {
        uint64_t e = r;
        while (e < total && tr.vid[e] == tr.vid[r]) ++e;
        tr.range[tr.vid[r]] = {r, e};
        r = e;
      }
    }
  }

  if (tr_.on) tr_.mark(3);
  // --- responses per requested vertex, in part order (QueryBaseProcessor::genBuckets order)
  const uint64_t cap = (uint64_t)(E.cfg.max_edge_returned_per_vertex <= 0 ? 0x7fffffff : E.cfg.max_edge_returned_per_vertex);
  const auto& dict = E.snap.strings;
  static const std::string kEmpty;
  auto str_of = [&](int64_t code) -> const std::string& {
    return (code >= 0 && (code & 1) == 0 && (uint64_t)(code / 2) < dict.size()) ? dict[code / 2] : kEmpty;
  };
  auto put_value = [&](RowBytes& w, int32_t type, int64_t bits) {
    switch (kindOfType(type)) {   // RowReader::getPropByName -> VariantType -> PropsCollector
      case VK_INT: w.put_int(bits); break;
      case VK_DOUBLE: w.put_double(bits); break;
      case VK_BOOL: w.put_bool(bits); break;
      case VK_STRING: w.put_string(str_of(bits)); break;
    }
  };
  if (stats) {
    stats->acc.assign(ret_index, StatAcc{});
    for (auto& tc : tctx)
      for (auto& pc : tc.props) stats->acc[pc.ret] = StatAcc{pc.name, pc.stat, kindOfType(pc.type) == VK_DOUBLE};
    for (auto& ec : ectx)
      for (auto& pc : ec.props)
        stats->acc[pc.ret] = StatAcc{pc.name, pc.stat, !pc.pik && kindOfType(pc.type) == VK_DOUBLE};
  }
  auto collect = [&](const PropCtx& pc, int64_t bits) {   // StatsCollector::collect*
    StatAcc& a = stats->acc[pc.ret];
    if (pc.pik == 1 || pc.pik == 2) return;                // collectVid: nothing
    if (pc.pik) { a.isum += bits; ++a.count; return; }    // _type / _rank: collectInt64
    switch (kindOfType(pc.type)) {
      case VK_INT: a.isum += bits; break;
      case VK_DOUBLE: { double d; memcpy(&d, &bits, 8); a.dsum += d; break; }
      default: break;                                      // bool / string: count only
    }
    ++a.count;
  };
  std::vector<uint64_t> order(rq->num_vids);
  for (uint64_t i = 0; i < rq->num_vids; ++i) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](uint64_t a, uint64_t b) { return rq->parts[a] < rq->parts[b]; });
  std::vector<int32_t> stat_failed;   // parts with a failed vertex (boundStats)
  // one requested vertex: its tag rows and RowSets (boundStats: its values collected) -> whether
  // it is returned; `edges` counts the rows it returned
  auto vertex = [&](uint64_t i, nbg_gn_response::Vertex& v, uint64_t& edges) -> bool {
    if (!part_ok(rq->parts[i])) return false;
    v.vid = rq->vids[i];
    const uint32_t d = dense[i];
    if (stats) {
      // QueryStatsProcessor::processVertex: a requested tag the vertex lacks fails the vertex
      // (ERR_KEY_NOT_FOUND -> E_UNKNOWN, BaseProcessor.inl:14-29), first failure per part
      bool missing = false;
      for (auto& tc : tctx) missing = missing || d == NO_ROW || !E.snap.tags.at(tc.tag).h_present[d];
      if (missing) {
        if (std::find(stat_failed.begin(), stat_failed.end(), rq->parts[i]) == stat_failed.end()) {
          stat_failed.push_back(rq->parts[i]);
          resp->failed.emplace_back(NBG_E_UNKNOWN, rq->parts[i]);
        }
        return false;
      }
    }
    if (d == NO_ROW) return false;   // no keys in this part: no edges, not returned
    for (auto& tc : tctx) {      // collectVertexProps: the tag's live record, returned props
      const DevTag& dtg = E.snap.tags.at(tc.tag);
      if (!dtg.h_present[d]) continue;
      if (stats) {
        if (dtg.h_present[d] == 1)
          for (auto& pc : tc.props) collect(pc, dtg.h_cols[pc.col][d]);
        continue;
      }
      RowBytes w;
      if (dtg.h_present[d] == 1)
        for (auto& pc : tc.props) put_value(w, pc.type, dtg.h_cols[pc.col][d]);
      if (w.cols > 0) v.tags.emplace_back(tc.tag, w.encode());
    }
    for (size_t k = 0; k < ectx.size(); ++k) {
      const EdgeCtx& ec = ectx[k];
      if (ec.props.empty()) continue;
      const TypeRows& tr = trows[k];
      auto it = tr.range.find(v.vid);
      // an older version passing before the first accepted live edge comes first (firstLoop)
      const std::vector<int64_t>* first_old = nullptr;
      if (auto ot = orows[k].by_vid.find(v.vid); ot != orows[k].by_vid.end()) {
        const int64_t j1 = it == tr.range.end() ? INT64_MAX : tr.eidx[it->second.first];
        if ((int64_t)ot->second.front().first < j1) first_old = &ot->second.front().second;
      }
      if (it == tr.range.end() && !first_old) continue;
      std::string rs;
      uint64_t lo = 0, hi = 0;
      RowBytes w;
      if (it != tr.range.end()) {
        lo = it->second.first;
        hi = std::min(it->second.second, it->second.first + cap - (first_old ? 1 : 0));
      }
      auto put_row = [&](const std::vector<int64_t>* row, uint64_t r) {
        w.clear();
        for (size_t p = 0; p < ec.props.size(); ++p) {
          const PropCtx& pc = ec.props[p];
          const int64_t x = row ? (*row)[p] : tr.vals[p][r];
          switch (pc.pik) {
            case 1: case 2: w.put_vid(x); break;
            case 3: case 4: w.put_int(x); break;
            default: put_value(w, pc.type, x);
          }
        }
        w.append_to(rs);
        ++edges;
      };
      if (stats) {
        if (first_old)
          for (size_t p = 0; p < ec.props.size(); ++p) collect(ec.props[p], (*first_old)[p]);
        for (uint64_t r = lo; r < hi; ++r)
          for (size_t p = 0; p < ec.props.size(); ++p) collect(ec.props[p], tr.vals[p][r]);
        edges += hi - lo + (first_old ? 1 : 0);
        continue;
      }
      if (first_old) put_row(first_old, 0);
      for (uint64_t r = lo; r < hi; ++r) put_row(nullptr, r);
      if (!rs.empty()) v.edges.emplace_back(ec.type, std::move(rs));
    }
    return !v.edges.empty();   // only vertices with edges (QueryBoundProcessor.cpp:104-107)
  };
  if (stats) {   // (collects into shared sums: in order, on this thread)
    for (uint64_t i : order) {
      nbg_gn_response::Vertex v;
      uint64_t e = 0;
      vertex(i, v, e);
      resp->edges += e;
    }
  } else {
    // the vertices' responses are independent: encoded in parallel (storaged's handler threads
    // split a request's vertices the same way, QueryBaseProcessor::genBuckets), kept in order
    const int64_t nq = (int64_t)order.size();
    std::vector<nbg_gn_response::Vertex> outv((size_t)nq);
    std::vector<uint64_t> ne((size_t)nq, 0);
    std::vector<uint8_t> keep((size_t)nq, 0);
    // A team of 4 (NBG_GN_THREADS; 0: the OpenMP default): a QueryBoundBenchmark request's encode
    // took 28-31 us with 4 threads against 50-56 with the box's 16 and 41-42 with 8, where waking
    // and joining the larger team cost more than its share of the work (profiles/r04_af_gn_team_ab.txt)
    static const int team = getenv("NBG_GN_THREADS") ? std::max(0, atoi(getenv("NBG_GN_THREADS"))) : 4;
#pragma omp parallel for schedule(dynamic, 16) if (nq >= 64) num_threads(team > 0 ? team : omp_get_max_threads())
    for (int64_t k = 0; k < nq; ++k) keep[(size_t)k] = vertex(order[(size_t)k], outv[(size_t)k], ne[(size_t)k]) ? 1 : 0;
    resp->vertices.reserve((size_t)nq);
    for (int64_t k = 0; k < nq; ++k) {
      resp->edges += ne[(size_t)k];
      if (keep[(size_t)k]) resp->vertices.push_back(std::move(outv[(size_t)k]));
    }
  }
  // --- onProcessFinished: schemas of the returned columns
  for (auto& tc : tctx) {
    nbg_gn_response::Sch s{tc.tag, {}};
    for (auto& pc : tc.props) s.cols.emplace_back(pc.name, pc.type);
    if (!s.cols.empty()) resp->vschema.push_back(std::move(s));
  }
  for (auto& ec : ectx) {
    nbg_gn_response::Sch s{ec.type, {}};
    for (auto& pc : ec.props) s.cols.emplace_back(pc.name, pc.type);
    if (!s.cols.empty()) resp->eschema.push_back(std::move(s));
  }
  if (tr_.on) {
    tr_.mark(4);
    tr_.done();
  }
  return NBG_OK;
}

extern "C" {

int32_t nbg_get_neighbors(nbg_engine* h, const nbg_gn_request* rq, nbg_gn_response** out) {
  if (!h || !rq || !out || (rq->num_vids && (!rq->vids || !rq->parts)) ||
      (rq->num_edge_types && !rq->edge_types) || (rq->num_return_columns && !rq->return_columns))
    return NBG_E_INVALID_ARGUMENT;
  *out = nullptr;
  Engine& E = h->e;
  std::lock_guard<std::mutex> lg(E.mu);
  if (!E.finalized) return E.fail(NBG_E_STATE, "engine not finalized");
  if (hipSetDevice(E.cfg.device) != hipSuccess) return E.fail(NBG_E_DEVICE, "hipSetDevice failed");
  const auto t0 = std::chrono::steady_clock::now();
  auto* r = new nbg_gn_response();
  int32_t rc = get_neighbors(E, rq, r);
  if (rc) { delete r; return rc; }
  r->latency_us = (int32_t)std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0)
                      .count();
  *out = r;
  return NBG_OK;
}

// ---- boundStats (StorageServiceHandler::future_boundStats -> QueryStatsProcessor)
struct nbg_stats_response {
  std::vector<std::pair<int32_t, int32_t>> failed;
  std::vector<std::pair<std::string, int32_t>> schema;   // (name, NBG_T_INT / NBG_T_DOUBLE)
  std::vector<int64_t> bits;                            // value per column (int64 or double bits)
  std::string data;                                     // the encoded row (RowWriter, schema-less)
  uint64_t edges = 0;
};

int32_t nbg_bound_stats(nbg_engine* h, const nbg_gn_request* rq, const int32_t* stats, nbg_stats_response** out) {
  if (!h || !rq || !out || (rq->num_return_columns && !stats) || (rq->num_vids && (!rq->vids || !rq->parts)) ||
      (rq->num_edge_types && !rq->edge_types) || (rq->num_return_columns && !rq->return_columns))
    return NBG_E_INVALID_ARGUMENT;
  *out = nullptr;
  Engine& E = h->e;
  std::lock_guard<std::mutex> lg(E.mu);
  if (!E.finalized) return E.fail(NBG_E_STATE, "engine not finalized");
  if (hipSetDevice(E.cfg.device) != hipSuccess) return E.fail(NBG_E_DEVICE, "hipSetDevice failed");
  nbg_gn_response tmp;
  StatsSink sink;
  int32_t rc = get_neighbors(E, rq, &tmp, stats, &sink);
  if (rc) return rc;
  auto* r = new nbg_stats_response();
  r->failed = tmp.failed;
  r->edges = tmp.edges;
  if (!sink.acc.empty() || r->failed.empty()) {   // not a request-level error
    // QueryStatsProcessor::calcResult (QueryStatsProcessor.cpp:16-63)
    RowBytes w;
    for (auto& a : sink.acc) {
      int64_t bits = 0;
      switch (a.stat) {
        case NBG_STAT_SUM:
          if (a.dbl) { memcpy(&bits, &a.dsum, 8); w.put_double(bits); r->schema.emplace_back(a.name, NBG_T_DOUBLE); }
          else { bits = a.isum; w.put_int(bits); r->schema.emplace_back(a.name, NBG_T_INT); }
          break;
        case NBG_STAT_COUNT:
          bits = a.count;
          w.put_int(bits);
          r->schema.emplace_back(a.name, NBG_T_INT);
          break;
        case NBG_STAT_AVG: {
          const double v = a.dbl ? a.dsum / a.count : (double)a.isum / a.count;
          memcpy(&bits, &v, 8);
          w.put_double(bits);
          r->schema.emplace_back(a.name, NBG_T_DOUBLE);
          break;
        }
        default: continue;   // no stat set: no column
      }
      r->bits.push_back(bits);
    }
    r->data = w.encode();
  }
  *out = r;
  return NBG_OK;
}
int32_t nbg_stats_num_failed(const nbg_stats_response* r) { return r ? (int32_t)r->failed.size() : -1; }
int32_t nbg_stats_failed(const nbg_stats_response* r, int32_t i, int32_t* code, int32_t* part) {
  if (!r || i < 0 || i >= (int32_t)r->failed.size() || !code || !part) return NBG_E_INVALID_ARGUMENT;
  *code = r->failed[i].first;
  *part = r->failed[i].second;
  return NBG_OK;
}
int32_t nbg_stats_num_cols(const nbg_stats_response* r) { return r ? (int32_t)r->schema.size() : -1; }
int32_t nbg_stats_col(const nbg_stats_response* r, int32_t c, const char** name, int32_t* type, int64_t* bits) {
  if (!r || c < 0 || c >= (int32_t)r->schema.size() || !name || !type || !bits) return NBG_E_INVALID_ARGUMENT;
  *name = r->schema[c].first.c_str();
  *type = r->schema[c].second;
  *bits = r->bits[c];
  return NBG_OK;
}
int32_t nbg_stats_data(const nbg_stats_response* r, const uint8_t** data, uint64_t* len) {
  if (!r || !data || !len) return NBG_E_INVALID_ARGUMENT;
  *data = reinterpret_cast<const uint8_t*>(r->data.data());
  *len = r->data.size();
  return NBG_OK;
}
void nbg_stats_free(nbg_stats_response* r) { delete r; }

int32_t nbg_gn_num_failed(const nbg_gn_response* r) { return r ? (int32_t)r->failed.size() : -1; }
int32_t nbg_gn_failed(const nbg_gn_response* r, int32_t i, int32_t* code, int32_t* part) {
  if (!r || i < 0 || i >= (int32_t)r->failed.size() || !code || !part) return NBG_E_INVALID_ARGUMENT;
  *code = r->failed[i].first;
  *part = r->failed[i].second;
  return NBG_OK;
}
int32_t nbg_gn_latency_us(const nbg_gn_response* r) { return r ? r->latency_us : -1; }
int32_t nbg_gn_num_schemas(const nbg_gn_response* r, int32_t is_edge) {
  return r ? (int32_t)(is_edge ? r->eschema : r->vschema).size() : -1;
}
int32_t nbg_gn_schema(const nbg_gn_response* r, int32_t is_edge, int32_t i, int32_t* id, int32_t* ncols) {
  if (!r || !id || !ncols) return NBG_E_INVALID_ARGUMENT;
  const auto& v = is_edge ? r->eschema : r->vschema;
  if (i < 0 || i >= (int32_t)v.size()) return NBG_E_INVALID_ARGUMENT;
  *id = v[i].id;
  *ncols = (int32_t)v[i].cols.size();
  return NBG_OK;
}
int32_t nbg_gn_schema_col(const nbg_gn_response* r, int32_t is_edge, int32_t i, int32_t c, const char** name,
                          int32_t* type) {
  if (!r || !name || !type) return NBG_E_INVALID_ARGUMENT;
  const auto& v = is_edge ? r->eschema : r->vschema;
  if (i < 0 || i >= (int32_t)v.size() || c < 0 || c >= (int32_t)v[i].cols.size()) return NBG_E_INVALID_ARGUMENT;
  *name = v[i].cols[c].first.c_str();
  *type = v[i].cols[c].second;
  return NBG_OK;
}
int64_t nbg_gn_num_vertices(const nbg_gn_response* r) { return r ? (int64_t)r->vertices.size() : -1; }
int64_t nbg_gn_vertex_id(const nbg_gn_response* r, int64_t i) {
  return (r && i >= 0 && i < (int64_t)r->vertices.size()) ? r->vertices[i].vid : 0;
}
int32_t nbg_gn_vertex_num_tags(const nbg_gn_response* r, int64_t i) {
  return (r && i >= 0 && i < (int64_t)r->vertices.size()) ? (int32_t)r->vertices[i].tags.size() : -1;
}
int32_t nbg_gn_vertex_num_edges(const nbg_gn_response* r, int64_t i) {
  return (r && i >= 0 && i < (int64_t)r->vertices.size()) ? (int32_t)r->vertices[i].edges.size() : -1;
}
static int32_t gn_item(const nbg_gn_response* r, int64_t i, int32_t k, bool edges, int32_t* id, const uint8_t** data,
                       uint64_t* len) {
  if (!r || i < 0 || i >= (int64_t)r->vertices.size() || !id || !data || !len) return NBG_E_INVALID_ARGUMENT;
  const auto& v = edges ? r->vertices[i].edges : r->vertices[i].tags;
  if (k < 0 || k >= (int32_t)v.size()) return NBG_E_INVALID_ARGUMENT;
  *id = v[k].first;
  *data = reinterpret_cast<const uint8_t*>(v[k].second.data());
  *len = v[k].second.size();
  return NBG_OK;
}
int32_t nbg_gn_vertex_tag(const nbg_gn_response* r, int64_t i, int32_t k, int32_t* tag, const uint8_t** data,
                          uint64_t* len) {
  return gn_item(r, i, k, false, tag, data, len);
}
int32_t nbg_gn_vertex_edges(const nbg_gn_response* r, int64_t i, int32_t k, int32_t* type, const uint8_t** data,
                            uint64_t* len) {
  return gn_item(r, i, k, true, type, data, len);
}
uint64_t nbg_gn_edges(const nbg_gn_response* r) { return r ? r->edges : 0; }
void nbg_gn_free(nbg_gn_response* r) { delete r; }

}  // extern "C"
