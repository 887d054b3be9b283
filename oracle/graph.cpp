// Test infrastructure (oracle) — graphd traversal executors restated:
//   GoExecutor (src/graph/GoExecutor.cpp:83-984)
//   FindPathExecutor (src/graph/FindPathExecutor.cpp:145-715)
#include <algorithm>
#include <functional>
#include <set>
#include <tuple>
#include "orc.h"

namespace orc {

namespace {

// ExpressionContext::add* collection done by Expression::prepare (Expressions.cpp:137-140, 314-400)
struct Needs {
  std::set<std::pair<std::string, std::string>> src, dst, alias;
};
void collect(const Expr* e, Needs& n) {
  if (!e) return;
  switch (e->kind) {
    case kSourceProp: n.src.insert({e->alias, e->prop}); break;
    case kDestProp: n.dst.insert({e->alias, e->prop}); break;
    case kAliasProp: case kEdgeRank: case kEdgeDstId: case kEdgeSrcId: case kEdgeType:
      n.alias.insert({e->alias, e->prop}); break;
    default: break;
  }
  collect(e->a.get(), n);
  collect(e->b.get(), n);
  for (auto& x : e->args) collect(x.get(), n);
}

// GoExecutor::VertexHolder (GoExecutor.cpp:986-1064)
struct VertexHolder {
  std::unordered_map<int64_t, std::unordered_map<int32_t, std::pair<Schema, std::string>>> data;
  void add(const QueryResponse& r) {
    for (auto& vd : r.vertices) {
      std::unordered_map<int32_t, std::pair<Schema, std::string>> m;
      for (auto& td : vd.tags) {
        auto it = r.vertexSchema.find(td.tag);
        if (it != r.vertexSchema.end()) m[td.tag] = {it->second, td.data};
      }
      data[vd.vid] = std::move(m);
    }
  }
  OptValue defaultFor(int32_t tid, const std::string& prop) const {
    for (auto& kv : data) {
      auto it = kv.second.find(tid);
      if (it != kv.second.end()) return defaultProp(it->second.first, prop);
    }
    return Status::Err("Unknown Vertex");
  }
  SType typeFor(int64_t vid, int32_t tid, const std::string& prop) const {
    auto it = data.find(vid);
    if (it != data.end()) {
      auto jt = it->second.find(tid);
      if (jt != it->second.end()) return jt->second.first.typeOf(prop);
    }
    for (auto& kv : data) {
      auto jt = kv.second.find(tid);
      if (jt != kv.second.end()) return jt->second.first.typeOf(prop);
    }
    return ST_UNKNOWN;
  }
  OptValue get(int64_t vid, int32_t tid, const std::string& prop) const {
    auto it = data.find(vid);
    if (it == data.end()) return defaultFor(tid, prop);
    auto jt = it->second.find(tid);
    if (jt == it->second.end()) return defaultFor(tid, prop);
    RowReader r(jt->second.second, &jt->second.first);
    auto v = r.get(prop);
    if (!v.ok()) return Status::Err("get prop failed");
    return v;
  }
};

// GoExecutor::processFinalResult getters (GoExecutor.cpp:851-945)
struct GoGetters : Getters {
  const Store& st;
  int32_t edgeType = 0;
  RowReader* row = nullptr;
  const Schema* rowSchema = nullptr;
  const std::unordered_map<int32_t, Schema>* edgeSchema = nullptr;
  const std::unordered_map<int32_t, Schema>* tagSchema = nullptr;
  const std::vector<TagData>* tagData = nullptr;
  const VertexHolder* holder = nullptr;
  bool saveType = false;
  SType* colType = nullptr;
  // InterimResultIndex (InterimResult.cpp:158-270) + VertexBackTracker (GoExecutor.h:169-188)
  const GoQuery* q = nullptr;
  const std::unordered_map<int64_t, size_t>* index = nullptr;
  const std::unordered_map<int64_t, int64_t>* tracker = nullptr;   // null when steps == 1
  int64_t srcVid = 0;
  explicit GoGetters(const Store& s) : st(s) {}

  OptValue inputProp(const std::string& prop) override {
    if (!index) return Status::Err("no input");
    int64_t root = srcVid;
    if (tracker) {
      auto t = tracker->find(srcVid);
      if (t == tracker->end()) return Status::Err("no root");
      root = t->second;
    }
    auto r = index->find(root);
    if (r == index->end()) return Status::Err("no input row");
    for (size_t c = 0; c < q->inputNames.size(); ++c)
      if (q->inputNames[c] == prop) return q->inputRows[r->second][c];
    return Status::Err("Prop `" + prop + "' not found");
  }

  OptValue aliasProp(const std::string& edge, const std::string& prop) override {
    auto et = st.edgeByName.find(edge);
    if (et == st.edgeByName.end()) return Status::Err("edge not found");
    if (saveType) *colType = rowSchema->typeOf(prop);
    if (edgeType != et->second) {
      auto it = edgeSchema->find(et->second);
      if (it == edgeSchema->end()) return Status::Err("get schema failed");
      return defaultProp(it->second, prop);
    }
    auto v = row->get(prop);
    if (!v.ok()) return Status::Err("get prop(" + edge + "." + prop + ") failed");
    return v;
  }
  OptValue srcTagProp(const std::string& tag, const std::string& prop) override {
    auto t = st.tagByName.find(tag);
    if (t == st.tagByName.end()) return Status::Err("tag not found");
    const TagData* td = nullptr;
    for (auto& x : *tagData) if (x.tag == t->second) { td = &x; break; }
    if (!td) return defaultProp(*rowSchema, prop);   // note: the edge row's schema (GoExecutor.cpp:896-898)
    auto sit = tagSchema->find(t->second);
    if (sit == tagSchema->end()) return Status::Err("no tag schema");
    if (saveType) *colType = sit->second.typeOf(prop);
    RowReader r(td->data, &sit->second);
    auto v = r.get(prop);
    if (!v.ok()) return Status::Err("get prop(" + tag + "." + prop + ") failed");
    return v;
  }
  OptValue dstTagProp(const std::string& tag, const std::string& prop) override {
    auto d = row->get("_dst");
    if (!d.ok()) return Status::Err("get prop failed");
    auto t = st.tagByName.find(tag);
    if (t == st.tagByName.end()) return Status::Err("tag not found");
    int64_t vid = std::get<0>(d.v);
    if (saveType) *colType = holder->typeFor(vid, t->second, prop);
    return holder->get(vid, t->second, prop);
  }
};

ResultSet goError(const std::string& m) { ResultSet r; r.code = E_EXECUTION_ERROR; r.err = m; return r; }

}  // namespace

// ---------------------------------------------------------------- GO
// GoExecutor::getEdgeNamesFromResp (GoExecutor.cpp:481-499) walks resp[0].edge_schema, a
// std::unordered_map (storage.thrift:104) that graphd decoded from storaged's own
// unordered_map (QueryBoundProcessor.cpp:139-158), which was filled by walking
// edgeContexts_ (unordered_map, QueryBaseProcessor.h:114) built from the request's types
// with std::inserter (QueryBaseProcessor.inl:46-57).  Restated hop by hop with the same
// libstdc++ containers.
std::vector<int32_t> responseEdgeSchemaOrder(const std::vector<int32_t>& reqTypes) {
  std::unordered_map<int32_t, std::vector<int>> edgeContexts;
  for (int32_t t : reqTypes) edgeContexts.insert(edgeContexts.end(), {t, std::vector<int>{}});
  std::unordered_map<int32_t, std::string> storagedSchema;
  for (const auto& ec : edgeContexts) {
    if (storagedSchema.find(ec.first) == storagedSchema.end()) storagedSchema.emplace(ec.first, "_dst");
  }
  std::unordered_map<int32_t, std::string> graphdSchema;   // thrift map decode
  for (const auto& kv : storagedSchema) graphdSchema.emplace(kv.first, kv.second);
  std::vector<int32_t> names;
  for (const auto& kv : graphdSchema) names.push_back(kv.first);
  return names;
}

// storaged's edgeContexts_ iteration order for the request's types: the order processVertex
// emits a vertex's edge data in (QueryBaseProcessor.inl:46-57)
std::vector<int32_t> edgeContextOrder(const std::vector<int32_t>& reqTypes) {
  std::unordered_map<int32_t, std::vector<int>> edgeContexts;
  for (int32_t t : reqTypes) edgeContexts.insert(edgeContexts.end(), {t, std::vector<int>{}});
  std::vector<int32_t> order;
  for (const auto& kv : edgeContexts) order.push_back(kv.first);
  return order;
}

ResultSet runGo(const Store& st, const GoQuery& q) {
  ResultSet out;
  // prepareOver (GoExecutor.cpp:197-263)
  std::vector<int32_t> etypes = q.etypes;
  if (q.overAll) {
    etypes.clear();
    for (auto& kv : st.edgeSchemas) if (kv.first > 0) etypes.push_back(kv.first);
    std::sort(etypes.begin(), etypes.end());
  }
  for (auto et : etypes) if (!st.edgeNames.count(et)) return goError("edge not found");
  // prepareWhere / prepareYield: decode expressions
  std::unique_ptr<Expr> filter;
  if (!q.where.empty()) {
    std::string err;
    filter = decodeExpr(reinterpret_cast<const uint8_t*>(q.where.data()), q.where.size(), &err);
    if (!filter) return goError("bad where: " + err);
  }
  std::vector<std::unique_ptr<Expr>> yields;
  std::vector<std::string> colNames = q.yieldNames;
  for (auto& y : q.yields) {
    std::string err;
    auto e = decodeExpr(reinterpret_cast<const uint8_t*>(y.data()), y.size(), &err);
    if (!e) return goError("bad yield: " + err);
    yields.push_back(std::move(e));
  }
  bool defaultOverAllYield = false;
  if (yields.empty()) {
    if (q.overAll) {
      defaultOverAllYield = true;   // finishExecution (GoExecutor.cpp:546-561)
    } else {
      for (auto et : etypes) {     // parser.yy:518-531: EdgeDstIdExpression(edge name)
        auto e = std::make_unique<Expr>();
        e->kind = kEdgeDstId; e->alias = st.edgeNames.at(et); e->prop = "_dst";
        yields.push_back(std::move(e));
        colNames.push_back(st.edgeNames.at(et) + "._dst");
      }
    }
  }
  if (defaultOverAllYield) {
    for (auto et : responseEdgeSchemaOrder(etypes)) {
      auto e = std::make_unique<Expr>();
      e->kind = kEdgeDstId; e->alias = st.edgeNames.at(et); e->prop = "_dst";
      yields.push_back(std::move(e));
      colNames.push_back(st.edgeNames.at(et) + "._dst");
    }
  }
  while (colNames.size() < yields.size()) colNames.push_back("col" + std::to_string(colNames.size()));
  out.colNames = colNames;
  Needs needs;
  collect(filter.get(), needs);
  for (auto& y : yields) collect(y.get(), needs);

  // setupStarts + DISTINCT on starts (GoExecutor.cpp:97-107)
  std::vector<int64_t> starts = q.starts;
  if (starts.empty()) return out;
  if (q.distinct) {
    std::unordered_set<int64_t> u(starts.begin(), starts.end());
    starts.assign(u.begin(), u.end());
  }
  uint32_t steps = q.steps;
  std::unordered_map<int64_t, size_t> index;   // vidToRowIndex_: the last row of each vid wins
  const bool hasInput = q.inputVidCol >= 0;
  if (hasInput)
    for (size_t r = 0; r < q.inputRows.size(); ++r) index[std::get<0>(q.inputRows[r][q.inputVidCol])] = r;
  std::unordered_map<int64_t, int64_t> tracker;

  // ---- processFinalResult + setupInterimResult + InterimResult::getRows (GoExecutor.cpp:707-984,
  // InterimResult.cpp:74-153).  The result schema comes from the first row the reference
  // evaluates: a column's type is the type the LAST prop getter of its expression set (operands
  // left before right, no short-circuit), a root cast's type, else the value's kind; every row is
  // then written through that schema (RowWriter's incompatible-type defaults) and read back by it
  // (a default of another length shifts the later columns; a read past the row's end, or a FLOAT
  // column, fails the query).  Which row is first follows hash-map order; this restatement fixes
  // it (as the engine does) to an edge of the first type in the request's edge-context order whose
  // source carries the $^ tags the columns read.
  auto finish = [&](const QueryResponse& resp, const VertexHolder* holder) -> ResultSet {
    GoGetters g(st);
    g.holder = holder;
    g.q = &q;
    g.index = hasInput ? &index : nullptr;
    g.tracker = steps > 1 ? &tracker : nullptr;
    struct Rec { std::vector<Value> v; int32_t type; };
    std::vector<Rec> recs;
    for (auto& vd : resp.vertices) {
      for (auto& ed : vd.edges) {
        const Schema& s = resp.edgeSchema.at(ed.type);
        for (auto& row : rowSetSplit(ed.data)) {
          RowReader r(row, &s);
          g.edgeType = ed.type; g.row = &r; g.rowSchema = &s; g.srcVid = vd.vid;
          g.edgeSchema = &resp.edgeSchema; g.tagSchema = &resp.vertexSchema; g.tagData = &vd.tags;
          g.saveType = false;
          if (filter) {
            auto v = filter->eval(g);
            if (!v.ok()) return goError(v.st.msg);
            if (!asBool(v.v)) continue;
          }
          Rec rc;
          rc.type = ed.type;
          for (auto& y : yields) {
            auto v = y->eval(g);
            if (!v.ok()) return goError(v.st.msg);
            rc.v.push_back(v.v);
          }
          recs.push_back(std::move(rc));
        }
      }
    }
    if (recs.empty()) return out;
    const int32_t t0 = edgeContextOrder(etypes)[0];
    const Schema* rowSchema = resp.edgeSchema.count(t0) ? &resp.edgeSchema.at(t0) : nullptr;
    // the last getter's type, post-order (GoExecutor.cpp:851-945 save the type as they run)
    std::function<void(const Expr*, SType*)> last = [&](const Expr* e, SType* t) {
      if (!e) return;
      last(e->a.get(), t);
      last(e->b.get(), t);
      for (auto& x : e->args) last(x.get(), t);
      switch (e->kind) {
        case kAliasProp: case kEdgeRank: case kEdgeDstId: case kEdgeSrcId:
          if (st.edgeByName.count(e->alias)) *t = rowSchema ? rowSchema->typeOf(e->prop) : ST_UNKNOWN;
          break;
        case kSourceProp: case kDestProp: {
          auto it = st.tagByName.find(e->alias);
          if (it == st.tagByName.end()) break;
          const Schema* ts = st.tagSchema(it->second);
          *t = ts ? ts->typeOf(e->prop) : ST_UNKNOWN;
          break;
        }
        case kInputProp: case kVariableProp: {
          static const SType km[4] = {ST_INT, ST_DOUBLE, ST_BOOL, ST_STRING};
          *t = ST_UNKNOWN;
          for (size_t c = 0; c < q.inputNames.size(); ++c)
            if (q.inputNames[c] == e->prop && c < q.inputKinds.size()) *t = km[q.inputKinds[c] & 3];
          break;
        }
        default: break;
      }
    };
    const Rec* first = &recs[0];
    for (auto& r : recs)
      if (r.type == t0) { first = &r; break; }
    Schema outSchema;
    bool floatCol = false;
    for (size_t i = 0; i < yields.size(); ++i) {
      SType t = ST_UNKNOWN;
      if (yields[i]->kind == kTypeCasting) {
        static const SType m[] = {ST_INT, ST_STRING, ST_DOUBLE, ST_INT, ST_BOOL, ST_TIMESTAMP};
        t = m[yields[i]->castType % 6];
      } else {
        last(yields[i].get(), &t);
      }
      if (t == ST_UNKNOWN) {
        static const SType m[] = {ST_INT, ST_DOUBLE, ST_BOOL, ST_STRING};
        t = m[first->v[i].index()];
      }
      floatCol = floatCol || t == ST_FLOAT;
      outSchema.cols.push_back({colNames[i], t});
    }
    if (floatCol) return goError("Unknown Type: 4");
    std::unordered_set<std::string> uniq;
    for (auto& r : recs) {
      RowWriter w(&outSchema);
      for (auto& v : r.v) w.putValue(v, ST_UNKNOWN);
      std::string enc = w.encode();
      if (q.distinct && !uniq.insert(enc).second) continue;
      RowReader back(enc, &outSchema);
      std::vector<Value> decoded;
      for (size_t i = 0; i < r.v.size(); ++i) {
        auto v = back.getIdx((int)i);
        if (!v.ok()) return goError("Get value from interim failed");
        decoded.push_back(v.v);
      }
      out.rows.push_back(std::move(decoded));
    }
    return out;
  };

  for (uint32_t cur = 1;; ++cur) {
    bool final = cur >= steps;
    // getStepOutProps (GoExecutor.cpp:587-630)
    std::vector<PropDef> props;
    for (auto et : etypes) props.push_back({3, et, "_dst"});
    if (final) {
      for (auto& sp : needs.src) {
        auto it = st.tagByName.find(sp.first);
        if (it == st.tagByName.end()) return goError("No schema found for '" + sp.first + "'");
        props.push_back({1, it->second, sp.second});
      }
      for (auto& ap : needs.alias) {
        auto it = st.edgeByName.find(ap.first);
        if (it == st.edgeByName.end() ||
            std::find(etypes.begin(), etypes.end(), it->second) == etypes.end())
          return goError("the edge was not found '" + ap.first + "'");
        props.push_back({3, it->second, ap.second});
      }
    }
    QueryResponse resp = getNeighbors(st, starts, etypes, "", props);
    for (auto& vd : resp.vertices)
      for (auto& ed : vd.edges) out.scanned += rowSetSplit(ed.data).size();
    // completeness == 0 -> error (GoExecutor.cpp:426-430)
    {
      std::unordered_set<int32_t> reqParts;
      for (auto v : starts) reqParts.insert(partOf(v, st.numParts));
      if (!resp.failed.empty() && resp.failed.size() >= reqParts.size()) return goError("Get neighbors failed");
    }
    if (!final || !needs.dst.empty()) {
      // getDstIdsFromResp (GoExecutor.cpp:501-541)
      std::unordered_set<int64_t> set;
      for (auto& vd : resp.vertices) {
        for (auto& ed : vd.edges) {
          const Schema& s = resp.edgeSchema.at(ed.type);
          for (auto& row : rowSetSplit(ed.data)) {
            RowReader r(row, &s);
            auto d = r.get("_dst");
            if (d.ok()) set.insert(std::get<0>(d.v));
            if (!final && d.ok()) {   // VertexBackTracker::add (GoExecutor.cpp:531-533)
              int64_t value = vd.vid;
              auto it = tracker.find(vd.vid);
              if (it != tracker.end()) value = it->second;
              tracker[std::get<0>(d.v)] = value;
            }
          }
        }
      }
      std::vector<int64_t> dst(set.begin(), set.end());
      if (dst.empty()) return out;   // onEmptyInputs
      if (!final) { starts = std::move(dst); continue; }
      // fetchVertexProps (GoExecutor.cpp:652-690)
      GNRequest vreq;
      for (auto v : dst) vreq.parts[partOf(v, st.numParts)].push_back(v);
      for (auto& dp : needs.dst) {
        auto it = st.tagByName.find(dp.first);
        if (it == st.tagByName.end()) return goError("No schema found for '" + dp.first + "'");
        vreq.returns.push_back({2, it->second, dp.second});
      }
      auto vresp = getVertexProps(st, vreq);
      VertexHolder holder;
      holder.add(vresp);
      // fallthrough to finish with holder
      return finish(resp, &holder);
    }
    // final step without $$ props
    VertexHolder holder;
    return finish(resp, &holder);
  }
}

// ---------------------------------------------------------------- FIND PATH
namespace {

using Neighbor = PathStep;   // (dst, type, rank)
using Frontiers = std::vector<std::pair<int64_t, std::vector<Neighbor>>>;

// FindPathExecutor::getFrom/ToFrontiers + doFilter (FindPathExecutor.cpp:456-613)
Frontiers frontiers(const Store& st, const std::vector<int64_t>& vids, const std::vector<int32_t>& types) {
  std::vector<PropDef> props;
  for (auto t : types) for (const char* p : {"_dst", "_type", "_rank"}) props.push_back({3, t, p});
  QueryResponse resp = getNeighbors(st, vids, types, "", props);
  Frontiers f;
  for (auto& vd : resp.vertices) {
    for (auto& ed : vd.edges) {
      const Schema& s = resp.edgeSchema.at(ed.type);
      std::vector<Neighbor> ns;
      for (auto& row : rowSetSplit(ed.data)) {
        RowReader r(row, &s);
        auto d = r.get("_dst"), t = r.get("_type"), k = r.get("_rank");
        ns.push_back({std::get<0>(d.v), static_cast<int32_t>(std::get<0>(t.v)), std::get<0>(k.v)});
      }
      f.emplace_back(vd.vid, std::move(ns));
    }
  }
  return f;
}

// buildPathRow (FindPathExecutor.cpp:644-702) into the canonical entry list
std::vector<int64_t> entryList(const Path& path) {
  std::vector<int64_t> out;
  size_t i = 0;
  for (; i < path.size(); ++i) {
    if (path[i].type < 0) { out.push_back(path[i].id); ++i; goto tail; }
    out.push_back(path[i].id); out.push_back(path[i].type); out.push_back(path[i].rank);
  }
  return out;
tail:
  for (; i < path.size(); ++i) {
    out.push_back(-path[i].type); out.push_back(path[i].rank); out.push_back(path[i].id);
  }
  return out;
}

// canonical order: lexicographic over [v0,t0,r0,v1,...], signed
bool lexLess(const std::vector<int64_t>& a, const std::vector<int64_t>& b) {
  return std::lexicographical_compare(a.begin(), a.end(), b.begin(), b.end());
}

}  // namespace

int32_t runFindPath(const Store& st, const FindPathQuery& q, std::vector<std::vector<int64_t>>& out) {
  out.clear();
  // VerticesClause::prepare dedups literal vids (src/parser/Clauses.cpp:51-92)
  auto dedup = [](const std::vector<int64_t>& v) {
    std::vector<int64_t> r; std::unordered_set<int64_t> s;
    for (auto x : v) if (s.insert(x).second) r.push_back(x);
    return r;
  };
  std::vector<int64_t> fromV = dedup(q.from), toV = dedup(q.to);
  std::vector<int32_t> types = q.etypes, opp;
  if (q.overAll) {
    types.clear();
    for (auto& kv : st.edgeSchemas) if (kv.first > 0) types.push_back(kv.first);
    std::sort(types.begin(), types.end());
  }
  for (auto t : types) opp.push_back(-t);
  uint32_t steps = q.upto / 2 + q.upto % 2;                       // :155
  std::unordered_set<int64_t> visitedFrom(fromV.begin(), fromV.end());
  std::unordered_set<int64_t> visitedTo(toV.begin(), toV.end());
  std::unordered_set<int64_t> targetNotFound(toV.begin(), toV.end());
  std::multimap<int64_t, Path> pathFrom, pathTo;
  for (auto v : fromV) pathFrom.emplace(v, Path{});
  for (auto v : toV) pathTo.emplace(v, Path{});
  std::multimap<int64_t, std::vector<int64_t>> finalPath;     // target -> entry list
  std::unordered_map<int64_t, size_t> finalLen;

  auto record = [&](int64_t target, const Path& p) {
    auto el = entryList(p);
    if (!q.shortest) { finalPath.emplace(target, std::move(el)); return; }
    auto it = finalPath.find(target);
    if (it == finalPath.end()) { finalPath.emplace(target, std::move(el)); finalLen[target] = p.size(); return; }
    // first found wins in the reference (iteration order); canonical: smallest among equal length
    if (p.size() == finalLen[target] && lexLess(el, it->second)) it->second = std::move(el);
  };

  for (uint32_t cur = 1;; ++cur) {
    if (fromV.empty() || toV.empty()) break;                     // :175-178
    Frontiers ff = frontiers(st, fromV, types);
    Frontiers tf = frontiers(st, toV, opp);
    // findPath (:218-290)
    visitedFrom.clear();
    std::multimap<int64_t, Path> pathF;
    for (auto& fr : ff) {
      for (auto& nb : fr.second) {
        int64_t dst = nb.id;
        if (visitedTo.count(dst)) {                               // meetOddPath (:292-333)
          auto rf = pathFrom.equal_range(fr.first);
          for (auto i = rf.first; i != rf.second; ++i) {
            auto rt = pathTo.equal_range(dst);
            for (auto j = rt.first; j != rt.second; ++j) {
              if (j->second.size() + i->second.size() > q.upto) continue;
              Path p = i->second;
              p.push_back({fr.first, nb.type, nb.rank});
              p.push_back({dst, -nb.type, nb.rank});
              p.insert(p.end(), j->second.begin(), j->second.end());
              int64_t target = p.back().id;
              if (q.shortest) targetNotFound.erase(target);
              record(target, p);
            }
          }
        }
        // updatePath FROM (:384-411)
        auto r = pathFrom.equal_range(fr.first);
        for (auto i = r.first; i != r.second; ++i) {
          Path p = i->second;
          p.push_back({fr.first, nb.type, nb.rank});
          pathF.emplace(dst, std::move(p));
        }
        visitedFrom.insert(dst);
      }
    }
    pathFrom = std::move(pathF);
    fromV.assign(visitedFrom.begin(), visitedFrom.end());
    visitedTo.clear();
    std::multimap<int64_t, Path> pathT;
    for (auto& fr : tf) {
      for (auto& nb : fr.second) {
        auto r = pathTo.equal_range(fr.first);
        for (auto i = r.first; i != r.second; ++i) {
          Path p = i->second;
          p.insert(p.begin(), PathStep{fr.first, nb.type, nb.rank});
          pathT.emplace(nb.id, std::move(p));
        }
        visitedTo.insert(nb.id);
      }
    }
    pathTo = std::move(pathT);
    toV.assign(visitedTo.begin(), visitedTo.end());
    std::sort(fromV.begin(), fromV.end());
    std::sort(toV.begin(), toV.end());
    std::vector<int64_t> inter;
    std::set_intersection(fromV.begin(), fromV.end(), toV.begin(), toV.end(), std::back_inserter(inter));
    if (!inter.empty()) {
      if (q.shortest && targetNotFound.empty()) break;
      for (auto id : inter) {                                      // meetEvenPath (:335-382)
        auto rf = pathFrom.equal_range(id);
        auto rt = pathTo.equal_range(id);
        for (auto i = rf.first; i != rf.second; ++i) {
          for (auto j = rt.first; j != rt.second; ++j) {
            if (j->second.size() + i->second.size() > q.upto) continue;
            Path p = i->second;
            if (!j->second.empty()) {
              PathStep s = j->second.front(); s.id = id; s.type = -s.type; p.push_back(s);
            } else if (!i->second.empty()) {
              PathStep s = i->second.back(); s.id = id; p.push_back(s);
            }
            p.insert(p.end(), j->second.begin(), j->second.end());
            int64_t target = p.back().id;
            if (q.shortest) {
              if (finalPath.count(target) && finalLen[target] < p.size()) continue;
              targetNotFound.erase(target);
            }
            record(target, p);
          }
        }
      }
    }
    if (cur >= steps || (q.shortest && targetNotFound.empty())) break;
  }
  for (auto& kv : finalPath) out.push_back(kv.second);
  std::sort(out.begin(), out.end(), lexLess);
  return 0;
}

// Canonical BFS restatement of SHORTEST (for graphs where the faithful enumerator explodes).
int32_t runShortestBfs(const Store& st, const FindPathQuery& q, std::vector<std::vector<int64_t>>& out) {
  out.clear();
  std::vector<int64_t> S, T;
  { std::unordered_set<int64_t> s; for (auto x : q.from) if (s.insert(x).second) S.push_back(x); }
  { std::unordered_set<int64_t> s; for (auto x : q.to) if (s.insert(x).second) T.push_back(x); }
  std::vector<int32_t> types = q.etypes;
  if (q.overAll) {
    types.clear();
    for (auto& kv : st.edgeSchemas) if (kv.first > 0) types.push_back(kv.first);
    std::sort(types.begin(), types.end());
  }
  // out-neighbours with storage semantics (latest version, edge cap)
  auto nbrs = [&](int64_t v, std::vector<PathStep>& res) {
    res.clear();
    int32_t part = partOf(v, st.numParts);
    if (!st.parts.count(part)) return;
    const auto& kvs = st.parts.at(part);
    for (auto t : types) {
      auto rng = st.prefixRange(part, edgePrefix(part, v, t));
      int64_t lr = -1, ld = 0; bool first = true; int cnt = 0;
      for (size_t i = rng.first; i < rng.second && cnt < st.maxEdgePerVertex; ++i) {
        int64_t rk = keyRank(kvs.key(i).data()), d = keyDst(kvs.key(i).data());
        if (!first && rk == lr && d == ld) continue;
        lr = rk; ld = d; first = false; ++cnt;
        res.push_back({d, t, rk});
      }
    }
  };
  std::unordered_set<int64_t> Sset(S.begin(), S.end());
  std::unordered_map<int64_t, uint32_t> dist;   // walk length >= 1 from S
  std::vector<std::vector<int64_t>> level(1, S);
  std::vector<PathStep> nb;
  for (uint32_t l = 1; l <= q.upto; ++l) {
    std::vector<int64_t> next;
    for (auto v : level[l - 1]) {
      nbrs(v, nb);
      for (auto& e : nb) if (!dist.count(e.id)) { dist[e.id] = l; next.push_back(e.id); }
    }
    level.push_back(std::move(next));
    if (level.back().empty()) break;
  }
  for (auto t : T) {
    auto it = dist.find(t);
    if (it == dist.end()) continue;
    uint32_t L = it->second;
    std::vector<std::unordered_set<int64_t>> B(L + 1);
    B[L].insert(t);
    for (int i = (int)L - 1; i >= 0; --i) {
      for (auto u : level[i]) {
        if (i > 0 && Sset.count(u)) continue;
        nbrs(u, nb);
        for (auto& e : nb) if (B[i + 1].count(e.id)) { B[i].insert(u); break; }
      }
    }
    std::vector<int64_t> path;
    int64_t v = *std::min_element(B[0].begin(), B[0].end());
    path.push_back(v);
    for (uint32_t i = 0; i < L; ++i) {
      nbrs(v, nb);
      bool have = false; PathStep best{};
      for (auto& e : nb) {
        if (!B[i + 1].count(e.id)) continue;
        if (!have || std::make_tuple(e.type, e.rank, e.id) < std::make_tuple(best.type, best.rank, best.id)) {
          best = e; have = true;
        }
      }
      path.push_back(best.type); path.push_back(best.rank); path.push_back(best.id);
      v = best.id;
    }
    out.push_back(std::move(path));
  }
  std::sort(out.begin(), out.end(), lexLess);
  return 0;
}

}  // namespace orc
