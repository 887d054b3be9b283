// Test infrastructure (oracle) — storaged read path restated:
//   QueryBaseProcessor::process / checkAndBuildContexts / checkExp / collectEdgeProps /
//   collectVertexProps / collectProps / genBuckets (src/storage/QueryBaseProcessor.inl)
//   QueryBoundProcessor::processVertex / processEdge(Impl) / onProcessFinished
//   (src/storage/QueryBoundProcessor.cpp:16-161)
//   StorageClient::getNeighbors + clusterIdsToHosts (src/storage/client/StorageClient.cpp:94-124,
//   StorageClient.h:240-260)
#include <algorithm>
#include <future>
#include <mutex>
#include "orc.h"

namespace orc {

const Schema* Store::edgeSchema(int32_t et, int64_t ver) const {
  auto it = edgeSchemas.find(et);
  if (it == edgeSchemas.end() || it->second.empty()) return nullptr;
  if (ver < 0) return &it->second.rbegin()->second;
  auto jt = it->second.find(ver);
  return jt == it->second.end() ? nullptr : &jt->second;
}
const Schema* Store::tagSchema(int32_t tag, int64_t ver) const {
  auto it = tagSchemas.find(tag);
  if (it == tagSchemas.end() || it->second.empty()) return nullptr;
  if (ver < 0) return &it->second.rbegin()->second;
  auto jt = it->second.find(ver);
  return jt == it->second.end() ? nullptr : &jt->second;
}

// RocksEngine::prefix (src/kvstore/RocksEngine.cpp:189-198): Seek(prefix), iterate while
// the key starts with prefix; bytewise (memcmp) comparator.
std::pair<size_t, size_t> Store::prefixRange(int32_t part, const std::string& prefix) const {
  auto it = parts.find(part);
  if (it == parts.end()) return {0, 0};
  const PartKV& v = it->second;
  size_t lo = 0, hi = v.size();
  while (lo < hi) {
    size_t mid = (lo + hi) / 2;
    if (v.key(mid) < std::string_view(prefix)) lo = mid + 1; else hi = mid;
  }
  size_t e = lo;
  while (e < v.size() && v.key(e).substr(0, prefix.size()) == prefix) ++e;
  return {lo, e};
}

// stable bytewise sort; identical keys keep the LAST write (RocksDB write-batch semantics)
void PartKV::finalize() {
  uint32_t n = (uint32_t)(koff.size() - 1);
  std::vector<uint32_t> idx(n);
  for (uint32_t i = 0; i < n; ++i) idx[i] = i;
  std::stable_sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) { return rkey(a) < rkey(b); });
  order.clear();
  order.reserve(n);
  for (uint32_t i = 0; i < n; ++i) {
    if (i + 1 < n && rkey(idx[i + 1]) == rkey(idx[i])) continue;
    order.push_back(idx[i]);
  }
}

namespace {

struct PropCtx {
  PropDef prop;
  SType type = ST_UNKNOWN;
  int pik = 0;            // 0 none, 1 src, 2 dst, 3 type, 4 rank
  bool returned = false;
  bool filtered = false;  // from a $^ filter
  int retIndex = -1;
  // StatsCollector state (Collector.h:76-109); the reference's sum_ starts as int64 0 and a
  // double value would hit boost::bad_get — restated here as a double sum
  int64_t isum = 0;
  double dsum = 0;
  int32_t count = 0;
  std::string tagName;
};
struct TagCtx { int32_t tag; std::vector<PropCtx> props; std::vector<std::string> filterNames; };
using TagFilters = std::map<std::pair<std::string, std::string>, Value>;

struct Processor {
  const Store& st;
  std::vector<TagCtx> tagCtx;
  // edgeContexts_: std::unordered_map in the reference; iteration order is unspecified,
  // so the oracle keeps request order (results are compared as sets).
  std::vector<std::pair<int32_t, std::vector<PropCtx>>> edgeCtx;
  std::unique_ptr<Expr> exp;
  std::mutex lock;
  bool stats = false;     // QueryStatsProcessor: collect into the PropCtx accumulators
  int retIndex = 0;
  // QueryBaseProcessor::validOperation (QueryBaseProcessor.inl:18-35)
  static bool validOp(SType t, int32_t stat) {
    if (stat != 1 && stat != 3) return true;
    return t == ST_INT || t == ST_VID || t == ST_TIMESTAMP || t == ST_FLOAT || t == ST_DOUBLE;
  }
  static void statCollect(const PropCtx& p, const Value& v) {
    auto& q = const_cast<PropCtx&>(p);
    switch (v.index()) {
      case 0: q.isum += std::get<0>(v); break;
      case 1: q.dsum += std::get<1>(v); break;
      default: break;
    }
    q.count++;
  }

  explicit Processor(const Store& s) : st(s) {}

  std::vector<PropCtx>* edgeProps(int32_t et) {
    for (auto& e : edgeCtx) if (e.first == et) return &e.second;
    return nullptr;
  }

  // QueryBaseProcessor::checkExp (QueryBaseProcessor.inl:172-290)
  bool checkExp(const Expr* e) {
    switch (e->kind) {
      case kPrimary: return true;
      case kFunctionCall: return false;
      case kUnary: case kTypeCasting: return checkExp(e->a.get());
      case kArithmetic: case kRelational: case kLogical:
        return checkExp(e->a.get()) && checkExp(e->b.get());
      case kSourceProp: {
        auto it = st.tagByName.find(e->alias);
        if (it == st.tagByName.end()) return false;
        const Schema* s = st.tagSchema(it->second);
        if (!s || s->find(e->prop) < 0) return false;
        SType ft = s->typeOf(e->prop);
        for (auto& tc : tagCtx) {
          if (tc.tag == it->second) {
            if (std::find(tc.filterNames.begin(), tc.filterNames.end(), e->prop) == tc.filterNames.end()) {
              PropCtx pc; pc.prop = {1, it->second, e->prop}; pc.type = ft; pc.filtered = true; pc.tagName = e->alias;
              tc.props.push_back(pc); tc.filterNames.push_back(e->prop);
            }
            return true;
          }
        }
        TagCtx tc; tc.tag = it->second;
        PropCtx pc; pc.prop = {1, it->second, e->prop}; pc.type = ft; pc.filtered = true; pc.tagName = e->alias;
        tc.props.push_back(pc); tc.filterNames.push_back(e->prop);
        tagCtx.push_back(std::move(tc));
        return true;
      }
      case kEdgeRank: case kEdgeDstId: case kEdgeSrcId: case kEdgeType: return true;
      case kAliasProp: {
        if (edgeCtx.empty()) return false;
        auto it = st.edgeByName.find(e->alias);
        if (it == st.edgeByName.end()) return false;
        if (it->second < 0) return false;
        const Schema* s = st.edgeSchema(it->second);
        if (!s || s->find(e->prop) < 0) return false;
        return true;
      }
      default: return false;
    }
  }

  // QueryBaseProcessor::checkAndBuildContexts (QueryBaseProcessor.inl:60-169)
  int32_t build(const GNRequest& req) {
    for (auto et : req.edgeTypes)
      if (!edgeProps(et)) edgeCtx.emplace_back(et, std::vector<PropCtx>{});
    for (const auto& col : req.returns) {
      PropCtx pc;
      if (col.owner == 1 || col.owner == 2) {
        const Schema* s = st.tagSchema(col.id);
        if (!s) return E_TAG_PROP_NOT_FOUND;
        SType ft = s->typeOf(col.name);
        if (ft == ST_UNKNOWN) return E_IMPROPER_DATA_TYPE;
        if (!validOp(ft, col.stat)) return E_IMPROPER_DATA_TYPE;
        pc.type = ft; pc.prop = col; pc.returned = true; pc.retIndex = retIndex++;
        bool found = false;
        for (auto& tc : tagCtx) if (tc.tag == col.id) { tc.props.push_back(pc); found = true; break; }
        if (!found) { TagCtx tc; tc.tag = col.id; tc.props.push_back(pc); tagCtx.push_back(std::move(tc)); }
      } else {
        int32_t et = col.id;
        if (col.name == "_src" || col.name == "_dst" || col.name == "_type" || col.name == "_rank") {
          pc.pik = col.name == "_src" ? 1 : col.name == "_dst" ? 2 : col.name == "_type" ? 3 : 4;
          pc.type = (pc.pik == 1 || pc.pik == 2) ? ST_VID : ST_INT;
        } else if (et > 0) {
          const Schema* s = st.edgeSchema(et);
          if (!s) return E_EDGE_PROP_NOT_FOUND;
          SType ft = s->typeOf(col.name);
          if (ft == ST_UNKNOWN) return E_IMPROPER_DATA_TYPE;
          pc.type = ft;
        } else {
          continue;   // "InBound has none props, skip it!"
        }
        if (!validOp(pc.type, col.stat)) return E_IMPROPER_DATA_TYPE;
        pc.prop = col; pc.returned = true; pc.retIndex = retIndex++;
        auto* v = edgeProps(et);
        if (!v) { edgeCtx.emplace_back(et, std::vector<PropCtx>{pc}); }
        else v->push_back(pc);
      }
    }
    if (!req.filter.empty()) {
      std::string err;
      exp = decodeExpr(reinterpret_cast<const uint8_t*>(req.filter.data()), req.filter.size(), &err);
      if (!exp) return E_INVALID_FILTER;
      if (!checkExp(exp.get())) return E_INVALID_FILTER;
    }
    return E_SUCCEEDED;
  }

  // QueryBaseProcessor::collectProps (QueryBaseProcessor.inl:293-351) with PropsCollector
  void collectProps(RowReader* reader, const char* key, const std::vector<PropCtx>& props,
                    TagFilters* tf, RowWriter& w) {
    for (const auto& p : props) {
      if (stats) {   // StatsCollector: collectVid does nothing; _type/_rank collectInt64
        switch (p.pik) {
          case 1: case 2: continue;
          case 3: statCollect(p, Value((int64_t)keyType(key))); continue;
          case 4: statCollect(p, Value(keyRank(key))); continue;
          default: break;
        }
      }
      switch (p.pik) {
        case 1: w.putVid(keySrc(key)); continue;
        case 2: w.putVid(keyDst(key)); continue;
        case 3: w.putInt(keyType(key)); continue;
        case 4: w.putInt(keyRank(key)); continue;
        default: break;
      }
      if (!reader) continue;
      auto v = reader->get(p.prop.name);
      if (!v.ok()) continue;   // "Skip the bad value"
      if (p.filtered && tf) (*tf)[{p.tagName, p.prop.name}] = v.v;
      if (p.returned && stats) { statCollect(p, v.v); continue; }
      if (p.returned) {
        switch (v.v.index()) {
          case 0: w.putInt(std::get<0>(v.v)); break;
          case 1: w.putDouble(std::get<1>(v.v)); break;
          case 2: w.putBool(std::get<2>(v.v)); break;
          default: w.putString(std::get<3>(v.v)); break;
        }
      }
    }
  }

  struct FilterGetters : Getters {
    const Store& st; int32_t edgeType; RowReader* reader; int64_t rank; TagFilters* tf;
    FilterGetters(const Store& s, int32_t et, RowReader* r, int64_t rk, TagFilters* t)
        : st(s), edgeType(et), reader(r), rank(rk), tf(t) {}
    // QueryBaseProcessor.inl:580-606
    OptValue aliasProp(const std::string& edge, const std::string& prop) override {
      auto it = st.edgeByName.find(edge);
      if (it == st.edgeByName.end() || it->second != edgeType) return Status::Err("ignore this edge");
      auto v = reader->get(prop);
      if (!v.ok()) return Status::Err("Invalid Prop");
      return v;
    }
    OptValue srcTagProp(const std::string& tag, const std::string& prop) override {
      auto it = tf->find({tag, prop});
      if (it == tf->end()) return Status::Err("Invalid Tag Filter");
      return it->second;
    }
    OptValue dstTagProp(const std::string&, const std::string&) override {
      return Status::Err("Unsupport get dst tag");
    }
    OptValue edgeRank() override { return Value(rank); }
  };

  // QueryBaseProcessor::collectEdgeProps (QueryBaseProcessor.inl:381-458)
  int32_t collectEdgeProps(int32_t part, int64_t vid, int32_t et, const std::vector<PropCtx>& props,
                           TagFilters* tf, std::string& rowset) {
    auto prefix = edgePrefix(part, vid, et);
    auto rng = st.prefixRange(part, prefix);
    if (rng.first == rng.second) return E_SUCCEEDED;
    const auto& kvs = st.parts.at(part);
    int64_t lastRank = -1, lastDst = 0;
    bool firstLoop = true;
    int cnt = 0;
    for (size_t i = rng.first; i < rng.second && cnt < st.maxEdgePerVertex; ++i) {
      std::string_view key = kvs.key(i);
      std::string_view val = kvs.val(i);
      int64_t rank = keyRank(key.data()), dst = keyDst(key.data());
      if (!firstLoop && rank == lastRank && lastDst == dst) continue;   // older version
      lastRank = rank; lastDst = dst;
      std::unique_ptr<RowReader> reader;
      if (et > 0 && !val.empty()) {
        reader = std::make_unique<RowReader>(val, st.edgeSchema(et, rowSchemaVer(val)));
        if (exp) {
          std::lock_guard<std::mutex> lg(lock);
          FilterGetters g(st, et, reader.get(), rank, tf);
          auto v = exp->eval(g);
          if (v.ok() && !asBool(v.v)) continue;   // errors keep the edge
        }
      }
      RowWriter w(nullptr);
      collectProps(reader.get(), key.data(), props, tf, w);
      rowSetAdd(rowset, w.encode());
      ++cnt;
      if (firstLoop) firstLoop = false;
    }
    return E_SUCCEEDED;
  }

  // QueryBaseProcessor::collectVertexProps (QueryBaseProcessor.inl:354-378)
  int32_t collectVertexProps(int32_t part, int64_t vid, int32_t tag, const std::vector<PropCtx>& props,
                             TagFilters* tf, RowWriter& w) {
    auto rng = st.prefixRange(part, vertexPrefix(part, vid, tag));
    if (rng.first == rng.second) return E_KEY_NOT_FOUND;
    const PartKV& kvs = st.parts.at(part);
    RowReader r(kvs.val(rng.first), st.tagSchema(tag, rowSchemaVer(kvs.val(rng.first))));
    collectProps(&r, kvs.key(rng.first).data(), props, tf, w);
    return E_SUCCEEDED;
  }

  // QueryBoundProcessor::processVertex (QueryBoundProcessor.cpp:64-111)
  int32_t processVertex(int32_t part, int64_t vid, bool onlyVertexProps, std::vector<VertexData>& out) {
    // every part 1..numParts of the space exists (possibly empty) on its host
    if (part < 1 || part > st.numParts) return E_PART_NOT_FOUND;
    VertexData vd; vd.vid = vid;
    TagFilters tf;
    for (auto& tc : tagCtx) {
      RowWriter w(nullptr);
      int32_t rc = collectVertexProps(part, vid, tc.tag, tc.props, &tf, w);
      if (rc == E_KEY_NOT_FOUND) continue;
      if (rc != E_SUCCEEDED) return rc;
      if (w.colNum > 0) vd.tags.push_back({tc.tag, w.encode()});   // writer.size() > 1
    }
    if (!onlyVertexProps) {
      for (auto& ec : edgeCtx) {
        if (ec.second.empty()) continue;
        std::string rs;
        int32_t rc = collectEdgeProps(part, vid, ec.first, ec.second, &tf, rs);
        if (rc != E_SUCCEEDED) return rc;
        if (!rs.empty()) vd.edges.push_back({ec.first, std::move(rs)});
      }
      if (vd.edges.empty()) return E_SUCCEEDED;   // only return the vertex if edges existed
    }
    std::lock_guard<std::mutex> lg(lock);
    out.push_back(std::move(vd));
    return E_SUCCEEDED;
  }

  // QueryBoundProcessor::onProcessFinished (QueryBoundProcessor.cpp:113-161)
  void finish(QueryResponse& resp) {
    for (auto& tc : tagCtx) {
      Schema s;
      for (auto& p : tc.props) if (p.returned) s.cols.push_back({p.prop.name, p.type});
      if (!s.cols.empty() && !resp.vertexSchema.count(tc.tag)) resp.vertexSchema.emplace(tc.tag, s);
    }
    resp.hasVertexSchema = !resp.vertexSchema.empty();
    for (auto& ec : edgeCtx) {
      Schema s;
      for (auto& p : ec.second) s.cols.push_back({p.prop.name, p.type});
      if (!s.cols.empty() && !resp.edgeSchema.count(ec.first)) resp.edgeSchema.emplace(ec.first, s);
    }
    resp.hasEdgeSchema = !resp.edgeSchema.empty();
  }
};

// QueryBaseProcessor::getBucketsNum/genBuckets (QueryBaseProcessor.inl:479-513)
std::vector<std::vector<std::pair<int32_t, int64_t>>> genBuckets(const Store& st, const GNRequest& req,
                                                                 const std::vector<int32_t>& partOrder) {
  int32_t n = 0;
  for (auto& p : req.parts) n += (int32_t)p.second.size();
  int32_t nb = std::min(std::max(1, n / st.minVerticesPerBucket), st.maxHandlersPerReq);
  std::vector<std::vector<std::pair<int32_t, int64_t>>> buckets(nb);
  int32_t per = n / nb, left = n % nb, bi = -1;
  size_t thr = per;
  for (auto part : partOrder) {
    for (auto vid : req.parts.at(part)) {
      if (bi < 0 || buckets[bi].size() >= thr) { ++bi; thr = bi < left ? per + 1 : per; }
      buckets[bi].emplace_back(part, vid);
    }
  }
  return buckets;
}

QueryResponse process(const Store& st, const GNRequest& req, bool onlyVertexProps) {
  QueryResponse resp;
  Processor proc(st);
  std::vector<int32_t> partOrder;
  for (auto& p : req.parts) partOrder.push_back(p.first);
  std::sort(partOrder.begin(), partOrder.end());
  int32_t rc = proc.build(req);
  if (rc != E_SUCCEEDED) {   // request-level error: one code per requested part (inl:529-535)
    for (auto p : partOrder) resp.failed.emplace_back(rc, p);
    return resp;
  }
  auto buckets = genBuckets(st, req, partOrder);
  std::vector<std::vector<std::pair<int32_t, int32_t>>> codes(buckets.size());
  auto work = [&](size_t b) {
    for (auto& pv : buckets[b]) {
      int32_t r = proc.processVertex(pv.first, pv.second, onlyVertexProps, resp.vertices);
      if (r != E_SUCCEEDED) codes[b].emplace_back(r, pv.first);
    }
  };
  if (st.threads > 1 && buckets.size() > 1) {
    std::vector<std::future<void>> fs;
    for (size_t b = 0; b < buckets.size(); ++b) fs.push_back(std::async(std::launch::async, work, b));
    for (auto& f : fs) f.get();
  } else {
    for (size_t b = 0; b < buckets.size(); ++b) work(b);
  }
  std::unordered_set<int32_t> failedParts;
  for (auto& cs : codes)
    for (auto& c : cs)
      if (!failedParts.count(c.second)) { failedParts.insert(c.second); resp.failed.push_back(c); }
  proc.finish(resp);
  return resp;
}

}  // namespace

QueryResponse getBound(const Store& st, const GNRequest& req) { return process(st, req, false); }

QueryResponse getVertexProps(const Store& st, const GNRequest& req) { return process(st, req, true); }

// QueryStatsProcessor::processVertex / onProcessFinished / calcResult
// (src/storage/QueryStatsProcessor.cpp:16-130): tag props of every requested vertex, edge props
// of every accepted edge, one row in retIndex order.
StatsResult boundStats(const Store& st, const GNRequest& req) {
  StatsResult res;
  Processor proc(st);
  proc.stats = true;
  std::vector<int32_t> partOrder;
  for (auto& p : req.parts) partOrder.push_back(p.first);
  std::sort(partOrder.begin(), partOrder.end());
  int32_t rc = proc.build(req);
  if (rc != E_SUCCEEDED) {
    for (auto p : partOrder) res.failed.emplace_back(rc, p);
    return res;
  }
  std::unordered_set<int32_t> failedParts;
  for (auto part : partOrder) {
    for (auto vid : req.parts.at(part)) {
      if (part < 1 || part > st.numParts) {
        if (failedParts.insert(part).second) res.failed.emplace_back(E_PART_NOT_FOUND, part);
        continue;
      }
      TagFilters tf;
      bool missing = false;   // QueryStatsProcessor::processVertex returns the tag's failure
      for (auto& tc : proc.tagCtx) {
        RowWriter w(nullptr);
        if (proc.collectVertexProps(part, vid, tc.tag, tc.props, &tf, w) != E_SUCCEEDED) { missing = true; break; }
      }
      if (missing) {   // ERR_KEY_NOT_FOUND -> E_UNKNOWN (BaseProcessor.inl:14-29), first per part
        if (failedParts.insert(part).second) res.failed.emplace_back(E_UNKNOWN, part);
        continue;
      }
      for (auto& ec : proc.edgeCtx) {
        if (ec.second.empty()) continue;
        std::string rs;
        proc.collectEdgeProps(part, vid, ec.first, ec.second, &tf, rs);
      }
    }
  }
  std::vector<const PropCtx*> props;
  for (auto& tc : proc.tagCtx)
    for (auto& p : tc.props) if (p.returned) props.push_back(&p);
  for (auto& ec : proc.edgeCtx)
    for (auto& p : ec.second) props.push_back(&p);
  std::sort(props.begin(), props.end(), [](const PropCtx* a, const PropCtx* b) { return a->retIndex < b->retIndex; });
  RowWriter w(nullptr);
  for (auto* p : props) {
    const bool dbl = p->type == ST_DOUBLE || p->type == ST_FLOAT;
    switch (p->prop.stat) {
      case 1:
        if (dbl) { w.putDouble(p->dsum); res.schema.cols.push_back({p->prop.name, ST_DOUBLE}); res.values.push_back(p->dsum); }
        else { w.putInt(p->isum); res.schema.cols.push_back({p->prop.name, ST_INT}); res.values.push_back(p->isum); }
        break;
      case 2:
        w.putInt(p->count); res.schema.cols.push_back({p->prop.name, ST_INT}); res.values.push_back((int64_t)p->count);
        break;
      case 3: {
        const double v = dbl ? p->dsum / p->count : static_cast<double>(p->isum) / p->count;
        w.putDouble(v); res.schema.cols.push_back({p->prop.name, ST_DOUBLE}); res.values.push_back(v);
        break;
      }
      default: break;
    }
  }
  res.data = w.encode();
  return res;
}

QueryResponse getNeighbors(const Store& st, const std::vector<int64_t>& vids,
                           const std::vector<int32_t>& etypes, const std::string& filter,
                           const std::vector<PropDef>& returns) {
  // clusterIdsToHosts: one request per storaged host holding all of that host's parts
  // (StorageClient.h:240-260); part p lives on host p % hosts (CreateSpaceProcessor.cpp:84-95).
  const int32_t H = std::max(1, st.hosts);
  std::vector<GNRequest> reqs(H);
  for (auto v : vids) {
    int32_t p = partOf(v, st.numParts);
    reqs[p % H].parts[p].push_back(v);
  }
  for (auto& r : reqs) { r.edgeTypes = etypes; r.filter = filter; r.returns = returns; }
  if (H == 1) return getBound(st, reqs[0]);
  // collectResponse (StorageClient.inl:73-160): fan out, gather
  std::vector<std::future<QueryResponse>> fs;
  for (auto& r : reqs) {
    if (r.parts.empty()) continue;
    fs.push_back(std::async(std::launch::async, [&st, &r]() { return getBound(st, r); }));
  }
  QueryResponse all;
  for (auto& f : fs) {
    QueryResponse q = f.get();
    all.failed.insert(all.failed.end(), q.failed.begin(), q.failed.end());
    for (auto& kv : q.vertexSchema) all.vertexSchema.emplace(kv.first, kv.second);
    for (auto& kv : q.edgeSchema) all.edgeSchema.emplace(kv.first, kv.second);
    for (auto& v : q.vertices) all.vertices.push_back(std::move(v));
  }
  all.hasVertexSchema = !all.vertexSchema.empty();
  all.hasEdgeSchema = !all.edgeSchema.empty();
  return all;
}

}  // namespace orc
