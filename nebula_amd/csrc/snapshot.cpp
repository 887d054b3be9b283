// Snapshot files: the finalized device snapshot written to disk and read back, so a storaged
// restart (or a second process serving the same parts) skips KV ingestion, version de-dup and
// the CSR build (SURVEY.md §8(f)4 "a CSR snapshot file for restart").
//
// The file holds what nbg_finalize derives from the kvstore records: schemas, the string
// dictionary, the vertex dictionary with home parts and visibility, per signed edge type the CSR
// offsets, neighbour ids, dst vids, ranks, property columns and decode flags, and the per-vertex
// tag columns.  Neighbour ids of a partitioned engine are global ids (owner * npad + local id),
// so the file is per rank and the loading engine must have the same parts / GPUs / rank and its
// communicator attached (tag columns are gathered again).  Narrow INT copies are re-derived.
// Format 2 also holds each type's superseded-version CSR (multi-version data: GetNeighbors' filtered
// walk reads the older versions until an edge is accepted, QueryBaseProcessor.inl:394-456), so a
// restored engine answers exactly as the KV-loaded one; format 1 files (no such CSR) still load.
#include <cstdio>
#include <cstring>

#include "engine.h"

using namespace nbg;

namespace {

constexpr char kMagic[8] = {'N', 'B', 'G', 'S', 'N', 'A', 'P', '2'};
constexpr char kMagic1[8] = {'N', 'B', 'G', 'S', 'N', 'A', 'P', '1'};   // format 1: no superseded versions

struct Out {
  FILE* f;
  bool ok = true;
  void raw(const void* p, size_t n) {
    if (ok && n && fwrite(p, 1, n, f) != n) ok = false;
  }
  template <class T>
  void put(T v) { raw(&v, sizeof v); }
  void str(const std::string& s) {
    put<uint32_t>((uint32_t)s.size());
    raw(s.data(), s.size());
  }
  template <class T>
  void vec(const std::vector<T>& v) {
    put<uint64_t>(v.size());
    raw(v.data(), v.size() * sizeof(T));
  }
};

struct In {
  FILE* f;
  bool ok = true;
  void raw(void* p, size_t n) {
    if (ok && n && fread(p, 1, n, f) != n) ok = false;
  }
  template <class T>
  T get() {
    T v{};
    raw(&v, sizeof v);
    return v;
  }
  std::string str() {
    const uint32_t n = get<uint32_t>();
    if (!ok || n > (1u << 30)) { ok = false; return {}; }
    std::string s(n, '\0');
    raw(&s[0], n);
    return s;
  }
  template <class T>
  std::vector<T> vec() {
    const uint64_t n = get<uint64_t>();
    if (!ok || n > (1ull << 40) / sizeof(T)) { ok = false; return {}; }
    std::vector<T> v(n);
    raw(v.data(), n * sizeof(T));
    return v;
  }
};

void put_schemas(Out& o, const std::map<int32_t, SchemaSet>& m) {
  o.put<uint32_t>((uint32_t)m.size());
  for (auto& kv : m) {
    o.put<int32_t>(kv.first);
    o.str(kv.second.name);
    o.put<uint32_t>((uint32_t)kv.second.versions.size());
    for (auto& v : kv.second.versions) {
      o.put<int64_t>(v.first);
      o.put<uint32_t>((uint32_t)v.second.cols.size());
      for (auto& c : v.second.cols) {
        o.str(c.name);
        o.put<int32_t>(c.type);
      }
    }
  }
}

bool get_schemas(In& in, std::map<int32_t, SchemaSet>& m) {
  m.clear();
  const uint32_t n = in.get<uint32_t>();
  for (uint32_t i = 0; in.ok && i < n; ++i) {
    const int32_t id = in.get<int32_t>();
    SchemaSet& ss = m[id];
    ss.name = in.str();
    const uint32_t nv = in.get<uint32_t>();
    for (uint32_t k = 0; in.ok && k < nv; ++k) {
      Schema s;
      s.version = in.get<int64_t>();
      const uint32_t nc = in.get<uint32_t>();
      for (uint32_t c = 0; in.ok && c < nc; ++c) {
        Column col;
        col.name = in.str();
        col.type = in.get<int32_t>();
        s.cols.push_back(col);
      }
      ss.versions[s.version] = s;
    }
  }
  return in.ok;
}

template <class T>
bool download(std::vector<T>& out, const T* dev, uint64_t n) {
  out.resize(n);
  return !n || hipMemcpy(out.data(), dev, n * sizeof(T), hipMemcpyDeviceToHost) == hipSuccess;
}

}  // namespace

namespace nbg {

int32_t Engine::save_snapshot(const char* path) {
  if (!finalized) return fail(NBG_E_STATE, "engine not finalized");
  FILE* f = fopen(path, "wb");
  if (!f) return fail(NBG_E_INVALID_ARGUMENT, std::string("cannot open ") + path);
  Out o{f};
  o.raw(kMagic, sizeof kMagic);
  o.put<int32_t>(cfg.num_parts);
  o.put<int32_t>(cfg.num_gpus);
  o.put<int32_t>(cfg.rank);
  o.put<uint64_t>(npad);
  put_schemas(o, edges);
  put_schemas(o, tags);
  o.put<uint64_t>(snap.strings.size());
  for (auto& s : snap.strings) o.str(s);
  o.vec(snap.h_vids);
  o.vec(snap.h_part);
  o.vec(snap.h_visible);
  o.put<uint32_t>((uint32_t)snap.types.size());
  bool dl = true;
  auto put_csr = [&](const DevEdgeType& dt) {
    const uint64_t E = dt.num_edges;
    o.put<uint64_t>(E);
    o.vec(dt.h_row_ptr);
    std::vector<uint32_t> col;
    std::vector<int64_t> v64;
    dl = dl && download(col, dt.col, E);
    o.vec(col);
    dl = dl && download(v64, dt.dst_vid, E);
    o.vec(v64);
    o.put<uint8_t>(dt.rank != nullptr);
    if (dt.rank) {
      dl = dl && download(v64, dt.rank, E);
      o.vec(v64);
    }
    o.put<uint32_t>((uint32_t)dt.props.size());
    for (size_t c = 0; c < dt.props.size(); ++c) {
      o.put<uint8_t>((uint8_t)dt.prop_kind[c]);
      dl = dl && download(v64, dt.props[c], E);
      o.vec(v64);
    }
    o.put<uint8_t>(dt.valid != nullptr);
    if (dt.valid) {
      std::vector<uint8_t> v8;
      dl = dl && download(v8, dt.valid, E);
      o.vec(v8);
    }
  };
  for (auto& kv : snap.types) {
    o.put<int32_t>(kv.first);
    put_csr(kv.second);
    o.put<uint8_t>(kv.second.old != nullptr);
    if (kv.second.old) {
      put_csr(*kv.second.old);
      o.vec(kv.second.old->h_grp);
    }
  }
  o.put<uint32_t>((uint32_t)snap.tags.size());
  for (auto& kv : snap.tags) {
    const DevTag& t = kv.second;
    o.put<int32_t>(t.tag);
    o.put<int32_t>(t.index);
    o.put<int32_t>(t.col_base);
    std::vector<uint8_t> kinds(t.kind.begin(), t.kind.end());
    o.vec(kinds);
    o.vec(t.h_present);
    for (auto& c : t.h_cols) o.vec(c);
  }
  o.raw(kMagic, sizeof kMagic);   // trailer: a truncated file is rejected
  const bool ok = o.ok && fclose(f) == 0;
  if (!dl) return fail(NBG_E_DEVICE, "snapshot download failed");
  return ok ? NBG_OK : fail(NBG_E_UNKNOWN, std::string("write failed: ") + path);
}

int32_t Engine::load_snapshot(const char* path) {
  if (finalized) return fail(NBG_E_STATE, "engine already finalized");
  if (partitioned() && !comm) return fail(NBG_E_STATE, "a partitioned engine needs nbg_comm_init before loading");
  FILE* f = fopen(path, "rb");
  if (!f) return fail(NBG_E_INVALID_ARGUMENT, std::string("cannot open ") + path);
  In in{f};
  auto bad = [&](const std::string& why) {
    fclose(f);
    free_snapshot();   // no partial device state survives a rejected file
    return fail(NBG_E_INVALID_ARGUMENT, "snapshot " + std::string(path) + ": " + why);
  };
  char magic[8];
  in.raw(magic, sizeof magic);
  const bool v1 = in.ok && !memcmp(magic, kMagic1, sizeof kMagic1);
  if (!in.ok || (!v1 && memcmp(magic, kMagic, sizeof kMagic))) return bad("not a snapshot file");
  const int32_t parts = in.get<int32_t>(), gpus = in.get<int32_t>(), rank = in.get<int32_t>();
  if (parts != cfg.num_parts || gpus != cfg.num_gpus || rank != cfg.rank)
    return bad("written for another partitioning (parts / GPUs / rank)");
  npad = in.get<uint64_t>();
  if (!get_schemas(in, edges) || !get_schemas(in, tags)) return bad("schemas");
  const uint64_t ns = in.get<uint64_t>();
  snap.strings.clear();
  for (uint64_t i = 0; in.ok && i < ns; ++i) snap.strings.push_back(in.str());
  snap.h_vids = in.vec<int64_t>();
  snap.h_part = in.vec<int32_t>();
  snap.h_visible = in.vec<uint8_t>();
  snap.nv = snap.h_vids.size();
  const uint64_t nv = snap.nv;
  if (!in.ok || snap.h_part.size() != nv || (!snap.h_visible.empty() && snap.h_visible.size() != nv))
    return bad("vertex tables");
  // dense() binary-searches the dictionary: strictly ascending vids
  for (uint64_t d = 1; d < nv; ++d)
    if (snap.h_vids[d - 1] >= snap.h_vids[d]) return bad("vertex dictionary not sorted");
  if (nv >= NO_ROW || (partitioned() && ((npad % PART_ALIGN) || nv > npad || (uint64_t)cfg.num_gpus * npad >= NO_ROW)))
    return bad("vertex id space");
  // neighbour ids index [nv) on one GPU, the global id space [G * npad) when partitioned
  const uint64_t id_space = partitioned() ? (uint64_t)cfg.num_gpus * npad : nv;
  // one CSR (a type's, or its superseded versions') read, validated and uploaded into dt
  auto get_csr = [&](DevEdgeType& dt, int32_t type, const char* what) -> int32_t {
    dt.type = type;
    dt.num_edges = in.get<uint64_t>();
    const uint64_t E = dt.num_edges;
    const std::string name = std::string(what) + " " + std::to_string(type);
    dt.h_row_ptr = in.vec<uint32_t>();
    std::vector<uint32_t> col = in.vec<uint32_t>();
    std::vector<int64_t> dvid = in.vec<int64_t>(), rk;
    const bool has_rank = in.get<uint8_t>() != 0;
    if (has_rank) rk = in.vec<int64_t>();
    const uint32_t nc = in.get<uint32_t>();
    std::vector<VKind> kinds;
    std::vector<std::vector<int64_t>> pc;
    for (uint32_t c = 0; in.ok && c < nc; ++c) {
      kinds.push_back((VKind)in.get<uint8_t>());
      pc.push_back(in.vec<int64_t>());
    }
    std::vector<uint8_t> valid;
    const bool has_valid = in.get<uint8_t>() != 0;
    if (has_valid) valid = in.vec<uint8_t>();
    bool sizes = dt.h_row_ptr.size() == nv + 1 && col.size() == E && dvid.size() == E && (!has_rank || rk.size() == E) &&
                 (!has_valid || valid.size() == E) && dt.h_row_ptr[nv] == E;
    for (auto& c : pc) sizes = sizes && c.size() == E;
    if (!in.ok || !sizes) return bad(name);
    if (dt.h_row_ptr[0] != 0) return bad(name + ": row offsets");
    for (uint64_t d = 0; d < nv; ++d)
      if (dt.h_row_ptr[d] > dt.h_row_ptr[d + 1]) return bad(name + ": row offsets");
    for (uint32_t c : col)
      if (c != NO_ROW && c >= id_space) return bad(name + ": neighbour id");
    for (VKind k : kinds)
      if (k > VK_STRING) return bad(name + ": column kind");
    if (!upload_type(dt, nv, col, dvid, has_rank ? &rk : nullptr, pc, has_valid ? &valid : nullptr, kinds)) {
      fclose(f);
      free_snapshot();
      return fail(NBG_E_OUT_OF_MEMORY, "device allocation failed for the snapshot");
    }
    return NBG_OK;
  };
  const uint32_t nt = in.get<uint32_t>();
  for (uint32_t k = 0; in.ok && k < nt; ++k) {
    const int32_t type = in.get<int32_t>();
    DevEdgeType& dt = snap.types[type];
    if (int32_t rc = get_csr(dt, type, "edge type")) return rc;
    if (!v1 && in.get<uint8_t>() != 0) {
      dt.old = new DevEdgeType();
      if (int32_t rc = get_csr(*dt.old, type, "superseded versions of edge type")) return rc;
      dt.old->h_grp = in.vec<uint32_t>();
      bool ok = in.ok && dt.old->h_grp.size() == dt.old->num_edges;
      for (uint32_t g : dt.old->h_grp) ok = ok && g < dt.num_edges;
      if (!ok) return bad("superseded versions of edge type " + std::to_string(type) + ": live edge index");
    }
  }
  const uint32_t ntag = in.get<uint32_t>();
  for (uint32_t k = 0; in.ok && k < ntag; ++k) {
    const int32_t tag = in.get<int32_t>();
    DevTag& t = snap.tags[tag];
    t.tag = tag;
    t.index = in.get<int32_t>();
    t.col_base = in.get<int32_t>();
    std::vector<uint8_t> kinds = in.vec<uint8_t>();
    t.kind.clear();
    for (uint8_t k : kinds) t.kind.push_back((VKind)k);
    t.h_present = in.vec<uint8_t>();
    t.h_cols.clear();
    for (size_t c = 0; in.ok && c < kinds.size(); ++c) t.h_cols.push_back(in.vec<int64_t>());
    if (!in.ok || t.h_present.size() != nv) return bad("tag " + std::to_string(tag));
    for (auto& c : t.h_cols)
      if (c.size() != nv) return bad("tag " + std::to_string(tag));
    for (uint8_t k : kinds)
      if (k > VK_STRING) return bad("tag " + std::to_string(tag) + ": column kind");
  }
  {   // tag slots index Snapshot::d_tpres / d_tcols: a permutation / disjoint column ranges
    std::vector<int> seen(snap.tags.size(), 0);
    int cols = 0;
    for (auto& kv : snap.tags) {
      const DevTag& t = kv.second;
      if (t.index < 0 || t.index >= (int)seen.size() || seen[t.index]++) return bad("tag table");
      cols += (int)t.kind.size();
    }
    std::vector<int> used(cols, 0);
    for (auto& kv : snap.tags) {
      const DevTag& t = kv.second;
      if (t.col_base < 0 || t.col_base + (int)t.kind.size() > cols) return bad("tag table");
      for (size_t c = 0; c < t.kind.size(); ++c)
        if (used[t.col_base + c]++) return bad("tag table");
    }
  }
  in.raw(magic, sizeof magic);
  if (!in.ok || memcmp(magic, v1 ? kMagic1 : kMagic, sizeof kMagic)) return bad("truncated");
  fclose(f);
  int32_t rc = upload_tags();
  if (!rc) rc = upload_vertices(snap.h_visible, snap.h_visible.empty());
  if (rc) {
    const std::string msg = last_error;
    free_snapshot();
    return fail(rc, msg);
  }
  finalized = true;
  return NBG_OK;
}

}  // namespace nbg

extern "C" {

int32_t nbg_snapshot_save(nbg_engine* h, const char* path) {
  if (!h || !path) return NBG_E_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lg(h->e.mu);
  if (hipSetDevice(h->e.cfg.device) != hipSuccess) return h->e.fail(NBG_E_DEVICE, "hipSetDevice failed");
  return h->e.save_snapshot(path);
}

int32_t nbg_snapshot_load(nbg_engine* h, const char* path) {
  if (!h || !path) return NBG_E_INVALID_ARGUMENT;
  Engine& E = h->e;
  std::lock_guard<std::mutex> lg(E.mu);
  if (hipSetDevice(E.cfg.device) != hipSuccess) return E.fail(NBG_E_DEVICE, "hipSetDevice failed");
  if (!E.stream && hipStreamCreateWithFlags(&E.stream, hipStreamNonBlocking) != hipSuccess)
    return E.fail(NBG_E_DEVICE, "hipStreamCreate failed");
  int32_t rc = E.load_snapshot(path);
  if (rc) return rc;
  return engine_ready(E);
}

}  // extern "C"
