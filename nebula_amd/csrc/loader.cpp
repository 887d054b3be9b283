// Loader: kvstore records (or bulk edge columns) -> device-resident CSR per signed edge type.
//
// What a storaged part holds (and what GetNeighbors reads back) is defined by
//   NebulaKeyUtils::edgeKey  (src/common/base/NebulaKeyUtils.cpp:28-47)
//   AddEdgesProcessor        (src/storage/AddEdgesProcessor.cpp:15-37)  version = BE(INT64_MAX-now)
//   RowWriter / RowReader    (src/dataman/RowWriter.cpp:49-75, RowReader.cpp:117-258)
//   collectEdgeProps         (src/storage/QueryBaseProcessor.inl:381-458)
// A prefix scan of (part, src, type) visits keys in memcmp order of (rank LE | dst LE |
// version BE) and keeps the first key of each (rank, dst) group.  The snapshot bakes exactly
// that view: rows sorted by (bswap64(rank), bswap64(dst)) as unsigned, one live edge per
// (src, type, rank, dst) — the one with the smallest version bytes (newest write); identical
// keys resolve to the record loaded last (write-batch overwrite).
#include <omp.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <numeric>
#include <parallel/algorithm>

#include "engine.h"

namespace nbg {

static inline uint64_t bswap64(uint64_t x) { return __builtin_bswap64(x); }

static int32_t hash_part(int64_t vid, int32_t parts) {
  return (int32_t)((uint64_t)vid % (uint64_t)parts + 1);
}

// ----------------------------------------------------------------------------- row decoding
// RowReader::processHeader + sequential field walk (RowReader.cpp:217-258, :307-375)
static bool decode_varint(const uint8_t* p, size_t avail, uint64_t& v, size_t& len) {
  v = 0;
  len = 0;
  for (int shift = 0; shift < 64 && len < avail; shift += 7) {
    uint8_t b = p[len++];
    v |= (uint64_t)(b & 0x7f) << shift;
    if (!(b & 0x80)) return true;
  }
  return false;
}

int64_t Engine::intern(const std::string& s) {
  auto it = pool_index.find(s);
  if (it != pool_index.end()) return it->second;
  int64_t id = (int64_t)pool.size();
  pool.push_back(s);
  pool_index.emplace(s, id);
  return id;
}

// Decodes a RowWriter value into the latest schema's column order.  Returns false if the row
// cannot be decoded (the reference would then fail reading the prop).
bool Engine::decode_row(const SchemaSet& ss, const uint8_t* v, size_t n, int64_t* out) {
  if (n == 0) return false;
  uint8_t h = v[0];
  size_t offBytes = (h & 0x07) + 1, verBytes = h >> 5;
  int64_t ver = 0;
  if (1 + verBytes > n) return false;
  for (size_t i = 0; i < verBytes; ++i) ver |= (int64_t)v[1 + i] << (8 * i);
  const Schema* sc = ss.at(ver);
  const Schema* latest = ss.latest();
  if (!sc || !latest) return false;
  size_t numOffsets = sc->cols.size() >> 4;
  size_t pos = 1 + verBytes + offBytes * numOffsets;
  if (pos > n) return false;
  std::vector<int64_t> vals(sc->cols.size());
  for (size_t c = 0; c < sc->cols.size(); ++c) {
    const uint8_t* p = v + pos;
    size_t avail = n - pos;
    switch (sc->cols[c].type) {
      case NBG_T_BOOL: if (avail < 1) return false; vals[c] = p[0] != 0; pos += 1; break;
      case NBG_T_INT: case NBG_T_TIMESTAMP: {
        uint64_t x; size_t l;
        if (!decode_varint(p, avail, x, l)) return false;
        vals[c] = (int64_t)x; pos += l; break;
      }
      case NBG_T_VID: if (avail < 8) return false; memcpy(&vals[c], p, 8); pos += 8; break;
      case NBG_T_FLOAT: {
        if (avail < 4) return false;
        float f; memcpy(&f, p, 4);
        double d = f; memcpy(&vals[c], &d, 8); pos += 4; break;
      }
      case NBG_T_DOUBLE: if (avail < 8) return false; memcpy(&vals[c], p, 8); pos += 8; break;
      case NBG_T_STRING: {
        uint64_t len; size_t l;
        if (!decode_varint(p, avail, len, l) || l + len > avail) return false;
        vals[c] = intern(std::string(reinterpret_cast<const char*>(p + l), len));
        pos += l + len; break;
      }
      default: return false;
    }
  }
  for (size_t c = 0; c < latest->cols.size(); ++c) {
    int k = sc == latest ? (int)c : sc->find(latest->cols[c].name);
    if (k < 0) return false;
    out[c] = vals[k];
  }
  return true;
}

// ----------------------------------------------------------------------------- ingest
int32_t Engine::load_part_kv(int32_t part, const uint8_t* kd, const uint64_t* ko, const uint8_t* vd,
                             const uint64_t* vo, uint64_t n) {
  if (finalized) return fail(NBG_E_STATE, "engine already finalized");
  if (cfg.num_gpus > 1 && part % cfg.num_gpus != cfg.rank) return NBG_OK;   // not served here
  std::vector<int64_t> props;
  for (uint64_t i = 0; i < n; ++i) {
    const uint8_t* k = kd + ko[i];
    uint64_t klen = ko[i + 1] - ko[i];
    const uint8_t* v = vd + vo[i];
    uint64_t vlen = vo[i + 1] - vo[i];
    if (klen < 4) continue;
    int32_t item;
    memcpy(&item, k, 4);
    if ((item & 0xFF) != 1) continue;   // NebulaKeyType::kData only
    if (klen == 40) {
      int32_t t;
      memcpy(&t, k + 12, 4);
      if (!(t & 0x40000000)) continue;
      int32_t type = t > 0 ? (t & (int32_t)0xBFFFFFFF) : t;
      int64_t src, rank, dst;
      uint64_t ver;
      memcpy(&src, k + 4, 8);
      memcpy(&rank, k + 16, 8);
      memcpy(&dst, k + 24, 8);
      memcpy(&ver, k + 32, 8);
      EdgeStage& st = stage[type];
      st.src.push_back(src);
      st.dst.push_back(dst);
      st.rank.push_back(rank);
      st.verkey.push_back(bswap64(ver));
      st.seq.push_back(seq++);
      st.part.push_back(item >> 8);
      if (type > 0) {
        auto es = edges.find(type);
        const Schema* latest = es == edges.end() ? nullptr : es->second.latest();
        size_t nc = latest ? latest->cols.size() : 0;
        if (st.props.size() < nc) st.props.resize(nc);
        props.assign(nc, 0);
        bool ok = latest && decode_row(es->second, v, vlen, props.data());
        for (size_t c = 0; c < nc; ++c) st.props[c].push_back(ok ? props[c] : 0);
        st.valid.push_back(ok ? 1 : 0);
      }
    } else if (klen == 24) {
      // vertex key (NebulaKeyUtils::vertexKey, NebulaKeyUtils.cpp:12-26): part | vid | tag | version
      int32_t tag;
      int64_t vid;
      uint64_t ver;
      memcpy(&vid, k + 4, 8);
      memcpy(&tag, k + 12, 4);
      memcpy(&ver, k + 16, 8);
      if (tag & 0x40000000) continue;
      TagStage& ts = tstage[tag];
      ts.vid.push_back(vid);
      ts.verkey.push_back(bswap64(ver));
      ts.seq.push_back(seq++);
      ts.part.push_back(item >> 8);
      auto sit = tags.find(tag);
      const Schema* latest = sit == tags.end() ? nullptr : sit->second.latest();
      size_t nc = latest ? latest->cols.size() : 0;
      if (ts.props.size() < nc) ts.props.resize(nc);
      props.assign(nc, 0);
      bool ok = latest && decode_row(sit->second, v, vlen, props.data());
      for (size_t c = 0; c < nc; ++c) ts.props[c].push_back(ok ? props[c] : 0);
      ts.valid.push_back(ok ? 1 : 0);
    }
  }
  return NBG_OK;
}

int32_t Engine::load_edges(int32_t type, const int64_t* src, const int64_t* dst, const int64_t* rank, uint64_t n,
                           const void* const* cols, int32_t ncols) {
  if (finalized) return fail(NBG_E_STATE, "engine already finalized");
  auto es = edges.find(type);
  if (type <= 0 || es == edges.end()) return fail(NBG_E_EDGE_PROP_NOT_FOUND, "edge type not registered");
  const Schema* latest = es->second.latest();
  if ((int32_t)latest->cols.size() != ncols) return fail(NBG_E_INVALID_ARGUMENT, "column count mismatch");
  for (auto& c : latest->cols)
    if (c.type == NBG_T_STRING) return fail(NBG_E_UNSUPPORTED, "bulk load of STRING columns");
  EdgeStage& out = stage[type];
  EdgeStage& in = stage[-type];
  if (out.props.size() < (size_t)ncols) out.props.resize(ncols);
  const uint64_t ver = bswap64((uint64_t)(INT64_MAX - 1));   // one version for the whole batch
  const int32_t P = cfg.num_parts, G = cfg.num_gpus;
  for (uint64_t i = 0; i < n; ++i) {
    int64_t r = rank ? rank[i] : 0;
    int32_t ps = hash_part(src[i], P), pd = hash_part(dst[i], P);
    if (G <= 1 || ps % G == cfg.rank) {
      out.src.push_back(src[i]);
      out.dst.push_back(dst[i]);
      out.rank.push_back(r);
      out.verkey.push_back(ver);
      out.seq.push_back(seq + i);
      out.part.push_back(ps);
      for (int32_t c = 0; c < ncols; ++c) {
        int64_t b = 0;
        switch (latest->cols[c].type) {
          case NBG_T_BOOL: b = static_cast<const uint8_t*>(cols[c])[i] != 0; break;
          case NBG_T_FLOAT: case NBG_T_DOUBLE: memcpy(&b, static_cast<const double*>(cols[c]) + i, 8); break;
          default: b = static_cast<const int64_t*>(cols[c])[i]; break;
        }
        out.props[c].push_back(b);
      }
      out.valid.push_back(1);
    }
    if (G <= 1 || pd % G == cfg.rank) {
      in.src.push_back(dst[i]);
      in.dst.push_back(src[i]);
      in.rank.push_back(r);
      in.verkey.push_back(ver);
      in.seq.push_back(seq + i);
      in.part.push_back(pd);
    }
  }
  seq += n;
  return NBG_OK;
}

// ----------------------------------------------------------------------------- finalize
namespace {
struct RowKey {   // memcmp order of (rank | dst | version) then newest load first
  uint64_t rank_be, dst_be, ver;
  uint64_t seq;
  uint64_t idx;
};
inline bool rowkey_less(const RowKey& a, const RowKey& b) {
  if (a.rank_be != b.rank_be) return a.rank_be < b.rank_be;
  if (a.dst_be != b.dst_be) return a.dst_be < b.dst_be;
  if (a.ver != b.ver) return a.ver < b.ver;
  return a.seq > b.seq;
}
}  // namespace

// Every rank learns every rank's sorted vertex dictionary (allgather over the communicator):
// npad = the largest dictionary rounded up to PART_ALIGN.
int32_t Engine::exchange_dictionary(const std::vector<int64_t>& local, std::vector<int64_t>* gdict,
                                    std::vector<uint64_t>* gcount) {
  if (!comm) return fail(NBG_E_STATE, "a partitioned engine (num_gpus > 1) needs nbg_comm_init before nbg_finalize");
  const uint64_t G = (uint64_t)cfg.num_gpus;
  uint64_t* d_cnt = nullptr;
  int64_t *d_loc = nullptr, *d_glob = nullptr;
  auto done = [&](int32_t rc, const std::string& msg) {
    for (void* p : {(void*)d_cnt, (void*)d_loc, (void*)d_glob})
      if (p) (void)hipFree(p);
    return rc ? fail(rc, msg) : NBG_OK;
  };
  const uint64_t nv = local.size();
  if (hipMalloc((void**)&d_cnt, (G + 1) * 8) != hipSuccess ||
      hipMemcpy(d_cnt + G, &nv, 8, hipMemcpyHostToDevice) != hipSuccess)
    return done(NBG_E_OUT_OF_MEMORY, "dictionary exchange: device allocation");
  if (comm->allgather(d_cnt + G, d_cnt, 8, stream) || hipStreamSynchronize(stream) != hipSuccess)
    return done(NBG_E_DEVICE, "dictionary exchange (counts): " + comm->last);
  gcount->assign(G, 0);
  if (hipMemcpy(gcount->data(), d_cnt, G * 8, hipMemcpyDeviceToHost) != hipSuccess)
    return done(NBG_E_DEVICE, "dictionary exchange: copy");
  uint64_t mx = 1;
  for (uint64_t c : *gcount) mx = std::max(mx, c);
  npad = (mx + PART_ALIGN - 1) / PART_ALIGN * PART_ALIGN;
  if (G * npad >= (uint64_t)NO_ROW) return done(NBG_E_UNSUPPORTED, "global id space exceeds 2^32-1 vertices");
  if (hipMalloc((void**)&d_loc, npad * 8) != hipSuccess || hipMalloc((void**)&d_glob, G * npad * 8) != hipSuccess)
    return done(NBG_E_OUT_OF_MEMORY, "dictionary exchange: device allocation");
  if (nv && hipMemcpy(d_loc, local.data(), nv * 8, hipMemcpyHostToDevice) != hipSuccess)
    return done(NBG_E_DEVICE, "dictionary exchange: upload");
  if (comm->allgather(d_loc, d_glob, npad * 8, stream) || hipStreamSynchronize(stream) != hipSuccess)
    return done(NBG_E_DEVICE, "dictionary exchange (vids): " + comm->last);
  gdict->resize(G * npad);
  if (hipMemcpy(gdict->data(), d_glob, G * npad * 8, hipMemcpyDeviceToHost) != hipSuccess)
    return done(NBG_E_DEVICE, "dictionary exchange: download");
  return done(NBG_OK, "");
}

// Tag records -> per-vertex columns (the live record of each (vid, tag) is the newest version,
// i.e. the first key of the vertex prefix, QueryBaseProcessor::collectVertexProps,
// QueryBaseProcessor.inl:354-378).  Partitioned engines gather every rank's columns into the
// global id space, so a `$$` read of a remote destination stays a local load.
int32_t Engine::build_tags(const std::vector<int64_t>& dict, const std::vector<int64_t>& remap) {
  const uint64_t nv = dict.size();
  int index = 0, col_base = 0;
  for (auto& kv : tags) {
    const int32_t tag = kv.first;
    const Schema* latest = kv.second.latest();
    const size_t nc = latest ? latest->cols.size() : 0;
    DevTag& dt = snap.tags[tag];
    dt.tag = tag;
    dt.index = index++;
    dt.col_base = col_base;
    col_base += (int)nc;
    dt.kind.clear();
    for (size_t c = 0; c < nc; ++c) dt.kind.push_back(kindOfType(latest->cols[c].type));
    dt.h_present.assign(nv, 0);
    dt.h_cols.assign(nc, std::vector<int64_t>(nv, 0));
    auto it = tstage.find(tag);
    if (it == tstage.end()) continue;
    const TagStage& ts = it->second;
    std::vector<int64_t> best(nv, -1);   // record index of the live version per vertex
    for (size_t i = 0; i < ts.vid.size(); ++i) {
      auto p = std::lower_bound(dict.begin(), dict.end(), ts.vid[i]);
      const uint64_t d = (uint64_t)(p - dict.begin());
      const int64_t b = best[d];
      if (b < 0 || ts.verkey[i] < ts.verkey[b] || (ts.verkey[i] == ts.verkey[b] && ts.seq[i] > ts.seq[b]))
        best[d] = (int64_t)i;
    }
    for (uint64_t d = 0; d < nv; ++d) {
      const int64_t b = best[d];
      if (b < 0) continue;
      dt.h_present[d] = ts.valid[b] ? 1 : 2;   // 2: record present, value undecodable
      for (size_t c = 0; c < nc && c < ts.props.size(); ++c) {
        int64_t x = ts.props[c][b];
        if (dt.kind[c] == VK_STRING && ts.valid[b]) x = remap[x];
        dt.h_cols[c][d] = x;
      }
    }
  }
  return upload_tags();
}

// DevTag host arrays (local dense ids) -> device arrays over the tag index space (single GPU: the
// dense ids; partitioned: all ranks' local rows gathered into the global id space).
int32_t Engine::upload_tags() {
  const uint64_t nv = snap.nv;
  const uint64_t G = (uint64_t)cfg.num_gpus;
  const uint64_t local = partitioned() ? npad : nv;          // rows of the local arrays
  const uint64_t space = partitioned() ? G * npad : nv;      // rows of the device arrays
  std::vector<int64_t*> all_cols;
  std::vector<uint8_t*> all_pres;
  void* d_stage = nullptr;
  auto up = [&](void** dst, const void* src, size_t bytes) -> bool {
    if (hipMalloc(dst, std::max<size_t>(bytes, 8)) != hipSuccess) return false;
    snap.device_bytes += bytes;
    if (!bytes) return true;
    if (!partitioned()) return !src || hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice) == hipSuccess;
    const size_t lb = bytes / G;
    if (hipMemcpy(d_stage, src, lb, hipMemcpyHostToDevice) != hipSuccess) return false;
    return comm->allgather(d_stage, *dst, lb, stream) == 0 && hipStreamSynchronize(stream) == hipSuccess;
  };
  if (partitioned() && hipMalloc(&d_stage, std::max<uint64_t>(local, 1) * 8) != hipSuccess)
    return fail(NBG_E_OUT_OF_MEMORY, "tag staging");
  int32_t rc = NBG_OK;
  std::vector<DevTag*> order(snap.tags.size(), nullptr);
  for (auto& kv : snap.tags) order[kv.second.index] = &kv.second;
  for (DevTag* dtp : order) {
    DevTag& dt = *dtp;
    std::vector<uint8_t> pres(local, 0);
    for (uint64_t d = 0; d < nv; ++d) pres[d] = dt.h_present[d] != 0;
    bool ok = up((void**)&dt.present, pres.data(), space);
    dt.cols.assign(dt.h_cols.size(), nullptr);
    std::vector<int64_t> buf(local, 0);
    for (size_t c = 0; ok && c < dt.h_cols.size(); ++c) {
      std::copy(dt.h_cols[c].begin(), dt.h_cols[c].end(), buf.begin());
      ok = up((void**)&dt.cols[c], buf.data(), space * 8);
    }
    if (!ok) { rc = fail(NBG_E_OUT_OF_MEMORY, "device allocation failed for tag columns"); break; }
    all_pres.push_back(dt.present);
    for (auto* p : dt.cols) all_cols.push_back(p);
  }
  if (d_stage) (void)hipFree(d_stage);
  if (rc) return rc;
  bool ok = hipMalloc((void**)&snap.d_tcols, std::max<size_t>(all_cols.size(), 1) * 8) == hipSuccess &&
            hipMalloc((void**)&snap.d_tpres, std::max<size_t>(all_pres.size(), 1) * 8) == hipSuccess;
  if (ok && !all_cols.empty())
    ok = hipMemcpy(snap.d_tcols, all_cols.data(), all_cols.size() * 8, hipMemcpyHostToDevice) == hipSuccess;
  if (ok && !all_pres.empty())
    ok = hipMemcpy(snap.d_tpres, all_pres.data(), all_pres.size() * 8, hipMemcpyHostToDevice) == hipSuccess;
  return ok ? NBG_OK : fail(NBG_E_OUT_OF_MEMORY, "device allocation failed for the tag tables");
}

// dense id -> vid table and the visibility flags
int32_t Engine::upload_vertices(const std::vector<uint8_t>& visible, bool all_visible) {
  const uint64_t nv = snap.nv;
  bool ok = hipMalloc((void**)&snap.d_vids, std::max<uint64_t>(nv, 1) * 8) == hipSuccess &&
            hipMemcpy(snap.d_vids, snap.h_vids.data(), nv * 8, hipMemcpyHostToDevice) == hipSuccess;
  snap.device_bytes += nv * 8;
  if (ok && !all_visible) {
    snap.h_visible = visible;
    ok = hipMalloc((void**)&snap.d_visible, nv) == hipSuccess &&
         hipMemcpy(snap.d_visible, visible.data(), nv, hipMemcpyHostToDevice) == hipSuccess;
    snap.device_bytes += nv;
  }
  return ok ? NBG_OK : fail(NBG_E_OUT_OF_MEMORY, "device allocation failed for the vertex table");
}

// Upload one signed type's CSR and columns (plus narrow copies of INT columns whose values fit
// 1 / 2 / 4 bytes, sign-extended on load: the final-step fast path reads those).  rank / valid:
// nullptr when every rank is 0 / every value decoded.
bool Engine::upload_type(DevEdgeType& dt, uint64_t nv, const std::vector<uint32_t>& col, const std::vector<int64_t>& dvid,
                         const std::vector<int64_t>* rk, const std::vector<std::vector<int64_t>>& pc,
                         const std::vector<uint8_t>* valid, const std::vector<VKind>& kinds) {
  const uint64_t E = dt.num_edges;
  const size_t nc = pc.size();
  auto up = [&](void** dst, const void* src, size_t bytes) -> bool {
    if (!bytes) bytes = 8;
    if (hipMalloc(dst, bytes) != hipSuccess) return false;
    snap.device_bytes += bytes;
    if (src && hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice) != hipSuccess) return false;
    return true;
  };
  bool ok = up((void**)&dt.row_ptr, dt.h_row_ptr.data(), (nv + 1) * 4) && up((void**)&dt.col, col.data(), E * 4) &&
            up((void**)&dt.dst_vid, dvid.data(), E * 8);
  if (ok && rk) ok = up((void**)&dt.rank, rk->data(), E * 8);
  dt.prop_kind = kinds;
  dt.props.assign(nc, nullptr);
  for (size_t c = 0; ok && c < nc; ++c) ok = up((void**)&dt.props[c], pc[c].data(), E * 8);
  dt.narrow.assign(nc, nullptr);
  dt.narrow_bytes.assign(nc, 0);
  for (size_t c = 0; ok && c < nc && E; ++c) {
    if (kinds[c] != VK_INT) continue;
    int64_t lo = INT64_MAX, hi = INT64_MIN;
#pragma omp parallel for reduction(min : lo) reduction(max : hi)
    for (int64_t i = 0; i < (int64_t)E; ++i) {
      lo = std::min(lo, pc[c][i]);
      hi = std::max(hi, pc[c][i]);
    }
    int bytes = 8;
    if (lo >= INT8_MIN && hi <= INT8_MAX) bytes = 1;
    else if (lo >= INT16_MIN && hi <= INT16_MAX) bytes = 2;
    else if (lo >= INT32_MIN && hi <= INT32_MAX) bytes = 4;
    if (bytes == 8) continue;
    std::vector<uint8_t> buf(E * (size_t)bytes);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)E; ++i) {
      const int64_t v = pc[c][i];
      if (bytes == 1) reinterpret_cast<int8_t*>(buf.data())[i] = (int8_t)v;
      else if (bytes == 2) reinterpret_cast<int16_t*>(buf.data())[i] = (int16_t)v;
      else reinterpret_cast<int32_t*>(buf.data())[i] = (int32_t)v;
    }
    ok = up(&dt.narrow[c], buf.data(), buf.size());
    dt.narrow_bytes[c] = bytes;
  }
  if (ok && valid) ok = up((void**)&dt.valid, valid->data(), E);
  if (ok && nc) ok = up((void**)&dt.d_props, dt.props.data(), nc * sizeof(int64_t*));
  uint32_t md = 0;
  for (uint64_t d = 0; d < nv; ++d) md = std::max(md, dt.h_row_ptr[d + 1] - dt.h_row_ptr[d]);
  dt.max_degree = (int)md;
  return ok;
}

int32_t Engine::finalize() {
  if (finalized) return fail(NBG_E_STATE, "engine already finalized");
  // 1. string dictionary: sorted; device code = 2 * rank
  std::vector<int64_t> remap(pool.size());
  {
    std::vector<int64_t> order(pool.size());
    std::iota(order.begin(), order.end(), 0);
    std::sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return pool[a] < pool[b]; });
    snap.strings.clear();
    for (auto id : order) {
      if (snap.strings.empty() || snap.strings.back() != pool[id]) snap.strings.push_back(pool[id]);
      remap[id] = 2 * (int64_t)(snap.strings.size() - 1);
    }
  }
  // 2. vertex dictionary: every vid that owns a row (src of any signed type)
  std::vector<int64_t> all;
  {
    size_t tot = 0;
    for (auto& kv : stage) tot += kv.second.src.size();
    all.reserve(tot);
    for (auto& kv : stage) all.insert(all.end(), kv.second.src.begin(), kv.second.src.end());
    for (auto& kv : tstage) all.insert(all.end(), kv.second.vid.begin(), kv.second.vid.end());
    __gnu_parallel::sort(all.begin(), all.end());
    all.erase(std::unique(all.begin(), all.end()), all.end());
  }
  const uint64_t nv = all.size();
  if (nv >= NO_ROW) return fail(NBG_E_UNSUPPORTED, "more than 2^32-1 vertices on one GPU");
  snap.nv = nv;
  snap.h_vids = all;
  auto dense = [&](int64_t vid) -> uint32_t {
    auto it = std::lower_bound(all.begin(), all.end(), vid);
    return (it != all.end() && *it == vid) ? (uint32_t)(it - all.begin()) : NO_ROW;
  };
  // dense id of every record's source (reused by the CSR build); home part per vertex — a vid
  // whose rows sit in two parts is not representable
  std::map<int32_t, std::vector<uint32_t>> src_dense;
  std::vector<int32_t> home(nv, 0);
  bool all_visible = true;
  bool split = false;
  for (auto& kv : stage) {
    auto& st = kv.second;
    auto& sd = src_dense[kv.first];
    sd.resize(st.src.size());
#pragma omp parallel for schedule(static) reduction(|| : split)
    for (int64_t i = 0; i < (int64_t)st.src.size(); ++i) {
      const uint32_t d = dense(st.src[i]);
      sd[i] = d;
      int32_t expected = 0;
      if (!__atomic_compare_exchange_n(&home[d], &expected, st.part[i], false, __ATOMIC_RELAXED, __ATOMIC_RELAXED) &&
          expected != st.part[i])
        split = true;
    }
  }
  for (auto& kv : tstage) {
    const TagStage& ts = kv.second;
    for (size_t i = 0; i < ts.vid.size(); ++i) {
      const uint32_t d = dense(ts.vid[i]);
      if (home[d] == 0) home[d] = ts.part[i];
      else if (home[d] != ts.part[i]) split = true;
    }
  }
  if (split) return fail(NBG_E_UNSUPPORTED, "vertex rows split across partitions");
  std::vector<uint8_t> visible(nv, 1);
  for (uint64_t d = 0; d < nv; ++d) {
    if (home[d] != hash_part(all[d], cfg.num_parts)) { visible[d] = 0; all_visible = false; }
  }
  snap.h_part = home;

  // 2b. partitioned mode: a global id space [G * npad) — rank q's vertices are q * npad + local
  // id — so a neighbour id names its owner (the rank serving its hash part) without a lookup.
  std::vector<int64_t> gdict;
  std::vector<uint64_t> gcount;
  if (partitioned()) {
    int32_t prc = exchange_dictionary(all, &gdict, &gcount);
    if (prc) return prc;
  }
  const int32_t G = cfg.num_gpus;
  auto gid = [&](int64_t vid) -> uint32_t {
    if (!partitioned()) return dense(vid);
    const uint64_t q = (uint64_t)(hash_part(vid, cfg.num_parts) % G);
    auto b = gdict.begin() + q * npad, e = b + gcount[q];
    auto it = std::lower_bound(b, e, vid);
    return (it != e && *it == vid) ? (uint32_t)(q * npad + (uint64_t)(it - b)) : NO_ROW;
  };

  // 3. per signed type: bucket by src, sort rows in key order, keep the live version
  int32_t rc = NBG_OK;
  for (auto& kv : stage) {
    const int32_t type = kv.first;
    EdgeStage& st = kv.second;
    const uint64_t n = st.src.size();
    std::vector<uint32_t> sd = std::move(src_dense[type]);
    std::vector<uint64_t> cnt(nv + 1, 0);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)n; ++i) __atomic_fetch_add(&cnt[sd[i] + 1], 1ull, __ATOMIC_RELAXED);
    for (uint64_t d = 0; d < nv; ++d) cnt[d + 1] += cnt[d];
    std::vector<RowKey> keys(n);
    {
      // bucket order inside a vertex does not matter: each bucket is sorted by rowkey_less
      // (a total order: load sequence breaks ties)
      std::vector<uint64_t> cur(cnt.begin(), cnt.end() - 1);
#pragma omp parallel for schedule(static)
      for (int64_t i = 0; i < (int64_t)n; ++i) {
        const uint64_t p = __atomic_fetch_add(&cur[sd[i]], 1ull, __ATOMIC_RELAXED);
        keys[p] = RowKey{bswap64((uint64_t)st.rank[i]), bswap64((uint64_t)st.dst[i]), st.verkey[i], st.seq[i],
                         (uint64_t)i};
      }
    }
    std::vector<uint32_t> live(nv + 1, 0);
#pragma omp parallel for schedule(dynamic, 4096)
    for (int64_t d = 0; d < (int64_t)nv; ++d) {
      auto b = keys.begin() + cnt[d], e = keys.begin() + cnt[d + 1];
      if (e - b > 1) std::sort(b, e, rowkey_less);
      uint32_t m = 0;
      for (auto it = b; it != e; ++it) {
        if (it != b && it->rank_be == (it - 1)->rank_be && it->dst_be == (it - 1)->dst_be) continue;
        b[m++] = *it;   // compact in place (m <= position)
      }
      live[d + 1] = m;
    }
    std::vector<uint64_t> rp(nv + 1, 0);
    for (uint64_t d = 0; d < nv; ++d) rp[d + 1] = rp[d] + live[d + 1];
    const uint64_t E = rp[nv];
    if (E >= 0xFFFFFFFFull) return fail(NBG_E_UNSUPPORTED, "more than 2^32-1 edges of one type on one GPU");
    DevEdgeType& dt = snap.types[type];
    dt.type = type;
    dt.num_edges = E;
    dt.h_row_ptr.resize(nv + 1);
    for (uint64_t d = 0; d <= nv; ++d) dt.h_row_ptr[d] = (uint32_t)rp[d];
    std::vector<uint32_t> col(E);
    std::vector<int64_t> dvid(E), rk(E);
    const size_t nc = type > 0 ? st.props.size() : 0;
    std::vector<std::vector<int64_t>> pc(nc, std::vector<int64_t>(E));
    std::vector<uint8_t> valid(type > 0 ? E : 0);
    bool any_rank = false, any_invalid = false;
    std::vector<VKind> kinds(nc, VK_INT);
    if (nc) {
      const Schema* latest = edges[type].latest();
      for (size_t c = 0; c < nc; ++c) kinds[c] = kindOfType(latest->cols[c].type);
    }
#pragma omp parallel for schedule(dynamic, 4096) reduction(|| : any_rank, any_invalid)
    for (int64_t d = 0; d < (int64_t)nv; ++d) {
      uint64_t o = rp[d];
      for (uint32_t m = 0; m < live[d + 1]; ++m) {
        const RowKey& k = keys[cnt[d] + m];
        uint64_t i = k.idx;
        col[o + m] = gid(st.dst[i]);
        dvid[o + m] = st.dst[i];
        rk[o + m] = st.rank[i];
        if (st.rank[i]) any_rank = true;
        for (size_t c = 0; c < nc; ++c) {
          int64_t b = st.props[c][i];
          if (kinds[c] == VK_STRING && st.valid[i]) b = remap[b];
          pc[c][o + m] = b;
        }
        if (type > 0) {
          valid[o + m] = st.valid[i];
          if (!st.valid[i]) any_invalid = true;
        }
      }
    }
    bool ok = upload_type(dt, nv, col, dvid, any_rank ? &rk : nullptr, pc, any_invalid ? &valid : nullptr, kinds);
    if (!ok) { rc = fail(NBG_E_OUT_OF_MEMORY, "device allocation failed for the snapshot"); break; }

    EdgeStage().src.swap(st.src);   // release staging as we go
    st = EdgeStage();
  }
  if (rc) return rc;
  rc = build_tags(all, remap);
  if (rc) return rc;
  rc = upload_vertices(visible, all_visible);
  if (rc) return rc;
  stage.clear();
  tstage.clear();
  pool.clear();
  pool_index.clear();
  finalized = true;
  return NBG_OK;
}

}  // namespace nbg
