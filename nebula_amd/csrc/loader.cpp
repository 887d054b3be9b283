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
// One staged record (KV path).  The optional columns of EdgeStage materialise on the first
// record that needs them, so bulk loads keep only src / dst / props.
static void stage_push(EdgeStage& st, int64_t src, int64_t dst, int64_t rank, uint64_t verkey, int32_t part,
                       int32_t parts) {
  const uint64_t n = st.size();
  if (n == 0 && st.verkey.empty()) st.ver0 = verkey;
  if (st.rank.empty() && rank != 0) st.rank.assign(n, 0);
  if (st.verkey.empty() && verkey != st.ver0) st.verkey.assign(n, st.ver0);
  if (st.part.empty() && part != hash_part(src, parts)) {
    st.part.resize(n);
    for (uint64_t i = 0; i < n; ++i) st.part[i] = hash_part(st.src[i], parts);
  }
  st.src.push_back(src);
  st.dst.push_back(dst);
  if (!st.rank.empty()) st.rank.push_back(rank);
  if (!st.verkey.empty()) st.verkey.push_back(verkey);
  if (!st.part.empty()) st.part.push_back(part);
}

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
      const uint64_t at = st.size();
      stage_push(st, src, dst, rank, bswap64(ver), item >> 8, cfg.num_parts);
      ++seq;
      if (type > 0) {
        auto es = edges.find(type);
        const Schema* latest = es == edges.end() ? nullptr : es->second.latest();
        size_t nc = latest ? latest->cols.size() : 0;
        if (st.props.size() < nc) st.props.resize(nc, std::vector<int64_t>(at, 0));
        props.assign(nc, 0);
        bool ok = latest && decode_row(es->second, v, vlen, props.data());
        for (size_t c = 0; c < nc; ++c) st.props[c].push_back(ok ? props[c] : 0);
        for (size_t c = nc; c < st.props.size(); ++c) st.props[c].push_back(0);
        if (!ok && st.valid.empty()) st.valid.assign(at, 1);
        if (!st.valid.empty()) st.valid.push_back(ok ? 1 : 0);
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

// The indices i in [0, n) with keep(i), ascending (parallel, two passes).
template <typename Keep>
static std::vector<uint64_t> kept_indices(uint64_t n, Keep keep) {
  const int T = omp_get_max_threads();
  std::vector<uint64_t> cnt(T + 1, 0);
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num();
    const uint64_t b = n * t / T, e = n * (t + 1) / T;
    uint64_t c = 0;
    for (uint64_t i = b; i < e; ++i) c += keep(i) ? 1 : 0;
    cnt[t + 1] = c;
  }
  for (int t = 0; t < T; ++t) cnt[t + 1] += cnt[t];
  std::vector<uint64_t> idx(cnt[T]);
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num();
    const uint64_t b = n * t / T, e = n * (t + 1) / T;
    uint64_t o = cnt[t];
    for (uint64_t i = b; i < e; ++i)
      if (keep(i)) idx[o++] = i;
  }
  return idx;
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
  const uint64_t ver = bswap64((uint64_t)(INT64_MAX - 1));   // one version for the whole batch
  const int32_t P = cfg.num_parts, G = cfg.num_gpus, R = cfg.rank;
  bool any_rank = false;
  if (rank) {
#pragma omp parallel for reduction(|| : any_rank)
    for (int64_t i = 0; i < (int64_t)n; ++i) any_rank = any_rank || rank[i] != 0;
  }
  // out-edges at src's part, in-edges (dst, -type, rank, src) with no props at dst's part
  for (int side = 0; side < 2; ++side) {
    EdgeStage& st = stage[side ? -type : type];
    const int64_t* a = side ? dst : src;
    const int64_t* b = side ? src : dst;
    const uint64_t at = st.size();
    if (at == 0 && st.verkey.empty()) st.ver0 = ver;
    if (st.verkey.empty() && ver != st.ver0) st.verkey.assign(at, st.ver0);
    if (any_rank && st.rank.empty()) st.rank.assign(at, 0);
    const bool with_props = side == 0;
    if (with_props && st.props.size() < (size_t)ncols) st.props.resize(ncols, std::vector<int64_t>(at, 0));
    // a partitioned rank keeps the records of the parts it serves (part % G == rank)
    std::vector<uint64_t> idx;
    if (G > 1) idx = kept_indices(n, [&](uint64_t i) { return hash_part(a[i], P) % G == R; });
    const uint64_t m = G > 1 ? idx.size() : n;
    // grow every column to its final size first (the parallel writes below index into them)
    st.src.resize(at + m);
    st.dst.resize(at + m);
    if (!st.rank.empty()) st.rank.resize(at + m);
    if (!st.verkey.empty()) st.verkey.resize(at + m);
    if (!st.part.empty()) st.part.resize(at + m);
    if (!st.valid.empty()) st.valid.resize(at + m);
    if (with_props)
      for (int32_t c = 0; c < ncols; ++c) st.props[c].resize(at + m);
    auto put = [&](uint64_t o, uint64_t i) {
      st.src[o] = a[i];
      st.dst[o] = b[i];
      if (!st.rank.empty()) st.rank[o] = rank ? rank[i] : 0;
      if (!st.verkey.empty()) st.verkey[o] = ver;
      if (!st.part.empty()) st.part[o] = hash_part(a[i], P);
      if (!st.valid.empty()) st.valid[o] = 1;
      if (with_props) {
        for (int32_t c = 0; c < ncols; ++c) {
          int64_t x = 0;
          switch (latest->cols[c].type) {
            case NBG_T_BOOL: x = static_cast<const uint8_t*>(cols[c])[i] != 0; break;
            case NBG_T_FLOAT: case NBG_T_DOUBLE: memcpy(&x, static_cast<const double*>(cols[c]) + i, 8); break;
            default: x = static_cast<const int64_t*>(cols[c])[i]; break;
          }
          st.props[c][o] = x;
        }
      }
    };
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < (int64_t)m; ++k) put(at + (uint64_t)k, G > 1 ? idx[k] : (uint64_t)k);
  }
  seq += n;
  return NBG_OK;
}

// ----------------------------------------------------------------------------- finalize
// Every rank learns every rank's sorted vertex dictionary (allgather over the communicator):
// npad = the largest dictionary rounded up to PART_ALIGN.
int32_t Engine::exchange_strings(std::vector<std::string>* strings) {
  if (!comm) return fail(NBG_E_STATE, "a partitioned engine (num_gpus > 1) needs nbg_comm_init before nbg_finalize");
  const uint64_t G = (uint64_t)cfg.num_gpus;
  std::string blob;   // [u32 length][bytes] per string
  for (const std::string& x : *strings) {
    const uint32_t n = (uint32_t)x.size();
    blob.append(reinterpret_cast<const char*>(&n), 4);
    blob += x;
  }
  uint64_t* d_cnt = nullptr;
  char *d_loc = nullptr, *d_glob = nullptr;
  auto done = [&](int32_t rc, const std::string& msg) {
    for (void* p : {(void*)d_cnt, (void*)d_loc, (void*)d_glob})
      if (p) (void)hipFree(p);
    return rc ? fail(rc, msg) : NBG_OK;
  };
  const uint64_t nb = blob.size();
  if (hipMalloc((void**)&d_cnt, (G + 1) * 8) != hipSuccess || hipMemcpy(d_cnt + G, &nb, 8, hipMemcpyHostToDevice) != hipSuccess)
    return done(NBG_E_OUT_OF_MEMORY, "string dictionary exchange: device allocation");
  if (comm->allgather(d_cnt + G, d_cnt, 8, stream) || hipStreamSynchronize(stream) != hipSuccess)
    return done(NBG_E_DEVICE, "string dictionary exchange (sizes): " + comm->last);
  std::vector<uint64_t> sizes(G);
  if (hipMemcpy(sizes.data(), d_cnt, G * 8, hipMemcpyDeviceToHost) != hipSuccess)
    return done(NBG_E_DEVICE, "string dictionary exchange: copy");
  uint64_t mx = 8;
  for (uint64_t c : sizes) mx = std::max(mx, (c + 7) / 8 * 8);
  if (hipMalloc((void**)&d_loc, mx) != hipSuccess || hipMalloc((void**)&d_glob, G * mx) != hipSuccess)
    return done(NBG_E_OUT_OF_MEMORY, "string dictionary exchange: device allocation");
  if (nb && hipMemcpy(d_loc, blob.data(), nb, hipMemcpyHostToDevice) != hipSuccess)
    return done(NBG_E_DEVICE, "string dictionary exchange: upload");
  if (comm->allgather(d_loc, d_glob, mx, stream) || hipStreamSynchronize(stream) != hipSuccess)
    return done(NBG_E_DEVICE, "string dictionary exchange (bytes): " + comm->last);
  std::string all(G * mx, '\0');
  if (hipMemcpy(&all[0], d_glob, G * mx, hipMemcpyDeviceToHost) != hipSuccess)
    return done(NBG_E_DEVICE, "string dictionary exchange: download");
  std::vector<std::string> u;
  for (uint64_t q = 0; q < G; ++q) {
    const char* p = all.data() + q * mx;
    for (uint64_t o = 0; o + 4 <= sizes[q];) {
      uint32_t n;
      memcpy(&n, p + o, 4);
      u.emplace_back(p + o + 4, n);
      o += 4 + n;
    }
  }
  std::sort(u.begin(), u.end());
  u.erase(std::unique(u.begin(), u.end()), u.end());
  *strings = std::move(u);
  return done(NBG_OK, "");
}

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
// Every rank's out-degree per positive type, all-gathered into the global id space on the host
// (G * npad 4-byte words per type: 134 MB at RMAT-26 over 8 ranks).
int32_t Engine::gather_degrees() {
  h_gdeg.clear();
  const uint64_t G = (uint64_t)cfg.num_gpus;
  uint32_t *d_loc = nullptr, *d_all = nullptr;
  auto done = [&](int32_t rc, const std::string& msg) {
    if (d_loc) (void)hipFree(d_loc);
    if (d_all) (void)hipFree(d_all);
    return rc ? fail(rc, msg) : NBG_OK;
  };
  if (hipMalloc((void**)&d_loc, npad * 4) != hipSuccess || hipMalloc((void**)&d_all, G * npad * 4) != hipSuccess)
    return done(NBG_E_OUT_OF_MEMORY, "degree all-gather: device allocation");
  // (every rank walks the same type list: the registered edge types, present locally or not)
  for (auto& kv : edges) {
    const int32_t t = kv.first;
    std::vector<uint32_t> deg(npad, 0);
    auto it = snap.types.find(t);
    if (it != snap.types.end() && it->second.h_row_ptr.size() == snap.nv + 1)
      for (uint64_t d = 0; d < snap.nv; ++d) deg[d] = it->second.h_row_ptr[d + 1] - it->second.h_row_ptr[d];
    if (hipMemcpy(d_loc, deg.data(), npad * 4, hipMemcpyHostToDevice) != hipSuccess)
      return done(NBG_E_DEVICE, "degree all-gather: upload");
    if (comm->allgather(d_loc, d_all, npad * 4, stream) || hipStreamSynchronize(stream) != hipSuccess)
      return done(NBG_E_DEVICE, "degree all-gather: " + comm->last);
    std::vector<uint32_t>& g = h_gdeg[t];
    g.resize(G * npad);
    if (hipMemcpy(g.data(), d_all, G * npad * 4, hipMemcpyDeviceToHost) != hipSuccess)
      return done(NBG_E_DEVICE, "degree all-gather: download");
  }
  return done(NBG_OK, "");
}

uint64_t Engine::first_hop_bound(int32_t type, const int64_t* starts, uint64_t n, uint32_t cap) const {
  auto it = h_gdeg.find(type);
  const uint64_t G = (uint64_t)cfg.num_gpus;
  if (it == h_gdeg.end() || h_gcount.size() != G || h_gdict.size() != G * npad || n > 4096) return UINT64_MAX;
  std::vector<uint64_t> per(G, 0);
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t q = (uint64_t)hash_part(starts[i], cfg.num_parts) % G;
    auto b = h_gdict.begin() + (int64_t)(q * npad), e = b + (int64_t)h_gcount[q];
    auto f = std::lower_bound(b, e, starts[i]);
    if (f == e || *f != starts[i]) continue;
    per[q] += std::min<uint64_t>(it->second[(uint64_t)(f - h_gdict.begin())], cap);
  }
  return *std::max_element(per.begin(), per.end());
}

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
  bool ok = true;
  if (!snap.d_vids) {   // (finalize builds the table on the device; a snapshot file uploads it)
    ok = hipMalloc((void**)&snap.d_vids, std::max<uint64_t>(nv, 1) * 8) == hipSuccess &&
         hipMemcpy(snap.d_vids, snap.h_vids.data(), nv * 8, hipMemcpyHostToDevice) == hipSuccess;
    snap.device_bytes += nv * 8;
  }
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
  const hipStream_t s = stream;
  // device temporaries of the build, released on every exit
  std::map<int32_t, int64_t*> d_src;
  std::vector<void*> tmp;
  auto cleanup = [&]() {
    for (auto& kv : d_src)
      if (kv.second) (void)hipFree(kv.second);
    d_src.clear();
    for (void* p : tmp)
      if (p) (void)hipFree(p);
    tmp.clear();
  };
  auto bail = [&](int32_t code, const std::string& msg) {
    cleanup();
    free_snapshot();
    return fail(code, msg);
  };
  auto hip = [&](hipError_t e, const char* what) -> bool {
    if (e == hipSuccess) return true;
    last_error = std::string(what) + ": " + hipGetErrorString(e);
    return false;
  };
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
    if (partitioned()) {   // one dictionary over all ranks: codes are rank-independent
      if (int32_t rc = exchange_strings(&snap.strings)) {
        const std::string msg = last_error;
        return bail(rc, msg);
      }
      for (size_t id = 0; id < pool.size(); ++id)
        remap[id] = 2 * (int64_t)(std::lower_bound(snap.strings.begin(), snap.strings.end(), pool[id]) - snap.strings.begin());
    }
  }
  // 2. vertex dictionary on the device: every vid that owns a row (the source of any signed
  // type's record, or a tag record): per-type sorted sets, then their union
  std::vector<int64_t> tag_vids;
  for (auto& kv : tstage) tag_vids.insert(tag_vids.end(), kv.second.vid.begin(), kv.second.vid.end());
  int64_t* d_dict = nullptr;
  uint64_t nv = 0;
  {
    std::vector<std::pair<int64_t*, uint64_t>> sets;
    uint64_t tot = tag_vids.size();
    for (auto& kv : stage) {
      const uint64_t n = kv.second.size();
      int64_t* d = nullptr;
      if (!hip(hipMalloc((void**)&d, std::max<uint64_t>(n, 1) * 8), "device allocation (sources)"))
        return bail(NBG_E_OUT_OF_MEMORY, last_error);
      d_src[kv.first] = d;
      if (n && !hip(hipMemcpyAsync(d, kv.second.src.data(), n * 8, hipMemcpyHostToDevice, s), "upload"))
        return bail(NBG_E_DEVICE, last_error);
      int64_t* u = nullptr;
      uint64_t nu = 0;
      if (!hip(bd_sort_unique(d, n, &u, &nu, s), "vertex dictionary")) return bail(NBG_E_DEVICE, last_error);
      tmp.push_back(u);
      sets.emplace_back(u, nu);
      tot += nu;
    }
    int64_t* cat = nullptr;
    if (!hip(hipMalloc((void**)&cat, std::max<uint64_t>(tot, 1) * 8), "device allocation (dictionary)"))
      return bail(NBG_E_OUT_OF_MEMORY, last_error);
    tmp.push_back(cat);
    uint64_t o = 0;
    for (auto& u : sets) {
      if (u.second && !hip(hipMemcpyAsync(cat + o, u.first, u.second * 8, hipMemcpyDeviceToDevice, s), "copy"))
        return bail(NBG_E_DEVICE, last_error);
      o += u.second;
    }
    if (!tag_vids.empty() &&
        !hip(hipMemcpyAsync(cat + o, tag_vids.data(), tag_vids.size() * 8, hipMemcpyHostToDevice, s), "upload"))
      return bail(NBG_E_DEVICE, last_error);
    if (!hip(bd_sort_unique(cat, tot, &d_dict, &nv, s), "vertex dictionary")) return bail(NBG_E_DEVICE, last_error);
    snap.d_vids = d_dict;   // the snapshot's dense id -> vid table
    snap.device_bytes += std::max<uint64_t>(nv, 1) * 8;
  }
  if (nv >= NO_ROW) return bail(NBG_E_UNSUPPORTED, "more than 2^32-1 vertices on one GPU");
  snap.nv = nv;
  std::vector<int64_t> all(nv);
  if (nv && !hip(hipMemcpy(all.data(), d_dict, nv * 8, hipMemcpyDeviceToHost), "download"))
    return bail(NBG_E_DEVICE, last_error);
  snap.h_vids = all;
  auto dense = [&](int64_t vid) -> uint32_t {
    auto it = std::lower_bound(all.begin(), all.end(), vid);
    return (it != all.end() && *it == vid) ? (uint32_t)(it - all.begin()) : NO_ROW;
  };
  // 2a. home part per vertex; a vid whose rows sit in two parts is not representable.  Records
  // loaded without an explicit part sit in their source's hash part.
  std::vector<int32_t> home(nv, 0);
  bool explicit_parts = false;
  for (auto& kv : stage) explicit_parts = explicit_parts || !kv.second.part.empty();
  for (auto& kv : tstage)
    for (size_t i = 0; i < kv.second.vid.size() && !explicit_parts; ++i)
      explicit_parts = kv.second.part[i] != hash_part(kv.second.vid[i], cfg.num_parts);
  bool split = false;
  if (explicit_parts) {
    int32_t* d_home = nullptr;
    if (!hip(hipMalloc((void**)&d_home, std::max<uint64_t>(nv, 1) * 4), "device allocation (home)"))
      return bail(NBG_E_OUT_OF_MEMORY, last_error);
    tmp.push_back(d_home);
    if (!hip(hipMemsetAsync(d_home, 0, std::max<uint64_t>(nv, 1) * 4, s), "memset"))
      return bail(NBG_E_DEVICE, last_error);
    for (auto& kv : stage) {
      bool sp = false;
      const EdgeStage& st = kv.second;
      if (!hip(bd_home(d_home, d_src[kv.first], st.part.empty() ? nullptr : st.part.data(), st.size(), d_dict, nv,
                       cfg.num_parts, &sp, s),
               "home parts"))
        return bail(NBG_E_DEVICE, last_error);
      split = split || sp;
    }
    if (nv && !hip(hipMemcpy(home.data(), d_home, nv * 4, hipMemcpyDeviceToHost), "download"))
      return bail(NBG_E_DEVICE, last_error);
    for (auto& kv : tstage) {
      const TagStage& ts = kv.second;
      for (size_t i = 0; i < ts.vid.size(); ++i) {
        const uint32_t d = dense(ts.vid[i]);
        if (home[d] == 0) home[d] = ts.part[i];
        else if (home[d] != ts.part[i]) split = true;
      }
    }
  } else {
#pragma omp parallel for schedule(static)
    for (int64_t d = 0; d < (int64_t)nv; ++d) home[d] = hash_part(all[d], cfg.num_parts);
  }
  if (split) return bail(NBG_E_UNSUPPORTED, "vertex rows split across partitions");
  bool all_visible = true;
  std::vector<uint8_t> visible(nv, 1);
  if (explicit_parts) {
    for (uint64_t d = 0; d < nv; ++d) {
      if (home[d] != hash_part(all[d], cfg.num_parts)) { visible[d] = 0; all_visible = false; }
    }
  }
  snap.h_part = home;

  // 2b. partitioned mode: a global id space [G * npad) — rank q's vertices are q * npad + local
  // id — so a neighbour id names its owner (the rank serving its hash part) without a lookup.
  GidMap gm;
  gm.dict = d_dict;
  gm.nv = nv;
  gm.parts = cfg.num_parts;
  gm.gpus = cfg.num_gpus;
  std::vector<int64_t> gdict;
  std::vector<uint64_t> gcount;
  if (partitioned()) {
    int32_t prc = exchange_dictionary(all, &gdict, &gcount);
    if (prc) {
      const std::string msg = last_error;
      return bail(prc, msg);
    }
    int64_t* d_g = nullptr;
    uint64_t* d_c = nullptr;
    if (!hip(hipMalloc((void**)&d_g, std::max<size_t>(gdict.size(), 1) * 8), "device allocation") ||
        !hip(hipMalloc((void**)&d_c, std::max<size_t>(gcount.size(), 1) * 8), "device allocation"))
      return bail(NBG_E_OUT_OF_MEMORY, last_error);
    tmp.push_back(d_g);
    tmp.push_back(d_c);
    if (!hip(hipMemcpy(d_g, gdict.data(), gdict.size() * 8, hipMemcpyHostToDevice), "upload") ||
        !hip(hipMemcpy(d_c, gcount.data(), gcount.size() * 8, hipMemcpyHostToDevice), "upload"))
      return bail(NBG_E_DEVICE, last_error);
    gm.gdict = d_g;
    gm.gcount = d_c;
    gm.npad = npad;
  }

  // 3. per signed type: CSR on the device (records sorted in key order, the live version kept)
  for (auto& kv : stage) {
    const int32_t type = kv.first;
    EdgeStage& st = kv.second;
    const size_t nc = type > 0 ? st.props.size() : 0;
    std::vector<VKind> kinds(nc, VK_INT);
    if (nc) {
      const Schema* latest = edges[type].latest();
      for (size_t c = 0; c < nc; ++c) kinds[c] = kindOfType(latest->cols[c].type);
    }
    for (size_t c = 0; c < nc; ++c) {   // string ids -> dictionary codes
      if (kinds[c] != VK_STRING) continue;
      std::vector<int64_t>& col = st.props[c];
#pragma omp parallel for schedule(static)
      for (int64_t i = 0; i < (int64_t)col.size(); ++i)
        if (st.valid.empty() || st.valid[i]) col[i] = remap[col[i]];
    }
    std::vector<const int64_t*> pcols(nc);
    for (size_t c = 0; c < nc; ++c) pcols[c] = st.props[c].data();
    TypeBuildIn in;
    in.n = st.size();
    in.d_src = d_src[type];
    in.dst = st.dst.data();
    in.rank = st.rank.empty() ? nullptr : st.rank.data();
    in.verkey = st.verkey.empty() ? nullptr : st.verkey.data();
    in.nprops = (int)nc;
    in.props = pcols.data();
    in.kinds = kinds.data();
    in.valid = (type > 0 && !st.valid.empty()) ? st.valid.data() : nullptr;
    DevEdgeType& dt = snap.types[type];
    dt.type = type;
    dt.prop_kind = kinds;
    uint64_t bytes = 0;
    std::string err;
    hipError_t he = bd_build_type(in, gm, s, &dt, &bytes, &err);
    if (he != hipSuccess) {
      if (err.empty()) err = std::string("snapshot build: ") + hipGetErrorString(he);
      return bail(he == hipErrorOutOfMemory ? NBG_E_OUT_OF_MEMORY
                                            : (he == hipErrorInvalidValue ? NBG_E_UNSUPPORTED : NBG_E_DEVICE),
                  err);
    }
    if (dt.num_edges >= 0xFFFFFFFFull) return bail(NBG_E_UNSUPPORTED, "more than 2^32-1 edges of one type on one GPU");
    snap.device_bytes += bytes;
    (void)hipFree(d_src[type]);   // release as we go
    d_src[type] = nullptr;
    st = EdgeStage();
  }
  cleanup();
  if (partitioned()) {
    h_gdict = std::move(gdict);
    h_gcount = std::move(gcount);
  }
  int32_t rc = partitioned() ? gather_degrees() : NBG_OK;
  if (!rc) rc = build_tags(all, remap);
  if (!rc) rc = upload_vertices(visible, all_visible);
  if (rc) {
    const std::string msg = last_error;
    free_snapshot();
    return fail(rc, msg);
  }
  stage.clear();
  tstage.clear();
  pool.clear();
  pool_index.clear();
  finalized = true;
  return NBG_OK;
}

}  // namespace nbg
