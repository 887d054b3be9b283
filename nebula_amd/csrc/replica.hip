// FIND PATH replica of a partitioned snapshot (collective, at finalize).
//
// A partitioned engine keeps GO on the partitioned snapshot (a hop = local expansion + one bitmap
// all-to-all).  FIND SHORTEST PATH on it costs a collective per BFS level and
// per greedy hop (~12 per pair) — latency that no xGMI link removes, so a pair
// would be slower at 8 GPUs than at 1.  HBM is large enough to avoid that: RMAT-26 is 35.5 GB
// on one MI355X (288 GB), and its path-relevant part (offsets, neighbour ids, neighbour vids,
// ranks of every signed type: no property columns) is ~26 GB.  So every rank also holds a
// REPLICA of the path CSRs over the GLOBAL vertex space, built once here from the ranks' own
// CSRs (never from the staged records, which stay partitioned in host memory), and FIND PATH
// then runs on one GPU with the single-engine kernels: no collective per pair, and each rank can
// answer a different pair (path.cpp, nbg.h).  The replica is built when it fits; otherwise
// (or with nbg_set_path_replica(e, 0) / NBG_PATH_REPLICA=0) the collective search is used.
//
// Build (every step stream-ordered; the ranks' data travel by the engine's communicator):
//   1. the global dictionary: every rank's sorted vids, all-gathered (G x npad) and merged into
//      one sorted array; a global dense id is a vid's rank in it, so smallest vid = smallest id
//      (the tie-break order of the single engine); g2d maps a global id (owner * npad + local)
//      to it;
//   2. per signed type: every rank's out-degrees (all-gathered) give the replica's offsets
//      (scan in global dense order) and each rank's own row starts (scan per segment); the
//      edges then travel in fixed chunks (all-gather, bounded scratch) and each received edge is
//      placed at its row's replica offset, its neighbour renumbered by g2d.  Rows keep key order.
//   3. visibility bytes are all-gathered and renumbered the same way.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <rocprim/rocprim.hpp>
#include <string>
#include <vector>

#include "engine.h"

namespace nbg {
namespace {

constexpr int RB = 256;
inline unsigned rgrid(uint64_t n) {
  const uint64_t b = (n + RB - 1) / RB;
  return (unsigned)(b ? (b < 65535 ? b : 65535) : 1);
}

#define RP_TRY(x)                                       \
  do {                                                  \
    const hipError_t e_ = (x);                          \
    if (e_ != hipSuccess) return fail(e_, #x);          \
  } while (0)

// the valid entries of the all-gathered dictionaries, packed: q's vids at [base[q], base[q] + cnt[q])
__global__ void k_rp_pack(const int64_t* __restrict__ gd, uint64_t npad, int G, const uint64_t* __restrict__ cnt,
                          const uint64_t* __restrict__ base, int64_t* __restrict__ out) {
  for (uint64_t g = (uint64_t)blockIdx.x * RB + threadIdx.x; g < (uint64_t)G * npad; g += (uint64_t)gridDim.x * RB) {
    const uint64_t q = g / npad, i = g - q * npad;
    if (i < cnt[q]) out[base[q] + i] = gd[g];
  }
}

// global id -> global dense id (the vid's position in the merged dictionary D), NO_ROW for padding
__global__ void k_rp_g2d(const int64_t* __restrict__ gd, uint64_t npad, int G, const uint64_t* __restrict__ cnt,
                         const int64_t* __restrict__ D, uint64_t N, uint32_t* __restrict__ g2d) {
  for (uint64_t g = (uint64_t)blockIdx.x * RB + threadIdx.x; g < (uint64_t)G * npad; g += (uint64_t)gridDim.x * RB) {
    const uint64_t q = g / npad, i = g - q * npad;
    uint32_t d = NO_ROW;
    if (i < cnt[q]) {
      const int64_t v = gd[g];
      uint64_t lo = 0, hi = N;
      while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (D[mid] < v) lo = mid + 1;
        else hi = mid;
      }
      d = (uint32_t)lo;
    }
    g2d[g] = d;
  }
}

// this rank's out-degrees over npad slots (0 past nv or without the type)
__global__ void k_rp_deg(const uint32_t* __restrict__ row_ptr, uint64_t nv, uint64_t npad, uint32_t* __restrict__ deg) {
  for (uint64_t i = (uint64_t)blockIdx.x * RB + threadIdx.x; i < npad; i += (uint64_t)gridDim.x * RB)
    deg[i] = (row_ptr && i < nv) ? row_ptr[i + 1] - row_ptr[i] : 0u;
}

// degree of every global dense id (scattered from the global ids)
__global__ void k_rp_scatter_deg(const uint32_t* __restrict__ gdeg, const uint32_t* __restrict__ g2d, uint64_t n,
                                 uint32_t* __restrict__ ddeg) {
  for (uint64_t g = (uint64_t)blockIdx.x * RB + threadIdx.x; g < n; g += (uint64_t)gridDim.x * RB)
    if (g2d[g] != NO_ROW) ddeg[g2d[g]] = gdeg[g];
}

struct ChunkArgs {
  const uint32_t* col;      // [G * C] received neighbour global ids
  const int64_t* dst;       // [G * C] neighbour vids
  const int64_t* rank;      // [G * C] ranks (nullable: all 0)
  uint64_t C, k0;           // chunk length, first edge index of the chunk
  int G;
  uint64_t npad;
  const uint64_t* ecount;   // [G] edges of the type on each rank
  const uint64_t* vcount;   // [G] vertices of each rank
  const uint32_t* goff;     // [G * npad] each rank's row starts (exclusive scan of its degrees)
  const uint32_t* g2d;
  const uint32_t* rp;       // replica offsets [N + 1]
  uint32_t* out_col;
  int64_t* out_dst;
  int64_t* out_rank;        // nullable
};

// each received edge -> its replica position (row found by binary search in the sender's starts)
__global__ void k_rp_place(ChunkArgs a) {
  for (uint64_t x = (uint64_t)blockIdx.x * RB + threadIdx.x; x < (uint64_t)a.G * a.C; x += (uint64_t)gridDim.x * RB) {
    const uint64_t q = x / a.C, e = a.k0 + (x - q * a.C);
    if (e >= a.ecount[q]) continue;
    const uint32_t* off = a.goff + q * a.npad;
    uint64_t lo = 0, hi = a.vcount[q];   // last row whose start is <= e
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if (off[mid] <= e) lo = mid + 1;
      else hi = mid;
    }
    const uint64_t i = lo - 1;
    const uint32_t d = a.g2d[q * a.npad + i];
    const uint64_t pos = (uint64_t)a.rp[d] + (e - off[i]);
    const uint32_t c = a.col[x];
    a.out_col[pos] = c == NO_ROW ? NO_ROW : a.g2d[c];
    a.out_dst[pos] = a.dst[x];
    if (a.out_rank) a.out_rank[pos] = a.rank ? a.rank[x] : 0;
  }
}

__global__ void k_rp_vis(const uint8_t* __restrict__ gvis, const uint32_t* __restrict__ g2d, uint64_t n,
                         uint8_t* __restrict__ out) {
  for (uint64_t g = (uint64_t)blockIdx.x * RB + threadIdx.x; g < n; g += (uint64_t)gridDim.x * RB)
    if (g2d[g] != NO_ROW) out[g2d[g]] = gvis[g];
}

__global__ void k_rp_vis_local(const uint8_t* __restrict__ vis, uint64_t nv, uint64_t npad, uint8_t* __restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * RB + threadIdx.x; i < npad; i += (uint64_t)gridDim.x * RB)
    out[i] = i < nv ? (vis ? vis[i] : 1) : 0;
}

struct Builder {
  Engine& E;
  Comm* cm;
  hipStream_t s;
  int G;
  uint64_t npad;
  std::vector<void*> tmp;
  std::string err;
  explicit Builder(Engine& e) : E(e), cm(e.comm.get()), s(e.stream), G(e.cfg.num_gpus), npad(e.npad) {}
  ~Builder() {
    (void)hipStreamSynchronize(s);
    for (void* p : tmp) (void)hipFree(p);
  }
  hipError_t fail(hipError_t e, const char* what) {
    if (err.empty()) err = std::string(what) + ": " + hipGetErrorString(e);
    return e;
  }
  template <class T>
  hipError_t get(T** p, uint64_t n) {
    void* q = nullptr;
    const hipError_t e = hipMalloc(&q, std::max<uint64_t>(n, 1) * sizeof(T));
    if (e != hipSuccess) return e;
    tmp.push_back(q);
    *p = static_cast<T*>(q);
    return hipSuccess;
  }
  // a device allocation kept by the replica (freed with it on failure by the caller)
  template <class T>
  hipError_t keep(T** p, uint64_t n, std::vector<void*>* owned) {
    void* q = nullptr;
    const hipError_t e = hipMalloc(&q, std::max<uint64_t>(n, 1) * sizeof(T));
    if (e != hipSuccess) return e;
    owned->push_back(q);
    *p = static_cast<T*>(q);
    return hipSuccess;
  }
  hipError_t gather(const void* send, void* recv, size_t bytes) {
    if (cm->allgather(send, recv, bytes, s)) {
      err = "all-gather: " + cm->last;
      return hipErrorUnknown;
    }
    return hipSuccess;
  }
  hipError_t scan(const uint32_t* in, uint32_t* out, uint64_t n) {
    size_t bytes = 0;
    RP_TRY(rocprim::exclusive_scan(nullptr, bytes, in, out, 0u, n, rocprim::plus<uint32_t>(), s));
    void* t = nullptr;
    RP_TRY(get(reinterpret_cast<uint8_t**>(&t), bytes));
    RP_TRY(rocprim::exclusive_scan(t, bytes, in, out, 0u, n, rocprim::plus<uint32_t>(), s));
    return hipSuccess;
  }
  template <class T>
  hipError_t host_all(T v, std::vector<T>* out) {   // all-gather of one value per rank
    T* d = nullptr;
    T* r = nullptr;
    RP_TRY(get(&d, 1));
    RP_TRY(get(&r, (uint64_t)G));
    RP_TRY(hipMemcpyAsync(d, &v, sizeof(T), hipMemcpyHostToDevice, s));
    RP_TRY(gather(d, r, sizeof(T)));
    out->resize(G);
    RP_TRY(hipMemcpyAsync(out->data(), r, G * sizeof(T), hipMemcpyDeviceToHost, s));
    return hipStreamSynchronize(s);
  }
};

// replica bytes this rank would hold (path CSRs over every rank's vertices and edges) and the
// build's peak scratch
uint64_t replica_bytes(const Engine& E, uint64_t n_all, uint64_t e_all_per_type, bool ranks, uint64_t chunk) {
  const uint64_t G = (uint64_t)E.cfg.num_gpus;
  uint64_t b = n_all * 9 + G * E.npad * 16;
  b += E.snap.types.size() * ((n_all + 1) * 4 + e_all_per_type * (12 + (ranks ? 8 : 0)));
  return b + G * chunk * 20 + chunk * 20;
}

}  // namespace

bool path_replica_wanted(const Engine& E) {
  if (E.path_replica_mode >= 0) return E.path_replica_mode != 0;
  const char* v = getenv("NBG_PATH_REPLICA");
  return !v || atoi(v) != 0;
}

void destroy_path_replica(Engine& E) {
  if (!E.rep) return;
  Engine& R = *E.rep;
  path_slots_release(R);
  if (R.ws) ws_destroy(R.ws);
  if (R.sp) sp_destroy(R.sp);
  R.free_snapshot();
  if (R.stream) (void)hipStreamDestroy(R.stream);
  E.rep.reset();
}

int32_t build_path_replica(Engine& E) {
  destroy_path_replica(E);
  if (!E.partitioned() || !E.comm) return NBG_OK;
  Builder B(E);
  const int G = B.G;
  const uint64_t npad = B.npad;
  const uint64_t CHUNK = getenv("NBG_REPLICA_CHUNK") ? strtoull(getenv("NBG_REPLICA_CHUNK"), nullptr, 10) : (1ull << 25);
  // ---- sizes, and whether every rank wants and can hold the replica (agreed: all or none)
  std::vector<uint64_t> vcount;
  if (B.host_all<uint64_t>(E.snap.nv, &vcount) != hipSuccess) return E.fail(NBG_E_DEVICE, "replica: " + B.err);
  std::vector<int32_t> types;   // union of the ranks' signed types (each rank lists up to 64)
  {
    int32_t mine[64] = {0};
    int k = 0;
    for (auto& kv : E.snap.types)
      if (k < 64) mine[k++] = kv.first;
    int32_t *d = nullptr, *r = nullptr;
    if (B.get(&d, 64) != hipSuccess || B.get(&r, 64 * (uint64_t)G) != hipSuccess ||
        hipMemcpyAsync(d, mine, sizeof(mine), hipMemcpyHostToDevice, B.s) != hipSuccess ||
        B.gather(d, r, sizeof(mine)) != hipSuccess)
      return E.fail(NBG_E_DEVICE, "replica: " + B.err);
    std::vector<int32_t> all(64 * (size_t)G);
    if (hipMemcpyAsync(all.data(), r, all.size() * 4, hipMemcpyDeviceToHost, B.s) != hipSuccess ||
        hipStreamSynchronize(B.s) != hipSuccess)
      return E.fail(NBG_E_DEVICE, "replica: type list");
    for (int32_t t : all)
      if (t && std::find(types.begin(), types.end(), t) == types.end()) types.push_back(t);
    std::sort(types.begin(), types.end());
  }
  uint64_t n_all = 0, e_max = 0;
  for (uint64_t c : vcount) n_all += c;
  bool any_rank = false;
  for (auto& kv : E.snap.types) any_rank = any_rank || kv.second.rank;
  std::vector<uint64_t> etot(types.size(), 0);
  std::vector<std::vector<uint64_t>> ecount(types.size());
  for (size_t k = 0; k < types.size(); ++k) {
    auto it = E.snap.types.find(types[k]);
    if (B.host_all<uint64_t>(it == E.snap.types.end() ? 0 : it->second.num_edges, &ecount[k]) != hipSuccess)
      return E.fail(NBG_E_DEVICE, "replica: " + B.err);
    for (uint64_t c : ecount[k]) etot[k] += c;
    e_max = std::max(e_max, etot[k]);
  }
  std::vector<uint64_t> ranks_any;
  if (B.host_all<uint64_t>(any_rank ? 1 : 0, &ranks_any) != hipSuccess) return E.fail(NBG_E_DEVICE, "replica: " + B.err);
  any_rank = false;
  for (uint64_t x : ranks_any) any_rank = any_rank || x;
  size_t free_b = 0, total_b = 0;
  (void)hipMemGetInfo(&free_b, &total_b);
  int32_t local = NBG_OK;
  if (!path_replica_wanted(E)) local = NBG_E_UNSUPPORTED;
  else if (e_max >= 0xFFFFFFFFull || n_all >= NO_ROW) local = NBG_E_UNSUPPORTED;
  else if (replica_bytes(E, n_all, e_max, any_rank, CHUNK) > free_b / 10 * 8) local = NBG_E_OUT_OF_MEMORY;
  int32_t agreed = NBG_OK;
  if (B.cm->agree(B.s, local, &agreed)) return E.fail(NBG_E_DEVICE, "replica agreement: " + B.cm->last);
  if (agreed) return NBG_OK;   // no replica on any rank: FIND PATH stays collective

  auto R = std::make_unique<Engine>();
  std::vector<void*> owned;   // the replica's device arrays until its snapshot holds them
  auto bail = [&](hipError_t e) {
    for (void* p : owned) (void)hipFree(p);
    // every rank reaches the same point of the build; a local failure here aborts the
    // communicator so the peers' pending collectives fail too
    B.cm->abort();
    return E.fail(e == hipErrorOutOfMemory ? NBG_E_OUT_OF_MEMORY : NBG_E_DEVICE, "path replica: " + B.err);
  };
#define RB_TRY(x)                                  \
  do {                                             \
    const hipError_t e__ = (x);                    \
    if (e__ != hipSuccess) {                       \
      if (B.err.empty()) B.err = #x;               \
      return bail(e__);                            \
    }                                              \
  } while (0)
  // ---- 1. global dictionary
  uint64_t *d_cnt = nullptr, *d_base = nullptr;
  RB_TRY(B.get(&d_cnt, G));
  RB_TRY(B.get(&d_base, G));
  std::vector<uint64_t> base(G, 0);
  for (int q = 1; q < G; ++q) base[q] = base[q - 1] + vcount[q - 1];
  RB_TRY(hipMemcpyAsync(d_cnt, vcount.data(), G * 8, hipMemcpyHostToDevice, B.s));
  RB_TRY(hipMemcpyAsync(d_base, base.data(), G * 8, hipMemcpyHostToDevice, B.s));
  int64_t *lv = nullptr, *gd = nullptr, *packed = nullptr, *D = nullptr;
  RB_TRY(B.get(&lv, npad));
  RB_TRY(B.get(&gd, (uint64_t)G * npad));
  RB_TRY(hipMemsetAsync(lv, 0, npad * 8, B.s));
  if (E.snap.nv) RB_TRY(hipMemcpyAsync(lv, E.snap.d_vids, E.snap.nv * 8, hipMemcpyDeviceToDevice, B.s));
  RB_TRY(B.gather(lv, gd, npad * 8));
  RB_TRY(B.get(&packed, n_all));
  hipLaunchKernelGGL(k_rp_pack, dim3(rgrid((uint64_t)G * npad)), dim3(RB), 0, B.s, gd, npad, G, d_cnt, d_base, packed);
  RB_TRY(hipGetLastError());
  uint64_t N = 0;
  RB_TRY(bd_sort_unique(packed, n_all, &D, &N, B.s));
  owned.push_back(D);
  if (N != n_all) {   // a vid held by two ranks: every rank sees the same gathered data, so all stop here
    for (void* p : owned) (void)hipFree(p);
    return NBG_OK;
  }
  uint32_t* g2d = nullptr;
  RB_TRY(B.get(&g2d, (uint64_t)G * npad));
  hipLaunchKernelGGL(k_rp_g2d, dim3(rgrid((uint64_t)G * npad)), dim3(RB), 0, B.s, gd, npad, G, d_cnt, D, N, g2d);
  RB_TRY(hipGetLastError());
  Snapshot& rs = R->snap;
  rs.nv = N;
  rs.d_vids = D;
  rs.h_vids.resize(N);
  RB_TRY(hipMemcpyAsync(rs.h_vids.data(), D, N * 8, hipMemcpyDeviceToHost, B.s));
  // ---- 2. per signed type
  uint32_t *ldeg = nullptr, *gdeg = nullptr, *goff = nullptr, *ddeg = nullptr;
  RB_TRY(B.get(&ldeg, npad));
  RB_TRY(B.get(&gdeg, (uint64_t)G * npad));
  RB_TRY(B.get(&goff, (uint64_t)G * npad));
  RB_TRY(B.get(&ddeg, N + 1));
  uint64_t* d_ecnt = nullptr;
  RB_TRY(B.get(&d_ecnt, G));
  uint32_t *s_col = nullptr, *r_col = nullptr;
  int64_t *s_dst = nullptr, *r_dst = nullptr, *s_rank = nullptr, *r_rank = nullptr;
  RB_TRY(B.get(&s_col, CHUNK));
  RB_TRY(B.get(&r_col, (uint64_t)G * CHUNK));
  RB_TRY(B.get(&s_dst, CHUNK));
  RB_TRY(B.get(&r_dst, (uint64_t)G * CHUNK));
  if (any_rank) {
    RB_TRY(B.get(&s_rank, CHUNK));
    RB_TRY(B.get(&r_rank, (uint64_t)G * CHUNK));
  }
  for (size_t k = 0; k < types.size(); ++k) {
    const int32_t t = types[k];
    auto it = E.snap.types.find(t);
    const DevEdgeType* lt = it == E.snap.types.end() ? nullptr : &it->second;
    hipLaunchKernelGGL(k_rp_deg, dim3(rgrid(npad)), dim3(RB), 0, B.s, lt ? lt->row_ptr : nullptr, E.snap.nv, npad, ldeg);
    RB_TRY(hipGetLastError());
    RB_TRY(B.gather(ldeg, gdeg, npad * 4));
    for (int q = 0; q < G; ++q) RB_TRY(B.scan(gdeg + (uint64_t)q * npad, goff + (uint64_t)q * npad, npad));
    RB_TRY(hipMemsetAsync(ddeg, 0, (N + 1) * 4, B.s));
    hipLaunchKernelGGL(k_rp_scatter_deg, dim3(rgrid((uint64_t)G * npad)), dim3(RB), 0, B.s, gdeg, g2d,
                       (uint64_t)G * npad, ddeg);
    RB_TRY(hipGetLastError());
    DevEdgeType dt;
    dt.type = t;
    dt.num_edges = etot[k];
    RB_TRY(B.keep(&dt.row_ptr, N + 1, &owned));
    RB_TRY(B.scan(ddeg, dt.row_ptr, N + 1));   // row_ptr[N] = the total (ddeg[N] == 0)
    RB_TRY(B.keep(&dt.col, etot[k], &owned));
    RB_TRY(B.keep(&dt.dst_vid, etot[k], &owned));
    if (any_rank) RB_TRY(B.keep(&dt.rank, etot[k], &owned));
    RB_TRY(hipMemcpyAsync(d_ecnt, ecount[k].data(), G * 8, hipMemcpyHostToDevice, B.s));
    uint64_t emax = 0;
    for (uint64_t c : ecount[k]) emax = std::max(emax, c);
    const uint64_t mine = lt ? lt->num_edges : 0;
    for (uint64_t k0 = 0; k0 < emax; k0 += CHUNK) {
      const uint64_t n = k0 < mine ? std::min<uint64_t>(CHUNK, mine - k0) : 0;
      if (n) {
        RB_TRY(hipMemcpyAsync(s_col, lt->col + k0, n * 4, hipMemcpyDeviceToDevice, B.s));
        RB_TRY(hipMemcpyAsync(s_dst, lt->dst_vid + k0, n * 8, hipMemcpyDeviceToDevice, B.s));
        if (any_rank) {
          if (lt->rank) RB_TRY(hipMemcpyAsync(s_rank, lt->rank + k0, n * 8, hipMemcpyDeviceToDevice, B.s));
          else RB_TRY(hipMemsetAsync(s_rank, 0, n * 8, B.s));
        }
      }
      RB_TRY(B.gather(s_col, r_col, CHUNK * 4));
      RB_TRY(B.gather(s_dst, r_dst, CHUNK * 8));
      if (any_rank) RB_TRY(B.gather(s_rank, r_rank, CHUNK * 8));
      ChunkArgs a;
      a.col = r_col;
      a.dst = r_dst;
      a.rank = r_rank;
      a.C = CHUNK;
      a.k0 = k0;
      a.G = G;
      a.npad = npad;
      a.ecount = d_ecnt;
      a.vcount = d_cnt;
      a.goff = goff;
      a.g2d = g2d;
      a.rp = dt.row_ptr;
      a.out_col = dt.col;
      a.out_dst = dt.dst_vid;
      a.out_rank = dt.rank;
      hipLaunchKernelGGL(k_rp_place, dim3(rgrid((uint64_t)G * CHUNK)), dim3(RB), 0, B.s, a);
      RB_TRY(hipGetLastError());
    }
    dt.h_row_ptr.resize(N + 1);
    RB_TRY(hipMemcpyAsync(dt.h_row_ptr.data(), dt.row_ptr, (N + 1) * 4, hipMemcpyDeviceToHost, B.s));
    RB_TRY(hipStreamSynchronize(B.s));
    uint32_t md = 0;
    for (uint64_t v = 0; v < N; ++v) md = std::max(md, dt.h_row_ptr[v + 1] - dt.h_row_ptr[v]);
    dt.max_degree = (int)md;
    rs.types[t] = std::move(dt);
    rs.device_bytes += (N + 1) * 4 + etot[k] * (12 + (any_rank ? 8 : 0));
  }
  // ---- 3. visibility
  {
    uint8_t *lvis = nullptr, *gvis = nullptr;
    RB_TRY(B.get(&lvis, npad));
    RB_TRY(B.get(&gvis, (uint64_t)G * npad));
    hipLaunchKernelGGL(k_rp_vis_local, dim3(rgrid(npad)), dim3(RB), 0, B.s, E.snap.d_visible, E.snap.nv, npad, lvis);
    RB_TRY(hipGetLastError());
    RB_TRY(B.gather(lvis, gvis, npad));
    std::vector<uint64_t> any_hidden;
    uint64_t hidden = 0;
    if (!E.snap.h_visible.empty())
      for (uint8_t v : E.snap.h_visible) hidden += v == 0;
    if (B.host_all<uint64_t>(hidden, &any_hidden) != hipSuccess) return bail(hipErrorUnknown);
    hidden = 0;
    for (uint64_t x : any_hidden) hidden += x;
    if (hidden) {
      RB_TRY(B.keep(&rs.d_visible, N, &owned));
      hipLaunchKernelGGL(k_rp_vis, dim3(rgrid((uint64_t)G * npad)), dim3(RB), 0, B.s, gvis, g2d, (uint64_t)G * npad,
                         rs.d_visible);
      RB_TRY(hipGetLastError());
      rs.h_visible.resize(N);
      RB_TRY(hipMemcpyAsync(rs.h_visible.data(), rs.d_visible, N, hipMemcpyDeviceToHost, B.s));
    }
  }
  RB_TRY(hipStreamSynchronize(B.s));
#undef RB_TRY
  owned.clear();   // the snapshot holds them now
  rs.device_bytes += N * 9;
  // ---- the replica engine: a single-GPU engine over the replica snapshot (no props, no tags)
  R->cfg = E.cfg;
  R->cfg.num_gpus = 1;
  R->cfg.rank = 0;
  R->edges = E.edges;
  R->tags = E.tags;
  R->prof_mode = E.prof_mode;
  R->finalized = true;
  if (hipStreamCreateWithFlags(&R->stream, hipStreamNonBlocking) != hipSuccess) {
    R->free_snapshot();
    return E.fail(NBG_E_DEVICE, "replica stream");
  }
  if (int32_t rc = engine_ready(*R)) {
    R->free_snapshot();
    (void)hipStreamDestroy(R->stream);
    return E.fail(rc, "path replica workspace: " + R->last_error);
  }
  E.rep = std::move(R);
  return NBG_OK;
}

}  // namespace nbg
