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
#include <unistd.h>
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

// the merged dictionary must hold every vid once (ranks own disjoint vertex sets)
__global__ void k_rp_dups(const int64_t* __restrict__ D, uint64_t n, uint32_t* __restrict__ dups) {
  for (uint64_t i = (uint64_t)blockIdx.x * RB + threadIdx.x + 1; i < n; i += (uint64_t)gridDim.x * RB)
    if (D[i] == D[i - 1]) atomicAdd(dups, 1u);
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

// the replica's scratch and kept arrays: every allocation of the build is made before its first
// data collective (a rank-local OOM after that point could only abort the communicator)
struct Builder {
  Engine& E;
  Comm* cm;
  hipStream_t s;
  int G;
  uint64_t npad;
  std::vector<void*> tmp;    // freed when the build ends
  std::vector<void*> kept;   // the replica's arrays (freed on failure, else held by its snapshot)
  bool oom = false;
  std::string err;
  explicit Builder(Engine& e) : E(e), cm(e.comm.get()), s(e.stream), G(e.cfg.num_gpus), npad(e.npad) {}
  ~Builder() {
    (void)hipStreamSynchronize(s);
    for (void* p : tmp) (void)hipFree(p);
    for (void* p : kept) (void)hipFree(p);
  }
  hipError_t fail(hipError_t e, const char* what) {
    if (err.empty()) err = std::string(what) + ": " + hipGetErrorString(e);
    return e;
  }
  template <class T>
  T* alloc(uint64_t n, std::vector<void*>& into) {
    if (oom) return nullptr;
    void* q = nullptr;
    if (hipMalloc(&q, std::max<uint64_t>(n, 1) * sizeof(T)) != hipSuccess) {
      oom = true;
      err = "hipMalloc of " + std::to_string(n * sizeof(T)) + " bytes";
      (void)hipGetLastError();
      return nullptr;
    }
    into.push_back(q);
    return static_cast<T*>(q);
  }
  template <class T>
  T* get(uint64_t n) { return alloc<T>(n, tmp); }
  template <class T>
  T* keep(uint64_t n) { return alloc<T>(n, kept); }
  hipError_t gather(const void* send, void* recv, size_t bytes) {
    if (cm->allgather(send, recv, bytes, s)) {
      err = "all-gather: " + cm->last;
      return hipErrorUnknown;
    }
    return hipSuccess;
  }
};

// a key naming the physical device this rank runs on (host name + PCI bus id): ranks sharing one
// GPU (the one-GPU rehearsals, in-process groups) share its free memory
uint64_t device_key(int dev) {
  char host[256] = {0};
  (void)gethostname(host, sizeof(host) - 1);
  char bus[64] = {0};
  (void)hipDeviceGetPCIBusId(bus, sizeof(bus) - 1, dev);
  uint64_t h = 1469598103934665603ull;
  for (const char* p : {static_cast<const char*>(host), static_cast<const char*>(bus)})
    for (; *p; ++p) h = (h ^ (uint8_t)*p) * 1099511628211ull;
  return h;
}

// replica bytes this rank would hold (path CSRs over every rank's vertices and edges) and the
// build's peak scratch
uint64_t replica_bytes(const Engine& E, uint64_t n_all, uint64_t e_all_per_type, uint64_t ntypes, bool ranks,
                       uint64_t chunk) {
  const uint64_t G = (uint64_t)E.cfg.num_gpus;
  uint64_t b = n_all * 26 + G * E.npad * 25;
  b += ntypes * ((n_all + 1) * 4 + e_all_per_type * (12 + (ranks ? 8 : 0)));
  return b + (G + 1) * chunk * (12 + (ranks ? 8 : 0));
}

// the share of this rank's free HBM the replica may take (NBG_REPLICA_FIT, default 0.8)
double replica_fit() {
  const char* v = getenv("NBG_REPLICA_FIT");
  const double f = v ? atof(v) : 0.8;
  return f > 0 && f <= 1 ? f : 0.8;
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
  Comm* const cm = E.comm.get();
  const int G = E.cfg.num_gpus;
  const uint64_t npad = E.npad;
  const hipStream_t st = E.stream;
  auto xfail = [&](const char* what) { return E.fail(NBG_E_DEVICE, std::string("replica ") + what + ": " + cm->last); };
  // ---- 1. sizes: host words through the communicator's own scratch (nothing allocated here)
  uint64_t hidden = 0;
  for (uint8_t v : E.snap.h_visible) hidden += v == 0;
  bool any_rank = false;
  for (auto& kv : E.snap.types) any_rank = any_rank || kv.second.rank;
  const uint64_t me_key = device_key(E.cfg.device);
  const uint64_t w1[5] = {E.snap.nv, E.snap.types.size(), any_rank ? 1ull : 0ull, hidden, me_key};
  std::vector<uint64_t> g1;
  if (cm->gather_u64(st, w1, 5, &g1)) return xfail("sizes");
  std::vector<uint64_t> vcount(G);
  uint64_t n_all = 0, max_types = 0, hidden_all = 0, coresident = 0;
  any_rank = false;
  for (int q = 0; q < G; ++q) {
    vcount[q] = g1[q * 5];
    n_all += vcount[q];
    max_types = std::max(max_types, g1[q * 5 + 1]);
    any_rank = any_rank || g1[q * 5 + 2];
    hidden_all += g1[q * 5 + 3];
    coresident += g1[q * 5 + 4] == me_key;
  }
  // (every rank decides the same from the same words: no agreement needed to skip)
  if (max_types == 0 || (uint64_t)G * max_types > GATHER_WORDS) return NBG_OK;
  std::vector<int32_t> types;   // union of the ranks' signed types, sorted
  {
    std::vector<uint64_t> mine(max_types, 0), all;
    size_t k = 0;
    for (auto& kv : E.snap.types) mine[k++] = (uint64_t)(uint32_t)kv.first;
    if (cm->gather_u64(st, mine.data(), max_types, &all)) return xfail("type list");
    for (uint64_t x : all)
      if (x && std::find(types.begin(), types.end(), (int32_t)(uint32_t)x) == types.end())
        types.push_back((int32_t)(uint32_t)x);
    std::sort(types.begin(), types.end());
  }
  if ((uint64_t)G * types.size() > GATHER_WORDS) return NBG_OK;
  std::vector<std::vector<uint64_t>> ecount(types.size(), std::vector<uint64_t>(G));
  std::vector<uint64_t> etot(types.size(), 0);
  uint64_t e_max = 0, e_rank_max = 0;
  {
    std::vector<uint64_t> mine(types.size(), 0), all;
    for (size_t k = 0; k < types.size(); ++k) {
      auto it = E.snap.types.find(types[k]);
      mine[k] = it == E.snap.types.end() ? 0 : it->second.num_edges;
    }
    if (cm->gather_u64(st, mine.data(), types.size(), &all)) return xfail("edge counts");
    for (size_t k = 0; k < types.size(); ++k) {
      for (int q = 0; q < G; ++q) {
        ecount[k][q] = all[(size_t)q * types.size() + k];
        etot[k] += ecount[k][q];
        e_rank_max = std::max(e_rank_max, ecount[k][q]);
      }
      e_max = std::max(e_max, etot[k]);
    }
  }
  const uint64_t CHUNK0 = getenv("NBG_REPLICA_CHUNK") ? strtoull(getenv("NBG_REPLICA_CHUNK"), nullptr, 10) : (1ull << 25);
  const uint64_t CHUNK = std::max<uint64_t>(1, std::min<uint64_t>(CHUNK0, e_rank_max));
  size_t free_b = 0, total_b = 0;
  (void)hipMemGetInfo(&free_b, &total_b);
  const uint64_t my_share = free_b / std::max<uint64_t>(coresident, 1);   // ranks sharing this GPU
  int32_t local = NBG_OK;
  if (!path_replica_wanted(E)) local = NBG_E_UNSUPPORTED;
  else if (e_max >= 0xFFFFFFFFull || n_all >= NO_ROW) local = NBG_E_UNSUPPORTED;
  else if ((double)replica_bytes(E, n_all, e_max, types.size(), any_rank, CHUNK) > (double)my_share * replica_fit())
    local = NBG_E_OUT_OF_MEMORY;
  int32_t agreed = NBG_OK;
  if (cm->agree(st, local, &agreed)) return xfail("agreement");
  if (agreed) return NBG_OK;   // no replica on any rank: FIND PATH stays collective

  // ---- 2. every allocation of the build and of the replica engine, then a second agreement: a
  //         rank that cannot allocate makes every rank go without the replica (not an abort)
  Builder B(E);
  const uint64_t N = n_all;   // (checked below: the ranks' dictionaries are disjoint)
  uint64_t* d_cnt = B.get<uint64_t>(G);
  uint64_t* d_base = B.get<uint64_t>(G);
  int64_t* lv = B.get<int64_t>(npad);
  int64_t* gd = B.get<int64_t>((uint64_t)G * npad);
  int64_t* packed = B.get<int64_t>(n_all);
  int64_t* D = B.keep<int64_t>(N);
  uint32_t* dups = B.get<uint32_t>(1);
  uint32_t* g2d = B.get<uint32_t>((uint64_t)G * npad);
  uint32_t* ldeg = B.get<uint32_t>(npad);
  uint32_t* gdeg = B.get<uint32_t>((uint64_t)G * npad);
  uint32_t* goff = B.get<uint32_t>((uint64_t)G * npad);
  uint32_t* ddeg = B.get<uint32_t>(N + 1);
  uint64_t* d_ecnt = B.get<uint64_t>(G);
  uint32_t* s_col = B.get<uint32_t>(CHUNK);
  uint32_t* r_col = B.get<uint32_t>((uint64_t)G * CHUNK);
  int64_t* s_dst = B.get<int64_t>(CHUNK);
  int64_t* r_dst = B.get<int64_t>((uint64_t)G * CHUNK);
  int64_t* s_rank = any_rank ? B.get<int64_t>(CHUNK) : nullptr;
  int64_t* r_rank = any_rank ? B.get<int64_t>((uint64_t)G * CHUNK) : nullptr;
  uint8_t* lvis = hidden_all ? B.get<uint8_t>(npad) : nullptr;
  uint8_t* gvis = hidden_all ? B.get<uint8_t>((uint64_t)G * npad) : nullptr;
  uint8_t* rvis = hidden_all ? B.keep<uint8_t>(N) : nullptr;
  size_t sort_bytes = 0, scan_bytes = 0, b2 = 0;
  (void)rocprim::radix_sort_keys(nullptr, sort_bytes, packed, D, n_all, 0, 64, st);
  (void)rocprim::exclusive_scan(nullptr, scan_bytes, ldeg, goff, 0u, npad, rocprim::plus<uint32_t>(), st);
  (void)rocprim::exclusive_scan(nullptr, b2, ddeg, ddeg, 0u, N + 1, rocprim::plus<uint32_t>(), st);
  scan_bytes = std::max(scan_bytes, b2);
  void* sort_tmp = B.get<uint8_t>(sort_bytes);
  void* scan_tmp = B.get<uint8_t>(scan_bytes);
  std::vector<DevEdgeType> dts(types.size());
  for (size_t k = 0; k < types.size(); ++k) {
    dts[k].type = types[k];
    dts[k].num_edges = etot[k];
    dts[k].row_ptr = B.keep<uint32_t>(N + 1);
    dts[k].col = B.keep<uint32_t>(etot[k]);
    dts[k].dst_vid = B.keep<int64_t>(etot[k]);
    if (any_rank) dts[k].rank = B.keep<int64_t>(etot[k]);
  }
  auto R = std::make_unique<Engine>();
  R->cfg = E.cfg;
  R->cfg.num_gpus = 1;
  R->cfg.rank = 0;
  std::string werr;
  if (!B.oom && hipStreamCreateWithFlags(&R->stream, hipStreamNonBlocking) != hipSuccess) {
    R->stream = nullptr;
    B.oom = true;
    B.err = "replica stream";
  }
  if (!B.oom && !(R->ws = ws_create(N + 1024, N, e_max, R->stream, &werr))) {
    B.oom = true;
    B.err = "replica workspace: " + werr;
  }
  auto drop_engine = [&]() {
    if (R->ws) ws_destroy(R->ws);
    R->ws = nullptr;
    if (R->stream) (void)hipStreamDestroy(R->stream);
    R->stream = nullptr;
  };
  if (cm->agree(st, B.oom ? NBG_E_OUT_OF_MEMORY : NBG_OK, &agreed)) {
    drop_engine();
    return xfail("allocation agreement");
  }
  if (agreed) {   // some rank could not hold it: every rank goes without (B frees the arrays)
    drop_engine();
    return NBG_OK;
  }

  // ---- 3. the build: from here on only a device or transport error fails, and it aborts the
  //         communicator (every rank reaches the same collectives)
  auto bail = [&](hipError_t e) {
    drop_engine();
    cm->abort();
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
  auto scan = [&](const uint32_t* in, uint32_t* out, uint64_t n) {
    size_t bytes = scan_bytes;
    return rocprim::exclusive_scan(scan_tmp, bytes, in, out, 0u, n, rocprim::plus<uint32_t>(), st);
  };
  // 3a. global dictionary
  std::vector<uint64_t> base(G, 0);
  for (int q = 1; q < G; ++q) base[q] = base[q - 1] + vcount[q - 1];
  RB_TRY(hipMemcpyAsync(d_cnt, vcount.data(), G * 8, hipMemcpyHostToDevice, st));
  RB_TRY(hipMemcpyAsync(d_base, base.data(), G * 8, hipMemcpyHostToDevice, st));
  RB_TRY(hipMemsetAsync(lv, 0, npad * 8, st));
  if (E.snap.nv) RB_TRY(hipMemcpyAsync(lv, E.snap.d_vids, E.snap.nv * 8, hipMemcpyDeviceToDevice, st));
  RB_TRY(B.gather(lv, gd, npad * 8));
  hipLaunchKernelGGL(k_rp_pack, dim3(rgrid((uint64_t)G * npad)), dim3(RB), 0, st, gd, npad, G, d_cnt, d_base, packed);
  RB_TRY(hipGetLastError());
  {
    size_t bytes = sort_bytes;
    RB_TRY(rocprim::radix_sort_keys(sort_tmp, bytes, packed, D, n_all, 0, 64, st));
  }
  RB_TRY(hipMemsetAsync(dups, 0, 4, st));
  hipLaunchKernelGGL(k_rp_dups, dim3(rgrid(N)), dim3(RB), 0, st, D, N, dups);
  RB_TRY(hipGetLastError());
  uint32_t h_dups = 0;
  RB_TRY(hipMemcpyAsync(&h_dups, dups, 4, hipMemcpyDeviceToHost, st));
  RB_TRY(hipStreamSynchronize(st));
  if (h_dups) {   // a vid held by two ranks: every rank sees the same gathered data, so all stop here
    drop_engine();
    return NBG_OK;
  }
  hipLaunchKernelGGL(k_rp_g2d, dim3(rgrid((uint64_t)G * npad)), dim3(RB), 0, st, gd, npad, G, d_cnt, D, N, g2d);
  RB_TRY(hipGetLastError());
  Snapshot& rs = R->snap;
  rs.nv = N;
  rs.d_vids = D;
  rs.h_vids.resize(N);
  RB_TRY(hipMemcpyAsync(rs.h_vids.data(), D, N * 8, hipMemcpyDeviceToHost, st));
  // 3b. per signed type
  for (size_t k = 0; k < types.size(); ++k) {
    const int32_t t = types[k];
    auto it = E.snap.types.find(t);
    const DevEdgeType* lt = it == E.snap.types.end() ? nullptr : &it->second;
    DevEdgeType& dt = dts[k];
    hipLaunchKernelGGL(k_rp_deg, dim3(rgrid(npad)), dim3(RB), 0, st, lt ? lt->row_ptr : nullptr, E.snap.nv, npad, ldeg);
    RB_TRY(hipGetLastError());
    RB_TRY(B.gather(ldeg, gdeg, npad * 4));
    for (int q = 0; q < G; ++q) RB_TRY(scan(gdeg + (uint64_t)q * npad, goff + (uint64_t)q * npad, npad));
    RB_TRY(hipMemsetAsync(ddeg, 0, (N + 1) * 4, st));
    hipLaunchKernelGGL(k_rp_scatter_deg, dim3(rgrid((uint64_t)G * npad)), dim3(RB), 0, st, gdeg, g2d,
                       (uint64_t)G * npad, ddeg);
    RB_TRY(hipGetLastError());
    RB_TRY(scan(ddeg, dt.row_ptr, N + 1));   // row_ptr[N] = the total (ddeg[N] == 0)
    RB_TRY(hipMemcpyAsync(d_ecnt, ecount[k].data(), G * 8, hipMemcpyHostToDevice, st));
    uint64_t emax = 0;
    for (uint64_t c : ecount[k]) emax = std::max(emax, c);
    const uint64_t mine = lt ? lt->num_edges : 0;
    for (uint64_t k0 = 0; k0 < emax; k0 += CHUNK) {
      const uint64_t n = k0 < mine ? std::min<uint64_t>(CHUNK, mine - k0) : 0;
      if (n) {
        RB_TRY(hipMemcpyAsync(s_col, lt->col + k0, n * 4, hipMemcpyDeviceToDevice, st));
        RB_TRY(hipMemcpyAsync(s_dst, lt->dst_vid + k0, n * 8, hipMemcpyDeviceToDevice, st));
        if (any_rank) {
          if (lt->rank) RB_TRY(hipMemcpyAsync(s_rank, lt->rank + k0, n * 8, hipMemcpyDeviceToDevice, st));
          else RB_TRY(hipMemsetAsync(s_rank, 0, n * 8, st));
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
      hipLaunchKernelGGL(k_rp_place, dim3(rgrid((uint64_t)G * CHUNK)), dim3(RB), 0, st, a);
      RB_TRY(hipGetLastError());
    }
    dt.h_row_ptr.resize(N + 1);
    RB_TRY(hipMemcpyAsync(dt.h_row_ptr.data(), dt.row_ptr, (N + 1) * 4, hipMemcpyDeviceToHost, st));
    RB_TRY(hipStreamSynchronize(st));
    uint32_t md = 0;
    for (uint64_t v = 0; v < N; ++v) md = std::max(md, dt.h_row_ptr[v + 1] - dt.h_row_ptr[v]);
    dt.max_degree = (int)md;
    rs.device_bytes += (N + 1) * 4 + etot[k] * (12 + (any_rank ? 8 : 0));
  }
  // 3c. visibility
  if (hidden_all) {
    hipLaunchKernelGGL(k_rp_vis_local, dim3(rgrid(npad)), dim3(RB), 0, st, E.snap.d_visible, E.snap.nv, npad, lvis);
    RB_TRY(hipGetLastError());
    RB_TRY(B.gather(lvis, gvis, npad));
    rs.d_visible = rvis;
    hipLaunchKernelGGL(k_rp_vis, dim3(rgrid((uint64_t)G * npad)), dim3(RB), 0, st, gvis, g2d, (uint64_t)G * npad, rvis);
    RB_TRY(hipGetLastError());
    rs.h_visible.resize(N);
    RB_TRY(hipMemcpyAsync(rs.h_visible.data(), rvis, N, hipMemcpyDeviceToHost, st));
  }
  RB_TRY(hipStreamSynchronize(st));
#undef RB_TRY
  for (size_t k = 0; k < types.size(); ++k) rs.types[types[k]] = std::move(dts[k]);
  B.kept.clear();   // the snapshot holds them now
  rs.device_bytes += N * 9;
  // ---- the replica engine: a single-GPU engine over the replica snapshot (no props, no tags);
  //      its workspace was made in step 2 (engine_ready's only step for a single engine)
  R->edges = E.edges;
  R->tags = E.tags;
  R->prof_mode = E.prof_mode;
  R->finalized = true;
  R->err_parent = &E;
  E.rep = std::move(R);
  return NBG_OK;
}

}  // namespace nbg
