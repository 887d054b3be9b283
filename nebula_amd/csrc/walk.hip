// FIND ALL PATH on the device (split from kernels.hip): the forward walk enumeration with
// backward-distance pruning, single engine and partitioned.
#include <hip/hip_runtime.h>
#include <cstring>
#include <vector>

#include "ws.h"

// ============================================================================= FIND ALL PATH
// FindPathExecutor with ALL returns every walk of 1..N hops from a source to a target over the
// OVER types, cycles included, each once (its odd/even meets decompose a walk uniquely,
// FindPathExecutor.cpp:218-411).  The device enumerates the walks forward, level by level, and
// prunes with the backward BFS distance to the targets (LAB label, computed by path.cpp): a walk
// of i hops is extended to d only if dist(d) <= N - i - 1, so every stored walk completes and the
// work is proportional to the output.  Level l holds, per walk, its last vertex, its parent walk
// in level l - 1, the edge (CSR index, OVER position); a walk ending on a target is also listed as
// a completion.  Each level is a count pass then a fill pass (exact allocation).
namespace nbg {
namespace {
constexpr int WALK_MAX = 32;   // UPTO bound of FIND ALL PATH on the device

struct WalkArgs {
  int ntypes;
  const uint32_t* row_ptr[MAX_TYPES_Q];
  const uint32_t* col[MAX_TYPES_Q];
  const uint8_t* visible;
  const uint32_t* lab;
  uint32_t epoch;
  uint32_t budget;                 // largest admissible distance to a target for the next vertex
  const uint32_t* vtx;             // level i: last vertex per walk
  uint64_t n;
  int fill;
  uint32_t* nvtx;                  // level i + 1 (fill pass)
  uint32_t* npar;
  uint32_t* neid;
  uint8_t* ntix;
  uint32_t* comp;                  // completions of level i + 1 (walk index)
  unsigned long long* cnt;         // [0] walks, [1] completions, [2] adjacency entries scanned
};

// One WAVE per walk: the lanes stride the last vertex's adjacency (coalesced `col` reads, 64
// label probes in flight), and the fill pass places a wave's admissible extensions with one
// atomic per 64 neighbours (ballot prefix).  A hub's adjacency is therefore 1/64 of the serial
// chain it was with a thread per walk.  Walk order inside a level is irrelevant (paths are
// sorted at the end), but the count and fill passes test the same predicate.
__global__ void __launch_bounds__(BLOCK) k_walk(WalkArgs a) {
  unsigned long long nw = 0, nc = 0, ns = 0;
  const int lane = threadIdx.x & 63;
  const unsigned long long lt = (1ull << lane) - 1ull;
  const uint64_t wave0 = ((uint64_t)blockIdx.x * BLOCK + threadIdx.x) >> 6;
  const uint64_t nwaves = ((uint64_t)gridDim.x * BLOCK) >> 6;
  for (uint64_t w = wave0; w < a.n; w += nwaves) {
    const uint32_t v = a.vtx[w];
    if (a.visible && !a.visible[v]) continue;
    for (int t = 0; t < a.ntypes; ++t) {
      const uint32_t b = a.row_ptr[t][v], e = a.row_ptr[t][v + 1];
      if (lane == 0) ns += e - b;
      for (uint32_t j0 = b; j0 < e; j0 += 64) {
        const uint32_t j = j0 + (uint32_t)lane;
        uint32_t d = NO_ROW;
        bool ok = false, done = false;
        if (j < e) {
          d = a.col[t][j];
          if (d != NO_ROW) {
            const uint32_t lb = a.lab[d];
            ok = (lb >> LVL_BITS) == a.epoch && (lb & MAX_PATH_LEN) <= a.budget;
            done = ok && (lb & MAX_PATH_LEN) == 0;
          }
        }
        if (!a.fill) {
          nw += ok;
          nc += done;
          continue;
        }
        const unsigned long long ob = __ballot(ok);
        if (!ob) continue;
        unsigned long long base = 0;
        if (lane == 0) base = atomicAdd(&a.cnt[0], (unsigned long long)__popcll(ob));
        base = __shfl(base, 0, 64);
        const unsigned long long pos = base + (unsigned long long)__popcll(ob & lt);
        if (ok) {
          a.nvtx[pos] = d;
          a.npar[pos] = (uint32_t)w;
          a.neid[pos] = j;
          a.ntix[pos] = (uint8_t)t;
        }
        const unsigned long long cb = __ballot(done);
        if (cb) {
          unsigned long long cbase = 0;
          if (lane == 0) cbase = atomicAdd(&a.cnt[1], (unsigned long long)__popcll(cb));
          cbase = __shfl(cbase, 0, 64);
          if (done) a.comp[cbase + (unsigned long long)__popcll(cb & lt)] = (uint32_t)pos;
        }
      }
    }
  }
  if (!a.fill) {
    for (int o = 32; o; o >>= 1) {
      nw += __shfl_xor(nw, o, 64);
      nc += __shfl_xor(nc, o, 64);
      ns += __shfl_xor(ns, o, 64);
    }
    if (lane == 0 && (nw | nc | ns)) {
      atomicAdd(&a.cnt[0], nw);
      atomicAdd(&a.cnt[1], nc);
      atomicAdd(&a.cnt[2], ns);
    }
  }
}

struct WalkLevels {
  const uint32_t* vtx[WALK_MAX + 1];
  const uint32_t* par[WALK_MAX + 1];
  const uint32_t* eid[WALK_MAX + 1];
  const uint8_t* tix[WALK_MAX + 1];
};
struct WalkTypes {
  const int64_t* rank[MAX_TYPES_Q];
  int32_t type[MAX_TYPES_Q];
};

// entry list [v0, t0, r0, v1, ..., vL] of every completion of level L
__global__ void __launch_bounds__(BLOCK) k_walk_emit(WalkLevels lv, WalkTypes wt, const uint32_t* __restrict__ comp,
                                                     uint64_t ncomp, int L, const int64_t* __restrict__ vids,
                                                     int64_t* __restrict__ out) {
  for (uint64_t c = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; c < ncomp; c += (uint64_t)gridDim.x * BLOCK) {
    uint32_t k = comp[c];
    int64_t* o = out + c * (uint64_t)(1 + 3 * L);
    for (int l = L; l >= 1; --l) {
      const int t = lv.tix[l][k];
      o[3 * l] = vids[lv.vtx[l][k]];
      o[3 * l - 2] = wt.type[t];
      o[3 * l - 1] = wt.rank[t] ? wt.rank[t][lv.eid[l][k]] : 0;
      k = lv.par[l][k];
    }
    o[0] = vids[lv.vtx[0][k]];
  }
}
}  // namespace

// Bump allocation from the workspace's walk arena (kept across queries, grown by doubling; an
// outgrown arena stays alive until the query's release(), earlier levels still live in it).
namespace {
struct WalkArena {
  Workspace* w;
  std::vector<void*> owned;
  size_t used = 0;
  explicit WalkArena(Workspace* ws) : w(ws) {}
  void release() {
    (void)ws_sync(w);
    for (void* p : owned) (void)hipFree(p);
    owned.clear();
  }
  hipError_t get(void** p, size_t b) {
    b = ((b ? b : 1) + 255) & ~(size_t)255;   // 256-byte aligned, never empty
    if (used + b > w->walk_cap || !w->walk_arena) {
      if (w->walk_arena) owned.push_back(w->walk_arena);
      size_t cap = w->walk_cap ? w->walk_cap : ((size_t)1 << 24);
      while (cap < b) cap *= 2;
      cap *= 2;
      w->walk_arena = nullptr;
      w->walk_cap = 0;
      hipError_t e = hipMalloc((void**)&w->walk_arena, cap);
      if (e != hipSuccess) return e;
      w->walk_cap = cap;
      used = 0;
    }
    *p = w->walk_arena + used;
    used += b;
    return hipSuccess;
  }
};
}  // namespace

hipError_t ws_all_paths(Workspace* w, const PathTypes& fwd, int lab, uint32_t epoch, const uint32_t* S, uint64_t nS,
                        uint32_t upto, const int64_t* d_vids, const uint8_t* visible, uint64_t max_walks,
                        std::vector<std::vector<int64_t>>* out, uint64_t* scanned) {
  if (upto > (uint32_t)WALK_MAX || fwd.n > MAX_TYPES_Q) return hipErrorInvalidValue;
  WalkArena arena(w);
  auto cleanup = [&]() { arena.release(); };
  auto alloc = [&](void** p, size_t b) { return arena.get(p, b); };
#define WALK_TRY(x)                      \
  do {                                   \
    hipError_t e_ = (x);                 \
    if (e_ != hipSuccess) {              \
      cleanup();                         \
      return e_;                         \
    }                                    \
  } while (0)
  WalkLevels lv{};
  std::vector<uint64_t> nlev(upto + 1, 0), ncomp(upto + 1, 0);
  std::vector<uint32_t*> comp(upto + 1, nullptr);
  uint32_t* v0 = nullptr;
  WALK_TRY(alloc((void**)&v0, nS * 4));
  WALK_TRY(hipMemcpy(v0, S, nS * 4, hipMemcpyHostToDevice));
  lv.vtx[0] = v0;
  nlev[0] = nS;
  unsigned long long* cnt = nullptr;
  WALK_TRY(alloc((void**)&cnt, 3 * 8));
  unsigned long long h[3];
  uint64_t total = nS;
  *scanned = 0;
  WalkArgs a{};
  a.ntypes = fwd.n;
  for (int t = 0; t < fwd.n; ++t) {
    a.row_ptr[t] = fwd.a[t].row_ptr;
    a.col[t] = fwd.a[t].col;
  }
  a.visible = visible;
  a.cnt = cnt;
  a.lab = w->lab[lab];
  a.epoch = epoch;
  uint32_t L = 0;
  for (uint32_t i = 0; i < upto && nlev[i]; ++i) {
    a.budget = upto - i - 1;
    a.vtx = lv.vtx[i];
    a.n = nlev[i];
    const unsigned grid = (unsigned)std::min<uint64_t>(cdiv(a.n, WAVES), 8192);   // a wave per walk
    a.fill = 0;
    WALK_TRY(hipMemsetAsync(cnt, 0, 3 * 8, w->stream));
    hipLaunchKernelGGL(k_walk, dim3(grid), dim3(BLOCK), 0, w->stream, a);
    WALK_TRY(hipGetLastError());
    WALK_TRY(hipMemcpyAsync(h, cnt, sizeof(h), hipMemcpyDeviceToHost, w->stream));
    WALK_TRY(ws_sync(w));
    *scanned += h[2];
    if (!h[0]) break;
    total += h[0];
    if (total > max_walks || h[0] >= 0xFFFFFFFFull) {
      cleanup();
      return hipErrorOutOfMemory;   // reported as "too many paths"
    }
    uint32_t *nv, *np, *ne, *cp;
    uint8_t* nt;
    WALK_TRY(alloc((void**)&nv, h[0] * 4));
    WALK_TRY(alloc((void**)&np, h[0] * 4));
    WALK_TRY(alloc((void**)&ne, h[0] * 4));
    WALK_TRY(alloc((void**)&nt, h[0]));
    WALK_TRY(alloc((void**)&cp, h[1] * 4));
    a.fill = 1;
    a.nvtx = nv;
    a.npar = np;
    a.neid = ne;
    a.ntix = nt;
    a.comp = cp;
    a.cnt = cnt;
    WALK_TRY(hipMemsetAsync(cnt, 0, 3 * 8, w->stream));
    hipLaunchKernelGGL(k_walk, dim3(grid), dim3(BLOCK), 0, w->stream, a);
    WALK_TRY(hipGetLastError());
    lv.vtx[i + 1] = nv;
    lv.par[i + 1] = np;
    lv.eid[i + 1] = ne;
    lv.tix[i + 1] = nt;
    comp[i + 1] = cp;
    nlev[i + 1] = h[0];
    ncomp[i + 1] = h[1];
    L = i + 1;
  }
  WalkTypes wt{};
  for (int t = 0; t < fwd.n; ++t) {
    wt.rank[t] = fwd.a[t].rank;
    wt.type[t] = fwd.type[t];
  }
  for (uint32_t l = 1; l <= L; ++l) {
    if (!ncomp[l]) continue;
    const uint64_t width = 1 + 3 * (uint64_t)l;
    int64_t* o = nullptr;
    WALK_TRY(alloc((void**)&o, ncomp[l] * width * 8));
    hipLaunchKernelGGL(k_walk_emit, dim3((unsigned)std::min<uint64_t>(cdiv(ncomp[l], BLOCK), 4096)), dim3(BLOCK), 0,
                       w->stream, lv, wt, comp[l], ncomp[l], (int)l, d_vids, o);
    WALK_TRY(hipGetLastError());
    std::vector<int64_t> host(ncomp[l] * width);
    WALK_TRY(hipMemcpyAsync(host.data(), o, host.size() * 8, hipMemcpyDeviceToHost, w->stream));
    WALK_TRY(ws_sync(w));
    for (uint64_t c = 0; c < ncomp[l]; ++c)
      out->emplace_back(host.begin() + (ptrdiff_t)(c * width), host.begin() + (ptrdiff_t)((c + 1) * width));
  }
#undef WALK_TRY
  cleanup();
  return hipSuccess;
}

// ----------------------------------------------------------------------------- FIND ALL PATH, partitioned
// The reference extends every path list through the storaged hosts that own the frontier's parts
// (FindPathExecutor::getFromFrontiers / getToFrontiers, FindPathExecutor.cpp:441-530, then
// findPath :218-290).  Here a walk is extended by the rank that owns its last vertex (only it
// holds that vertex's out-edges), and every level is REPLICATED: each rank appends the walks it
// extended to its own block of the next level, one all-gather makes the level whole on every rank.
// A walk record carries what the entry list needs (the neighbour's global id and vid, the edge's
// OVER position and rank), so the ranks emit identical path lists without another exchange.  The
// pruning distances (backward BFS levels, labelled at each vertex's owner) are all-gathered once as
// one byte per global id.
namespace {
struct WalkRec {        // 32 bytes; gid == NO_ROW: an unused slot of a rank's block
  uint32_t gid;         // last vertex (global id)
  uint32_t par;         // parent walk in the previous level
  int32_t tix;          // OVER position of the last edge
  uint32_t pad;
  int64_t rnk;          // the last edge's rank
  int64_t vid;          // the last vertex's vid
};
static_assert(sizeof(WalkRec) == 32, "walk record layout");

struct WalkPartArgs {
  int ntypes;
  const uint32_t* row_ptr[MAX_TYPES_Q];
  const uint32_t* col[MAX_TYPES_Q];
  const int64_t* dst_vid[MAX_TYPES_Q];
  const int64_t* rank[MAX_TYPES_Q];
  const uint8_t* visible;
  const uint8_t* gdist;            // [G * npad] distance to a target, 0xFF = none within reach
  uint32_t budget;
  uint32_t gbase, npad;            // this rank's global id range [gbase, gbase + npad)
  const WalkRec* lv;               // level i (every rank's blocks)
  uint64_t n;
  int fill;
  WalkRec* out;                    // this rank's block of level i + 1 (fill pass)
  unsigned long long* cnt;         // [0] walks, [1] completions, [2] adjacency entries scanned
};

// distance byte per local vertex (the rank's npad block of the global id space)
__global__ void __launch_bounds__(BLOCK) k_walk_dist(const uint32_t* __restrict__ lab, uint32_t epoch, uint64_t nv,
                                                     uint64_t npad, uint8_t* __restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < npad; i += (uint64_t)gridDim.x * BLOCK) {
    uint8_t d = 0xFF;
    if (i < nv) {
      const uint32_t lb = lab[i];
      if ((lb >> LVL_BITS) == epoch) d = (uint8_t)(lb & MAX_PATH_LEN);
    }
    out[i] = d;
  }
}

// k_walk over the rank's own walks of a replicated level (a wave per walk, as k_walk)
__global__ void __launch_bounds__(BLOCK) k_walk_part(WalkPartArgs a) {
  unsigned long long nw = 0, nc = 0, ns = 0;
  const int lane = threadIdx.x & 63;
  const unsigned long long lt = (1ull << lane) - 1ull;
  const uint64_t wave0 = ((uint64_t)blockIdx.x * BLOCK + threadIdx.x) >> 6;
  const uint64_t nwaves = ((uint64_t)gridDim.x * BLOCK) >> 6;
  for (uint64_t w = wave0; w < a.n; w += nwaves) {
    const uint32_t g = a.lv[w].gid;
    const uint32_t v = g - a.gbase;   // unsigned: another rank's vertex (or NO_ROW) is >= npad
    if (g == NO_ROW || v >= a.npad) continue;
    if (a.visible && !a.visible[v]) continue;
    for (int t = 0; t < a.ntypes; ++t) {
      const uint32_t b = a.row_ptr[t][v], e = a.row_ptr[t][v + 1];
      if (lane == 0) ns += e - b;
      for (uint32_t j0 = b; j0 < e; j0 += 64) {
        const uint32_t j = j0 + (uint32_t)lane;
        uint32_t d = NO_ROW;
        bool ok = false, done = false;
        if (j < e) {
          d = a.col[t][j];
          if (d != NO_ROW) {
            const uint32_t dist = a.gdist[d];
            ok = dist <= a.budget;
            done = ok && dist == 0;
          }
        }
        if (!a.fill) {
          nw += ok;
          nc += done;
          continue;
        }
        const unsigned long long ob = __ballot(ok);
        if (!ob) continue;
        unsigned long long base = 0;
        if (lane == 0) base = atomicAdd(&a.cnt[0], (unsigned long long)__popcll(ob));
        base = __shfl(base, 0, 64);
        if (ok) {
          WalkRec r;
          r.gid = d;
          r.par = (uint32_t)w;
          r.tix = t;
          r.pad = 0;
          r.rnk = a.rank[t] ? a.rank[t][j] : 0;
          r.vid = a.dst_vid[t][j];
          a.out[base + (unsigned long long)__popcll(ob & lt)] = r;
        }
      }
    }
  }
  if (!a.fill) {
    for (int o = 32; o; o >>= 1) {
      nw += __shfl_xor(nw, o, 64);
      nc += __shfl_xor(nc, o, 64);
      ns += __shfl_xor(ns, o, 64);
    }
    if (lane == 0 && (nw | nc | ns)) {
      atomicAdd(&a.cnt[0], nw);
      atomicAdd(&a.cnt[1], nc);
      atomicAdd(&a.cnt[2], ns);
    }
  }
}

struct WalkPartLevels {
  const WalkRec* lv[WALK_MAX + 1];
};

// entry list [v0, t0, r0, v1, ..., vL] of every level-L walk that ends on a target
__global__ void __launch_bounds__(BLOCK) k_walk_emit_part(WalkPartLevels lv, WalkTypes wt, uint64_t n, int L,
                                                          const uint8_t* __restrict__ gdist,
                                                          unsigned long long* __restrict__ cnt,
                                                          int64_t* __restrict__ out) {
  for (uint64_t c = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; c < n; c += (uint64_t)gridDim.x * BLOCK) {
    WalkRec r = lv.lv[L][c];
    if (r.gid == NO_ROW || gdist[r.gid] != 0) continue;
    const unsigned long long pos = atomicAdd(cnt, 1ull);
    int64_t* o = out + pos * (uint64_t)(1 + 3 * L);
    for (int l = L; l >= 1; --l) {
      o[3 * l] = r.vid;
      o[3 * l - 2] = wt.type[r.tix];
      o[3 * l - 1] = r.rnk;
      r = lv.lv[l - 1][r.par];
    }
    o[0] = r.vid;
  }
}
}  // namespace

hipError_t ws_all_paths_part(Workspace* w, const PathTypes& fwd, int lab, uint32_t epoch, const uint32_t* Sgid,
                             const int64_t* Svid, uint64_t nS, uint32_t upto, uint64_t nv, const uint8_t* visible,
                             uint64_t max_walks, std::vector<std::vector<int64_t>>* out, uint64_t* scanned) {
  if (!w->comm || upto > (uint32_t)WALK_MAX || fwd.n > MAX_TYPES_Q) return hipErrorInvalidValue;
  const int G = w->comm->world;
  const uint64_t npad = w->npad;
  WalkArena arena(w);
#define WALK_TRY(x)                      \
  do {                                   \
    hipError_t e_ = (x);                 \
    if (e_ != hipSuccess) {              \
      arena.release();                   \
      return e_;                         \
    }                                    \
  } while (0)
#define WALK_COMM(x)                     \
  do {                                   \
    if (x) {                             \
      arena.release();                   \
      return hipErrorUnknown;            \
    }                                    \
  } while (0)
  // pruning distances over the global id space
  uint8_t *dloc = nullptr, *gdist = nullptr;
  WALK_TRY(arena.get((void**)&dloc, npad));
  WALK_TRY(arena.get((void**)&gdist, (size_t)G * npad));
  hipLaunchKernelGGL(k_walk_dist, dim3((unsigned)std::min<uint64_t>(cdiv(npad, BLOCK), 4096)), dim3(BLOCK), 0,
                     w->stream, w->lab[lab], epoch, nv, npad, dloc);
  WALK_TRY(hipGetLastError());
  WALK_COMM(w->comm->allgather(dloc, gdist, npad, w->stream));
  // level 0: the sources, replicated
  std::vector<WalkRec> h0(nS);
  for (uint64_t i = 0; i < nS; ++i) h0[i] = WalkRec{Sgid[i], 0, 0, 0, 0, Svid[i]};
  WalkPartLevels lv{};
  std::vector<uint64_t> nlev(upto + 1, 0), ncomp(upto + 1, 0);
  WalkRec* l0 = nullptr;
  WALK_TRY(arena.get((void**)&l0, nS * sizeof(WalkRec)));
  WALK_TRY(hipMemcpyAsync(l0, h0.data(), nS * sizeof(WalkRec), hipMemcpyHostToDevice, w->stream));
  lv.lv[0] = l0;
  nlev[0] = nS;
  unsigned long long *cnt = nullptr, *all = nullptr;
  WALK_TRY(arena.get((void**)&cnt, 3 * 8));
  WALK_TRY(arena.get((void**)&all, (size_t)G * 3 * 8));
  std::vector<unsigned long long> h(3 * (size_t)G);
  uint64_t total = nS;
  *scanned = 0;
  WalkPartArgs a{};
  a.ntypes = fwd.n;
  for (int t = 0; t < fwd.n; ++t) {
    a.row_ptr[t] = fwd.a[t].row_ptr;
    a.col[t] = fwd.a[t].col;
    a.dst_vid[t] = fwd.a[t].dst_vid;
    a.rank[t] = fwd.a[t].rank;
  }
  a.visible = visible;
  a.gdist = gdist;
  a.gbase = (uint32_t)(w->comm->rank * npad);
  a.npad = (uint32_t)npad;
  a.cnt = cnt;
  uint32_t L = 0;
  for (uint32_t i = 0; i < upto && nlev[i]; ++i) {
    a.budget = upto - i - 1;
    a.lv = lv.lv[i];
    a.n = nlev[i];
    const unsigned grid = (unsigned)std::min<uint64_t>(cdiv(a.n, WAVES), 8192);
    a.fill = 0;
    WALK_TRY(hipMemsetAsync(cnt, 0, 3 * 8, w->stream));
    hipLaunchKernelGGL(k_walk_part, dim3(grid), dim3(BLOCK), 0, w->stream, a);
    WALK_TRY(hipGetLastError());
    WALK_COMM(w->comm->allgather(cnt, all, 3 * 8, w->stream));
    WALK_TRY(hipMemcpyAsync(h.data(), all, h.size() * 8, hipMemcpyDeviceToHost, w->stream));
    WALK_TRY(ws_sync(w));
    uint64_t walks = 0, comps = 0, maxc = 0;
    for (int q = 0; q < G; ++q) {
      walks += h[3 * q];
      comps += h[3 * q + 1];
      *scanned += h[3 * q + 2];
      maxc = std::max<uint64_t>(maxc, h[3 * q]);
    }
    if (!walks) break;   // the same on every rank (summed counts)
    total += walks;
    if (total > max_walks || (uint64_t)G * maxc >= 0xFFFFFFFFull) {
      arena.release();
      return hipErrorOutOfMemory;   // reported as "too many paths"
    }
    WalkRec *mine = nullptr, *lvl = nullptr;
    WALK_TRY(arena.get((void**)&mine, maxc * sizeof(WalkRec)));
    WALK_TRY(arena.get((void**)&lvl, (size_t)G * maxc * sizeof(WalkRec)));
    WALK_TRY(hipMemsetAsync(mine, 0xFF, maxc * sizeof(WalkRec), w->stream));   // unused slots: gid NO_ROW
    a.fill = 1;
    a.out = mine;
    WALK_TRY(hipMemsetAsync(cnt, 0, 3 * 8, w->stream));
    hipLaunchKernelGGL(k_walk_part, dim3(grid), dim3(BLOCK), 0, w->stream, a);
    WALK_TRY(hipGetLastError());
    WALK_COMM(w->comm->allgather(mine, lvl, maxc * sizeof(WalkRec), w->stream));
    lv.lv[i + 1] = lvl;
    nlev[i + 1] = (uint64_t)G * maxc;
    ncomp[i + 1] = comps;
    L = i + 1;
  }
  WalkTypes wt{};
  for (int t = 0; t < fwd.n; ++t) wt.type[t] = fwd.type[t];
  for (uint32_t l = 1; l <= L; ++l) {
    if (!ncomp[l]) continue;
    const uint64_t width = 1 + 3 * (uint64_t)l;
    int64_t* o = nullptr;
    WALK_TRY(arena.get((void**)&o, ncomp[l] * width * 8));
    WALK_TRY(hipMemsetAsync(cnt, 0, 8, w->stream));
    hipLaunchKernelGGL(k_walk_emit_part, dim3((unsigned)std::min<uint64_t>(cdiv(nlev[l], BLOCK), 4096)), dim3(BLOCK),
                       0, w->stream, lv, wt, nlev[l], (int)l, gdist, cnt, o);
    WALK_TRY(hipGetLastError());
    std::vector<int64_t> host(ncomp[l] * width);
    WALK_TRY(hipMemcpyAsync(host.data(), o, host.size() * 8, hipMemcpyDeviceToHost, w->stream));
    WALK_TRY(ws_sync(w));
    for (uint64_t c = 0; c < ncomp[l]; ++c)
      out->emplace_back(host.begin() + (ptrdiff_t)(c * width), host.begin() + (ptrdiff_t)((c + 1) * width));
  }
#undef WALK_COMM
#undef WALK_TRY
  arena.release();
  return hipSuccess;
}
}  // namespace nbg
