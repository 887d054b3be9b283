// FIND SHORTEST / ALL PATH under max_edge_returned_per_vertex (gfx950 kernels + host driver).
//
// FindPathExecutor reads both frontiers through getNeighbors (FindPathExecutor.cpp:441-530), so
// storaged caps each (vertex, edge type) at the first K edges in key order
// (QueryBaseProcessor.inl:394-398): the from side walks the first K out-edges of a vertex, the
// to side the first K in-edges (-type) of a vertex.  With a cap the two sides no longer see
// mirror images of one graph, and the reference's semantics become those of its own rounds:
//   * round c expands the from-frontier F_{c-1} over capped out-rows and the to-frontier T_{c-1}
//     over capped in-rows; the frontiers are the SETS of every vertex a walk of exactly c steps
//     reaches (visitedFrom / visitedTo are cleared each round, :229-262), so walks may revisit
//     vertices;
//   * odd meet (:226-236): a from-edge u -> x with x in T_{c-1}, a walk of 2c - 1 edges whose
//     first c edges are capped out-edges and last c - 1 capped in-edges;
//   * even meet (:264-279): F_c ∩ T_c, c out-edges then c in-edges;
//   * a walk of L edges is therefore valid when its first ceil(L/2) edges come from the capped
//     out-rows and the rest from the capped in-rows.
// SHORTEST keeps, per target, the walks of the first round that reaches it (minimum L), and this
// engine returns the lexicographically smallest entry list among them (as for the uncapped
// search, path.cpp).  ALL returns every valid walk of 1..UPTO edges.
//
// Device design (one engine or a partitioned one, the same code):
//   * sets are bitmaps over the global id space (single engine: the dense ids), REPLICATED on
//     every rank: a rank expands the members it owns into a full-width bitmap, one all-to-all
//     hands segment q to rank q, the owner ORs the G segments and one all-gather replicates the
//     result; every decision below reads replicated data, so every rank takes the same branches;
//   * SHORTEST, per target t: F_c (shared by the targets) and T_c from {t}; the first meet fixes L
//     and h = ceil(L/2); B_h = F_h ∩ T_{L-h}; B_i = { u in F_i : a capped out-edge of u enters
//     B_{i+1} } for i < h (a pull over the owned members of F_i); positions past h are T_{L-i};
//     the greedy walks from min vid(B_0): a hop before h takes the minimum (type, rank, vid) of
//     the current vertex's capped out-row into B_{i+1}; a hop after h the minimum over the B_{i+1}
//     members whose capped in-row holds the current vertex; per-rank minima are all-gathered;
//   * ALL: the from-walks (capped out-rows, ceil(N/2) levels) and to-walks (capped in-rows,
//     floor(N/2) levels) are enumerated as replicated walk records (each level extended by the
//     owners of the walks' last vertices and all-gathered, as ws_all_paths_part), and the walks of
//     each length are the hash join of a from-level and a to-level on the meeting vertex, emitted
//     as entry lists on the device.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "nbg_internal.h"

namespace nbg {
namespace {

constexpr int CB = 256;   // block size
constexpr int CAP_LEVELS = 64;

inline uint64_t cdivc(uint64_t a, uint64_t b) { return (a + b - 1) / b; }
inline unsigned gridc(uint64_t n, unsigned cap = 4096) {
  const uint64_t b = cdivc(n ? n : 1, CB);
  return (unsigned)(b < cap ? b : cap);
}

struct CapCsr {                 // the CSRs of one search direction, OVER order
  int n;
  int32_t type[MAX_TYPES_Q];    // signed type (negative: in-edges)
  const uint32_t* row_ptr[MAX_TYPES_Q];
  const uint32_t* col[MAX_TYPES_Q];
  const int64_t* dst_vid[MAX_TYPES_Q];
  const int64_t* rank[MAX_TYPES_Q];
};

struct Cand {                   // one greedy candidate; gid < 0: none
  int64_t type, rank, vid, gid;
};

__device__ __forceinline__ bool cand_less(const Cand& a, const Cand& b) {
  if (a.gid < 0) return false;
  if (b.gid < 0) return true;
  if (a.type != b.type) return a.type < b.type;
  if (a.rank != b.rank) return a.rank < b.rank;
  return a.vid < b.vid;
}

__device__ __forceinline__ bool bit(const unsigned long long* bm, uint32_t g) { return (bm[g >> 6] >> (g & 63)) & 1ull; }

__device__ __forceinline__ uint32_t capped_end(const uint32_t* rp, uint32_t v, uint32_t K, uint32_t* b) {
  *b = rp[v];
  const uint32_t e = rp[v + 1];
  return e - *b > K ? *b + K : e;
}

__device__ void wave_add(unsigned long long* ctr, unsigned long long v) {
  for (int o = 32; o; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0 && v) atomicAdd(ctr, v);
}

// Y |= bits of the capped neighbours of X's members owned here (local ids [0, nv), global id
// gbase + v)
__global__ void __launch_bounds__(CB) k_cap_expand(CapCsr cs, const unsigned long long* __restrict__ X,
                                                   unsigned long long* __restrict__ Y, uint64_t nv, uint32_t gbase,
                                                   uint32_t K, const uint8_t* __restrict__ visible,
                                                   unsigned long long* scanned) {
  unsigned long long ns = 0;
  for (uint64_t v = (uint64_t)blockIdx.x * CB + threadIdx.x; v < nv; v += (uint64_t)gridDim.x * CB) {
    if (!bit(X, gbase + (uint32_t)v) || (visible && !visible[v])) continue;
    for (int t = 0; t < cs.n; ++t) {
      uint32_t b;
      const uint32_t e = capped_end(cs.row_ptr[t], (uint32_t)v, K, &b);
      ns += e - b;
      for (uint32_t j = b; j < e; ++j) {
        const uint32_t d = cs.col[t][j];
        if (d != NO_ROW) atomicOr(Y + (d >> 6), 1ull << (d & 63));
      }
    }
  }
  wave_add(scanned, ns);
}

// out (the rank's segment) = OR of the G received segments
__global__ void __launch_bounds__(CB) k_cap_or(const unsigned long long* __restrict__ recv, int G, uint64_t words,
                                               unsigned long long* __restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * CB + threadIdx.x; i < words; i += (uint64_t)gridDim.x * CB) {
    unsigned long long x = 0;
    for (int q = 0; q < G; ++q) x |= recv[(uint64_t)q * words + i];
    out[i] = x;
  }
}

__global__ void __launch_bounds__(CB) k_cap_and(const unsigned long long* __restrict__ A,
                                                const unsigned long long* __restrict__ B, uint64_t words,
                                                unsigned long long* __restrict__ out, unsigned long long* count) {
  unsigned long long c = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * CB + threadIdx.x; i < words; i += (uint64_t)gridDim.x * CB) {
    const unsigned long long x = A[i] & B[i];
    if (out) out[i] = x;
    c += (unsigned long long)__popcll(x);
  }
  wave_add(count, c);
}

__global__ void k_cap_set(const uint32_t* __restrict__ ids, uint64_t n, unsigned long long* __restrict__ bm) {
  for (uint64_t i = (uint64_t)blockIdx.x * CB + threadIdx.x; i < n; i += (uint64_t)gridDim.x * CB) {
    const uint32_t g = ids[i];
    if (g != NO_ROW) atomicOr(bm + (g >> 6), 1ull << (g & 63));
  }
}

// B_i (the rank's segment, local bit v) = { v in F_i owned here : a capped out-edge of v enters Bn }
__global__ void __launch_bounds__(CB) k_cap_pull(CapCsr cs, const unsigned long long* __restrict__ F,
                                                 const unsigned long long* __restrict__ Bn, uint64_t nv,
                                                 uint32_t gbase, uint32_t K, const uint8_t* __restrict__ visible,
                                                 unsigned long long* __restrict__ seg) {
  for (uint64_t v = (uint64_t)blockIdx.x * CB + threadIdx.x; v < nv; v += (uint64_t)gridDim.x * CB) {
    if (!bit(F, gbase + (uint32_t)v) || (visible && !visible[v])) continue;
    bool hit = false;
    for (int t = 0; t < cs.n && !hit; ++t) {
      uint32_t b;
      const uint32_t e = capped_end(cs.row_ptr[t], (uint32_t)v, K, &b);
      for (uint32_t j = b; j < e && !hit; ++j) {
        const uint32_t d = cs.col[t][j];
        hit = d != NO_ROW && bit(Bn, d);
      }
    }
    if (hit) atomicOr(seg + (v >> 6), 1ull << (v & 63));
  }
}

__device__ void block_min_store(Cand c, Cand* out) {
  __shared__ Cand s[CB];
  s[threadIdx.x] = c;
  __syncthreads();
  for (int o = CB / 2; o; o >>= 1) {
    if ((int)threadIdx.x < o && cand_less(s[threadIdx.x + o], s[threadIdx.x])) s[threadIdx.x] = s[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = s[0];
}

// hop before h: the minimum (type, rank, vid) capped out-edge of local vertex v into Bn (one
// workgroup; v == NO_ROW: another rank owns the vertex, no candidate)
__global__ void __launch_bounds__(CB) k_cap_hop_out(CapCsr cs, uint32_t v, uint32_t K,
                                                    const unsigned long long* __restrict__ Bn, Cand* out) {
  Cand best{0, 0, 0, -1};
  if (v != NO_ROW) {
    for (int t = 0; t < cs.n; ++t) {
      uint32_t b;
      const uint32_t e = capped_end(cs.row_ptr[t], v, K, &b);
      for (uint32_t j = b + threadIdx.x; j < e; j += CB) {
        const uint32_t d = cs.col[t][j];
        if (d == NO_ROW || !bit(Bn, d)) continue;
        Cand c{cs.type[t], cs.rank[t] ? cs.rank[t][j] : 0, cs.dst_vid[t][j], (int64_t)d};
        if (cand_less(c, best)) best = c;
      }
    }
  }
  block_min_store(best, out);
}

// hop after h: over the owned members w of Bn, the capped in-row entries naming the current
// vertex (global id cur): candidate (type, rank, vid(w)); per-workgroup minima into part[]
__global__ void __launch_bounds__(CB) k_cap_hop_in(CapCsr cs, uint32_t cur, uint32_t K,
                                                   const unsigned long long* __restrict__ Bn, uint64_t nv,
                                                   uint32_t gbase, const uint8_t* __restrict__ visible,
                                                   const int64_t* __restrict__ vids, Cand* part) {
  Cand best{0, 0, 0, -1};
  for (uint64_t w = (uint64_t)blockIdx.x * CB + threadIdx.x; w < nv; w += (uint64_t)gridDim.x * CB) {
    if (!bit(Bn, gbase + (uint32_t)w) || (visible && !visible[w])) continue;
    for (int t = 0; t < cs.n; ++t) {
      uint32_t b;
      const uint32_t e = capped_end(cs.row_ptr[t], (uint32_t)w, K, &b);
      for (uint32_t j = b; j < e; ++j) {
        if (cs.col[t][j] != cur) continue;
        Cand c{-(int64_t)cs.type[t], cs.rank[t] ? cs.rank[t][j] : 0, vids[w], (int64_t)(gbase + w)};
        if (cand_less(c, best)) best = c;
      }
    }
  }
  block_min_store(best, part + blockIdx.x);
}

__global__ void __launch_bounds__(CB) k_cap_reduce(const Cand* __restrict__ in, uint64_t n, Cand* out) {
  Cand best{0, 0, 0, -1};
  for (uint64_t i = threadIdx.x; i < n; i += CB)
    if (cand_less(in[i], best)) best = in[i];
  block_min_store(best, out);
}

// B_0 members among the sources: the one with the smallest vid (vid in .vid, gid in .gid)
__global__ void k_cap_pick_source(const unsigned long long* __restrict__ B0, const uint32_t* __restrict__ sg,
                                  const int64_t* __restrict__ sv, uint64_t n, Cand* out) {
  if (threadIdx.x || blockIdx.x) return;
  Cand best{0, 0, 0, -1};
  for (uint64_t i = 0; i < n; ++i)
    if (sg[i] != NO_ROW && bit(B0, sg[i]) && (best.gid < 0 || sv[i] < best.vid)) best = Cand{0, 0, sv[i], sg[i]};
  *out = best;
}

// ---------------------------------------------------------------------------- FIND ALL PATH
struct CRec {        // 32 bytes; gid == NO_ROW: an unused slot of a rank's block
  uint32_t gid;      // last vertex (global id)
  uint32_t par;      // parent walk in the previous level
  int32_t tix;       // OVER position of the last edge
  uint32_t pad;
  int64_t rnk;       // the last edge's rank
  int64_t vid;       // the last vertex's vid
};
static_assert(sizeof(CRec) == 32, "walk record layout");

// extend the owned walks of a replicated level by the last vertex's capped rows (count / fill)
__global__ void __launch_bounds__(CB) k_cap_walk(CapCsr cs, const CRec* __restrict__ lv, uint64_t n, uint64_t nv,
                                                 uint32_t gbase, uint32_t K, const uint8_t* __restrict__ visible,
                                                 int fill, CRec* __restrict__ out, unsigned long long* cnt) {
  unsigned long long nw = 0, ns = 0;
  for (uint64_t w = (uint64_t)blockIdx.x * CB + threadIdx.x; w < n; w += (uint64_t)gridDim.x * CB) {
    const uint32_t g = lv[w].gid;
    const uint32_t v = g - gbase;   // unsigned: another rank's vertex (or NO_ROW) is >= nv
    if (g == NO_ROW || v >= nv || (visible && !visible[v])) continue;
    for (int t = 0; t < cs.n; ++t) {
      uint32_t b;
      const uint32_t e = capped_end(cs.row_ptr[t], v, K, &b);
      ns += e - b;
      for (uint32_t j = b; j < e; ++j) {
        const uint32_t d = cs.col[t][j];
        if (d == NO_ROW) continue;
        if (!fill) {
          ++nw;
          continue;
        }
        const unsigned long long pos = atomicAdd(cnt, 1ull);
        CRec r;
        r.gid = d;
        r.par = (uint32_t)w;
        r.tix = t;
        r.pad = 0;
        r.rnk = cs.rank[t] ? cs.rank[t][j] : 0;
        r.vid = cs.dst_vid[t][j];
        out[pos] = r;
      }
    }
  }
  if (!fill) {
    wave_add(cnt, nw);
    wave_add(cnt + 1, ns);
  }
}

struct CapLevels {
  const CRec* lv[CAP_LEVELS];
};
struct CapTypeVals {
  int64_t type[MAX_TYPES_Q];   // entry-list type of each OVER position (positive)
};

__device__ __forceinline__ uint64_t hslot(uint32_t g, uint64_t mask) {
  uint64_t x = (uint64_t)g * 0x9E3779B97F4A7C15ull;
  return (x >> 32) & mask;
}

// hash table of the to-walks of one level by their last vertex: key[slot] = gid, head[slot] =
// first walk, nxt[walk] = next walk with the same gid
__global__ void __launch_bounds__(CB) k_cap_join_build(const CRec* __restrict__ tw, uint64_t n, uint32_t* key,
                                                       uint32_t* head, uint32_t* nxt, uint64_t mask) {
  for (uint64_t k = (uint64_t)blockIdx.x * CB + threadIdx.x; k < n; k += (uint64_t)gridDim.x * CB) {
    const uint32_t g = tw[k].gid;
    if (g == NO_ROW) continue;
    uint64_t s = hslot(g, mask);
    for (;;) {
      const uint32_t old = atomicCAS(key + s, NO_ROW, g);
      if (old == NO_ROW || old == g) break;
      s = (s + 1) & mask;
    }
    nxt[k] = atomicExch(head + s, (uint32_t)k);
  }
}

__device__ __forceinline__ uint32_t join_head(const uint32_t* key, const uint32_t* head, uint64_t mask, uint32_t g) {
  uint64_t s = hslot(g, mask);
  for (;;) {
    const uint32_t k = key[s];
    if (k == g) return head[s];
    if (k == NO_ROW) return NO_ROW;
    s = (s + 1) & mask;
  }
}

// walks = a from-walk of level c (ending at x) followed by a to-walk of level g starting at x:
// count pass (emit == nullptr) or emission of [v0, t0, r0, ..., vL] (L = c + g)
__global__ void __launch_bounds__(CB) k_cap_join(CapLevels fw, int c, CapLevels tw, int g, uint64_t nf,
                                                 const uint32_t* __restrict__ key, const uint32_t* __restrict__ head,
                                                 const uint32_t* __restrict__ nxt, uint64_t mask, CapTypeVals ft,
                                                 CapTypeVals bt, unsigned long long* cnt, int64_t* __restrict__ emit) {
  unsigned long long total = 0;
  const int L = c + g;
  for (uint64_t f = (uint64_t)blockIdx.x * CB + threadIdx.x; f < nf; f += (uint64_t)gridDim.x * CB) {
    const CRec fr = fw.lv[c][f];
    if (fr.gid == NO_ROW) continue;
    for (uint32_t k = join_head(key, head, mask, fr.gid); k != NO_ROW; k = nxt[k]) {
      if (!emit) {
        ++total;
        continue;
      }
      int64_t* o = emit + atomicAdd(cnt, 1ull) * (uint64_t)(1 + 3 * L);
      CRec r = fr;
      for (int l = c; l >= 1; --l) {
        o[3 * l] = r.vid;
        o[3 * l - 2] = ft.type[r.tix];
        o[3 * l - 1] = r.rnk;
        r = fw.lv[l - 1][r.par];
      }
      o[0] = r.vid;
      // to-walk record at level l: vertex a_l reached from a_{l-1} through a_{l-1}'s in-row,
      // i.e. the edge a_l -> a_{l-1}
      CRec q = tw.lv[g][k];
      for (int l = g; l >= 1; --l) {
        const CRec p = tw.lv[l - 1][q.par];
        const int pos = c + (g - l);   // a_l sits at entry position pos
        o[3 * pos + 1] = bt.type[q.tix];
        o[3 * pos + 2] = q.rnk;
        o[3 * pos + 3] = p.vid;
        q = p;
      }
    }
  }
  if (!emit) wave_add(cnt, total);
}

// ---------------------------------------------------------------------------- host side
struct Arena {
  hipStream_t s;
  std::vector<void*> owned;
  ~Arena() {
    (void)hipStreamSynchronize(s);
    for (void* p : owned) (void)hipFree(p);
  }
  template <class T>
  hipError_t get(T** p, size_t count) {
    void* q = nullptr;
    const hipError_t e = hipMalloc(&q, (count ? count : 1) * sizeof(T));
    if (e != hipSuccess) return e;
    owned.push_back(q);
    *p = static_cast<T*>(q);
    return hipSuccess;
  }
};

#define CAP_TRY(x)                   \
  do {                               \
    const hipError_t e_ = (x);       \
    if (e_ != hipSuccess) return e_; \
  } while (0)

struct Ctx {
  const CapEnv& env;
  Arena arena;
  uint64_t words;        // bitmap words over the global id space
  uint64_t seg_words;    // words of one rank's segment
  uint32_t gbase;
  unsigned long long* ctr = nullptr;   // [4] device counters
  unsigned long long* h_ctr = nullptr; // pinned mirror
  unsigned long long* recv = nullptr;  // [words] all-to-all receive buffer
  unsigned long long* seg = nullptr;   // [seg_words] the rank's segment
  Cand* cand = nullptr;                // [CAND_N] greedy scratch
  Cand* h_cand = nullptr;
  uint64_t scanned = 0;
  static constexpr int HOP_GRID = 1024;
  static constexpr int CAND_N = HOP_GRID + 2 + 256;

  explicit Ctx(const CapEnv& e) : env(e), arena{e.stream} {
    const uint64_t G = (uint64_t)env.world;
    seg_words = G > 1 ? env.npad / 64 : cdivc(env.nv ? env.nv : 1, 64);
    words = seg_words * G;
    gbase = (uint32_t)((uint64_t)env.rank * (G > 1 ? env.npad : 0));
  }
  // A failure only this rank saw (an allocation, a device error) leaves its peers in or on their
  // way to the next collective: abort the communicator so that they fail too (comm.cpp).  Failures
  // decided on replicated data (`agreed`) happen on every rank at the same point.
  bool ok = false, agreed = false;
  ~Ctx() {
    if (!ok && !agreed && env.comm) env.comm->abort();
    (void)wait();
    if (h_ctr) (void)hipHostFree(h_ctr);
    if (h_cand) (void)hipHostFree(h_cand);
  }
  hipError_t init() {
    CAP_TRY(arena.get(&ctr, 4));
    CAP_TRY(hipMemsetAsync(ctr, 0, 4 * 8, env.stream));   // ctr[3]: adjacency entries scanned
    CAP_TRY(hipHostMalloc((void**)&h_ctr, 4 * sizeof(unsigned long long)));
    CAP_TRY(arena.get(&cand, CAND_N));
    CAP_TRY(hipHostMalloc((void**)&h_cand, sizeof(Cand)));
    if (env.world > 1) {
      CAP_TRY(arena.get(&recv, words));
      CAP_TRY(arena.get(&seg, seg_words));
    }
    return hipSuccess;
  }
  hipError_t wait() {
    if (env.comm) return env.comm->wait(env.stream) == 0 ? hipSuccess : hipErrorLaunchTimeOut;
    return hipStreamSynchronize(env.stream);
  }
  hipError_t comm_err() { return hipErrorUnknown; }
  // (into `a`, default the search's arena: a per-target arena keeps a multi-target search's
  // memory at one target's bitmaps)
  hipError_t bitmap(unsigned long long** p, Arena* a = nullptr) {
    CAP_TRY((a ? a : &arena)->get(p, words));
    return hipMemsetAsync(*p, 0, words * 8, env.stream);
  }
  // replicate a bitmap whose bits were set by every rank anywhere in the global id space
  hipError_t reduce_or(unsigned long long* Y) {
    if (env.world == 1) return hipSuccess;
    if (env.comm->alltoall(Y, recv, seg_words * 8, env.stream)) return comm_err();
    hipLaunchKernelGGL(k_cap_or, dim3(gridc(seg_words)), dim3(CB), 0, env.stream, recv, env.world, seg_words, seg);
    CAP_TRY(hipGetLastError());
    if (env.comm->allgather(seg, Y, seg_words * 8, env.stream)) return comm_err();
    return hipSuccess;
  }
  // replicate a bitmap whose rank segment (local bits) was written into `seg`
  hipError_t gather_seg(unsigned long long* local, unsigned long long* Y) {
    if (env.world == 1) return hipSuccess;   // local == Y
    if (env.comm->allgather(local, Y, seg_words * 8, env.stream)) return comm_err();
    return hipSuccess;
  }
  hipError_t expand(const CapCsr& cs, const unsigned long long* X, unsigned long long** Y, Arena* a = nullptr) {
    CAP_TRY(bitmap(Y, a));
    hipLaunchKernelGGL(k_cap_expand, dim3(gridc(env.nv, 8192)), dim3(CB), 0, env.stream, cs, X, *Y, env.nv, gbase,
                       env.K, env.visible, ctr + 3);
    CAP_TRY(hipGetLastError());
    CAP_TRY(reduce_or(*Y));
    return hipSuccess;
  }
  // |A ∩ B| (replicated inputs: the same on every rank); out (nullable) = A ∩ B
  hipError_t and_count(const unsigned long long* A, const unsigned long long* B, unsigned long long* out,
                       uint64_t* n) {
    CAP_TRY(hipMemsetAsync(ctr, 0, 8, env.stream));
    hipLaunchKernelGGL(k_cap_and, dim3(gridc(words)), dim3(CB), 0, env.stream, A, B, words, out, ctr);
    CAP_TRY(hipGetLastError());
    CAP_TRY(hipMemcpyAsync(h_ctr, ctr, 8, hipMemcpyDeviceToHost, env.stream));
    CAP_TRY(wait());
    *n = h_ctr[0];
    return hipSuccess;
  }
  hipError_t set_ids(const std::vector<uint32_t>& ids, unsigned long long** bm, Arena* a = nullptr) {
    CAP_TRY(bitmap(bm, a));
    if (ids.empty()) return hipSuccess;
    uint32_t* d = nullptr;
    CAP_TRY((a ? a : &arena)->get(&d, ids.size()));
    CAP_TRY(hipMemcpyAsync(d, ids.data(), ids.size() * 4, hipMemcpyHostToDevice, env.stream));
    hipLaunchKernelGGL(k_cap_set, dim3(gridc(ids.size())), dim3(CB), 0, env.stream, d, (uint64_t)ids.size(), *bm);
    CAP_TRY(hipGetLastError());
    return wait();   // `ids` may be a temporary
  }
  // minimum of the ranks' candidates at cand[src] -> h_cand (synchronous)
  hipError_t agree_cand(int src) {
    Cand* all = cand + HOP_GRID + 2;
    if (env.world > 1) {
      if (env.comm->allgather(cand + src, all, sizeof(Cand), env.stream)) return comm_err();
      hipLaunchKernelGGL(k_cap_reduce, dim3(1), dim3(CB), 0, env.stream, all, (uint64_t)env.world, cand + src);
      CAP_TRY(hipGetLastError());
    }
    CAP_TRY(hipMemcpyAsync(h_cand, cand + src, sizeof(Cand), hipMemcpyDeviceToHost, env.stream));
    return wait();
  }
  // the expansions' scanned entries (device counter) + the host-counted walks; marks success
  hipError_t finish(uint64_t* out) {
    CAP_TRY(hipMemcpyAsync(h_ctr + 3, ctr + 3, 8, hipMemcpyDeviceToHost, env.stream));
    CAP_TRY(wait());
    *out = scanned + h_ctr[3];
    ok = true;
    return hipSuccess;
  }
  uint32_t local_of(int64_t gid) const {
    const uint64_t v = (uint64_t)gid - gbase;
    return gid >= 0 && v < env.nv ? (uint32_t)v : NO_ROW;
  }
};

CapCsr csr_of(const PathTypes& pt) {
  CapCsr c{};
  c.n = pt.n;
  for (int k = 0; k < pt.n; ++k) {
    c.type[k] = pt.type[k];
    c.row_ptr[k] = pt.a[k].row_ptr;
    c.col[k] = pt.a[k].col;
    c.dst_vid[k] = pt.a[k].dst_vid;
    c.rank[k] = pt.a[k].rank;
  }
  return c;
}

}  // namespace

hipError_t cap_shortest(const CapEnv& env, const PathTypes& fwd, const PathTypes& bwd,
                        const std::vector<uint32_t>& Sgid, const std::vector<int64_t>& Svid,
                        const std::vector<uint32_t>& Tgid, uint32_t upto, std::vector<std::vector<int64_t>>* out,
                        uint64_t* scanned) {
  Ctx x(env);
  CAP_TRY(x.init());
  const CapCsr cf = csr_of(fwd), cb = csr_of(bwd);
  const uint32_t steps = upto / 2 + upto % 2;   // FindPathExecutor.cpp:155
  std::vector<unsigned long long*> F;           // from-frontiers, shared by the targets
  unsigned long long* f0 = nullptr;
  CAP_TRY(x.set_ids(Sgid, &f0));
  F.push_back(f0);
  auto from_level = [&](uint32_t c) -> hipError_t {
    while (F.size() <= c) {
      unsigned long long* y = nullptr;
      CAP_TRY(x.expand(cf, F.back(), &y));
      F.push_back(y);
    }
    return hipSuccess;
  };
  uint32_t* d_sg = nullptr;
  int64_t* d_sv = nullptr;
  CAP_TRY(x.arena.get(&d_sg, Sgid.size()));
  CAP_TRY(x.arena.get(&d_sv, Svid.size()));
  CAP_TRY(hipMemcpyAsync(d_sg, Sgid.data(), Sgid.size() * 4, hipMemcpyHostToDevice, env.stream));
  CAP_TRY(hipMemcpyAsync(d_sv, Svid.data(), Svid.size() * 8, hipMemcpyHostToDevice, env.stream));
  for (uint32_t t : Tgid) {
    Arena ta{env.stream};   // this target's to-side levels and B-sets, freed before the next target
    std::vector<unsigned long long*> T;
    unsigned long long* t0 = nullptr;
    CAP_TRY(x.set_ids(std::vector<uint32_t>{t}, &t0, &ta));
    T.push_back(t0);
    uint32_t L = 0;
    for (uint32_t c = 1; c <= steps && !L; ++c) {
      CAP_TRY(from_level(c));
      uint64_t n = 0;
      CAP_TRY(x.and_count(F[c], T[c - 1], nullptr, &n));   // odd meet: 2c - 1 edges
      if (n) { L = 2 * c - 1; break; }
      uint64_t nf = 0;
      CAP_TRY(x.and_count(F[c], F[c], nullptr, &nf));
      if (2 * c > upto && c == steps) break;
      unsigned long long* y = nullptr;
      CAP_TRY(x.expand(cb, T[c - 1], &y, &ta));
      T.push_back(y);
      uint64_t nt = 0;
      CAP_TRY(x.and_count(y, y, nullptr, &nt));
      if (2 * c <= upto) {
        CAP_TRY(x.and_count(F[c], y, nullptr, &n));   // even meet: 2c edges
        if (n) { L = 2 * c; break; }
      }
      if (!nf || !nt) break;   // an empty frontier ends the search (FindPathExecutor.cpp:175-178)
    }
    if (!L) continue;
    const uint32_t h = (L + 1) / 2;
    // B-sets: B[L] = {t}, B[i] = T[L - i] for i > h, B[h] = F[h] ∩ T[L - h], pulled below h
    std::vector<unsigned long long*> B(L + 1, nullptr);
    for (uint32_t i = h + 1; i <= L; ++i) B[i] = T[L - i];
    unsigned long long* bh = nullptr;
    CAP_TRY(x.bitmap(&bh, &ta));
    uint64_t nb = 0;
    CAP_TRY(x.and_count(F[h], T[L - h], bh, &nb));
    B[h] = bh;
    for (int i = (int)h - 1; i >= 0; --i) {
      unsigned long long* bi = nullptr;
      CAP_TRY(x.bitmap(&bi, &ta));
      unsigned long long* local = bi;   // single engine: the segment is the whole bitmap
      if (env.world > 1) {
        CAP_TRY(hipMemsetAsync(x.seg, 0, x.seg_words * 8, env.stream));
        local = x.seg;
      }
      hipLaunchKernelGGL(k_cap_pull, dim3(gridc(env.nv, 8192)), dim3(CB), 0, env.stream, cf, F[i], B[i + 1], env.nv,
                         x.gbase, env.K, env.visible, local);
      CAP_TRY(hipGetLastError());
      CAP_TRY(x.gather_seg(local, bi));
      B[i] = bi;
    }
    // greedy: v0 = the smallest source vid in B[0], then the minimum (type, rank, vid) per hop
    hipLaunchKernelGGL(k_cap_pick_source, dim3(1), dim3(1), 0, env.stream, B[0], d_sg, d_sv, (uint64_t)Sgid.size(),
                       x.cand);
    CAP_TRY(hipGetLastError());
    CAP_TRY(hipMemcpyAsync(x.h_cand, x.cand, sizeof(Cand), hipMemcpyDeviceToHost, env.stream));
    CAP_TRY(x.wait());
    if (x.h_cand->gid < 0) {
      x.agreed = true;
      return hipErrorNotFound;
    }
    std::vector<int64_t> p;
    p.push_back(x.h_cand->vid);
    int64_t cur = x.h_cand->gid;
    for (uint32_t i = 0; i < L; ++i) {
      const int src = Ctx::HOP_GRID;
      if (i < h) {
        hipLaunchKernelGGL(k_cap_hop_out, dim3(1), dim3(CB), 0, env.stream, cf, x.local_of(cur), env.K, B[i + 1],
                           x.cand + src);
      } else {
        const unsigned g = gridc(env.nv, Ctx::HOP_GRID);
        hipLaunchKernelGGL(k_cap_hop_in, dim3(g), dim3(CB), 0, env.stream, cb, (uint32_t)cur, env.K, B[i + 1],
                           env.nv, x.gbase, env.visible, env.vids, x.cand);
        CAP_TRY(hipGetLastError());
        hipLaunchKernelGGL(k_cap_reduce, dim3(1), dim3(CB), 0, env.stream, x.cand, (uint64_t)g, x.cand + src);
      }
      CAP_TRY(hipGetLastError());
      CAP_TRY(x.agree_cand(src));
      const Cand c = *x.h_cand;
      if (c.gid < 0) {   // the B-sets promised an edge (replicated: every rank sees it)
        x.agreed = true;
        return hipErrorNotFound;
      }
      p.push_back(c.type);
      p.push_back(c.rank);
      p.push_back(c.vid);
      cur = c.gid;
    }
    out->push_back(std::move(p));
  }
  return x.finish(scanned);
}

hipError_t cap_all(const CapEnv& env, const PathTypes& fwd, const PathTypes& bwd, const std::vector<uint32_t>& Sgid,
                   const std::vector<int64_t>& Svid, const std::vector<uint32_t>& Tgid,
                   const std::vector<int64_t>& Tvid, uint32_t upto, uint64_t max_walks,
                   std::vector<std::vector<int64_t>>* out, uint64_t* scanned) {
  if (upto >= CAP_LEVELS) return hipErrorInvalidValue;
  Ctx x(env);
  CAP_TRY(x.init());
  const CapCsr cf = csr_of(fwd), cb = csr_of(bwd);
  const uint32_t H = upto / 2 + upto % 2, G2 = upto / 2;
  uint64_t total = 0;
  // one walk family: level 0 = the endpoints, level l + 1 = every capped extension of level l
  auto walks = [&](const CapCsr& cs, const std::vector<uint32_t>& gid, const std::vector<int64_t>& vid,
                   uint32_t levels, CapLevels* lv, std::vector<uint64_t>* nlev) -> hipError_t {
    std::vector<CRec> h0(gid.size());
    for (size_t i = 0; i < gid.size(); ++i) h0[i] = CRec{gid[i], 0, 0, 0, 0, vid[i]};
    CRec* l0 = nullptr;
    CAP_TRY(x.arena.get(&l0, h0.size()));
    CAP_TRY(hipMemcpyAsync(l0, h0.data(), h0.size() * sizeof(CRec), hipMemcpyHostToDevice, env.stream));
    lv->lv[0] = l0;
    nlev->assign(levels + 1, 0);
    (*nlev)[0] = h0.size();
    unsigned long long* all = nullptr;
    CAP_TRY(x.arena.get(&all, 2 * (size_t)env.world));
    std::vector<unsigned long long> hc(2 * (size_t)env.world);
    for (uint32_t l = 0; l < levels && (*nlev)[l]; ++l) {
      const uint64_t n = (*nlev)[l];
      const unsigned grid = gridc(n, 8192);
      CAP_TRY(hipMemsetAsync(x.ctr, 0, 16, env.stream));
      hipLaunchKernelGGL(k_cap_walk, dim3(grid), dim3(CB), 0, env.stream, cs, lv->lv[l], n, env.nv, x.gbase, env.K,
                         env.visible, 0, (CRec*)nullptr, x.ctr);
      CAP_TRY(hipGetLastError());
      if (env.world > 1) {
        if (env.comm->allgather(x.ctr, all, 16, env.stream)) return x.comm_err();
      } else {
        CAP_TRY(hipMemcpyAsync(all, x.ctr, 16, hipMemcpyDeviceToDevice, env.stream));
      }
      CAP_TRY(hipMemcpyAsync(hc.data(), all, hc.size() * 8, hipMemcpyDeviceToHost, env.stream));
      CAP_TRY(x.wait());
      uint64_t sum = 0, maxc = 0;
      for (int q = 0; q < env.world; ++q) {
        sum += hc[2 * q];
        maxc = std::max<uint64_t>(maxc, hc[2 * q]);
        if (q == env.rank) x.scanned += hc[2 * q + 1];
      }
      if (!sum) break;   // the same on every rank
      total += sum;
      if (total > max_walks || (uint64_t)env.world * maxc >= 0xFFFFFFFFull) {
        x.agreed = true;   // summed counts: every rank stops here
        return hipErrorOutOfMemory;
      }
      CRec *mine = nullptr, *lvl = nullptr;
      CAP_TRY(x.arena.get(&mine, maxc));
      CAP_TRY(hipMemsetAsync(mine, 0xFF, maxc * sizeof(CRec), env.stream));   // unused slots: gid NO_ROW
      CAP_TRY(hipMemsetAsync(x.ctr, 0, 8, env.stream));
      hipLaunchKernelGGL(k_cap_walk, dim3(grid), dim3(CB), 0, env.stream, cs, lv->lv[l], n, env.nv, x.gbase, env.K,
                         env.visible, 1, mine, x.ctr);
      CAP_TRY(hipGetLastError());
      if (env.world > 1) {
        CAP_TRY(x.arena.get(&lvl, (size_t)env.world * maxc));
        if (env.comm->allgather(mine, lvl, maxc * sizeof(CRec), env.stream)) return x.comm_err();
      } else {
        lvl = mine;
      }
      lv->lv[l + 1] = lvl;
      (*nlev)[l + 1] = (uint64_t)env.world * maxc;
    }
    return x.wait();   // h0 is uploaded before it goes
  };
  CapLevels fw{}, tw{};
  std::vector<uint64_t> nf, nt;
  CAP_TRY(walks(cf, Sgid, Svid, H, &fw, &nf));
  CAP_TRY(walks(cb, Tgid, Tvid, G2, &tw, &nt));
  CapTypeVals ft{}, bt{};
  for (int k = 0; k < fwd.n; ++k) ft.type[k] = fwd.type[k];
  for (int k = 0; k < bwd.n; ++k) bt.type[k] = -(int64_t)bwd.type[k];
  // lengths L = 2c - 1 (from level c, to level c - 1) and L = 2c (c, c)
  for (uint32_t L = 1; L <= upto; ++L) {
    const int c = (int)((L + 1) / 2), g = (int)L - c;
    if (!nf[c] || !nt[g]) continue;
    uint64_t M = 1;
    while (M < 2 * nt[g]) M <<= 1;
    uint32_t *key = nullptr, *head = nullptr, *nxt = nullptr;
    CAP_TRY(x.arena.get(&key, M));
    CAP_TRY(x.arena.get(&head, M));
    CAP_TRY(x.arena.get(&nxt, nt[g]));
    CAP_TRY(hipMemsetAsync(key, 0xFF, M * 4, env.stream));
    CAP_TRY(hipMemsetAsync(head, 0xFF, M * 4, env.stream));
    hipLaunchKernelGGL(k_cap_join_build, dim3(gridc(nt[g])), dim3(CB), 0, env.stream, tw.lv[g], nt[g], key, head, nxt,
                       M - 1);
    CAP_TRY(hipGetLastError());
    CAP_TRY(hipMemsetAsync(x.ctr, 0, 8, env.stream));
    hipLaunchKernelGGL(k_cap_join, dim3(gridc(nf[c])), dim3(CB), 0, env.stream, fw, c, tw, g, nf[c], key, head, nxt,
                       M - 1, ft, bt, x.ctr, (int64_t*)nullptr);
    CAP_TRY(hipGetLastError());
    CAP_TRY(hipMemcpyAsync(x.h_ctr, x.ctr, 8, hipMemcpyDeviceToHost, env.stream));
    CAP_TRY(x.wait());
    const uint64_t np = x.h_ctr[0];
    if (!np) continue;
    if (np > max_walks) {
      x.agreed = true;
      return hipErrorOutOfMemory;
    }
    const uint64_t width = 1 + 3 * (uint64_t)L;
    int64_t* o = nullptr;
    CAP_TRY(x.arena.get(&o, np * width));
    CAP_TRY(hipMemsetAsync(x.ctr, 0, 8, env.stream));
    hipLaunchKernelGGL(k_cap_join, dim3(gridc(nf[c])), dim3(CB), 0, env.stream, fw, c, tw, g, nf[c], key, head, nxt,
                       M - 1, ft, bt, x.ctr, o);
    CAP_TRY(hipGetLastError());
    std::vector<int64_t> host(np * width);
    CAP_TRY(hipMemcpyAsync(host.data(), o, host.size() * 8, hipMemcpyDeviceToHost, env.stream));
    CAP_TRY(x.wait());
    for (uint64_t i = 0; i < np; ++i)
      out->emplace_back(host.begin() + (ptrdiff_t)(i * width), host.begin() + (ptrdiff_t)((i + 1) * width));
  }
  return x.finish(scanned);
}

}  // namespace nbg
