// FIND SHORTEST PATH for one (source, target) pair in ONE persistent launch (single engine).
//
// Same semantics and result as path.cpp's bidirectional search (FindPathExecutor.cpp:145-411
// restated: minimal hop count, UPTO N, one path per target, ties broken by the lexicographically
// smallest entry list [v0, t0, r0, v1, ...]), but the level loop, the direction choice, the
// meet / termination tests, the B-set recovery and the greedy reconstruction all run on the
// device: the host enqueues one launch and one copy of the result block per pair, and waits once.
//
// Work is cut into ITEMS — runs of <= 64 consecutive CSR entries of one OVER type — produced
// when a vertex is claimed (its edges over the side's CSRs, split into 64-entry runs), so every
// level is a flat list of equal-sized items: a wave takes SP_U items per iteration, lane l owns
// entry l of each, and hubs spread over all waves with no merge-path pass and no degree scan.
//
// Workgroup 0 is the leader: it runs every small phase (<= SP_SMALL items) alone, and for a big
// phase publishes the phase parameters (agent-scope release, then the generation word) so that
// every workgroup takes its share; followers poll the generation word (sc1 loads + s_sleep),
// acquire, work, release and arrive on a counter the leader waits for.  Every spin is bounded
// (SpCtl::err = 2 and all workgroups leave).  Labels are epoch-stamped (epoch << LVL_BITS |
// level) like path.cpp's, read with agent-scope loads (sc1: the L1 may hold a stale line of a
// label another workgroup or an earlier phase claimed) and claimed with CAS.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "nbg_internal.h"

#define HIP_TRY_SP(x)                     \
  do {                                    \
    hipError_t e_ = (x);                  \
    if (e_ != hipSuccess) return e_;      \
  } while (0)

namespace nbg {
namespace {

constexpr int SP_THREADS = 512;
constexpr int SP_WAVES = SP_THREADS / 64;
constexpr int SP_U = 8;                 // items per wave pass (their loads in flight together)
constexpr int SP_PASS = SP_WAVES * SP_U;   // items per workgroup pass
constexpr uint32_t SP_CH = 64;          // CSR entries per item
constexpr uint64_t SP_SMALL = 2 * SP_PASS;   // a phase with at most this many items runs on the leader alone
constexpr uint32_t SP_GREEDY_SMALL = 4096;   // greedy hop: adjacency the leader scans alone
constexpr int SP_MAX_WGS = 256;

enum SpOp : uint32_t { OP_LEVEL = 1, OP_BSET = 2, OP_GREEDY = 3, OP_EXIT = 4 };
enum SpList : int { L_F0 = 0, L_F1 = 1, L_B0 = 2, L_B1 = 3, L_M0 = 4, L_M1 = 5, SP_NLISTS = 6 };

}  // namespace

// Device control block of one persistent query (zeroed once; per-query words reset by the leader).
// The polled generation word, the arrival counter and each accumulator sit on cache lines of
// their own: 63 pollers on the line that the level's atomics hit would serialise both.
struct alignas(128) SpWord {
  unsigned long long v;
  unsigned long long pad[15];
};
struct SpCtl {
  SpWord gen;                      // released phase: (q << 24) | phase
  SpWord arrive;                   // follower arrivals (reset at query start)
  SpWord err;                      // 1 reconstruction failure, 2 spin bound hit, 3 list overflow
  SpWord out_n, dsum, meet_n, meet_items, edges;   // phase accumulators (leader zeroes them)
  // phase parameters (leader writes, releases, bumps gen)
  alignas(128) unsigned long long op, side, src, n, dst, pos, cur, stamp, mstamp;
  alignas(128) unsigned long long gpart[4 * SP_MAX_WGS];   // greedy: per-workgroup minimum
};

// What a query reads besides its scalars: in device memory (uploaded when it changes), never a
// kernel argument — device code indexes its arrays with run-time indices, which on a by-value
// kernel argument would force a private (scratch) copy per lane.
struct SpArgs {
  SpTypes fwd, bwd;
  const uint8_t* visible;
  const int64_t* vids;
  uint32_t* lab_f;
  uint32_t* lab_b;
  uint32_t* lab_m;
  uint64_t* list[SP_NLISTS];
  uint64_t list_cap;
  SpCtl* ctl;
  SpResult* res;
};
struct SpQ {                       // per-query scalars (kernel argument, then LDS)
  uint32_t s, t, upto;
  uint32_t ef, eb, em;             // this query's epochs
  unsigned long long q;            // query sequence number (generation encoding)
  unsigned long long spin_limit;
};

namespace {

__device__ __forceinline__ uint32_t ld1(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld1(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st1(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st1(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint32_t stamp_of(uint32_t epoch, uint32_t level) { return (epoch << LVL_BITS) | level; }
__device__ __forceinline__ bool live(uint32_t lab, uint32_t epoch) { return (lab >> LVL_BITS) == epoch; }

// item: [j0:32][len-1:8][type index:8]
__device__ __forceinline__ uint64_t item_make(uint32_t j0, uint32_t len, uint32_t t) {
  return ((uint64_t)j0 << 32) | ((uint64_t)(len - 1) << 8) | t;
}

__device__ __forceinline__ uint32_t wave_incl_scan32(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

// Items of vertex x over a side's CSRs (visible vertices only): count and edge total.
__device__ __forceinline__ void vertex_items(const SpTypes& T, const uint8_t* visible, uint32_t x, uint32_t* nitems,
                                             uint32_t* nedges) {
  uint32_t ni = 0, ne = 0;
  if (x != NO_ROW && (!visible || visible[x])) {
    for (int t = 0; t < T.n; ++t) {
      const uint32_t d = T.row_ptr[t][x + 1] - T.row_ptr[t][x];
      ni += (d + SP_CH - 1) / SP_CH;
      ne += d;
    }
  }
  *nitems = ni;
  *nedges = ne;
}

// Writes items [first, total) step `stride` of vertex x over T at out[base + k]: item k is the
// k-th 64-entry run of x's rows, types in OVER order.  Row ranges are read once per type (a hub's
// thousands of items are then plain stores).
__device__ __forceinline__ void write_items(const SpTypes& T, uint32_t x, uint64_t* out, uint64_t base, uint32_t first,
                                            uint32_t stride, uint32_t total) {
  int64_t k0 = 0;   // items of the earlier types
  for (int t = 0; t < T.n && k0 < (int64_t)total; ++t) {
    const uint32_t rs = T.row_ptr[t][x], re = T.row_ptr[t][x + 1];
    const int64_t ni = (re - rs + SP_CH - 1) / SP_CH;
    // the first k >= k0 with k = first (mod stride)
    int64_t k = (int64_t)first >= k0 ? (int64_t)first
                                     : k0 + (((int64_t)first - k0) % (int64_t)stride + stride) % (int64_t)stride;
    for (; k < k0 + ni && k < (int64_t)total; k += stride) {
      const uint32_t j0 = rs + (uint32_t)(k - k0) * SP_CH;
      const uint32_t len = re - j0 < SP_CH ? re - j0 : SP_CH;
      out[base + (uint64_t)k] = item_make(j0, len, (uint32_t)t);
    }
    k0 += ni;
  }
}

// Appends, for every lane with want != 0, vertex x's items over T to list `out` (counter *n):
// one returning atomic per wave; vertices with many items are written by the whole wave.
__device__ __forceinline__ void wave_append(const SpTypes& T, uint32_t x, bool want, uint32_t nitems, uint64_t* out,
                                            unsigned long long* n, uint64_t cap, unsigned long long* err) {
  const int lane = threadIdx.x & 63;
  const uint32_t c = want ? nitems : 0;
  const uint32_t inc = wave_incl_scan32(c);
  const uint32_t tot = __shfl(inc, 63, 64);
  if (!tot) return;
  unsigned long long base = 0;
  if (lane == 0) base = atomicAdd(n, (unsigned long long)tot);
  base = __shfl(base, 0, 64);
  if (base + tot > cap) {
    if (lane == 0) atomicOr(err, 3ull);
    return;
  }
  const uint64_t mine = base + inc - c;
  const bool big = c > 8;
  if (c && !big) write_items(T, x, out, mine, 0, 1, c);
  unsigned long long bm = __ballot(big);
  while (bm) {   // hubs: the whole wave writes their items
    const int l = __ffsll((long long)bm) - 1;
    bm &= bm - 1;
    const uint32_t hx = __shfl(x, l, 64);
    const uint64_t hb = __shfl(mine, l, 64);
    const uint32_t hc = __shfl(c, l, 64);
    write_items(T, hx, out, hb, (uint32_t)lane, 64, hc);
  }
}

#ifndef SP_SUBTRACE
#define SP_SUBTRACE 0
#endif

struct LevelCfg {
  const SpTypes* T;          // CSRs expanded (side's direction)
  const SpTypes* N;          // CSRs of the claimed vertices' items (next level of the same side)
  const SpTypes* M;          // CSRs of a meet vertex's B-set items (in-edges)
  uint32_t* lab;             // claimed label
  uint32_t epoch, stamp;
  bool exact;                // already claimed = lab == stamp (B-sets: one LAB_M epoch, many positions)
  const uint32_t* rlab;      // restriction (B-set): claim u only if rlab[u] == rstamp
  uint32_t rstamp;
  const uint32_t* olab;      // other side's labels (meet test), nullable
  uint32_t oepoch;
  uint32_t mstamp;           // LAB_M stamp of a meet vertex
  bool append;               // append the claimed vertices' items (N) to dst
};

// Per-workgroup scratch of run_level's aggregated append.
struct LevelLds {
  uint32_t wave_tot[SP_WAVES];
  unsigned long long base;
  uint32_t total;
};

// Items of the claimed vertices of one lane (up to SP_U of them) over T, from their row ranges.
__device__ __forceinline__ uint32_t lane_items(const SpTypes& T, const uint32_t (&x)[SP_U], uint32_t cmask,
                                               const uint8_t* visible, uint32_t (&ni)[SP_U], unsigned long long* dsum,
                                               uint32_t (&rs0)[SP_U], uint32_t (&re0)[SP_U]) {
  uint32_t vis[SP_U];
#pragma unroll
  for (int u = 0; u < SP_U; ++u) vis[u] = ((cmask >> u) & 1u) && (!visible || visible[x[u]]);
  uint32_t c = 0;
#pragma unroll
  for (int u = 0; u < SP_U; ++u) ni[u] = 0;
  for (int t = 0; t < T.n; ++t) {
    uint32_t rs[SP_U], re[SP_U];
#pragma unroll
    for (int u = 0; u < SP_U; ++u) {   // every row range of this type in flight at once
      rs[u] = vis[u] ? T.row_ptr[t][x[u]] : 0u;
      re[u] = vis[u] ? T.row_ptr[t][x[u] + 1] : 0u;
    }
#pragma unroll
    for (int u = 0; u < SP_U; ++u) {
      const uint32_t d = re[u] - rs[u];
      ni[u] += (d + SP_CH - 1) / SP_CH;
      *dsum += d;
      if (t == 0) {
        rs0[u] = rs[u];
        re0[u] = re[u];
      }
    }
  }
#pragma unroll
  for (int u = 0; u < SP_U; ++u) c += ni[u];
  return c;
}

// One phase over the items of list `src` (n items): workgroup wg of nwg takes passes of SP_PASS
// items (SP_U per wave; lane l owns entry l of each item).  Per pass: every neighbour's labels in
// flight at once, the CAS claims, the claimed vertices' row ranges, then ONE atomic per workgroup
// reserves the pass's output items (block scan in LDS).
__device__ __forceinline__ void run_level(const SpArgs& A, const LevelCfg& C, const uint64_t* src, uint64_t n, uint64_t* dst,
                          int wg, int nwg, LevelLds* L) {
  SpCtl* ctl = A.ctl;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  unsigned long long edges = 0, dsum = 0;
  const bool tr = SP_SUBTRACE && wg == 0 && threadIdx.x == 0;   // (build with -DSP_SUBTRACE=1 to time sub-steps)
  unsigned long long tp = tr ? (unsigned long long)wall_clock64() : 0ull;
  auto mark = [&](int k, const uint32_t* dep) {   // (dep: a value the step produced, so the clock waits for it)
    if (!tr) return;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    const unsigned long long now = (unsigned long long)wall_clock64() + (dep ? (*dep & 0u) : 0u);
    A.res->sub[k] += now - tp;
    tp = now;
  };
  for (uint64_t p0 = (uint64_t)wg * SP_PASS; p0 < n; p0 += (uint64_t)nwg * SP_PASS) {   // uniform per workgroup
    const uint64_t i0 = p0 + (uint64_t)wv * SP_U;
    if (tr) A.res->sub[7] += 1;
    uint64_t it = 0;
    if (lane < SP_U && i0 + lane < n) it = src[i0 + lane];
    uint32_t x[SP_U];
#pragma unroll
    for (int u = 0; u < SP_U; ++u) {
      const uint64_t iu = __shfl(it, u, 64);
      x[u] = NO_ROW;
      if (i0 + u < n) {
        const uint32_t j0 = (uint32_t)(iu >> 32), len = (uint32_t)((iu >> 8) & 0xFF) + 1, t = (uint32_t)(iu & 0xFF);
        if ((uint32_t)lane < len) {
          x[u] = C.T->col[t][(uint64_t)j0 + lane];
          ++edges;
        }
      }
    }
    mark(0, &x[0]);
    // labels (claim, restriction, other side) of every neighbour in flight together
    uint32_t old[SP_U], rl[SP_U], ol[SP_U];
#pragma unroll
    for (int u = 0; u < SP_U; ++u) {
      const bool v = x[u] != NO_ROW;
      old[u] = v ? ld1(C.lab + x[u]) : 0u;
      rl[u] = (v && C.rlab) ? ld1(C.rlab + x[u]) : C.rstamp;
      ol[u] = (v && C.olab) ? ld1(C.olab + x[u]) : 0u;
    }
    mark(1, &old[0]);
    uint32_t claimed = 0, meet = 0;
#pragma unroll
    for (int u = 0; u < SP_U; ++u) {
      if (x[u] == NO_ROW || rl[u] != C.rstamp) continue;
      if (C.exact ? old[u] == C.stamp : live(old[u], C.epoch)) continue;
      if (atomicCAS(C.lab + x[u], old[u], C.stamp) != old[u]) continue;
      claimed |= 1u << u;
      if (C.olab && live(ol[u], C.oepoch)) meet |= 1u << u;
    }
    // output items of the claimed vertices: one reservation per workgroup pass
    mark(2, &claimed);
    uint32_t ni[SP_U];
#pragma unroll
    for (int u = 0; u < SP_U; ++u) ni[u] = 0;
    uint32_t rs0[SP_U], re0[SP_U];
    const uint32_t c = C.append ? lane_items(*C.N, x, claimed, A.visible, ni, &dsum, rs0, re0) : 0u;
    mark(3, &c);
    const uint32_t incl = wave_incl_scan32(c);
    if (lane == 63) L->wave_tot[wv] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t run = 0;
      for (int k = 0; k < SP_WAVES; ++k) {
        const uint32_t w_ = L->wave_tot[k];
        L->wave_tot[k] = run;
        run += w_;
      }
      L->total = run;
      L->base = run ? atomicAdd(&ctl->out_n.v, (unsigned long long)run) : 0ull;
      if (run && L->base + run > A.list_cap) atomicOr(&ctl->err.v, 3ull);
    }
    __syncthreads();
    const bool room = L->base + L->total <= A.list_cap;
    uint64_t mine = L->base + L->wave_tot[wv] + incl - c;
    __syncthreads();   // wave_tot / base are rewritten by the next pass
    mark(4, nullptr);
    if (room && C.N->n == 1) {   // one type: the row ranges are in registers already
      uint64_t off[SP_U];
#pragma unroll
      for (int u = 0; u < SP_U; ++u) {
        off[u] = mine;
        mine += ni[u];
        if (ni[u] && ni[u] <= 8)
          for (uint32_t k = 0; k < ni[u]; ++k) {
            const uint32_t j0 = rs0[u] + k * SP_CH;
            dst[off[u] + k] = item_make(j0, re0[u] - j0 < SP_CH ? re0[u] - j0 : SP_CH, 0u);
          }
      }
#pragma unroll
      for (int u = 0; u < SP_U; ++u) {   // vertices with many items: the whole wave writes them
        unsigned long long bm = __ballot(ni[u] > 8);
        while (bm) {
          const int l = __ffsll((long long)bm) - 1;
          bm &= bm - 1;
          if (tr) A.res->sub[6] += 1ull << 40;
          const uint32_t hs = __shfl(rs0[u], l, 64), he = __shfl(re0[u], l, 64), hc = __shfl(ni[u], l, 64);
          const uint64_t hb = __shfl(off[u], l, 64);
          for (uint32_t k = (uint32_t)lane; k < hc; k += 64) {
            const uint32_t j0 = hs + k * SP_CH;
            dst[hb + k] = item_make(j0, he - j0 < SP_CH ? he - j0 : SP_CH, 0u);
          }
        }
      }
    } else if (room) {
      bool big = false;
#pragma unroll
      for (int u = 0; u < SP_U; ++u) big |= ni[u] > 8;
      if (!big) {
#pragma unroll
        for (int u = 0; u < SP_U; ++u)
          if (ni[u]) {
            write_items(*C.N, x[u], dst, mine, 0, 1, ni[u]);
            mine += ni[u];
          }
      }
      unsigned long long bm = __ballot(big);
      while (bm) {   // lanes with a hub among their vertices: the whole wave writes their items
        const int l = __ffsll((long long)bm) - 1;
        bm &= bm - 1;
        if (tr) A.res->sub[6] += 1ull << 40;
        uint64_t b = __shfl(mine, l, 64);
#pragma unroll
        for (int u = 0; u < SP_U; ++u) {
          const uint32_t hx = __shfl(x[u], l, 64), hc = __shfl(ni[u], l, 64);
          if (hc) write_items(*C.N, hx, dst, b, (uint32_t)lane, 64, hc);
          b += hc;
        }
      }
    }
    mark(5, nullptr);
    if (C.olab && __ballot(meet != 0)) {   // rare: a meet vertex gets LAB_M and its in-edge items
      uint32_t mi[SP_U];
      unsigned long long md = 0;
#pragma unroll
      for (int u = 0; u < SP_U; ++u)
        if ((meet >> u) & 1u) st1(A.lab_m + x[u], C.mstamp);
      uint32_t mrs[SP_U], mre[SP_U];
      const uint32_t mc = lane_items(*C.M, x, meet, A.visible, mi, &md, mrs, mre);
      const uint32_t minc = wave_incl_scan32(mc);
      const uint32_t mtot = __shfl(minc, 63, 64);
      const uint32_t nmeet = (uint32_t)__popc(meet);
      uint32_t mcount = nmeet;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) mcount += __shfl_xor(mcount, o, 64);
      unsigned long long mb = 0;
      if (lane == 0) {
        atomicAdd(&ctl->meet_n.v, (unsigned long long)mcount);
        if (mtot) mb = atomicAdd(&ctl->meet_items.v, (unsigned long long)mtot);
      }
      mb = __shfl(mb, 0, 64);
      if (mb + mtot <= A.list_cap) {
        uint64_t m = mb + minc - mc;
#pragma unroll
        for (int u = 0; u < SP_U; ++u)
          if (mi[u]) {
            write_items(*C.M, x[u], A.list[L_M0], m, 0, 1, mi[u]);
            m += mi[u];
          }
      } else if (lane == 0) {
        atomicOr(&ctl->err.v, 3ull);
      }
    }
  }
  mark(6, nullptr);
  // wave totals: one atomic each
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    edges += __shfl_xor(edges, o, 64);
    dsum += __shfl_xor(dsum, o, 64);
  }
  if (lane == 0) {
    if (edges) atomicAdd(&ctl->edges.v, edges);
    if (dsum) atomicAdd(&ctl->dsum.v, dsum);
  }
}

struct Cand {
  int64_t t, r, v;
  uint32_t d;
};
__device__ __forceinline__ bool cand_less(const Cand& a, const Cand& b) {
  if (a.t != b.t) return a.t < b.t;
  if (a.r != b.r) return a.r < b.r;
  return a.v < b.v;
}

// Greedy hop `pos` from vertex c: the minimum (type, rank, dst vid) out-edge into B[pos + 1].
__device__ __forceinline__ Cand greedy_scan(const SpArgs& A, const SpQ& Q, uint32_t c, int pos, int L, int kf, int wg, int nwg,
                            Cand* lds) {
  const Cand none{INT64_MAX, INT64_MAX, INT64_MAX, NO_ROW};
  Cand best = none;
  const uint32_t want_m = stamp_of(Q.em, (uint32_t)(pos + 1));
  const uint32_t want_b = stamp_of(Q.eb, (uint32_t)(L - pos - 1));
  const bool by_m = pos + 1 <= kf;
  if (c != NO_ROW && (!A.visible || A.visible[c])) {
    const uint64_t g = (uint64_t)wg * SP_THREADS + threadIdx.x, G = (uint64_t)nwg * SP_THREADS;
    const uint32_t* lab = by_m ? A.lab_m : A.lab_b;
    const uint32_t want = by_m ? want_m : want_b;
    for (int t = 0; t < A.fwd.n; ++t) {
      const uint32_t rs = A.fwd.row_ptr[t][c], re = A.fwd.row_ptr[t][c + 1];
      for (uint64_t j0 = rs + g; j0 < re; j0 += 4 * G) {   // 4 edges per thread in flight
        uint32_t w[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) w[k] = j0 + k * G < re ? A.fwd.col[t][j0 + k * G] : NO_ROW;
        uint32_t l[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) l[k] = w[k] != NO_ROW ? ld1(lab + w[k]) : 0u;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (w[k] == NO_ROW || l[k] != want) continue;
          const uint64_t j = j0 + k * G;
          Cand x{(int64_t)A.fwd.type[t], A.fwd.rank[t] ? A.fwd.rank[t][j] : 0, A.fwd.dst_vid[t][j], w[k]};
          if (cand_less(x, best)) best = x;
        }
      }
    }
  }
  // block minimum
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    Cand x;
    x.t = __shfl_down(best.t, o, 64);
    x.r = __shfl_down(best.r, o, 64);
    x.v = __shfl_down(best.v, o, 64);
    x.d = __shfl_down(best.d, o, 64);
    if ((threadIdx.x & 63) + o < 64 && cand_less(x, best)) best = x;
  }
  if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < SP_WAVES; ++i)
      if (cand_less(lds[i], best)) best = lds[i];
    lds[SP_WAVES] = best;
  }
  __syncthreads();
  best = lds[SP_WAVES];
  __syncthreads();
  return best;
}

// ---------------------------------------------------------------- leader / follower protocol
// every storing wave drained, the workgroup joined, then one lane's agent release
__device__ __forceinline__ void wg_release() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

__device__ __forceinline__ void wg_acquire() {
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

struct PhaseView {   // the leader's phase parameters, as every workgroup reads them
  uint32_t op, side, src, dst, pos, cur;
  uint64_t n;
  uint32_t stamp, mstamp;
  uint32_t L, kf;
};

__device__ __forceinline__ void run_phase(const SpArgs& A, const SpQ& Q, const PhaseView& P, int wg, int nwg,
                                          Cand* lds, LevelLds* L) {
  if (P.op == OP_GREEDY) {
    Cand b = greedy_scan(A, Q, P.cur, (int)P.pos, (int)P.L, (int)P.kf, wg, nwg, lds);
    if (threadIdx.x == 0) {
      unsigned long long* part = A.ctl->gpart + 4 * wg;
      part[0] = (unsigned long long)b.t;
      part[1] = (unsigned long long)b.r;
      part[2] = (unsigned long long)b.v;
      part[3] = b.d;
    }
    return;
  }
  if (P.op != OP_LEVEL && P.op != OP_BSET) return;
  LevelCfg C{};
  if (P.op == OP_LEVEL) {
    const bool fw = P.side == 0;
    C.T = fw ? &A.fwd : &A.bwd;
    C.N = C.T;
    C.M = &A.bwd;
    C.lab = fw ? A.lab_f : A.lab_b;
    C.epoch = fw ? Q.ef : Q.eb;
    C.stamp = P.stamp;
    C.olab = fw ? A.lab_b : A.lab_f;
    C.oepoch = fw ? Q.eb : Q.ef;
    C.mstamp = P.mstamp;
    C.append = true;
  } else {
    // B[pos] from B[pos + 1] through in-edges, restricted to forward level pos, claimed in LAB_M
    C.T = &A.bwd;
    C.N = &A.bwd;
    C.lab = A.lab_m;
    C.exact = true;
    C.stamp = P.stamp;
    C.rlab = A.lab_f;
    C.rstamp = stamp_of(Q.ef, P.pos);
    C.append = P.pos >= 2;   // B[1]'s in-edges are not needed (B[0] = {s})
  }
  run_level(A, C, A.list[P.src], P.n, A.list[P.dst], wg, nwg, L);
}

}  // namespace

__global__ void __launch_bounds__(SP_THREADS) k_sp_pair(const SpArgs* __restrict__ Ap, SpQ qarg) {
  __shared__ PhaseView sP;
  __shared__ Cand lds[SP_WAVES + 1];
  __shared__ LevelLds sL;
  __shared__ int sQuit;
  __shared__ SpQ Q;
  if (threadIdx.x == 0) Q = qarg;
  __syncthreads();
  const SpArgs& A = *Ap;
  SpCtl* ctl = A.ctl;
  const unsigned long long g0 = Q.q << 24;
  const int nwg = gridDim.x;
  if (blockIdx.x != 0) {
    // ------------------------------------------------ follower
    unsigned long long seen = g0;
    for (;;) {
      if (threadIdx.x == 0) {
        unsigned long long g = ld1(&ctl->gen.v);
        unsigned long long spins = 0;
        while (g == seen || g < g0) {   // (< g0: a generation of an earlier query)
          if (++spins > Q.spin_limit) { atomicOr(&ctl->err.v, 2ull); g = 0; break; }
          __builtin_amdgcn_s_sleep(2);
          g = ld1(&ctl->gen.v);
        }
        sQuit = g == 0;
        seen = g;
      }
      __syncthreads();
      if (sQuit) return;
      wg_acquire();
      if (threadIdx.x == 0) {
        sP.op = (uint32_t)ctl->op;
        sP.side = (uint32_t)ctl->side;
        sP.src = (uint32_t)ctl->src;
        sP.n = ctl->n;
        sP.dst = (uint32_t)ctl->dst;
        sP.pos = (uint32_t)ctl->pos;
        sP.cur = (uint32_t)ctl->cur;
        sP.stamp = (uint32_t)ctl->stamp;
        sP.mstamp = (uint32_t)ctl->mstamp;
        sP.L = (uint32_t)(ctl->mstamp >> 32);
        sP.kf = (uint32_t)(ctl->stamp >> 32);
      }
      __syncthreads();
      const PhaseView P = sP;
      if (P.op == OP_EXIT) return;
      run_phase(A, Q, P, (int)blockIdx.x, nwg, lds, &sL);
      wg_release();
      if (threadIdx.x == 0) atomicAdd(&ctl->arrive.v, 1ull);
      __syncthreads();
    }
  }
  // -------------------------------------------------- leader
  __shared__ unsigned long long sAcc[6];
  unsigned long long phase = 0, big_phases = 0;
  bool failed = false;
  unsigned ntr = 0;
  auto trace = [&](unsigned long long kind) {   // thread 0
    if (ntr < 40) A.res->trace[ntr++] = (kind << 56) | ((unsigned long long)wall_clock64() & ((1ull << 56) - 1));
  };
  if (threadIdx.x == 0) trace(0);
  // run one phase: alone when small, else published to every workgroup
  auto phase_run = [&](PhaseView P, bool big) {
    if (threadIdx.x == 0) {
      st1(&ctl->out_n.v, 0ull);
      st1(&ctl->dsum.v, 0ull);
      st1(&ctl->meet_n.v, 0ull);
      st1(&ctl->meet_items.v, 0ull);
      st1(&ctl->edges.v, 0ull);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (big && nwg > 1 && !failed) {
      if (threadIdx.x == 0) {
        ctl->op = P.op;
        ctl->side = P.side;
        ctl->src = P.src;
        ctl->n = P.n;
        ctl->dst = P.dst;
        ctl->pos = P.pos;
        ctl->cur = P.cur;
        ctl->stamp = ((unsigned long long)P.kf << 32) | P.stamp;
        ctl->mstamp = ((unsigned long long)P.L << 32) | P.mstamp;
      }
      wg_release();
      if (threadIdx.x == 0) st1(&ctl->gen.v, g0 | ++phase);
      __syncthreads();
      run_phase(A, Q, P, 0, nwg, lds, &sL);
      ++big_phases;
      if (threadIdx.x == 0) {
        const unsigned long long want = big_phases * (unsigned long long)(nwg - 1);
        unsigned long long spins = 0;
        while (ld1(&ctl->arrive.v) < want) {
          if (++spins > Q.spin_limit) { atomicOr(&ctl->err.v, 2ull); break; }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      __syncthreads();
      wg_acquire();
    } else {
      run_phase(A, Q, P, 0, 1, lds, &sL);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      trace((unsigned long long)P.op * 2 + (big && nwg > 1 ? 1 : 0));
      sAcc[0] = ld1(&ctl->out_n.v);
      sAcc[1] = ld1(&ctl->dsum.v);
      sAcc[2] = ld1(&ctl->meet_n.v);
      sAcc[3] = ld1(&ctl->meet_items.v);
      sAcc[4] = ld1(&ctl->edges.v);
      sAcc[5] = ld1(&ctl->err.v);
    }
    __syncthreads();
    failed = failed || sAcc[5] != 0;
  };

  // ---- set-up: labels of s and t, their items
  if (threadIdx.x == 0) {
    st1(&ctl->arrive.v, 0ull);
    st1(&ctl->err.v, 0ull);
    st1(&ctl->out_n.v, 0ull);
    st1(&ctl->meet_items.v, 0ull);
    A.res->L = 0;
    A.res->edges = 0;
    A.res->err = 0;
    A.res->levels = 0;
    for (int k = 0; k < 8; ++k) A.res->sub[k] = 0;
  }
  __syncthreads();
  uint32_t nis = 0, nes = 0, nit = 0, net = 0;
  if (threadIdx.x == 0) {
    st1(A.lab_f + Q.s, stamp_of(Q.ef, 0));
    st1(A.lab_b + Q.t, stamp_of(Q.eb, 0));
  }
  vertex_items(A.fwd, A.visible, Q.s, &nis, &nes);
  vertex_items(A.bwd, A.visible, Q.t, &nit, &net);
  if (threadIdx.x < 64) {   // wave 0 writes both item lists
    write_items(A.fwd, Q.s, A.list[L_F0], 0, (uint32_t)threadIdx.x, 64, nis);
    write_items(A.bwd, Q.t, A.list[L_B0], 0, (uint32_t)threadIdx.x, 64, nit);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) trace(1);
  uint64_t nF = nis, nB = nit, dsf = nes, dsb = net, edges = 0;
  int fcur = L_F0, bcur = L_B0, kf = 0, kb = 0;
  bool met = false;
  uint64_t n_meet_items = 0;
  int levels = 0;
  if (dsf && dsb) {
    while ((uint32_t)(kf + kb) < Q.upto && !failed) {
      const bool fw = dsf <= dsb;
      PhaseView P{};
      P.op = OP_LEVEL;
      P.side = fw ? 0 : 1;
      P.src = (uint32_t)(fw ? fcur : bcur);
      P.dst = P.src ^ 1u;
      P.n = fw ? nF : nB;
      P.stamp = fw ? stamp_of(Q.ef, (uint32_t)kf + 1) : stamp_of(Q.eb, (uint32_t)kb + 1);
      P.mstamp = stamp_of(Q.em, fw ? (uint32_t)kf + 1 : (uint32_t)kf);
      phase_run(P, P.n > SP_SMALL);
      ++levels;
      edges += sAcc[4];
      if (fw) { fcur ^= 1; nF = sAcc[0]; dsf = sAcc[1]; ++kf; }
      else { bcur ^= 1; nB = sAcc[0]; dsb = sAcc[1]; ++kb; }
      if (sAcc[2]) { met = true; n_meet_items = sAcc[3]; break; }
      if (sAcc[0] == 0) break;   // a side has no further edges: no path
    }
  }
  const int L = kf + kb;
  bool ok = met && !failed;
  // ---- B-sets over the forward positions kf - 1 .. 1 (B[kf] = the meet set, stamped at meet)
  int mcur = L_M0;
  uint64_t nM = n_meet_items;
  for (int i = kf - 1; ok && i >= 1; --i) {
    PhaseView P{};
    P.op = OP_BSET;
    P.src = (uint32_t)mcur;
    P.dst = (uint32_t)(mcur == L_M0 ? L_M1 : L_M0);
    P.n = nM;
    P.pos = (uint32_t)i;
    P.stamp = stamp_of(Q.em, (uint32_t)i);
    phase_run(P, P.n > SP_SMALL);
    mcur = (int)P.dst;
    nM = sAcc[0];
    ok = !failed;
  }
  // ---- greedy reconstruction from s
  uint32_t c = Q.s;
  if (ok && threadIdx.x == 0) A.res->path[0] = A.vids[Q.s];
  for (int pos = 0; ok && pos < L; ++pos) {
    uint32_t deg = 0;
    if (!A.visible || A.visible[c])
      for (int t = 0; t < A.fwd.n; ++t) deg += A.fwd.row_ptr[t][c + 1] - A.fwd.row_ptr[t][c];
    PhaseView P{};
    P.op = OP_GREEDY;
    P.pos = (uint32_t)pos;
    P.cur = c;
    P.L = (uint32_t)L;
    P.kf = (uint32_t)kf;
    const bool big = deg > SP_GREEDY_SMALL && nwg > 1 && !failed;
    Cand mine{INT64_MAX, INT64_MAX, INT64_MAX, NO_ROW};
    if (big) {
      phase_run(P, true);
    } else {   // the leader alone: its block minimum is the answer
      mine = greedy_scan(A, Q, c, pos, L, kf, 0, 1, lds);
      if (threadIdx.x == 0) trace((unsigned long long)OP_GREEDY * 2);
    }
    if (threadIdx.x == 0) {
      Cand best = mine;
      for (int k = 0; big && k < nwg; ++k) {
        const unsigned long long* q = ctl->gpart + 4 * k;
        Cand x{(int64_t)ld1(q), (int64_t)ld1(q + 1), (int64_t)ld1(q + 2), (uint32_t)ld1(q + 3)};
        if (cand_less(x, best)) best = x;
      }
      lds[0] = best;
      if (best.d != NO_ROW) {
        A.res->path[1 + 3 * pos] = best.t;
        A.res->path[2 + 3 * pos] = best.r;
        A.res->path[3 + 3 * pos] = best.v;
      }
    }
    __syncthreads();
    c = lds[0].d;
    __syncthreads();
    if (c == NO_ROW) {
      ok = false;
      if (threadIdx.x == 0) atomicOr(&ctl->err.v, 1ull);
    }
  }
  // ---- result, release the followers
  if (threadIdx.x == 0) {
    A.res->L = ok ? (unsigned long long)L : 0ull;
    A.res->edges = edges;
    A.res->err = ld1(&ctl->err.v);
    A.res->levels = (unsigned long long)levels;
    trace(15);
    A.res->ntrace = ntr;
    if (nwg > 1) {   // EXIT: written through (sc1) and drained before the generation word
      st1(&ctl->op, (unsigned long long)OP_EXIT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      st1(&ctl->gen.v, g0 | ++phase);
    }
  }
}

// ---------------------------------------------------------------------------- host side
struct SpCtx {
  hipStream_t stream = nullptr;
  uint64_t nv = 0, cap = 0, edge_cap = 0;
  ChainCtx* chain = nullptr;       // the level-loop buffers (first SP_CHAIN query)
  int mode = SP_PERSISTENT;        // of the query in flight
  uint32_t* lab[3] = {};
  uint32_t epoch = 0;
  uint64_t* list[SP_NLISTS] = {};
  SpCtl* ctl = nullptr;
  SpResult* d_res = nullptr;
  SpResult* h_res = nullptr;
  hipEvent_t done = nullptr;
  unsigned long long q = 0;
  int wgs = 64;
  SpArgs* d_args = nullptr;        // the query's SpArgs in device memory
  SpArgs* h_args = nullptr;        // pinned staging
  SpArgs cached{};                 // what d_args holds
  bool args_valid = false;
  // NBG_SP_TRACE=1: per phase kind, launches and device ticks (printed by sp_destroy)
  bool tracing = false;
  double tick_us = 0.01;
  unsigned long long tr_n[16] = {}, tr_ticks[16] = {}, queries = 0, total_ticks = 0, sub[8] = {};
  double host_us = 0;              // level loop: host time enqueueing a query's chain
  unsigned long long host_n = 0;
  int prof = 0;                    // nbg_profile mode, applied to the chain when it is created
};

hipError_t sp_reserve_chain(SpCtx* c) {
  if (c->chain) return hipSuccess;
  std::string err;
  c->chain = chain_create(c->nv, c->edge_cap, c->stream, &err);
  if (!c->chain) return hipErrorOutOfMemory;
  if (c->prof) chain_profile(c->chain, c->prof);
  return hipSuccess;
}

void sp_profile(SpCtx* c, int mode) {
  if (!c) return;
  c->prof = mode;
  if (c->chain) chain_profile(c->chain, mode);
}

void sp_profile_accum(const SpCtx* c, double* launches, double* ms, double* bytes) {
  if (c && c->chain) chain_profile_accum(c->chain, launches, ms, bytes);
}

SpCtx* sp_create(uint64_t nv, uint64_t item_cap, uint64_t edge_cap, hipStream_t s, std::string* err) {
  auto* c = new SpCtx();
  c->stream = s;
  c->nv = nv;
  c->cap = item_cap;
  c->edge_cap = edge_cap;
  const char* e = getenv("NBG_SP_WGS");
  c->wgs = e ? std::max(1, std::min(SP_MAX_WGS, atoi(e))) : 64;
  c->tracing = getenv("NBG_SP_TRACE") && atoi(getenv("NBG_SP_TRACE")) != 0;
  {
    int dev = 0, khz = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) == hipSuccess && khz > 0)
      c->tick_us = 1000.0 / khz;
  }
  hipError_t he = hipSuccess;
  auto M = [&](void** p, size_t b) { if (he == hipSuccess) he = hipMalloc(p, b); };
  for (auto& l : c->lab) M((void**)&l, (nv + 1) * 4);
  M((void**)&c->ctl, sizeof(SpCtl));
  M((void**)&c->d_res, sizeof(SpResult));
  M((void**)&c->d_args, sizeof(SpArgs));
  if (he == hipSuccess) he = hipHostMalloc((void**)&c->h_args, sizeof(SpArgs), hipHostMallocDefault);
  if (he == hipSuccess) he = hipHostMalloc((void**)&c->h_res, sizeof(SpResult), hipHostMallocDefault);
  if (he == hipSuccess) he = hipEventCreateWithFlags(&c->done, hipEventDisableTiming);
  for (auto& l : c->lab)
    if (he == hipSuccess) he = hipMemsetAsync(l, 0, (nv + 1) * 4, s);
  if (he == hipSuccess) he = hipMemsetAsync(c->ctl, 0, sizeof(SpCtl), s);
  if (he == hipSuccess) he = hipStreamSynchronize(s);
  if (he != hipSuccess) {
    if (err) *err = std::string("shortest-path workspace: ") + hipGetErrorString(he);
    sp_destroy(c);
    return nullptr;
  }
  return c;
}

void sp_destroy(SpCtx* c) {
  if (!c) return;
  if (c->tracing && c->host_n)
    fprintf(stderr, "[sp trace] level loop: %llu queries, %.2f us host enqueue each\n", c->host_n,
            c->host_us / c->host_n);
  if (c->tracing && c->queries) {
    static const char* names[16] = {"launch", "setup", "level", "level*", "bset", "bset*", "greedy", "greedy*",
                                    "", "", "", "", "", "", "", "end"};
    fprintf(stderr, "[sp trace] %llu queries, %.2f us per query on the device (* = all workgroups)\n",
            c->queries, c->total_ticks * c->tick_us / c->queries);
    for (int k = 1; k < 16; ++k)
      if (c->tr_n[k])
        fprintf(stderr, "[sp trace]   %-8s %8llu phases  %8.2f us each  %8.2f us per query\n", names[k], c->tr_n[k],
                c->tr_ticks[k] * c->tick_us / c->tr_n[k], c->tr_ticks[k] * c->tick_us / c->queries);
    static const char* subs[8] = {"items+col", "labels", "claim", "rows", "reserve", "write", "tail", ""};
    for (int k = 0; k < 7; ++k)
      fprintf(stderr, "[sp trace]   leader %-9s %8.2f us per query\n", subs[k],
              (c->sub[k] & ((1ull << 40) - 1)) * c->tick_us / c->queries);
    fprintf(stderr, "[sp trace]   leader passes %.1f, hub lanes %.1f per query\n", (double)c->sub[7] / c->queries,
            (double)(c->sub[6] >> 40) / c->queries);
  }
  for (auto* l : c->lab)
    if (l) (void)hipFree(l);
  for (auto* l : c->list)
    if (l) (void)hipFree(l);
  chain_destroy(c->chain);
  if (c->ctl) (void)hipFree(c->ctl);
  if (c->d_args) (void)hipFree(c->d_args);
  if (c->h_args) (void)hipHostFree(c->h_args);
  if (c->d_res) (void)hipFree(c->d_res);
  if (c->h_res) (void)hipHostFree(c->h_res);
  if (c->done) (void)hipEventDestroy(c->done);
  delete c;
}

hipError_t sp_launch(SpCtx* c, int mode, const SpTypes& fwd, const SpTypes& bwd, const uint8_t* visible,
                     const int64_t* vids, uint32_t s, uint32_t t, uint32_t upto) {
  if (upto > MAX_PATH_LEN || s == NO_ROW || t == NO_ROW) return hipErrorInvalidValue;
  if (++c->epoch >= (1u << (32 - LVL_BITS))) {   // wrap: clear the labels once
    for (auto* l : c->lab) HIP_TRY_SP(hipMemsetAsync(l, 0, (c->nv + 1) * 4, c->stream));
    c->epoch = 1;
  }
  c->mode = mode;
  if (mode == SP_CHAIN) {
    if (!c->chain) {
      std::string err;
      c->chain = chain_create(c->nv, c->edge_cap, c->stream, &err);
      if (!c->chain) return hipErrorOutOfMemory;
      if (c->prof) chain_profile(c->chain, c->prof);
    }
    const auto t0 = std::chrono::steady_clock::now();
    HIP_TRY_SP(chain_launch(c->chain, fwd, bwd, visible, vids, c->lab, c->epoch, s, t, upto));
    const hipError_t e = hipEventRecord(c->done, c->stream);
    if (c->tracing) {
      c->host_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
      ++c->host_n;
    }
    return e;
  }
  if (!c->list[0]) {
    HIP_TRY_SP(hipStreamSynchronize(c->stream));
    for (auto& l : c->list) HIP_TRY_SP(hipMalloc((void**)&l, std::max<uint64_t>(c->cap, 1) * 8));
  }
  SpArgs a;
  memset(&a, 0, sizeof(a));   // compared bytewise: no indeterminate padding
  a.fwd = fwd;
  a.bwd = bwd;
  a.visible = visible;
  a.vids = vids;
  a.lab_f = c->lab[0];
  a.lab_b = c->lab[1];
  a.lab_m = c->lab[2];
  for (int i = 0; i < SP_NLISTS; ++i) a.list[i] = c->list[i];
  a.list_cap = c->cap;
  a.ctl = c->ctl;
  a.res = c->d_res;
  if (!c->args_valid || memcmp(&a, &c->cached, sizeof(a)) != 0) {
    // the staging buffer may still feed an earlier upload: drain the stream first (rare)
    HIP_TRY_SP(hipStreamSynchronize(c->stream));
    memcpy(c->h_args, &a, sizeof(a));
    HIP_TRY_SP(hipMemcpyAsync(c->d_args, c->h_args, sizeof(a), hipMemcpyHostToDevice, c->stream));
    c->cached = a;
    c->args_valid = true;
  }
  SpQ q{};
  q.s = s;
  q.t = t;
  q.upto = upto;
  q.ef = q.eb = q.em = c->epoch;
  q.q = ++c->q;
  q.spin_limit = 1ull << 24;   // ~10 s of polling: a stuck phase ends the query with err = 2
  hipLaunchKernelGGL(k_sp_pair, dim3((unsigned)c->wgs), dim3(SP_THREADS), 0, c->stream, (const SpArgs*)c->d_args, q);
  HIP_TRY_SP(hipGetLastError());
  HIP_TRY_SP(hipMemcpyAsync(c->h_res, c->d_res, sizeof(SpResult), hipMemcpyDeviceToHost, c->stream));
  return hipEventRecord(c->done, c->stream);
}

// n one-pair queries on n slots that share one stream, as one batched chain (spchain.hip); each
// slot's sp_wait then completes its own query.
hipError_t sp_launch_batch(SpCtx* const* cs, int n, const SpPair* pairs) {
  if (n < 1) return hipSuccess;
  std::vector<ChainCtx*> chains(n);
  std::vector<ChainQuery> qs(n);
  for (int p = 0; p < n; ++p) {
    SpCtx* c = cs[p];
    const SpPair& x = pairs[p];
    if (x.upto > MAX_PATH_LEN || x.s == NO_ROW || x.t == NO_ROW || c->stream != cs[0]->stream) return hipErrorInvalidValue;
    if (++c->epoch >= (1u << (32 - LVL_BITS))) {
      for (auto* l : c->lab) HIP_TRY_SP(hipMemsetAsync(l, 0, (c->nv + 1) * 4, c->stream));
      c->epoch = 1;
    }
    c->mode = SP_CHAIN;
    if (!c->chain) {
      std::string err;
      c->chain = chain_create(c->nv, c->edge_cap, c->stream, &err);
      if (!c->chain) return hipErrorOutOfMemory;
      if (c->prof) chain_profile(c->chain, c->prof);
    }
    chains[p] = c->chain;
    qs[p] = ChainQuery{x.fwd, x.bwd, x.visible, x.vids, c->lab, c->epoch, x.s, x.t, x.upto};
  }
  HIP_TRY_SP(chain_launch_batch(chains.data(), n, qs.data()));
  for (int p = 0; p < n; ++p) HIP_TRY_SP(hipEventRecord(cs[p]->done, cs[p]->stream));
  return hipSuccess;
}

bool sp_ready(SpCtx* c) { return hipEventQuery(c->done) == hipSuccess; }

hipError_t sp_wait(SpCtx* c, SpResult* out) {
  hipError_t e;
  while ((e = hipEventQuery(c->done)) == hipErrorNotReady) {
  }
  if (e != hipSuccess) return e;
  if (c->mode == SP_CHAIN) {
    while (!chain_more(c->chain, &e)) {   // a continuation batch: wait for it too
      if (e == hipSuccess) e = hipEventRecord(c->done, c->stream);
      if (e != hipSuccess) return e;
      while ((e = hipEventQuery(c->done)) == hipErrorNotReady) {
      }
      if (e != hipSuccess) return e;
    }
    chain_result(c->chain, out);
    chain_profile_done(c->chain, *out);
    return hipSuccess;
  }
  memcpy(out, c->h_res, sizeof(SpResult));
  if (c->tracing && out->ntrace >= 2) {
    const unsigned long long mask = (1ull << 56) - 1;
    unsigned long long prev = out->trace[0] & mask;
    for (unsigned long long i = 1; i < out->ntrace && i < 40; ++i) {
      const unsigned long long k = out->trace[i] >> 56, t = out->trace[i] & mask;
      c->tr_n[k & 15] += 1;
      c->tr_ticks[k & 15] += t - prev;
      prev = t;
    }
    c->total_ticks += prev - (out->trace[0] & mask);
    for (int k = 0; k < 8; ++k) c->sub[k] += out->sub[k];
    ++c->queries;
  }
  return hipSuccess;
}

}  // namespace nbg
