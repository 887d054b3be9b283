// FIND SHORTEST PATH for one (source, target) pair as a DEVICE-DRIVEN LEVEL LOOP (single engine).
//
// Same semantics and result as path.cpp's bidirectional() (FindPathExecutor.cpp:173-290
// restated: minimal hop count, UPTO N, one path per target, ties broken by the lexicographically
// smallest entry list [v0, t0, r0, v1, ...]).  The host enqueues a FIXED chain per pair —
//   k_ch_setup, UPTO x k_ch_level(BFS), UPTO-1 x k_ch_level(B-set), UPTO x k_ch_hop, one copy —
// and waits once.  Every launch reads what it has to do (the direction, the frontier list, its
// stamps, whether the search is over) from a device state block (ChState) that the LAST
// workgroup of the previous launch wrote (ticket counter), so no launch waits for the host and
// launches past the end of the search return at once.
//
// Frontier lists carry their edge space (the packed-atomic protocol of kernels.hip's lists):
// entry i = vertex ids[i], its edges at positions [seg_end[i] - deg, seg_end[i]) of the list's
// edge space starting at CSR row seg_rs[i], plus the merge-path split of every TILE boundary
// (tsplit).  A vertex is appended with its edge space when it is CLAIMED (CAS on its label), so
// a level is one launch: merge-path tiles over (entries + edges), neighbour gather, claims,
// appends.  One OVER type per direction (path.cpp sends other requests to the host loop).
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstring>
#include <string>

#include "nbg_internal.h"

#define HIP_TRY_CH(x)                     \
  do {                                    \
    hipError_t e_ = (x);                  \
    if (e_ != hipSuccess) return e_;      \
  } while (0)

namespace nbg {
namespace {

constexpr int CH_BLOCK = 256;
constexpr int CH_WAVES = CH_BLOCK / 64;
constexpr int CH_VT = 8;                  // merge-path items per lane per tile
constexpr int CH_TILE = 64 * CH_VT;       // items (entries + edges) per wave tile
constexpr int CH_HOP_WGS = 64;            // workgroups scanning one greedy hop
constexpr int CH_HOP_U = 4;               // neighbours per thread in flight (greedy)

enum ChListId : int { CL_F0 = 0, CL_F1 = 1, CL_B0 = 2, CL_B1 = 3, CL_M = 4, CH_NLISTS = 5 };
// B-set lists reuse the forward lists (the forward frontier is dead once the sides met)
constexpr int CL_S0 = CL_F0;

}  // namespace

struct ChList {
  uint32_t* ids;
  uint32_t* seg_end;    // inclusive edge prefix of the list
  uint32_t* seg_rs;     // CSR row start
  uint32_t* tsplit;     // merge-path split per tile
};

struct ChState {        // device; the prefix up to gpart is copied back per query
  unsigned long long acc[CH_NLISTS];   // packed (entries << 32 | edges) per list
  unsigned long long meets;            // meet vertices of the meeting level
  unsigned long long ticket;           // workgroups done (the last one does the bookkeeping)
  unsigned long long edges;            // BFS edges expanded
  unsigned long long err;              // 1 reconstruction failure, 3 list overflow
  unsigned long long levels;
  unsigned long long gticket, gv;      // greedy hop: workgroups done, current vertex
  unsigned long long ds[2];            // edge totals of the current forward / backward frontier
  uint32_t cur[2], kf, kb, done, met, L, dir;
  long long path[1 + 3 * MAX_PATH_LEN];
  unsigned long long gpart[4 * CH_HOP_WGS];
};

struct ChArgs {         // device memory (indexed at run time: never a by-value kernel argument)
  const uint32_t* row_ptr[2];          // [0] forward (out-edges), [1] backward (in-edges)
  const uint32_t* col[2];
  const int64_t* dst_vid;              // forward: greedy candidates
  const int64_t* rank;
  int64_t type;
  const uint8_t* visible;
  const int64_t* vids;
  uint32_t* lab[3];                    // forward, backward, B-set (LAB_M)
  ChList list[CH_NLISTS];
  uint64_t list_cap, tsplit_cap;
  ChState* st;
};

struct ChQ {
  uint32_t s, t, upto;
  uint32_t ef, eb, em;
};

namespace {

__device__ __forceinline__ uint32_t stamp_of(uint32_t epoch, uint32_t level) { return (epoch << LVL_BITS) | level; }
__device__ __forceinline__ bool live(uint32_t lab, uint32_t epoch) { return (lab >> LVL_BITS) == epoch; }
__device__ __forceinline__ unsigned long long ld_agent(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint32_t scan_incl(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}

// degree of v over direction `side` (0 for an invisible vertex), *rs its row start
__device__ __forceinline__ uint32_t vdeg(const ChArgs& A, int side, uint32_t v, uint32_t* rs) {
  if (v == NO_ROW || (A.visible && !A.visible[v])) {
    *rs = 0;
    return 0;
  }
  const uint32_t r = A.row_ptr[side][v];
  *rs = r;
  return A.row_ptr[side][v + 1] - r;
}

// Entry pos of list L: vertex v, its deg edges ending at edge offset end, from row rs; the tile
// boundaries its merge-path range [pos + end - deg, pos + end] covers get their split.
__device__ __forceinline__ void list_put(const ChArgs& A, const ChList& L, uint32_t pos, uint32_t v, uint32_t end,
                                         uint32_t deg, uint32_t rs) {
  L.ids[pos] = v;
  L.seg_end[pos] = end;
  L.seg_rs[pos] = rs;
  const uint64_t lo = (uint64_t)pos + end - deg, hi = (uint64_t)pos + end;
  for (uint64_t t = (lo + CH_TILE - 1) / CH_TILE; t * CH_TILE <= hi && t < A.tsplit_cap; ++t) L.tsplit[t] = pos;
}

// Appends, per lane, the vertices x[i] with bit i of `m` and a nonzero degree (dg[i], rs[i]) to
// list `li`: one packed atomic per wave for positions and edge offsets.
__device__ __forceinline__ void wave_append(const ChArgs& A, int li, const uint32_t (&x)[CH_VT], uint32_t m,
                                            const uint32_t (&dg)[CH_VT], const uint32_t (&rs)[CH_VT]) {
  const int lane = threadIdx.x & 63;
  uint32_t c = 0, d = 0;
#pragma unroll
  for (int i = 0; i < CH_VT; ++i)
    if (((m >> i) & 1u) && dg[i]) {
      ++c;
      d += dg[i];
    }
  const uint32_t ic = scan_incl(c), id = scan_incl(d);
  const uint32_t tc = __shfl(ic, 63, 64), td = __shfl(id, 63, 64);
  if (!tc) return;   // wave-uniform
  unsigned long long old = 0;
  if (lane == 0) old = atomicAdd(&A.st->acc[li], ((unsigned long long)tc << 32) | td);
  old = __shfl(old, 0, 64);
  if ((old >> 32) + tc > A.list_cap) {
    if (lane == 0) atomicOr(&A.st->err, 3ull);
    return;
  }
  uint32_t pos = (uint32_t)(old >> 32) + ic - c;
  uint32_t end = (uint32_t)old + id - d;
  const ChList L = A.list[li];
#pragma unroll
  for (int i = 0; i < CH_VT; ++i)
    if (((m >> i) & 1u) && dg[i]) {
      end += dg[i];
      list_put(A, L, pos++, x[i], end, dg[i], rs[i]);
    }
}

// The last workgroup of a launch to finish (ticket) gets true, with the other workgroups'
// writes visible.
__device__ __forceinline__ bool last_workgroup(unsigned long long* ticket) {
  __shared__ int s_last;
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    s_last = atomicAdd(ticket, 1ull) == gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last) return false;
  __threadfence();
  return true;
}

}  // namespace

// Set-up (one workgroup): the state block, the labels of s and t, the one-entry lists {s}, {t}.
__global__ void __launch_bounds__(CH_BLOCK) k_ch_setup(const ChArgs* __restrict__ Ap, ChQ q) {
  const ChArgs& A = *Ap;
  ChState* st = A.st;
  uint32_t rsf, rsb;
  const uint32_t dsf = vdeg(A, 0, q.s, &rsf), dsb = vdeg(A, 1, q.t, &rsb);
  for (uint64_t t = threadIdx.x; t * CH_TILE <= dsf && t < A.tsplit_cap; t += CH_BLOCK) A.list[CL_F0].tsplit[t] = 0;
  for (uint64_t t = threadIdx.x; t * CH_TILE <= dsb && t < A.tsplit_cap; t += CH_BLOCK) A.list[CL_B0].tsplit[t] = 0;
  if (threadIdx.x != 0) return;
  for (int i = 0; i < CH_NLISTS; ++i) st->acc[i] = 0;
  st->meets = st->ticket = st->edges = st->err = st->levels = st->gticket = 0;
  st->cur[0] = st->cur[1] = 0;
  st->kf = st->kb = st->met = st->L = 0;
  st->ds[0] = dsf;
  st->ds[1] = dsb;
  st->dir = dsf <= dsb ? 0u : 1u;
  st->done = !dsf || !dsb;
  A.lab[0][q.s] = stamp_of(q.ef, 0);
  A.lab[1][q.t] = stamp_of(q.eb, 0);
  if (dsf) {
    const ChList& F = A.list[CL_F0];
    F.ids[0] = q.s;
    F.seg_end[0] = dsf;
    F.seg_rs[0] = rsf;
    st->acc[CL_F0] = (1ull << 32) | dsf;
  }
  if (dsb) {
    const ChList& B = A.list[CL_B0];
    B.ids[0] = q.t;
    B.seg_end[0] = dsb;
    B.seg_rs[0] = rsb;
    st->acc[CL_B0] = (1ull << 32) | dsb;
  }
  st->gv = q.s;
  st->path[0] = A.vids[q.s];
}

// One level: mode 0 = the next BFS level (side from ChState::dir), mode 1 = B-set step k
// (B[kf - 1 - k] from B[kf - k] through in-edges, restricted to forward level kf - 1 - k).
__global__ void __launch_bounds__(CH_BLOCK) k_ch_level(const ChArgs* __restrict__ Ap, ChQ q, int mode, int k) {
  __shared__ uint32_t sEndAll[CH_WAVES][CH_TILE + 2];
  __shared__ uint32_t sRsAll[CH_WAVES][CH_TILE + 1];
  __shared__ uint16_t sSegAll[CH_WAVES][CH_TILE];
  const ChArgs& A = *Ap;
  ChState* st = A.st;
  const bool bfs = mode == 0;
  // ---- what this launch does (every workgroup reads the same state: uniform)
  const uint32_t kf = st->kf, kb = st->kb;
  int side, src, dst;
  uint32_t* lab;
  uint32_t epoch = 0, stamp, oepoch = 0, mstamp = 0, rstamp = 0;
  const uint32_t* olab = nullptr;
  const uint32_t* rlab = nullptr;
  bool append = true;
  if (bfs) {
    if (st->done) return;
    side = (int)st->dir;
    src = side * 2 + (int)st->cur[side];
    dst = src ^ 1;
    lab = A.lab[side];
    epoch = side ? q.eb : q.ef;
    stamp = stamp_of(epoch, (side ? kb : kf) + 1);
    olab = A.lab[side ^ 1];
    oepoch = side ? q.ef : q.eb;
    mstamp = stamp_of(q.em, side ? kf : kf + 1);
  } else {
    if (!st->met || kf < 2u + (uint32_t)k) return;
    const uint32_t pos = kf - 1 - (uint32_t)k;
    side = 1;
    src = k == 0 ? CL_M : CL_S0 + ((k - 1) & 1);
    dst = CL_S0 + (k & 1);
    lab = A.lab[2];
    epoch = q.em;   // (as the host loop: a vertex with any B-set stamp of this query is taken)
    stamp = stamp_of(q.em, pos);
    rlab = A.lab[0];
    rstamp = stamp_of(q.ef, pos);
    append = pos >= 2;   // B[1]'s in-edges are not needed (B[0] = {s})
  }
  const unsigned long long packed = st->acc[src];
  const uint64_t n = packed >> 32, total = packed & 0xFFFFFFFFull;
  const ChList S = A.list[src];
  const uint32_t* __restrict__ col = A.col[side];
  const uint64_t npath = n + total, ntiles = (npath + CH_TILE - 1) / CH_TILE;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t* const sEnd = sEndAll[w];
  uint32_t* const sRs = sRsAll[w];
  uint16_t* const sSeg = sSegAll[w];
  for (uint64_t t = (uint64_t)blockIdx.x * CH_WAVES + w; t < ntiles; t += (uint64_t)gridDim.x * CH_WAVES) {
    uint64_t sp = 0;
    if (lane == 0) sp = S.tsplit[t];
    if (lane == 1) sp = (t + 1) * CH_TILE >= npath ? n : S.tsplit[t + 1];
    const uint64_t a0 = uniform64(__shfl(sp, 0, 64)), a1 = uniform64(__shfl(sp, 1, 64));
    const uint64_t d0 = t * CH_TILE, d1 = d0 + CH_TILE < npath ? d0 + CH_TILE : npath;
    const uint64_t b0 = d0 - a0, b1 = d1 - a1;
    const int na = (int)(a1 - a0), nb = (int)(b1 - b0);
    // the tile's window: sEnd[k] = seg_end[a0 - 1 + k], sRs[k] = seg_rs[a0 + k]
    for (int kk = lane; kk <= na + 1; kk += 64) {
      const int64_t i = (int64_t)a0 - 1 + kk;
      sEnd[kk] = i < 0 ? 0u : (i < (int64_t)n ? S.seg_end[i] : 0xFFFFFFFFu);
      if (kk <= na) sRs[kk] = (uint64_t)(i + 1) < n ? S.seg_rs[i + 1] : 0u;
    }
    wave_lds_sync();
    const uint32_t* Aend = sEnd + 1;   // Aend[j] = end of entry a0 + j
    {   // lane-level merge path: the entry of every edge item
      const int diag = lane * CH_VT, dmax = na + nb;
      if (diag < dmax) {
        int lo = diag > nb ? diag - nb : 0, hi = diag < na ? diag : na;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if ((uint64_t)Aend[mid] <= b0 + (uint64_t)(diag - 1 - mid)) lo = mid + 1;
          else hi = mid;
        }
        int ai = lo, bi = diag - lo;
#pragma unroll
        for (int kk = 0; kk < CH_VT; ++kk) {
          if (ai + bi >= dmax) break;
          if (ai < na && (bi >= nb || (uint64_t)Aend[ai] <= b0 + (uint64_t)bi)) {
            ++ai;
          } else {
            sSeg[bi] = (uint16_t)ai;
            ++bi;
          }
        }
      }
    }
    wave_lds_sync();
    // neighbours, all loads in flight together
    uint32_t x[CH_VT];
#pragma unroll
    for (int i = 0; i < CH_VT; ++i) {
      const int kk = i * 64 + lane;
      x[i] = NO_ROW;
      if (kk < nb) {
        const uint32_t s = sSeg[kk];
        x[i] = col[(uint64_t)sRs[s] + (b0 + kk - (uint64_t)sEnd[s])];
      }
    }
    uint32_t old[CH_VT], gate[CH_VT];
#pragma unroll
    for (int i = 0; i < CH_VT; ++i) {
      old[i] = x[i] != NO_ROW ? lab[x[i]] : 0u;
      gate[i] = (x[i] != NO_ROW && rlab) ? rlab[x[i]] : rstamp;
    }
    wave_lds_sync();   // (the next tile rewrites the window)
    uint32_t cm = 0;
#pragma unroll
    for (int i = 0; i < CH_VT; ++i) {
      if (x[i] == NO_ROW || gate[i] != rstamp) continue;
      if (live(old[i], epoch)) continue;
      if (atomicCAS(lab + x[i], old[i], stamp) != old[i]) continue;
      cm |= 1u << i;
    }
    if (!__ballot(cm != 0)) continue;
    uint32_t mm = 0;
    if (bfs) {
      uint32_t ol[CH_VT];
#pragma unroll
      for (int i = 0; i < CH_VT; ++i) ol[i] = ((cm >> i) & 1u) ? olab[x[i]] : 0u;
#pragma unroll
      for (int i = 0; i < CH_VT; ++i)
        if (((cm >> i) & 1u) && live(ol[i], oepoch)) mm |= 1u << i;
    }
    if (append) {
      uint32_t dg[CH_VT], rs[CH_VT];
#pragma unroll
      for (int i = 0; i < CH_VT; ++i) dg[i] = ((cm >> i) & 1u) ? vdeg(A, side, x[i], &rs[i]) : (rs[i] = 0, 0u);
      wave_append(A, dst, x, cm, dg, rs);
    }
    if (__ballot(mm != 0)) {   // the sides met: LAB_M stamps, the meet list over in-edges
      uint32_t dg[CH_VT], rs[CH_VT];
      uint32_t nm = 0;
#pragma unroll
      for (int i = 0; i < CH_VT; ++i) {
        dg[i] = 0;
        rs[i] = 0;
        if ((mm >> i) & 1u) {
          A.lab[2][x[i]] = mstamp;
          dg[i] = vdeg(A, 1, x[i], &rs[i]);
          ++nm;
        }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) nm += __shfl_xor(nm, o, 64);
      if (lane == 0) atomicAdd(&st->meets, (unsigned long long)nm);
      wave_append(A, CL_M, x, mm, dg, rs);
    }
  }
  // ---- bookkeeping by the last workgroup: the next launch's parameters
  if (!last_workgroup(&st->ticket) || threadIdx.x != 0) return;
  st->ticket = 0;
  if (!bfs) {
    if (k >= 1) st->acc[src] = 0;   // the list the next B-set step appends to
    return;
  }
  const unsigned long long nn = ld_agent(&st->acc[dst]);
  const uint32_t nkf = kf + (side == 0), nkb = kb + (side == 1);
  st->cur[side] ^= 1u;
  st->acc[src] = 0;   // this side's next level appends here
  st->kf = nkf;
  st->kb = nkb;
  const unsigned long long ds = nn & 0xFFFFFFFFull, dso = st->ds[side ^ 1];
  st->ds[side] = ds;
  st->edges += total;
  st->levels += 1;
  const unsigned long long err = ld_agent(&st->err);
  if (err) {
    st->done = 1;
  } else if (ld_agent(&st->meets)) {
    st->met = 1;
    st->L = nkf + nkb;
    st->done = 1;
    st->acc[CL_F0] = st->acc[CL_F1] = 0;   // the B-set lists
  } else if ((nn >> 32) == 0 || nkf + nkb >= q.upto) {
    st->done = 1;   // a side has no further edges, or UPTO reached: no path
  }
  st->dir = (side == 0 ? ds <= dso : dso <= ds) ? 0u : 1u;
}

// Greedy hop pos (CH_HOP_WGS workgroups): the minimum (type, rank, dst vid) out-edge of the
// current vertex into B[pos + 1]; the last workgroup reduces, records the hop, moves on.
__global__ void __launch_bounds__(CH_BLOCK) k_ch_hop(const ChArgs* __restrict__ Ap, ChQ q, int pos) {
  struct Cand {
    int64_t t, r, v;
    uint32_t d;
  };
  __shared__ Cand lds[CH_WAVES + 1];
  const ChArgs& A = *Ap;
  ChState* st = A.st;
  if (!st->met || (uint32_t)pos >= st->L || st->err) return;
  const uint32_t c = (uint32_t)st->gv, L = st->L, kf = st->kf;
  auto less = [](const Cand& a, const Cand& b) {
    if (a.t != b.t) return a.t < b.t;
    if (a.r != b.r) return a.r < b.r;
    return a.v < b.v;
  };
  const Cand none{INT64_MAX, INT64_MAX, INT64_MAX, NO_ROW};
  Cand best = none;
  const bool by_m = (uint32_t)pos + 1 <= kf;
  const uint32_t* vlab = by_m ? A.lab[2] : A.lab[1];
  const uint32_t want = by_m ? stamp_of(q.em, (uint32_t)pos + 1) : stamp_of(q.eb, L - (uint32_t)pos - 1);
  if (c != NO_ROW && (!A.visible || A.visible[c])) {
    const uint32_t rs = A.row_ptr[0][c], re = A.row_ptr[0][c + 1];
    const uint64_t g = (uint64_t)blockIdx.x * CH_BLOCK + threadIdx.x, G = (uint64_t)gridDim.x * CH_BLOCK;
    for (uint64_t j0 = rs + g; j0 < re; j0 += CH_HOP_U * G) {
      uint32_t wv[CH_HOP_U], lv[CH_HOP_U];
#pragma unroll
      for (int u = 0; u < CH_HOP_U; ++u) wv[u] = j0 + u * G < re ? A.col[0][j0 + u * G] : NO_ROW;
#pragma unroll
      for (int u = 0; u < CH_HOP_U; ++u) lv[u] = wv[u] != NO_ROW ? vlab[wv[u]] : 0u;
#pragma unroll
      for (int u = 0; u < CH_HOP_U; ++u) {
        if (wv[u] == NO_ROW || lv[u] != want) continue;
        const uint64_t j = j0 + u * G;
        const Cand x{A.type, A.rank ? A.rank[j] : 0, A.dst_vid[j], wv[u]};
        if (less(x, best)) best = x;
      }
    }
  }
  auto block_min = [&](Cand b) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      Cand y;
      y.t = __shfl_down(b.t, o, 64);
      y.r = __shfl_down(b.r, o, 64);
      y.v = __shfl_down(b.v, o, 64);
      y.d = __shfl_down(b.d, o, 64);
      if ((threadIdx.x & 63) + o < 64 && less(y, b)) b = y;
    }
    if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = b;
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int i = 1; i < CH_WAVES; ++i)
        if (less(lds[i], b)) b = lds[i];
      lds[CH_WAVES] = b;
    }
    __syncthreads();
    b = lds[CH_WAVES];
    __syncthreads();
    return b;
  };
  best = block_min(best);
  if (threadIdx.x == 0) {
    unsigned long long* part = st->gpart + 4 * blockIdx.x;
    part[0] = (unsigned long long)best.t;
    part[1] = (unsigned long long)best.r;
    part[2] = (unsigned long long)best.v;
    part[3] = best.d;
  }
  if (!last_workgroup(&st->gticket)) return;
  Cand r = none;
  if (threadIdx.x < gridDim.x) {
    const unsigned long long* p = st->gpart + 4 * threadIdx.x;
    r = Cand{(int64_t)ld_agent(p), (int64_t)ld_agent(p + 1), (int64_t)ld_agent(p + 2), (uint32_t)ld_agent(p + 3)};
  }
  r = block_min(r);
  if (threadIdx.x != 0) return;
  st->gticket = 0;
  if (r.d == NO_ROW) {
    st->err |= 1ull;
    st->gv = NO_ROW;
    return;
  }
  st->path[1 + 3 * pos] = r.t;
  st->path[2 + 3 * pos] = r.r;
  st->path[3 + 3 * pos] = r.v;
  st->gv = r.d;
}

// ---------------------------------------------------------------------------- host side
struct ChainCtx {
  hipStream_t stream = nullptr;
  uint64_t nv = 0, list_cap = 0, tsplit_cap = 0;
  ChList list[CH_NLISTS] = {};
  ChState* d_st = nullptr;
  ChState* h_st = nullptr;
  ChArgs* d_args = nullptr;
  ChArgs* h_args = nullptr;
  ChArgs cached{};
  bool args_valid = false;
  unsigned grid = 512;
};

static constexpr size_t CH_COPY = offsetof(ChState, gpart);

ChainCtx* chain_create(uint64_t nv, uint64_t edge_cap, hipStream_t s, std::string* err) {
  auto* c = new ChainCtx();
  c->stream = s;
  c->nv = nv;
  c->list_cap = nv + 1;
  c->tsplit_cap = (nv + 1 + edge_cap) / CH_TILE + 2;
  const char* g = getenv("NBG_SP_GRID");
  if (g && atoi(g) > 0) c->grid = (unsigned)atoi(g);
  hipError_t he = hipSuccess;
  auto M = [&](void** p, size_t b) { if (he == hipSuccess) he = hipMalloc(p, b); };
  for (auto& L : c->list) {
    M((void**)&L.ids, c->list_cap * 4);
    M((void**)&L.seg_end, c->list_cap * 4);
    M((void**)&L.seg_rs, c->list_cap * 4);
    M((void**)&L.tsplit, c->tsplit_cap * 4);
  }
  M((void**)&c->d_st, sizeof(ChState));
  M((void**)&c->d_args, sizeof(ChArgs));
  if (he == hipSuccess) he = hipHostMalloc((void**)&c->h_st, sizeof(ChState), hipHostMallocDefault);
  if (he == hipSuccess) he = hipHostMalloc((void**)&c->h_args, sizeof(ChArgs), hipHostMallocDefault);
  if (he == hipSuccess) he = hipMemsetAsync(c->d_st, 0, sizeof(ChState), s);
  if (he == hipSuccess) he = hipStreamSynchronize(s);
  if (he != hipSuccess) {
    if (err) *err = std::string("shortest-path level-loop workspace: ") + hipGetErrorString(he);
    chain_destroy(c);
    return nullptr;
  }
  return c;
}

void chain_destroy(ChainCtx* c) {
  if (!c) return;
  for (auto& L : c->list)
    for (uint32_t* p : {L.ids, L.seg_end, L.seg_rs, L.tsplit})
      if (p) (void)hipFree(p);
  if (c->d_st) (void)hipFree(c->d_st);
  if (c->d_args) (void)hipFree(c->d_args);
  if (c->h_st) (void)hipHostFree(c->h_st);
  if (c->h_args) (void)hipHostFree(c->h_args);
  delete c;
}

hipError_t chain_launch(ChainCtx* c, const SpTypes& fwd, const SpTypes& bwd, const uint8_t* visible,
                        const int64_t* vids, uint32_t* const lab[3], uint32_t epoch, uint32_t s, uint32_t t,
                        uint32_t upto) {
  if (fwd.n != 1 || bwd.n != 1 || upto < 1 || upto > MAX_PATH_LEN) return hipErrorInvalidValue;
  ChArgs a;
  memset(&a, 0, sizeof(a));   // compared bytewise: no indeterminate padding
  a.row_ptr[0] = fwd.row_ptr[0];
  a.row_ptr[1] = bwd.row_ptr[0];
  a.col[0] = fwd.col[0];
  a.col[1] = bwd.col[0];
  a.dst_vid = fwd.dst_vid[0];
  a.rank = fwd.rank[0];
  a.type = fwd.type[0];
  a.visible = visible;
  a.vids = vids;
  for (int i = 0; i < 3; ++i) a.lab[i] = lab[i];
  for (int i = 0; i < CH_NLISTS; ++i) a.list[i] = c->list[i];
  a.list_cap = c->list_cap;
  a.tsplit_cap = c->tsplit_cap;
  a.st = c->d_st;
  if (!c->args_valid || memcmp(&a, &c->cached, sizeof(a)) != 0) {
    HIP_TRY_CH(hipStreamSynchronize(c->stream));   // the staging buffer may still feed an earlier upload
    memcpy(c->h_args, &a, sizeof(a));
    HIP_TRY_CH(hipMemcpyAsync(c->d_args, c->h_args, sizeof(a), hipMemcpyHostToDevice, c->stream));
    c->cached = a;
    c->args_valid = true;
  }
  const ChArgs* A = c->d_args;
  const ChQ q{s, t, upto, epoch, epoch, epoch};
  hipLaunchKernelGGL(k_ch_setup, dim3(1), dim3(CH_BLOCK), 0, c->stream, A, q);
  for (uint32_t i = 0; i < upto; ++i)
    hipLaunchKernelGGL(k_ch_level, dim3(c->grid), dim3(CH_BLOCK), 0, c->stream, A, q, 0, (int)i);
  for (uint32_t k = 0; k + 2 <= upto; ++k)   // B-set steps: kf - 1 - k >= 1 needs kf >= k + 2
    hipLaunchKernelGGL(k_ch_level, dim3(c->grid), dim3(CH_BLOCK), 0, c->stream, A, q, 1, (int)k);
  for (uint32_t p = 0; p < upto; ++p)
    hipLaunchKernelGGL(k_ch_hop, dim3(CH_HOP_WGS), dim3(CH_BLOCK), 0, c->stream, A, q, (int)p);
  HIP_TRY_CH(hipGetLastError());
  return hipMemcpyAsync(c->h_st, c->d_st, CH_COPY, hipMemcpyDeviceToHost, c->stream);
}

// the copied state -> SpResult (after the stream reached the copy)
void chain_result(const ChainCtx* c, SpResult* out) {
  const ChState& h = *c->h_st;
  out->err = h.err;
  out->edges = h.edges;
  out->levels = h.levels;
  out->L = (h.met && !h.err) ? h.L : 0;
  out->ntrace = 0;
  if (out->L) memcpy(out->path, h.path, (1 + 3 * (size_t)out->L) * sizeof(long long));
}

}  // namespace nbg
