// FIND SHORTEST PATH for one (source, target) pair as a DEVICE-DRIVEN LEVEL LOOP (single engine).
//
// Same semantics and result as path.cpp's bidirectional() (FindPathExecutor.cpp:173-290
// restated: minimal hop count, UPTO N, one path per target, ties broken by the lexicographically
// smallest entry list [v0, t0, r0, v1, ...]).  The host enqueues a chain per pair —
//   K x k_ch_step (the first starts the search; the last stores the result into mapped host
//   memory), plus k_ch_hop launches only when a continuation needs them —
// and waits once.  Step launch i derives what it does from the state snapshot of launch i - 1
// (snap[i - 1]) and that launch's results (its output-list and meet counters, lacc / lmeet[i - 1]),
// which are final at the launch boundary: the BFS level loop (direction = the side with the
// smaller edge total, meet / empty / UPTO tests), then the B-set steps, and once the search is
// over the greedy path walk (a launch finding nothing left returns at once).  Workgroup 0 stores
// the derived snapshot for launch i + 1, so no launch waits for the host or for a last-workgroup
// ticket.  K follows the recent queries (launches used); a query that needs more gets a
// continuation batch.
//
// Frontier lists carry their edge space (the packed-atomic protocol of kernels.hip's lists):
// entry i = vertex ids[i], its edges at positions [seg_end[i] - deg, seg_end[i]) of the list's
// edge space starting at CSR row seg_rs[i], plus the merge-path split of every TILE boundary
// (tsplit).  A vertex is appended with its edge space when it is CLAIMED (CAS on its label), so
// a level is one launch: merge-path tiles over (entries + edges), neighbour gather, claims,
// appends.  The first B-set step (B[kf - 1] from the meet set B[kf]) runs either way round:
// push = the in-edges of B[kf] into forward level kf - 1, pull = the out-edges of forward level
// kf - 1 into B[kf], whichever edge total is smaller (same set).  One OVER type per direction
// (path.cpp sends other requests to the host loop).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
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
// merge-path items per lane per tile.  A level's critical path is
// the slowest wave's chain of dependent accesses, so shorter tiles spread a level over more waves:
// RMAT-26 10k pairs, p50 0.131 ms at 8, 0.110 at 4, 0.107 at 2 (0.104 with a 256-workgroup step
// grid), 0.103 at 1 but p99 0.30-0.34 ms and batched -17 % (profiles/r03_vt2_sp_vt_ab.txt,
// r03_fin2_sp_vt2_batch_ab.txt)
constexpr int CH_VT = 2;                  // the batched chains' tiles (k_ch_step_b)
constexpr int CH_VT1 = 1;                 // the one-pair chains' tiles (k_ch_step<1>)
constexpr int CH_TILE_MIN = 64 * CH_VT1;  // (tile splits are allocated for the shorter tiles)
constexpr int CH_HOP_WGS = 64;            // workgroups scanning one greedy hop
constexpr int CH_HOP_U = 4;               // neighbours per thread in flight (greedy)
constexpr int CH_MAXS = 2 * MAX_PATH_LEN + 2;   // step launches of one query, at most

// Same-launch meets of a two-sided level are exchanged through LAB_M under tag epochs: the query's
// LAB_M epoch (< 2^24, sp.hip's next_epoch) with bit 25 (forward claim) or bit 24 (backward claim)
constexpr uint32_t CH_TAG_F = 1u << 25, CH_TAG_B = 1u << 24;
static_assert(CH_TAG_F < (1u << (32 - LVL_BITS)), "tag epochs fit the label's epoch field");

enum ChListId : int { CL_F0 = 0, CL_F1 = 1, CL_B0 = 2, CL_B1 = 3, CL_M = 4, CH_NLISTS = 5 };
enum ChPhase : uint32_t { PH_BFS = 0, PH_BSET = 1, PH_DONE = 2 };
// profiled launch kinds (nbg_profile_read names: kChainKernelNames)
enum ChKind : int { CHK_STEP = 0, CHK_HOP, CHK_STEP_B, CHK_ROLL, CH_NKINDS };

}  // namespace

struct ChList {
  uint32_t* ids;
  uint32_t* seg_end;    // inclusive edge prefix of the list
  uint32_t* seg_rs;     // CSR row start
  uint32_t* tsplit;     // merge-path split per tile
};

struct ChSnap {         // the search state before one step launch
  uint32_t phase, kf, kb, dir, met, L, bstep, err;
  uint32_t cur[2];                     // current list of each side (F0/F1, B0/B1)
  uint32_t both;                       // BFS: this step expands both sides (ChQ::both_items)
  uint32_t spare;
  unsigned long long cnt[2];           // packed (entries << 32 | edges) of each side's current list
  unsigned long long fprev;            // ... of the forward list one level back
  unsigned long long bcnt;             // ... of the B-set step's source list
  unsigned long long edges;            // BFS edges expanded so far
  unsigned long long levels;
  unsigned long long abytes;           // algorithmic bytes of the step launches so far (SURVEY §8(d)
                                       // B_SP: 4|F| ids + 8|F| row offsets + 4 E neighbour ids + 4 per
                                       // vertex appended, for every level and B-set step)
};

// A query's counters.  Two sets, used by alternate queries of a context (ChQ::par): the launch
// that writes a query's result zeroes the OTHER set — the next query's — so the next query needs
// no set-up launch, and nothing of the current query (whose workgroups may still be reading its
// own set) is touched.
struct ChCtr {
  unsigned long long lacc[CH_MAXS];    // packed output list of step launch i (both sides: forward's)
  unsigned long long lmeet[CH_MAXS];   // meet vertices found by step launch i (both sides: at position kf)
  unsigned long long lacc2[CH_MAXS];   // both sides: the backward output list
  unsigned long long lmeet2[CH_MAXS];  // both sides: meets at position kf + 1 (claimed by both sides)
  unsigned long long macc;             // packed meet list (over in-edges)
  unsigned long long err;              // 1 reconstruction failure, 3 list overflow
  unsigned long long hlaunch;          // greedy launches that did work
  unsigned long long busy;             // step launches that ran a step
  // greedy hub hop: workgroups done (the last one reduces and resets it).  Per query, so a hop
  // whose workgroups disagreed about their count (a failed query) cannot leave the next query's
  // hops a stale ticket
  unsigned long long gticket;
};

struct ChState {        // device; the host reads what the result launch derives from it (ChOut)
  ChCtr c[2];
  unsigned long long gerr;             // CH_GUARD builds: bit 8 + site of a bounds violation
  // greedy launch h starts from hstart[h] = (position << 32 | current vertex) and exactly one of
  // its workgroups writes hstart[h + 1]: state that no launch mutates while its own workgroups
  // may still read it (workgroups of one launch start at different times).  Greedy launches are
  // the step launches that find the search over (hop_first) and then the k_ch_hop launches.
  unsigned long long hstart[2 * CH_MAXS + 2];
  // step launch i starts at step first[i] (a BFS level or B-set step; first[0] = 0) and writes
  // first[i + 1]: one step, or none (the search is over)
  unsigned long long first[CH_MAXS + 1];
  ChSnap snap[CH_MAXS];
  long long path[1 + 3 * MAX_PATH_LEN];
  unsigned long long gpart[4 * CH_HOP_WGS];
  // hub hops inside the walking workgroup's launch (ch_hop<true>): the walker posts job k of greedy
  // launch h as hjob = (tag << 32 | h << 16 | k << 8 | pos) after its row range hjob_rng; helper
  // workgroup b stores its share's minimum into hpart[4b..4b+3] and then htag[b] = the job word.
  // Every word is tagged by the batch, launch and job, so nothing is reset between launches.
  unsigned long long hjob, hjob_rng;
  unsigned long long htag[CH_HOP_WGS];
  unsigned long long hpart[4 * CH_HOP_WGS];
  // (ChQ::tag << 32 | launch index) of the launch in which this query's walk ended (or found nothing
  // to walk): a batched chain's LATER launches give the pair one workgroup (ch_batch_work).  Written
  // inside a launch, so the launch that writes it must not act on it (its workgroups start at
  // different times and must all derive the same split), and written ONCE per query: the launches
  // after the walk's end find the same vertex and would rewrite it with their own index, which a
  // late-starting workgroup of such a launch read as "not over before this launch" while its
  // early peers had read the old value — two splits of one launch (round 6: a hub hop's ticket
  // then never reached its count, and every later query of that context failed)
  unsigned long long walk_end;
};

// What the host reads after a chain, stored by its last launch (ch_out) straight into mapped
// pinned memory (a hipMemcpyAsync of the 17 KB ChState went down the copy engine's path: ~130 us
// per pair on MI355X against ~3 us for a kernel's stores, profiles/r03_l_d2h_probe.json).
struct ChOut {
  ChSnap F;                            // the state after the last step launch
  unsigned long long err;              // ChState::err
  unsigned long long hpos;             // hstart[hops] (position << 32 | vertex)
  unsigned long long hlaunch;
  unsigned long long busy;             // ChState::busy
  unsigned long long tag;              // ChQ::tag of the batch whose launch stored this
  long long path[1 + 3 * MAX_PATH_LEN];
  unsigned long long wake;             // = tag, stored last (system-scope release): the host polls it
};

struct ChArgs {         // device memory (indexed at run time: never a by-value kernel argument)
  const uint32_t* row_ptr[2];          // [0] forward (out-edges), [1] backward (in-edges)
  const uint32_t* col[2];
  const int64_t* dst_vid;              // forward: greedy candidates
  const int64_t* rank;
  int64_t type;
  const uint8_t* visible;
  const int64_t* vids;
  uint32_t* lab[3];                    // forward, backward, B-set (LAB_M): words 0, 1, 2 of each
                                       // vertex's CH_LAB_WORDS-word record (index lrec(v))
  ChList list[CH_NLISTS];
  uint64_t list_cap, tsplit_cap;
  uint64_t nv, ne[2];                  // vertices, edges per direction (bounds of the checked build)
  ChState* st;
};

struct ChQ {
  uint32_t s, t, upto;
  uint32_t ef, eb, em;
  uint32_t par;                        // the query's counter set (ChState::c)
  uint32_t tag;                        // this batch of launches (ChOut::tag: which batch stored)
  uint32_t both_items;                 // a BFS level expands both sides when each has at most this many
                                       // items (entries + edges) and UPTO allows two levels (0: never)
  uint32_t job_wait;                   // ch_hop<true>: the walker's wait for its helpers' answers to a
                                       // hub job (steady-counter ticks; then the next launch spreads it)
};

// Both sides in one launch: while both frontiers are small a level's launch costs the same for one
// side or two (its time is the dependent chain of one tile, not the items), so two levels take one
// launch.  Forward claims level kf + 1, backward level kb + 1, at once.  The shortest length is
// kf + kb + 1 when a vertex at forward level kf gets backward level kb + 1 (the backward claims test
// the forward labels, which this launch does not write at level <= kf: a complete, race-free meet
// set at position kf; every such path also has one); otherwise kf + kb + 2 when a vertex is claimed
// by both sides in this launch — each claimer then exchanges its side's tag into the vertex's LAB_M
// word, and the later of the two exchanges (one location: a total modification order) returns the
// earlier one's tag: the meet set at position kf + 1 is complete too (LAB_M stamps only; the first
// B-set step then pulls).
__host__ __device__ __forceinline__ uint32_t both_next(const ChSnap& s, uint32_t upto, uint32_t items) {
  const unsigned long long a = (s.cnt[0] >> 32) + (s.cnt[0] & 0xFFFFFFFFull);
  const unsigned long long b = (s.cnt[1] >> 32) + (s.cnt[1] & 0xFFFFFFFFull);
  return items && s.kf + s.kb + 2 <= upto && a <= items && b <= items ? 1u : 0u;
}

// The state after step launch `i` (snapshot p before it, its results from st): every step launch
// and the host derive it the same way.
__host__ __device__ __forceinline__ ChSnap ch_advance(const ChSnap& p, unsigned long long out, unsigned long long meets,
                                              unsigned long long macc, unsigned long long err, uint32_t upto,
                                              unsigned long long out2, unsigned long long meets2, uint32_t items) {
  ChSnap s = p;
  constexpr unsigned long long M32 = 0xFFFFFFFFull;
  auto bytes_of = [](unsigned long long src, unsigned long long dst) {
    return 12ull * (src >> 32) + 4ull * (src & M32) + 4ull * (dst >> 32);
  };
  s.both = 0;
  if (p.phase == PH_BFS && p.both) {   // both sides expanded: forward `out`, backward `out2`
    s.abytes += bytes_of(p.cnt[0], out) + bytes_of(p.cnt[1], out2);
    s.edges += (p.cnt[0] & M32) + (p.cnt[1] & M32);
    s.levels += 2;
    // the backward side advanced in every case
    s.cnt[1] = out2;
    s.cur[1] ^= 1u;
    ++s.kb;
    if (err) {
      s.phase = PH_DONE;
      s.err = 1;
    } else if (meets) {   // length kf + kb (+1): meet set at forward position kf, listed (push)
      s.met = 1;
      s.L = s.kf + s.kb;
      s.bstep = 0;
      s.bcnt = macc;
      s.fprev = M32;      // (the forward side's other list now holds level kf + 1: no pull)
      s.phase = s.kf >= 2 ? PH_BSET : PH_DONE;
    } else {
      s.fprev = p.cnt[0];
      s.cnt[0] = out;
      s.cur[0] ^= 1u;
      ++s.kf;
      if (meets2) {       // length kf + kb (+2): meet set at position kf + 1, LAB_M stamps only (pull)
        s.met = 1;
        s.L = s.kf + s.kb;
        s.bstep = 0;
        s.bcnt = M32;
        s.phase = s.kf >= 2 ? PH_BSET : PH_DONE;
      } else if ((out >> 32) == 0 || (out2 >> 32) == 0 || s.kf + s.kb >= upto) {
        s.phase = PH_DONE;
      } else {
        s.dir = (s.cnt[0] & M32) <= (s.cnt[1] & M32) ? 0u : 1u;
        s.both = both_next(s, upto, items);
      }
    }
  } else if (p.phase == PH_BFS) {
    // (constant indices only: a runtime index into the snapshot's arrays puts it in scratch memory)
    const bool fwd = p.dir == 0;
    const unsigned long long pc = fwd ? p.cnt[0] : p.cnt[1];
    s.abytes += bytes_of(pc, out);
    s.edges += pc & 0xFFFFFFFFull;
    s.levels += 1;
    if (fwd) {
      s.fprev = p.cnt[0];
      s.cnt[0] = out;
      s.cur[0] ^= 1u;
      ++s.kf;
    } else {
      s.cnt[1] = out;
      s.cur[1] ^= 1u;
      ++s.kb;
    }
    if (err) {
      s.phase = PH_DONE;
      s.err = 1;
    } else if (meets) {
      s.met = 1;
      s.L = s.kf + s.kb;
      s.bstep = 0;
      s.bcnt = macc;
      s.phase = s.kf >= 2 ? PH_BSET : PH_DONE;
    } else if ((out >> 32) == 0 || s.kf + s.kb >= upto) {
      s.phase = PH_DONE;   // a side has no further edges, or UPTO reached: no path
    } else {
      s.dir = (s.cnt[0] & 0xFFFFFFFFull) <= (s.cnt[1] & 0xFFFFFFFFull) ? 0u : 1u;
      s.both = both_next(s, upto, items);
    }
  } else if (p.phase == PH_BSET) {
    // (the source list of this B-set step, as ch_step chose it: pull from the forward level or push)
    const bool pull = p.bstep == 0 && (p.fprev & M32) < (p.bcnt & M32);
    s.abytes += bytes_of(pull ? p.fprev : p.bcnt, out);
    s.bcnt = out;
    s.bstep += 1;
    if (err) {
      s.phase = PH_DONE;
      s.err = 1;
    } else if (s.bstep + 1 >= s.kf) {
      s.phase = PH_DONE;   // B[kf - 1] .. B[1] are there
    }
  }
  return s;
}

namespace {

// CH_GUARD=1 (a debugging build, `make EXTRA=-DCH_GUARD=1`): every indexed access is checked
// against its array's size; a violation sets bit 8 + site of ChState::err instead of touching
// memory, and the query fails with that code.
#ifndef CH_GUARD
#define CH_GUARD 0
#endif

template <typename T>
__device__ __forceinline__ T gld(const T* p, uint64_t i, uint64_t n, int site, ChState* st) {
  if (CH_GUARD && i >= n) {
    atomicOr(&st->gerr, 1ull << (8 + site));
    return T(0);
  }
  return p[i];
}
template <typename T>
__device__ __forceinline__ void gst(T* p, uint64_t i, uint64_t n, T v, int site, ChState* st) {
  if (CH_GUARD && i >= n) {
    atomicOr(&st->gerr, 1ull << (8 + site));
    return;
  }
  p[i] = v;
}

__device__ __forceinline__ uint32_t stamp_of(uint32_t epoch, uint32_t level) { return (epoch << LVL_BITS) | level; }
__device__ __forceinline__ bool live(uint32_t lab, uint32_t epoch) { return (lab >> LVL_BITS) == epoch; }
// word v of a label array: a vertex's three labels are one record (ChArgs::lab)
__device__ __forceinline__ uint64_t lrec(uint64_t v) { return v * CH_LAB_WORDS; }
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
  if (v == NO_ROW || (A.visible && !gld(A.visible, v, A.nv, 0, A.st))) {
    *rs = 0;
    return 0;
  }
  const uint32_t r = gld(A.row_ptr[side], v, A.nv + 1, 1, A.st);
  *rs = r;
  return gld(A.row_ptr[side], (uint64_t)v + 1, A.nv + 1, 1, A.st) - r;
}

// vdeg with every load issued at once (visibility and both row offsets), for a vertex that may
// not be claimed: its loads then travel with the claim's instead of after it
__device__ __forceinline__ uint32_t vdeg_spec(const ChArgs& A, int side, uint32_t v, uint32_t* rs) {
  if (v == NO_ROW) {
    *rs = 0;
    return 0;
  }
  const uint8_t vis = A.visible ? gld(A.visible, v, A.nv, 0, A.st) : (uint8_t)1;
  const uint32_t r = gld(A.row_ptr[side], v, A.nv + 1, 1, A.st);
  const uint32_t e = gld(A.row_ptr[side], (uint64_t)v + 1, A.nv + 1, 1, A.st);
  *rs = vis ? r : 0u;
  return vis ? e - r : 0u;
}

// Entry pos of list L: vertex v, its deg edges ending at edge offset end, from row rs; the tile
// boundaries its merge-path range [pos + end - deg, pos + end] covers get their split.
constexpr uint32_t CH_SPLITS_SOLO = 4;   // an entry covering more tile boundaries: the wave writes them

// Entry pos of list L: vertex v, its deg edges ending at edge offset end, from row rs.  The tile
// boundaries its merge-path range [pos + end - deg, pos + end] covers, [*t0, *t1), get the entry
// as their split; up to CH_SPLITS_SOLO of them are written here, the caller spreads the rest.
template <int VT>
__device__ __forceinline__ void list_put(const ChArgs& A, const ChList& L, uint32_t pos, uint32_t v, uint32_t end,
                                         uint32_t deg, uint32_t rs, uint64_t* t0, uint64_t* t1) {
  gst(L.ids, pos, A.list_cap, v, 2, A.st);
  gst(L.seg_end, pos, A.list_cap, end, 2, A.st);
  gst(L.seg_rs, pos, A.list_cap, rs, 2, A.st);
  const uint64_t lo = (uint64_t)pos + end - deg, hi = (uint64_t)pos + end;
  const uint64_t a = (lo + (64 * VT) - 1) / (64 * VT);
  const uint64_t b = hi / (64 * VT) + 1 < A.tsplit_cap ? hi / (64 * VT) + 1 : A.tsplit_cap;
  *t0 = a;
  *t1 = a < b ? b : a;
  if (*t1 - *t0 <= CH_SPLITS_SOLO) {
    for (uint64_t t = a; t < b; ++t) L.tsplit[t] = pos;
    *t1 = *t0;
  }
}

// Appends, per lane, the vertices x[i] with bit i of `m` and a nonzero degree (dg[i], rs[i]) to
// list L (counter *acc): one packed atomic per wave for positions and edge offsets; the tile
// splits of hubs (entries spanning many tiles) are written by the whole wave, lane-strided.
template <int VT>
__device__ __forceinline__ void wave_append(const ChArgs& A, const ChList& L, unsigned long long* acc,
                                            unsigned long long* err, const uint32_t (&x)[VT], uint32_t m,
                                            const uint32_t (&dg)[VT], const uint32_t (&rs)[VT]) {
  const int lane = threadIdx.x & 63;
  uint32_t c = 0, d = 0;
#pragma unroll
  for (int i = 0; i < VT; ++i)
    if (((m >> i) & 1u) && dg[i]) {
      ++c;
      d += dg[i];
    }
  const uint32_t ic = scan_incl(c), id = scan_incl(d);
  const uint32_t tc = __shfl(ic, 63, 64), td = __shfl(id, 63, 64);
  if (!tc) return;   // wave-uniform
  unsigned long long old = 0;
  if (lane == 0) old = atomicAdd(acc, ((unsigned long long)tc << 32) | td);
  old = __shfl(old, 0, 64);
  if ((old >> 32) + tc > A.list_cap) {
    if (lane == 0) atomicOr(err, 3ull);
    return;
  }
  uint32_t pos = (uint32_t)(old >> 32) + ic - c;
  uint32_t end = (uint32_t)old + id - d;
#pragma unroll
  for (int i = 0; i < VT; ++i) {
    uint64_t t0 = 0, t1 = 0;
    uint32_t p = pos;
    if (((m >> i) & 1u) && dg[i]) {
      end += dg[i];
      list_put<VT>(A, L, pos++, x[i], end, dg[i], rs[i], &t0, &t1);
    }
    unsigned long long bm = __ballot(t1 > t0);
    while (bm) {   // hubs of this round: the wave writes their tile splits
      const int l = __ffsll((long long)bm) - 1;
      bm &= bm - 1;
      const uint64_t a = __shfl(t0, l, 64), b = __shfl(t1, l, 64);
      const uint32_t hp = __shfl(p, l, 64);
      for (uint64_t t = a + (uint64_t)lane; t < b; t += 64) L.tsplit[t] = hp;
    }
  }
}

// The snapshot step i runs under: snap[0] (set-up) or derived from step i - 1.
__device__ __forceinline__ ChSnap snap_for(const ChState* st, const ChQ& q, int i) {
  if (i == 0) return st->snap[0];
  const ChCtr& C = st->c[q.par];
  return ch_advance(st->snap[i - 1], C.lacc[i - 1], C.lmeet[i - 1], C.macc, C.err, q.upto, C.lacc2[i - 1],
                    C.lmeet2[i - 1], q.both_items);
}

}  // namespace

// The first step needs no set-up launch: every workgroup of step launch 0 derives the search's
// start from (s, t) — the one-entry lists {s}, {t} are the registers below, not list memory, and
// s / t count as labelled (level 0 of their side) before workgroup 0 stores their labels — and
// workgroup 0 stores what later launches read: the labels of s and t, the lists {s} and {t} (the
// B-set steps and the greedy read them), snapshot 0, the greedy's start.  The counters are zero
// (the previous query's result launch zeroed this query's set; chain_prepare does it after a
// query that did not finish).
struct ChFirst {
  uint32_t dsf, rsf, dsb, rsb;   // degree and row start of s (forward) and t (backward)
};

__device__ __forceinline__ ChSnap first_snap(const ChArgs& A, const ChQ& q, ChFirst* f) {
  f->dsf = vdeg_spec(A, 0, q.s, &f->rsf);
  f->dsb = vdeg_spec(A, 1, q.t, &f->rsb);
  ChSnap s;
  memset(&s, 0, sizeof(s));
  s.phase = f->dsf && f->dsb ? PH_BFS : PH_DONE;
  s.dir = f->dsf <= f->dsb ? 0u : 1u;
  s.cnt[0] = (1ull << 32) | f->dsf;
  s.cnt[1] = (1ull << 32) | f->dsb;
  s.both = s.phase == PH_BFS ? both_next(s, q.upto, q.both_items) : 0u;
  return s;
}

__device__ __forceinline__ void first_store(const ChArgs& A, const ChQ& q, const ChFirst& f, const ChSnap& s) {
  ChState* st = A.st;
  st->snap[0] = s;
  A.lab[0][lrec(q.s)] = stamp_of(q.ef, 0);
  A.lab[1][lrec(q.t)] = stamp_of(q.eb, 0);
  const ChList& F = A.list[CL_F0];
  F.ids[0] = q.s;
  F.seg_end[0] = f.dsf;
  F.seg_rs[0] = f.rsf;
  const ChList& B = A.list[CL_B0];
  B.ids[0] = q.t;
  B.seg_end[0] = f.dsb;
  B.seg_rs[0] = f.rsb;
  st->hstart[0] = q.s;   // position 0, vertex s
  st->path[0] = gld(A.vids, q.s, A.nv, 16, st);
}

// Step j (snapshot P, not DONE): a BFS level or a B-set step.
//   BFS, side d: expand side d's current list over d's CSR; claim unlabelled neighbours with the
//     side's next level stamp, append them to d's other list, and record meets (claimed vertices
//     the other side already labelled: LAB_M stamp, meet list over in-edges).
//   B-set step k: B[kf - 1 - k] = vertices of forward level kf - 1 - k with an edge into
//     B[kf - k], claimed in LAB_M (push: in-edges of B[kf - k]; pull, k == 0 only: out-edges of
//     forward level kf - 1).
// (bid, nblk: this workgroup among the query's workgroups of the launch; NW waves per workgroup)
// (first: step 0, whose source list {s} or {t} is f0's registers — by value: a pointer to it
// selected at run time put it in scratch memory)
template <int NW, int VT>
__device__ __forceinline__ void ch_level(const ChArgs& A, const ChQ& q, const ChSnap& P, int i, uint32_t bid,
                                         uint32_t nblk, bool first, const ChFirst f0) {
  __shared__ uint32_t sEndAll[NW][(64 * VT) + 2];
  __shared__ uint32_t sRsAll[NW][(64 * VT) + 1];
  __shared__ uint16_t sSegAll[NW][(64 * VT)];
  ChState* st = A.st;
  const bool bfs = P.phase == PH_BFS;
  const bool both = bfs && P.both;   // forward level kf + 1 and backward level kb + 1 in one launch
  // ---- this launch's lists, labels and stamps (uniform; a two-sided level's backward tiles switch
  //      to the backward side's below)
  int side;              // CSR expanded
  ChList S, D;           // source list, output list
  unsigned long long scnt;
  uint32_t* lab;         // claimed label
  uint32_t epoch, stamp, oepoch = 0, mstamp = 0, rstamp = 0;
  const uint32_t* olab = nullptr;   // BFS: meet test
  const uint32_t* rlab = nullptr;   // push B-set: restriction to a forward level
  const uint32_t* tlab = nullptr;   // pull B-set: the neighbour must be in B[kf] (LAB_M == tstamp)
  uint32_t tstamp = 0;
  int oside;             // CSR of the output list's edge space
  bool append = true;
  if (bfs) {
    side = both ? 0 : (int)P.dir;
    const int src = side * 2 + (int)(side ? P.cur[1] : P.cur[0]);
    S = A.list[src];
    D = A.list[src ^ 1];
    scnt = side ? P.cnt[1] : P.cnt[0];
    lab = A.lab[side];
    epoch = side ? q.eb : q.ef;
    stamp = stamp_of(epoch, (side ? P.kb : P.kf) + 1);
    olab = A.lab[side ^ 1];
    oepoch = side ? q.ef : q.eb;
    mstamp = stamp_of(q.em, side ? P.kf : P.kf + 1);
    oside = side;
  } else {
    const uint32_t k = P.bstep, pos = P.kf - 1 - k;
    lab = A.lab[2];
    epoch = q.em;   // (as the host loop: a vertex with any B-set stamp of this query is taken)
    stamp = stamp_of(q.em, pos);
    append = pos >= 2;   // B[1]'s in-edges are not needed (B[0] = {s})
    oside = 1;
    D = A.list[CL_B0 + (int)(k & 1)];   // the backward lists are free once the sides met
    const bool pull = k == 0 && (P.fprev & 0xFFFFFFFFull) < (P.bcnt & 0xFFFFFFFFull);
    if (pull) {   // forward level kf - 1 is the forward side's other list
      side = 0;
      S = A.list[CL_F0 + (int)(P.cur[0] ^ 1u)];
      scnt = P.fprev;
      tlab = A.lab[2];
      tstamp = stamp_of(q.em, P.kf);
    } else {
      side = 1;
      S = A.list[k == 0 ? CL_M : CL_B0 + (int)((k - 1) & 1)];
      scnt = P.bcnt;
      rlab = A.lab[0];
      rstamp = stamp_of(q.ef, pos);
    }
  }
  const bool pull = tlab != nullptr;
  ChCtr& C = st->c[q.par];
  unsigned long long* out_acc = &C.lacc[i];
  // step 0: the one entry of the source list (s forward, t backward) from registers; s and t are
  // labelled level 0 of their sides (workgroup 0 stores those labels during this launch)
  uint32_t f_deg = first ? (side ? f0.dsb : f0.dsf) : 0u;
  uint32_t f_rs = first ? (side ? f0.rsb : f0.rsf) : 0u;
  uint32_t f_own = first ? (side ? q.t : q.s) : NO_ROW, f_other = first ? (side ? q.s : q.t) : NO_ROW;
  uint64_t n = scnt >> 32, total = scnt & 0xFFFFFFFFull;
  const uint32_t* __restrict__ col = A.col[side];
  uint64_t npath = n + total, ntiles = (npath + (64 * VT) - 1) / (64 * VT);
  // a two-sided level: tiles [0, nt0) are the forward side's, [nt0, nt0 + nt1) the backward's.
  // Meets: a backward claim of a vertex at forward level kf (l1stamp; LAB_M stamp kf, the meet list,
  // lmeet) or a vertex both sides claim in this launch (found by the exchange of mytag / otag in its
  // LAB_M word; LAB_M stamp kf + 1, lmeet2); forward claims of vertices at backward level <= kb are
  // no meets here
  const uint64_t nt0 = ntiles;
  const uint64_t nt1 = both ? (((P.cnt[1] >> 32) + (P.cnt[1] & 0xFFFFFFFFull)) + (64 * VT) - 1) / (64 * VT) : 0;
  const uint32_t l1stamp = stamp_of(q.ef, P.kf), l2m = stamp_of(q.em, P.kf + 1);
  // same-launch meet tags in LAB_M (tag epochs: never a query's live epoch, distinct per query)
  uint32_t mytag = stamp_of(q.em | CH_TAG_F, P.kf + 1), otag = stamp_of(q.em | CH_TAG_B, P.kb + 1);
  if (both) mstamp = 0;   // (forward tiles record no position-kf meets)
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t* const sEnd = sEndAll[w];
  uint32_t* const sRs = sRsAll[w];
  uint16_t* const sSeg = sSegAll[w];
  // tile t -> workgroup t % nblk, wave (t / nblk) % NW: the tiles of a level spread over as many
  // CUs as it has tiles (up to the grid) before any CU gets a second one.  A tile's random loads
  // and atomics (8 per lane) queue at its CU, so tiles packed 4 to a workgroup had 4 waves' misses
  // in one CU's queue while most CUs idled
  for (uint64_t tg = (uint64_t)w * nblk + bid; tg < nt0 + nt1; tg += (uint64_t)nblk * NW) {
    uint64_t t = tg;
    if (both && tg >= nt0 && side == 0) {   // (wave-uniform) the backward side's tiles from here on
      t = tg - nt0;
      side = 1;
      const int src = 2 + (int)P.cur[1];
      S = A.list[src];
      D = A.list[src ^ 1];
      scnt = P.cnt[1];
      lab = A.lab[1];
      epoch = q.eb;
      stamp = stamp_of(q.eb, P.kb + 1);
      olab = A.lab[0];
      oepoch = q.ef;
      mstamp = stamp_of(q.em, P.kf);
      oside = 1;
      out_acc = &C.lacc2[i];
      f_deg = first ? f0.dsb : 0u;
      f_rs = first ? f0.rsb : 0u;
      f_own = first ? q.t : NO_ROW;
      f_other = first ? q.s : NO_ROW;
      n = scnt >> 32;
      total = scnt & 0xFFFFFFFFull;
      col = A.col[1];
      npath = n + total;
      ntiles = nt1;
      const uint32_t tt = mytag;
      mytag = otag;
      otag = tt;
    } else if (both && side == 1) {
      t = tg - nt0;
    }
    uint32_t c[VT];   // the vertex a claim is about: the neighbour, or (pull) the list entry
    uint32_t cm = 0, mm = 0;
    // once this level has met, its claims are not expanded again: their appends are skipped
    // (read now, used after the claims: the load is off the critical path).  A two-sided level
    // runs to its end (a meet at position kf + 1 needs every claim of both sides)
    const unsigned long long met_now = bfs && !both ? ld_agent(&C.lmeet[i]) : 0ull;
    uint64_t sp = 0;
    if (first) {   // one entry: every tile's split is 0, the last tile's end is 1
      sp = lane == 1 && (t + 1) * (64 * VT) >= npath ? n : 0;
    } else if (ntiles > 1) {
      if (lane == 0) sp = gld(S.tsplit, t, A.tsplit_cap, 3, st);
      if (lane == 1) sp = (t + 1) * (64 * VT) >= npath ? n : gld(S.tsplit, t + 1, A.tsplit_cap, 3, st);
    } else {
      sp = lane == 1 ? n : 0;   // one tile: no split to read
    }
    const uint64_t a0 = uniform64(__shfl(sp, 0, 64)), a1 = uniform64(__shfl(sp, 1, 64));
    const uint64_t d0 = t * (64 * VT), d1 = d0 + (64 * VT) < npath ? d0 + (64 * VT) : npath;
    // a split that does not describe this tile (stale list memory) skips it and fails the search
    // (ChCtr::err bit 4, "device search aborted") instead of indexing out of bounds
    const bool bad = !(a0 <= a1 && a1 <= n && a1 - a0 <= d1 - d0 && d1 - a1 <= total && d0 - a0 <= d1 - a1);
    if (bad && lane == 0) atomicOr(&C.err, 4ull);
    const uint64_t b0 = bad ? 0 : d0 - a0, b1 = bad ? 0 : d1 - a1;
    const int na = bad ? 0 : (int)(a1 - a0), nb = bad ? 0 : (int)(b1 - b0);
    // the tile's window: sEnd[k] = seg_end[a0 - 1 + k], sRs[k] = seg_rs[a0 + k]
    for (int kk = lane; kk <= na + 1; kk += 64) {
      const int64_t e = (int64_t)a0 - 1 + kk;
      if (first) {
        sEnd[kk] = e < 0 ? 0u : (e < (int64_t)n ? f_deg : 0xFFFFFFFFu);
        if (kk <= na) sRs[kk] = (uint64_t)(e + 1) < n ? f_rs : 0u;
      } else {
        sEnd[kk] = e < 0 ? 0u : (e < (int64_t)n ? gld(S.seg_end, (uint64_t)e, A.list_cap, 4, st) : 0xFFFFFFFFu);
        if (kk <= na) sRs[kk] = (uint64_t)(e + 1) < n ? gld(S.seg_rs, (uint64_t)(e + 1), A.list_cap, 4, st) : 0u;
      }
    }
    wave_lds_sync();
    const uint32_t* Aend = sEnd + 1;   // Aend[j] = end of entry a0 + j
    {   // lane-level merge path: the entry of every edge item
      const int diag = lane * VT, dmax = na + nb;
      if (diag < dmax) {
        int lo = diag > nb ? diag - nb : 0, hi = diag < na ? diag : na;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if ((uint64_t)Aend[mid] <= b0 + (uint64_t)(diag - 1 - mid)) lo = mid + 1;
          else hi = mid;
        }
        int ai = lo, bi = diag - lo;
#pragma unroll
        for (int kk = 0; kk < VT; ++kk) {
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
    // neighbours (and, pulling, the list entry each edge belongs to), all loads in flight
    uint32_t x[VT], seg[VT];
#pragma unroll
    for (int j = 0; j < VT; ++j) {
      const int kk = j * 64 + lane;
      x[j] = NO_ROW;
      seg[j] = 0;
      if (kk < nb) {
        const uint32_t s = sSeg[kk];
        seg[j] = s;
        x[j] = gld(col, (uint64_t)sRs[s] + (b0 + kk - (uint64_t)sEnd[s]), A.ne[side], 5, st);
      }
    }
    wave_lds_sync();   // (the next tile rewrites the window)
    if (pull) {
      uint32_t tl[VT], vis[VT];
#pragma unroll
      for (int j = 0; j < VT; ++j) {
        tl[j] = x[j] != NO_ROW ? gld(tlab, lrec(x[j]), lrec(A.nv), 6, st) : 0u;
        vis[j] = x[j] != NO_ROW && A.visible ? gld(A.visible, x[j], A.nv, 6, st) : 1u;
      }
#pragma unroll
      for (int j = 0; j < VT; ++j)
        c[j] = (x[j] != NO_ROW && tl[j] == tstamp && vis[j]) ? gld(S.ids, a0 + seg[j], A.list_cap, 7, st) : NO_ROW;
    } else {
#pragma unroll
      for (int j = 0; j < VT; ++j) c[j] = x[j];
    }
    uint32_t old[VT], gate[VT];
    // a BFS level before its meet: the other side's label and the degree / row start of EVERY
    // neighbour are loaded with its own label, so the meet test and the append do not wait for
    // two more round trips after the claim (the extra loads are cheap: a level runs far below the
    // HBM bandwidth, profiles/r03_t_sp_step_pmc.txt)
    const bool spec = bfs && !met_now;   // (wave-uniform)
    uint32_t sol[VT], sdg[VT], srs[VT];
#pragma unroll
    for (int j = 0; j < VT; ++j) {
      old[j] = c[j] != NO_ROW ? gld(lab, lrec(c[j]), lrec(A.nv), 8, st) : 0u;
      gate[j] = (c[j] != NO_ROW && rlab) ? gld(rlab, lrec(c[j]), lrec(A.nv), 8, st) : rstamp;
      sol[j] = 0;
      sdg[j] = 0;
      srs[j] = 0;
      if (spec && c[j] != NO_ROW) {
        sol[j] = gld(olab, lrec(c[j]), lrec(A.nv), 9, st);
        sdg[j] = vdeg_spec(A, oside, c[j], &srs[j]);
      }
      if (first) {   // (the stores of these labels may still be in flight)
        if (c[j] == f_own) old[j] = stamp_of(epoch, 0);
        if (c[j] == f_other) sol[j] = stamp_of(oepoch, 0);
      }
    }
    if (met_now) {
      // the level has met: only meet vertices matter now (B[kf] is the met set; this level's other
      // labels are read by nothing), so the other side's label is tested before claiming
      uint32_t ol[VT];
#pragma unroll
      for (int j = 0; j < VT; ++j) {
        ol[j] = (c[j] != NO_ROW && !live(old[j], epoch)) ? gld(olab, lrec(c[j]), lrec(A.nv), 9, st) : 0u;
        if (first && c[j] == f_other) ol[j] = stamp_of(oepoch, 0);
      }
#pragma unroll
      for (int j = 0; j < VT; ++j) {
        if (c[j] == NO_ROW || live(old[j], epoch) || !live(ol[j], oepoch)) continue;
        if (CH_GUARD && c[j] >= A.nv) continue;
        if (atomicCAS(lab + lrec(c[j]), old[j], stamp) != old[j]) continue;
        mm |= 1u << j;
      }
    } else {
#pragma unroll
      for (int j = 0; j < VT; ++j) {
        if (c[j] == NO_ROW || gate[j] != rstamp || live(old[j], epoch)) continue;
        if (CH_GUARD && c[j] >= A.nv) continue;
        if (atomicCAS(lab + lrec(c[j]), old[j], stamp) != old[j]) continue;
        cm |= 1u << j;
      }
    }
    if (spec && !both) {   // meet test: the claimed vertices the other side has labelled
#pragma unroll
      for (int j = 0; j < VT; ++j)
        if (((cm >> j) & 1u) && live(sol[j], oepoch)) mm |= 1u << j;
    } else if (both) {
      uint32_t m2 = 0;
#pragma unroll
      for (int j = 0; j < VT; ++j) {
        if (!((cm >> j) & 1u)) continue;
        uint32_t o = sol[j];
        if (side == 1 && o == l1stamp) {   // backward level kb + 1 at forward level kf
          mm |= 1u << j;
          continue;
        }
        // claimed by the other side in this launch too: both claimers exchange their side's tag into
        // the vertex's ONE LAB_M word, so the later exchange in that word's modification order
        // returns the earlier one's tag (a relaxed RMW reads the latest value of its location; a
        // re-read of the other side's label after our own CAS would be the two-address store-buffer
        // pattern, which the memory model lets both claimers miss)
        const uint32_t prev = atomicExch(A.lab[2] + lrec(c[j]), mytag);
        if (prev == otag) m2 |= 1u << j;
      }
      if (__ballot(m2 != 0)) {
        uint32_t n2 = 0;
#pragma unroll
        for (int j = 0; j < VT; ++j)
          if ((m2 >> j) & 1u) {
            // (the one claimer that saw the other's tag; after both exchanges, so the stamp stays)
            __hip_atomic_store(A.lab[2] + lrec(c[j]), l2m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ++n2;
          }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) n2 += __shfl_xor(n2, o, 64);
        if (lane == 0) atomicAdd(&C.lmeet2[i], (unsigned long long)n2);
      }
    }
    if (!__ballot((cm | mm) != 0)) continue;
    // appends: one packed atomic per wave and list (aggregating them per workgroup behind two
    // barriers measured 4 % slower, profiles/r03_v_sp_wg_append_ab.txt)
    const uint32_t am = append && !met_now ? cm : 0u;
    uint32_t dg[VT], rs[VT];
#pragma unroll
    for (int j = 0; j < VT; ++j) {
      dg[j] = 0;
      rs[j] = 0;
      if ((am >> j) & 1u) {
        if (spec) {
          dg[j] = sdg[j];
          rs[j] = srs[j];
        } else {
          dg[j] = vdeg(A, oside, c[j], &rs[j]);
        }
      }
    }
    if (append && !met_now) wave_append<VT>(A, D, out_acc, &C.err, c, am, dg, rs);   // (a wave-uniform condition)
    // the sides met: LAB_M stamps, the meet list over in-edges, the level's meet count
    uint32_t nm = 0;
#pragma unroll
    for (int j = 0; j < VT; ++j) {
      dg[j] = 0;
      rs[j] = 0;
      if ((mm >> j) & 1u) {
        gst(A.lab[2], lrec(c[j]), lrec(A.nv), mstamp, 10, st);
        dg[j] = vdeg(A, 1, c[j], &rs[j]);
        ++nm;
      }
    }
    if (__ballot(mm != 0)) {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) nm += __shfl_xor(nm, o, 64);
      if (lane == 0) atomicAdd(&C.lmeet[i], (unsigned long long)nm);
      wave_append<VT>(A, A.list[CL_M], &C.macc, &C.err, c, mm, dg, rs);
    }
  }
}

// Items (entries + edges) of the source list of step P (as ch_level picks it).
__device__ __forceinline__ uint64_t step_items(const ChSnap& P) {
  unsigned long long c;
  if (P.phase == PH_BFS && P.both) {
    return (P.cnt[0] >> 32) + (P.cnt[0] & 0xFFFFFFFFull) + (P.cnt[1] >> 32) + (P.cnt[1] & 0xFFFFFFFFull);
  } else if (P.phase == PH_BFS) {
    c = P.dir ? P.cnt[1] : P.cnt[0];
  } else {
    const bool pull = P.bstep == 0 && (P.fprev & 0xFFFFFFFFull) < (P.bcnt & 0xFFFFFFFFull);
    c = pull ? P.fprev : P.bcnt;
  }
  return (c >> 32) + (c & 0xFFFFFFFFull);
}

// Step launch i: step first[i] (= i while the search is on) over the whole grid.  (Round 4's solo
// steps — small steps run back to back by workgroup 0 — measured neutral and were removed in
// round 6.)  Returns false when the search was over before this launch (a greedy launch then).
template <int NW, int VT>
__device__ __forceinline__ bool ch_step(const ChArgs& A, const ChQ& q, int i, uint32_t bid, uint32_t nblk) {
  ChState* st = A.st;
  ChCtr& C = st->c[q.par];
  // launch i runs step i while the search is on (first[i] == i, one step per launch): that
  // snapshot's loads are issued with first[i]'s, not after it (one memory round trip, not two,
  // before the level starts); a launch past the search reloads
  uint32_t j = 0;
  ChFirst f0{};
  ChSnap P;
  if (i == 0) {
    P = first_snap(A, q, &f0);
  } else {
    j = (uint32_t)st->first[i];
    const ChSnap Ps = snap_for(st, q, i);
    P = j == (uint32_t)i ? Ps : snap_for(st, q, (int)j);
  }
  const bool lead = bid == 0 && threadIdx.x == 0;
  if (i == 0 && bid == 0) {
    // the splits of {s} and {t} for later launches (a backward level from {t}, a pull B-set step
    // from {s}): one entry, so every tile's split is 0
    for (uint64_t t = threadIdx.x; t * (64 * VT) <= f0.dsf && t < A.tsplit_cap; t += CH_BLOCK) A.list[CL_F0].tsplit[t] = 0;
    for (uint64_t t = threadIdx.x; t * (64 * VT) <= f0.dsb && t < A.tsplit_cap; t += CH_BLOCK) A.list[CL_B0].tsplit[t] = 0;
    if (lead) first_store(A, q, f0, P);
  }
  if (P.phase == PH_DONE) {
    if (lead) st->first[i + 1] = j;
    return false;
  }
  if (lead) {
    C.busy += 1;
    if (j > 0) st->snap[j] = P;   // (step j + 1 derives its snapshot from it; snap[0]: first_store)
    st->first[i + 1] = j + 1;
  }
  ch_level<NW, VT>(A, q, P, (int)j, bid, nblk, j == 0, f0);
  return true;
}

namespace {

struct Cand {
  int64_t t, r, v;
  uint32_t d;
};
__device__ __forceinline__ bool cand_less(const Cand& a, const Cand& b) {
  if (a.t != b.t) return a.t < b.t;
  if (a.r != b.r) return a.r < b.r;
  return a.v < b.v;
}
constexpr uint32_t CH_SOLO_DEG = 4 * CH_BLOCK * CH_HOP_U;   // a hop one workgroup takes alone

// Workgroup-wide minimum (every thread gets it).
__device__ __forceinline__ Cand block_min(Cand b, Cand* lds) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    Cand y;
    y.t = __shfl_down(b.t, o, 64);
    y.r = __shfl_down(b.r, o, 64);
    y.v = __shfl_down(b.v, o, 64);
    y.d = __shfl_down(b.d, o, 64);
    if ((threadIdx.x & 63) + o < 64 && cand_less(y, b)) b = y;
  }
  if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = b;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < CH_WAVES; ++k)
      if (cand_less(lds[k], b)) b = lds[k];
    lds[CH_WAVES] = b;
  }
  __syncthreads();
  b = lds[CH_WAVES];
  __syncthreads();
  return b;
}

// Workgroup-wide minimum with ONE barrier (the solo walk's hops): each wave reduces, writes its
// candidate to slot set `par` (alternating per hop, so a wave still reading the previous hop's
// slots is never overwritten), and every thread reduces the CH_WAVES slots itself.
__device__ __forceinline__ Cand block_min1(Cand b, Cand (*slots)[CH_WAVES], uint32_t par) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    Cand y;
    y.t = __shfl_down(b.t, o, 64);
    y.r = __shfl_down(b.r, o, 64);
    y.v = __shfl_down(b.v, o, 64);
    y.d = __shfl_down(b.d, o, 64);
    if ((threadIdx.x & 63) + o < 64 && cand_less(y, b)) b = y;
  }
  if ((threadIdx.x & 63) == 0) slots[par][threadIdx.x >> 6] = b;
  __syncthreads();
  b = slots[par][0];
#pragma unroll
  for (int k = 1; k < CH_WAVES; ++k)
    if (cand_less(slots[par][k], b)) b = slots[par][k];
  return b;
}

// This thread's best candidate among c's out-edges [rs + g, re) step G into B[pos + 1].
__device__ __forceinline__ Cand hop_scan(const ChArgs& A, const uint32_t* vlab, uint32_t want, uint32_t rs,
                                         uint32_t re, uint64_t g, uint64_t G) {
  Cand best{INT64_MAX, INT64_MAX, INT64_MAX, NO_ROW};
  for (uint64_t j0 = rs + g; j0 < re; j0 += CH_HOP_U * G) {
    // (an edge's dst vid and rank are loaded with its neighbour id, not after the label test: one
    // dependent round trip less per hop, for 8-16 bytes more per scanned edge)
    uint32_t wv[CH_HOP_U], lv[CH_HOP_U];
    int64_t dv[CH_HOP_U], rk[CH_HOP_U];
#pragma unroll
    for (int u = 0; u < CH_HOP_U; ++u) {
      const uint64_t j = j0 + u * G;
      const bool in = j < re;
      wv[u] = in ? gld(A.col[0], j, A.ne[0], 11, A.st) : NO_ROW;
      dv[u] = in ? gld(A.dst_vid, j, A.ne[0], 13, A.st) : 0;
      rk[u] = in && A.rank ? gld(A.rank, j, A.ne[0], 13, A.st) : 0;
    }
#pragma unroll
    for (int u = 0; u < CH_HOP_U; ++u) lv[u] = wv[u] != NO_ROW ? gld(vlab, lrec(wv[u]), lrec(A.nv), 12, A.st) : 0u;
#pragma unroll
    for (int u = 0; u < CH_HOP_U; ++u) {
      if (wv[u] == NO_ROW || lv[u] != want) continue;
      const Cand x{A.type, rk[u], dv[u], wv[u]};
      if (cand_less(x, best)) best = x;
    }
  }
  return best;
}

}  // namespace

// Hub hops in the walk's launch (COOP): the workgroups that are not walking wait for the walker's
// jobs instead of returning.  Every wait is bounded (wall clock): a helper gives up after
// CH_HELP_IDLE without a job, the walker after CH_JOB_WAIT without every helper's answer, and then
// leaves the hub to the next launch's spread scan as before.  Only one-pair chains use it (a
// launch of at most CH_HOP_WGS walking workgroups per query, far below the chip's residency); a
// batch's pairs do not all have their workgroups resident together.
constexpr long long CH_HELP_IDLE = 20000;   // steady-counter ticks (100 MHz: 200 us)
constexpr uint32_t CH_JOB_WAIT = 10000;     // (100 us; ChQ::job_wait, NBG_SP_JOB_WAIT)
constexpr unsigned CH_JOB_END = 255;        // the job number of "the walk is over"

__device__ __forceinline__ unsigned long long job_word(const ChQ& q, int h, unsigned k, uint32_t pos) {
  return ((unsigned long long)q.tag << 32) | ((unsigned long long)(h & 0xFFFF) << 16) | ((k & 0xFFu) << 8) | (pos & 0xFFu);
}

// The walker's end of the walk in launch h (thread 0): the helpers return.
__device__ __forceinline__ void post_end(ChState* st, const ChQ& q, int h) {
  __hip_atomic_store(&st->hjob, job_word(q, h, CH_JOB_END, 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Greedy hops (CH_HOP_WGS workgroups), launch h of the query.  The state after step launch
// `last` says whether the sides met and the path length L; the launch starts from hstart[h] =
// (pos, c): hop pos (< L) takes the minimum (type, rank, dst vid) out-edge of the current vertex c
// into B[pos + 1] (B[pos + 1] = LAB_M stamp pos + 1 for positions <= kf, backward level
// L - pos - 1 beyond).  A hub's hop is scanned by every workgroup and reduced by the last one to
// finish; small hops are taken by one workgroup alone (workgroup 0, or the reducing one after a
// hub), which walks on until the path is complete.  A hub met on the way is spread over the
// other workgroups as a job (COOP), or (no COOP, or a job unanswered) left to the next launch.
// The walker writes hstart[h + 1].  Returns true in that one writing workgroup (every thread):
// it is the launch's last to touch the query's state, so it may also store the result.  COOP
// (one query per launch): true only where the result is final — the walk ended in this launch,
// or there was nothing to walk and this is the first greedy launch — and every launch is given
// the result block, so the host wakes as soon as the walk ends; the chain's later launches find
// the walk over and return without storing.
// (bid, nblk: this workgroup among the query's nblk <= CH_HOP_WGS workgroups of the launch)
template <bool COOP>
__device__ __forceinline__ bool ch_hop(const ChArgs& A, const ChQ& q, int nl, int h, uint32_t bid, uint32_t nblk) {
  __shared__ Cand lds[CH_WAVES + 1];
  __shared__ Cand hop_slots[2][CH_WAVES];
  __shared__ int s_last;
  __shared__ unsigned long long s_job[2];
  ChState* st = A.st;
  ChCtr& C = st->c[q.par];
  const ChSnap F = snap_for(st, q, (int)st->first[nl]);   // the state after the nl step launches
  const unsigned long long H = st->hstart[h];
  uint32_t pos = (uint32_t)(H >> 32), c = (uint32_t)H;
  auto finish = [&](uint32_t p, uint32_t v) {   // (thread 0 of the one writer)
    st->hstart[h + 1] = ((unsigned long long)p << 32) | v;
    if ((v == NO_ROW || !F.met || F.err || p >= F.L) && (ld_agent(&st->walk_end) >> 32) != q.tag)
      st->walk_end = ((unsigned long long)q.tag << 32) | (uint32_t)nl;
  };
  if (!F.met || F.phase != PH_DONE || F.err || pos >= F.L || c == NO_ROW) {
    if (bid == 0 && threadIdx.x == 0) finish(pos, c);
    return bid == 0 && (!COOP || h == 0);   // (COOP: the walk's own launch stored, unless none ran)
  }
  const uint32_t L = F.L, kf = F.kf;
  const Cand none{INT64_MAX, INT64_MAX, INT64_MAX, NO_ROW};
  auto range = [&](uint32_t v, uint32_t* rs, uint32_t* re) {   // (the three loads issued together)
    *rs = *re = 0;
    if (v != NO_ROW) {
      const uint32_t a = gld(A.row_ptr[0], v, A.nv + 1, 14, st);
      const uint32_t b = gld(A.row_ptr[0], (uint64_t)v + 1, A.nv + 1, 14, st);
      if (!A.visible || gld(A.visible, v, A.nv, 14, st)) {
        *rs = a;
        *re = b;
      }
    }
  };
  auto want_of = [&](uint32_t p, const uint32_t** vlab) {
    const bool by_m = p + 1 <= kf;
    *vlab = by_m ? A.lab[2] : A.lab[1];
    return by_m ? stamp_of(q.em, p + 1) : stamp_of(q.eb, L - p - 1);
  };
  // record hop p (thread 0): false when it has no candidate (reconstruction failure)
  auto record = [&](uint32_t p, const Cand& r) {
    if (r.d == NO_ROW) {
      atomicOr(&C.err, 1ull);
      finish(p, NO_ROW);
      return false;
    }
    gst(st->path, 1 + 3 * (uint64_t)p, 1 + 3 * (uint64_t)MAX_PATH_LEN, (long long)r.t, 15, st);
    gst(st->path, 2 + 3 * (uint64_t)p, 1 + 3 * (uint64_t)MAX_PATH_LEN, (long long)r.r, 15, st);
    gst(st->path, 3 + 3 * (uint64_t)p, 1 + 3 * (uint64_t)MAX_PATH_LEN, (long long)r.v, 15, st);
    return true;
  };
  // a helper: jobs 1, 2, ... of this launch until the end of the walk (or CH_HELP_IDLE without one)
  auto help = [&]() {
    for (unsigned k = 1; k < CH_JOB_END; ++k) {
      if (threadIdx.x == 0) {
        const long long t0 = wall_clock64();
        const unsigned long long mine = job_word(q, h, 0, 0) >> 16;   // (tag, launch)
        unsigned long long a = 0;
        for (;;) {
          const unsigned long long x = __hip_atomic_load(&st->hjob, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if ((x >> 16) == mine && ((x >> 8) & 0xFFu) >= k) {
            a = x;
            break;
          }
          if (wall_clock64() - t0 > CH_HELP_IDLE) break;
          __builtin_amdgcn_s_sleep(1);
        }
        s_job[0] = a;
        if (a) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          s_job[1] = ld_agent(&st->hjob_rng);
        }
      }
      __syncthreads();
      const unsigned long long a = s_job[0], rng = s_job[1];
      __syncthreads();   // (thread 0 rewrites s_job for the next job)
      if (!a || ((a >> 8) & 0xFFu) != k) return;   // the end, or no job within CH_HELP_IDLE
      const uint32_t* vlab;
      const uint32_t want = want_of((uint32_t)(a & 0xFFu), &vlab);
      Cand best = hop_scan(A, vlab, want, (uint32_t)rng, (uint32_t)(rng >> 32), (uint64_t)bid * CH_BLOCK + threadIdx.x,
                           (uint64_t)nblk * CH_BLOCK);
      best = block_min(best, lds);
      if (threadIdx.x == 0) {
        unsigned long long* part = st->hpart + 4 * bid;
        part[0] = (unsigned long long)best.t;
        part[1] = (unsigned long long)best.r;
        part[2] = (unsigned long long)best.v;
        part[3] = best.d;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __hip_atomic_store(&st->htag[bid], a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  };
  uint32_t rs, re;
  range(c, &rs, &re);
  if (re - rs > CH_SOLO_DEG) {   // a hub: every workgroup scans a share
    const uint32_t* vlab;
    const uint32_t want = want_of(pos, &vlab);
    Cand best = hop_scan(A, vlab, want, rs, re, (uint64_t)bid * CH_BLOCK + threadIdx.x, (uint64_t)nblk * CH_BLOCK);
    best = block_min(best, lds);
    if (threadIdx.x == 0) {
      unsigned long long* part = st->gpart + 4 * bid;
      part[0] = (unsigned long long)best.t;
      part[1] = (unsigned long long)best.r;
      part[2] = (unsigned long long)best.v;
      part[3] = best.d;
      __threadfence();
      s_last = atomicAdd(&C.gticket, 1ull) == nblk - 1;
    }
    __syncthreads();
    if (!s_last) {
      if (COOP) help();
      return false;
    }
    __threadfence();
    Cand r = none;
    if (threadIdx.x < nblk) {
      const unsigned long long* p = st->gpart + 4 * threadIdx.x;
      r = Cand{(int64_t)ld_agent(p), (int64_t)ld_agent(p + 1), (int64_t)ld_agent(p + 2), (uint32_t)ld_agent(p + 3)};
    }
    r = block_min(r, lds);
    if (threadIdx.x == 0) {
      C.gticket = 0;
      s_last = record(pos, r);
      if (COOP && !s_last) post_end(st, q, h);
    }
    __syncthreads();
    if (!s_last) return true;   // (a reconstruction failure: recorded and finished)
    c = r.d;
    ++pos;
  } else if (bid != 0) {
    if (COOP) help();
    return false;
  }
  // this workgroup alone: small hops, and (COOP) hubs' hops as jobs for the others
  if (threadIdx.x == 0) C.hlaunch += 1;
  uint32_t par = 0;   // block_min1's slot set, alternating per reduction
  unsigned jobs = 0;
  while (pos < L) {
    range(c, &rs, &re);
    const uint32_t* vlab;
    const uint32_t want = want_of(pos, &vlab);
    Cand r;
    if (re - rs > CH_SOLO_DEG) {   // a hub
      if (!COOP || nblk < 2 || jobs + 1 >= CH_JOB_END) break;   // the next launch spreads it
      const unsigned long long a = job_word(q, h, ++jobs, pos);
      if (threadIdx.x == 0) {
        __hip_atomic_store(&st->hjob_rng, (unsigned long long)rs | ((unsigned long long)re << 32), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __hip_atomic_store(&st->hjob, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      r = block_min(hop_scan(A, vlab, want, rs, re, (uint64_t)bid * CH_BLOCK + threadIdx.x, (uint64_t)nblk * CH_BLOCK),
                    lds);
      // wave 0 collects the helpers' answers: lane l waits for htag[l] == a (bounded)
      if (threadIdx.x < 64) {
        const uint32_t l = threadIdx.x;
        const long long t0 = wall_clock64();
        bool all = false;
        for (;;) {
          const bool ok = l >= nblk || l == bid || ld_agent(&st->htag[l]) == a;
          all = __all(ok);
          if (all || wall_clock64() - t0 > (long long)q.job_wait) break;
          __builtin_amdgcn_s_sleep(1);
        }
        Cand x = none;
        if (all) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          if (l < nblk && l != bid) {
            const unsigned long long* p = st->hpart + 4 * l;
            x = Cand{(int64_t)ld_agent(p), (int64_t)ld_agent(p + 1), (int64_t)ld_agent(p + 2), (uint32_t)ld_agent(p + 3)};
          }
        }
        if (l == 0) {
          if (cand_less(r, x)) x = r;   // (the walker's own share)
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
          Cand y;
          y.t = __shfl_down(x.t, o, 64);
          y.r = __shfl_down(x.r, o, 64);
          y.v = __shfl_down(x.v, o, 64);
          y.d = __shfl_down(x.d, o, 64);
          if (l + o < 64 && cand_less(y, x)) x = y;
        }
        if (l == 0) {
          hop_slots[0][0] = x;
          s_last = all;
        }
      }
      __syncthreads();
      const bool answered = s_last;
      r = hop_slots[0][0];
      __syncthreads();
      if (!answered) break;   // a helper did not answer in time: the next launch spreads it
    } else {
      // (one barrier per reduction: every thread has the minimum, so none waits for thread 0's record)
      r = block_min1(hop_scan(A, vlab, want, rs, re, threadIdx.x, CH_BLOCK), hop_slots, par);
      par ^= 1u;
    }
    if (threadIdx.x == 0) record(pos, r);
    if (r.d == NO_ROW) {   // (a reconstruction failure: recorded and finished)
      if (COOP && threadIdx.x == 0) post_end(st, q, h);
      return true;
    }
    c = r.d;
    ++pos;
  }
  if (threadIdx.x == 0) {
    finish(pos, c);
    if (COOP) post_end(st, q, h);
  }
  return !COOP || pos >= L;   // (COOP: a walk left at a hub is stored by the launch that ends it)
}

// The first greedy launch of the query: the first step launch that finds the search over (busy =
// the step launches that ran a step), never launch 0 (it stores the greedy's start).
__device__ __forceinline__ int hop_first(const ChCtr& C) {
  const int b = (int)C.busy;
  return b > 1 ? b : 1;
}

// ---------------------------------------------------------------------------- kernels
// The chain's result (the state after `steps` step launches; the greedy's position hstart[hend])
// into the host's ChOut (one workgroup; vector stores over the mapped pinned page), and the next
// query's counter set zeroed.
__device__ __forceinline__ void ch_out(const ChArgs& A, const ChQ& q, int steps, int hend, ChOut* out) {
  ChState* st = A.st;
  __syncthreads();   // (the writing workgroup's own stores: the path, hstart)
  const ChSnap F = snap_for(st, q, (int)st->first[steps]);
  const ChCtr& C = st->c[q.par];
  const uint32_t L = F.met && F.L <= MAX_PATH_LEN ? F.L : 0;
  for (uint32_t k = threadIdx.x; k < 1 + 3 * L; k += blockDim.x) out->path[k] = st->path[k];
  if (threadIdx.x == 0) {
    out->F = F;
    out->err = C.err | st->gerr;
    out->hpos = st->hstart[hend];
    out->tag = q.tag;
    out->hlaunch = C.hlaunch;
    out->busy = C.busy;
  }
  unsigned long long* nxt = reinterpret_cast<unsigned long long*>(&st->c[q.par ^ 1u]);
  for (uint32_t k = threadIdx.x; k < sizeof(ChCtr) / 8; k += blockDim.x) nxt[k] = 0;
  // the host's wake-up: every thread's stores released to system scope, then the tag
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // (release only, at system scope: no cache invalidation)
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(&out->wake, q.tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// One query per launch (the chain of one pair): step launch 0 starts the search (no set-up
// launch), and the batch's last hop launch stores the result (no result launch) ...
// (at most 2 waves per SIMD: 256 VGPRs, no spills; a one-pair launch has 128 workgroups of 4 waves,
// 2 waves per CU, so the occupancy bound costs nothing.  16-wave workgroups, tried for more waves
// per big level, were slower: RMAT-26 p50 0.137 -> 0.197 ms, profiles/r03_n_sp_block_ab.txt)
// Step launch i: a search step, or — the search over — greedy launch i - hop_first (its first
// CH_HOP_WGS workgroups), so the walk runs in the launches that used to return at once.  (out:
// where ch_hop says the result is final — COOP: the launch that ends the walk; else the batch's
// last launch, when the search was over before it.)
template <int NW, int VT, bool COOP>
__device__ __forceinline__ void ch_any(const ChArgs& A, const ChQ& q, int i, uint32_t bid, uint32_t nblk, ChOut* out) {
  if (ch_step<NW, VT>(A, q, i, bid, nblk) || i == 0 || bid >= (uint32_t)CH_HOP_WGS) return;
  const int h = i - hop_first(A.st->c[q.par]);
  if (ch_hop<COOP>(A, q, i, h, bid, nblk < (uint32_t)CH_HOP_WGS ? nblk : (uint32_t)CH_HOP_WGS) && out)
    ch_out(A, q, i, h + 1, out);
}

// VT: items per lane of a chain tile — 1 for one-pair chains (a level's critical path is the slowest
// wave's chain of dependent accesses, so shorter tiles cut the latency: RMAT-26 p50 0.0871-0.0876
// -> 0.0818-0.0836 ms, profiles/r05_u_sp_vt1_ab.txt), 2 for batched chains and their continuations
// (2-item tiles keep the batched rate: 37.3-37.7 k -> 41.2-41.5 k pairs/s)
template <int VT>
__global__ void __launch_bounds__(CH_BLOCK) __attribute__((amdgpu_waves_per_eu(2))) k_ch_step(const ChArgs* __restrict__ Ap, ChQ q, int i, ChOut* out) {
  ch_any<CH_WAVES, VT, true>(*Ap, q, i, blockIdx.x, gridDim.x, out);
}

// Greedy launches of a continuation: launch j after the nl step launches is greedy launch
// nl - hop_first + j; the one that ends the walk stores the result.
__global__ void __launch_bounds__(CH_BLOCK) k_ch_hop(const ChArgs* __restrict__ Ap, ChQ q, int nl, int j, ChOut* out) {
  const int h = nl - hop_first(Ap->st->c[q.par]) + j;
  if (ch_hop<true>(*Ap, q, nl, h, blockIdx.x, gridDim.x) && out) ch_out(*Ap, q, nl, h + 1, out);
}

// ... or up to CH_BMAX queries per launch (a batch of pairs, each with its own workspace, state and
// labels): query p takes workgroups [p * per, (p + 1) * per) of every launch of the chain, so one
// launch latency serves the whole batch.
constexpr int CH_BMAX = 32;
struct ChBatch {
  const ChArgs* A[CH_BMAX];
  ChState* st[CH_BMAX];                // (A[p]->st, passed by value: the allocation's loads start at once)
  ChQ q[CH_BMAX];
  ChOut* out[CH_BMAX];
  int n;
  uint32_t per;                        // fixed split: workgroups per pair (alloc == 0)
  uint32_t alloc;                      // 1: the grid is split by each pair's work in this launch
  uint32_t walk_items;                 // the work a pair whose search is over counts as (its walk)
};

// A pair's work in step launch i of a batch: the items of the step it runs (0 before launch 1:
// every pair starts from one vertex per side), or walk_items once its search is over.  Every
// workgroup derives it from the state the previous launch left, so all agree.
__device__ __forceinline__ unsigned long long ch_batch_work(const ChBatch& b, int p, int i) {
  if (i == 0) return 1;
  const ChState* st = b.st[p];
  const unsigned long long j = ld_agent(&st->first[i]);
  const unsigned long long we = ld_agent(&st->walk_end);
  const ChSnap P = snap_for(st, b.q[p], i);
  if ((we >> 32) == b.q[p].tag && (uint32_t)we < (uint32_t)i) return 0;   // walk over before launch i
  if (j != (unsigned long long)i || P.phase == PH_DONE) return b.walk_items;
  return step_items(P) + 1;
}

// Launch i of a batch: pair p takes nblk workgroups from `first` on.  alloc: 1 + (G - n) * work_p /
// sum(work) workgroups each (a launch lasts as long as its slowest pair's step, so a pair's share
// follows its step's size; a fixed 64 per pair left a hub level on 64 workgroups while most of
// the grid returned at once); else the fixed `per`.
__device__ __forceinline__ bool ch_batch_slot(const ChBatch& b, int i, uint32_t* p, uint32_t* bid, uint32_t* nblk) {
  if (!b.alloc) {
    *p = blockIdx.x / b.per;
    *bid = blockIdx.x % b.per;
    *nblk = b.per;
    return (int)*p < b.n;
  }
  __shared__ uint32_t s_sel[3];
  if (threadIdx.x < 64) {
    const int l = threadIdx.x;
    const unsigned long long w = l < b.n ? ch_batch_work(b, l, i) : 0ull;
    unsigned long long W = w;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) W += __shfl_xor(W, o, 64);
    const uint32_t G = gridDim.x, spare = G > (uint32_t)b.n ? G - (uint32_t)b.n : 0u;
    const uint32_t a = l < b.n ? 1u + (uint32_t)(W ? ((unsigned long long)spare * w) / W : 0ull) : 0u;
    const uint32_t incl = scan_incl(a), excl = incl - a;
    if (l == 0) s_sel[0] = 0xFFFFFFFFu;
    __builtin_amdgcn_wave_barrier();
    if (a && blockIdx.x >= excl && blockIdx.x < incl) {
      s_sel[0] = (uint32_t)l;
      s_sel[1] = blockIdx.x - excl;
      s_sel[2] = a;
    }
  }
  __syncthreads();
  *p = __builtin_amdgcn_readfirstlane(s_sel[0]);   // (uniform: kernel-argument arrays indexed by SGPRs)
  *bid = __builtin_amdgcn_readfirstlane(s_sel[1]);
  *nblk = __builtin_amdgcn_readfirstlane(s_sel[2]);
  __syncthreads();   // (ch_level reuses LDS; s_sel is read once)
  return *p != 0xFFFFFFFFu;
}

// (2 waves/SIMD: no spills; batched 33.3-33.9k -> 34.7-35.0k pairs/s, profiles/r03_y_sp_spec_ab.txt)
__global__ void __launch_bounds__(CH_BLOCK) __attribute__((amdgpu_waves_per_eu(2))) k_ch_step_b(ChBatch b, int i, int last) {
  uint32_t p, bid, nblk;
  if (ch_batch_slot(b, i, &p, &bid, &nblk))
    ch_any<CH_WAVES, CH_VT, false>(*b.A[p], b.q[p], i, bid, nblk, last ? b.out[p] : nullptr);
}

// ---------------------------------------------------------------------------- rolling batches
// A batch of 32 pairs ran the whole chain UPTO allows (2 UPTO launches) although a pair needs 4
// on average: most of each launch's slots sat idle behind the batch's longest search.  A rolling
// run keeps `nslots` contexts (slots) busy over a queue of n pairs: when a slot's pair has stored
// its result, the slot takes the next queued pair in the next launch, whose workgroups start that
// pair's step 0 beside the other slots' later steps.  Every workgroup derives launch i's
// assignment from state final at the launch boundary — the previous launch's assignment (R, one
// buffer per launch parity: launch i reads s[(i - 1) & 1] and its workgroup 0 writes s[i & 1]) and
// each slot's walk_end — so all agree.  A pair runs under its local launch index i - i0, with its
// own tag (tag0 + its index), counter set (its ordinal in the slot & 1: the previous pair's result
// launch zeroed it) and label epoch (ebase + ordinal + 1).  Its result is stored, straight into
// its own mapped ChOut, by the launch in which its walk ends.
constexpr int CH_RMAX = CH_ROLL_SLOTS;         // slots of a rolling run (one wave's lanes)
static_assert(CH_RMAX <= 64, "one lane per slot");
constexpr uint32_t CH_RNONE = 0xFFFFFFFFu;     // an idle slot (the queue is empty)
constexpr uint32_t CH_RDEAD = 0xFFFFFFFEu;     // a slot whose pair reached CH_MAXS launches (retired)
struct ChRollSlot {
  uint32_t p, i0, o, pad;                      // pair, its first launch, its ordinal in the slot
};
constexpr int CH_RTRACE = 4096;                // launches whose work NBG_SP_TRACE=2 records
struct ChRollState {                           // device
  ChRollSlot s[2][CH_RMAX];
  uint32_t qhead[2];                           // pairs handed out by launch i's assignment
  unsigned long long wmax[CH_RTRACE], wsum[CH_RTRACE];   // launch i's largest and total work (trace)
};
struct ChRollPair {
  uint32_t s, t;
};
struct ChRoll {
  const ChArgs* A[CH_RMAX];
  ChState* st[CH_RMAX];
  uint32_t ebase[CH_RMAX];
  const ChRollPair* pairs;                     // device [n]
  ChOut* outs;                                 // mapped pinned [n]
  ChRollState* R;
  unsigned long long* prog;                    // mapped pinned: ((i + 1) << 1) | (every pair done)
  uint32_t n, nslots, tag0, upto, both, walk_items;
};

__device__ __forceinline__ ChQ roll_q(const ChRoll& r, int l, uint32_t p, uint32_t o, uint32_t s, uint32_t t) {
  const uint32_t e = r.ebase[l] + o + 1;
  return ChQ{s, t, r.upto, e, e, e, o & 1u, r.tag0 + p, r.both, 0u};
}

// (2 waves per SIMD, as k_ch_step_b; VT: items per lane of a tile, NBG_SP_ROLL_VT)
template <int VT>
__global__ void __launch_bounds__(CH_BLOCK) __attribute__((amdgpu_waves_per_eu(2))) k_ch_roll(ChRoll r, int i) {
  __shared__ uint32_t s_sel[6];
  __shared__ int s_end;
  if (threadIdx.x < 64) {
    const int l = threadIdx.x;
    const bool slot = l < (int)r.nslots;
    ChRollSlot a{CH_RNONE, 0, 0, 0};
    uint32_t qh;
    if (i == 0) {
      if (slot && (uint32_t)l < r.n) a.p = (uint32_t)l;
      qh = r.n < r.nslots ? r.n : r.nslots;
    } else {
      const ChRollSlot pv = slot ? r.R->s[(i - 1) & 1][l] : a;
      const uint32_t qp = r.R->qhead[(i - 1) & 1];
      bool take = false;
      if (slot && pv.p < r.n) {
        const unsigned long long we = ld_agent(&r.st[l]->walk_end);
        if ((we >> 32) == r.tag0 + pv.p && (uint32_t)we < (uint32_t)i - pv.i0) take = true;   // stored before launch i
        else if ((uint32_t)i - pv.i0 >= (uint32_t)CH_MAXS) a = ChRollSlot{CH_RDEAD, 0, pv.o, 0};
        else a = pv;
      } else if (slot) {
        take = pv.p == CH_RNONE;
        a = pv;
      }
      const unsigned long long m = __ballot(take);
      if (take) {
        const uint32_t np = qp + (uint32_t)__popcll(m & ((1ull << l) - 1ull));
        const uint32_t no = pv.p == CH_RNONE ? pv.o : pv.o + 1;   // (an idle slot keeps its next ordinal)
        a = ChRollSlot{np < r.n ? np : CH_RNONE, (uint32_t)i, no, 0};
      }
      const uint32_t t = qp + (uint32_t)__popcll(m);
      qh = t < r.n ? t : r.n;
    }
    // this launch's work per active slot (as ch_batch_work) and the grid's split
    const bool act = slot && a.p < r.n;
    unsigned long long w = 0;
    if (act) {
      const int li = i - (int)a.i0;
      if (li == 0) {
        w = 1;
      } else {
        const ChState* st = r.st[l];
        const ChQ q = roll_q(r, l, a.p, a.o, 0, 0);
        const unsigned long long j = ld_agent(&st->first[li]);
        const ChSnap P = snap_for(st, q, li);
        w = (j != (unsigned long long)li || P.phase == PH_DONE) ? r.walk_items : step_items(P) + 1;
      }
    }
    unsigned long long W = w, Wm = w;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      W += __shfl_xor(W, o, 64);
      const unsigned long long y = __shfl_xor(Wm, o, 64);
      Wm = y > Wm ? y : Wm;
    }
    const uint32_t nact = (uint32_t)__popcll(__ballot(act));
    const uint32_t G = gridDim.x, spare = G > nact ? G - nact : 0u;
    const uint32_t na = act ? 1u + (uint32_t)(W ? ((unsigned long long)spare * w) / W : 0ull) : 0u;
    const uint32_t incl = scan_incl(na), excl = incl - na;
    if (l == 0) s_sel[0] = CH_RNONE;
    __builtin_amdgcn_wave_barrier();
    if (na && blockIdx.x >= excl && blockIdx.x < incl) {
      s_sel[0] = (uint32_t)l;
      s_sel[1] = blockIdx.x - excl;
      s_sel[2] = na;
      s_sel[3] = a.p;
      s_sel[4] = a.i0;
      s_sel[5] = a.o;
    }
    if (blockIdx.x == 0) {   // the assignment for launch i + 1 to derive its own from
      if (slot) r.R->s[i & 1][l] = a;
      if (l == 0) {
        r.R->qhead[i & 1] = qh;
        if (i < CH_RTRACE) {
          r.R->wmax[i] = Wm;
          r.R->wsum[i] = W;
        }
        __hip_atomic_store(r.prog, ((unsigned long long)(i + 1) << 1) | (qh >= r.n && nact == 0 ? 1ull : 0ull),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
  __syncthreads();
  const uint32_t l = __builtin_amdgcn_readfirstlane(s_sel[0]);
  const uint32_t bid = __builtin_amdgcn_readfirstlane(s_sel[1]), nblk = __builtin_amdgcn_readfirstlane(s_sel[2]);
  const uint32_t p = __builtin_amdgcn_readfirstlane(s_sel[3]), i0 = __builtin_amdgcn_readfirstlane(s_sel[4]);
  const uint32_t o = __builtin_amdgcn_readfirstlane(s_sel[5]);
  __syncthreads();   // (ch_level reuses LDS)
  if (l == CH_RNONE) return;
  const ChRollPair pr = r.pairs[p];
  const ChQ q = roll_q(r, (int)l, p, o, pr.s, pr.t);
  const ChArgs& A = *r.A[l];
  const int li = i - (int)i0;
  if (ch_step<CH_WAVES, VT>(A, q, li, bid, nblk) || li == 0 || bid >= (uint32_t)CH_HOP_WGS) return;
  const int h = li - hop_first(A.st->c[q.par]);
  if (!ch_hop<false>(A, q, li, h, bid, nblk < (uint32_t)CH_HOP_WGS ? nblk : (uint32_t)CH_HOP_WGS)) return;
  // the launch's writer: the result is final when the walk ended in this launch (walk_end is
  // written once per query, by the writer, which reads its own store back)
  if (threadIdx.x == 0) s_end = ld_agent(&A.st->walk_end) == (((unsigned long long)q.tag << 32) | (uint32_t)li);
  __syncthreads();
  if (s_end) ch_out(A, q, li, h + 1, r.outs + p);
}

// Zeroes both counter sets of every slot (block b: slot b) before a rolling run.
__global__ void __launch_bounds__(CH_BLOCK) k_ch_roll_init(ChRoll r) {
  unsigned long long* c = reinterpret_cast<unsigned long long*>(r.st[blockIdx.x]->c);
  for (uint32_t k = threadIdx.x; k < 2 * sizeof(ChCtr) / 8; k += blockDim.x) c[k] = 0;
}

// ---------------------------------------------------------------------------- host side
// A rolling run's buffers (kept by the run's first context, grown to the largest run)
struct RollBuf {
  ChRollState* R = nullptr;
  ChRollPair* d_pairs = nullptr;
  ChRollPair* h_pairs = nullptr;   // pinned staging of the pairs' upload
  ChOut* h_outs = nullptr;         // mapped pinned: every pair's result
  ChOut* d_outs = nullptr;
  unsigned long long* h_prog = nullptr;   // mapped pinned progress word
  unsigned long long* d_prog = nullptr;
  uint32_t cap = 0;
  uint32_t tag_next = 1u << 31;    // pair tags (a context's own chains count theirs from 1)
  void release() {
    if (R) (void)hipFree(R);
    if (d_pairs) (void)hipFree(d_pairs);
    if (h_pairs) (void)hipHostFree(h_pairs);
    if (h_outs) (void)hipHostFree(h_outs);
    if (h_prog) (void)hipHostFree(h_prog);
    R = nullptr;
    d_pairs = h_pairs = nullptr;
    h_outs = d_outs = nullptr;
    h_prog = d_prog = nullptr;
    cap = 0;
  }
};

struct ChainCtx {
  hipStream_t stream = nullptr;
  uint64_t nv = 0, list_cap = 0, tsplit_cap = 0;
  ChList list[CH_NLISTS] = {};
  ChState* d_st = nullptr;
  ChOut* h_out = nullptr;          // mapped pinned: the chain's last launch stores the result here
  ChOut* d_out = nullptr;          // its device address
  ChArgs* d_args = nullptr;
  ChArgs* h_args = nullptr;
  ChArgs cached{};
  bool args_valid = false;
  // step launch grid: most levels are a few tiles, so the launch's own cost (workgroups to
  // dispatch, each reading the state snapshot first) dominates; RMAT-26 10k-pair sweep
  // (profiles/r02_x_sp_grid_sweep.json): p50 0.159 ms at 512, 0.151 at 256, 0.148 at 128 and 96,
  // 0.154 at 32.  With 2-item-per-lane tiles (more tiles per level) 256: 0.104-0.106 against
  // 0.109-0.113 at 128 (profiles/r03_vt3_sp_grid_ab.txt, r03_fin2_sp_vt2_batch_ab.txt).
  // NBG_SP_GRID overrides.
  unsigned grid = 256;
  // ChQ::both_items (NBG_SP_BOTH; 0: one side per level).  RMAT-26 10 k pairs, round 6 (label
  // records): 16384 -> 32768 p50 0.0746-0.0748 -> 0.0736-0.0739 ms, p99 0.212-0.213 -> 0.210-0.212,
  // 65536 no better (profiles/r06_ae_sp_both_threshold_ab.txt)
  uint32_t both = 32768;
  // the query in flight: what has been enqueued
  ChQ q{};
  int steps = 0, hops = 0;
  uint32_t par = 0;                // the query's counter set (ChQ::par)
  bool clean = true;               // the next query's counter set is zero
  // recent queries: launches used (search steps + greedy launches; sizes the next chain)
  double ema_launches = 6;
  uint32_t tag_seq = 0;            // ChQ::tag of the next batch
  unsigned long long batches = 0, queries = 0;
  uint32_t qbatches = 0;           // batches the query in flight has used (1: no continuation)
  // nbg_profile: HIP events around the chain's launches (mode 1 every launch, 2 step launches only)
  int prof = 0;
  bool last_batched = false;       // the query in flight ran in a batched chain
  bool walk_cap = false;           // the walk did not end within CH_MAXS greedy launches (an error)
  struct RollBuf* roll = nullptr;  // rolling runs led by this context (chain_roll)
  struct PRec { int kind; hipEvent_t a, b; };
  std::vector<PRec> pend;
  std::vector<hipEvent_t> pool;
  double launches[CH_NKINDS] = {}, ms[CH_NKINDS] = {}, bytes[CH_NKINDS] = {};
  hipEvent_t ev() {
    if (!pool.empty()) { hipEvent_t e = pool.back(); pool.pop_back(); return e; }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
  }
  // one launch between two events (kind: CHK_*), when profiling that kind
  template <class F>
  void timed(int kind, F&& launch) {
    if (!prof || (prof == 2 && kind != CHK_STEP && kind != CHK_STEP_B && kind != CHK_ROLL)) { launch(); return; }
    PRec r{kind, ev(), ev()};
    (void)hipEventRecord(r.a, stream);
    launch();
    (void)hipEventRecord(r.b, stream);
    pend.push_back(r);
  }
  void flush() {   // (a host woken by the result's flag may be ahead of the last event)
    if (!pend.empty()) (void)hipEventSynchronize(pend.back().b);
    for (auto& r : pend) {
      float t = 0;
      if (hipEventElapsedTime(&t, r.a, r.b) == hipSuccess) ms[r.kind] += t;
      launches[r.kind] += 1;
      pool.push_back(r.a);
      pool.push_back(r.b);
    }
    pend.clear();
  }
};

ChainCtx* chain_create(uint64_t nv, uint64_t edge_cap, hipStream_t s, std::string* err, uint64_t list_cap) {
  auto* c = new ChainCtx();
  c->stream = s;
  c->nv = nv;
  c->list_cap = list_cap && list_cap < nv + 1 ? list_cap : nv + 1;
  c->tsplit_cap = (nv + 1 + edge_cap) / CH_TILE_MIN + 2;
  const char* g = getenv("NBG_SP_GRID");
  if (g && atoi(g) > 0) c->grid = (unsigned)atoi(g);
  const char* bo = getenv("NBG_SP_BOTH");
  if (bo) c->both = (uint32_t)strtoul(bo, nullptr, 10);
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
  if (he == hipSuccess) he = hipHostMalloc((void**)&c->h_out, sizeof(ChOut), hipHostMallocMapped | hipHostMallocCoherent);
  if (he == hipSuccess) he = hipHostGetDevicePointer((void**)&c->d_out, c->h_out, 0);
  if (he == hipSuccess) c->h_out->wake = 0;
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
  if (getenv("NBG_SP_TRACE") && c->queries)
    fprintf(stderr, "[sp trace] level loop: %llu queries, %.3f batches each, chain sized for %.2f launches\n",
            c->queries, (double)c->batches / c->queries, c->ema_launches);
  for (auto& L : c->list)
    for (uint32_t* p : {L.ids, L.seg_end, L.seg_rs, L.tsplit})
      if (p) (void)hipFree(p);
  if (c->d_st) (void)hipFree(c->d_st);
  if (c->d_args) (void)hipFree(c->d_args);
  if (c->h_out) (void)hipHostFree(c->h_out);
  if (c->h_args) (void)hipHostFree(c->h_args);
  if (c->roll) {
    c->roll->release();
    delete c->roll;
  }
  for (auto& r : c->pend) { (void)hipEventDestroy(r.a); (void)hipEventDestroy(r.b); }
  for (auto e : c->pool) (void)hipEventDestroy(e);
  delete c;
}

// Enqueue step launches [steps, steps + k) then h greedy launches.  The launch in which the walk
// ends stores the result (ch_hop<true>); a batch that ends before that stores nothing, so the
// stored tag stays the previous batch's and chain_more continues.
static hipError_t chain_batch(ChainCtx* c, int k, int h) {
  const ChArgs* A = c->d_args;
  c->q.tag = ++c->tag_seq;
  h = std::min(h, CH_MAXS - c->hops);
  for (int j = 0; j < k; ++j, ++c->steps)
    c->timed(CHK_STEP, [&] {
      // (a batched query's continuation keeps its chain's tile size: its lists' splits are per tile)
      if (c->last_batched)
        hipLaunchKernelGGL(k_ch_step<CH_VT>, dim3(c->grid), dim3(CH_BLOCK), 0, c->stream, A, c->q, c->steps, c->d_out);
      else
        hipLaunchKernelGGL(k_ch_step<CH_VT1>, dim3(c->grid), dim3(CH_BLOCK), 0, c->stream, A, c->q, c->steps, c->d_out);
    });
  for (int j = 0; j < h; ++j, ++c->hops)
    c->timed(CHK_HOP, [&] {
      hipLaunchKernelGGL(k_ch_hop, dim3(CH_HOP_WGS), dim3(CH_BLOCK), 0, c->stream, A, c->q, c->steps, c->hops, c->d_out);
    });
  ++c->batches;
  ++c->qbatches;
  return hipGetLastError();
}

// The query's arguments into c (uploaded when they changed) and its ChQ; nothing launched.
// The CSRs, labels and buffers of c's queries into its device ChArgs (uploaded when they changed).
static hipError_t chain_args(ChainCtx* c, const SpTypes& fwd, const SpTypes& bwd, const uint8_t* visible,
                             const int64_t* vids, uint32_t* const lab[3]) {
  if (fwd.n != 1 || bwd.n != 1) return hipErrorInvalidValue;
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
  a.nv = c->nv;
  a.ne[0] = fwd.ne[0];
  a.ne[1] = bwd.ne[0];
  a.st = c->d_st;
  if (!c->args_valid || memcmp(&a, &c->cached, sizeof(a)) != 0) {
    HIP_TRY_CH(hipStreamSynchronize(c->stream));   // the staging buffer may still feed an earlier upload
    memcpy(c->h_args, &a, sizeof(a));
    HIP_TRY_CH(hipMemcpyAsync(c->d_args, c->h_args, sizeof(a), hipMemcpyHostToDevice, c->stream));
    c->cached = a;
    c->args_valid = true;
  }
  return hipSuccess;
}

static hipError_t chain_prepare(ChainCtx* c, const SpTypes& fwd, const SpTypes& bwd, const uint8_t* visible,
                                const int64_t* vids, uint32_t* const lab[3], uint32_t epoch, uint32_t s, uint32_t t,
                                uint32_t upto) {
  if (upto < 1 || upto > MAX_PATH_LEN) return hipErrorInvalidValue;
  HIP_TRY_CH(chain_args(c, fwd, bwd, visible, vids, lab));
  c->par ^= 1u;
  // (NBG_SP_JOB_WAIT, read per query: a test sets 0 so that every hub job goes unanswered and the
  // fallback — the next launch's spread scan — runs)
  const char* jw = getenv("NBG_SP_JOB_WAIT");
  c->q = ChQ{s, t, upto, epoch, epoch, epoch, c->par, 0, c->both,
             jw ? (uint32_t)strtoul(jw, nullptr, 10) : CH_JOB_WAIT};
  c->steps = c->hops = 0;
  c->last_batched = false;
  c->walk_cap = false;
  c->qbatches = 0;
  ++c->queries;
  // the previous query's result launch zeroed this query's counters, unless it never ran
  if (!c->clean) HIP_TRY_CH(hipMemsetAsync(&c->d_st->c[c->par], 0, sizeof(ChCtr), c->stream));
  c->clean = false;
  return hipSuccess;
}

// Step launches a query can use: its search steps (at most 2 UPTO - 1) and one launch past them,
// in which the greedy walk (or, with no path, the result) runs.
static int chain_max(const ChainCtx* c) { return 2 * (int)c->q.upto; }

// chain length for c's query: sized by the recent queries, at their rounded-up mean.  The launch
// that ends the walk stores the result (ch_hop<true>), so the launches past it cost the next
// query a few us at most, while a chain one launch short costs a host round trip: RMAT-26 10 k
// pairs, p50 0.0761 / 0.0753 ms one launch under the mean and 0.0766 / 0.0763 at it, p90 0.142 /
// 0.140 against 0.1325 / 0.1317, six in flight 23.7-25.4 k against 28.7 k pairs/s
// (profiles/r05_zb_sp_store_early_ab.txt).  NBG_SP_KPAD adds launches (negative: fewer).  A longer
// query continues (chain_more).
static int chain_length(const ChainCtx* c) {
  static const int kpad = getenv("NBG_SP_KPAD") ? atoi(getenv("NBG_SP_KPAD")) : 0;
  return std::min(chain_max(c), std::max(2, (int)std::ceil(c->ema_launches) + kpad));
}

// dmin: min(out-degree of s, in-degree of t) when the caller knows it.  An endpoint of degree 1
// (a third of the RMAT-26 bench pairs) leaves its side a one-vertex frontier per level, so those
// searches run longer: 6.5 % of them needed a continuation (a host round trip) against 0.4 % for
// degree 2-3 and none above (tools/sp_tail_probe.py, profiles/r06_d_sp_tail.txt); their chains
// get NBG_SP_LOWDEG_PAD (1) more launches.
hipError_t chain_launch(ChainCtx* c, const SpTypes& fwd, const SpTypes& bwd, const uint8_t* visible,
                        const int64_t* vids, uint32_t* const lab[3], uint32_t epoch, uint32_t s, uint32_t t,
                        uint32_t upto, uint64_t dmin) {
  HIP_TRY_CH(chain_prepare(c, fwd, bwd, visible, vids, lab, epoch, s, t, upto));
  const char* lp = getenv("NBG_SP_LOWDEG_PAD");
  const int pad = dmin == 1 ? (lp ? atoi(lp) : 1) : 0;
  return chain_batch(c, std::min(chain_max(c), chain_length(c) + pad), 0);
}

// n <= CH_BMAX queries (contexts on one stream) in one chain of batched launches; each context
// then continues (chain_more) and completes (chain_result) on its own.
hipError_t chain_launch_batch(ChainCtx* const* cs, int n, const ChainQuery* qs) {
  if (n < 1 || n > CH_BMAX) return hipErrorInvalidValue;
  ChBatch b;
  memset(&b, 0, sizeof(b));
  b.n = n;
  static const unsigned per_env = getenv("NBG_SP_BATCH_WGS") ? (unsigned)atoi(getenv("NBG_SP_BATCH_WGS")) : 0u;
  // (2048 workgroups for a full batch: 64 per pair at 32 pairs, 39.4-40.5 k pairs/s against
  // 34.3-34.7 k at 32 per pair with 2-item tiles, profiles/r03_fin2_sp_vt2_batch_ab.txt)
  b.per = per_env ? per_env : std::max(64u, 2048u / (unsigned)n);
  // NBG_SP_BATCH_ALLOC (default 1): split the grid by each pair's step size; NBG_SP_BATCH_GRID
  // workgroups per launch then (default 512: two per CU, every one resident at 2 waves per SIMD),
  // NBG_SP_WALK_ITEMS the share of a walking pair
  // (read per batch: one getenv per 32 pairs)
  const int alloc_env = getenv("NBG_SP_BATCH_ALLOC") ? atoi(getenv("NBG_SP_BATCH_ALLOC")) : 1;
  const unsigned grid_env = getenv("NBG_SP_BATCH_GRID") ? (unsigned)atoi(getenv("NBG_SP_BATCH_GRID")) : 512u;
  const unsigned walk_env = getenv("NBG_SP_WALK_ITEMS") ? (unsigned)atoi(getenv("NBG_SP_WALK_ITEMS")) : 16384u;
  b.alloc = alloc_env ? 1u : 0u;
  b.walk_items = walk_env;
  const unsigned grid = b.alloc ? std::max<unsigned>(grid_env, (unsigned)n) : (unsigned)n * b.per;
  int k = 1;
  for (int p = 0; p < n; ++p) {
    ChainCtx* c = cs[p];
    if (c->stream != cs[0]->stream) return hipErrorInvalidValue;
    const ChainQuery& x = qs[p];
    HIP_TRY_CH(chain_prepare(c, *x.fwd, *x.bwd, x.visible, x.vids, x.lab, x.epoch, x.s, x.t, x.upto));
    c->q.tag = ++c->tag_seq;
    b.A[p] = c->d_args;
    b.st[p] = c->d_st;
    b.q[p] = c->q;
    b.out[p] = c->d_out;
    // the whole chain at once (every search step UPTO allows and one launch past them, which
    // walks the greedy path): a continuation would cost the batch a host round trip per context,
    // while a launch past a query's end returns at once
    k = std::max(k, chain_max(c));
  }
  const hipStream_t st = cs[0]->stream;
  ChainCtx* c0 = cs[0];   // (the batch's launch events are kept by its first context)
  for (int j = 0; j < k; ++j)
    c0->timed(CHK_STEP_B, [&] {
      hipLaunchKernelGGL(k_ch_step_b, dim3(grid), dim3(CH_BLOCK), 0, st, b, j, j + 1 == k);
    });
  HIP_TRY_CH(hipGetLastError());
  for (int p = 0; p < n; ++p) {
    ChainCtx* c = cs[p];
    c->last_batched = true;
    // a query needing fewer launches than the batch's longest ran past its end: its launches
    // returned at once (the search over, nothing left to walk), as in chain_batch
    c->steps = k;
    c->hops = 0;
    ++c->batches;
    ++c->qbatches;
  }
  return hipSuccess;
}

// A rolling run (k_ch_roll): n pairs (s[k], t[k]) of one query shape over nslots contexts that
// share one stream; every pair's result into results[k].  The host keeps NBG_SP_ROLL_AHEAD (4)
// launches queued past the one the device has started (the progress word, written at each
// launch's start), and stops when a launch finds every pair done; the launches queued past that
// return at once.  A pair whose walk did not end within CH_MAXS launches of its own (not
// reachable at UPTO <= CH_ROLL_UPTO) gets CH_ERR_WALK_CAP, and its slot takes no more pairs.
static void out_result(const ChOut& h, bool walk_cap, SpResult* out);

hipError_t chain_roll(const ChainSlot* slots, int nslots, const SpTypes& fwd, const SpTypes& bwd,
                      const uint8_t* visible, const int64_t* vids, const uint32_t* s, const uint32_t* t, uint32_t n,
                      uint32_t upto, SpResult* results) {
  if (nslots < 1 || nslots > CH_RMAX || upto < 1 || upto > CH_ROLL_UPTO) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  ChainCtx* c0 = slots[0].c;
  const hipStream_t st = c0->stream;
  ChRoll r;
  memset(&r, 0, sizeof(r));
  for (int l = 0; l < nslots; ++l) {
    ChainCtx* c = slots[l].c;
    if (c->stream != st) return hipErrorInvalidValue;
    HIP_TRY_CH(chain_args(c, fwd, bwd, visible, vids, slots[l].lab));
    r.A[l] = c->d_args;
    r.st[l] = c->d_st;
    r.ebase[l] = slots[l].ebase;
  }
  if (!c0->roll) c0->roll = new RollBuf();
  RollBuf& B = *c0->roll;
  if (B.cap < n) {   // (the previous run has completed: the buffers are idle)
    B.release();
    hipError_t he = hipMalloc((void**)&B.R, sizeof(ChRollState));
    if (he == hipSuccess) he = hipMalloc((void**)&B.d_pairs, (size_t)n * sizeof(ChRollPair));
    if (he == hipSuccess) he = hipHostMalloc((void**)&B.h_pairs, (size_t)n * sizeof(ChRollPair), hipHostMallocDefault);
    if (he == hipSuccess)
      he = hipHostMalloc((void**)&B.h_outs, (size_t)n * sizeof(ChOut), hipHostMallocMapped | hipHostMallocCoherent);
    if (he == hipSuccess) he = hipHostGetDevicePointer((void**)&B.d_outs, B.h_outs, 0);
    if (he == hipSuccess)
      he = hipHostMalloc((void**)&B.h_prog, sizeof(unsigned long long), hipHostMallocMapped | hipHostMallocCoherent);
    if (he == hipSuccess) he = hipHostGetDevicePointer((void**)&B.d_prog, B.h_prog, 0);
    if (he != hipSuccess) {
      B.release();
      return he;
    }
    B.cap = n;
  }
  for (uint32_t k = 0; k < n; ++k) B.h_pairs[k] = ChRollPair{s[k], t[k]};
  HIP_TRY_CH(hipMemcpyAsync(B.d_pairs, B.h_pairs, (size_t)n * sizeof(ChRollPair), hipMemcpyHostToDevice, st));
  __atomic_store_n(B.h_prog, 0ull, __ATOMIC_RELEASE);
  if (B.tag_next > 0xF0000000u - n) B.tag_next = 1u << 31;
  r.pairs = B.d_pairs;
  r.outs = B.d_outs;
  r.R = B.R;
  r.prog = B.d_prog;
  r.n = n;
  r.nslots = (uint32_t)nslots;
  r.tag0 = B.tag_next;
  B.tag_next += n;
  r.upto = upto;
  r.both = c0->both;
  // (read per run, as the fixed batches read theirs per batch).  RMAT-26, 10 k pairs
  // (profiles/r06_i_sp_roll_grid_vt.txt, r06_j_*): 4-item tiles on 1024 workgroups 50.6-54.9 k
  // pairs/s against 44.6-45.0 k with the fixed batches' 2-item tiles on 512 (8-item tiles 47.6-49.1 k)
  const unsigned grid_env = getenv("NBG_SP_ROLL_GRID") ? (unsigned)atoi(getenv("NBG_SP_ROLL_GRID")) : 1024u;
  const unsigned walk_env = getenv("NBG_SP_WALK_ITEMS") ? (unsigned)atoi(getenv("NBG_SP_WALK_ITEMS")) : 16384u;
  const int ahead = getenv("NBG_SP_ROLL_AHEAD") ? std::max(1, atoi(getenv("NBG_SP_ROLL_AHEAD"))) : 4;
  const int vt = getenv("NBG_SP_ROLL_VT") ? atoi(getenv("NBG_SP_ROLL_VT")) : 4;
  auto kern = vt == 8 ? k_ch_roll<8> : vt == 4 ? k_ch_roll<4> : vt == 1 ? k_ch_roll<1> : k_ch_roll<2>;
  const auto t_start = std::chrono::steady_clock::now();
  r.walk_items = walk_env;
  const unsigned grid = std::max(grid_env, (unsigned)nslots);
  hipLaunchKernelGGL(k_ch_roll_init, dim3(nslots), dim3(CH_BLOCK), 0, st, r);
  HIP_TRY_CH(hipGetLastError());
  // launches: at most CH_MAXS per pair on each slot (a safety bound; a run takes ~4-5 per pair / nslots)
  const uint64_t cap = ((uint64_t)n + (uint64_t)nslots) * CH_MAXS;
  uint64_t enq = 0;
  // NBG_SP_TRACE=2: an event before every launch, and each launch's work (largest pair, total)
  static const bool trace2 = getenv("NBG_SP_TRACE") && atoi(getenv("NBG_SP_TRACE")) == 2;
  std::vector<hipEvent_t> tev;
  for (unsigned spin = 1;; ++spin) {
    const unsigned long long pw = __atomic_load_n(B.h_prog, __ATOMIC_ACQUIRE);
    if (pw & 1ull) break;
    const uint64_t seen = pw >> 1;   // launches started
    if (enq < seen + (uint64_t)ahead && enq < cap) {
      const int i = (int)enq;
      if (trace2 && i < CH_RTRACE) {
        tev.push_back(c0->ev());
        (void)hipEventRecord(tev.back(), st);
      }
      c0->timed(CHK_ROLL, [&] { hipLaunchKernelGGL(kern, dim3(grid), dim3(CH_BLOCK), 0, st, r, i); });
      HIP_TRY_CH(hipGetLastError());
      ++enq;
      continue;
    }
    if ((spin & 1023) == 0) {   // a failed launch never writes progress: its error ends the run
      const hipError_t e = hipStreamQuery(st);
      if (e != hipErrorNotReady && e != hipSuccess) return e;
      if (e == hipSuccess && enq >= cap) break;   // (not reachable: every pair ends within the bound)
    }
  }
  if (trace2) {
    tev.push_back(c0->ev());
    (void)hipEventRecord(tev.back(), st);
  }
  HIP_TRY_CH(hipStreamSynchronize(st));
  if (trace2 && tev.size() > 1) {   // per launch: duration against its largest pair's work (log2 buckets)
    const size_t nl = tev.size() - 1;
    std::vector<unsigned long long> wm(nl), ws(nl);
    (void)hipMemcpy(wm.data(), B.R->wmax, nl * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(ws.data(), B.R->wsum, nl * 8, hipMemcpyDeviceToHost);
    double cnt[48] = {}, ms[48] = {}, sum[48] = {};
    for (size_t k = 0; k < nl; ++k) {
      float t = 0;
      (void)hipEventElapsedTime(&t, tev[k], tev[k + 1]);
      int b = 0;
      while (b < 47 && (1ull << (b + 1)) <= wm[k]) ++b;
      cnt[b] += 1;
      ms[b] += t;
      sum[b] += (double)ws[k];
    }
    double tot = 0;
    for (int b = 0; b < 48; ++b) tot += ms[b];
    for (int b = 0; b < 48; ++b)
      if (cnt[b])
        fprintf(stderr, "[sp roll launches] largest pair work in [2^%d, 2^%d): %5.0f launches, %8.2f us each, %5.1f%% of the time, mean total work %.0f\n",
                b, b + 1, cnt[b], 1e3 * ms[b] / cnt[b], 100.0 * ms[b] / tot, sum[b] / cnt[b]);
    fprintf(stderr, "[sp roll launches] %zu launches, %.3f ms\n", nl, tot);
    for (auto e : tev) c0->pool.push_back(e);
  }
  if (getenv("NBG_SP_TRACE"))
    fprintf(stderr, "[sp roll] %u pairs, %d slots, %llu launches enqueued, done at launch %llu, %.3f ms\n", n, nslots,
            (unsigned long long)enq, (unsigned long long)(__atomic_load_n(B.h_prog, __ATOMIC_ACQUIRE) >> 1),
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count());
  double abytes = 0;
  for (uint32_t k = 0; k < n; ++k) {
    const ChOut& h = B.h_outs[k];
    const bool stored = __atomic_load_n(&h.wake, __ATOMIC_ACQUIRE) == (unsigned long long)(r.tag0 + k);
    out_result(h, !stored, &results[k]);
    results[k].launches = stored ? h.busy + std::max(1ull, h.hlaunch) : 0;
    results[k].batches = 1;
    abytes += stored ? (double)h.F.abytes : 0.0;
  }
  for (int l = 0; l < nslots; ++l) {
    ChainCtx* c = slots[l].c;
    c->clean = false;   // (the next one-pair query zeroes its counter set)
    c->queries += 1;
  }
  if (c0->prof) {
    c0->flush();
    c0->bytes[CHK_ROLL] += abytes;
  }
  return hipSuccess;
}

// After a batch's copy completed: the query's final state, or false with a continuation batch
// enqueued (the caller waits again).
bool chain_woken(const ChainCtx* c) {
  return c && c->h_out && __atomic_load_n(&c->h_out->wake, __ATOMIC_ACQUIRE) == c->q.tag;
}

bool chain_more(ChainCtx* c, hipError_t* he) {
  *he = hipSuccess;
  const ChOut& h = *c->h_out;
  const ChSnap F = h.F;
  if (h.tag != c->q.tag || F.phase != PH_DONE) {
    // the batch ended inside the search (its last launch stored nothing): NBG_SP_KMORE (2) more
    // launches, or the rest if fewer — most such searches ended in the batch's last launch or
    // need one more step, and the launches past a search's end cost ~3 us each; a search still
    // not over continues again.  The batch's last launch stores if the search was over before it.
    if (c->steps >= chain_max(c)) {
      // a search has at most 2 UPTO - 1 steps, so it is over: the walk stopped at a hub whose job
      // went unanswered in the chain's last launch.  Greedy continuation launches (k_ch_hop): each
      // takes at least one hop (a hub's spread over its workgroups), the one that ends the walk
      // stores the result, and the ones past it return at once
      const int left = CH_MAXS - c->hops;
      if (left <= 0) {   // (not reachable: every greedy launch advances the walk)
        c->walk_cap = true;
        return true;
      }
      *he = chain_batch(c, 0, std::min(left, (int)c->q.upto));
      return false;
    }
    static const int kmore = getenv("NBG_SP_KMORE") ? std::max(1, atoi(getenv("NBG_SP_KMORE"))) : 2;
    *he = chain_batch(c, std::min(chain_max(c) - c->steps, kmore), 0);
    return false;
  }
  const uint32_t hpos = (uint32_t)(h.hpos >> 32);
  if (F.met && !F.err && !h.err && hpos < F.L) {
    if (c->hops >= CH_MAXS) {
      c->walk_cap = true;
      return true;
    }
    *he = chain_batch(c, 0, (int)F.L - (int)hpos);
    return false;
  }
  c->clean = true;   // (its result launch zeroed the next query's counters)
  // launches used (search steps, then the greedy's, at least one); decay toward this query's needs
  const double used = (double)h.busy + (double)std::max(1ull, h.hlaunch);
  c->ema_launches = 0.9 * c->ema_launches + 0.1 * (used + 0.3);
  return true;
}

// a stored result -> SpResult (walk_cap: the walk never ended)
static void out_result(const ChOut& h, bool walk_cap, SpResult* out) {
  const ChSnap& F = h.F;
  out->err = h.err;
  out->edges = F.edges;
  out->levels = F.levels;
  out->abytes = F.abytes;
  const uint32_t hpos = (uint32_t)(h.hpos >> 32);
  out->L = (F.met && !h.err && hpos == F.L && !walk_cap) ? F.L : 0;
  if (walk_cap) {
    out->err = CH_ERR_WALK_CAP;
  } else if (F.met && !h.err && hpos != F.L) {
    out->err = 2;   // (cannot happen: the hops were enqueued)
  }
  if (out->L) memcpy(out->path, h.path, (1 + 3 * (size_t)out->L) * sizeof(long long));
}

// the final state -> SpResult
void chain_result(const ChainCtx* c, SpResult* out) {
  const ChOut& h = *c->h_out;
  out_result(h, c->walk_cap, out);
  out->launches = (unsigned long long)(c->steps + c->hops);
  out->batches = c->qbatches;
  // NBG_SP_TRACE=2: one line per query (the chain's step and greedy launches, path length)
  static const bool per_query = getenv("NBG_SP_TRACE") && atoi(getenv("NBG_SP_TRACE")) == 2;
  if (per_query)
    fprintf(stderr, "[sp q] steps %d hops %d busy %llu hlaunch %llu L %llu\n", c->steps, c->hops, h.busy, h.hlaunch,
            (unsigned long long)out->L);
}

// nbg_profile over the chain: mode 0 off, 1 every launch, 2 step launches only (counters reset)
void chain_profile(ChainCtx* c, int mode) {
  c->flush();
  c->prof = mode;
  for (int k = 0; k < CH_NKINDS; ++k) c->launches[k] = c->ms[k] = c->bytes[k] = 0;
}

// after chain_result: resolve the query's launch events and credit its algorithmic bytes to the
// step launches that moved them (setup and greedy hops touch O(path) bytes)
void chain_profile_done(ChainCtx* c, const SpResult& r) {
  if (!c->prof) return;
  c->flush();
  c->bytes[c->last_batched ? CHK_STEP_B : CHK_STEP] += (double)r.abytes;
}

static_assert(CH_NKINDS == CHAIN_KINDS, "chain kinds");
const char* const kChainKernelNames[CH_NKINDS] = {"k_ch_step", "k_ch_hop", "k_ch_step_b", "k_ch_roll"};

void chain_profile_accum(const ChainCtx* c, double* launches, double* ms, double* bytes) {
  for (int k = 0; k < CH_NKINDS; ++k) {
    launches[k] += c->launches[k];
    ms[k] += c->ms[k];
    bytes[k] += c->bytes[k];
  }
}

}  // namespace nbg
