// nebula_amd — gfx950 (CDNA4) kernels for the GO N STEPS / FIND PATH hot path.
//
// A query is enqueued on the workspace stream with NO host synchronisation until its end:
// every size the kernels need (frontier size n, edges of the current expansion, next frontier
// size) lives in a device-resident QState and grids are sized from host-known upper bounds.
//
// Per hop over one edge type (CSR):
//   k_degree      frontier degrees (row_ptr gathers, capped by max_edge_returned_per_vertex)
//                 + block-local inclusive scan                       (wave64 shuffles + LDS)
//   k_scan_blocks exclusive scan of the per-block totals (one workgroup); publishes the total
//   k_expand<M>   persistent, load-balanced expansion over merge-path tiles: a tile owns TILE
//                 path items (frontier segments + edges) whatever the degree skew, its split is
//                 found by a wave-wide 64-ary search over the global scan; items are processed striped
//                 across the block so neighbour / property reads are coalesced.
//                 M = MARK  (steps 1..N-1: set next-frontier byte flags, idempotent plain stores)
//                 M = FINAL (step N: WHERE/YIELD bytecode per edge, wave-ballot compaction, rows
//                           appended to one of NSHARD per-shard regions: one atomic per
//                           tile on a sharded counter, never a single hot word; simple
//                           `col <cmp> const` / leaf-yield programs skip the interpreter)
//   k_flag_count / k_scan_blocks / k_flag_write  dense compaction of the byte flags into the
//                 next (sorted) frontier, clearing the flags in the same pass.
// Semantics follow QueryBaseProcessor::collectEdgeProps (version de-dup is done at load,
// neighbours are in memcmp key order, the cap counts edges in that order) and
// GoExecutor::getDstIdsFromResp (per-step dst SET, no global visited set).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "nbg_internal.h"

namespace nbg {

constexpr int BLOCK = 256;
constexpr int WAVES = BLOCK / 64;
constexpr int SCAN_ITEMS = 8;                    // k_degree: items per thread
constexpr int SCAN_TILE = BLOCK * SCAN_ITEMS;    // 2048 frontier entries per block
constexpr int SCAN_SHIFT = 11;
constexpr int FLAG_BYTES = BLOCK * 16;           // k_flag_*: bytes per block
constexpr int EXPAND_GRID = 2048;                // persistent k_expand grid (8 blocks / CU)

enum KernelId { K_DEGREE = 0, K_SCAN, K_EXPAND_MARK, K_FLAG_COUNT, K_FLAG_WRITE, K_EXPAND_FINAL, K_BFS,
                K_GATHER, K_DEGSUM, K_GREEDY, K_STAMP, K_PACK, K_ALLTOALL, K_BITS_COUNT, K_BITS_WRITE, K_COUNT };
static const char* const kKernelNames[K_COUNT] = {"k_degree", "k_scan_blocks", "k_expand<MARK>", "k_flag_count",
                                                  "k_flag_write", "k_expand<FINAL>", "k_expand<BFS>", "k_gather",
                                                  "k_degsum", "k_path_greedy", "k_stamp", "k_pack_bits",
                                                  "alltoall(xGMI)", "k_bits_count", "k_bits_write"};
constexpr int BITS_BLOCK = BLOCK * 64;           // k_bits_*: vertices (bits) per block

struct Prof {
  bool on = false;
  struct Rec { int kid, step, tix; hipEvent_t a, b; double cols, kout; bool path; };
  std::vector<Rec> pending;
  std::vector<hipEvent_t> pool;
  uint64_t launches[K_COUNT] = {};
  double ms[K_COUNT] = {};
  double bytes[K_COUNT] = {};
  hipEvent_t get() {
    if (!pool.empty()) { hipEvent_t e = pool.back(); pool.pop_back(); return e; }
    hipEvent_t e;
    (void)hipEventCreate(&e);
    return e;
  }
};

struct Workspace {
  Prof prof;
  hipStream_t stream = nullptr;
  uint64_t cap_frontier = 0;      // entries in each frontier / scan buffer
  uint64_t nv = 0;
  uint32_t* frontier[2] = {nullptr, nullptr};
  int cur = 0;
  uint32_t* seg_end = nullptr;    // block-local inclusive scan of degrees
  uint32_t* seg_rs = nullptr;     // row start per frontier entry
  uint32_t* block_sum = nullptr;  // per-block totals -> exclusive prefix (in place)
  uint64_t cap_blocks = 0;
  uint8_t* flags = nullptr;       // [nv rounded up to FLAG_BYTES], kept all-zero between steps
  uint64_t flag_bytes = 0;
  uint32_t* flag_blocks = nullptr;
  QState* q = nullptr;            // device query state
  QState* h_q = nullptr;          // pinned host mirror
  uint32_t* h_starts = nullptr;   // pinned staging for start ids
  uint64_t cap_starts = 0;
  Ins* h_prog = nullptr;          // pinned staging for programs
  int64_t* rows = nullptr;        // [ncols][cap_rows]
  uint64_t cap_rows = 0;
  int ncols_alloc = 0;
  int64_t** d_row_cols = nullptr; // device array of column pointers
  Ins* d_prog = nullptr;          // [MAX_TYPES_Q][MAX_PROGRAM]
  // FIND PATH (allocated on first use)
  PState* ps = nullptr;
  PState* h_ps = nullptr;         // pinned mirror
  uint32_t* lab[NUM_LABS] = {};   // [nv] epoch-stamped labels
  uint32_t epoch[NUM_LABS] = {};
  uint32_t* slot[PSLOTS] = {};    // frontier / B-set / meet lists
  uint64_t slot_cap = 0;
  uint32_t* pscratch = nullptr;   // claim shards
  uint64_t pscratch_cap = 0;
  int64_t* d_path = nullptr;      // [1 + 3 MAX_PATH_LEN]
  int64_t* h_path = nullptr;
  uint32_t* h_stage = nullptr;    // pinned [PSLOTS][STAGE] upload staging (one upload per slot per query)
  int rec = 0;                    // next PState expansion record
  // partitioned mode: flags cover the global id space [world * npad), one
  // bitmap segment of npad bits per owner rank is exchanged per hop
  Comm* comm = nullptr;
  uint64_t npad = 0;
  unsigned long long* sendbits = nullptr;   // [world * npad / 64]
  unsigned long long* recvbits = nullptr;   // [world * npad / 64]
  unsigned long long* mbits = nullptr;      // [npad / 64] OR of the received segments
  unsigned long long* gst = nullptr;        // [GST_N] globally reduced query statistics
  unsigned long long* h_gst = nullptr;
};

// ----------------------------------------------------------------------------- helpers
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

// Exclusive block scan of one value per thread; *total gets the block sum.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* total, uint32_t* lds) {
  uint32_t inc = wave_incl_scan(v);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 63) lds[w] = inc;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < WAVES; ++i) {
    uint32_t s = lds[i];
    pre += (i < w) ? s : 0u;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return pre + inc - v;
}

// ----------------------------------------------------------------------------- k_degree
// `reset` (nullable): NSHARD counters zeroed by block 0 (the BFS claim shards of the previous
// expansion, consumed by k_gather before this launch in stream order).
__global__ void __launch_bounds__(BLOCK) k_degree(const uint32_t* __restrict__ frontier,
                                                  const unsigned long long* __restrict__ np,
                                                  const uint32_t* __restrict__ row_ptr,
                                                  const uint8_t* __restrict__ visible, uint32_t cap,
                                                  uint32_t* __restrict__ seg_end, uint32_t* __restrict__ seg_rs,
                                                  uint32_t* __restrict__ block_sum, unsigned long long* reset,
                                                  unsigned long long* n_rec) {
  __shared__ uint32_t lds[WAVES];
  const uint64_t n = *np;
  if (blockIdx.x == 0) {
    if (reset && threadIdx.x < NSHARD) reset[threadIdx.x] = 0;
    if (n_rec && threadIdx.x == 0) *n_rec = n;
  }
  if ((uint64_t)blockIdx.x * SCAN_TILE >= n) return;
  const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_ITEMS;
  uint32_t deg[SCAN_ITEMS], rs[SCAN_ITEMS];
  uint32_t sum = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    uint64_t i = base + k;
    uint32_t d = 0, r = 0;
    if (i < n) {
      uint32_t v = frontier[i];
      if (v != NO_ROW && (!visible || visible[v])) {
        r = row_ptr[v];
        d = row_ptr[v + 1] - r;
        d = d < cap ? d : cap;
      }
    }
    deg[k] = d;
    rs[k] = r;
    sum += d;
  }
  uint32_t total;
  uint32_t pre = block_excl_scan(sum, &total, lds);
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    uint64_t i = base + k;
    pre += deg[k];
    if (i < n) {
      seg_end[i] = pre;   // inclusive, block-local
      seg_rs[i] = rs[k];
    }
  }
  if (threadIdx.x == 0) block_sum[blockIdx.x] = total;
}

// One workgroup: exclusive scan of nb uint32 in place.  nb = fixed_nb, or ceil(*np / 2048) when
// fixed_nb == 0.  The grand total goes to *total_out and is added to *accum (stats, nullable).
__global__ void __launch_bounds__(1024) k_scan_blocks(uint32_t* __restrict__ v, const unsigned long long* np,
                                                      uint64_t fixed_nb, unsigned long long* total_out,
                                                      unsigned long long* accum) {
  __shared__ uint64_t lds[16];
  __shared__ uint64_t carry;
  const uint64_t nb = fixed_nb ? fixed_nb : (*np + SCAN_TILE - 1) / SCAN_TILE;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint64_t base = 0; base < nb; base += 1024) {
    uint64_t i = base + threadIdx.x;
    uint64_t x = i < nb ? v[i] : 0;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t inc = x;
    for (int o = 1; o < 64; o <<= 1) {
      uint64_t t = __shfl_up(inc, o, 64);
      if (lane >= o) inc += t;
    }
    if (lane == 63) lds[w] = inc;
    __syncthreads();
    uint64_t pre = 0, tot = 0;
    for (int k = 0; k < 16; ++k) {
      pre += (k < w) ? lds[k] : 0;
      tot += lds[k];
    }
    uint64_t c = carry;
    if (i < nb) v[i] = (uint32_t)(c + pre + inc - x);
    __syncthreads();
    if (threadIdx.x == 0) carry = c + tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    *total_out = carry;
    if (accum) *accum += carry;
  }
}

__device__ __forceinline__ uint32_t seg_end_at(const uint32_t* __restrict__ seg_end,
                                               const uint32_t* __restrict__ block_pre, uint64_t i) {
  return seg_end[i] + block_pre[i >> SCAN_SHIFT];
}

// Merge-path split: number of frontier segments fully consumed in the first d path items, i.e.
// the smallest i with NOT(end(i) <= d-1-i).  Computed by one whole wave as a 64-ary search:
// each round the 64 lanes probe 64 evenly spaced candidates in parallel (one memory round trip)
// and a ballot narrows the range 64x, so a split costs ceil(log64(n)) <= 5 round trips instead
// of ~25 dependent loads of a binary search.
__device__ __forceinline__ uint64_t wave_merge_split(const uint32_t* __restrict__ seg_end,
                                                     const uint32_t* __restrict__ block_pre, uint64_t n,
                                                     uint64_t total, uint64_t d) {
  const int lane = threadIdx.x & 63;
  uint64_t lo = d > total ? d - total : 0;
  uint64_t hi = d < n ? d : n;
  while (lo < hi) {
    const uint64_t step = (hi - lo + 63) >> 6;
    const uint64_t p = lo + (uint64_t)lane * step;
    bool t = p < hi && (uint64_t)seg_end_at(seg_end, block_pre, p) <= d - 1 - p;
    const int c = __popcll(__ballot(t));
    const uint64_t nlo = c > 0 ? lo + (uint64_t)(c - 1) * step + 1 : lo;
    uint64_t nhi = lo + (uint64_t)c * step;
    if (nhi > hi) nhi = hi;
    lo = nlo;
    hi = nhi;
  }
  return lo;
}

// Fast path for the common final-step program shape: WHERE absent or `col <cmp> const` on an
// INT column, YIELD columns that are plain edge fields / key props / constants.  No
// interpreter, no LDS registers; the generic bytecode path handles everything else.
struct FastProg {
  int enabled;
  int where_col;           // -1: no WHERE
  int where_op;            // 0 LT 1 LE 2 GT 3 GE 4 EQ 5 NE (int64)
  int64_t where_const;
  int ykind[MAX_YIELDS];   // 0 DST, 1 SRC, 2 RANK, 3 COL, 4 CONST
  int ycol[MAX_YIELDS];
};

__device__ __forceinline__ bool cmp_i(int op, int64_t x, int64_t y) {
  switch (op) {
    case 0: return x < y;
    case 1: return x <= y;
    case 2: return x > y;
    case 3: return x >= y;
    case 4: return x == y;
    default: return x != y;
  }
}

// ----------------------------------------------------------------------------- bytecode
struct EdgeCtx {
  uint64_t j;       // edge index in CSR
  uint32_t v;       // source dense id
};

__device__ __forceinline__ double as_f(int64_t x) { return __longlong_as_double(x); }
__device__ __forceinline__ int64_t fbits(double d) { return __double_as_longlong(d); }

// Evaluate instructions [pc0, pc1) for this lane.  Registers live in LDS, one 8-byte slot per
// lane per register ([reg][BLOCK]); instruction fetch is wave-uniform (scalar loads).
__device__ __forceinline__ void run_program(const Ins* __restrict__ prog, int pc0, int pc1, const EdgeCtx& c,
                                            const ExpandArgs& a, int64_t* __restrict__ regs, bool active,
                                            bool& err) {
  const int tid = threadIdx.x;
  for (int pc = pc0; pc < pc1; ++pc) {
    const Ins ins = prog[pc];
    int64_t x = regs[ins.a * BLOCK + tid];
    int64_t y = regs[ins.b * BLOCK + tid];
    int64_t r = 0;
    switch (ins.op) {
      case OP_CONST: r = ins.imm; break;
      case OP_COL: r = active ? a.props[ins.aux][c.j] : 0; break;
      case OP_COLV:
        if (active) {
          if (!a.valid[c.j]) err = true;
          r = a.props[ins.aux][c.j];
        }
        break;
      case OP_DST: r = active ? a.dst_vid[c.j] : 0; break;
      case OP_SRC: r = active ? a.vids[c.v] : 0; break;
      case OP_RANK: r = (active && a.rank) ? a.rank[c.j] : 0; break;
      case OP_ERR: err = true; break;
      case OP_ADD_I: r = (int64_t)((uint64_t)x + (uint64_t)y); break;
      case OP_SUB_I: r = (int64_t)((uint64_t)x - (uint64_t)y); break;
      case OP_MUL_I: r = (int64_t)((uint64_t)x * (uint64_t)y); break;
      case OP_DIV_I:
      case OP_MOD_I:
        if (y == 0 || (x == INT64_MIN && y == -1)) { err = true; r = 0; }
        else r = ins.op == OP_DIV_I ? x / y : x % y;
        break;
      case OP_XOR_I: r = x ^ y; break;
      case OP_NEG_I: r = (int64_t)(0ull - (uint64_t)x); break;
      case OP_LT_I: r = x < y; break;
      case OP_LE_I: r = x <= y; break;
      case OP_GT_I: r = x > y; break;
      case OP_GE_I: r = x >= y; break;
      case OP_EQ_I: r = x == y; break;
      case OP_NE_I: r = x != y; break;
      case OP_ADD_F: r = fbits(as_f(x) + as_f(y)); break;
      case OP_SUB_F: r = fbits(as_f(x) - as_f(y)); break;
      case OP_MUL_F: r = fbits(as_f(x) * as_f(y)); break;
      case OP_DIV_F: r = fbits(as_f(x) / as_f(y)); break;
      case OP_MOD_F: r = fbits(fmod(as_f(x), as_f(y))); break;
      case OP_XOR_F: r = (int64_t)llround(as_f(x)) ^ (int64_t)llround(as_f(y)); break;
      case OP_NEG_F: r = fbits(-as_f(x)); break;
      // boost::variant: >, <=, >= derive from < (NaN makes <= and >= true)
      case OP_LT_F: r = as_f(x) < as_f(y); break;
      case OP_LE_F: r = !(as_f(y) < as_f(x)); break;
      case OP_GT_F: r = as_f(y) < as_f(x); break;
      case OP_GE_F: r = !(as_f(x) < as_f(y)); break;
      case OP_EQ_F: r = fabs(as_f(x) - as_f(y)) < 1e-8; break;
      case OP_NE_F: r = !(fabs(as_f(x) - as_f(y)) < 1e-8); break;
      case OP_I2F: r = fbits((double)x); break;
      case OP_B2I: r = x != 0; break;
      case OP_B2F: r = fbits(x != 0 ? 1.0 : 0.0); break;
      case OP_F2I: r = (int64_t)as_f(x); break;
      case OP_NOT: r = x == 0; break;
      case OP_TRUTHY_I: r = x != 0; break;
      case OP_TRUTHY_F: r = as_f(x) != 0.0; break;
      case OP_TRUTHY_S: r = x == ins.imm; break;
      case OP_AND: r = (x != 0) && (y != 0); break;
      case OP_OR: r = (x != 0) || (y != 0); break;
      case OP_XORB: r = (x != 0) != (y != 0); break;
      default: break;
    }
    regs[ins.d * BLOCK + tid] = r;
  }
}

// ----------------------------------------------------------------------------- k_expand
enum Mode { MARK = 0, FINAL = 1, BFS = 2 };

// BFS-mode expansion (FIND SHORTEST PATH): every neighbour w is claimed at most once per epoch by
// a CAS on its label (epoch << LVL_BITS | level); winners are appended, one atomic per tile on a
// sharded counter, to NSHARD regions of `out` that k_gather then packs into the next frontier.
struct BfsParams {
  uint32_t* lab;                  // claim labels
  uint32_t stamp;                 // claimed label value
  uint32_t epoch;                 // a label is live when (lab >> LVL_BITS) == epoch
  const uint32_t* rlab;           // restriction (nullable): claim w only if rlab[w] == rstamp
  uint32_t rstamp;
  const uint32_t* mlab;           // meet test (nullable): a claimed w with a live mlab label met
  uint32_t mepoch;                //   the other search side
  uint32_t* mout;                 // meets: mout[w] = mstamp, w appended to meet_list
  uint32_t mstamp;
  uint32_t* meet_list;
  unsigned long long* meet_n;
  const uint32_t* tlab;           // targets (nullable): claimed w with tlab[w] == tstamp counts
  uint32_t tstamp;
  unsigned long long* found;
  uint32_t* out;                  // shard regions [NSHARD][shard_cap]
  uint64_t shard_cap;
  unsigned long long* shard_cnt;  // [NSHARD]
};

struct FinalParams {
  const Ins* prog;
  int where_len;
  int where_reg;          // -1 none
  int prog_len;           // WHERE + YIELD instructions
  int nyields;
  int yield_reg[MAX_YIELDS];
  int64_t yield_const[MAX_YIELDS];
  int64_t** out_cols;
  uint64_t region_base;   // first row of this type's region
  uint64_t shard_cap;     // rows per shard region
  unsigned long long* shard_rows;   // [NSHARD] counters of this type
  unsigned long long* err_flag;
  FastProg fast;
};

template <int M>
__global__ void __launch_bounds__(BLOCK) k_expand(ExpandArgs a, const unsigned long long* __restrict__ np,
                                                  const unsigned long long* __restrict__ totp,
                                                  const uint32_t* __restrict__ seg_end,
                                                  const uint32_t* __restrict__ block_pre,
                                                  const uint32_t* __restrict__ seg_rs, uint8_t* __restrict__ flags,
                                                  FinalParams fp, BfsParams bp) {
  __shared__ uint32_t sEnd[TILE + 2];   // seg_end for i in [a0-1, a1]
  __shared__ uint32_t sRs[TILE + 1];    // seg_rs for i in [a0, a1]
  __shared__ uint32_t sSeg[TILE];       // segment of each edge item in this tile
  __shared__ uint32_t sCnt[VT * WAVES]; // FINAL: passing items per (iteration, wave) -> offsets
  __shared__ uint64_t sSplit[2];
  __shared__ uint64_t sBase;
  extern __shared__ int64_t regs[];     // FINAL generic path: [nregs][BLOCK]

  const uint64_t n = *np;
  const uint64_t total = *totp;
  const uint64_t npath = n + total;
  const uint64_t ntiles = (npath + TILE - 1) / TILE;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  bool anyErr = false;

  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const uint64_t d0 = t * TILE;
    const uint64_t d1 = (d0 + TILE < npath) ? d0 + TILE : npath;
    if (w < 2) {
      uint64_t sp = wave_merge_split(seg_end, block_pre, n, total, w ? d1 : d0);
      if (lane == 0) sSplit[w] = sp;
    }
    __syncthreads();
    const uint64_t a0 = sSplit[0], a1 = sSplit[1];
    const uint64_t b0 = d0 - a0, b1 = d1 - a1;
    const int na = (int)(a1 - a0), nb = (int)(b1 - b0);

    // stage the tile's segment ends / row starts in LDS
    for (int k = threadIdx.x; k <= na + 1; k += BLOCK) {
      int64_t i = (int64_t)a0 - 1 + k;
      sEnd[k] = (i < 0) ? 0u : (i < (int64_t)n ? seg_end_at(seg_end, block_pre, (uint64_t)i) : 0xFFFFFFFFu);
    }
    for (int k = threadIdx.x; k <= na; k += BLOCK) {
      uint64_t i = a0 + k;
      sRs[k] = i < n ? seg_rs[i] : 0u;
    }
    __syncthreads();
    const uint32_t* A = sEnd + 1;   // A[k] = end of segment a0 + k

    // thread-level merge path over this tile: assign a segment to every edge item
    {
      int diag = threadIdx.x * VT;
      int dmax = na + nb;
      if (diag < dmax) {
        int lo = diag > nb ? diag - nb : 0;
        int hi = diag < na ? diag : na;
        while (lo < hi) {
          int mid = (lo + hi) >> 1;
          if ((uint64_t)A[mid] <= b0 + (uint64_t)(diag - 1 - mid)) lo = mid + 1;
          else hi = mid;
        }
        int ai = lo, bi = diag - lo;
#pragma unroll
        for (int k = 0; k < VT; ++k) {
          if (ai + bi >= dmax) break;
          if (ai < na && (bi >= nb || (uint64_t)A[ai] <= b0 + (uint64_t)bi)) {
            ++ai;
          } else {
            sSeg[bi] = (uint32_t)ai;
            ++bi;
          }
        }
      }
    }
    __syncthreads();

    if (M == MARK) {
      for (int k = threadIdx.x; k < nb; k += BLOCK) {
        uint32_t s = sSeg[k];
        uint64_t e = b0 + k;
        uint64_t j = (uint64_t)sRs[s] + (e - (uint64_t)sEnd[s]);   // sEnd[s] = start of segment a0+s
        uint32_t u = a.col[j];
        if (u != NO_ROW) flags[u] = 1;
      }
    } else if (M == BFS) {
      uint32_t wv[VT];
      uint32_t cmask = 0, mmask = 0;
#pragma unroll
      for (int i = 0; i < VT; ++i) {
        const int k = i * BLOCK + threadIdx.x;
        wv[i] = NO_ROW;
        if (k < nb) {
          uint32_t s = sSeg[k];
          wv[i] = a.col[(uint64_t)sRs[s] + (b0 + k - (uint64_t)sEnd[s])];
        }
      }
#pragma unroll
      for (int i = 0; i < VT; ++i) {
        const uint32_t x = wv[i];
        if (x == NO_ROW) continue;
        if (bp.rlab && bp.rlab[x] != bp.rstamp) continue;
        const uint32_t old = bp.lab[x];
        if ((old >> LVL_BITS) == bp.epoch) continue;
        if (atomicCAS(bp.lab + x, old, bp.stamp) != old) continue;
        cmask |= 1u << i;
        if (bp.mlab && (bp.mlab[x] >> LVL_BITS) == bp.mepoch) mmask |= 1u << i;
        if (bp.tlab && bp.tlab[x] == bp.tstamp) atomicAdd(bp.found, 1ull);
      }
#pragma unroll
      for (int i = 0; i < VT; ++i) {
        unsigned long long bal = __ballot((cmask >> i) & 1u);
        if (lane == 0) sCnt[i * WAVES + w] = (uint32_t)__popcll(bal);
      }
      __syncthreads();
      const uint64_t shard = t % NSHARD;
      if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (int k = 0; k < VT * WAVES; ++k) {
          uint32_t c = sCnt[k];
          sCnt[k] = run;
          run += c;
        }
        sBase = run ? atomicAdd(bp.shard_cnt + shard, (unsigned long long)run) : 0ull;
      }
      __syncthreads();
      uint32_t* const region = bp.out + shard * bp.shard_cap + sBase;
      for (int i = 0; i < VT; ++i) {
        const bool c = (cmask >> i) & 1u;
        unsigned long long bal = __ballot(c);
        if (c) region[sCnt[i * WAVES + w] + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull))] = wv[i];
        const bool m = (mmask >> i) & 1u;
        unsigned long long mb = __ballot(m);
        if (mb) {
          unsigned long long base = 0;
          if (lane == 0) base = atomicAdd(bp.meet_n, (unsigned long long)__popcll(mb));
          base = __shfl(base, 0, 64);
          if (m) {
            bp.meet_list[base + (uint32_t)__popcll(mb & ((1ull << lane) - 1ull))] = wv[i];
            bp.mout[wv[i]] = bp.mstamp;
          }
        }
      }
    } else {
      // phase A: WHERE for every item of the tile (VT items per thread, striped)
      uint64_t jj[VT];
      uint32_t vv[VT];
      uint32_t pmask = 0;
#pragma unroll
      for (int i = 0; i < VT; ++i) {
        const int k = i * BLOCK + threadIdx.x;
        jj[i] = 0;
        vv[i] = 0;
        if (k < nb) {
          uint32_t s = sSeg[k];
          jj[i] = (uint64_t)sRs[s] + (b0 + k - (uint64_t)sEnd[s]);
          vv[i] = s;
        }
      }
      if (fp.fast.enabled) {
        if (fp.fast.where_col < 0) {
#pragma unroll
          for (int i = 0; i < VT; ++i) pmask |= (uint32_t)(i * BLOCK + (int)threadIdx.x < nb) << i;
        } else {
          const int64_t* __restrict__ wc = a.props[fp.fast.where_col];
          int64_t x[VT];
#pragma unroll
          for (int i = 0; i < VT; ++i) x[i] = (i * BLOCK + (int)threadIdx.x < nb) ? wc[jj[i]] : 0;
#pragma unroll
          for (int i = 0; i < VT; ++i)
            pmask |= (uint32_t)((i * BLOCK + (int)threadIdx.x < nb) && cmp_i(fp.fast.where_op, x[i],
                                                                               fp.fast.where_const)) << i;
        }
      } else {
        for (int i = 0; i < VT; ++i) {
          const int k = i * BLOCK + threadIdx.x;
          const bool active = k < nb;
          bool pass = active;
          if (fp.where_reg >= 0) {
            bool werr = false;
            EdgeCtx c{jj[i], active ? a.frontier[a0 + vv[i]] : 0u};
            run_program(fp.prog, 0, fp.where_len, c, a, regs, active, werr);
            pass = active && !werr && regs[fp.where_reg * BLOCK + threadIdx.x] != 0;
            if (active && werr) anyErr = true;
          }
          pmask |= (uint32_t)pass << i;
        }
      }
      // one atomic per tile on a sharded counter: offsets for (iteration, wave) in item order
#pragma unroll
      for (int i = 0; i < VT; ++i) {
        unsigned long long bal = __ballot((pmask >> i) & 1u);
        if (lane == 0) sCnt[i * WAVES + w] = (uint32_t)__popcll(bal);
      }
      __syncthreads();
      const uint64_t shard = t % NSHARD;
      if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (int k = 0; k < VT * WAVES; ++k) {
          uint32_t c = sCnt[k];
          sCnt[k] = run;
          run += c;
        }
        sBase = run ? atomicAdd(fp.shard_rows + shard, (unsigned long long)run) : 0ull;
      }
      __syncthreads();
      // phase B: YIELD for the passing items, written at their final rows
      const uint64_t region = fp.region_base + shard * fp.shard_cap + sBase;
      int64_t* const* cols = fp.out_cols;
      for (int i = 0; i < VT; ++i) {
        const bool pass = (pmask >> i) & 1u;
        unsigned long long bal = __ballot(pass);
        if (!bal) continue;
        const uint64_t row = region + sCnt[i * WAVES + w] + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
        if (fp.fast.enabled) {
          if (pass) {
            for (int y = 0; y < fp.nyields; ++y) {
              int64_t val;
              switch (fp.fast.ykind[y]) {
                case 0: val = a.dst_vid[jj[i]]; break;
                case 1: val = a.vids[a.frontier[a0 + vv[i]]]; break;
                case 2: val = a.rank ? a.rank[jj[i]] : 0; break;
                case 3: val = a.props[fp.fast.ycol[y]][jj[i]]; break;
                default: val = fp.yield_const[y]; break;
              }
              cols[y][row] = val;
            }
          }
        } else {
          bool yerr = false;
          EdgeCtx c{jj[i], pass ? a.frontier[a0 + vv[i]] : 0u};
          run_program(fp.prog, fp.where_len, fp.prog_len, c, a, regs, pass, yerr);
          if (pass && yerr) anyErr = true;
          if (pass) {
            for (int y = 0; y < fp.nyields; ++y) {
              int r = fp.yield_reg[y];
              cols[y][row] = r >= 0 ? regs[r * BLOCK + threadIdx.x] : fp.yield_const[y];
            }
          }
        }
      }
    }
    __syncthreads();   // LDS reuse by the next tile
  }
  if (M == FINAL && anyErr) atomicOr(fp.err_flag, 1ull);
}

// ----------------------------------------------------------------------------- flag compaction
__global__ void __launch_bounds__(BLOCK) k_flag_count(const uint8_t* __restrict__ flags, uint64_t nbytes,
                                                      uint32_t* __restrict__ block_cnt) {
  __shared__ uint32_t lds[WAVES];
  uint64_t off = (uint64_t)blockIdx.x * FLAG_BYTES + threadIdx.x * 16;
  uint32_t c = 0;
  if (off < nbytes) {
    uint4 q = *reinterpret_cast<const uint4*>(flags + off);
    uint32_t ws[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) c += __popc(ws[i] & 0x01010101u);
  }
  uint32_t tot;
  block_excl_scan(c, &tot, lds);
  if (threadIdx.x == 0) block_cnt[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(BLOCK) k_flag_write(uint8_t* __restrict__ flags, uint64_t nbytes, uint64_t nv,
                                                      const uint32_t* __restrict__ block_pre,
                                                      uint32_t* __restrict__ out) {
  __shared__ uint32_t lds[WAVES];
  uint64_t off = (uint64_t)blockIdx.x * FLAG_BYTES + threadIdx.x * 16;
  uint32_t ws[4] = {0, 0, 0, 0};
  uint32_t c = 0;
  if (off < nbytes) {
    uint4 q = *reinterpret_cast<const uint4*>(flags + off);
    ws[0] = q.x; ws[1] = q.y; ws[2] = q.z; ws[3] = q.w;
#pragma unroll
    for (int i = 0; i < 4; ++i) c += __popc(ws[i] & 0x01010101u);
  }
  uint32_t tot;
  uint32_t pre = block_excl_scan(c, &tot, lds) + block_pre[blockIdx.x];
  if (c) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if ((ws[i >> 2] >> ((i & 3) * 8)) & 1u) {
        uint64_t v = off + i;
        if (v < nv) out[pre++] = (uint32_t)v;
      }
    }
    *reinterpret_cast<uint4*>(flags + off) = make_uint4(0, 0, 0, 0);
  }
}

// ----------------------------------------------------------------------------- partitioned exchange
// Pack the byte flags of the global id space into a bitmap (one 64-bit word per 64 flags) and
// clear them.  Segment q of the bitmap (npad bits) holds the next-frontier candidates owned by
// rank q; the all-to-all hands every owner the G segments that concern it.
__global__ void __launch_bounds__(BLOCK) k_pack_bits(uint8_t* __restrict__ flags, uint64_t nwords,
                                                     unsigned long long* __restrict__ bits) {
  const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (i >= nwords) return;
  uint4* p = reinterpret_cast<uint4*>(flags + i * 64);
  unsigned long long m = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint4 q = p[k];
    const uint32_t ws[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {   // flag bytes are 0 or 1
      const uint32_t x = ws[j];
      const unsigned long long b = (x & 1u) | ((x >> 7) & 2u) | ((x >> 14) & 4u) | ((x >> 21) & 8u);
      m |= b << (k * 16 + j * 4);
    }
  }
  bits[i] = m;
  if (m) {
#pragma unroll
    for (int k = 0; k < 4; ++k) p[k] = make_uint4(0, 0, 0, 0);
  }
}

// Owner side: OR the G received segments (one per sending rank) of this rank's id range; the
// union is the global per-step dst SET restricted to the owner (getDstIdsFromResp).
__global__ void __launch_bounds__(BLOCK) k_bits_count(const unsigned long long* __restrict__ recv, int world,
                                                      uint64_t seg_words, uint64_t nv,
                                                      unsigned long long* __restrict__ merged,
                                                      uint32_t* __restrict__ block_cnt) {
  __shared__ uint32_t lds[WAVES];
  const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  unsigned long long m = 0;
  for (int q = 0; q < world; ++q) m |= recv[(uint64_t)q * seg_words + i];
  const uint64_t lo = i * 64;
  if (lo >= nv) m = 0;
  else if (nv - lo < 64) m &= (1ull << (nv - lo)) - 1ull;
  merged[i] = m;
  uint32_t tot;
  block_excl_scan((uint32_t)__popcll(m), &tot, lds);
  if (threadIdx.x == 0) block_cnt[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(BLOCK) k_bits_write(const unsigned long long* __restrict__ merged,
                                                      const uint32_t* __restrict__ block_pre,
                                                      uint32_t* __restrict__ out) {
  __shared__ uint32_t lds[WAVES];
  const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  unsigned long long m = merged[i];
  uint32_t tot;
  uint32_t pre = block_excl_scan((uint32_t)__popcll(m), &tot, lds) + block_pre[blockIdx.x];
  while (m) {
    const int b = __ffsll((long long)m) - 1;
    out[pre++] = (uint32_t)(i * 64 + b);
    m &= m - 1;
  }
}

// Query statistics every rank needs globally: [err, step_n[0..MAX_STEPS+1], Σ_types e_st[s]].
constexpr int GST_N = 1 + 2 * (MAX_STEPS + 2);
__global__ void k_gstats(const QState* __restrict__ q, int ntypes, unsigned long long* __restrict__ g) {
  const int s = threadIdx.x;
  if (s == 0) g[0] = q->err ? 1ull : 0ull;
  if (s < MAX_STEPS + 2) {
    g[1 + s] = q->step_n[s];
    unsigned long long e = 0;
    for (int t = 0; t < ntypes; ++t) e += q->e_st[s][t];
    g[1 + (MAX_STEPS + 2) + s] = e;
  }
}

// ============================================================================= host side
static inline uint64_t cdiv(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

#define HIP_TRY(x)                         \
  do {                                     \
    hipError_t e_ = (x);                   \
    if (e_ != hipSuccess) return e_;       \
  } while (0)

// Kernel timing: an event pair around each launch on the workspace stream, resolved after the
// query's single host synchronisation (byte counts need the device-side sizes).
static hipEvent_t prof_begin(Workspace* w) {
  if (!w->prof.on) return nullptr;
  hipEvent_t a = w->prof.get();
  (void)hipEventRecord(a, w->stream);
  return a;
}
static void prof_end(Workspace* w, hipEvent_t a, int kid, int step, int tix, double cols = 0, double kout = 0) {
  if (!a) return;
  hipEvent_t b = w->prof.get();
  (void)hipEventRecord(b, w->stream);
  w->prof.pending.push_back({kid, step, tix, a, b, cols, kout, false});
}
// algorithmic bytes per kernel (SURVEY.md §8(d) B_GO terms)
static double prof_bytes(const Prof::Rec& r, const QState& q) {
  switch (r.kid) {
    case K_DEGREE: return 12.0 * (double)q.step_n[r.step];                 // 4|F| ids + 8|F| row_ptr
    case K_EXPAND_MARK: return 4.0 * (double)q.e_st[r.step][r.tix];        // 4 E_s neighbour ids
    case K_FLAG_WRITE: return 4.0 * (double)q.step_n[r.step + 1];          // write F_{s+1}
    case K_BITS_WRITE: return 4.0 * (double)q.step_n[r.step + 1];
    case K_PACK: case K_ALLTOALL: case K_BITS_COUNT: return r.cols;       // fixed sizes (set at launch)
    case K_EXPAND_FINAL: {
      double rows = 0;
      for (int s = 0; s < NSHARD; ++s) rows += (double)q.rows[r.tix][s];
      // SURVEY §8(d) B_GO final-step terms: 4 E_N neighbour ids + 8 E_N per WHERE/YIELD edge
      // property column + 8 k per emitted row
      return (double)q.e_st[r.step][r.tix] * (4.0 + 8.0 * r.cols) + 8.0 * rows * r.kout;
    }
    default: return 0.0;
  }
}
// FIND PATH launches: r.step indexes the per-query expansion records of PState (B_SP terms:
// 4|F| ids + 8|F| row_ptr, 4 E neighbour ids, 4 per claimed vertex written)
static double prof_bytes_path(const Prof::Rec& r, const PState& p) {
  const int i = r.step < PATH_REC ? r.step : PATH_REC - 1;
  switch (r.kid) {
    case K_DEGREE: return 12.0 * (double)p.ln[i];
    case K_BFS: return 4.0 * (double)p.le[i];
    case K_GATHER: return 8.0 * (double)p.lc[i];
    case K_DEGSUM: return 12.0 * (double)p.ln[i];
    default: return 0.0;
  }
}
static void prof_flush(Workspace* w, const QState* q, const PState* ps = nullptr) {
  for (auto& r : w->prof.pending) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
      w->prof.launches[r.kid]++;
      w->prof.ms[r.kid] += ms;
      if (r.path) {
        if (ps) w->prof.bytes[r.kid] += prof_bytes_path(r, *ps);
      } else if (q) {
        w->prof.bytes[r.kid] += prof_bytes(r, *q);
      }
    }
    w->prof.pool.push_back(r.a);
    w->prof.pool.push_back(r.b);
  }
  w->prof.pending.clear();
}

void ws_profile(Workspace* w, bool on) {
  if (!w) return;
  prof_flush(w, nullptr);
  w->prof.on = on;
  if (on) {
    for (int k = 0; k < K_COUNT; ++k) { w->prof.launches[k] = 0; w->prof.ms[k] = 0; w->prof.bytes[k] = 0; }
  }
}

int ws_profile_read(Workspace* w, nbg_kernel_stat* out, int cap) {
  if (!w) return 0;
  int n = 0;
  for (int k = 0; k < K_COUNT && n < cap; ++k) {
    out[n].name = kKernelNames[k];
    out[n].launches = w->prof.launches[k];
    out[n].total_ms = w->prof.ms[k];
    out[n].algo_bytes = w->prof.bytes[k];
    ++n;
  }
  return n;
}

Workspace* ws_create(uint64_t max_frontier, uint64_t nv, hipStream_t s, std::string* err) {
  auto* w = new Workspace();
  w->stream = s;
  w->nv = nv;
  w->cap_frontier = max_frontier < 1024 ? 1024 : max_frontier;
  w->cap_blocks = cdiv(w->cap_frontier, SCAN_TILE) + 1;
  w->flag_bytes = cdiv(nv + 1, FLAG_BYTES) * FLAG_BYTES;
  uint64_t fblocks = w->flag_bytes / FLAG_BYTES + 1;
  if (fblocks > w->cap_blocks) w->cap_blocks = fblocks;
  hipError_t e = hipSuccess;
  auto M = [&](void** p, size_t b) { if (e == hipSuccess) e = hipMalloc(p, b); };
  M((void**)&w->frontier[0], w->cap_frontier * 4);
  M((void**)&w->frontier[1], w->cap_frontier * 4);
  M((void**)&w->seg_end, w->cap_frontier * 4);
  M((void**)&w->seg_rs, w->cap_frontier * 4);
  M((void**)&w->block_sum, w->cap_blocks * 4);
  M((void**)&w->flags, w->flag_bytes);
  M((void**)&w->flag_blocks, w->cap_blocks * 4);
  M((void**)&w->q, sizeof(QState));
  M((void**)&w->d_prog, (size_t)MAX_TYPES_Q * MAX_PROGRAM * sizeof(Ins));
  M((void**)&w->d_row_cols, MAX_YIELDS * sizeof(int64_t*));
  if (e == hipSuccess) e = hipHostMalloc((void**)&w->h_q, sizeof(QState), hipHostMallocDefault);
  if (e == hipSuccess) e = hipHostMalloc((void**)&w->h_prog, (size_t)MAX_TYPES_Q * MAX_PROGRAM * sizeof(Ins),
                                         hipHostMallocDefault);
  if (e == hipSuccess) e = hipMemsetAsync(w->flags, 0, w->flag_bytes, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    if (err) *err = std::string("workspace allocation failed: ") + hipGetErrorString(e);
    ws_destroy(w);
    return nullptr;
  }
  return w;
}

void ws_destroy(Workspace* w) {
  if (!w) return;
  for (void* p : {(void*)w->frontier[0], (void*)w->frontier[1], (void*)w->seg_end, (void*)w->seg_rs,
                  (void*)w->block_sum, (void*)w->flags, (void*)w->flag_blocks, (void*)w->q, (void*)w->rows,
                  (void*)w->d_row_cols, (void*)w->d_prog})
    if (p) (void)hipFree(p);
  for (void* p : {(void*)w->h_q, (void*)w->h_starts, (void*)w->h_prog, (void*)w->h_ps, (void*)w->h_path,
                  (void*)w->h_stage})
    if (p) (void)hipHostFree(p);
  for (void* p : {(void*)w->sendbits, (void*)w->recvbits, (void*)w->mbits, (void*)w->gst})
    if (p) (void)hipFree(p);
  if (w->h_gst) (void)hipHostFree(w->h_gst);
  for (void* p : {(void*)w->ps, (void*)w->pscratch, (void*)w->d_path})
    if (p) (void)hipFree(p);
  for (auto* p : w->lab)
    if (p) (void)hipFree(p);
  for (auto* p : w->slot)
    if (p) (void)hipFree(p);
  for (auto& r : w->prof.pending) { (void)hipEventDestroy(r.a); (void)hipEventDestroy(r.b); }
  for (auto e : w->prof.pool) (void)hipEventDestroy(e);
  delete w;
}

uint64_t ws_cap_frontier(Workspace* w) { return w->cap_frontier; }
int64_t* ws_row_col(Workspace* w, int c) { return w->rows + (uint64_t)c * w->cap_rows; }
const QState* ws_host_state(Workspace* w) { return w->h_q; }
const uint32_t* ws_current_frontier(Workspace* w) { return w->frontier[w->cur]; }

hipError_t ws_reserve_rows(Workspace* w, uint64_t rows, int ncols) {
  if (rows <= w->cap_rows && ncols <= w->ncols_alloc) return hipSuccess;
  HIP_TRY(hipStreamSynchronize(w->stream));
  if (w->rows) HIP_TRY(hipFree(w->rows));
  w->rows = nullptr;
  uint64_t cap = rows < 1024 ? 1024 : rows;
  if (cap < w->cap_rows) cap = w->cap_rows;
  int nc = ncols < 1 ? 1 : ncols;
  if (nc < w->ncols_alloc) nc = w->ncols_alloc;
  HIP_TRY(hipMalloc((void**)&w->rows, cap * nc * sizeof(int64_t)));
  w->cap_rows = cap;
  w->ncols_alloc = nc;
  int64_t* cols[MAX_YIELDS];
  for (int c = 0; c < MAX_YIELDS; ++c) cols[c] = w->rows + (uint64_t)(c < nc ? c : 0) * cap;
  HIP_TRY(hipMemcpy(w->d_row_cols, cols, sizeof(cols), hipMemcpyHostToDevice));
  return hipSuccess;
}

hipError_t ws_begin_query(Workspace* w, const uint32_t* starts, uint64_t n, const std::vector<TypeProgram>* progs) {
  if (n > w->cap_frontier) return hipErrorInvalidValue;
  if (n > w->cap_starts) {
    if (w->h_starts) HIP_TRY(hipHostFree(w->h_starts));
    w->cap_starts = n + n / 2 + 1024;
    HIP_TRY(hipHostMalloc((void**)&w->h_starts, w->cap_starts * 4, hipHostMallocDefault));
  }
  // the previous query on this workspace has completed (its end synchronised the stream)
  memcpy(w->h_starts, starts, n * 4);
  memset(w->h_q, 0, sizeof(QState));
  w->h_q->n = n;
  w->h_q->step_n[1] = n;
  w->cur = 0;
  HIP_TRY(hipMemcpyAsync(w->frontier[0], w->h_starts, n * 4, hipMemcpyHostToDevice, w->stream));
  HIP_TRY(hipMemcpyAsync(w->q, w->h_q, sizeof(QState), hipMemcpyHostToDevice, w->stream));
  if (progs && !progs->empty()) {
    size_t k = 0;
    for (auto& p : *progs) {
      memcpy(w->h_prog + k * MAX_PROGRAM, p.code.data(), p.code.size() * sizeof(Ins));
      ++k;
    }
    HIP_TRY(hipMemcpyAsync(w->d_prog, w->h_prog, k * MAX_PROGRAM * sizeof(Ins), hipMemcpyHostToDevice, w->stream));
  }
  return hipSuccess;
}

// Enqueue k_degree + k_scan_blocks for the current frontier (n <= n_bound) over one type.
static hipError_t enqueue_scan(Workspace* w, const ExpandArgs& a, uint64_t n_bound, int step, int tix) {
  uint64_t nb = cdiv(n_bound ? n_bound : 1, SCAN_TILE);
  hipEvent_t p = prof_begin(w);
  hipLaunchKernelGGL(k_degree, dim3((unsigned)nb), dim3(BLOCK), 0, w->stream, w->frontier[w->cur], &w->q->n,
                     a.row_ptr, a.visible, a.cap, w->seg_end, w->seg_rs, w->block_sum,
                     (unsigned long long*)nullptr, (unsigned long long*)nullptr);
  prof_end(w, p, K_DEGREE, step, tix);
  p = prof_begin(w);
  hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(1024), 0, w->stream, w->block_sum, &w->q->n, (uint64_t)0,
                     &w->q->total, &w->q->e_st[step][tix]);
  prof_end(w, p, K_SCAN, step, tix);
  return hipGetLastError();
}

static unsigned expand_grid(uint64_t n_bound, uint64_t e_bound) {
  uint64_t tiles = cdiv(n_bound + e_bound + 1, TILE);
  return (unsigned)(tiles < EXPAND_GRID ? (tiles ? tiles : 1) : EXPAND_GRID);
}

hipError_t ws_expand_mark(Workspace* w, const ExpandArgs& a0, uint64_t n_bound, uint64_t e_bound, int step, int tix) {
  if (step > MAX_STEPS || tix >= MAX_TYPES_Q) return hipErrorInvalidValue;
  HIP_TRY(enqueue_scan(w, a0, n_bound, step, tix));
  ExpandArgs a = a0;
  a.frontier = w->frontier[w->cur];
  FinalParams fp{};
  hipEvent_t p = prof_begin(w);
  hipLaunchKernelGGL(k_expand<MARK>, dim3(expand_grid(n_bound, e_bound)), dim3(BLOCK), 0, w->stream, a, &w->q->n,
                     &w->q->total, w->seg_end, w->block_sum, w->seg_rs, w->flags, fp, BfsParams{});
  prof_end(w, p, K_EXPAND_MARK, step, tix);
  return hipGetLastError();
}

hipError_t ws_compact(Workspace* w, int step) {
  uint64_t nb = w->flag_bytes / FLAG_BYTES;
  uint32_t* next = w->frontier[w->cur ^ 1];
  hipEvent_t p = prof_begin(w);
  hipLaunchKernelGGL(k_flag_count, dim3((unsigned)nb), dim3(BLOCK), 0, w->stream, w->flags, w->flag_bytes,
                     w->flag_blocks);
  prof_end(w, p, K_FLAG_COUNT, step, 0);
  p = prof_begin(w);
  hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(1024), 0, w->stream, w->flag_blocks, &w->q->n, nb, &w->q->n,
                     &w->q->step_n[step + 1]);
  prof_end(w, p, K_SCAN, step, 0);
  p = prof_begin(w);
  hipLaunchKernelGGL(k_flag_write, dim3((unsigned)nb), dim3(BLOCK), 0, w->stream, w->flags, w->flag_bytes, w->nv,
                     w->flag_blocks, next);
  prof_end(w, p, K_FLAG_WRITE, step, 0);
  w->cur ^= 1;
  return hipGetLastError();
}

// distinct 8-byte edge property columns a program reads per edge (WHERE + YIELD)
static int edge_columns_read(const TypeProgram& prog) {
  uint64_t seen = 0;
  int n = 0;
  for (auto& ins : prog.code) {
    if (ins.op != OP_COL && ins.op != OP_COLV) continue;
    const uint64_t bit = 1ull << (ins.aux & 63);
    if (!(seen & bit)) { seen |= bit; ++n; }
  }
  return n;
}

// Recognise the FastProg shapes in the compiled bytecode (see FastProg).
static FastProg detect_fast(const TypeProgram& prog, const ExpandArgs& a) {
  FastProg f{};
  f.enabled = 0;
  f.where_col = -1;
  auto leaf_col = [&](const Ins& i) {
    return i.op == OP_COL || (i.op == OP_COLV && a.valid == nullptr);
  };
  if (prog.where_reg >= 0) {
    if (prog.where_len != 3) return f;
    const Ins &i0 = prog.code[0], &i1 = prog.code[1], &c = prog.code[2];
    static const int kOps[6] = {OP_LT_I, OP_LE_I, OP_GT_I, OP_GE_I, OP_EQ_I, OP_NE_I};
    static const int kSwap[6] = {2, 3, 0, 1, 4, 5};   // const <op> col  ==  col <swap(op)> const
    int op = -1;
    for (int k = 0; k < 6; ++k)
      if (c.op == kOps[k]) op = k;
    if (op < 0 || c.d != prog.where_reg) return f;
    const Ins* colI = nullptr;
    const Ins* constI = nullptr;
    if (leaf_col(i0) && i1.op == OP_CONST) { colI = &i0; constI = &i1; }
    else if (i0.op == OP_CONST && leaf_col(i1)) { colI = &i1; constI = &i0; }
    else return f;
    if (c.a == colI->d && c.b == constI->d) f.where_op = op;
    else if (c.a == constI->d && c.b == colI->d) f.where_op = kSwap[op];
    else return f;
    f.where_col = colI->aux;
    f.where_const = constI->imm;
  }
  const int ny = (int)prog.yield_reg.size();
  int pc = prog.where_len;
  for (int y = 0; y < ny; ++y) {
    if (prog.yield_reg[y] < 0) { f.ykind[y] = 4; continue; }
    if (pc >= (int)prog.code.size()) return f;
    const Ins& i = prog.code[pc++];
    if (i.d != prog.yield_reg[y]) return f;
    if (i.op == OP_DST) f.ykind[y] = 0;
    else if (i.op == OP_SRC) f.ykind[y] = 1;
    else if (i.op == OP_RANK) f.ykind[y] = 2;
    else if (leaf_col(i)) { f.ykind[y] = 3; f.ycol[y] = i.aux; }
    else return f;
  }
  if (pc != (int)prog.code.size()) return f;
  f.enabled = 1;
  return f;
}

uint64_t ws_shard_cap(uint64_t n_bound, uint64_t e_bound) {
  uint64_t tiles = cdiv(n_bound + e_bound + 1, TILE);
  return cdiv(tiles, NSHARD) * TILE;
}

hipError_t ws_expand_final(Workspace* w, const ExpandArgs& a0, uint64_t n_bound, uint64_t e_bound, int step, int tix,
                           const TypeProgram& prog, uint64_t region_base, uint64_t shard_cap) {
  if (step > MAX_STEPS || tix >= MAX_TYPES_Q) return hipErrorInvalidValue;
  HIP_TRY(enqueue_scan(w, a0, n_bound, step, tix));
  ExpandArgs a = a0;
  a.frontier = w->frontier[w->cur];
  FinalParams fp{};
  fp.prog = w->d_prog + (size_t)tix * MAX_PROGRAM;
  fp.where_len = prog.where_len;
  fp.where_reg = prog.where_reg;
  fp.prog_len = (int)prog.code.size();
  fp.nyields = (int)prog.yield_reg.size();
  for (int y = 0; y < fp.nyields; ++y) {
    fp.yield_reg[y] = prog.yield_reg[y];
    fp.yield_const[y] = prog.yield_const[y];
  }
  fp.out_cols = w->d_row_cols;
  fp.region_base = region_base;
  fp.shard_cap = shard_cap;
  fp.shard_rows = &w->q->rows[tix][0];
  fp.err_flag = &w->q->err;
  fp.fast = detect_fast(prog, a);
  size_t lds = fp.fast.enabled ? 0 : (size_t)(prog.nregs > 0 ? prog.nregs : 1) * BLOCK * sizeof(int64_t);
  hipEvent_t p = prof_begin(w);
  hipLaunchKernelGGL(k_expand<FINAL>, dim3(expand_grid(n_bound, e_bound)), dim3(BLOCK), lds, w->stream, a, &w->q->n,
                     &w->q->total, w->seg_end, w->block_sum, w->seg_rs, w->flags, fp, BfsParams{});
  prof_end(w, p, K_EXPAND_FINAL, step, tix, (double)edge_columns_read(prog), (double)fp.nyields);
  return hipGetLastError();
}

// Scan-only expansion (final step whose WHERE folded to false still counts E_N).
hipError_t ws_scan_only(Workspace* w, const ExpandArgs& a, uint64_t n_bound, int step, int tix) {
  return enqueue_scan(w, a, n_bound, step, tix);
}

hipError_t ws_end_query(Workspace* w) {
  HIP_TRY(hipMemcpyAsync(w->h_q, w->q, sizeof(QState), hipMemcpyDeviceToHost, w->stream));
  HIP_TRY(hipStreamSynchronize(w->stream));
  prof_flush(w, w->h_q);
  return hipSuccess;
}

// ----------------------------------------------------------------------------- partitioned mode
hipError_t ws_set_partition(Workspace* w, Comm* comm, uint64_t npad) {
  if (!comm || npad % BITS_BLOCK) return hipErrorInvalidValue;
  const uint64_t G = (uint64_t)comm->world;
  HIP_TRY(hipStreamSynchronize(w->stream));
  w->comm = comm;
  w->npad = npad;
  if (w->flags) HIP_TRY(hipFree(w->flags));
  w->flags = nullptr;
  w->flag_bytes = G * npad;                     // multiple of FLAG_BYTES (npad % BITS_BLOCK == 0)
  HIP_TRY(hipMalloc((void**)&w->flags, w->flag_bytes));
  HIP_TRY(hipMemsetAsync(w->flags, 0, w->flag_bytes, w->stream));
  HIP_TRY(hipMalloc((void**)&w->sendbits, G * npad / 8));
  HIP_TRY(hipMalloc((void**)&w->recvbits, G * npad / 8));
  HIP_TRY(hipMalloc((void**)&w->mbits, npad / 8));
  HIP_TRY(hipMalloc((void**)&w->gst, GST_N * sizeof(unsigned long long)));
  HIP_TRY(hipHostMalloc((void**)&w->h_gst, GST_N * sizeof(unsigned long long), hipHostMallocDefault));
  const uint64_t nb = npad / BITS_BLOCK + 1;
  if (nb > w->cap_blocks) {
    if (w->flag_blocks) HIP_TRY(hipFree(w->flag_blocks));
    w->flag_blocks = nullptr;
    w->cap_blocks = nb;
    HIP_TRY(hipMalloc((void**)&w->flag_blocks, nb * 4));
    HIP_TRY(hipFree(w->block_sum));
    w->block_sum = nullptr;
    HIP_TRY(hipMalloc((void**)&w->block_sum, nb * 4));
  }
  return hipStreamSynchronize(w->stream);
}

// After all OVER types of a non-final step marked their candidates (global ids) in the flags:
// pack -> all-to-all of npad-bit segments -> owner OR + compaction into the next local frontier.
hipError_t ws_exchange(Workspace* w, int step) {
  if (!w->comm) return hipErrorInvalidValue;
  const uint64_t G = (uint64_t)w->comm->world;
  const uint64_t nwords = G * w->npad / 64, seg_words = w->npad / 64, nb = w->npad / BITS_BLOCK;
  hipEvent_t p = prof_begin(w);
  hipLaunchKernelGGL(k_pack_bits, dim3((unsigned)cdiv(nwords, BLOCK)), dim3(BLOCK), 0, w->stream, w->flags, nwords,
                     w->sendbits);
  prof_end(w, p, K_PACK, step, 0, (double)(G * w->npad) + (double)(G * w->npad / 8));
  HIP_TRY(hipGetLastError());
  p = prof_begin(w);
  if (w->comm->alltoall(w->sendbits, w->recvbits, w->npad / 8, w->stream)) return hipErrorUnknown;
  prof_end(w, p, K_ALLTOALL, step, 0, (double)((G - 1) * w->npad / 8));
  p = prof_begin(w);
  hipLaunchKernelGGL(k_bits_count, dim3((unsigned)nb), dim3(BLOCK), 0, w->stream, w->recvbits, (int)G, seg_words,
                     w->nv, w->mbits, w->flag_blocks);
  prof_end(w, p, K_BITS_COUNT, step, 0, (double)(G * w->npad / 8) + (double)(w->npad / 8));
  p = prof_begin(w);
  hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(1024), 0, w->stream, w->flag_blocks, &w->q->n, nb, &w->q->n,
                     &w->q->step_n[step + 1]);
  prof_end(w, p, K_SCAN, step, 0);
  p = prof_begin(w);
  hipLaunchKernelGGL(k_bits_write, dim3((unsigned)nb), dim3(BLOCK), 0, w->stream, w->mbits, w->flag_blocks,
                     w->frontier[w->cur ^ 1]);
  prof_end(w, p, K_BITS_WRITE, step, 0);
  w->cur ^= 1;
  return hipGetLastError();
}

// Global query statistics (err flag, |F_s|, E_s summed over ranks), synchronised with the query
// end; valid in ws_host_gstats() after ws_end_query.
hipError_t ws_global_stats(Workspace* w, int ntypes) {
  if (!w->comm) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_gstats, dim3(1), dim3(64), 0, w->stream, w->q, ntypes, w->gst);
  HIP_TRY(hipGetLastError());
  if (w->comm->allreduce_sum_u64(w->gst, GST_N, w->stream)) return hipErrorUnknown;
  return hipMemcpyAsync(w->h_gst, w->gst, GST_N * sizeof(unsigned long long), hipMemcpyDeviceToHost, w->stream);
}

void ws_host_gstats(Workspace* w, unsigned long long* err, unsigned long long* step_n, unsigned long long* esum) {
  *err = w->h_gst[0];
  for (int s = 0; s < MAX_STEPS + 2; ++s) {
    step_n[s] = w->h_gst[1 + s];
    esum[s] = w->h_gst[1 + (MAX_STEPS + 2) + s];
  }
}


// ============================================================================= FIND SHORTEST PATH
// Bidirectional BFS over epoch-stamped labels (path.cpp drives it level by level):
//   k_expand<BFS>  claims neighbours (CAS on the label), detects meets, appends to claim shards
//   k_gather       packs the NSHARD claim regions into the next frontier list
//   k_degsum       degree sum of a frontier (which side to expand next)
//   k_stamp        label a list (sources, targets, level-0 vertices)
//   k_path_greedy  lexicographically smallest shortest path through the B-sets (one workgroup)

__global__ void __launch_bounds__(BLOCK) k_stamp(const uint32_t* __restrict__ ids,
                                                 const unsigned long long* __restrict__ np,
                                                 uint32_t* __restrict__ lab, uint32_t stamp) {
  const uint64_t n = *np;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (uint64_t)gridDim.x * BLOCK) {
    uint32_t v = ids[i];
    if (v != NO_ROW) lab[v] = stamp;
  }
}

__global__ void __launch_bounds__(BLOCK) k_gather(const uint32_t* __restrict__ scratch, uint64_t shard_cap,
                                                  const unsigned long long* __restrict__ shard_cnt,
                                                  uint32_t* __restrict__ out, unsigned long long* n_out,
                                                  unsigned long long* c_rec) {
  __shared__ unsigned long long pre[NSHARD + 1];
  if (threadIdx.x == 0) {
    unsigned long long run = 0;
    for (int s = 0; s < NSHARD; ++s) {
      pre[s] = run;
      run += shard_cnt[s];
    }
    pre[NSHARD] = run;
    if (blockIdx.x == 0) {
      *n_out = run;
      if (c_rec) *c_rec = run;
    }
  }
  __syncthreads();
  for (int s = 0; s < NSHARD; ++s) {
    const uint64_t cnt = pre[s + 1] - pre[s];
    const uint32_t* src = scratch + (uint64_t)s * shard_cap;
    uint32_t* dst = out + pre[s];
    for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < cnt; i += (uint64_t)gridDim.x * BLOCK)
      dst[i] = src[i];
  }
}

struct DegsumArgs {
  int ntypes;
  const uint32_t* row_ptr[MAX_TYPES_Q];
  const uint8_t* visible;
  uint32_t cap;
};

__global__ void __launch_bounds__(BLOCK) k_degsum(const uint32_t* __restrict__ f,
                                                  const unsigned long long* __restrict__ np, DegsumArgs d,
                                                  unsigned long long* out, unsigned long long* n_rec) {
  __shared__ unsigned long long lds[WAVES];
  const uint64_t n = *np;
  if (n_rec && blockIdx.x == 0 && threadIdx.x == 0) *n_rec = n;
  unsigned long long sum = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (uint64_t)gridDim.x * BLOCK) {
    uint32_t v = f[i];
    if (v == NO_ROW || (d.visible && !d.visible[v])) continue;
    for (int t = 0; t < d.ntypes; ++t) {
      uint32_t deg = d.row_ptr[t][v + 1] - d.row_ptr[t][v];
      sum += deg < d.cap ? deg : d.cap;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_down(sum, o, 64);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) lds[w] = sum;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int i = 0; i < WAVES; ++i) t += lds[i];
    if (t) atomicAdd(out, t);
  }
}

struct GreedyArgs {
  int ntypes;
  int32_t type[MAX_TYPES_Q];
  const uint32_t* row_ptr[MAX_TYPES_Q];
  const uint32_t* col[MAX_TYPES_Q];
  const int64_t* dst_vid[MAX_TYPES_Q];
  const int64_t* rank[MAX_TYPES_Q];
  const uint8_t* visible;
  const int64_t* vids;
  uint32_t cap;
  int L, kf;
  const uint32_t* lab_m;
  uint32_t em;
  const uint32_t* lab_b;
  uint32_t eb;
  const uint32_t* starts;
  const unsigned long long* nstarts;
  int64_t* out;                 // [v0, t0, r0, v1, ...]
  unsigned long long* err;
};

struct Cand {                   // (type, rank, vid) key + dense id of the vertex
  int64_t t, r, v;
  uint32_t d;
};
__device__ __forceinline__ bool cand_less(const Cand& x, const Cand& y) {
  if (x.t != y.t) return x.t < y.t;
  if (x.r != y.r) return x.r < y.r;
  return x.v < y.v;
}
__device__ __forceinline__ Cand shfl_cand(const Cand& c, int o) {
  Cand r;
  r.t = __shfl_down(c.t, o, 64);
  r.r = __shfl_down(c.r, o, 64);
  r.v = __shfl_down(c.v, o, 64);
  r.d = __shfl_down(c.d, o, 64);
  return r;
}
constexpr int GREEDY_BLOCK = 1024;

// Block-wide minimum; every thread gets the result.  INT64_MAX type marks "no candidate".
__device__ Cand block_min(Cand c, Cand* lds) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    Cand x = shfl_cand(c, o);
    if (cand_less(x, c)) c = x;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) lds[w] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    Cand b = lds[0];
    for (int i = 1; i < GREEDY_BLOCK / 64; ++i)
      if (cand_less(lds[i], b)) b = lds[i];
    lds[GREEDY_BLOCK / 64] = b;
  }
  __syncthreads();
  Cand r = lds[GREEDY_BLOCK / 64];
  __syncthreads();
  return r;
}

// Position pos (1..L) of a shortest path is valid for w when w is in B[pos]: positions <= kf
// carry a LAB_M stamp (the backward B-set passes over the forward levels), positions > kf the
// backward BFS level L - pos.
__device__ __forceinline__ bool greedy_valid(const GreedyArgs& g, uint32_t w, int pos) {
  if (w == NO_ROW) return false;
  if (pos <= g.kf) return g.lab_m[w] == ((g.em << LVL_BITS) | (uint32_t)pos);
  return g.lab_b[w] == ((g.eb << LVL_BITS) | (uint32_t)(g.L - pos));
}

__global__ void __launch_bounds__(GREEDY_BLOCK) k_path_greedy(GreedyArgs g) {
  __shared__ Cand lds[GREEDY_BLOCK / 64 + 1];
  const Cand none{INT64_MAX, INT64_MAX, INT64_MAX, NO_ROW};
  // v0 = smallest vid among the start candidates (dense ids are in vid order)
  Cand c = none;
  const uint64_t ns = *g.nstarts;
  for (uint64_t i = threadIdx.x; i < ns; i += GREEDY_BLOCK) {
    uint32_t d = g.starts[i];
    if (d != NO_ROW && (int64_t)d < c.t) c = Cand{(int64_t)d, 0, 0, d};
  }
  c = block_min(c, lds);
  uint32_t v = c.d;
  if (v == NO_ROW) {
    if (threadIdx.x == 0) *g.err = 1;
    return;
  }
  if (threadIdx.x == 0) g.out[0] = g.vids[v];
  for (int pos = 0; pos < g.L; ++pos) {
    Cand best = none;
    if (!g.visible || g.visible[v]) {
      for (int t = 0; t < g.ntypes; ++t) {
        const uint32_t rs = g.row_ptr[t][v];
        uint32_t deg = g.row_ptr[t][v + 1] - rs;
        deg = deg < g.cap ? deg : g.cap;
        for (uint32_t k = threadIdx.x; k < deg; k += GREEDY_BLOCK) {
          const uint64_t j = (uint64_t)rs + k;
          const uint32_t w = g.col[t][j];
          if (!greedy_valid(g, w, pos + 1)) continue;
          Cand x{(int64_t)g.type[t], g.rank[t] ? g.rank[t][j] : 0, g.dst_vid[t][j], w};
          if (cand_less(x, best)) best = x;
        }
      }
    }
    best = block_min(best, lds);
    if (best.d == NO_ROW) {
      if (threadIdx.x == 0) *g.err = 1;
      return;
    }
    if (threadIdx.x == 0) {
      g.out[1 + 3 * pos] = best.t;
      g.out[2 + 3 * pos] = best.r;
      g.out[3 + 3 * pos] = best.v;
    }
    v = best.d;
  }
}

// ----------------------------------------------------------------------------- path host side
constexpr uint64_t STAGE = 4096;
static hipEvent_t prof_begin_p(Workspace* w) { return prof_begin(w); }
static void prof_end_p(Workspace* w, hipEvent_t a, int kid, int rec) {
  if (!a) return;
  hipEvent_t b = w->prof.get();
  (void)hipEventRecord(b, w->stream);
  w->prof.pending.push_back({kid, rec, 0, a, b, 0, 0, true});
}

hipError_t ws_path_begin(Workspace* w, uint64_t scratch_entries, uint64_t list_entries) {
  if (!w->ps) {
    HIP_TRY(hipMalloc((void**)&w->ps, sizeof(PState)));
    HIP_TRY(hipHostMalloc((void**)&w->h_ps, sizeof(PState), hipHostMallocDefault));
    HIP_TRY(hipMalloc((void**)&w->d_path, (1 + 3 * MAX_PATH_LEN) * sizeof(int64_t)));
    HIP_TRY(hipHostMalloc((void**)&w->h_path, (1 + 3 * MAX_PATH_LEN) * sizeof(int64_t), hipHostMallocDefault));
    HIP_TRY(hipHostMalloc((void**)&w->h_stage, (size_t)PSLOTS * STAGE * sizeof(uint32_t), hipHostMallocDefault));
    for (int l = 0; l < NUM_LABS; ++l) {
      HIP_TRY(hipMalloc((void**)&w->lab[l], (w->nv + 1) * sizeof(uint32_t)));
      HIP_TRY(hipMemsetAsync(w->lab[l], 0, (w->nv + 1) * sizeof(uint32_t), w->stream));
      w->epoch[l] = 0;
    }
  }
  if (list_entries > w->slot_cap) {
    HIP_TRY(hipStreamSynchronize(w->stream));
    for (auto*& p : w->slot) {
      if (p) HIP_TRY(hipFree(p));
      p = nullptr;
    }
    w->slot_cap = list_entries;
    for (auto*& p : w->slot) HIP_TRY(hipMalloc((void**)&p, w->slot_cap * sizeof(uint32_t)));
  }
  if (scratch_entries > w->pscratch_cap) {
    HIP_TRY(hipStreamSynchronize(w->stream));
    if (w->pscratch) HIP_TRY(hipFree(w->pscratch));
    w->pscratch = nullptr;
    w->pscratch_cap = scratch_entries;
    HIP_TRY(hipMalloc((void**)&w->pscratch, w->pscratch_cap * sizeof(uint32_t)));
  }
  w->rec = 0;
  return hipMemsetAsync(w->ps, 0, sizeof(PState), w->stream);
}

uint32_t ws_path_epoch(Workspace* w, int l) {
  if (++w->epoch[l] >= (1u << (32 - LVL_BITS))) {   // wrap: clear the labels once
    (void)hipMemsetAsync(w->lab[l], 0, (w->nv + 1) * sizeof(uint32_t), w->stream);
    w->epoch[l] = 1;
  }
  return w->epoch[l];
}

uint32_t* ws_path_slot(Workspace* w, int s) { return w->slot[s]; }

hipError_t ws_path_upload(Workspace* w, int s, const uint32_t* ids, uint64_t n) {
  if (n > w->slot_cap) return hipErrorInvalidValue;
  if (n <= STAGE) {   // common case: no synchronisation
    uint32_t* st = w->h_stage + (size_t)s * STAGE;
    memcpy(st, ids, n * 4);
    w->h_ps->n[s] = n;
    if (n) HIP_TRY(hipMemcpyAsync(w->slot[s], st, n * 4, hipMemcpyHostToDevice, w->stream));
    return hipMemcpyAsync(&w->ps->n[s], &w->h_ps->n[s], sizeof(unsigned long long), hipMemcpyHostToDevice,
                          w->stream);
  }
  if (n > w->cap_starts) {
    HIP_TRY(hipStreamSynchronize(w->stream));
    if (w->h_starts) HIP_TRY(hipHostFree(w->h_starts));
    w->cap_starts = n + n / 2 + 1024;
    HIP_TRY(hipHostMalloc((void**)&w->h_starts, w->cap_starts * 4, hipHostMallocDefault));
  }
  // the staging buffer may still feed an earlier copy of this query
  HIP_TRY(hipStreamSynchronize(w->stream));
  memcpy(w->h_starts, ids, n * 4);
  w->h_ps->n[s] = n;
  HIP_TRY(hipMemcpyAsync(w->slot[s], w->h_starts, n * 4, hipMemcpyHostToDevice, w->stream));
  return hipMemcpyAsync(&w->ps->n[s], &w->h_ps->n[s], sizeof(unsigned long long), hipMemcpyHostToDevice,
                        w->stream);
}

hipError_t ws_path_stamp(Workspace* w, int s, uint64_t n_bound, int l, uint32_t stamp) {
  unsigned nb = (unsigned)cdiv(n_bound ? n_bound : 1, BLOCK);
  if (nb > 1024) nb = 1024;
  hipEvent_t p = prof_begin_p(w);
  hipLaunchKernelGGL(k_stamp, dim3(nb), dim3(BLOCK), 0, w->stream, w->slot[s], &w->ps->n[s], w->lab[l], stamp);
  prof_end_p(w, p, K_STAMP, 0);
  return hipGetLastError();
}

hipError_t ws_path_degsum(Workspace* w, int s, uint64_t n_bound, const PathTypes& pt, int side) {
  DegsumArgs d{};
  d.ntypes = pt.n;
  for (int t = 0; t < pt.n; ++t) d.row_ptr[t] = pt.a[t].row_ptr;
  d.visible = pt.n ? pt.a[0].visible : nullptr;
  d.cap = pt.n ? pt.a[0].cap : 0xFFFFFFFFu;
  unsigned nb = (unsigned)cdiv(n_bound ? n_bound : 1, BLOCK);
  if (nb > 2048) nb = 2048;
  const int rec = w->rec < PATH_REC ? w->rec++ : PATH_REC - 1;
  HIP_TRY(hipMemsetAsync(&w->ps->dsum[side], 0, sizeof(unsigned long long), w->stream));
  hipEvent_t p = prof_begin_p(w);
  hipLaunchKernelGGL(k_degsum, dim3(nb), dim3(BLOCK), 0, w->stream, w->slot[s], &w->ps->n[s], d,
                     &w->ps->dsum[side], &w->ps->ln[rec]);
  prof_end_p(w, p, K_DEGSUM, rec);
  return hipGetLastError();
}

hipError_t ws_path_level(Workspace* w, const PathTypes& pt, int src, uint64_t n_bound, uint64_t e_bound, int dst,
                         const PathLevel& lv) {
  // claim shards: a shard's count is bounded by its tiles over all types of this level
  uint64_t shard_cap = 0;
  for (int t = 0; t < pt.n; ++t) shard_cap += ws_shard_cap(n_bound, e_bound);
  if (shard_cap * NSHARD > w->pscratch_cap) {
    HIP_TRY(hipStreamSynchronize(w->stream));
    if (w->pscratch) HIP_TRY(hipFree(w->pscratch));
    w->pscratch = nullptr;
    w->pscratch_cap = shard_cap * NSHARD;
    HIP_TRY(hipMalloc((void**)&w->pscratch, w->pscratch_cap * sizeof(uint32_t)));
  }
  BfsParams bp{};
  bp.lab = w->lab[lv.lab];
  bp.stamp = lv.stamp;
  bp.epoch = lv.stamp >> LVL_BITS;
  if (lv.rlab >= 0) { bp.rlab = w->lab[lv.rlab]; bp.rstamp = lv.rstamp; }
  if (lv.mlab >= 0) {
    bp.mlab = w->lab[lv.mlab];
    bp.mepoch = lv.mepoch;
    bp.mout = w->lab[LAB_M];
    bp.mstamp = lv.mstamp;
    bp.meet_list = w->slot[lv.meet_slot];
    bp.meet_n = &w->ps->n[lv.meet_slot];
  }
  if (lv.tlab >= 0) { bp.tlab = w->lab[lv.tlab]; bp.tstamp = lv.tstamp; bp.found = &w->ps->found; }
  bp.out = w->pscratch;
  bp.shard_cap = shard_cap;
  bp.shard_cnt = w->ps->shard;
  const int rec = w->rec < PATH_REC ? w->rec++ : PATH_REC - 1;
  for (int t = 0; t < pt.n; ++t) {
    ExpandArgs a = pt.a[t];
    a.frontier = w->slot[src];
    uint64_t nb = cdiv(n_bound ? n_bound : 1, SCAN_TILE);
    hipEvent_t p = prof_begin_p(w);
    hipLaunchKernelGGL(k_degree, dim3((unsigned)nb), dim3(BLOCK), 0, w->stream, w->slot[src], &w->ps->n[src],
                       a.row_ptr, a.visible, a.cap, w->seg_end, w->seg_rs, w->block_sum,
                       t == 0 ? w->ps->shard : (unsigned long long*)nullptr, &w->ps->ln[rec]);
    prof_end_p(w, p, K_DEGREE, rec);
    p = prof_begin_p(w);
    hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(1024), 0, w->stream, w->block_sum, &w->ps->n[src], (uint64_t)0,
                       &w->ps->total, &w->ps->le[rec]);
    prof_end_p(w, p, K_SCAN, rec);
    p = prof_begin_p(w);
    hipLaunchKernelGGL(k_expand<BFS>, dim3(expand_grid(n_bound, e_bound)), dim3(BLOCK), 0, w->stream, a,
                       &w->ps->n[src], &w->ps->total, w->seg_end, w->block_sum, w->seg_rs, (uint8_t*)nullptr,
                       FinalParams{}, bp);
    prof_end_p(w, p, K_BFS, rec);
  }
  uint64_t gb = cdiv(n_bound + e_bound + 1, (uint64_t)BLOCK * 4);
  unsigned grid = (unsigned)(gb < 1 ? 1 : (gb > 1024 ? 1024 : gb));
  hipEvent_t p = prof_begin_p(w);
  hipLaunchKernelGGL(k_gather, dim3(grid), dim3(BLOCK), 0, w->stream, w->pscratch, shard_cap, w->ps->shard,
                     w->slot[dst], &w->ps->n[dst], &w->ps->lc[rec]);
  prof_end_p(w, p, K_GATHER, rec);
  return hipGetLastError();
}

int ws_path_last_rec(Workspace* w) { return w->rec - 1; }

hipError_t ws_path_read_label(Workspace* w, int l, uint32_t v, uint32_t* out) {
  HIP_TRY(hipMemcpyAsync(w->h_stage, w->lab[l] + v, sizeof(uint32_t), hipMemcpyDeviceToHost, w->stream));
  HIP_TRY(hipStreamSynchronize(w->stream));
  *out = w->h_stage[0];
  return hipSuccess;
}

hipError_t ws_path_greedy(Workspace* w, const PathTypes& pt, const PathGreedy& pg) {
  if (pg.L < 1 || pg.L > (int)MAX_PATH_LEN) return hipErrorInvalidValue;
  GreedyArgs g{};
  g.ntypes = pt.n;
  for (int t = 0; t < pt.n; ++t) {
    g.type[t] = pt.type[t];
    g.row_ptr[t] = pt.a[t].row_ptr;
    g.col[t] = pt.a[t].col;
    g.dst_vid[t] = pt.a[t].dst_vid;
    g.rank[t] = pt.a[t].rank;
  }
  g.visible = pt.n ? pt.a[0].visible : nullptr;
  g.vids = pt.n ? pt.a[0].vids : nullptr;
  g.cap = pt.n ? pt.a[0].cap : 0xFFFFFFFFu;
  g.L = pg.L;
  g.kf = pg.kf;
  g.lab_m = w->lab[LAB_M];
  g.em = pg.em;
  g.lab_b = w->lab[LAB_B];
  g.eb = pg.eb;
  g.starts = w->slot[pg.start_slot];
  g.nstarts = &w->ps->n[pg.start_slot];
  g.out = w->d_path;
  g.err = &w->ps->err;
  hipEvent_t p = prof_begin_p(w);
  hipLaunchKernelGGL(k_path_greedy, dim3(1), dim3(GREEDY_BLOCK), 0, w->stream, g);
  prof_end_p(w, p, K_GREEDY, 0);
  return hipGetLastError();
}

hipError_t ws_path_sync(Workspace* w, PState* out, int64_t* path, int path_len) {
  HIP_TRY(hipMemcpyAsync(w->h_ps, w->ps, sizeof(PState), hipMemcpyDeviceToHost, w->stream));
  if (path && path_len > 0)
    HIP_TRY(hipMemcpyAsync(w->h_path, w->d_path, (size_t)path_len * sizeof(int64_t), hipMemcpyDeviceToHost,
                           w->stream));
  HIP_TRY(hipStreamSynchronize(w->stream));
  if (out) *out = *w->h_ps;
  if (path && path_len > 0) memcpy(path, w->h_path, (size_t)path_len * sizeof(int64_t));
  // resolve timing of the launches since the last sync (record indices stay valid per query)
  prof_flush(w, nullptr, w->h_ps);
  return hipSuccess;
}

}  // namespace nbg
