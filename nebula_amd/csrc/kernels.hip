// nebula_amd — gfx950 (CDNA4) kernels for the GO N STEPS / FIND PATH hot path.
//
// Per hop over one edge type (CSR):
//   k_degree      frontier degrees (row_ptr gathers, capped by max_edge_returned_per_vertex)
//                 + block-local inclusive scan                       (wave64 shuffles + LDS)
//   k_scan_blocks exclusive scan of the per-block totals (one workgroup)
//   k_partition   merge-path split of (frontier segments ⊕ edges) into equal tiles
//   k_expand<M>   load-balanced expansion: each tile owns TILE path items whatever the degree
//                 skew; items are processed striped across the block so neighbour reads are
//                 coalesced.  M = MARK (intermediate steps: set next-frontier byte flags) or
//                 FINAL (evaluate the WHERE/YIELD bytecode per edge, wave-ballot compaction of
//                 the emitted rows, one atomic per block-iteration).
//   k_flag_count / k_flag_write  dense compaction of the byte flags into the next (sorted)
//                 frontier, clearing the flags in the same pass.
// Semantics follow QueryBaseProcessor::collectEdgeProps (version de-dup is done at load,
// neighbours are in memcmp key order, the cap counts edges in that order) and
// GoExecutor::getDstIdsFromResp (per-step dst SET, no global visited set).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

#include "nbg_internal.h"

namespace nbg {

constexpr int BLOCK = 256;
constexpr int WAVES = BLOCK / 64;
constexpr int SCAN_ITEMS = 8;                    // k_degree: items per thread
constexpr int SCAN_TILE = BLOCK * SCAN_ITEMS;    // 2048 frontier entries per block
constexpr int SCAN_SHIFT = 11;
constexpr int VT = 4;                            // k_expand: path items per thread
constexpr int TILE = BLOCK * VT;                 // 1024 path items per tile
constexpr int FLAG_BYTES = BLOCK * 16;           // k_flag_*: bytes per block

enum KernelId { K_DEGREE = 0, K_SCAN, K_PARTITION, K_EXPAND_MARK, K_FLAG_COUNT, K_FLAG_WRITE, K_EXPAND_FINAL,
                K_BFS, K_COUNT };
static const char* const kKernelNames[K_COUNT] = {"k_degree", "k_scan_blocks", "k_partition", "k_expand<MARK>",
                                                  "k_flag_count", "k_flag_write", "k_expand<FINAL>", "k_expand<BFS>"};

struct Prof {
  bool on = false;
  struct Rec { int kid; hipEvent_t a, b; double bytes; };
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
  uint32_t* seg_end = nullptr;    // block-local inclusive scan of degrees
  uint32_t* seg_rs = nullptr;     // row start per frontier entry
  uint32_t* block_sum = nullptr;  // per-block totals -> exclusive prefix (in place)
  uint64_t cap_blocks = 0;
  uint32_t* part = nullptr;       // merge-path tile splits
  uint64_t cap_tiles = 0;
  uint8_t* flags = nullptr;       // [nv rounded up to FLAG_BYTES], kept all-zero between steps
  uint64_t flag_bytes = 0;
  uint32_t* flag_blocks = nullptr;
  uint64_t* counters = nullptr;   // [0] total, [1] row counter, [2] error, [3] scratch
  uint64_t* h_pinned = nullptr;   // pinned readback
  int64_t* rows = nullptr;        // [ncols][cap_rows]
  uint64_t cap_rows = 0;
  int ncols_alloc = 0;
  int64_t** d_row_cols = nullptr; // device array of column pointers
  Ins* d_prog = nullptr;
};

#define HIP_TRY(x)                         \
  do {                                     \
    hipError_t e_ = (x);                   \
    if (e_ != hipSuccess) return e_;       \
  } while (0)

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
__global__ void __launch_bounds__(BLOCK) k_degree(const uint32_t* __restrict__ frontier, uint64_t n,
                                                  const uint32_t* __restrict__ row_ptr,
                                                  const uint8_t* __restrict__ visible, uint32_t cap,
                                                  uint32_t* __restrict__ seg_end, uint32_t* __restrict__ seg_rs,
                                                  uint32_t* __restrict__ block_sum) {
  __shared__ uint32_t lds[WAVES];
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

// One workgroup: exclusive scan of nb uint32 in place; out[0] = grand total (uint64).
__global__ void __launch_bounds__(1024) k_scan_blocks(uint32_t* __restrict__ v, uint64_t nb,
                                                      uint64_t* __restrict__ out) {
  __shared__ uint64_t lds[16];
  __shared__ uint64_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint64_t base = 0; base < nb; base += 1024) {
    uint64_t i = base + threadIdx.x;
    uint64_t x = i < nb ? v[i] : 0;
    // wave inclusive scan (64-bit)
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
  if (threadIdx.x == 0) out[0] = carry;
}

__device__ __forceinline__ uint32_t seg_end_at(const uint32_t* __restrict__ seg_end,
                                               const uint32_t* __restrict__ block_pre, uint64_t i) {
  return seg_end[i] + block_pre[i >> SCAN_SHIFT];
}

// ----------------------------------------------------------------------------- k_partition
__global__ void k_partition(const uint32_t* __restrict__ seg_end, const uint32_t* __restrict__ block_pre,
                            uint64_t n, uint64_t total, uint64_t ntiles, uint32_t* __restrict__ part) {
  uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t > ntiles) return;
  uint64_t d = t * TILE;
  if (d > n + total) d = n + total;
  uint64_t lo = d > total ? d - total : 0;
  uint64_t hi = d < n ? d : n;
  while (lo < hi) {
    uint64_t mid = (lo + hi) >> 1;
    if ((uint64_t)seg_end_at(seg_end, block_pre, mid) <= d - 1 - mid) lo = mid + 1;
    else hi = mid;
  }
  part[t] = (uint32_t)lo;
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
enum Mode { MARK = 0, FINAL = 1 };

struct FinalParams {
  const Ins* prog;
  int where_len;
  int where_reg;          // -1 none
  int prog_len;           // WHERE + YIELD instructions
  int nyields;
  int yield_reg[MAX_YIELDS];
  int64_t yield_const[MAX_YIELDS];
  int64_t** out_cols;
  uint64_t row_base;
  uint64_t* row_counter;
  uint64_t* err_flag;
};

template <int M>
__global__ void __launch_bounds__(BLOCK) k_expand(ExpandArgs a, const uint32_t* __restrict__ seg_end,
                                                  const uint32_t* __restrict__ block_pre,
                                                  const uint32_t* __restrict__ seg_rs,
                                                  const uint32_t* __restrict__ part, uint64_t total,
                                                  uint8_t* __restrict__ flags, FinalParams fp) {
  __shared__ uint32_t sEnd[TILE + 2];   // seg_end for i in [a0-1, a1]
  __shared__ uint32_t sRs[TILE + 1];    // seg_rs for i in [a0, a1]
  __shared__ uint32_t sSeg[TILE];       // segment of each edge item in this tile
  __shared__ uint32_t sWave[WAVES];
  __shared__ uint64_t sBase;
  extern __shared__ int64_t regs[];     // FINAL: [MAX_REGS][BLOCK]

  const uint64_t t = blockIdx.x;
  const uint64_t n = a.n;
  const uint64_t d0 = t * TILE;
  const uint64_t d1 = (d0 + TILE < n + total) ? d0 + TILE : n + total;
  const uint64_t a0 = part[t], a1 = part[t + 1];
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
  } else {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    bool anyErr = false;
    for (int k0 = 0; k0 < nb; k0 += BLOCK) {
      int k = k0 + threadIdx.x;
      bool active = k < nb;
      EdgeCtx c{0, 0};
      if (active) {
        uint32_t s = sSeg[k];
        uint64_t e = b0 + k;
        c.j = (uint64_t)sRs[s] + (e - (uint64_t)sEnd[s]);
        c.v = a.frontier[a0 + s];
      }
      bool werr = false, pass = active;
      if (fp.where_reg >= 0) {
        run_program(fp.prog, 0, fp.where_len, c, a, regs, active, werr);
        pass = active && !werr && regs[fp.where_reg * BLOCK + threadIdx.x] != 0;
      }
      bool yerr = false;
      // the YIELD programs follow the WHERE part; they run for passing lanes only
      run_program(fp.prog, fp.where_len, fp.prog_len, c, a, regs, pass, yerr);
      if (active && (werr || (pass && yerr))) anyErr = true;

      unsigned long long bal = __ballot(pass);
      uint32_t wcount = __popcll(bal);
      uint32_t lpre = __popcll(bal & ((1ull << lane) - 1ull));
      if (lane == 0) sWave[w] = wcount;
      __syncthreads();
      uint32_t wpre = 0, btot = 0;
#pragma unroll
      for (int i = 0; i < WAVES; ++i) {
        wpre += (i < w) ? sWave[i] : 0u;
        btot += sWave[i];
      }
      if (threadIdx.x == 0 && btot) sBase = atomicAdd((unsigned long long*)fp.row_counter, (unsigned long long)btot);
      __syncthreads();
      if (pass) {
        uint64_t row = fp.row_base + sBase + wpre + lpre;
        for (int y = 0; y < fp.nyields; ++y) {
          int r = fp.yield_reg[y];
          fp.out_cols[y][row] = r >= 0 ? regs[r * BLOCK + threadIdx.x] : fp.yield_const[y];
        }
      }
      __syncthreads();
    }
    if (anyErr) atomicOr((unsigned long long*)fp.err_flag, 1ull);
  }
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

// ============================================================================= host wrappers
static inline uint64_t cdiv(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

// Kernel timing: an event pair around each launch on the workspace stream, resolved at the
// next host synchronisation point.
static hipEvent_t prof_begin(Workspace* w) {
  if (!w->prof.on) return nullptr;
  hipEvent_t a = w->prof.get();
  (void)hipEventRecord(a, w->stream);
  return a;
}
static void prof_end(Workspace* w, hipEvent_t a, int kid, double bytes) {
  if (!a) return;
  hipEvent_t b = w->prof.get();
  (void)hipEventRecord(b, w->stream);
  w->prof.pending.push_back({kid, a, b, bytes});
}
static void prof_flush(Workspace* w) {
  for (auto& r : w->prof.pending) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
      w->prof.launches[r.kid]++;
      w->prof.ms[r.kid] += ms;
      w->prof.bytes[r.kid] += r.bytes;
    }
    w->prof.pool.push_back(r.a);
    w->prof.pool.push_back(r.b);
  }
  w->prof.pending.clear();
}

void ws_profile(Workspace* w, bool on) {
  if (!w) return;
  prof_flush(w);
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
  M((void**)&w->counters, 8 * sizeof(uint64_t));
  M((void**)&w->d_prog, MAX_PROGRAM * sizeof(Ins));
  M((void**)&w->d_row_cols, MAX_YIELDS * sizeof(int64_t*));
  if (e == hipSuccess) e = hipHostMalloc((void**)&w->h_pinned, 64, hipHostMallocDefault);
  if (e == hipSuccess) e = hipMemsetAsync(w->flags, 0, w->flag_bytes, s);
  if (e == hipSuccess) e = hipMemsetAsync(w->counters, 0, 8 * sizeof(uint64_t), s);
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
                  (void*)w->block_sum, (void*)w->part, (void*)w->flags, (void*)w->flag_blocks,
                  (void*)w->counters, (void*)w->rows, (void*)w->d_row_cols, (void*)w->d_prog})
    if (p) (void)hipFree(p);
  if (w->h_pinned) (void)hipHostFree(w->h_pinned);
  delete w;
}

uint32_t* ws_frontier(Workspace* w, int which) { return w->frontier[which]; }
int64_t** ws_row_cols(Workspace* w) { return w->d_row_cols; }
int64_t* ws_row_col(Workspace* w, int c) { return w->rows + (uint64_t)c * w->cap_rows; }
Ins* ws_program(Workspace* w) { return w->d_prog; }

hipError_t ws_reserve_rows(Workspace* w, uint64_t rows, int ncols) {
  if (rows <= w->cap_rows && ncols <= w->ncols_alloc) return hipSuccess;
  if (w->rows) HIP_TRY(hipFree(w->rows));
  w->rows = nullptr;
  uint64_t cap = rows < 1024 ? 1024 : rows + rows / 8;
  int nc = ncols < 1 ? 1 : ncols;
  HIP_TRY(hipMalloc((void**)&w->rows, cap * nc * sizeof(int64_t)));
  w->cap_rows = cap;
  w->ncols_alloc = nc;
  int64_t* cols[MAX_YIELDS];
  for (int c = 0; c < MAX_YIELDS; ++c) cols[c] = w->rows + (uint64_t)(c < nc ? c : 0) * cap;
  HIP_TRY(hipMemcpyAsync(w->d_row_cols, cols, sizeof(cols), hipMemcpyHostToDevice, w->stream));
  return hipStreamSynchronize(w->stream);
}

static hipError_t ensure_tiles(Workspace* w, uint64_t ntiles) {
  if (ntiles + 2 <= w->cap_tiles) return hipSuccess;
  if (w->part) HIP_TRY(hipFree(w->part));
  w->cap_tiles = ntiles + 2 + ntiles / 4;
  return hipMalloc((void**)&w->part, w->cap_tiles * sizeof(uint32_t));
}

hipError_t k_degree_scan(Workspace* w, const ExpandArgs& a, uint64_t* total) {
  if (a.n == 0) { *total = 0; return hipSuccess; }
  if (a.n > w->cap_frontier) return hipErrorInvalidValue;
  uint64_t nb = cdiv(a.n, SCAN_TILE);
  hipEvent_t p = prof_begin(w);
  hipLaunchKernelGGL(k_degree, dim3((unsigned)nb), dim3(BLOCK), 0, w->stream, a.frontier, a.n, a.row_ptr,
                     a.visible, a.cap, w->seg_end, w->seg_rs, w->block_sum);
  prof_end(w, p, K_DEGREE, 12.0 * (double)a.n);   // 4|F| ids + 8|F| row_ptr pairs
  p = prof_begin(w);
  hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(1024), 0, w->stream, w->block_sum, nb, w->counters);
  prof_end(w, p, K_SCAN, 0.0);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(w->h_pinned, w->counters, 8, hipMemcpyDeviceToHost, w->stream));
  HIP_TRY(hipStreamSynchronize(w->stream));
  prof_flush(w);
  *total = w->h_pinned[0];
  return hipSuccess;
}

static hipError_t launch_partition(Workspace* w, const ExpandArgs& a, uint64_t total, uint64_t* ntiles_out) {
  uint64_t ntiles = cdiv(a.n + total, TILE);
  HIP_TRY(ensure_tiles(w, ntiles));
  hipEvent_t p = prof_begin(w);
  hipLaunchKernelGGL(k_partition, dim3((unsigned)cdiv(ntiles + 1, 256)), dim3(256), 0, w->stream, w->seg_end,
                     w->block_sum, a.n, total, ntiles, w->part);
  prof_end(w, p, K_PARTITION, 0.0);
  *ntiles_out = ntiles;
  return hipGetLastError();
}

hipError_t k_expand_mark(Workspace* w, const ExpandArgs& a, uint64_t total) {
  if (total == 0) return hipSuccess;
  uint64_t ntiles;
  HIP_TRY(launch_partition(w, a, total, &ntiles));
  FinalParams fp{};
  hipEvent_t p = prof_begin(w);
  hipLaunchKernelGGL(k_expand<MARK>, dim3((unsigned)ntiles), dim3(BLOCK), 0, w->stream, a, w->seg_end,
                     w->block_sum, w->seg_rs, w->part, total, w->flags, fp);
  prof_end(w, p, K_EXPAND_MARK, 4.0 * (double)total);   // 4 E_s neighbour ids
  return hipGetLastError();
}

hipError_t k_compact(Workspace* w, uint64_t nv, uint32_t* next, uint64_t* count) {
  uint64_t nb = w->flag_bytes / FLAG_BYTES;
  hipEvent_t p = prof_begin(w);
  hipLaunchKernelGGL(k_flag_count, dim3((unsigned)nb), dim3(BLOCK), 0, w->stream, w->flags, w->flag_bytes,
                     w->flag_blocks);
  prof_end(w, p, K_FLAG_COUNT, 0.0);
  p = prof_begin(w);
  hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(1024), 0, w->stream, w->flag_blocks, nb, w->counters);
  prof_end(w, p, K_SCAN, 0.0);
  p = prof_begin(w);
  hipLaunchKernelGGL(k_flag_write, dim3((unsigned)nb), dim3(BLOCK), 0, w->stream, w->flags, w->flag_bytes, nv,
                     w->flag_blocks, next);
  prof_end(w, p, K_FLAG_WRITE, 0.0);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(w->h_pinned, w->counters, 8, hipMemcpyDeviceToHost, w->stream));
  HIP_TRY(hipStreamSynchronize(w->stream));
  *count = w->h_pinned[0];
  if (!w->prof.pending.empty()) w->prof.pending.back().bytes = 4.0 * (double)*count;   // write F_{s+1}
  prof_flush(w);
  return hipSuccess;
}

// distinct 8-byte edge columns a program reads per edge (props, _dst, _rank)
static int edge_columns_read(const TypeProgram& prog) {
  uint64_t seen = 0;
  int n = 0;
  for (auto& ins : prog.code) {
    int key = -1;
    if (ins.op == OP_COL || ins.op == OP_COLV) key = 2 + (ins.aux & 31);
    else if (ins.op == OP_DST) key = 0;
    else if (ins.op == OP_RANK) key = 1;
    if (key >= 0 && !(seen & (1ull << key))) { seen |= 1ull << key; ++n; }
  }
  return n;
}

hipError_t k_expand_final(Workspace* w, const ExpandArgs& a, uint64_t total, const TypeProgram& prog,
                          const Ins* d_prog, int64_t** d_out_cols, uint64_t row_base, uint64_t* rows_out,
                          int* err_out) {
  *rows_out = 0;
  *err_out = 0;
  if (total == 0) return hipSuccess;
  uint64_t ntiles;
  HIP_TRY(launch_partition(w, a, total, &ntiles));
  FinalParams fp{};
  fp.prog = d_prog;
  fp.where_len = prog.where_len;
  fp.where_reg = prog.where_reg;
  fp.prog_len = (int)prog.code.size();
  fp.nyields = (int)prog.yield_reg.size();
  int kout = 0;
  for (int y = 0; y < fp.nyields; ++y) {
    fp.yield_reg[y] = prog.yield_reg[y];
    fp.yield_const[y] = prog.yield_const[y];
    kout += 1;
  }
  fp.out_cols = d_out_cols;
  fp.row_base = row_base;
  fp.row_counter = w->counters + 1;
  fp.err_flag = w->counters + 2;
  HIP_TRY(hipMemsetAsync(w->counters + 1, 0, 2 * sizeof(uint64_t), w->stream));
  size_t lds = (size_t)(prog.nregs > 0 ? prog.nregs : 1) * BLOCK * sizeof(int64_t);
  hipEvent_t p = prof_begin(w);
  hipLaunchKernelGGL(k_expand<FINAL>, dim3((unsigned)ntiles), dim3(BLOCK), lds, w->stream, a, w->seg_end,
                     w->block_sum, w->seg_rs, w->part, total, w->flags, fp);
  prof_end(w, p, K_EXPAND_FINAL, 8.0 * (double)total * edge_columns_read(prog));
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(w->h_pinned, w->counters, 24, hipMemcpyDeviceToHost, w->stream));
  HIP_TRY(hipStreamSynchronize(w->stream));
  *rows_out = w->h_pinned[1];
  *err_out = w->h_pinned[2] != 0;
  if (!w->prof.pending.empty()) w->prof.pending.back().bytes += 8.0 * (double)*rows_out * kout;   // R * 8k
  prof_flush(w);
  return hipSuccess;
}

}  // namespace nbg
