// Workspace of a GO / FIND PATH query slot and the helpers the kernel files share (kernels.hip,
// walk.hip).  Internal to libnbg.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#include "nbg_internal.h"

namespace nbg {

constexpr int BLOCK = 256;
constexpr int WAVES = BLOCK / 64;
constexpr int FLAG_ALIGN = 1024 * 16;           // flag array granularity (k_compact workgroup)
constexpr int EXPAND_GRID = 2048;                // persistent k_expand grid (8 blocks / CU)

enum KernelId { K_RELIST = 0, K_EXPAND_MARK, K_COMPACT, K_EXPAND_FINAL, K_BFS, K_GATHER, K_DEGSUM, K_GREEDY,
                K_STAMP, K_PACK, K_ALLTOALL, K_BITS_COMPACT, K_ROOTS, K_COUNT };
[[maybe_unused]] static const char* const kKernelNames[K_COUNT] = {"k_relist", "k_expand<MARK>", "k_compact", "k_expand<FINAL>",
                                                  "k_expand<BFS>", "k_gather", "k_degsum", "k_greedy",
                                                  "k_stamp", "k_pack_bits", "alltoall(xGMI)", "k_bits_compact",
                                                  "alltoallv(roots)"};
constexpr int BITS_BLOCK = BLOCK * 16;           // k_bits_compact: vertices (bits) per block
constexpr uint64_t RW_BLOCK = 4 * BLOCK;          // root packing: bitmap words per prefix block

struct InlineIds {                 // a short start list passed by value in the kernel arguments
  uint32_t n;
  uint32_t id[INLINE_STARTS];
};

struct Prof {
  bool on = false;
  uint32_t mask = ~0u;     // kernels timed (bit per KernelId)
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
  // edge space of a list, two sets: frontier[i]'s list carries set i; k_relist writes into the
  // set of the current frontier (free by then); claim-mode MARK builds the next list in the other
  uint32_t* seg_end = nullptr;    // set 0: inclusive scan of degrees
  uint32_t* seg_rs = nullptr;     // set 0: row start per frontier entry
  uint32_t* seg_end1 = nullptr;   // set 1
  uint32_t* seg_rs1 = nullptr;
  uint32_t* tsplit1 = nullptr;
  uint32_t* seen = nullptr;       // [nv + 1] claim stamps of the per-step dst SET (single engine)
  uint32_t seen_stamp = 0;        // last stamp handed out
  uint32_t step_stamp = 0;        // stamp of the current step (all its OVER types)
  // partitioned roots ($- / $var props read after 2+ steps): MARKB writes them over the global
  // id space (bt_out); a hop sends only the roots of the vertices whose bits it sends, packed in
  // bit order (bt_pack -> bt_recv), at offsets from the bitmaps' popcount prefixes (ws_roots)
  int64_t* bt_out = nullptr;
  int64_t* bt_pack = nullptr;
  int64_t* bt_recv = nullptr;
  uint32_t* bt_pre = nullptr;     // [2][world * npad / 64] popcount before each word in its RW_BLOCK
  uint32_t* bt_boff = nullptr;    // [2][blocks] then the block's offset in its rank segment
  uint64_t* bt_disp = nullptr;    // [2][world] packed displacements: sent, received
  uint64_t* h_btc = nullptr;      // mapped pinned [2][world] counts: sent to / received from rank q
  uint64_t* d_btc = nullptr;
  bool bt_active = false;         // this query tracks roots: the hop exchange carries them
  // partitioned DISTINCT exchange scratch (row owners, counts, send / receive buffers)
  uint32_t* xown = nullptr;
  uint64_t xown_cap = 0;
  unsigned long long* xcnt = nullptr;
  uint64_t xcnt_cap = 0;
  int64_t* xsend = nullptr;
  int64_t* xrecv = nullptr;
  uint64_t xsend_cap = 0, xrecv_cap = 0;
  bool mark_flags = false;        // this query: byte flags + k_compact instead of claims
  bool env_flags = false;         // NBG_MARK_FLAGS=1: always flags
  uint32_t* rlist = nullptr;      // k_relist output list
  uint8_t* flags = nullptr;       // [nv rounded up to FLAG_ALIGN], kept all-zero between steps
  uint64_t flag_bytes = 0;
  uint32_t* tsplit = nullptr;      // [cap_tiles] merge-path split per tile (compaction-produced frontiers)
  uint32_t* blk_rows = nullptr;    // [MAX_TYPES_Q][EXPAND_GRID] final-step rows per workgroup
  uint32_t* h_blk_rows = nullptr;  // pinned mirror (valid after ws_end_query)
  unsigned final_grid[MAX_TYPES_Q] = {};
  uint64_t cap_tiles = 0;
  uint64_t e_max = 0;              // edges of the longest list the tiles cover (beside cap_frontier entries)
  bool seg_ready = false;          // the compaction list carries the first OVER type's edge space
  const unsigned long long* list_acc = nullptr;   // packed size of frontier[cur] (null: q->n, plain)
  int pr = 0, pc = 0;              // ping-pong parity of the relist / compaction accumulators
  uint64_t start_n = 0;            // step-1 list: start ids (inline in the kernel arguments when short)
  bool start_inline = false;
  InlineIds inl{};
  uint64_t prog_stmt = 0;          // statement whose programs d_prog holds
  std::vector<Ins> prog_img;      // ... and their words (upload skipped when a statement's equal them)
  std::vector<uint32_t> prog_lens;
  QState* q = nullptr;            // device query state
  QState* h_q = nullptr;          // pinned host mirror (mapped: k_q_out stores into it)
  QState* d_hq = nullptr;         // its device address
  int64_t* h_small = nullptr;     // mapped pinned: [0] = rows + 1 when packed, then the cells
  int64_t* d_small = nullptr;     // its device address
  // the host's wake-up (NBG_WAKE, default flag): the end-of-query kernel stores wake_seq into
  // the mapped word h_wake after its host-visible stores; the host polls it instead of an event
  unsigned long long* h_wake = nullptr;
  unsigned long long* d_wake = nullptr;
  unsigned int* d_ticket = nullptr;   // last-workgroup ticket of a multi-workgroup end kernel
  unsigned long long wake_seq = 0;
  bool wake_armed = false;            // the enqueued end kernel will store wake_seq
  bool wake_flag = true;              // ws_set_wake: the next end kernel may arm it
  bool q_reset = false;               // the enqueued end kernel zeroes QState behind its copy
  uint32_t* h_starts = nullptr;   // pinned staging for start ids
  uint64_t cap_starts = 0;
  Ins* h_prog = nullptr;          // pinned staging for programs
  int64_t* rows = nullptr;        // [ncols][cap_rows]
  uint64_t cap_rows = 0;
  int ncols_alloc = 0;
  int64_t** d_row_cols = nullptr; // device array of column pointers
  // YIELD DISTINCT scratch (grown on demand): open-addressing row table, keep flags, segments
  unsigned long long* dtab = nullptr;
  uint64_t dtab_cap = 0;
  uint8_t* dkeep = nullptr;
  uint64_t dkeep_cap = 0;
  uint64_t* dseg = nullptr;
  uint64_t dseg_cap = 0;
  uint32_t* dcnt = nullptr;
  uint8_t* dkinds = nullptr;
  int64_t* bt = nullptr;         // VertexBackTracker roots [nv] (queries with $- / $var props)
  uint8_t* walk_arena = nullptr;  // FIND ALL PATH level arrays (grow-only)
  size_t walk_cap = 0;
  Ins* d_prog = nullptr;          // [MAX_TYPES_Q][MAX_PROGRAM]
  char* sarena = nullptr;         // derived strings of the query's rows (OP_SOUT; grow-only)
  uint64_t sarena_cap = 0;
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
  int ppr = 0;                    // ping-pong parity of the path relist accumulators
  // partitioned mode: flags cover the global id space [world * npad), one
  // bitmap segment of npad bits per owner rank is exchanged per hop
  Comm* comm = nullptr;
  uint64_t npad = 0;
  unsigned long long* sendbits = nullptr;   // [world * npad / 64]
  unsigned long long* recvbits = nullptr;   // [world * npad / 64]
  unsigned long long* gst = nullptr;        // [GST_N] globally reduced query statistics
  hipEvent_t done_ev = nullptr;             // ws_wait's completion event
  unsigned long long* pgst = nullptr;       // [PG_N] globally reduced FIND PATH sizes
  unsigned long long* h_pgst = nullptr;
  // partitioned greedy (allocated on first use): per-block minima, this rank's record, every
  // rank's records, the path and {current global id, error} — the hops run without host waits
  void* g_part = nullptr;
  int64_t* g_rec = nullptr;
  int64_t* g_all = nullptr;
  int64_t* g_path = nullptr;
  unsigned long long* g_cur = nullptr;
  int64_t* h_gpath = nullptr;               // pinned: path + {cur, err}
  unsigned long long* ar_buf = nullptr;     // ws_allreduce_host scratch (grow-only)
  uint64_t ar_cap = 0;
  bool hop_bits = false;                    // this hop's MARKs set sendbits directly (no pack)
  uint64_t hop_slots = 0;                   // this hop sends slot arrays of this stride (0: bitmaps)
  uint64_t* fetch_meta = nullptr;           // ws_fetch_rows staging (grow-only)
  size_t fetch_meta_cap = 0;
  int64_t* fetch_out = nullptr;
  size_t fetch_out_cap = 0;
  unsigned long long* h_gst = nullptr;
};

// Wait for the workspace's stream.  A partitioned workspace's stream runs collectives: the wait
// is bounded by the communicator timeout and aborts the communicator when a peer never arrives.
[[maybe_unused]] static hipError_t ws_sync(Workspace* w) {
  if (!w->comm) return hipStreamSynchronize(w->stream);
  return w->comm->wait(w->stream) == 0 ? hipSuccess : hipErrorLaunchTimeOut;
}

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

// Exclusive scan of one value per thread over an NT-thread block; *total gets the block sum.
template <int NT = BLOCK>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* total, uint32_t* lds) {
  uint32_t inc = wave_incl_scan(v);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 63) lds[w] = inc;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) {
    uint32_t s = lds[i];
    pre += (i < w) ? s : 0u;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return pre + inc - v;
}

[[maybe_unused]] static inline uint64_t cdiv(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

#define HIP_TRY(x)                         \
  do {                                     \
    hipError_t e_ = (x);                   \
    if (e_ != hipSuccess) return e_;       \
  } while (0)

// Kernel timing: an event pair around each launch on the workspace stream, resolved after the
// query's single host synchronisation (byte counts need the device-side sizes).
[[maybe_unused]] static hipEvent_t prof_begin(Workspace* w, int kid) {
  if (!w->prof.on || !((w->prof.mask >> kid) & 1u)) return nullptr;
  hipEvent_t a = w->prof.get();
  (void)hipEventRecord(a, w->stream);
  return a;
}
[[maybe_unused]] static void prof_end(Workspace* w, hipEvent_t a, int kid, int step, int tix, double cols = 0, double kout = 0) {
  if (!a) return;
  hipEvent_t b = w->prof.get();
  (void)hipEventRecord(b, w->stream);
  w->prof.pending.push_back({kid, step, tix, a, b, cols, kout, false});
}

}  // namespace nbg
