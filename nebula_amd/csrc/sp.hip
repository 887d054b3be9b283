// A one-pair FIND SHORTEST PATH slot (single engine): the labels and the device-driven level
// loop of spchain.hip, with the event the host waits on.  path.cpp hands the slot a pair; the
// chain runs the search, the B-sets and the greedy reconstruction on the device (semantics of
// FindPathExecutor.cpp:145-411: minimal hop count, UPTO N, one path per target, the
// lexicographically smallest entry list [v0, t0, r0, v1, ...] among the shortest).
//
// (A single persistent launch with grid-wide phase barriers was measured slower than the launch
// chain and removed in round 4; DESIGN.md §5 keeps the record.)
#include <hip/hip_runtime.h>

#include <algorithm>
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

// ---------------------------------------------------------------------------- host side
struct SpCtx {
  hipStream_t stream = nullptr;
  uint64_t nv = 0, cap = 0, edge_cap = 0;
  uint64_t list_cap = 0;           // the chain's list capacity (0: nv + 1)
  ChainCtx* chain = nullptr;       // the level-loop buffers (first query)
  uint32_t* lab_rec = nullptr;     // (nv + 1) label records of CH_LAB_WORDS words
  uint32_t* lab[3] = {};           // forward, backward, B-set labels: words 0, 1, 2 of the records
  uint32_t epoch = 0;
  hipEvent_t done = nullptr;
  int prof = 0;                    // nbg_profile mode, applied to the chain when it is created
};

static size_t lab_bytes(uint64_t nv) { return (size_t)(nv + 1) * CH_LAB_WORDS * 4; }

hipError_t sp_reserve_chain(SpCtx* c) {
  if (c->chain) return hipSuccess;
  std::string err;
  c->chain = chain_create(c->nv, c->edge_cap, c->stream, &err, c->list_cap);
  if (!c->chain) return hipErrorOutOfMemory;
  if (c->prof) chain_profile(c->chain, c->prof);
  return hipSuccess;
}

void sp_set_list_cap(SpCtx* c, uint64_t list_cap) {
  if (c && !c->chain) c->list_cap = list_cap;
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
  hipError_t he = hipSuccess;
  he = hipMalloc((void**)&c->lab_rec, lab_bytes(nv));
  for (int i = 0; i < 3 && he == hipSuccess; ++i) c->lab[i] = c->lab_rec + i;
  if (he == hipSuccess) he = hipEventCreateWithFlags(&c->done, hipEventDisableTiming);
  if (he == hipSuccess) he = hipMemsetAsync(c->lab_rec, 0, lab_bytes(nv), s);
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
  if (c->lab_rec) (void)hipFree(c->lab_rec);
  chain_destroy(c->chain);
  if (c->done) (void)hipEventDestroy(c->done);
  delete c;
}

static hipError_t next_epoch(SpCtx* c) {
  // wrap (clear the labels once) below 2^24: spchain.hip's same-launch meet tags use the epochs
  // with bit 24 or 25 set
  if (++c->epoch >= (1u << 24)) {
    HIP_TRY_SP(hipMemsetAsync(c->lab_rec, 0, lab_bytes(c->nv), c->stream));
    c->epoch = 1;
  }
  return hipSuccess;
}

hipError_t sp_launch(SpCtx* c, const SpTypes& fwd, const SpTypes& bwd, const uint8_t* visible, const int64_t* vids,
                     uint32_t s, uint32_t t, uint32_t upto, uint64_t dmin) {
  if (upto > MAX_PATH_LEN || s == NO_ROW || t == NO_ROW) return hipErrorInvalidValue;
  HIP_TRY_SP(next_epoch(c));
  HIP_TRY_SP(sp_reserve_chain(c));
  HIP_TRY_SP(chain_launch(c->chain, fwd, bwd, visible, vids, c->lab, c->epoch, s, t, upto, dmin));
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
    HIP_TRY_SP(next_epoch(c));
    HIP_TRY_SP(sp_reserve_chain(c));
    chains[p] = c->chain;
    qs[p] = ChainQuery{x.fwd, x.bwd, x.visible, x.vids, c->lab, c->epoch, x.s, x.t, x.upto};
  }
  HIP_TRY_SP(chain_launch_batch(chains.data(), n, qs.data()));
  for (int p = 0; p < n; ++p) HIP_TRY_SP(hipEventRecord(cs[p]->done, cs[p]->stream));
  return hipSuccess;
}

// n pairs over nslots slots as one rolling run (spchain.hip chain_roll): each slot reserves n + 2
// label epochs (its pairs' ordinals are below n + 1), clearing its labels first when they would
// reach the tag bits
hipError_t sp_roll(SpCtx* const* cs, int nslots, const SpTypes& fwd, const SpTypes& bwd, const uint8_t* visible,
                   const int64_t* vids, const uint32_t* s, const uint32_t* t, uint32_t n, uint32_t upto,
                   SpResult* results) {
  if (nslots < 1 || nslots > CH_ROLL_SLOTS || n >= (1u << 22)) return hipErrorInvalidValue;
  std::vector<ChainSlot> sl(nslots);
  for (int l = 0; l < nslots; ++l) {
    SpCtx* c = cs[l];
    if (c->stream != cs[0]->stream) return hipErrorInvalidValue;
    HIP_TRY_SP(sp_reserve_chain(c));
    if (c->epoch + n + 2 >= (1u << 24)) {
      HIP_TRY_SP(hipMemsetAsync(c->lab_rec, 0, lab_bytes(c->nv), c->stream));
      c->epoch = 0;
    }
    sl[l] = ChainSlot{c->chain, c->lab, c->epoch};
    c->epoch += n + 2;
  }
  return chain_roll(sl.data(), nslots, fwd, bwd, visible, vids, s, t, n, upto, results);
}

// NBG_WAKE=event: wait for the event behind the batch only (the A/B baseline)
static bool wake_by_flag() {
  static const bool on = !(getenv("NBG_WAKE") && strcmp(getenv("NBG_WAKE"), "event") == 0);
  return on;
}

static bool blocking_sync() {   // NBG_BLOCKING_SYNC: the waits block instead of polling
  static const bool on = getenv("NBG_BLOCKING_SYNC") != nullptr;
  return on;
}

bool sp_ready(SpCtx* c) { return (wake_by_flag() && chain_woken(c->chain)) || hipEventQuery(c->done) == hipSuccess; }

// The batch's end: its last launch's wake word (the result is readable before the launch has
// retired and the event behind it is signalled), or the event — a batch that ended inside the
// search stores nothing, and a failed launch ends the wait with its error.
static hipError_t wait_batch(SpCtx* c) {
  if (blocking_sync()) return hipEventSynchronize(c->done);
  const bool flag = wake_by_flag();
  for (unsigned k = 1;; ++k) {
    if (flag && chain_woken(c->chain)) {
      (void)hipEventQuery(c->done);   // (lets the runtime retire what it has finished)
      return hipSuccess;
    }
    if (!flag || (k & 255) == 0) {
      const hipError_t e = hipEventQuery(c->done);
      if (e != hipErrorNotReady) return e;
    }
  }
}

hipError_t sp_wait(SpCtx* c, SpResult* out) {
  hipError_t e = wait_batch(c);
  if (e != hipSuccess) return e;
  while (!chain_more(c->chain, &e)) {   // a continuation batch: wait for it too
    if (e == hipSuccess) e = hipEventRecord(c->done, c->stream);
    if (e != hipSuccess) return e;
    if ((e = wait_batch(c)) != hipSuccess) return e;
  }
  if (e != hipSuccess) return e;
  chain_result(c->chain, out);
  chain_profile_done(c->chain, *out);
  return hipSuccess;
}

}  // namespace nbg
