// The final GO step for the statement shape that dominates GO traffic: WHERE `col <cmp> const`
// (or none) over one edge column and YIELDs that are `_dst` or constants — the bench's
// `GO 3 STEPS ... WHERE e.w < 50 YIELD e._dst`, GoExecutor::processFinalResult
// (src/graph/GoExecutor.cpp:803-984) with the storage filter of QueryBaseProcessor.inl:444-448.
//
// Same contract as k_expand<FINALD> (kernels.hip): the final frontier list with its edge space
// and merge-path tile splits in, rows appended to each workgroup's own region through an LDS
// cursor, blk_rows[workgroup] out.  What differs is the instruction budget per tile.  FINALD's
// waves were issue-bound, not memory-bound: ~400 instructions per 256-item tile, half of them
// scalar (the lane-level merge path's divergent binary search and per-item branches, SGPR spills
// of its large argument block), with the SIMDs issuing about every cycle
// (profiles/r02_r_pmc_sq_stall_rmat26.json: 56.7 M VALU + 57.6 M SALU per RMAT-26 launch).
// Here a tile's edge items find their frontier entry without a search:
//   * each entry of the tile's window with edges in the tile sets the bit of its first edge's tile
//     position in a 256-bit head mask (4 words in LDS) and stores its (row start - edge offset)
//     at its rank among those entries (ballot prefix counts);
//   * an item's entry is then the number of head bits at or before it: a popcount of the masked
//     word plus the earlier words', so its CSR index is two popcounts, one LDS read and one add.
// (Round 5's first version tagged heads with the tile count and carried the last head forward
// with a DPP max-scan per item row: 12 VALU per item where the popcounts take 4.)
// The WHERE column width and the single-_dst YIELD are template parameters: no per-tile switch.
#include <hip/hip_runtime.h>

#include "nbg_internal.h"

namespace nbg {
namespace {

constexpr int FB = 256;        // threads per workgroup
constexpr int FW = FB / 64;    // waves per workgroup
constexpr int FV = VT;         // items per lane: a tile is the producers' TILE
static_assert(FV == 4 && TILE == 256, "the head mask is 4 words of 64 tile positions");

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// A load the compiler issues where it is written: a relaxed wave-scope atomic load is a plain
// global_load that is never sunk into a conditional block (the select of a plain load's value
// became a branch around the load with a wait inside it, one memory round trip per load)
template <typename T>
__device__ __forceinline__ T ld(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

template <int WB>
struct WType { using T = int64_t; };
template <> struct WType<1> { using T = int8_t; };
template <> struct WType<2> { using T = int16_t; };
template <> struct WType<4> { using T = int32_t; };

}  // namespace

// WB: the WHERE column's stored width (0: no WHERE).  ONE: the only YIELD is _dst.  (Outside the
// anonymous namespace so profilers name it nbg::k_final_dst<WB, ONE>.)
template <int WB, bool ONE>
__global__ void __launch_bounds__(FB) __attribute__((amdgpu_waves_per_eu(8)))
k_final_dst(FinalDstArgs a) {
  __shared__ unsigned long long sMaskAll[FW][FV];   // tile positions where an entry's edges start
  __shared__ uint32_t sDeltaAll[FW][TILE + 1];      // head rank (1-based) -> row start - edge offset
  __shared__ unsigned long long sBase;          // rows this workgroup wrote
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  unsigned long long* const sMask = sMaskAll[w];
  uint32_t* const sDelta = sDeltaAll[w];
  const uint64_t g = (uint64_t)gridDim.x * FW;
  uint64_t t = (uint64_t)blockIdx.x * FW + w;   // adjacent tiles in one workgroup (shared lines)
  // merge-path split of tile tt: entries consumed before its start (which 0) / its end (which 1).
  // A tile's split is wave-uniform: read through the scalar cache (address space 4), so its wait
  // is on lgkmcnt and never on the vector memory counter that the row stores share
  const __attribute__((address_space(4))) uint32_t* const tsplit =
      (const __attribute__((address_space(4))) uint32_t*)a.tsplit;
  // the splits of this wave's first two tiles are loaded with the list's size, not after it (one
  // memory round trip less before the stream starts; the size then says which of them are used)
  const uint64_t tmax = a.tsplit_n ? a.tsplit_n - 1 : 0;
  auto clampt = [&](uint64_t x) { return x < tmax ? x : tmax; };
  const uint32_t sp0 = tsplit[clampt(t)], sp1 = tsplit[clampt(t + 1)];
  const uint32_t sq0 = tsplit[clampt(t + g)], sq1 = tsplit[clampt(t + g + 1)];
  const unsigned long long packed = *a.acc;   // (list entries << 32 | edges)
  const uint64_t n = packed >> 32, total = packed & 0xFFFFFFFFull;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (a.stat_e) *a.stat_e += total;
    if (a.stat_n) *a.stat_n = n;
  }
  if (threadIdx.x == 0) sBase = 0;
  __syncthreads();
  const uint64_t npath = n + total;
  const uint64_t ntiles = (npath + TILE - 1) / TILE;
  auto split_of = [&](uint64_t tt, int which) -> uint64_t {
    if (which == 0) return tsplit[tt];
    return (tt + 1) * TILE >= npath ? n : tsplit[tt + 1];
  };
  // lane k's window entry s = k of the tile starting at entry s0: the raw edge offsets where it
  // starts (the end of entry s0 - 1 + k) and ends, and its row start, loaded at clamped indices
  // with no branch; `window` applies the bounds when the values are used (a select right after
  // a load is a wait for it: the prefetch would be waited for in the tile that issued it)
  // (32-bit: a list holds fewer than 2^32 - 2 * TILE entries, ws_cap_frontier; q = s + 1)
  const uint32_t n32 = (uint32_t)n;
  auto stage = [&](uint64_t s0, uint32_t* x0, uint32_t* x1, uint32_t* rr) {
    const uint32_t q = (uint32_t)s0 + (uint32_t)lane;
    const uint32_t c0 = q == 0 ? 0u : (q - 1 < n32 ? q - 1 : n32 - 1);
    const uint32_t c1 = q < n32 ? q : n32 - 1;
    *x0 = ld(a.seg_end + c0);
    *x1 = ld(a.seg_end + c1);
    *rr = ld(a.seg_rs + c1);
  };
  auto window = [&](uint64_t s0, uint32_t x0, uint32_t x1, uint32_t rr, uint32_t* st, uint32_t* en, uint32_t* r) {
    const uint32_t q = (uint32_t)s0 + (uint32_t)lane;
    *st = q == 0 ? 0u : (q - 1 < n32 ? x0 : 0xFFFFFFFFu);
    *en = q < n32 ? x1 : 0xFFFFFFFFu;
    *r = q < n32 ? rr : 0u;
  };
  const typename WType<WB>::T* const wcol = static_cast<const typename WType<WB>::T*>(a.wcol);
  // the WHERE `lo <= x <= hi` (!= where_neg) over a column of at most 4 bytes, as one 32-bit
  // compare: the bounds clamped to int32 (the values' range), an empty range as the full range
  // with the negation flipped, then (uint32)(x - lo) <= hi - lo
  int64_t wlo = a.lo, whi = a.hi;
  bool wneg = a.where_neg != 0;
  if (wlo < INT32_MIN) wlo = INT32_MIN;
  if (whi > INT32_MAX) whi = INT32_MAX;
  if (wlo > whi) {
    wlo = INT32_MIN;
    whi = INT32_MAX;
    wneg = !wneg;
  }
  const uint32_t wbase = (uint32_t)(int32_t)wlo, wspan = (uint32_t)(whi - wlo);
  // rows of one tile at `region`, in item order (ballots of the pass masks).  One predicated
  // store per item slot, none skipped by a branch: the count of memory instructions after the
  // tile's loads is fixed, so the wait for those loads is vmcnt(FV * nyields) and never waits for
  // these stores (one counter retires loads and stores in issue order)
  auto store_rows = [&](const int64_t (&dv)[FV], uint32_t pm, uint64_t region) {
    uint32_t off = 0;
#pragma unroll
    for (int i = 0; i < FV; ++i) {
      const bool pass = (pm >> i) & 1u;
      const unsigned long long bal = __ballot(pass);
      const uint64_t row = region + off + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
      off += (uint32_t)__popcll(bal);
      if constexpr (ONE) {
        if (pass) a.out[0][row] = dv[i];
      } else {
        for (int y = 0; y < a.nyields; ++y)
          if (pass) a.out[y][row] = ((a.const_mask >> y) & 1u) ? a.yconst[y] : dv[i];
      }
    }
  };
  int64_t pdv[FV];   // the previous tile's _dst values, pass mask and first row (stored behind the
  uint32_t ppm = 0;  // next tile's loads: one vmcnt retires loads and stores in issue order)
  uint64_t preg = 0;
#pragma unroll
  for (int i = 0; i < FV; ++i) pdv[i] = 0;
  uint64_t a0 = 0, a1 = 0, n0 = 0, n1 = 0;   // splits of tiles t and t + g
  uint32_t e_pre = 0, f_pre = 0, r_pre = 0;   // lane's window entry of tile t
  if (t < ntiles) {
    a0 = sp0;
    a1 = (t + 1) * TILE >= npath ? n : sp1;
    if (t + g < ntiles) {
      n0 = sq0;
      n1 = (t + g + 1) * TILE >= npath ? n : sq1;
    }
    stage(a0, &e_pre, &f_pre, &r_pre);
  }
  // lanes at or below this one: the popcount mask of an item's own head word
  const unsigned long long le = ~0ull >> (63 - lane);
  for (; t < ntiles; t += g) {
    const uint64_t d0 = t * TILE;
    const uint64_t d1 = d0 + TILE < npath ? d0 + TILE : npath;
    // a split that does not describe this tile (stale list memory) skips it and fails the query
    // (SPLIT_BAD) instead of indexing out of bounds
    const bool bad = !(a0 <= a1 && a1 <= n && a1 - a0 <= d1 - d0 && d1 - a1 <= total && d0 - a0 <= d1 - a1);
    if (bad && lane == 0) atomicOr(a.err_flag, SPLIT_BAD);
    const uint32_t b0 = bad ? 0u : (uint32_t)(d0 - a0), b1 = bad ? 0u : (uint32_t)(d1 - a1);
    const int na = bad ? 0 : (int)(a1 - a0);
    const int nb = (int)(b1 - b0);
    // ---- head bits and deltas of the window's entries 0..na that have edges in the tile (64
    //      at a time; past the first 64 — tiles of many low-degree entries — loaded here).  The
    //      previous tile's mask reads are earlier LDS instructions of this wave: in order
    if (lane < FV) sMask[lane] = 0;
    uint32_t heads = 0;
    for (int c = 0; c * 64 <= na; ++c) {   // (wave-uniform)
      const int s = c * 64 + lane;
      uint32_t x0 = e_pre, x1 = f_pre, rr = r_pre, st, en, rs;
      if (c > 0) stage(a0 + (uint64_t)c * 64, &x0, &x1, &rr);
      window(a0 + (uint64_t)c * 64, x0, x1, rr, &st, &en, &rs);
      const uint32_t lo = st > b0 ? st : b0, hi = en < b1 ? en : b1;
      const bool head = s <= na && lo < hi;
      const unsigned long long hb = __ballot(head);
      if (head) {
        const uint32_t p = lo - b0;   // < nb <= TILE
        sDelta[heads + 1 + (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(hb >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((uint32_t)hb, 0u))] = rs - st;
        atomicOr(&sMask[p >> 6], 1ull << (p & 63));
      }
      heads += (uint32_t)__popcll(hb);
    }
    // prefetch tile t + g's window and tile t + 2g's split
    const uint64_t na0 = n0, na1 = n1;
    if (t + g < ntiles) {
      stage(na0, &e_pre, &f_pre, &r_pre);
      if (t + 2 * g < ntiles) {
        n0 = split_of(t + 2 * g, 0);
        n1 = split_of(t + 2 * g, 1);
      }
    }
    wave_lds_sync();
    // ---- every item's entry (the head bits at or before it: item 0 of a tile with edges is
    //      always a head) and CSR index; an item past the tile's edges may count 0 (sDelta[0]: any
    //      value, its index is replaced below)
    uint32_t jj[FV];
    {
      uint32_t before = 0;
#pragma unroll
      for (int i = 0; i < FV; ++i) {
        const unsigned long long m = sMask[i];
        const uint32_t c = before + (uint32_t)__popcll(m & le);
        before += (uint32_t)__popcll(m);
        jj[i] = b0 + (uint32_t)(i * 64 + lane) + sDelta[c];
      }
    }
    wave_lds_sync();   // (the next tile rewrites the window)
    // ---- loads: every item's _dst, then its WHERE value, all in flight before the first wait.
    //      No branch around them (a branch made each narrow load wait for itself, four round
    //      trips per tile): an item past the tile's edges reads the tile's first edge instead
    int64_t dv[FV];
    typename WType<WB>::T x[FV];
    {
      // item 0 is an edge of the tile when it has any; else edge 0 of the CSR (the host passes
      // columns of at least one element)
      const uint32_t jsafe = nb > 0 ? (uint32_t)__builtin_amdgcn_readfirstlane((int)jj[0]) : 0u;
#pragma unroll
      for (int i = 0; i < FV; ++i)
        if (i * 64 + lane >= nb) jj[i] = jsafe;
#pragma unroll
      for (int i = 0; i < FV; ++i) dv[i] = ld(a.dst_vid + jj[i]);
      if constexpr (WB != 0) {
#pragma unroll
        for (int i = 0; i < FV; ++i) x[i] = ld(wcol + jj[i]);
      }
    }
    store_rows(pdv, ppm, preg);   // the previous tile's rows, behind this tile's loads
    uint32_t pm = 0;
#pragma unroll
    for (int i = 0; i < FV; ++i) {
      const bool act = i * 64 + lane < nb;
      bool pass = act;
      if constexpr (WB == 8) {
        const int64_t v = (int64_t)x[i];
        pass = act & (((v >= a.lo) & (v <= a.hi)) != (a.where_neg != 0));
      } else if constexpr (WB != 0) {
        pass = act & (((uint32_t)(int32_t)x[i] - wbase <= wspan) != wneg);
      }
      pm |= (uint32_t)pass << i;
    }
    uint32_t run = 0;
#pragma unroll
    for (int i = 0; i < FV; ++i) run += (uint32_t)__popcll(__ballot((pm >> i) & 1u));
    unsigned long long base = 0;
    if (lane == 0 && run) base = atomicAdd(&sBase, (unsigned long long)run);
    base = ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(base >> 32), 0) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)base, 0);
#pragma unroll
    for (int i = 0; i < FV; ++i) pdv[i] = dv[i];
    ppm = pm;
    preg = a.region_base + (uint64_t)blockIdx.x * a.blk_cap + base;
    a0 = na0;
    a1 = na1;
  }
  store_rows(pdv, ppm, preg);   // the wave's last tile
  __syncthreads();              // every wave of the workgroup has reserved its rows
  if (threadIdx.x == 0) a.blk_rows[blockIdx.x] = (uint32_t)sBase;
}

namespace {

template <int WB>
void launch_wb(const FinalDstArgs& a, bool one, unsigned grid, hipStream_t s) {
  if (one) hipLaunchKernelGGL((k_final_dst<WB, true>), dim3(grid), dim3(FB), 0, s, a);
  else hipLaunchKernelGGL((k_final_dst<WB, false>), dim3(grid), dim3(FB), 0, s, a);
}

}  // namespace

hipError_t launch_final_dst(const FinalDstArgs& a, int wbytes, bool one, unsigned grid, hipStream_t s) {
  switch (wbytes) {
    case 0: launch_wb<0>(a, one, grid, s); break;
    case 1: launch_wb<1>(a, one, grid, s); break;
    case 2: launch_wb<2>(a, one, grid, s); break;
    case 4: launch_wb<4>(a, one, grid, s); break;
    case 8: launch_wb<8>(a, one, grid, s); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace nbg
