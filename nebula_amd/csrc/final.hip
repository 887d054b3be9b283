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
//   * each entry of the tile's window writes its index at the tile position of its first edge
//     (a "head"), tagged with the wave's tile count so the head array is never cleared;
//   * a wave-wide max-scan (DPP row shifts and row broadcasts) carries the last head forward, so
//     every item knows its entry;
//   * the entry's (row start - edge offset) was stored beside it, so an item's CSR index is one
//     LDS read and one add.
// The WHERE column width and the single-_dst YIELD are template parameters: no per-tile switch.
#include <hip/hip_runtime.h>

#include "nbg_internal.h"

namespace nbg {
namespace {

constexpr int FB = 256;        // threads per workgroup
constexpr int FW = FB / 64;    // waves per workgroup
constexpr int FV = VT;         // items per lane: a tile is the producers' TILE
constexpr uint32_t HEAD_BITS = 9;   // an entry index within a tile's window: 0..TILE
static_assert(TILE + 1 <= (1 << HEAD_BITS), "head index width");

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// max with the value DPP brings from another lane (lanes without a source, or in rows the mask
// leaves out, read 0: the identity of max over indices)
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t max_dpp(uint32_t v) {
  const uint32_t t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xf, false);
  return v > t ? v : t;
}

// inclusive max-scan over the wave's 64 lanes: within rows of 16 (row_shr 1, 2, 4, 8), then
// row 15 into rows 1 and 3 (row_bcast:15) and lane 31 into rows 2 and 3 (row_bcast:31)
__device__ __forceinline__ uint32_t wave_max_scan(uint32_t v) {
  v = max_dpp<0x111, 0xf>(v);
  v = max_dpp<0x112, 0xf>(v);
  v = max_dpp<0x114, 0xf>(v);
  v = max_dpp<0x118, 0xf>(v);
  v = max_dpp<0x142, 0xa>(v);
  v = max_dpp<0x143, 0xc>(v);
  return v;
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

// WB: the WHERE column's stored width (0: no WHERE).  ONE: the only YIELD is _dst.
template <int WB, bool ONE>
__global__ void __launch_bounds__(FB) __attribute__((amdgpu_waves_per_eu(8)))
k_final_dst(FinalDstArgs a) {
  __shared__ uint32_t sHeadAll[FW][TILE];       // tile position -> (tag << HEAD_BITS | entry)
  __shared__ uint32_t sDeltaAll[FW][TILE + 1];  // entry -> row start - edge offset
  __shared__ unsigned long long sBase;          // rows this workgroup wrote
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t* const sHead = sHeadAll[w];
  uint32_t* const sDelta = sDeltaAll[w];
  const unsigned long long packed = *a.acc;   // (list entries << 32 | edges)
  const uint64_t n = packed >> 32, total = packed & 0xFFFFFFFFull;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (a.stat_e) *a.stat_e += total;
    if (a.stat_n) *a.stat_n = n;
  }
  for (int k = lane; k < TILE; k += 64) sHead[k] = 0;   // (tag 0 is never a tile's)
  if (threadIdx.x == 0) sBase = 0;
  __syncthreads();
  const uint64_t npath = n + total;
  const uint64_t ntiles = (npath + TILE - 1) / TILE;
  const uint64_t g = (uint64_t)gridDim.x * FW;
  // merge-path split of tile tt: entries consumed before its start (which 0) / its end (which 1).
  // A tile's split is wave-uniform: read through the scalar cache (address space 4), so its wait
  // is on lgkmcnt and never on the vector memory counter that the row stores share
  const __attribute__((address_space(4))) uint32_t* const tsplit =
      (const __attribute__((address_space(4))) uint32_t*)a.tsplit;
  auto split_of = [&](uint64_t tt, int which) -> uint64_t {
    if (which == 0) return tsplit[tt];
    return (tt + 1) * TILE >= npath ? n : tsplit[tt + 1];
  };
  // lane k's window entry s = k of the tile starting at entry s0: the raw edge offsets where it
  // starts (the end of entry s0 - 1 + k) and ends, and its row start, loaded at clamped indices
  // with no branch; `window` applies the bounds when the values are used (a select right after
  // a load is a wait for it: the prefetch would be waited for in the tile that issued it)
  auto stage = [&](uint64_t s0, uint32_t* x0, uint32_t* x1, uint32_t* rr) {
    const int64_t i = (int64_t)s0 - 1 + lane;
    const uint64_t c0 = i < 0 ? 0 : ((uint64_t)i < n ? (uint64_t)i : n - 1);
    const uint64_t c1 = (uint64_t)(i + 1) < n ? (uint64_t)(i + 1) : n - 1;
    *x0 = ld(a.seg_end + c0);
    *x1 = ld(a.seg_end + c1);
    *rr = ld(a.seg_rs + c1);
  };
  auto window = [&](uint64_t s0, uint32_t x0, uint32_t x1, uint32_t rr, uint32_t* st, uint32_t* en, uint32_t* r) {
    const int64_t i = (int64_t)s0 - 1 + lane;
    *st = i < 0 ? 0u : ((uint64_t)i < n ? x0 : 0xFFFFFFFFu);
    *en = (uint64_t)(i + 1) < n ? x1 : 0xFFFFFFFFu;
    *r = (uint64_t)(i + 1) < n ? rr : 0u;
  };
  const typename WType<WB>::T* const wcol = static_cast<const typename WType<WB>::T*>(a.wcol);
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
      const uint64_t row = region + off + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
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
  uint64_t t = (uint64_t)blockIdx.x * FW + w;   // adjacent tiles in one workgroup (shared lines)
  uint64_t a0 = 0, a1 = 0, n0 = 0, n1 = 0;   // splits of tiles t and t + g
  uint32_t e_pre = 0, f_pre = 0, r_pre = 0;   // lane's window entry of tile t
  if (t < ntiles) {
    a0 = split_of(t, 0);
    a1 = split_of(t, 1);
    if (t + g < ntiles) {
      n0 = split_of(t + g, 0);
      n1 = split_of(t + g, 1);
    }
    stage(a0, &e_pre, &f_pre, &r_pre);
  }
  uint32_t tag = 0;
  for (; t < ntiles; t += g) {
    if (++tag == (1u << (32 - HEAD_BITS))) {   // (unreachable in practice: 2^23 tiles on one wave)
      for (int k = lane; k < TILE; k += 64) sHead[k] = 0;
      tag = 1;
    }
    const uint64_t d0 = t * TILE;
    const uint64_t d1 = d0 + TILE < npath ? d0 + TILE : npath;
    const uint32_t b0 = (uint32_t)(d0 - a0), b1 = (uint32_t)(d1 - a1);
    const int na = (int)(a1 - a0);
    const int nb = (int)(b1 - b0);
    // ---- heads and deltas of the window's entries 0..na (64 at a time; past the first 64 —
    //      tiles of many low-degree entries — loaded here)
    for (int c = 0; c * 64 <= na; ++c) {   // (wave-uniform)
      const int s = c * 64 + lane;
      uint32_t x0 = e_pre, x1 = f_pre, rr = r_pre, st, en, rs;
      if (c > 0) stage(a0 + (uint64_t)c * 64, &x0, &x1, &rr);
      window(a0 + (uint64_t)c * 64, x0, x1, rr, &st, &en, &rs);
      if (s <= na) {
        sDelta[s] = rs - st;
        const uint32_t lo = st > b0 ? st : b0, hi = en < b1 ? en : b1;
        if (lo < hi) sHead[lo - b0] = (tag << HEAD_BITS) | (uint32_t)s;
      }
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
    // ---- every item's entry (the last head at or before it) and CSR index
    uint32_t jj[FV];
    uint32_t carry = 0;
#pragma unroll
    for (int i = 0; i < FV; ++i) {
      const int k = i * 64 + lane;
      const uint32_t h = sHead[k];
      uint32_t s = (h >> HEAD_BITS) == tag ? (h & ((1u << HEAD_BITS) - 1u)) : 0u;
      s = wave_max_scan(s);
      s = s > carry ? s : carry;
      carry = (uint32_t)__builtin_amdgcn_readlane((int)s, 63);
      jj[i] = b0 + (uint32_t)k + sDelta[s];
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
      if constexpr (WB != 0) {
        const int64_t v = (int64_t)x[i];
        pass = act & (((v >= a.lo) & (v <= a.hi)) != (a.where_neg != 0));
      }
      pm |= (uint32_t)pass << i;
    }
    uint32_t run = 0;
#pragma unroll
    for (int i = 0; i < FV; ++i) run += (uint32_t)__popcll(__ballot((pm >> i) & 1u));
    unsigned long long base = 0;
    if (lane == 0 && run) base = atomicAdd(&sBase, (unsigned long long)run);
    base = __shfl(base, 0, 64);
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
