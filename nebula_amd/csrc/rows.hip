// nebula_amd — result rows on the device (gfx950): packing row segments into columns (to the
// device or straight into pinned host memory), the order-independent row digest, and YIELD
// DISTINCT (single engine: an open-addressing row table; partitioned: rows hashed to an owner
// rank, one all-to-all, deduplicated there).  GoExecutor.cpp:771-778 (DISTINCT), graph.thrift
// :107-114 (the rows an ExecutionResponse carries).  Split out of kernels.hip in round 6.
#include <hip/hip_runtime.h>
#include <array>
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <vector>

#include "ws.h"

namespace nbg {

// ----------------------------------------------------------------------------- row packing
// Gathers the segments of a GO result (one per producing workgroup and type) into contiguous
// columns: segment k = rows [seg[3k], seg[3k] + seg[3k+1]) of every column, written at seg[3k+2].
__global__ void __launch_bounds__(BLOCK) k_pack_rows(const uint64_t* __restrict__ seg, int nseg,
                                                     int64_t* const* __restrict__ cols, int ncols,
                                                     int64_t* __restrict__ out, uint64_t total) {
  for (int k = blockIdx.x; k < nseg; k += gridDim.x) {
    const uint64_t b = seg[3 * k], len = seg[3 * k + 1], o = seg[3 * k + 2];
    for (int c = 0; c < ncols; ++c)
      for (uint64_t i = threadIdx.x; i < len; i += BLOCK) out[(uint64_t)c * total + o + i] = cols[c][b + i];
  }
}

// k_pack_rows into host memory (the pinned block, over the host link): 16-byte stores wherever the
// destination is 16-byte aligned (a 16-byte store per lane reaches ~54 GB/s into pinned memory,
// the DMA engine ~30, profiles/r03_q_d2h_bw_probe.json)
__global__ void __launch_bounds__(BLOCK) k_pack_rows_host(const uint64_t* __restrict__ seg, int nseg,
                                                          int64_t* const* __restrict__ cols, int ncols,
                                                          int64_t* __restrict__ out, uint64_t total) {
  for (int k = blockIdx.x; k < nseg; k += gridDim.x) {
    const uint64_t b = seg[3 * k], len = seg[3 * k + 1], o = seg[3 * k + 2];
    for (int c = 0; c < ncols; ++c) {
      const int64_t* src = cols[c] + b;
      int64_t* dst = out + (uint64_t)c * total + o;
      const uint64_t head = ((uintptr_t)dst & 15) ? 1 : 0;   // (8-byte aligned: at most one odd cell)
      if (head && threadIdx.x == 0 && len) dst[0] = src[0];
      const uint64_t body = len > head ? (len - head) / 2 : 0;
      const int64_t* s2 = src + head;
      longlong2* d2 = reinterpret_cast<longlong2*>(dst + head);
      for (uint64_t i = threadIdx.x; i < body; i += BLOCK) d2[i] = make_longlong2(s2[2 * i], s2[2 * i + 1]);
      const uint64_t done = head + 2 * body;
      if (done < len && threadIdx.x == 0) dst[done] = src[done];
    }
  }
}

// Order-independent digest of a result: per row h = splitmix64-chain of its 8-byte cell
// payloads (column order), summed and xor-ed over the rows (out = {rows, xor, sum}).
__device__ __forceinline__ uint64_t splitmix64_d(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void __launch_bounds__(BLOCK) k_rows_digest(const uint64_t* __restrict__ seg, int nseg,
                                                       int64_t* const* __restrict__ cols, int ncols,
                                                       unsigned long long* __restrict__ out) {
  unsigned long long n = 0, x = 0, sum = 0;
  for (int k = blockIdx.x; k < nseg; k += gridDim.x) {
    const uint64_t b = seg[3 * k], len = seg[3 * k + 1];
    for (uint64_t i = threadIdx.x; i < len; i += BLOCK) {
      uint64_t h = 0;
      for (int c = 0; c < ncols; ++c) h = splitmix64_d(h ^ (uint64_t)cols[c][b + i]);
      ++n;
      x ^= h;
      sum += h;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {   // wave64 reduction
    n += __shfl_xor(n, o);
    x ^= __shfl_xor(x, o);
    sum += __shfl_xor(sum, o);
  }
  if ((threadIdx.x & 63) == 0 && n) {
    atomicAdd(&out[0], n);
    atomicXor(&out[1], x);
    atomicAdd(&out[2], sum);
  }
}

// ----------------------------------------------------------------------------- YIELD DISTINCT
// GoExecutor::setupInterimResult keeps the first row of each distinct encoded row
// (GoExecutor.cpp:771-778).  A row's identity here is its value kinds (per OVER type) plus its
// 8-byte payloads — the encoded row up to the RowWriter framing.  k_distinct_mark inserts every
// row into an open-addressing table (CAS on an empty slot; a lost race re-compares), flagging the
// winners; k_distinct_compact then compacts each result segment in place, stably.
// seg[4k..4k+3] = (first row, rows, flag offset, OVER type index); kinds[type * MAX_YIELDS + c].
__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

__global__ void __launch_bounds__(BLOCK) k_distinct_mark(const uint64_t* __restrict__ seg, int nseg,
                                                         int64_t* const* __restrict__ cols, int ncols,
                                                         const uint8_t* __restrict__ kinds,
                                                         unsigned long long* __restrict__ tab, uint64_t tmask,
                                                         uint8_t* __restrict__ keep) {
  for (int k = blockIdx.x; k < nseg; k += gridDim.x) {
    const uint64_t b = seg[4 * k], len = seg[4 * k + 1], fo = seg[4 * k + 2];
    const uint32_t ty = (uint32_t)seg[4 * k + 3];
    for (uint64_t i = threadIdx.x; i < len; i += BLOCK) {
      const uint64_t row = b + i;
      uint64_t h = 0x6E6562756C61ull;
      for (int c = 0; c < ncols; ++c)
        h = mix64(h ^ (uint64_t)cols[c][row] ^ ((uint64_t)kinds[ty * MAX_YIELDS + c] << 61) ^ (uint64_t)c);
      const unsigned long long me = ((unsigned long long)ty << 48) | (row + 1);
      bool kept = false;
      for (uint64_t p = h & tmask;; p = (p + 1) & tmask) {
        unsigned long long cur = tab[p];
        if (cur == 0ull) {
          cur = atomicCAS(tab + p, 0ull, me);
          if (cur == 0ull) { kept = true; break; }
        }
        const uint64_t orow = (cur & ((1ull << 48) - 1)) - 1;
        const uint32_t oty = (uint32_t)(cur >> 48);
        bool eq = true;
        for (int c = 0; c < ncols && eq; ++c)
          eq = cols[c][orow] == cols[c][row] && kinds[oty * MAX_YIELDS + c] == kinds[ty * MAX_YIELDS + c];
        if (eq) break;
      }
      keep[fo + i] = kept ? 1 : 0;
    }
  }
}

__global__ void __launch_bounds__(BLOCK) k_distinct_compact(const uint64_t* __restrict__ seg, int nseg,
                                                            int64_t* const* __restrict__ cols, int ncols,
                                                            const uint8_t* __restrict__ keep,
                                                            uint32_t* __restrict__ counts) {
  __shared__ uint32_t wsum[WAVES];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int k = blockIdx.x; k < nseg; k += gridDim.x) {
    const uint64_t b = seg[4 * k], len = seg[4 * k + 1], fo = seg[4 * k + 2];
    uint64_t out = 0;
    for (uint64_t c0 = 0; c0 < len; c0 += BLOCK) {
      const uint64_t i = c0 + threadIdx.x;
      const bool kp = i < len && keep[fo + i];
      int64_t v[MAX_YIELDS];
#pragma unroll
      for (int c = 0; c < MAX_YIELDS; ++c)
        if (c < ncols && kp) v[c] = cols[c][b + i];
      const unsigned long long bal = __ballot(kp);
      if (lane == 0) wsum[wv] = (uint32_t)__popcll(bal);
      __syncthreads();   // every read of this chunk precedes its writes (positions <= reads)
      uint32_t before = 0, tot = 0;
      for (int x = 0; x < WAVES; ++x) {
        if (x < wv) before += wsum[x];
        tot += wsum[x];
      }
      if (kp) {
        const uint64_t dst = b + out + before + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
#pragma unroll
        for (int c = 0; c < MAX_YIELDS; ++c)
          if (c < ncols) cols[c][dst] = v[c];
      }
      out += tot;
      __syncthreads();
    }
    if (threadIdx.x == 0) counts[k] = (uint32_t)out;
  }
}

// Partitioned DISTINCT: every row goes to the rank its identity hashes to (equal rows meet at one
// owner, whatever rank produced them); the owners then deduplicate locally.
// seg as for k_distinct_mark, with seg[4k + 2] = the segment's first row in the global row order.
__device__ __forceinline__ uint64_t row_hash(int64_t* const* cols, int ncols, const uint8_t* kinds, uint32_t ty,
                                            uint64_t row) {
  uint64_t h = 0x6E6562756C61ull;
  for (int c = 0; c < ncols; ++c)
    h = mix64(h ^ (uint64_t)cols[c][row] ^ ((uint64_t)kinds[ty * MAX_YIELDS + c] << 61) ^ (uint64_t)c);
  return h;
}

__global__ void __launch_bounds__(BLOCK) k_row_route(const uint64_t* __restrict__ seg, int nseg,
                                                     int64_t* const* __restrict__ cols, int ncols,
                                                     const uint8_t* __restrict__ kinds, int world, int ntypes,
                                                     uint32_t* __restrict__ owner,
                                                     unsigned long long* __restrict__ cnt) {
  for (int k = blockIdx.x; k < nseg; k += gridDim.x) {
    const uint64_t b = seg[4 * k], len = seg[4 * k + 1], go = seg[4 * k + 2];
    const uint32_t ty = (uint32_t)seg[4 * k + 3];
    for (uint64_t i = threadIdx.x; i < len; i += BLOCK) {
      const uint32_t q = (uint32_t)(row_hash(cols, ncols, kinds, ty, b + i) >> 33) % (uint32_t)world;
      owner[go + i] = q;
      atomicAdd(&cnt[(uint64_t)q * ntypes + ty], 1ull);
    }
  }
}

// send[(q * maxc + base[q][ty] + cursor) * ncols + c] <- row; rows of one (owner, type) contiguous
__global__ void __launch_bounds__(BLOCK) k_row_pack(const uint64_t* __restrict__ seg, int nseg,
                                                    int64_t* const* __restrict__ cols, int ncols,
                                                    const uint32_t* __restrict__ owner, int ntypes,
                                                    const unsigned long long* __restrict__ base,
                                                    unsigned long long* __restrict__ cursor, uint64_t maxc,
                                                    int64_t* __restrict__ send) {
  for (int k = blockIdx.x; k < nseg; k += gridDim.x) {
    const uint64_t b = seg[4 * k], len = seg[4 * k + 1], go = seg[4 * k + 2];
    const uint32_t ty = (uint32_t)seg[4 * k + 3];
    for (uint64_t i = threadIdx.x; i < len; i += BLOCK) {
      const uint32_t q = owner[go + i];
      const uint64_t slot = (uint64_t)q * ntypes + ty;
      const uint64_t pos = base[slot] + atomicAdd(&cursor[slot], 1ull);
      int64_t* o = send + ((uint64_t)q * maxc + pos) * ncols;
      for (int c = 0; c < ncols; ++c) o[c] = cols[c][b + i];
    }
  }
}

// received rows of rank r (recv[(r * maxc + j) * ncols ..], j < n_r, type-major) -> the result
// columns at place[r * ntypes + ty] + (j - first row of that type)
__global__ void __launch_bounds__(BLOCK) k_row_unpack(const int64_t* __restrict__ recv, int world, int ntypes,
                                                      uint64_t maxc, int ncols,
                                                      const unsigned long long* __restrict__ rcnt,
                                                      const unsigned long long* __restrict__ place,
                                                      int64_t* const* __restrict__ cols) {
  const int r = blockIdx.y;
  uint64_t n = 0;
  for (int t = 0; t < ntypes; ++t) n += rcnt[(uint64_t)r * ntypes + t];
  for (uint64_t j = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; j < n; j += (uint64_t)gridDim.x * BLOCK) {
    uint64_t k = j;
    int t = 0;
    while (k >= rcnt[(uint64_t)r * ntypes + t]) k -= rcnt[(uint64_t)r * ntypes + t++];
    const uint64_t dst = place[(uint64_t)r * ntypes + t] + k;
    const int64_t* in = recv + ((uint64_t)r * maxc + j) * ncols;
    for (int c = 0; c < ncols; ++c) cols[c][dst] = in[c];
  }
}

// ============================================================================= host side
// YIELD DISTINCT over the result segments (synchronous): rows of each segment compacted in place,
// new row counts per segment in `counts`.  segs: (first row, rows, OVER type index).
hipError_t ws_distinct(Workspace* w, const std::vector<std::array<uint64_t, 3>>& segs, int ncols,
                       const std::vector<std::vector<VKind>>& kinds, std::vector<uint32_t>* counts) {
  counts->assign(segs.size(), 0);
  if (segs.empty() || !ncols) return hipSuccess;
  if (kinds.size() > (size_t)MAX_TYPES_Q) return hipErrorInvalidValue;
  uint64_t total = 0;
  std::vector<uint64_t> meta;
  for (auto& sg : segs) {
    meta.insert(meta.end(), {sg[0], sg[1], total, sg[2]});
    total += sg[1];
  }
  if (!total) return hipSuccess;
  uint64_t tcap = 1024;
  while (tcap < 2 * total) tcap <<= 1;
  HIP_TRY(ws_sync(w));
  if (tcap > w->dtab_cap) {
    if (w->dtab) HIP_TRY(hipFree(w->dtab));
    w->dtab = nullptr;
    HIP_TRY(hipMalloc((void**)&w->dtab, tcap * 8));
    w->dtab_cap = tcap;
  }
  if (total > w->dkeep_cap) {
    if (w->dkeep) HIP_TRY(hipFree(w->dkeep));
    w->dkeep = nullptr;
    HIP_TRY(hipMalloc((void**)&w->dkeep, total));
    w->dkeep_cap = total;
  }
  if (segs.size() > w->dseg_cap) {
    if (w->dseg) HIP_TRY(hipFree(w->dseg));
    if (w->dcnt) HIP_TRY(hipFree(w->dcnt));
    w->dseg = nullptr;
    w->dcnt = nullptr;
    HIP_TRY(hipMalloc((void**)&w->dseg, segs.size() * 32));
    HIP_TRY(hipMalloc((void**)&w->dcnt, segs.size() * 4));
    w->dseg_cap = segs.size();
  }
  if (!w->dkinds) HIP_TRY(hipMalloc((void**)&w->dkinds, MAX_TYPES_Q * MAX_YIELDS));
  uint8_t hk[MAX_TYPES_Q * MAX_YIELDS] = {};
  for (size_t t = 0; t < kinds.size(); ++t)
    for (size_t c = 0; c < kinds[t].size() && c < (size_t)MAX_YIELDS; ++c) hk[t * MAX_YIELDS + c] = (uint8_t)kinds[t][c];
  HIP_TRY(hipMemcpy(w->dkinds, hk, sizeof(hk), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(w->dseg, meta.data(), meta.size() * 8, hipMemcpyHostToDevice));
  HIP_TRY(hipMemsetAsync(w->dtab, 0, tcap * 8, w->stream));
  const unsigned grid = (unsigned)std::min<uint64_t>(segs.size(), 8192);
  hipLaunchKernelGGL(k_distinct_mark, dim3(grid), dim3(BLOCK), 0, w->stream, w->dseg, (int)segs.size(), w->d_row_cols,
                     ncols, w->dkinds, w->dtab, tcap - 1, w->dkeep);
  HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL(k_distinct_compact, dim3(grid), dim3(BLOCK), 0, w->stream, w->dseg, (int)segs.size(),
                     w->d_row_cols, ncols, w->dkeep, w->dcnt);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(counts->data(), w->dcnt, segs.size() * 4, hipMemcpyDeviceToHost, w->stream));
  return ws_sync(w);
}

hipError_t ws_distinct_exchange(Workspace* w, const std::vector<std::array<uint64_t, 3>>& segs, int ncols,
                                const std::vector<std::vector<VKind>>& kinds, std::vector<DistinctBlock>* out,
                                int32_t status, int32_t* gstatus) {
  *gstatus = NBG_OK;
  Comm* comm = w->comm;
  const int G = comm ? comm->world : 1, me = comm ? comm->rank : 0;
  const int T = (int)kinds.size();
  if (!comm || T < 1 || T > MAX_TYPES_Q || ncols < 1) return hipErrorInvalidValue;
  uint64_t total = 0;
  std::vector<uint64_t> meta;
  for (auto& sg : segs) {
    meta.insert(meta.end(), {sg[0], sg[1], total, sg[2]});
    total += sg[1];
  }
  HIP_TRY(ws_sync(w));
  // scratch: owners, counts [G][T] local and gathered, bases, cursors
  auto grow = [&](void** p, uint64_t* cap, uint64_t need) -> hipError_t {
    if (need <= *cap) return hipSuccess;
    if (*p) HIP_TRY(hipFree(*p));
    *p = nullptr;
    *cap = need + need / 2 + 4096;
    return hipMalloc(p, *cap);
  };
  const uint64_t GT = (uint64_t)G * T;
  HIP_TRY(grow((void**)&w->xown, &w->xown_cap, std::max<uint64_t>(total, 1) * 4));
  // each rank's counts carry its status word (the local dedup pass): a failure reaches every rank
  // with the counts, so the exchange needs no agreement of its own
  const uint64_t GS = GT + 1;
  HIP_TRY(grow((void**)&w->xcnt, &w->xcnt_cap, (GS + (uint64_t)G * GS + 2 * GT) * 8));
  unsigned long long* cnt = w->xcnt;            // [G][T] this rank's rows per (owner, type), then its status
  unsigned long long* all = cnt + GS;           // [G ranks][G][T + status]
  unsigned long long* base = all + (uint64_t)G * GS;
  unsigned long long* cursor = base + GT;
  if (!w->dkinds) HIP_TRY(hipMalloc((void**)&w->dkinds, MAX_TYPES_Q * MAX_YIELDS));
  uint8_t hk[MAX_TYPES_Q * MAX_YIELDS] = {};
  for (int t = 0; t < T; ++t)
    for (size_t c = 0; c < kinds[t].size() && c < (size_t)MAX_YIELDS; ++c) hk[t * MAX_YIELDS + c] = (uint8_t)kinds[t][c];
  HIP_TRY(hipMemcpy(w->dkinds, hk, sizeof(hk), hipMemcpyHostToDevice));
  if (segs.size() > w->dseg_cap) {
    if (w->dseg) HIP_TRY(hipFree(w->dseg));
    if (w->dcnt) HIP_TRY(hipFree(w->dcnt));
    w->dseg = nullptr;
    w->dcnt = nullptr;
    HIP_TRY(hipMalloc((void**)&w->dseg, segs.size() * 32));
    HIP_TRY(hipMalloc((void**)&w->dcnt, segs.size() * 4));
    w->dseg_cap = segs.size();
  }
  if (!meta.empty()) HIP_TRY(hipMemcpy(w->dseg, meta.data(), meta.size() * 8, hipMemcpyHostToDevice));
  HIP_TRY(hipMemsetAsync(cnt, 0, GT * 8, w->stream));
  const unsigned long long st_word = (unsigned long long)(long long)status;
  HIP_TRY(hipMemcpyAsync(cnt + GT, &st_word, 8, hipMemcpyHostToDevice, w->stream));
  const unsigned grid = (unsigned)std::min<uint64_t>(std::max<size_t>(segs.size(), 1), 8192);
  if (!segs.empty()) {
    hipLaunchKernelGGL(k_row_route, dim3(grid), dim3(BLOCK), 0, w->stream, w->dseg, (int)segs.size(), w->d_row_cols,
                       ncols, w->dkinds, G, T, w->xown, cnt);
    HIP_TRY(hipGetLastError());
  }
  if (comm->allgather(cnt, all, GS * 8, w->stream)) return hipErrorUnknown;
  HIP_TRY(ws_sync(w));
  std::vector<unsigned long long> h_all((uint64_t)G * GS);
  HIP_TRY(hipMemcpy(h_all.data(), all, h_all.size() * 8, hipMemcpyDeviceToHost));
  for (int r = 0; r < G; ++r)   // the first failing rank's code, on every rank: nothing more is exchanged
    if (h_all[(uint64_t)r * GS + GT]) {
      *gstatus = (int32_t)(long long)h_all[(uint64_t)r * GS + GT];
      return hipSuccess;
    }
  auto at = [&](int r, int q, int t) { return h_all[(uint64_t)r * GS + (uint64_t)q * T + t]; };
  uint64_t maxc = 1;
  for (int r = 0; r < G; ++r)
    for (int q = 0; q < G; ++q) {
      uint64_t n = 0;
      for (int t = 0; t < T; ++t) n += at(r, q, t);
      maxc = std::max(maxc, n);
    }
  std::vector<unsigned long long> h_base(GT);
  for (int q = 0; q < G; ++q) {
    uint64_t o = 0;
    for (int t = 0; t < T; ++t) {
      h_base[(uint64_t)q * T + t] = o;
      o += at(me, q, t);
    }
  }
  HIP_TRY(hipMemcpy(base, h_base.data(), GT * 8, hipMemcpyHostToDevice));
  HIP_TRY(hipMemsetAsync(cursor, 0, GT * 8, w->stream));
  const uint64_t xbytes = (uint64_t)G * maxc * ncols * 8;
  HIP_TRY(grow((void**)&w->xsend, &w->xsend_cap, xbytes));
  HIP_TRY(grow((void**)&w->xrecv, &w->xrecv_cap, xbytes));
  if (!segs.empty()) {
    hipLaunchKernelGGL(k_row_pack, dim3(grid), dim3(BLOCK), 0, w->stream, w->dseg, (int)segs.size(), w->d_row_cols,
                       ncols, w->xown, T, base, cursor, maxc, w->xsend);
    HIP_TRY(hipGetLastError());
  }
  if (comm->alltoall(w->xsend, w->xrecv, maxc * ncols * 8, w->stream)) return hipErrorUnknown;
  HIP_TRY(ws_sync(w));
  // this rank's rows by type: type t's block b = rows received from rank b
  out->assign(T, DistinctBlock{});
  std::vector<unsigned long long> h_rcnt(GT), h_place(GT);
  uint64_t region = 0;
  for (int t = 0; t < T; ++t) {
    uint64_t cap = 0;
    for (int r = 0; r < G; ++r) cap = std::max<uint64_t>(cap, at(r, me, t));
    (*out)[t].region = region;
    (*out)[t].blk_cap = cap;
    (*out)[t].counts.assign(G, 0);
    for (int r = 0; r < G; ++r) {
      h_rcnt[(uint64_t)r * T + t] = at(r, me, t);
      h_place[(uint64_t)r * T + t] = region + (uint64_t)r * cap;
    }
    region += (uint64_t)G * cap;
  }
  HIP_TRY(ws_reserve_rows(w, std::max<uint64_t>(region, 1), ncols));
  HIP_TRY(hipMemcpy(base, h_rcnt.data(), GT * 8, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(cursor, h_place.data(), GT * 8, hipMemcpyHostToDevice));
  if (region) {
    hipLaunchKernelGGL(k_row_unpack, dim3((unsigned)std::min<uint64_t>((maxc + BLOCK - 1) / BLOCK, 4096), (unsigned)G),
                       dim3(BLOCK), 0, w->stream, w->xrecv, G, T, maxc, ncols, base, cursor, w->d_row_cols);
    HIP_TRY(hipGetLastError());
  }
  // the owner's deduplication over what it received
  std::vector<std::array<uint64_t, 3>> rsegs;
  std::vector<std::pair<int, int>> where;
  for (int t = 0; t < T; ++t)
    for (int r = 0; r < G; ++r) {
      const uint64_t n = at(r, me, t);
      if (!n) continue;
      rsegs.push_back({(*out)[t].region + (uint64_t)r * (*out)[t].blk_cap, n, (uint64_t)t});
      where.emplace_back(t, r);
    }
  std::vector<uint32_t> kept;
  HIP_TRY(ws_distinct(w, rsegs, ncols, kinds, &kept));
  for (size_t k = 0; k < rsegs.size(); ++k) (*out)[where[k].first].counts[where[k].second] = kept[k];
  return hipSuccess;
}

// Synchronous: packs `segs` (begin, len) of the workspace's row columns into host columns.
hipError_t ws_fetch_rows(Workspace* w, const std::vector<std::pair<uint64_t, uint64_t>>& segs, int ncols,
                         uint64_t total, int64_t* const* host_cols) {
  if (!total || !ncols) return hipSuccess;
  std::vector<uint64_t> meta;
  uint64_t o = 0;
  for (auto& sg : segs) {
    if (!sg.second) continue;
    meta.push_back(sg.first);
    meta.push_back(sg.second);
    meta.push_back(o);
    o += sg.second;
  }
  if (o != total) return hipErrorInvalidValue;
  // grow-only staging in the workspace (no allocation / free, which would wait for the device, per
  // fetch)
  auto grow = [&](void** p, size_t* cap, size_t bytes) -> hipError_t {
    if (bytes <= *cap) return hipSuccess;
    if (*p) {
      hipError_t se = ws_sync(w);
      if (se != hipSuccess) return se;
      (void)hipFree(*p);
      *p = nullptr;
      *cap = 0;
    }
    hipError_t ae = hipMalloc(p, bytes);
    if (ae == hipSuccess) *cap = bytes;
    return ae;
  };
  hipError_t e = grow((void**)&w->fetch_meta, &w->fetch_meta_cap, meta.size() * 8);
  if (e == hipSuccess) e = grow((void**)&w->fetch_out, &w->fetch_out_cap, total * ncols * 8);
  uint64_t* d_meta = w->fetch_meta;
  int64_t* d_out = w->fetch_out;
  if (e == hipSuccess) e = hipMemcpyAsync(d_meta, meta.data(), meta.size() * 8, hipMemcpyHostToDevice, w->stream);
  if (e == hipSuccess) {
    const int nseg = (int)(meta.size() / 3);
    hipLaunchKernelGGL(k_pack_rows, dim3((unsigned)(nseg < 4096 ? nseg : 4096)), dim3(BLOCK), 0, w->stream, d_meta,
                       nseg, (int64_t* const*)w->d_row_cols, ncols, d_out, total);
    e = hipGetLastError();
  }
  bool contiguous = true;   // host columns back to back (a pinned block): one copy for all of them
  for (int c = 1; c < ncols; ++c) contiguous = contiguous && host_cols[c] == host_cols[0] + (uint64_t)c * total;
  if (contiguous && e == hipSuccess)
    e = hipMemcpyAsync(host_cols[0], d_out, total * (uint64_t)ncols * 8, hipMemcpyDeviceToHost, w->stream);
  for (int c = 0; !contiguous && e == hipSuccess && c < ncols; ++c)
    e = hipMemcpyAsync(host_cols[c], d_out + (uint64_t)c * total, total * 8, hipMemcpyDeviceToHost, w->stream);
  if (e == hipSuccess) e = ws_sync(w);
  return e;
}

// Rows into a pinned host block (columns back to back, `total` rows each): packed by the device
// straight into the block over the host link (16-byte stores), or — for results of 32 MB and
// more — packed on the device and DMAed (above; ~50 GB/s either way at that size,
// profiles/r03_r_host_delivered_ab.txt, while a copy-engine transfer of a small result costs
// ~130 us of latency, r03_m_d2h_probe.json).  NBG_FETCH=direct / dma forces one of them.
hipError_t ws_fetch_rows_pinned(Workspace* w, const std::vector<std::pair<uint64_t, uint64_t>>& segs, int ncols,
                                uint64_t total, int64_t* host_block) {
  if (!total || !ncols) return hipSuccess;
  static const char* mode = getenv("NBG_FETCH");
  const bool big = total * (uint64_t)ncols * 8 >= (32ull << 20);
  const bool dma = mode ? strcmp(mode, "direct") != 0 : big;
  void* dptr = nullptr;
  if (dma || hipHostGetDevicePointer(&dptr, host_block, 0) != hipSuccess || !dptr) {
    std::vector<int64_t*> hc(ncols);
    for (int c = 0; c < ncols; ++c) hc[c] = host_block + (uint64_t)c * total;
    return ws_fetch_rows(w, segs, ncols, total, hc.data());
  }
  std::vector<uint64_t> meta;
  uint64_t o = 0;
  for (auto& sg : segs) {
    if (!sg.second) continue;
    meta.push_back(sg.first);
    meta.push_back(sg.second);
    meta.push_back(o);
    o += sg.second;
  }
  if (o != total) return hipErrorInvalidValue;
  if (meta.size() * 8 > w->fetch_meta_cap) {
    if (w->fetch_meta) {
      HIP_TRY(ws_sync(w));
      (void)hipFree(w->fetch_meta);
      w->fetch_meta = nullptr;
      w->fetch_meta_cap = 0;
    }
    HIP_TRY(hipMalloc((void**)&w->fetch_meta, meta.size() * 8));
    w->fetch_meta_cap = meta.size() * 8;
  }
  HIP_TRY(hipMemcpyAsync(w->fetch_meta, meta.data(), meta.size() * 8, hipMemcpyHostToDevice, w->stream));
  const int nseg = (int)(meta.size() / 3);
  hipLaunchKernelGGL(k_pack_rows_host, dim3((unsigned)(nseg < 4096 ? nseg : 4096)), dim3(BLOCK), 0, w->stream,
                     w->fetch_meta, nseg, (int64_t* const*)w->d_row_cols, ncols, static_cast<int64_t*>(dptr), total);
  HIP_TRY(hipGetLastError());
  return ws_sync(w);
}

hipError_t ws_rows_digest(Workspace* w, const std::vector<std::pair<uint64_t, uint64_t>>& segs, int ncols,
                          uint64_t out[3]) {
  out[0] = out[1] = out[2] = 0;
  std::vector<uint64_t> meta;
  for (auto& sg : segs) {
    if (!sg.second) continue;
    meta.push_back(sg.first);
    meta.push_back(sg.second);
    meta.push_back(0);
  }
  if (meta.empty() || !ncols) return hipSuccess;
  uint64_t* d_meta = nullptr;
  unsigned long long* d_out = nullptr;
  hipError_t e = hipMalloc((void**)&d_meta, meta.size() * 8);
  if (e == hipSuccess) e = hipMalloc((void**)&d_out, 3 * 8);
  if (e == hipSuccess) e = hipMemcpyAsync(d_meta, meta.data(), meta.size() * 8, hipMemcpyHostToDevice, w->stream);
  if (e == hipSuccess) e = hipMemsetAsync(d_out, 0, 3 * 8, w->stream);
  if (e == hipSuccess) {
    const int nseg = (int)(meta.size() / 3);
    hipLaunchKernelGGL(k_rows_digest, dim3((unsigned)(nseg < 8192 ? nseg : 8192)), dim3(BLOCK), 0, w->stream, d_meta,
                       nseg, (int64_t* const*)w->d_row_cols, ncols, d_out);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(out, d_out, 3 * 8, hipMemcpyDeviceToHost, w->stream);
  if (e == hipSuccess) e = ws_sync(w);
  if (d_meta) (void)hipFree(d_meta);
  if (d_out) (void)hipFree(d_out);
  return e;
}

}  // namespace nbg
