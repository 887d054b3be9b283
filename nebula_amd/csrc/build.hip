// Device-side snapshot build: staged kvstore records -> CSR / CSC per signed edge type, in HBM.
//
// loader.cpp's finalize hands every signed type's staged records (load order) to bd_build_type.
// What a storaged prefix scan would return per (part, src, type) is computed with data-parallel
// passes instead of per-vertex host sorts:
//   * the vertex dictionary is the sorted set of every record's source (radix sort + unique);
//   * a record permutation is sorted by stable LSD radix passes, least significant key first:
//       load order descending (identical keys: the later write wins), version bytes ascending
//       (newest version first), bswap64(dst), bswap64(rank), dense source id —
//     i.e. memcmp order of the 40-byte edge key (NebulaKeyUtils.cpp:28-47) within each source;
//   * the first record of every (src, rank, dst) group is the live edge (the version skip of
//     QueryBaseProcessor.inl:394-408); flags -> exclusive scan -> one scatter writes the CSR;
//   * neighbour ids are binary searches into the (global) dictionary.
// The sorts are rocPRIM's device radix sort (load path only; the traversal kernels are in
// kernels.hip).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <rocprim/rocprim.hpp>

#include "nbg_internal.h"

namespace nbg {
namespace {

constexpr int BT = 256;

unsigned grid_for(uint64_t n) {
  const uint64_t g = (n + BT - 1) / BT;
  return (unsigned)std::min<uint64_t>(std::max<uint64_t>(g, 1), 1u << 18);
}

#define GRID_STRIDE(i, n) \
  for (uint64_t i = (uint64_t)blockIdx.x * BT + threadIdx.x; i < (n); i += (uint64_t)gridDim.x * BT)

__device__ inline uint64_t lower_bound_i64(const int64_t* a, uint64_t n, int64_t v) {
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__device__ inline uint64_t lower_bound_u32(const uint32_t* a, uint64_t n, uint32_t v) {
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__device__ inline uint32_t gid_of(const GidMap& g, int64_t v) {
  if (!g.gdict) {
    const uint64_t r = lower_bound_i64(g.dict, g.nv, v);
    return (r < g.nv && g.dict[r] == v) ? (uint32_t)r : NO_ROW;
  }
  const uint64_t q = ((uint64_t)v % (uint64_t)g.parts + 1) % (uint64_t)g.gpus;   // owner: part % G
  const int64_t* b = g.gdict + q * g.npad;
  const uint64_t c = g.gcount[q];
  const uint64_t r = lower_bound_i64(b, c, v);
  return (r < c && b[r] == v) ? (uint32_t)(q * g.npad + r) : NO_ROW;
}

__global__ void k_iota_desc(uint32_t* p, uint64_t n) {
  GRID_STRIDE(i, n) p[i] = (uint32_t)(n - 1 - i);
}

template <bool BSWAP>
__global__ void k_gather_key(uint64_t* out, const uint64_t* key, const uint32_t* perm, uint64_t n) {
  GRID_STRIDE(i, n) {
    const uint64_t k = key[perm[i]];
    out[i] = BSWAP ? __builtin_bswap64(k) : k;
  }
}

__global__ void k_gather_u32(uint32_t* out, const uint32_t* key, const uint32_t* perm, uint64_t n) {
  GRID_STRIDE(i, n) out[i] = key[perm[i]];
}

__global__ void k_dense(uint32_t* sd, const int64_t* vids, uint64_t n, const int64_t* dict, uint64_t nv) {
  GRID_STRIDE(i, n) sd[i] = (uint32_t)lower_bound_i64(dict, nv, vids[i]);   // every source is in dict
}

// home part of every vertex (the part its records sit in); a vertex with records in two parts
// is not representable (split)
__global__ void k_home(int32_t* home, const uint32_t* sd, const int64_t* src, const int32_t* part, uint64_t n,
                       int32_t parts, unsigned* split) {
  bool bad = false;
  GRID_STRIDE(i, n) {
    const int32_t p = part ? part[i] : (int32_t)((uint64_t)src[i] % (uint64_t)parts + 1);
    const int32_t old = atomicCAS(&home[sd[i]], 0, p);
    bad |= old != 0 && old != p;
  }
  if (bad) atomicOr(split, 1u);
}

__global__ void k_live(uint32_t* live, const uint32_t* sd_sorted, const uint32_t* perm, const int64_t* dst,
                       const int64_t* rank, uint64_t n) {
  GRID_STRIDE(i, n) {
    bool l = i == 0;
    if (!l) {
      const uint32_t a = perm[i], b = perm[i - 1];
      l = sd_sorted[i] != sd_sorted[i - 1] || dst[a] != dst[b] || (rank && rank[a] != rank[b]);
    }
    live[i] = l;
  }
}

// superseded versions: a record that is not its group's live edge but the first of its own
// (src, rank, dst, version) run (identical keys: only the last write exists)
__global__ void k_old(uint32_t* old, const uint32_t* live, const uint32_t* perm, const uint64_t* ver, uint64_t n) {
  GRID_STRIDE(i, n) old[i] = !live[i] && ver[perm[i]] != ver[perm[i - 1]];
}

__global__ void k_row_ptr(uint32_t* row_ptr, const uint32_t* sd_sorted, const uint32_t* pos, uint64_t n, uint64_t nv,
                          uint32_t E) {
  GRID_STRIDE(d, nv + 1) {
    const uint64_t r = lower_bound_u32(sd_sorted, n, (uint32_t)d);
    row_ptr[d] = r < n ? pos[r] : E;
  }
}

struct EmitArgs {
  const uint32_t* perm;
  const uint32_t* live;
  const uint32_t* pos;
  const int64_t* dst;
  const int64_t* rank;
  const uint8_t* valid;
  const int64_t* const* pin;    // [nprops] staged columns
  int64_t* const* pout;         // [nprops] CSR columns
  int nprops;
  uint32_t* col;
  int64_t* dvid;
  int64_t* rank_out;
  uint8_t* valid_out;
  GidMap g;
  unsigned* flags;              // bit 0: a live rank != 0, bit 1: a live undecodable value
  const uint32_t* gpos;         // superseded versions: the live edges' positions (grp = gpos - 1)
  uint32_t* grp;
};

__global__ void k_emit(EmitArgs a, uint64_t n) {
  unsigned fl = 0;
  GRID_STRIDE(i, n) {
    if (!a.live[i]) continue;
    const uint32_t o = a.pos[i];
    const uint32_t j = a.perm[i];
    const int64_t v = a.dst[j];
    a.col[o] = gid_of(a.g, v);
    a.dvid[o] = v;
    if (a.grp) a.grp[o] = a.gpos[i] - 1;
    if (a.rank) {
      const int64_t r = a.rank[j];
      a.rank_out[o] = r;
      fl |= r != 0 ? 1u : 0u;
    }
    for (int c = 0; c < a.nprops; ++c) a.pout[c][o] = a.pin[c][j];
    if (a.valid) {
      const uint8_t ok = a.valid[j];
      a.valid_out[o] = ok;
      fl |= ok ? 0u : 2u;
    }
  }
  if (fl) atomicOr(a.flags, fl);
}

template <typename T>
__global__ void k_narrow(T* out, const int64_t* in, uint64_t n) {
  GRID_STRIDE(i, n) out[i] = (T)in[i];
}

// ---------------------------------------------------------------------------------- helpers
struct Scratch {   // device temporaries of one build step, released together
  std::vector<void*> ptrs;
  hipError_t err = hipSuccess;
  template <typename T>
  T* alloc(uint64_t count) {
    void* p = nullptr;
    if (err == hipSuccess) err = hipMalloc(&p, std::max<uint64_t>(count, 1) * sizeof(T));
    if (err == hipSuccess) ptrs.push_back(p);
    return static_cast<T*>(p);
  }
  void release(void* p) {
    auto it = std::find(ptrs.begin(), ptrs.end(), p);
    if (it != ptrs.end()) {
      (void)hipFree(p);
      ptrs.erase(it);
    }
  }
  ~Scratch() {
    for (void* p : ptrs) (void)hipFree(p);
  }
};

#define BD_TRY(x)                           \
  do {                                      \
    hipError_t e_ = (x);                    \
    if (e_ != hipSuccess) return e_;        \
  } while (0)

// stable sort of (key, perm) pairs by the low `bits` bits of key; keys/perm are double buffers
template <typename K>
hipError_t sort_pairs(Scratch& sc, rocprim::double_buffer<K>& keys, rocprim::double_buffer<uint32_t>& perm,
                      uint64_t n, unsigned bits, hipStream_t s) {
  size_t bytes = 0;
  BD_TRY(rocprim::radix_sort_pairs(nullptr, bytes, keys, perm, n, 0, bits, s));
  void* tmp = sc.alloc<uint8_t>(bytes);
  BD_TRY(sc.err);
  BD_TRY(rocprim::radix_sort_pairs(tmp, bytes, keys, perm, n, 0, bits, s));
  sc.release(tmp);
  return hipSuccess;
}

unsigned bits_for(uint64_t v) {   // bits to represent values in [0, v]
  unsigned b = 1;
  while (b < 64 && (v >> b)) ++b;
  return b;
}

}  // namespace

// Sorted unique values of `n` device int64s (the input is left unchanged) -> *out (hipMalloc'd,
// exactly *n_out entries).
hipError_t bd_sort_unique(const int64_t* d_in, uint64_t n, int64_t** out, uint64_t* n_out, hipStream_t s) {
  *out = nullptr;
  *n_out = 0;
  Scratch sc;
  int64_t* sorted = sc.alloc<int64_t>(n);
  int64_t* uniq = sc.alloc<int64_t>(n);
  uint64_t* cnt = sc.alloc<uint64_t>(1);
  BD_TRY(sc.err);
  uint64_t u = 0;
  if (n) {
    size_t bytes = 0;
    BD_TRY(rocprim::radix_sort_keys(nullptr, bytes, d_in, sorted, n, 0, 64, s));
    void* tmp = sc.alloc<uint8_t>(bytes);
    BD_TRY(sc.err);
    BD_TRY(rocprim::radix_sort_keys(tmp, bytes, d_in, sorted, n, 0, 64, s));
    sc.release(tmp);
    bytes = 0;
    BD_TRY(rocprim::unique(nullptr, bytes, sorted, uniq, cnt, n, rocprim::equal_to<int64_t>(), s));
    tmp = sc.alloc<uint8_t>(bytes);
    BD_TRY(sc.err);
    BD_TRY(rocprim::unique(tmp, bytes, sorted, uniq, cnt, n, rocprim::equal_to<int64_t>(), s));
    BD_TRY(hipMemcpyAsync(&u, cnt, 8, hipMemcpyDeviceToHost, s));
    BD_TRY(hipStreamSynchronize(s));
  }
  int64_t* res = nullptr;
  BD_TRY(hipMalloc((void**)&res, std::max<uint64_t>(u, 1) * 8));
  if (u) {
    hipError_t e = hipMemcpyAsync(res, uniq, u * 8, hipMemcpyDeviceToDevice, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) { (void)hipFree(res); return e; }
  }
  *out = res;
  *n_out = u;
  return hipSuccess;
}

hipError_t bd_home(int32_t* d_home, const int64_t* d_src, const int32_t* part, uint64_t n, const int64_t* d_dict,
                   uint64_t nv, int32_t parts, bool* split, hipStream_t s) {
  *split = false;
  if (!n) return hipSuccess;
  Scratch sc;
  uint32_t* sd = sc.alloc<uint32_t>(n);
  unsigned* flag = sc.alloc<unsigned>(1);
  int32_t* d_part = part ? sc.alloc<int32_t>(n) : nullptr;
  BD_TRY(sc.err);
  if (part) BD_TRY(hipMemcpyAsync(d_part, part, n * 4, hipMemcpyHostToDevice, s));
  BD_TRY(hipMemsetAsync(flag, 0, 4, s));
  k_dense<<<grid_for(n), BT, 0, s>>>(sd, d_src, n, d_dict, nv);
  k_home<<<grid_for(n), BT, 0, s>>>(d_home, sd, d_src, d_part, n, parts, flag);
  BD_TRY(hipGetLastError());
  unsigned h = 0;
  BD_TRY(hipMemcpyAsync(&h, flag, 4, hipMemcpyDeviceToHost, s));
  BD_TRY(hipStreamSynchronize(s));
  *split = h != 0;
  return hipSuccess;
}

hipError_t bd_build_type(const TypeBuildIn& in, const GidMap& gm, hipStream_t s, DevEdgeType* out, uint64_t* bytes_out,
                         std::string* err) {
  const uint64_t n = in.n;
  const uint64_t nv = gm.nv;
  *bytes_out = 0;
  if (n >= 0xFFFFFFFFull) {
    *err = "more than 2^32-1 staged records of one edge type on one GPU";
    return hipErrorInvalidValue;
  }
  Scratch sc;
  // ---- 1. dense source ids, the permutation sort
  uint32_t* sd = sc.alloc<uint32_t>(n);
  uint32_t* perm0 = sc.alloc<uint32_t>(n);
  uint32_t* perm1 = sc.alloc<uint32_t>(n);
  uint64_t* key0 = sc.alloc<uint64_t>(n);
  uint64_t* key1 = sc.alloc<uint64_t>(n);
  int64_t* dst = sc.alloc<int64_t>(n);
  int64_t* rank = in.rank ? sc.alloc<int64_t>(n) : nullptr;
  BD_TRY(sc.err);
  if (n) {
    k_dense<<<grid_for(n), BT, 0, s>>>(sd, in.d_src, n, gm.dict, nv);
    BD_TRY(hipMemcpyAsync(dst, in.dst, n * 8, hipMemcpyHostToDevice, s));
    if (rank) BD_TRY(hipMemcpyAsync(rank, in.rank, n * 8, hipMemcpyHostToDevice, s));
    k_iota_desc<<<grid_for(n), BT, 0, s>>>(perm0, n);
    BD_TRY(hipGetLastError());
  }
  rocprim::double_buffer<uint32_t> perm(perm0, perm1);
  rocprim::double_buffer<uint64_t> keys(key0, key1);
  uint64_t* ver_keep = nullptr;
  if (n && in.verkey) {   // version bytes (BE), ascending = newest first
    uint64_t* ver = sc.alloc<uint64_t>(n);
    BD_TRY(sc.err);
    BD_TRY(hipMemcpyAsync(ver, in.verkey, n * 8, hipMemcpyHostToDevice, s));
    k_gather_key<false><<<grid_for(n), BT, 0, s>>>(keys.current(), ver, perm.current(), n);
    BD_TRY(sort_pairs(sc, keys, perm, n, 64, s));
    ver_keep = ver;   // (the superseded versions are told apart by it below)
  }
  if (n) {   // dst bytes LE, compared as memcmp = bswap64 as unsigned
    k_gather_key<true><<<grid_for(n), BT, 0, s>>>(keys.current(), reinterpret_cast<const uint64_t*>(dst),
                                                  perm.current(), n);
    BD_TRY(sort_pairs(sc, keys, perm, n, 64, s));
  }
  if (n && rank) {
    k_gather_key<true><<<grid_for(n), BT, 0, s>>>(keys.current(), reinterpret_cast<const uint64_t*>(rank),
                                                  perm.current(), n);
    BD_TRY(sort_pairs(sc, keys, perm, n, 64, s));
  }
  // dense source id: 32-bit keys in the key buffers
  rocprim::double_buffer<uint32_t> skeys(reinterpret_cast<uint32_t*>(keys.current()),
                                         reinterpret_cast<uint32_t*>(keys.alternate()));
  if (n) {
    k_gather_u32<<<grid_for(n), BT, 0, s>>>(skeys.current(), sd, perm.current(), n);
    BD_TRY(sort_pairs(sc, skeys, perm, n, bits_for(nv), s));
  }
  sc.release(sd);
  const uint32_t* sd_sorted = skeys.current();
  // ---- 2. live flags -> positions
  uint32_t* live = reinterpret_cast<uint32_t*>(skeys.alternate());
  uint32_t* pos = sc.alloc<uint32_t>(n);
  BD_TRY(sc.err);
  uint32_t E = 0;
  if (n) {
    k_live<<<grid_for(n), BT, 0, s>>>(live, sd_sorted, perm.current(), dst, rank, n);
    size_t bytes = 0;
    BD_TRY(rocprim::exclusive_scan(nullptr, bytes, live, pos, 0u, n, rocprim::plus<uint32_t>(), s));
    void* tmp = sc.alloc<uint8_t>(bytes);
    BD_TRY(sc.err);
    BD_TRY(rocprim::exclusive_scan(tmp, bytes, live, pos, 0u, n, rocprim::plus<uint32_t>(), s));
    uint32_t tail[2];
    BD_TRY(hipMemcpyAsync(&tail[0], pos + n - 1, 4, hipMemcpyDeviceToHost, s));
    BD_TRY(hipMemcpyAsync(&tail[1], live + n - 1, 4, hipMemcpyDeviceToHost, s));
    BD_TRY(hipStreamSynchronize(s));
    sc.release(tmp);
    E = tail[0] + tail[1];
  }
  // ---- 3. CSR arrays
  DevEdgeType& dt = *out;
  dt.num_edges = E;
  uint64_t dev = 0;
  auto keep = [&](void** p, uint64_t b) -> hipError_t {
    dev += std::max<uint64_t>(b, 8);
    return hipMalloc(p, std::max<uint64_t>(b, 8));
  };
  BD_TRY(keep((void**)&dt.row_ptr, (nv + 1) * 4));
  BD_TRY(keep((void**)&dt.col, (uint64_t)E * 4));
  BD_TRY(keep((void**)&dt.dst_vid, (uint64_t)E * 8));
  if (rank) BD_TRY(keep((void**)&dt.rank, (uint64_t)E * 8));
  if (in.valid) BD_TRY(keep((void**)&dt.valid, E));
  dt.props.assign(in.nprops, nullptr);
  for (int c = 0; c < in.nprops; ++c) BD_TRY(keep((void**)&dt.props[c], (uint64_t)E * 8));
  k_row_ptr<<<grid_for(nv + 1), BT, 0, s>>>(dt.row_ptr, sd_sorted, pos, n, nv, E);
  BD_TRY(hipGetLastError());
  // staged columns on the device (one at a time would cap memory; all at once keeps one emit pass)
  std::vector<int64_t*> pin(in.nprops, nullptr);
  for (int c = 0; c < in.nprops; ++c) {
    pin[c] = sc.alloc<int64_t>(n);
    BD_TRY(sc.err);
    if (n) BD_TRY(hipMemcpyAsync(pin[c], in.props[c], n * 8, hipMemcpyHostToDevice, s));
  }
  uint8_t* valid = in.valid ? sc.alloc<uint8_t>(n) : nullptr;
  int64_t** d_pin = sc.alloc<int64_t*>(std::max(in.nprops, 1));
  int64_t** d_pout = sc.alloc<int64_t*>(std::max(in.nprops, 1));
  unsigned* flags = sc.alloc<unsigned>(1);
  BD_TRY(sc.err);
  if (valid && n) BD_TRY(hipMemcpyAsync(valid, in.valid, n, hipMemcpyHostToDevice, s));
  if (in.nprops) {
    BD_TRY(hipMemcpyAsync(d_pin, pin.data(), in.nprops * 8, hipMemcpyHostToDevice, s));
    BD_TRY(hipMemcpyAsync(d_pout, dt.props.data(), in.nprops * 8, hipMemcpyHostToDevice, s));
  }
  BD_TRY(hipMemsetAsync(flags, 0, 4, s));
  if (n) {
    EmitArgs a{};
    a.perm = perm.current();
    a.live = live;
    a.pos = pos;
    a.dst = dst;
    a.rank = rank;
    a.valid = valid;
    a.pin = d_pin;
    a.pout = d_pout;
    a.nprops = in.nprops;
    a.col = dt.col;
    a.dvid = dt.dst_vid;
    a.rank_out = dt.rank;
    a.valid_out = dt.valid;
    a.g = gm;
    a.flags = flags;
    k_emit<<<grid_for(n), BT, 0, s>>>(a, n);
    BD_TRY(hipGetLastError());
  }
  unsigned fl = 0;
  BD_TRY(hipMemcpyAsync(&fl, flags, 4, hipMemcpyDeviceToHost, s));
  dt.h_row_ptr.resize(nv + 1);
  BD_TRY(hipMemcpyAsync(dt.h_row_ptr.data(), dt.row_ptr, (nv + 1) * 4, hipMemcpyDeviceToHost, s));
  BD_TRY(hipStreamSynchronize(s));
  if (dt.rank && !(fl & 1)) {   // every live rank is 0: no rank column
    (void)hipFree(dt.rank);
    dt.rank = nullptr;
    dev -= std::max<uint64_t>((uint64_t)E * 8, 8);
  }
  if (dt.valid && !(fl & 2)) {
    (void)hipFree(dt.valid);
    dt.valid = nullptr;
    dev -= std::max<uint64_t>(E, 8);
  }
  // ---- 3b. superseded versions (multi-version data): their own CSR, each tagged with its group
  if (ver_keep && n > 1) {
    uint32_t* oflag = sc.alloc<uint32_t>(n);
    uint32_t* opos = sc.alloc<uint32_t>(n);
    BD_TRY(sc.err);
    BD_TRY(hipMemsetAsync(oflag, 0, 4, s));
    k_old<<<grid_for(n - 1), BT, 0, s>>>(oflag + 1, live + 1, perm.current() + 1, ver_keep, n - 1);
    BD_TRY(hipGetLastError());
    size_t bytes = 0;
    BD_TRY(rocprim::exclusive_scan(nullptr, bytes, oflag, opos, 0u, n, rocprim::plus<uint32_t>(), s));
    void* tmp = sc.alloc<uint8_t>(bytes);
    BD_TRY(sc.err);
    BD_TRY(rocprim::exclusive_scan(tmp, bytes, oflag, opos, 0u, n, rocprim::plus<uint32_t>(), s));
    uint32_t tail[2];
    BD_TRY(hipMemcpyAsync(&tail[0], opos + n - 1, 4, hipMemcpyDeviceToHost, s));
    BD_TRY(hipMemcpyAsync(&tail[1], oflag + n - 1, 4, hipMemcpyDeviceToHost, s));
    BD_TRY(hipStreamSynchronize(s));
    sc.release(tmp);
    const uint32_t NO = tail[0] + tail[1];
    if (NO) {
      auto* od = new DevEdgeType();
      dt.old = od;
      od->type = dt.type;
      od->num_edges = NO;
      BD_TRY(keep((void**)&od->row_ptr, (nv + 1) * 4));
      BD_TRY(keep((void**)&od->col, (uint64_t)NO * 4));
      BD_TRY(keep((void**)&od->dst_vid, (uint64_t)NO * 8));
      if (dt.rank) BD_TRY(keep((void**)&od->rank, (uint64_t)NO * 8));
      if (in.valid) BD_TRY(keep((void**)&od->valid, NO));
      od->props.assign(in.nprops, nullptr);
      for (int c = 0; c < in.nprops; ++c) BD_TRY(keep((void**)&od->props[c], (uint64_t)NO * 8));
      uint32_t* grp = sc.alloc<uint32_t>(NO);
      BD_TRY(sc.err);
      k_row_ptr<<<grid_for(nv + 1), BT, 0, s>>>(od->row_ptr, sd_sorted, opos, n, nv, NO);
      if (in.nprops) BD_TRY(hipMemcpyAsync(d_pout, od->props.data(), in.nprops * 8, hipMemcpyHostToDevice, s));
      EmitArgs a{};
      a.perm = perm.current();
      a.live = oflag;
      a.pos = opos;
      a.dst = dst;
      a.rank = dt.rank ? rank : nullptr;
      a.valid = valid;
      a.pin = d_pin;
      a.pout = d_pout;
      a.nprops = in.nprops;
      a.col = od->col;
      a.dvid = od->dst_vid;
      a.rank_out = od->rank;
      a.valid_out = od->valid;
      a.g = gm;
      a.flags = flags;
      a.gpos = pos;
      a.grp = grp;
      k_emit<<<grid_for(n), BT, 0, s>>>(a, n);
      BD_TRY(hipGetLastError());
      od->h_row_ptr.resize(nv + 1);
      od->h_grp.resize(NO);
      BD_TRY(hipMemcpyAsync(od->h_row_ptr.data(), od->row_ptr, (nv + 1) * 4, hipMemcpyDeviceToHost, s));
      BD_TRY(hipMemcpyAsync(od->h_grp.data(), grp, (uint64_t)NO * 4, hipMemcpyDeviceToHost, s));
      od->narrow.assign(in.nprops, nullptr);
      od->narrow_bytes.assign(in.nprops, 0);
      od->prop_kind = dt.prop_kind;
      if (in.nprops) BD_TRY(keep((void**)&od->d_props, (uint64_t)in.nprops * 8));
      if (in.nprops) BD_TRY(hipMemcpyAsync(od->d_props, od->props.data(), in.nprops * 8, hipMemcpyHostToDevice, s));
      BD_TRY(hipStreamSynchronize(s));
      uint32_t md = 0;
      for (uint64_t d = 0; d < nv; ++d) md = std::max(md, od->h_row_ptr[d + 1] - od->h_row_ptr[d]);
      od->max_degree = (int)md;
    }
  }
  // ---- 4. narrow copies of INT columns (read by the final-step fast path)
  dt.narrow.assign(in.nprops, nullptr);
  dt.narrow_bytes.assign(in.nprops, 0);
  for (int c = 0; c < in.nprops && E; ++c) {
    if (in.kinds[c] != VK_INT) continue;
    int64_t* mm = sc.alloc<int64_t>(2);
    BD_TRY(sc.err);
    size_t bytes = 0;
    BD_TRY(rocprim::reduce(nullptr, bytes, dt.props[c], mm, INT64_MAX, E, rocprim::minimum<int64_t>(), s));
    void* tmp = sc.alloc<uint8_t>(bytes);
    BD_TRY(sc.err);
    BD_TRY(rocprim::reduce(tmp, bytes, dt.props[c], mm, INT64_MAX, E, rocprim::minimum<int64_t>(), s));
    BD_TRY(rocprim::reduce(tmp, bytes, dt.props[c], mm + 1, INT64_MIN, E, rocprim::maximum<int64_t>(), s));
    int64_t h[2];
    BD_TRY(hipMemcpyAsync(h, mm, 16, hipMemcpyDeviceToHost, s));
    BD_TRY(hipStreamSynchronize(s));
    sc.release(tmp);
    int w = 8;
    if (h[0] >= INT8_MIN && h[1] <= INT8_MAX) w = 1;
    else if (h[0] >= INT16_MIN && h[1] <= INT16_MAX) w = 2;
    else if (h[0] >= INT32_MIN && h[1] <= INT32_MAX) w = 4;
    if (w == 8) continue;
    BD_TRY(keep(&dt.narrow[c], (uint64_t)E * w));
    if (w == 1) k_narrow<int8_t><<<grid_for(E), BT, 0, s>>>((int8_t*)dt.narrow[c], dt.props[c], E);
    else if (w == 2) k_narrow<int16_t><<<grid_for(E), BT, 0, s>>>((int16_t*)dt.narrow[c], dt.props[c], E);
    else k_narrow<int32_t><<<grid_for(E), BT, 0, s>>>((int32_t*)dt.narrow[c], dt.props[c], E);
    BD_TRY(hipGetLastError());
    dt.narrow_bytes[c] = w;
  }
  if (in.nprops) BD_TRY(keep((void**)&dt.d_props, (uint64_t)in.nprops * 8));
  if (in.nprops) BD_TRY(hipMemcpyAsync(dt.d_props, dt.props.data(), in.nprops * 8, hipMemcpyHostToDevice, s));
  BD_TRY(hipStreamSynchronize(s));
  uint32_t md = 0;
  for (uint64_t d = 0; d < nv; ++d) md = std::max(md, dt.h_row_ptr[d + 1] - dt.h_row_ptr[d]);
  dt.max_degree = (int)md;
  *bytes_out = dev;
  return hipSuccess;
}

}  // namespace nbg
