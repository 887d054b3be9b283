// nebula_amd — gfx950 (CDNA4) kernels for the GO N STEPS / FIND PATH hot path (this file: the GO
// pipeline, YIELD DISTINCT, the partitioned exchange, FIND SHORTEST PATH's host-driven levels;
// final.hip: the lean final step; walk.hip: FIND ALL PATH; spchain.hip: the one-pair SHORTEST
// chain; ws.h: the query slot's workspace).
//
// A query is enqueued on the workspace stream with NO host synchronisation until its end:
// every size the kernels need (frontier size n, edges of the current expansion, next frontier
// size) lives in a device-resident QState and grids are sized from host-known upper bounds.
//
// Per hop over one edge type (CSR):
//   k_relist      the start list's entries with edges, their degree prefix, row starts and the
//                 merge-path split of every tile (one packed atomic per workgroup: no scan pass)
//   k_expand<M>   persistent, load-balanced expansion over merge-path tiles: a tile owns TILE
//                 path items (frontier entries + edges) whatever the degree skew; its split is
//                 read from the list, items are striped across lanes so neighbour / property
//                 reads are coalesced.
//                 M = MARK  (steps 1..N-1: claim each neighbour for the step's SET and append the
//                           winners, with their edge space over the next step, to the next list)
//                 M = FINAL (step N: WHERE/YIELD per edge, rows appended to the workgroup's own
//                           region: no global atomics; `col <cmp> const` / leaf-yield programs skip
//                           the interpreter, and the dominant shape runs k_final_dst, final.hip)
// A prepared GO 3 STEPS query over one edge type is three launches: MARK, MARK, FINAL.
// Semantics follow QueryBaseProcessor::collectEdgeProps (version de-dup is done at load,
// neighbours are in memcmp key order, the cap counts edges in that order) and
// GoExecutor::getDstIdsFromResp (per-step dst SET, no global visited set).
#include <hip/hip_runtime.h>
#include <array>
#include <cstddef>

#include <cstdio>
#include <cstring>
#include <vector>

#include "ws.h"

namespace nbg {


// ----------------------------------------------------------------------------- frontier lists
// Every frontier list an expansion consumes is produced together with its edge space: entry i
// owns edges [seg_end[i] - deg_i, seg_end[i]) (deg capped by max_edge_returned_per_vertex), row
// start seg_rs[i], and the merge-path split of every TILE boundary it covers (tsplit).  List
// positions and edge offsets are handed out per workgroup by ONE 64-bit atomicAdd on a packed
// accumulator (count << 32 | degree sum): no separate scan pass, no fences, no grid barrier.
// Lists are therefore in workgroup-arrival order (id order inside a workgroup); frontier order
// is irrelevant to GoExecutor's semantics (a per-step SET, GoExecutor.cpp:501-541).
// The degree sum fits the low word: a step's frontier is a set (Σ deg <= E < 2^32 per type) and
// the host checks the start list (which keeps duplicates) before launching.
struct DegSrc {                    // the CSR whose degrees the list carries (row_ptr null: none)
  const uint32_t* row_ptr;
  const uint8_t* visible;
  uint32_t cap;
};

struct ListOut {
  uint32_t* ids;
  uint32_t* seg_end;               // inclusive degree prefix (global)
  uint32_t* seg_rs;                // row start
  uint32_t* tsplit;                // merge-path split per tile
  unsigned long long* acc;         // packed (entries << 32 | edges); zero before the launch
  unsigned long long* zero_next;   // the other accumulator of the ping-pong pair, zeroed here
  unsigned long long* stat_n;      // frontier size of this step (input count), nullable
};

__device__ __forceinline__ uint32_t vdeg(const DegSrc& ds, uint32_t v, uint32_t* rs) {
  if (!ds.row_ptr || v == NO_ROW || (ds.visible && !ds.visible[v])) { *rs = 0; return 0; }
  const uint32_t r = ds.row_ptr[v];
  const uint32_t d = ds.row_ptr[v + 1] - r;
  *rs = r;
  return d < ds.cap ? d : ds.cap;
}

// Entry i owns merge-path positions [i + start_i, i + end_i] (its edges, then its terminator);
// the split of tile t (entries consumed before position t * TILE) is the entry whose range holds
// t * TILE, so each entry records the tile boundaries it covers and k_expand reads its split.
// An entry covering up to SPLITS_SOLO boundaries writes them itself; a hub's (one boundary per
// 256 edges: a vertex of degree 10^6 covers ~4000) are left in [*t0, *t1) for wave_splits, which
// spreads them over the wave's lanes — one lane storing them serially cost a claim-mode MARK step
// ~40 us whenever the claimed set held a hub (RMAT-26 step 2: 50-60 us for 292 claims or 282 k).
constexpr uint64_t SPLITS_SOLO = 4;
__device__ __forceinline__ void record_splits(uint32_t* tsplit, uint32_t i, uint32_t end_incl, uint32_t deg,
                                              uint64_t* t0, uint64_t* t1) {
  const uint64_t lo = (uint64_t)i + end_incl - deg, hi = (uint64_t)i + end_incl;
  const uint64_t a = (lo + TILE - 1) / TILE, b = hi / TILE + 1;
  if (b - a <= SPLITS_SOLO) {
    for (uint64_t t = a; t < b; ++t) tsplit[t] = i;
    return;
  }
  *t0 = a;
  *t1 = b;
}

// The hub boundaries of one round of list_put calls (every lane of the wave takes part; a lane
// without an entry passes t0 == t1): each hub's boundaries are stored lane-strided by the wave.
__device__ __forceinline__ void wave_splits(uint32_t* tsplit, uint64_t t0, uint64_t t1, uint32_t pos) {
  unsigned long long bm = __ballot(t1 > t0);
  const uint64_t lane = threadIdx.x & 63;
  while (bm) {
    const int l = __ffsll((long long)bm) - 1;
    bm &= bm - 1;
    const uint64_t a = __shfl(t0, l, 64), b = __shfl(t1, l, 64);
    const uint32_t p = __shfl(pos, l, 64);
    for (uint64_t t = a + lane; t < b; t += 64) tsplit[t] = p;
  }
}

// Block-wide reservation: exclusive per-thread offsets (*pc list position, *pd edge offset).
template <int NT>
__device__ __forceinline__ void reserve(uint32_t c, uint32_t d, unsigned long long* acc, uint32_t* pc, uint32_t* pd) {
  __shared__ uint32_t lds[NT / 64];
  __shared__ unsigned long long s_old;
  uint32_t tc, td;
  const uint32_t xc = block_excl_scan<NT>(c, &tc, lds);
  const uint32_t xd = block_excl_scan<NT>(d, &td, lds);
  if (threadIdx.x == 0) s_old = (tc | td) ? atomicAdd(acc, ((unsigned long long)tc << 32) | td) : 0ull;
  __syncthreads();
  *pc = (uint32_t)(s_old >> 32) + xc;
  *pd = (uint32_t)s_old + xd;
}

// One list entry; a hub's tile boundaries come back in [*t0, *t1) for wave_splits (t0 == t1 else).
__device__ __forceinline__ void list_put(const ListOut& o, const DegSrc& ds, uint32_t pos, uint32_t v, uint32_t* pd,
                                         uint32_t dg, uint32_t rs, uint64_t* t0, uint64_t* t1) {
  o.ids[pos] = v;
  if (ds.row_ptr) {
    *pd += dg;
    o.seg_end[pos] = *pd;
    o.seg_rs[pos] = rs;
    record_splits(o.tsplit, pos, *pd, dg, t0, t1);
  }
}

// k_relist: a list (start ids, an earlier list, a FIND PATH frontier) -> the list of its entries
// with edges over one CSR.  Entries without edges are dropped (they expand to nothing).
constexpr int RL_ITEMS = 8;
constexpr int RL_TILE = BLOCK * RL_ITEMS;
// Input count: *in_n (packed when in_packed), or n_val when in_n is null; ids: in[], or the
// start ids inside the kernel arguments when in is null (n_val <= INLINE_STARTS).
__global__ void __launch_bounds__(BLOCK) k_relist(const uint32_t* __restrict__ in, const unsigned long long* in_n,
                                                  int in_packed, uint32_t n_val, InlineIds inl, DegSrc ds, ListOut o,
                                                  unsigned long long* reset) {
  __shared__ uint32_t sIn[INLINE_STARTS];
  const uint64_t n = in_n ? (in_packed ? (*in_n >> 32) : *in_n) : n_val;
  if (!in) {   // uniform: stage the inline ids (constant indices only, no scratch)
#pragma unroll
    for (int k = 0; k < INLINE_STARTS; ++k)
      if (threadIdx.x == k) sIn[k] = inl.id[k];
    __syncthreads();
  }
  if (blockIdx.x == 0) {
    if (threadIdx.x == 0) {
      *o.zero_next = 0;
      if (o.stat_n) *o.stat_n = n;
    }
    if (reset && threadIdx.x == 0) *reset = 0;   // the length of the list the expansion appends to
  }
  const uint64_t base = (uint64_t)blockIdx.x * RL_TILE + (uint64_t)threadIdx.x * RL_ITEMS;
  if ((uint64_t)blockIdx.x * RL_TILE >= n) return;
  uint32_t v[RL_ITEMS], dg[RL_ITEMS], rs[RL_ITEMS];
  uint32_t c = 0, d = 0;
#pragma unroll
  for (int k = 0; k < RL_ITEMS; ++k) {
    v[k] = base + k < n ? (in ? in[base + k] : sIn[base + k]) : NO_ROW;
    dg[k] = vdeg(ds, v[k], &rs[k]);
    c += dg[k] ? 1u : 0u;
    d += dg[k];
  }
  uint32_t pc, pd;
  reserve<BLOCK>(c, d, o.acc, &pc, &pd);
#pragma unroll
  for (int k = 0; k < RL_ITEMS; ++k) {
    uint64_t t0 = 0, t1 = 0;
    const uint32_t p = pc;
    if (dg[k]) list_put(o, ds, pc++, v[k], &pd, dg[k], rs[k], &t0, &t1);
    wave_splits(o.tsplit, t0, t1, p);
  }
}

// k_compact: next frontier = the byte flags set by k_expand<MARK> (the per-step dst SET),
// listed with the degrees of the next step's first OVER type; clears the flags.  Every flagged
// vertex is kept (this list is the frontier for every OVER type).  16 flag bytes per thread,
// their degree gathers all in flight at once.
constexpr int CP_THREADS = 1024;
constexpr int CP_BYTES = CP_THREADS * 16;        // flag bytes per workgroup
__global__ void __launch_bounds__(CP_THREADS) k_compact(uint8_t* __restrict__ flags, DegSrc ds, ListOut o) {
  if (blockIdx.x == 0 && threadIdx.x == 0) *o.zero_next = 0;
  const uint64_t off = (uint64_t)blockIdx.x * CP_BYTES + (uint64_t)threadIdx.x * 16;
  uint4* p = reinterpret_cast<uint4*>(flags + off);
  const uint4 q = *p;
  const uint32_t ws[4] = {q.x, q.y, q.z, q.w};
  uint32_t c = 0, d = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) c += __popc(ws[j] & 0x01010101u);
  uint32_t dg[16], rs[16];
#pragma unroll
  for (int b = 0; b < 16; ++b) {
    const bool set = (ws[b >> 2] >> ((b & 3) * 8)) & 1u;
    dg[b] = set ? vdeg(ds, (uint32_t)(off + b), &rs[b]) : 0u;
    d += dg[b];
  }
  uint32_t pc, pd;
  reserve<CP_THREADS>(c, d, o.acc, &pc, &pd);
#pragma unroll
  for (int b = 0; b < 16; ++b) {   // (every lane: wave_splits is wave-wide)
    uint64_t t0 = 0, t1 = 0;
    const uint32_t pp = pc;
    if ((ws[b >> 2] >> ((b & 3) * 8)) & 1u) list_put(o, ds, pc++, (uint32_t)(off + b), &pd, dg[b], rs[b], &t0, &t1);
    wave_splits(o.tsplit, t0, t1, pp);
  }
  *p = make_uint4(0, 0, 0, 0);
}

// Fast path for the common final-step program shape: WHERE absent or `col <cmp> const` on an
// INT column, YIELD columns that are plain edge fields / key props / constants.  No
// interpreter, no LDS registers; the generic bytecode path handles everything else.
__device__ __forceinline__ int64_t load_col(const void* p, int bytes, uint32_t j) {
  switch (bytes) {   // uniform
    case 1: return reinterpret_cast<const int8_t*>(p)[j];
    case 2: return reinterpret_cast<const int16_t*>(p)[j];
    case 4: return reinterpret_cast<const int32_t*>(p)[j];
    default: return reinterpret_cast<const int64_t*>(p)[j];
  }
}

// VT loads of a column of type T (sign-extended), all in flight at once
template <typename T, int V = VT>
__device__ __forceinline__ void load_narrow(const void* p, const uint32_t* jj, int nb, int lane, int64_t* x) {
  const T* c = reinterpret_cast<const T*>(p);
#pragma unroll
  for (int i = 0; i < V; ++i) x[i] = (i * 64 + lane < nb) ? (int64_t)c[jj[i]] : 0;
}

struct FastProg {
  int enabled;
  int has_where;
  int where_neg;           // pass = (lo <= x && x <= hi) != where_neg   (branch-free `col <op> const`)
  int64_t lo, hi;
  const void* wcol;        // WHERE column (device pointer, resolved on the host) ...
  int wbytes;              // ... at this width (1/2/4: narrow copy of an INT column; 8)
  int ykind[MAX_YIELDS];   // 0 DST, 1 SRC, 2 RANK, 3 COL, 4 CONST, 5 the edge's CSR index
  const void* ycol[MAX_YIELDS];
  int ybytes[MAX_YIELDS];
  int dst_yield;           // some YIELD is _dst
};

// ----------------------------------------------------------------------------- bytecode
struct EdgeCtx {
  uint64_t j;       // edge index in CSR
  uint32_t v;       // source dense id
};

__device__ __forceinline__ double as_f(int64_t x) { return __longlong_as_double(x); }
__device__ __forceinline__ int64_t fbits(double d) { return __double_as_longlong(d); }

// ----------------------------------------------------------------------------- derived strings
// A piece list (exprc.cpp emit_pieces) streamed byte by byte: dictionary strings from the
// snapshot's string bytes, constants from the program's data, INT pieces as decimal digits
// computed in place (no per-lane buffer), BOOL pieces as "true" / "false".
__constant__ unsigned long long kPow10[20] = {1ull, 10ull, 100ull, 1000ull, 10000ull, 100000ull, 1000000ull,
                                              10000000ull, 100000000ull, 1000000000ull, 10000000000ull,
                                              100000000000ull, 1000000000000ull, 10000000000000ull,
                                              100000000000000ull, 1000000000000000ull, 10000000000000000ull,
                                              100000000000000000ull, 1000000000000000000ull,
                                              10000000000000000000ull};
__constant__ char kTrueFalse[10] = "truefalse";

struct PieceView {
  const char* p;     // the bytes, or nullptr: the decimal of u (negative when neg)
  uint64_t u;
  uint32_t len;
  uint32_t nd, neg;
};

__device__ __forceinline__ PieceView piece_view(const Ins& pc, const char* dbase, const DevStrings& S,
                                                const int64_t* regs, int tid, bool& bad) {
  PieceView v{dbase, 0, 0, 0, 0};
  const int64_t x = regs[pc.d * BLOCK + tid];
  switch (pc.op) {
    case PC_DICT:
      // -1: "" absent from the dictionary (the schema default of a string prop)
      if (((uint64_t)x >> 60) == 1) {   // a string materialised in the arena (OP_SMAT)
        const uint64_t at = (uint64_t)(x & (STR_ARENA - 1));
        if (!S.arena || at + 16 > S.arena_cap) {
          bad = true;
        } else {
          v.p = S.arena + at + 16;
          v.len = (uint32_t)*reinterpret_cast<const uint64_t*>(S.arena + at + 8);
        }
      } else if (((uint64_t)x >> 61) == 1) {   // (is_input_code) an input string absent from the dictionary (STR_INPUT | index)
        const uint64_t i = (uint64_t)(x & (STR_INPUT - 1));
        if (i >= S.xn) {
          bad = true;
        } else {
          v.p = S.xbytes + S.xoff[i];
          v.len = S.xoff[i + 1] - S.xoff[i];
        }
      } else if (x != -1) {
        if (x < 0 || (x & 1) || (uint64_t)(x >> 1) >= S.n) {
          bad = true;
        } else {
          const uint64_t i = (uint64_t)x >> 1;
          v.p = S.bytes + S.off[i];
          v.len = S.off[i + 1] - S.off[i];
        }
      }
      break;
    case PC_CONST: v.p = dbase + pc.aux; v.len = (uint32_t)pc.imm; break;
    case PC_BOOL: v.p = kTrueFalse + (x ? 0 : 4); v.len = x ? 4u : 5u; break;
    case PC_VIEW: bad = true; break;   // (a view inside a flat list: never emitted)
    default: {   // PC_INT: folly::to<std::string>(int64_t)
      v.p = nullptr;
      v.neg = x < 0;
      v.u = v.neg ? 0ull - (uint64_t)x : (uint64_t)x;
      uint32_t nd = 1;
      while (nd < 20 && v.u >= kPow10[nd]) ++nd;
      v.nd = nd;
      v.len = nd + v.neg;
    }
  }
  return v;
}

__device__ __forceinline__ uint32_t piece_byte(const PieceView& v, uint32_t i) {
  if (v.p) return (uint8_t)v.p[i];
  if (v.neg) {
    if (!i) return '-';
    --i;
  }
  return '0' + (uint32_t)((v.u / kPow10[v.nd - 1 - i]) % 10);
}

// A flat piece list (no views): the inner list of a view, a pad list
struct FlatIter {
  const Ins* list;   // the pieces
  const char* dbase;
  int n, k;
  uint32_t i;
  PieceView v;
};

__device__ __forceinline__ void flat_open(FlatIter& it, const Ins* data, int32_t hdr, const DevStrings& S,
                                          const int64_t* regs, int tid, bool& bad) {
  const Ins h = data[hdr];
  it.list = data + h.aux;
  it.dbase = reinterpret_cast<const char*>(data);
  it.n = h.d;
  it.k = 0;
  it.i = 0;
  it.v = PieceView{it.dbase, 0, 0, 0, 0};
  if (it.n) it.v = piece_view(it.list[0], it.dbase, S, regs, tid, bad);
}

// the next byte (-1 at the end)
__device__ __forceinline__ int flat_next(FlatIter& it, const DevStrings& S, const int64_t* regs, int tid, bool& bad) {
  while (it.i >= it.v.len) {
    if (++it.k >= it.n) return -1;
    it.v = piece_view(it.list[it.k], it.dbase, S, regs, tid, bad);
    it.i = 0;
  }
  return (int)piece_byte(it.v, it.i++);
}

__device__ void flat_skip(FlatIter& it, uint64_t m, const DevStrings& S, const int64_t* regs, int tid, bool& bad) {
  while (m) {
    if (it.i < it.v.len) {
      const uint32_t d = (uint64_t)(it.v.len - it.i) < m ? it.v.len - it.i : (uint32_t)m;
      it.i += d;
      m -= d;
    } else {
      if (++it.k >= it.n) return;
      it.v = piece_view(it.list[it.k], it.dbase, S, regs, tid, bad);
      it.i = 0;
    }
  }
}

__device__ uint64_t flat_len(const Ins* data, int32_t hdr, const DevStrings& S, const int64_t* regs, int tid,
                             bool& bad) {
  const Ins h = data[hdr];
  uint64_t n = 0;
  for (int k = 0; k < h.d; ++k) n += piece_view(data[h.aux + k], reinterpret_cast<const char*>(data), S, regs, tid, bad).len;
  return n;
}

// byte m of a flat list (a pad: read cyclically, one piece walk per byte; pads are short)
__device__ uint32_t flat_byte_at(const Ins* data, int32_t hdr, uint64_t m, const DevStrings& S, const int64_t* regs,
                                 int tid, bool& bad) {
  const Ins h = data[hdr];
  for (int k = 0; k < h.d; ++k) {
    const PieceView v = piece_view(data[h.aux + k], reinterpret_cast<const char*>(data), S, regs, tid, bad);
    if (m < v.len) return piece_byte(v, (uint32_t)m);
    m -= v.len;
  }
  return 0;
}

// A PC_VIEW piece (FunctionManager.cpp:249-409 over its inner list's bytes, L of them): `pre` pad
// bytes, the inner bytes [w0, w0 + mid) case-mapped, `post` pad bytes.  The reference's failures
// (lpad / rpad to a negative length: a size_t that never stops padding; an empty pad) and results
// over 2^31 bytes set `bad` (an evaluation error).
struct ViewGeom {
  uint64_t w0, pre, mid, post, padlen;
  uint32_t cs;   // the inner bytes: 0 as is, 1 tolower, 2 toupper ("C" locale: ASCII letters)
  uint32_t oc;   // every byte, pads included (an outer lower / upper over this view)
};

__device__ ViewGeom view_geom(const Ins& pc, const Ins* data, const DevStrings& S, const int64_t* regs, int tid,
                              bool& bad) {
  ViewGeom g{0, 0, 0, 0, 0, (uint32_t)(pc.imm >> 32) & 3u, (uint32_t)(pc.imm >> 34) & 3u};
  const uint64_t L = flat_len(data, pc.aux, S, regs, tid, bad);
  const int32_t padh = (int32_t)(pc.imm & 0xFFFFFFFFll);
  const int64_t na = regs[pc.d * BLOCK + tid], nb = regs[pc.b * BLOCK + tid];
  g.mid = L;
  switch (pc.a) {
    case VF_LOWER: g.cs = 1; break;
    case VF_UPPER: g.cs = 2; break;
    case VF_TRIM:
    case VF_LTRIM:
    case VF_RTRIM: {   // find_first_not_of(" ") / find_last_not_of(" ") + 1
      FlatIter it;
      flat_open(it, data, pc.aux, S, regs, tid, bad);
      uint64_t first = L, last = 0;
      for (uint64_t k = 0; k < L; ++k)
        if (flat_next(it, S, regs, tid, bad) != ' ') {
          if (first == L) first = k;
          last = k + 1;
        }
      g.w0 = pc.a == VF_RTRIM ? 0 : first;
      const uint64_t end = pc.a == VF_LTRIM ? L : last;
      g.mid = end > g.w0 ? end - g.w0 : 0;
      break;
    }
    case VF_LEFT: g.mid = na <= 0 ? 0 : ((uint64_t)na < L ? (uint64_t)na : L); break;
    case VF_RIGHT: {
      const uint64_t k = na <= 0 ? 0 : ((uint64_t)na < L ? (uint64_t)na : L);
      g.w0 = L - k;
      g.mid = k;
      break;
    }
    case VF_LPAD:
    case VF_RPAD: {
      if (na < 0) {
        bad = true;
        g.mid = 0;
        break;
      }
      if ((uint64_t)na < L) {
        g.mid = (uint64_t)na;
        break;
      }
      const uint64_t need = (uint64_t)na - L;
      g.padlen = flat_len(data, padh, S, regs, tid, bad);
      if (need && !g.padlen) {
        bad = true;
        break;
      }
      if (pc.a == VF_LPAD) g.pre = need;
      else g.post = need;
      break;
    }
    default: {   // VF_SUBSTR
      const uint64_t ast = na == INT64_MIN ? 1ull << 63 : (uint64_t)(na < 0 ? -na : na);
      if (ast > L || nb <= 0 || na == 0) {
        g.mid = 0;
      } else {
        g.w0 = na > 0 ? (uint64_t)na - 1 : L - ast;
        const uint64_t room = L - g.w0;
        g.mid = (uint64_t)nb < room ? (uint64_t)nb : room;
      }
    }
  }
  if (g.pre + g.mid + g.post >= (1ull << 31)) {
    bad = true;
    g.pre = g.post = 0;
    g.mid = 0;
  }
  return g;
}

// A view being read: out of line (view_open / view_next / view_len are calls) so that the string
// ops that never meet a view keep the registers they had; the inlined paths only test a piece's
// kind.  `bad` travels in return values (no escaping reference).
struct ViewIter {
  FlatIter in;  // the inner list, positioned at the window
  int32_t padh;
  uint32_t padlen, pre, mid, total, pos, cs, oc;
};

// false: bad
__device__ __noinline__ bool view_open(ViewIter* w, const Ins pc, const Ins* data, const DevStrings* S,
                                       const int64_t* regs, int tid) {
  bool bad = false;
  const ViewGeom g = view_geom(pc, data, *S, regs, tid, bad);
  flat_open(w->in, data, pc.aux, *S, regs, tid, bad);
  flat_skip(w->in, g.w0, *S, regs, tid, bad);
  w->padh = (int32_t)(pc.imm & 0xFFFFFFFFll);
  w->padlen = (uint32_t)g.padlen;
  w->pre = (uint32_t)g.pre;
  w->mid = (uint32_t)g.mid;
  w->total = (uint32_t)(g.pre + g.mid + g.post);
  w->pos = 0;
  w->cs = g.cs;
  w->oc = g.oc;
  return !bad;
}

// the view's next byte; -1 at its end, -2 bad
__device__ __noinline__ int view_next(ViewIter* w, const Ins* data, const DevStrings* S, const int64_t* regs,
                                      int tid) {
  if (w->pos >= w->total) return -1;
  bool bad = false;
  const uint32_t p = w->pos++;
  int c;
  if (p < w->pre) {
    c = (int)flat_byte_at(data, w->padh, p % w->padlen, *S, regs, tid, bad);
  } else if (p - w->pre < w->mid) {
    c = flat_next(w->in, *S, regs, tid, bad);
    if (c < 0) c = 0;
    if (w->cs == 1 && c >= 'A' && c <= 'Z') c += 32;
    if (w->cs == 2 && c >= 'a' && c <= 'z') c -= 32;
  } else {
    c = (int)flat_byte_at(data, w->padh, (p - w->pre - w->mid) % w->padlen, *S, regs, tid, bad);
  }
  if (w->oc == 1 && c >= 'A' && c <= 'Z') c += 32;
  if (w->oc == 2 && c >= 'a' && c <= 'z') c -= 32;
  return bad ? -2 : c;
}

// the view's length; -1: bad
__device__ __noinline__ int64_t view_len(const Ins pc, const Ins* data, const DevStrings* S, const int64_t* regs,
                                         int tid) {
  bool bad = false;
  const ViewGeom g = view_geom(pc, data, *S, regs, tid, bad);
  return bad ? -1 : (int64_t)(g.pre + g.mid + g.post);
}

// A derived string's piece list streamed byte by byte, views included
struct StrIter {
  FlatIter o;   // the list; its current piece when not in a view
  ViewIter vw;
  const Ins* data;
  bool view;
};

__device__ __forceinline__ void str_open(StrIter& it, const Ins* data, int32_t hdr, const DevStrings&,
                                         const int64_t*, int, bool&) {
  const Ins h = data[hdr];
  it.o.list = data + h.aux;
  it.o.dbase = reinterpret_cast<const char*>(data);
  it.o.n = h.d;
  it.o.k = -1;
  it.o.i = 0;
  it.o.v = PieceView{it.o.dbase, 0, 0, 0, 0};
  it.data = data;
  it.view = false;
}

// the next byte (-1 at the end)
__device__ __forceinline__ int str_next(StrIter& it, const DevStrings& S, const int64_t* regs, int tid, bool& bad) {
  for (;;) {
    if (it.view) {
      const int c = view_next(&it.vw, it.data, &S, regs, tid);
      if (c >= 0) return c;
      bad = bad || c == -2;
      it.view = false;
    } else if (it.o.i < it.o.v.len) {
      return (int)piece_byte(it.o.v, it.o.i++);
    }
    if (++it.o.k >= it.o.n) return -1;
    const Ins pc = it.o.list[it.o.k];
    if (pc.op == PC_VIEW) {
      bad = !view_open(&it.vw, pc, it.data, &S, regs, tid) || bad;
      it.view = true;
    } else {
      it.o.v = piece_view(pc, it.o.dbase, S, regs, tid, bad);
      it.o.i = 0;
    }
  }
}

__device__ __forceinline__ uint64_t str_len(const Ins* data, int32_t hdr, const DevStrings& S, const int64_t* regs,
                                            int tid, bool& bad) {
  const Ins h = data[hdr];
  uint64_t n = 0;
  for (int k = 0; k < h.d; ++k) {
    const Ins pc = data[h.aux + k];
    if (pc.op == PC_VIEW) {
      const int64_t l = view_len(pc, data, &S, regs, tid);
      bad = bad || l < 0;
      n += l < 0 ? 0 : (uint64_t)l;
    } else {
      n += piece_view(pc, reinterpret_cast<const char*>(data), S, regs, tid, bad).len;
    }
  }
  return n;
}

// std::string::compare of two piece lists: <0, 0, >0
__device__ int str_cmp(const Ins* data, int32_t ha, int32_t hb, const DevStrings& S, const int64_t* regs, int tid,
                       bool& bad) {
  StrIter x, y;
  str_open(x, data, ha, S, regs, tid, bad);
  str_open(y, data, hb, S, regs, tid, bad);
  for (;;) {
    const int cx = str_next(x, S, regs, tid, bad), cy = str_next(y, S, regs, tid, bad);
    if (cx != cy) return cx < cy ? -1 : 1;   // (the end, -1, sorts first: a prefix is smaller)
    if (cx < 0) return 0;
  }
}

__device__ __forceinline__ bool is_space(int ch) { return ch == ' ' || (ch >= '\t' && ch <= '\r'); }

// strtoll(s, &end, 10) consuming the whole string, no overflow (Expression::toInt of a string,
// as exprc.cpp cast_value restates folly::to<int64_t>); false = evaluation error
__device__ bool str_to_int(StrIter& it, const DevStrings& S, const int64_t* regs, int tid, bool& bad, int64_t* out) {
  int ch = str_next(it, S, regs, tid, bad);
  while (ch >= 0 && is_space(ch)) ch = str_next(it, S, regs, tid, bad);
  bool neg = false;
  if (ch == '+' || ch == '-') {
    neg = ch == '-';
    ch = str_next(it, S, regs, tid, bad);
  }
  if (ch < '0' || ch > '9') return false;
  uint64_t u = 0;
  const uint64_t lim = neg ? (1ull << 63) : (1ull << 63) - 1;
  bool over = false;
  for (; ch >= '0' && ch <= '9'; ch = str_next(it, S, regs, tid, bad)) {
    const uint64_t d = (uint64_t)(ch - '0');
    if (u > (lim - d) / 10) over = true;
    else u = u * 10 + d;
  }
  if (ch >= 0 || over) return false;
  *out = neg ? (int64_t)(0ull - u) : (int64_t)u;
  return true;
}

// strtod(s, &end) consuming the whole string, for decimal forms whose value is exact in the
// fast path (<= 19 significant digits, m * 10^e with m < 2^53 and |e| <= 22, both exact, so the
// one rounding is IEEE's); other spellings (hex, inf, nan, longer mantissas) return false
__device__ bool str_to_double(StrIter& it, const DevStrings& S, const int64_t* regs, int tid, bool& bad, double* out) {
  int ch = str_next(it, S, regs, tid, bad);
  while (ch >= 0 && is_space(ch)) ch = str_next(it, S, regs, tid, bad);
  bool neg = false;
  if (ch == '+' || ch == '-') {
    neg = ch == '-';
    ch = str_next(it, S, regs, tid, bad);
  }
  uint64_t m = 0;
  int sig = 0, e10 = 0;
  bool any = false;
  for (; ch >= '0' && ch <= '9'; ch = str_next(it, S, regs, tid, bad)) {
    any = true;
    if (m || ch != '0') {
      if (sig >= 19) return false;
      m = m * 10 + (uint64_t)(ch - '0');
      ++sig;
    }
  }
  if (ch == '.') {
    ch = str_next(it, S, regs, tid, bad);
    for (; ch >= '0' && ch <= '9'; ch = str_next(it, S, regs, tid, bad)) {
      any = true;
      if (m || ch != '0') {
        if (sig >= 19) return false;
        m = m * 10 + (uint64_t)(ch - '0');
        ++sig;
      }
      --e10;
    }
  }
  if (!any) return false;
  if (ch == 'e' || ch == 'E') {
    ch = str_next(it, S, regs, tid, bad);
    bool eneg = false;
    if (ch == '+' || ch == '-') {
      eneg = ch == '-';
      ch = str_next(it, S, regs, tid, bad);
    }
    if (ch < '0' || ch > '9') return false;   // strtod would stop before the 'e'
    int ex = 0;
    for (; ch >= '0' && ch <= '9'; ch = str_next(it, S, regs, tid, bad)) ex = ex < 100000 ? ex * 10 + (ch - '0') : ex;
    e10 += eneg ? -ex : ex;
  }
  if (ch >= 0) return false;
  double v;
  if (m == 0) {
    v = 0.0;
  } else {
    if (m > (1ull << 53)) return false;
    if (e10 > 22 && e10 <= 22 + 15) {   // m * 10^(e10 - 22) may still be exact
      const uint64_t k = kPow10[e10 - 22];
      if (m > (1ull << 53) / k) return false;
      m *= k;
      e10 = 22;
    }
    if (e10 < -22 || e10 > 22) return false;
    v = e10 >= 0 ? (double)m * (double)kPow10[e10] : (double)m / (double)kPow10[-e10];
  }
  *out = neg ? -v : v;
  return true;
}

// libstdc++'s std::_Hash_bytes (the 64-bit MurmurHash2 variant under std::hash<std::string> and
// std::hash<double>), seed 0xc70f6907: 8-byte little-endian words, then the tail bytes
constexpr uint64_t HB_MUL = 0xc6a4a7935bd1e995ull;
__device__ __forceinline__ uint64_t hb_shift_mix(uint64_t v) { return v ^ (v >> 47); }
__device__ __forceinline__ uint64_t hb_word(uint64_t h, uint64_t w) {
  return (h ^ (hb_shift_mix(w * HB_MUL) * HB_MUL)) * HB_MUL;
}
__device__ __forceinline__ uint64_t hb_final(uint64_t h, uint64_t tail, uint64_t ntail) {
  if (ntail) h = (h ^ tail) * HB_MUL;
  return hb_shift_mix(hb_shift_mix(h) * HB_MUL);
}
__device__ uint64_t str_hash_bytes(const Ins* data, int32_t hdr, const DevStrings& S, const int64_t* regs, int tid,
                                   bool& bad) {
  const uint64_t len = str_len(data, hdr, S, regs, tid, bad);
  uint64_t h = 0xc70f6907ull ^ (len * HB_MUL), w = 0;
  StrIter it;
  str_open(it, data, hdr, S, regs, tid, bad);
  for (uint64_t k = 0; k < len; ++k) {
    w |= (uint64_t)(uint32_t)str_next(it, S, regs, tid, bad) << (8 * (k & 7));
    if ((k & 7) == 7) {
      h = hb_word(h, w);
      w = 0;
    }
  }
  return hb_final(h, w, len & 7);
}
__device__ __forceinline__ uint64_t hash_double_bits(int64_t bits) {   // std::hash<double>
  if (as_f(bits) == 0.0) return 0;   // (+0.0 and -0.0)
  return hb_final(hb_word(0xc70f6907ull ^ (8 * HB_MUL), (uint64_t)bits), 0, 0);
}

// glibc strcasecmp over two piece lists: the difference of the first differing lowered bytes (a
// string's end reads as 0, so a proper prefix compares as the shorter one's NUL)
__device__ int64_t str_casecmp(const Ins* data, int32_t ha, int32_t hb, const DevStrings& S, const int64_t* regs,
                               int tid, bool& bad) {
  StrIter x, y;
  str_open(x, data, ha, S, regs, tid, bad);
  str_open(y, data, hb, S, regs, tid, bad);
  for (;;) {
    int cx = str_next(x, S, regs, tid, bad), cy = str_next(y, S, regs, tid, bad);
    if (cx < 0) cx = 0;
    if (cy < 0) cy = 0;
    const int lx = cx >= 'A' && cx <= 'Z' ? cx + 32 : cx, ly = cy >= 'A' && cy <= 'Z' ? cy + 32 : cy;
    if (lx != ly || cx == 0) return lx - ly;
  }
}

// rand32 / rand64 (FunctionManager.cpp:186-230 over folly::Random): a value per evaluation from
// the query's seed, the edge and the instruction (random in the reference too; the ranges and the
// integer conversions are what is restated)
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9e3779b97f4a7c15ull;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}
__device__ int64_t rand_value(uint64_t seed, uint64_t j, uint32_t v, int pc, int nargs, bool r64, int64_t a0,
                              int64_t a1) {
  const uint64_t r = splitmix64(seed ^ splitmix64(j * 0x100000001b3ull + v) ^ ((uint64_t)pc << 56));
  if (!r64) {
    const uint32_t u = (uint32_t)r;
    if (nargs == 0) return (int64_t)(int32_t)u;
    const uint32_t lo = nargs == 2 ? (uint32_t)a0 : 0u, hi = (uint32_t)(nargs == 2 ? a1 : a0);
    if (lo == hi) return 0;   // folly: an empty range
    const uint32_t got = lo + (uint32_t)(((uint64_t)u * (uint32_t)(hi - lo)) >> 32);
    return nargs == 1 ? (int64_t)(int32_t)got : (int64_t)got;
  }
  if (nargs == 0) return (int64_t)r;
  const uint64_t lo = nargs == 2 ? (uint64_t)a0 : 0ull, hi = (uint64_t)(nargs == 2 ? a1 : a0);
  if (lo == hi) return 0;
  return (int64_t)(lo + __umul64hi(r, hi - lo));
}

// OP_SMAT: the piece list's bytes into an arena entry ([u64 0][u64 len][bytes]), STR_ARENA | its
// offset (read back by the same lane through a PC_DICT piece)
__device__ int64_t str_mat(const Ins* data, int32_t hdr, const DevStrings& S, const int64_t* regs, int tid, bool& bad,
                           bool& err) {
  const uint64_t len = str_len(data, hdr, S, regs, tid, bad);
  const uint64_t need = 16 + ((len + 7) & ~7ull);
  const uint64_t at = atomicAdd(S.arena_used, (unsigned long long)need);
  if (!S.arena || at + need > S.arena_cap) {   // the host fails the query with E_OUT_OF_MEMORY
    if (S.err_flag) atomicOr(S.err_flag, ARENA_OVERFLOW);
    err = true;
    return STR_ARENA | (STR_ARENA - 1);   // (no entry: a reader sees an offset past the arena)
  }
  char* e = S.arena + at;
  StrIter it;
  str_open(it, data, hdr, S, regs, tid, bad);
  for (uint64_t i = 0; i < len; ++i) e[16 + i] = (char)str_next(it, S, regs, tid, bad);
  *reinterpret_cast<uint64_t*>(e) = 0;
  *reinterpret_cast<uint64_t*>(e + 8) = len;
  return STR_ARENA | (int64_t)at;
}

// OP_SOUT: the derived string into the arena; its canonical code (dictionary code when the
// dictionary holds it, else STR_DERIVED | content hash, str_derived_code)
__device__ int64_t str_store(const Ins* data, int32_t hdr, const DevStrings& S, const int64_t* regs, int tid,
                             bool& bad, bool& err) {
  const uint64_t len = str_len(data, hdr, S, regs, tid, bad);
  const uint64_t need = 16 + ((len + 7) & ~7ull);
  const uint64_t at = atomicAdd(S.arena_used, (unsigned long long)need);
  if (!S.arena || at + need > S.arena_cap) {   // the host fails the query with E_OUT_OF_MEMORY
    if (S.err_flag) atomicOr(S.err_flag, ARENA_OVERFLOW);
    err = true;
    return 0;
  }
  char* e = S.arena + at;
  StrIter it;
  str_open(it, data, hdr, S, regs, tid, bad);
  uint64_t h = STR_HASH_INIT;
  for (uint64_t i = 0; i < len; ++i) {
    const int ch = str_next(it, S, regs, tid, bad);
    e[16 + i] = (char)ch;
    h = str_hash_step(h, (uint8_t)ch);
  }
  const int64_t code = str_derived_code(h, len);
  *reinterpret_cast<int64_t*>(e) = code;
  *reinterpret_cast<uint64_t*>(e + 8) = len;
  // the dictionary's code when it holds the string (so a value has one code, whatever made it)
  uint64_t lo = 0, hi = S.n;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    const uint32_t b = S.off[mid], n = S.off[mid + 1] - b;
    int c = 0;
    for (uint32_t i = 0; i < n && i < len && !c; ++i) {
      const uint32_t x = (uint8_t)S.bytes[b + i], y = (uint8_t)e[16 + i];
      c = x < y ? -1 : x > y ? 1 : 0;
    }
    if (!c) c = n < len ? -1 : n > len ? 1 : 0;
    if (c == 0) return (int64_t)(2 * mid);
    if (c < 0) lo = mid + 1;
    else hi = mid;
  }
  return code;
}

// Evaluate instructions [pc0, pc1) for this lane.  Registers live in LDS, one 8-byte slot per
// lane per register ([reg][BLOCK]); instruction fetch is wave-uniform (scalar loads).  `data`:
// the program's piece lists and constant bytes (derived strings).
__device__ __forceinline__ void run_program(const Ins* __restrict__ prog, const Ins* __restrict__ data, int pc0,
                                            int pc1, const EdgeCtx& c, const ExpandArgs& a,
                                            int64_t* __restrict__ regs, bool active, bool& err, uint32_t& tbits) {
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
      case OP_TAGS:
      case OP_TAGS_E:
        if (active) {
          const uint32_t v = a.gbase + c.v;
          if (a.tpres[ins.aux >> 16][v]) r = a.tcols[ins.aux & 0xFFFF][v];
          else if (ins.op == OP_TAGS) r = ins.imm;
          else err = true;
        }
        break;
      case OP_TAGD:
        if (active) {
          const uint32_t v = a.col[c.j];
          if (v != NO_ROW && a.tpres[ins.aux >> 16][v]) {
            r = a.tcols[ins.aux & 0xFFFF][v];
          } else {
            r = ins.imm;
            tbits |= 1u << (MAX_TAG_BITS + (ins.aux >> 16));
          }
        }
        break;
      case OP_EIDX: r = (int64_t)c.j; break;
      case OP_INPUT:
        if (active) {
          // getPropFromInterim (GoExecutor.cpp:1066-1075): the row of the source's root
          const int64_t root = a.bt_in ? a.bt_in[c.v] : a.vids[c.v];
          uint64_t lo = 0, hi = a.in_n;
          while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (a.in_ids[mid] < root) lo = mid + 1;
            else hi = mid;
          }
          if (lo < a.in_n && a.in_ids[lo] == root) r = a.in_cols[ins.aux][lo];
          else err = true;
        }
        break;
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
      case OP_S2I:
      case OP_S2F: {
        const bool dbl = ins.op == OP_S2F;
        if (x >= 0 && !(x & 1) && (uint64_t)(x >> 1) < a.str.n &&
            (a.str.s2ok[x >> 1] & (dbl ? 2 : 1))) {
          r = dbl ? a.str.s2f[x >> 1] : a.str.s2i[x >> 1];
        } else if (active) {
          err = true;   // not a number ("" too)
        }
        break;
      }
      case OP_SCMP:
        if (active) {
          bool bad = false;
          const int cm = str_cmp(data, ins.aux, (int32_t)ins.imm, a.str, regs, tid, bad);
          switch (ins.a) {   // EK_REL op: < <= > >= == !=
            case 0: r = cm < 0; break;
            case 1: r = cm <= 0; break;
            case 2: r = cm > 0; break;
            case 3: r = cm >= 0; break;
            case 4: r = cm == 0; break;
            default: r = cm != 0; break;
          }
          err = err || bad;
        }
        break;
      case OP_SPARSE_I:
      case OP_SPARSE_F:
        if (active) {
          bool bad = false;
          StrIter it;
          str_open(it, data, ins.aux, a.str, regs, tid, bad);
          bool ok;
          if (ins.op == OP_SPARSE_I) {
            ok = str_to_int(it, a.str, regs, tid, bad, &r);
          } else {
            double v = 0.0;
            ok = str_to_double(it, a.str, regs, tid, bad, &v);
            r = fbits(v);
          }
          err = err || bad || !ok;
        }
        break;
      case OP_SEMPTY:
        if (active) {
          bool bad = false;
          r = str_len(data, ins.aux, a.str, regs, tid, bad) == 0;
          err = err || bad;
        }
        break;
      case OP_SOUT:
        if (active) {
          bool bad = false;
          r = str_store(data, ins.aux, a.str, regs, tid, bad, err);
          err = err || bad;
        }
        break;
      case OP_SMAT:
        if (active) {
          bool bad = false;
          r = str_mat(data, ins.aux, a.str, regs, tid, bad, err);
          err = err || bad;
        }
        break;
      case OP_ISIN_I: r = (y != 0) || x == ins.imm; break;
      case OP_ISIN_F: r = (y != 0) || as_f(x) == as_f(ins.imm); break;
      case OP_EQX_F: r = as_f(x) == as_f(y); break;
      case OP_ABS_F: r = fbits(fabs(as_f(x))); break;
      case OP_FLOOR_F: r = fbits(floor(as_f(x))); break;
      case OP_CEIL_F: r = fbits(ceil(as_f(x))); break;
      case OP_ROUND_F: r = fbits(round(as_f(x))); break;
      case OP_SQRT_F: r = fbits(sqrt(as_f(x))); break;
      case OP_MATH1_F: {
        const double v = as_f(x);
        double o;
        switch (ins.aux) {
          case 0: o = cbrt(v); break;
          case 1: o = exp(v); break;
          case 2: o = exp2(v); break;
          case 3: o = log(v); break;
          case 4: o = log2(v); break;
          case 5: o = log10(v); break;
          case 6: o = sin(v); break;
          case 7: o = asin(v); break;
          case 8: o = cos(v); break;
          case 9: o = acos(v); break;
          case 10: o = tan(v); break;
          default: o = atan(v); break;
        }
        r = fbits(o);
        break;
      }
      case OP_MATH2_F: r = fbits(ins.aux == 0 ? pow(as_f(x), as_f(y)) : hypot(as_f(x), as_f(y))); break;
      case OP_HASH_F: r = (int64_t)hash_double_bits(x); break;
      case OP_HASH_S:
      case OP_SLEN:
      case OP_SCASE:
        if (active) {
          bool bad = false;
          if (ins.op == OP_HASH_S) r = (int64_t)str_hash_bytes(data, ins.aux, a.str, regs, tid, bad);
          else if (ins.op == OP_SLEN) r = (int64_t)str_len(data, ins.aux, a.str, regs, tid, bad);
          else r = str_casecmp(data, ins.aux, (int32_t)ins.imm, a.str, regs, tid, bad);
          err = err || bad;
        }
        break;
      case OP_RAND: r = rand_value(a.rand_seed, c.j, c.v, pc, ins.aux & 3, (ins.aux & 4) != 0, x, y); break;
      case OP_NOW: r = a.now_sec; break;
      default: break;

    }
    regs[ins.d * BLOCK + tid] = r;
  }
}

// ----------------------------------------------------------------------------- k_expand
// FINALF: the final step with a FastProg program (no interpreter: fewer registers, 8 waves/SIMD)
// FINALD: FINALF whose YIELDs are only _dst / constants; a tile's rows are stored after the NEXT
// tile's loads are issued, so waiting for those loads never waits for this tile's stores (on
// CDNA one counter, vmcnt, retires loads and stores in issue order)
// MARKB: MARK that also records each reached vertex's root (VertexBackTracker::add, last write
// wins as in the reference's unordered iteration) for queries that read $- / $var props
// FINALY: FINALF with many YIELD columns (getBound's rows): the loads of YG columns of every item
// in flight together, at 4 waves/SIMD for the registers they need
enum Mode { MARK = 0, FINAL = 1, BFS = 2, FINALF = 3, FINALD = 4, MARKB = 5, FINALY = 6 };

struct DegsumArgs {
  int ntypes;
  const uint32_t* row_ptr[MAX_TYPES_Q];
  const uint8_t* visible;
  uint32_t cap;
};

__device__ unsigned long long degree_of(const DegsumArgs& d, uint32_t v) {
  if (v == NO_ROW || (d.visible && !d.visible[v])) return 0;
  unsigned long long sum = 0;
  for (int t = 0; t < d.ntypes; ++t) {
    const uint32_t deg = d.row_ptr[t][v + 1] - d.row_ptr[t][v];
    sum += deg < d.cap ? deg : d.cap;
  }
  return sum;
}

// BFS-mode expansion (FIND SHORTEST PATH): every neighbour w is claimed at most once per epoch by
// a CAS on its label (epoch << LVL_BITS | level); winners are appended, one atomic per wave tile,
// straight to the next frontier list (`out`, count `*out_n`).  With `dsum` set, each tile also
// adds its claimed vertices' degrees over `deg` (the next level's bound and direction) with one
// atomic.
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
  uint32_t* out;                  // next frontier list (a level claims <= nv vertices)
  unsigned long long* out_n;      // its length, zero before the level
  DegsumArgs deg;
  unsigned long long* dsum;       // nullable
  // MARK claim mode (lab != nullptr): claimed neighbours go to this list with their edge space
  // over nds (the next step's first OVER type); nlist.zero_next is zeroed by workgroup 0
  ListOut nlist;
  DegSrc nds;
  // MARK on a partitioned engine (non-null): neighbours set their bit of the global id space in
  // this bitmap (the hop's all-to-all send buffer) instead of a byte flag — no pack pass
  unsigned long long* bits;
  // ... or, for a level whose edge total is small (non-null): the neighbour of edge e (its
  // position in the list's edge space) goes to slot e of its owner's segment, as the owner's
  // local id — sparse[owner * sp_stride + e]; slots start as NO_ROW.  No atomics.
  uint32_t* sparse;
  uint32_t sp_stride;
  uint32_t sp_npad;
};

struct FinalParams {
  const Ins* prog;
  int where_len;
  int where_reg;          // -1 none
  int prog_len;           // WHERE + YIELD instructions
  int nyields;
  int yield_reg[MAX_YIELDS];
  int64_t yield_const[MAX_YIELDS];
  int64_t* out_cols[MAX_YIELDS];   // by value: global stores, no pointer loads per row
  uint64_t region_base;   // first row of this type's region
  uint64_t blk_cap;       // rows per workgroup region (each workgroup appends to its own region)
  uint32_t* blk_rows;     // [gridDim.x] rows written per workgroup
  unsigned long long* err_flag;
  uint32_t probe_mask;             // tags read through $$ (presence probed for every final edge)
  int keep_on_error;               // storage-side filter: an evaluation error keeps the edge
  unsigned long long* tag_bits;    // QState::tagbits
  FastProg fast;
};

// MARK claim mode: the per-step dst SET (GoExecutor::getDstIdsFromResp, GoExecutor.cpp:501-541)
// as claims — the first expansion of the step to CAS a neighbour's stamp to the step's stamp
// owns it — and the owners appended to the next frontier list together with their edge space
// over the next step's first OVER type: one packed atomic per wave for list positions and edge
// offsets.  A vertex without edges there is kept (the list is the frontier of every OVER type).
__device__ __forceinline__ void claim_append(const uint32_t (&u)[VT], const BfsParams& bp, int lane) {
  uint32_t dg[VT], rs[VT], cmask = 0;
#pragma unroll
  for (int i = 0; i < VT; ++i) {
    dg[i] = 0;
    rs[i] = 0;
    const uint32_t x = u[i];
    if (x == NO_ROW) continue;
    const uint32_t old = bp.lab[x];
    if (old == bp.stamp) continue;
    if (atomicCAS(bp.lab + x, old, bp.stamp) != old) continue;
    cmask |= 1u << i;
    dg[i] = vdeg(bp.nds, x, &rs[i]);
  }
  uint32_t c = (uint32_t)__popc(cmask), d = 0;
#pragma unroll
  for (int i = 0; i < VT; ++i) d += dg[i];
  const uint32_t ic = wave_incl_scan(c), id = wave_incl_scan(d);
  const uint32_t tc = __shfl(ic, 63, 64), td = __shfl(id, 63, 64);
  if (!tc) return;   // wave-uniform
  unsigned long long old = 0;
  if (lane == 0) old = atomicAdd(bp.nlist.acc, ((unsigned long long)tc << 32) | td);
  old = __shfl(old, 0, 64);
  uint32_t pos = (uint32_t)(old >> 32) + ic - c;
  uint32_t pd = (uint32_t)old + id - d;
#pragma unroll
  for (int i = 0; i < VT; ++i) {
    uint64_t t0 = 0, t1 = 0;
    const uint32_t p = pos;
    if ((cmask >> i) & 1u) list_put(bp.nlist, bp.nds, pos++, u[i], &pd, dg[i], rs[i], &t0, &t1);
    wave_splits(bp.nlist.tsplit, t0, t1, p);
  }
}

// Merge-path split of tile t: entries consumed before position t * TILE (which 0) or before the
// tile's end (which 1).
__device__ __forceinline__ uint64_t tile_split(const uint32_t* __restrict__ tsplit, uint64_t t, int which,
                                               uint64_t npath, uint64_t n) {
  if (which == 0) return tsplit[t];
  return (t + 1) * TILE >= npath ? n : tsplit[t + 1];
}

// Lane k's entry of a tile's window: seg_end[a0 - 1 + k] (k <= na + 1) and seg_rs[a0 + k].
__device__ __forceinline__ void stage_pre(const uint32_t* __restrict__ seg_end, const uint32_t* __restrict__ seg_rs,
                                          uint64_t n, uint64_t a0, uint64_t a1, int k, uint32_t* e, uint32_t* r) {
  const int na = (int)(a1 - a0);
  if (k <= na + 1) {
    const int64_t i = (int64_t)a0 - 1 + k;
    *e = i < 0 ? 0u : (i < (int64_t)n ? seg_end[i] : 0xFFFFFFFFu);
  }
  if (k <= na) {
    const uint64_t i = a0 + k;
    *r = i < n ? seg_rs[i] : 0u;
  }
}

__device__ __forceinline__ uint64_t uniform64(uint64_t v) {   // a wave-uniform value, in SGPRs
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}

// LDS written by some lanes of a wave and read by others: complete the wave's LDS operations.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Wave-tiled, load-balanced expansion.  Every WAVE owns whole tiles of TILE = 64 * VT merge-path
// items (frontier entries + edges) and runs them without workgroup barriers: its segment window,
// merge-path assignment and row offsets live in its own LDS slice and registers, so the 32 waves
// of a CU progress independently and the memory latency of one is hidden by the others.  While
// a wave processes tile t, the split of tile t + 2g and the window of tile t + g are in flight
// (software pipeline, registers).  Items are processed striped across the wave's lanes so
// neighbour / property reads are coalesced.
struct NoInline {};
template <bool INL>
using InlineArg = typename std::conditional<INL, InlineList, NoInline>::type;

// INL: the list is the query's start list, passed in the kernel arguments (InlineList) and
// staged in LDS; its tile splits are counted directly (<= INLINE_STARTS entries).
// V: merge-path items per lane (the tile is 64 * V items).  Producers split their lists per
// TILE = 64 * VT; a V = 2 * VT instantiation reads every other split.  (FINALD with V = 8 at 5 or
// 6 waves per SIMD measured 307-338 us per RMAT-26 launch against 222 us at V = 4 and 8 waves,
// profiles/r02_q_final_vt8_ab.json: the default V = VT is the only one launched.)
template <int M, bool INL = false, int V = VT>
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(M == FINAL || M == FINALY ? 4 : (V > VT ? 6 : 8))))
k_expand(ExpandArgs a, const unsigned long long* __restrict__ acc, const uint32_t* __restrict__ seg_end,
         const uint32_t* __restrict__ seg_rs, uint8_t* __restrict__ flags, FinalParams fp, BfsParams bp,
         unsigned long long* stat_e, unsigned long long* stat_n, InlineArg<INL> il) {
  __shared__ uint32_t sEndAll[WAVES][64 * V + 2];   // per wave: seg_end for i in [a0-1, a1]
  __shared__ uint32_t sRsAll[WAVES][64 * V + 1];    // per wave: seg_rs for i in [a0, a1]
  __shared__ uint16_t sSegAll[WAVES][64 * V];       // per wave: segment of each edge item
  __shared__ unsigned long long sBase;            // FINAL: rows this workgroup wrote (LDS cursor)
  extern __shared__ int64_t regs[];               // FINAL generic path: [nregs][BLOCK]

  __shared__ uint32_t sIl[INL ? 3 * INLINE_STARTS : 1];   // INL: end[], rs[], id[] of the start list
  uint64_t n, total;   // list entries, edges
  if constexpr (INL) {
    n = il.n;
    total = il.total;
#pragma unroll
    for (int k = 0; k < INLINE_STARTS; ++k)   // constant kernel-argument offsets (no scratch copy)
      if (threadIdx.x == k) {
        sIl[k] = il.end[k];
        sIl[INLINE_STARTS + k] = il.rs[k];
        sIl[2 * INLINE_STARTS + k] = il.id[k];
      }
    __syncthreads();
  } else {
    const unsigned long long packed = *acc;   // (list entries << 32 | edges) of the list a.frontier
    n = packed >> 32;
    total = packed & 0xFFFFFFFFull;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (stat_e) *stat_e += total;
    if (stat_n) {
      if constexpr (INL) *stat_n = il.n_in;
      else *stat_n = n;
    }
  }
  const uint64_t npath = n + total;
  constexpr uint64_t TV = 64 * V;   // items per tile
  static_assert(TV % TILE == 0, "tiles are whole producer tiles");
  const uint64_t ntiles = (npath + TV - 1) / TV;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: scalar registers
  uint32_t* const sEnd = sEndAll[w];
  uint32_t* const sRs = sRsAll[w];
  uint16_t* const sSeg = sSegAll[w];
  bool anyErr = false;
  uint32_t tbits = 0;              // FINAL: $$ holder bits (QState::tagbits)
  // merge-path split of tile tt (which 0: entries before its start; 1: before its end)
  auto split_of = [&](uint64_t tt, int which) -> uint64_t {
    if constexpr (INL) {
      const uint64_t p = (tt + (uint64_t)which) * TV;
      if (which == 1 && p >= npath) return n;
      uint64_t c = 0;   // entries whose span [j + start_j, j + end_j] ends before p
      for (uint32_t j = 0; j < (uint32_t)n; ++j) c += (uint64_t)j + sIl[j] < p;
      return c;
    } else {
      // producer splits every TILE items: this tile's boundaries are every (TV / TILE)-th of them
      if (which == 0) return a.tsplit[tt * (TV / TILE)];
      return (tt + 1) * TV >= npath ? n : a.tsplit[(tt + 1) * (TV / TILE)];
    }
  };
  // lane k's entry of a tile's segment-end window (seg_end[a0 - 1 + k]) and row starts (seg_rs[a0 + k])
  auto stage = [&](uint64_t s0, uint64_t s1, uint32_t* e, uint32_t* r) {
    if constexpr (INL) {
      const int na_ = (int)(s1 - s0);
      if (lane <= na_ + 1) {
        const int64_t i = (int64_t)s0 - 1 + lane;
        *e = i < 0 ? 0u : (i < (int64_t)n ? sIl[i] : 0xFFFFFFFFu);
      }
      if (lane <= na_) *r = s0 + lane < n ? sIl[INLINE_STARTS + s0 + lane] : 0u;
    } else {
      stage_pre(seg_end, seg_rs, n, s0, s1, lane, e, r);
    }
  };
  // the list's vertex at position i
  auto list_id = [&](uint64_t i) -> uint32_t {
    if constexpr (INL) return sIl[2 * INLINE_STARTS + i];
    else return a.frontier[i];
  };
  constexpr bool kFinal = M == FINAL || M == FINALF || M == FINALD || M == FINALY;
  constexpr bool kFast = M == FINALF || M == FINALD || M == FINALY;
  constexpr bool kDefer = M == FINALD;
  int64_t pdv[V];                 // FINALD: the previous tile's _dst values, pass mask, first row
  uint32_t ppm = 0;
  uint64_t preg = 0;
#pragma unroll
  for (int i = 0; i < V; ++i) pdv[i] = 0;
  uint32_t pu[V];                 // MARK: the previous tile's neighbours (flags not yet set)
#pragma unroll
  for (int i = 0; i < V; ++i) pu[i] = NO_ROW;
  int64_t* const* ycols = fp.out_cols;
  // rows of one tile: ballot-ordered positions from `region`, YIELD y = _dst or a constant
  auto store_dst_rows = [&](const int64_t* vdv, uint32_t pm, uint64_t region) {
    uint32_t off = 0;
#pragma unroll
    for (int i = 0; i < V; ++i) {
      const bool pass = (pm >> i) & 1u;
      const unsigned long long bal = __ballot(pass);
      if (!bal) continue;
      const uint64_t row = region + off + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
      off += (uint32_t)__popcll(bal);
      if (pass)
        for (int y = 0; y < fp.nyields; ++y) ycols[y][row] = fp.fast.ykind[y] == 0 ? vdv[i] : fp.yield_const[y];
    }
  };
  if (kFinal) {
    if (threadIdx.x == 0) sBase = 0;
    __syncthreads();
  }
  if ((M == MARK || M == MARKB) && bp.nlist.zero_next && blockIdx.x == 0 && threadIdx.x == 0) *bp.nlist.zero_next = 0;
  const uint64_t g = (uint64_t)gridDim.x * WAVES;
  // MARK: tile t -> workgroup t % grid first (a step's few tiles spread over CUs, each CU's miss
  // queue serving one wave's random claims; see spchain.hip); the final step keeps adjacent tiles
  // in one workgroup (they share lines at their boundaries; an XCD-major order measured -4 %,
  // DESIGN.md §5)
  uint64_t t = (M == MARK || M == MARKB) ? (uint64_t)w * gridDim.x + blockIdx.x : (uint64_t)blockIdx.x * WAVES + w;
  uint64_t sp_next = 0;            // lanes 0, 1: split (start, end) of tile t + g
  uint64_t a0 = 0, a1 = 0;         // split of tile t
  uint32_t e_pre = 0, r_pre = 0;   // lane's entry of tile t's segment-end window / row starts
  if (t < ntiles) {
    uint64_t sp = 0;
    if (lane < 2) {
      sp = split_of(t, lane);
      if (t + g < ntiles) sp_next = split_of(t + g, lane);
    }
    a0 = uniform64(__shfl(sp, 0, 64));
    a1 = uniform64(__shfl(sp, 1, 64));
    stage(a0, a1, &e_pre, &r_pre);
  }
  for (; t < ntiles; t += g) {
    const uint64_t d0 = t * TV;
    const uint64_t d1 = (d0 + TV < npath) ? d0 + TV : npath;
    // a split read from memory must describe this tile (entries within the list, in order, no more
    // of them than the tile has items, its edges within the list's): a stale one skips the tile and
    // fails the query (SPLIT_BAD) instead of indexing out of bounds
    const bool bad = !(a0 <= a1 && a1 <= n && a1 - a0 <= d1 - d0 && d1 - a1 <= total && d0 - a0 <= d1 - a1);
    if (bad && lane == 0 && fp.err_flag) atomicOr(fp.err_flag, SPLIT_BAD);
    const uint64_t b0 = bad ? 0 : d0 - a0, b1 = bad ? 0 : d1 - a1;
    const int na = bad ? 0 : (int)(a1 - a0), nb = bad ? 0 : (int)(b1 - b0);

    // the wave's window in LDS (entries past the prefetch loaded directly)
    if (lane <= na + 1) sEnd[lane] = e_pre;
    if (lane <= na) sRs[lane] = r_pre;
    if constexpr (!INL) {   // (an inline list has <= INLINE_STARTS entries: the prefetch covers it)
      for (int k = lane + 64; k <= na + 1; k += 64) {
        const uint64_t i = a0 - 1 + (uint64_t)k;
        sEnd[k] = i < n ? seg_end[i] : 0xFFFFFFFFu;
        if (k <= na) sRs[k] = i + 1 < n ? seg_rs[i + 1] : 0u;
      }
    }
    // prefetch tile t + g's window and tile t + 2g's split
    uint64_t na0 = 0, na1 = 0;
    if (t + g < ntiles) {
      na0 = uniform64(__shfl(sp_next, 0, 64));
      na1 = uniform64(__shfl(sp_next, 1, 64));
      stage(na0, na1, &e_pre, &r_pre);
      if (lane < 2 && t + 2 * g < ntiles) sp_next = split_of(t + 2 * g, lane);
    }
    wave_lds_sync();
    const uint32_t* A = sEnd + 1;   // A[k] = end of segment a0 + k

    // lane-level merge path over this tile: assign a segment to every edge item
    {
      const int diag = lane * V;
      const int dmax = na + nb;
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
        for (int k = 0; k < V; ++k) {
          if (ai + bi >= dmax) break;
          if (ai < na && (bi >= nb || (uint64_t)A[ai] <= b0 + (uint64_t)bi)) {
            ++ai;
          } else {
            sSeg[bi] = (uint16_t)ai;
            ++bi;
          }
        }
      }
    }
    wave_lds_sync();

    if constexpr (M == MARKB) {
      uint32_t u[V];
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const int k = i * 64 + lane;
        u[i] = NO_ROW;
        if (k < nb) {
          const uint32_t s = sSeg[k];
          u[i] = a.col[(uint64_t)sRs[s] + (b0 + k - (uint64_t)sEnd[s])];
          if (u[i] == NO_ROW) continue;
          const uint32_t src = list_id(a0 + s);
          a.bt[u[i]] = a.bt_first ? a.vids[src] : a.bt_in[src];
          if (!bp.lab) flags[u[i]] = 1;
        }
      }
      if (bp.lab) claim_append(u, bp, lane);
    } else if constexpr (M == MARK) {
      uint32_t u[V];   // all neighbour loads in flight before the flag stores / claims
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const int k = i * 64 + lane;
        u[i] = NO_ROW;
        if (k < nb) {
          const uint32_t s = sSeg[k];
          u[i] = a.col[(uint64_t)sRs[s] + (b0 + k - (uint64_t)sEnd[s])];   // sEnd[s] = start of a0+s
        }
      }
      if (bp.lab) {
        claim_append(u, bp, lane);
      } else if (bp.sparse) {
#pragma unroll
        for (int i = 0; i < V; ++i) {
          if (u[i] == NO_ROW) continue;
          const uint32_t q = u[i] / bp.sp_npad;
          bp.sparse[(uint64_t)q * bp.sp_stride + b0 + (uint64_t)(i * 64 + lane)] = u[i] - q * bp.sp_npad;
        }
      } else {
        // the previous tile's flags behind this tile's loads (see FINALD)
#pragma unroll
        for (int i = 0; i < V; ++i) {
          if (pu[i] != NO_ROW) {
            if (bp.bits) atomicOr(bp.bits + (pu[i] >> 6), 1ull << (pu[i] & 63));
            else flags[pu[i]] = 1;
          }
          pu[i] = u[i];
        }
      }
    } else if constexpr (M == BFS) {
      uint32_t wv[V];
      uint32_t cmask = 0, mmask = 0;
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const int k = i * 64 + lane;
        wv[i] = NO_ROW;
        if (k < nb) {
          const uint32_t s = sSeg[k];
          wv[i] = a.col[(uint64_t)sRs[s] + (b0 + k - (uint64_t)sEnd[s])];
        }
      }
#pragma unroll
      for (int i = 0; i < V; ++i) {
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
      // one atomic per wave tile on the list length
      uint32_t pre[V], run = 0;
#pragma unroll
      for (int i = 0; i < V; ++i) {
        pre[i] = run;
        run += (uint32_t)__popcll(__ballot((cmask >> i) & 1u));
      }
      unsigned long long base = 0;
      if (lane == 0 && run) base = atomicAdd(bp.out_n, (unsigned long long)run);
      base = __shfl(base, 0, 64);
      uint32_t* const region = bp.out + base;
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const bool c = (cmask >> i) & 1u;
        const unsigned long long bal = __ballot(c);
        if (c) region[pre[i] + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull))] = wv[i];
        const bool m = (mmask >> i) & 1u;
        const unsigned long long mb = __ballot(m);
        if (mb) {
          unsigned long long mbase = 0;
          if (lane == 0) mbase = atomicAdd(bp.meet_n, (unsigned long long)__popcll(mb));
          mbase = __shfl(mbase, 0, 64);
          if (m) {
            bp.meet_list[mbase + (uint32_t)__popcll(mb & ((1ull << lane) - 1ull))] = wv[i];
            bp.mout[wv[i]] = bp.mstamp;
          }
        }
      }
      if (bp.dsum && run) {
        unsigned long long ds = 0;
#pragma unroll
        for (int i = 0; i < V; ++i)
          if ((cmask >> i) & 1u) ds += degree_of(bp.deg, wv[i]);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) ds += __shfl_down(ds, o, 64);
        if (lane == 0 && ds) atomicAdd(bp.dsum, ds);
      }
    } else {
      // phase A: WHERE for every item of the tile (V items per lane, striped)
      uint32_t jj[V];      // edge index in the CSR (< 2^32 per type)
      uint32_t vv[V];
      int64_t dv[V];       // fast path: _dst prefetched with the WHERE column (one round trip)
      uint32_t pmask = 0;
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const int k = i * 64 + lane;
        jj[i] = 0;
        vv[i] = 0;
        if (k < nb) {
          const uint32_t s = sSeg[k];
          jj[i] = sRs[s] + (uint32_t)(b0 + k - (uint64_t)sEnd[s]);
          vv[i] = s;
        }
      }
      if (kFast) {
        // all loads of the tile in flight at once; the comparison is branch-free
        int64_t x[V];
#pragma unroll
        for (int i = 0; i < V; ++i) {
          const bool act = i * 64 + lane < nb;
          dv[i] = (act && fp.fast.dst_yield) ? a.dst_vid[jj[i]] : 0;
        }
        // the WHERE column at its stored width (narrow copy of an INT column when it fits)
        switch (fp.fast.has_where ? fp.fast.wbytes : 0) {
          case 1: load_narrow<int8_t, V>(fp.fast.wcol, jj, nb, lane, x); break;
          case 2: load_narrow<int16_t, V>(fp.fast.wcol, jj, nb, lane, x); break;
          case 4: load_narrow<int32_t, V>(fp.fast.wcol, jj, nb, lane, x); break;
          case 8: load_narrow<int64_t, V>(fp.fast.wcol, jj, nb, lane, x); break;
          default:
#pragma unroll
            for (int i = 0; i < V; ++i) x[i] = 0;
        }
        if (kDefer) {   // the previous tile's rows, behind this tile's loads
          store_dst_rows(pdv, ppm, preg);
          ppm = 0;
        }
#pragma unroll
        for (int i = 0; i < V; ++i) {
          const bool act = i * 64 + lane < nb;
          const bool in = (x[i] >= fp.fast.lo) & (x[i] <= fp.fast.hi);
          const bool pass = act & (!fp.fast.has_where | (in != (fp.fast.where_neg != 0)));
          pmask |= (uint32_t)pass << i;
        }
      } else {
        for (int i = 0; i < V; ++i) {
          const int k = i * 64 + lane;
          const bool active = k < nb;
          bool pass = active;
          if (fp.probe_mask && active) {   // the holder: every final destination's tags
            const uint32_t d = a.col[jj[i]];
            if (d != NO_ROW)
              for (uint32_t m = fp.probe_mask; m; m &= m - 1) {
                const int t = __builtin_ctz(m);
                if (a.tpres[t][d]) tbits |= 1u << t;
              }
          }
          if (fp.where_reg >= 0) {
            bool werr = false;
            EdgeCtx c{jj[i], active ? list_id(a0 + vv[i]) : 0u};
            run_program(fp.prog, fp.prog + fp.prog_len, 0, fp.where_len, c, a, regs, active, werr, tbits);
            if (fp.keep_on_error) {
              pass = active && (werr || regs[fp.where_reg * BLOCK + threadIdx.x] != 0);
            } else {
              pass = active && !werr && regs[fp.where_reg * BLOCK + threadIdx.x] != 0;
              if (active && werr) anyErr = true;
            }
          }
          pmask |= (uint32_t)pass << i;
        }
      }
      // row offsets in item order: wave-uniform prefix over the V ballots, then one LDS atomic
      // on the workgroup's cursor (rows go to the workgroup's own region: no global atomics)
      uint32_t run = 0;
#pragma unroll
      for (int i = 0; i < V; ++i) run += (uint32_t)__popcll(__ballot((pmask >> i) & 1u));
      unsigned long long base = 0;
      if (lane == 0 && run) base = atomicAdd(&sBase, (unsigned long long)run);
      base = __shfl(base, 0, 64);
      // phase B: YIELD for the passing items, written at their final rows
      const uint64_t region = fp.region_base + (uint64_t)blockIdx.x * fp.blk_cap + base;
      if (kDefer) {   // stored behind the next tile's loads (or after the loop)
#pragma unroll
        for (int i = 0; i < V; ++i) pdv[i] = dv[i];
        ppm = pmask;
        preg = region;
      }
      int64_t* const* cols = fp.out_cols;   // kernel-argument array
      uint32_t off = 0;                     // rows of the earlier items of this tile
      if (M == FINALY) {
        // YG YIELD columns at a time, with the loads of all their cells in flight together (a
        // load-store pair per cell left one memory round trip per cell on the critical path)
        constexpr int YG = 4;
        for (int y0 = 0; y0 < fp.nyields; y0 += YG) {
          int64_t val[YG][V];
#pragma unroll
          for (int u = 0; u < YG; ++u) {
            const int y = y0 + u;
            if (y >= fp.nyields) break;   // (uniform)
            const int kind = fp.fast.ykind[y];
#pragma unroll
            for (int i = 0; i < V; ++i) {
              val[u][i] = 0;
              if (!((pmask >> i) & 1u)) continue;
              switch (kind) {
                case 0: val[u][i] = dv[i]; break;
                case 1: val[u][i] = a.vids[list_id(a0 + vv[i])]; break;
                case 2: val[u][i] = a.rank ? a.rank[jj[i]] : 0; break;
                case 3: val[u][i] = load_col(fp.fast.ycol[y], fp.fast.ybytes[y], jj[i]); break;
                case 5: val[u][i] = (int64_t)jj[i]; break;
                default: val[u][i] = fp.yield_const[y]; break;
              }
            }
          }
          uint32_t roff = 0;
#pragma unroll
          for (int i = 0; i < V; ++i) {
            const bool pass = (pmask >> i) & 1u;
            const unsigned long long bal = __ballot(pass);
            const uint64_t row = region + roff + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
            roff += (uint32_t)__popcll(bal);
            if (!pass) continue;
#pragma unroll
            for (int u = 0; u < YG; ++u)
              if (y0 + u < fp.nyields) cols[y0 + u][row] = val[u][i];
          }
        }
      }
#pragma unroll
      for (int i = 0; i < V && !kDefer && M != FINALY; ++i) {
        const bool pass = (pmask >> i) & 1u;
        const unsigned long long bal = __ballot(pass);
        if (!bal) continue;
        const uint64_t row = region + off + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
        off += (uint32_t)__popcll(bal);
        if (kFast) {
          if (pass) {
            for (int y = 0; y < fp.nyields; ++y) {
              int64_t val;
              switch (fp.fast.ykind[y]) {
                case 0: val = dv[i]; break;
                case 1: val = a.vids[list_id(a0 + vv[i])]; break;
                case 2: val = a.rank ? a.rank[jj[i]] : 0; break;
                case 3: val = load_col(fp.fast.ycol[y], fp.fast.ybytes[y], jj[i]); break;
                case 5: val = (int64_t)jj[i]; break;
                default: val = fp.yield_const[y]; break;
              }
              cols[y][row] = val;
            }
          }
        } else
        {
          bool yerr = false;
          EdgeCtx c{jj[i], pass ? list_id(a0 + vv[i]) : 0u};
          run_program(fp.prog, fp.prog + fp.prog_len, fp.where_len, fp.prog_len, c, a, regs, pass, yerr, tbits);
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
    a0 = na0;
    a1 = na1;
  }
  if (kDefer) store_dst_rows(pdv, ppm, preg);   // the wave's last tile
  if (M == MARK) {
#pragma unroll
    for (int i = 0; i < V; ++i)
      if (pu[i] != NO_ROW) {
        if (bp.bits) atomicOr(bp.bits + (pu[i] >> 6), 1ull << (pu[i] & 63));
        else flags[pu[i]] = 1;
      }
  }
  if (kFinal) {
    __syncthreads();   // every wave of the workgroup has reserved its rows
    if (threadIdx.x == 0) fp.blk_rows[blockIdx.x] = (uint32_t)sBase;
    if (anyErr) atomicOr(fp.err_flag, 1ull);
    if (M == FINAL && fp.probe_mask) {
      // OR over the wave, one atomic per wave with bits
      uint32_t x = tbits;
      for (int o = 32; o; o >>= 1) x |= (uint32_t)__shfl_xor((int)x, o, 64);
      if (lane == 0 && x) atomicOr(fp.tag_bits, (unsigned long long)x);
    }
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
// union is the global per-step dst SET restricted to the owner (getDstIdsFromResp).  Listed as
// k_compact does: 16 vertices (bits) per thread.
// rt.recv (nullable): the roots each rank sent for this rank's vertices, packed per sending rank
// in bit order (k_rt_pack); a vertex reached from several ranks takes the highest such rank's
// (the reference's last write is arbitrary as well)
struct RootsIn {
  const int64_t* recv;    // packed roots, rank q's from disp[world + q]
  const uint32_t* pre;    // popcount prefixes of the received bitmap (k_rt_prefix, second half)
  const uint32_t* boff;   // block offsets (k_rt_offsets, second half)
  const uint64_t* disp;
  uint64_t nwords;        // words of one bitmap (world * npad / 64)
};
__global__ void __launch_bounds__(BLOCK) k_bits_compact(const unsigned long long* __restrict__ recv, int world,
                                                        uint64_t seg_words, uint64_t nv, DegSrc ds, ListOut o,
                                                        RootsIn rt, int64_t* __restrict__ bt_in) {
  if (blockIdx.x == 0 && threadIdx.x == 0) *o.zero_next = 0;
  const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;   // 16-bit slice index
  const uint64_t word = i >> 2;
  const int sh = (int)(i & 3) * 16;
  unsigned long long m64 = 0;
  for (int q = 0; q < world; ++q) m64 |= recv[(uint64_t)q * seg_words + word];
  uint32_t m = (uint32_t)(m64 >> sh) & 0xFFFFu;
  const uint64_t lo = i * 16;
  if (lo >= nv) m = 0;
  else if (nv - lo < 16) m &= (1u << (nv - lo)) - 1u;
  uint32_t dg[16], rs[16], d = 0;
#pragma unroll
  for (int b = 0; b < 16; ++b) {
    dg[b] = ((m >> b) & 1u) ? vdeg(ds, (uint32_t)(lo + b), &rs[b]) : 0u;
    d += dg[b];
  }
  uint32_t pc, pd;
  reserve<BLOCK>((uint32_t)__popc(m), d, o.acc, &pc, &pd);
#pragma unroll
  for (int b = 0; b < 16; ++b) {
    uint64_t t0 = 0, t1 = 0;
    const uint32_t pp = pc;
    if ((m >> b) & 1u) list_put(o, ds, pc++, (uint32_t)(lo + b), &pd, dg[b], rs[b], &t0, &t1);
    wave_splits(o.tsplit, t0, t1, pp);
  }
  if (rt.recv && m) {
    for (int b = 0; b < 16; ++b) {
      if (!((m >> b) & 1u)) continue;
      for (int q = world - 1; q >= 0; --q) {
        const uint64_t rw = (uint64_t)q * seg_words + word;
        const unsigned long long bits = recv[rw];
        if (!((bits >> (sh + b)) & 1ull)) continue;
        const uint64_t at = rt.disp[world + q] + rt.boff[(rt.nwords + rw) / RW_BLOCK] + rt.pre[rt.nwords + rw] +
                            (uint64_t)__popcll(bits & ((1ull << (sh + b)) - 1ull));
        bt_in[lo + b] = rt.recv[at];
        break;
      }
    }
  }
}

// Owner side of a small hop's slot exchange (ws_set_hop_slots): recv = world segments of `stride`
// local ids (NO_ROW: empty).  A vertex may arrive several times, so each arrival is claimed
// against the step's stamp (CAS); the winners are listed, with their edge space over ds, as
// k_bits_compact lists a bitmap's (the union is getDstIdsFromResp's per-step set).
constexpr int SC_ITEMS = 4;
__global__ void __launch_bounds__(BLOCK) k_slots_compact(const uint32_t* __restrict__ recv, uint64_t slots,
                                                         uint32_t* __restrict__ lab, uint32_t stamp, uint64_t nv,
                                                         DegSrc ds, ListOut o) {
  if (blockIdx.x == 0 && threadIdx.x == 0) *o.zero_next = 0;
  const uint64_t base = ((uint64_t)blockIdx.x * BLOCK + threadIdx.x) * SC_ITEMS;
  uint32_t v[SC_ITEMS], dg[SC_ITEMS], rs[SC_ITEMS], c = 0, d = 0;
#pragma unroll
  for (int k = 0; k < SC_ITEMS; ++k) v[k] = base + k < slots ? recv[base + k] : NO_ROW;
#pragma unroll
  for (int k = 0; k < SC_ITEMS; ++k) {
    if (v[k] >= nv) {   // (NO_ROW, or an id past this rank's vertices: dropped)
      v[k] = NO_ROW;
    } else {
      const uint32_t old = lab[v[k]];
      if (old == stamp || atomicCAS(lab + v[k], old, stamp) != old) v[k] = NO_ROW;
    }
    dg[k] = v[k] != NO_ROW ? vdeg(ds, v[k], &rs[k]) : 0u;
    c += v[k] != NO_ROW ? 1u : 0u;
    d += dg[k];
  }
  uint32_t pc, pd;
  reserve<BLOCK>(c, d, o.acc, &pc, &pd);
#pragma unroll
  for (int k = 0; k < SC_ITEMS; ++k) {   // (every lane: wave_splits is wave-wide)
    uint64_t t0 = 0, t1 = 0;
    const uint32_t pp = pc;
    if (v[k] != NO_ROW) list_put(o, ds, pc++, v[k], &pd, dg[k], rs[k], &t0, &t1);
    wave_splits(o.tsplit, t0, t1, pp);
  }
}

// Partitioned roots, 1 of 3: the popcount before every bitmap word within its block of RW_BLOCK
// words, and each block's total, over the send bitmap (blocks [0, nb)) and the received one
// ([nb, 2 nb)); 4 words per thread.
__global__ void __launch_bounds__(BLOCK) k_rt_prefix(const unsigned long long* __restrict__ sb,
                                                     const unsigned long long* __restrict__ rb, uint64_t nb,
                                                     uint32_t* __restrict__ pre, uint32_t* __restrict__ bsum) {
  __shared__ uint32_t s_w[WAVES];
  const uint64_t blk = blockIdx.x;
  const unsigned long long* src = blk < nb ? sb : rb;
  const uint64_t w0 = (blk < nb ? blk : blk - nb) * RW_BLOCK + threadIdx.x * 4;
  uint32_t c[4], t = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    c[k] = (uint32_t)__popcll(src[w0 + k]);
    t += c[k];
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t inc = wave_incl_scan(t);
  if (lane == 63) s_w[wv] = inc;
  __syncthreads();
  uint32_t run = inc - t;
  for (int k = 0; k < wv; ++k) run += s_w[k];
  uint32_t* out = pre + blk * RW_BLOCK + threadIdx.x * 4;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    out[k] = run;
    run += c[k];
  }
  if (threadIdx.x == BLOCK - 1) bsum[blk] = run;
}

// 2 of 3 (one workgroup): block totals -> offsets within their rank segment (spb blocks each;
// segments 0..world-1 of the send bitmap, then world..2 world-1 of the received one), the
// per-rank counts (cnt: mapped host memory, the host sizes the exchange from them) and the
// packed displacements.
__global__ void __launch_bounds__(BLOCK) k_rt_offsets(uint32_t* __restrict__ bsum, uint64_t spb, int world,
                                                      uint64_t* __restrict__ disp, uint64_t* cnt) {
  __shared__ uint32_t s_w[WAVES];
  __shared__ unsigned long long s_run;
  __shared__ unsigned long long s_cnt[2 * AGREE_WORDS];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int g = 0; g < 2 * world; ++g) {
    if (threadIdx.x == 0) s_run = 0;
    __syncthreads();
    uint32_t* b = bsum + (uint64_t)g * spb;
    for (uint64_t k0 = 0; k0 < spb; k0 += BLOCK) {
      const uint64_t k = k0 + threadIdx.x;
      const uint32_t v = k < spb ? b[k] : 0u;
      const uint32_t inc = wave_incl_scan(v);
      if (lane == 63) s_w[wv] = inc;
      __syncthreads();
      uint32_t base = 0, tot = 0;
      for (int j = 0; j < WAVES; ++j) {
        if (j < wv) base += s_w[j];
        tot += s_w[j];
      }
      const unsigned long long run = s_run;
      if (k < spb) b[k] = (uint32_t)(run + base + inc - v);
      __syncthreads();
      if (threadIdx.x == 0) s_run = run + tot;
      __syncthreads();
    }
    if (threadIdx.x == 0) s_cnt[g] = s_run;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int h = 0; h < 2; ++h) {
      unsigned long long d = 0;
      for (int q = 0; q < world; ++q) {
        disp[h * world + q] = d;
        d += s_cnt[h * world + q];
      }
    }
  }
  for (int g = threadIdx.x; g < 2 * world; g += BLOCK) cnt[g] = s_cnt[g];
}

// 3 of 3: the roots of the set bits of the send bitmap, packed per destination rank in bit order.
__global__ void __launch_bounds__(BLOCK) k_rt_pack(const unsigned long long* __restrict__ sb, uint64_t nwords,
                                                   uint64_t seg_words, const uint32_t* __restrict__ pre,
                                                   const uint32_t* __restrict__ boff, const uint64_t* __restrict__ disp,
                                                   const int64_t* __restrict__ bt_out, int64_t* __restrict__ pack) {
  const uint64_t w = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (w >= nwords) return;
  unsigned long long m = sb[w];
  if (!m) return;
  uint64_t at = disp[w / seg_words] + boff[w / RW_BLOCK] + pre[w];
  const int64_t* src = bt_out + w * 64;
  while (m) {
    pack[at++] = src[__ffsll((long long)m) - 1];
    m &= m - 1;
  }
}

// Stats of an expansion that is not launched (final step whose WHERE folded to false).
__global__ void k_note(const unsigned long long* __restrict__ acc, unsigned long long* stat_e,
                       unsigned long long* stat_n) {
  const unsigned long long v = *acc;
  *stat_e += v & 0xFFFFFFFFull;
  if (stat_n) *stat_n = v >> 32;
}

// Query statistics every rank needs globally: [err, step_n[0..MAX_STEPS+1], Σ_types e_st[s]].
// Then one counter per QState::tagbits bit (summed: > 0 is the OR over ranks), then one status
// word per rank (the rank's local status of the query: its own word, the others 0).
constexpr int GST_N0 = 1 + 2 * (MAX_STEPS + 2);
constexpr int GST_N = GST_N0 + 2 * MAX_TAG_BITS;
__global__ void k_gst_status(unsigned long long* __restrict__ g, int world, int rank, long long status) {
  for (int r = threadIdx.x; r < world; r += blockDim.x) g[GST_N + r] = r == rank ? (unsigned long long)status : 0ull;
}
__global__ void k_gstats(const QState* __restrict__ q, int ntypes, unsigned long long* __restrict__ g) {
  const int s = threadIdx.x;
  if (s == 0) g[0] = q->err ? 1ull : 0ull;
  if (s < 2 * MAX_TAG_BITS) g[GST_N0 + s] = (q->tagbits >> s) & 1ull;
  if (s < MAX_STEPS + 2) {
    g[1 + s] = q->step_n[s];
    unsigned long long e = 0;
    for (int t = 0; t < ntypes; ++t) e += q->e_st[s][t];
    g[1 + (MAX_STEPS + 2) + s] = e;
  }
}

// ============================================================================= host side
// algorithmic bytes per kernel (SURVEY.md §8(d) B_GO terms)
static double prof_bytes(const Workspace* w, const Prof::Rec& r, const QState& q) {
  switch (r.kid) {
    case K_RELIST: return 12.0 * (double)q.step_n[r.step];                 // 4|F| ids + 8|F| row_ptr
    case K_EXPAND_MARK: return 4.0 * (double)q.e_st[r.step][r.tix];        // 4 E_s neighbour ids
    // next frontier: 4|F_{s+1}| ids written + the fused degree pass of the next step (12|F_{s+1}|)
    case K_COMPACT: case K_BITS_COMPACT: return 16.0 * (double)q.step_n[r.step + 1];
    case K_PACK: case K_ALLTOALL: case K_ROOTS: return r.cols;             // sizes known at launch
    case K_EXPAND_FINAL: {
      double rows = 0;
      for (unsigned b = 0; b < w->final_grid[r.tix]; ++b) rows += (double)w->h_blk_rows[(size_t)r.tix * EXPAND_GRID + b];
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
    case K_RELIST: return 12.0 * (double)p.ln[i];
    case K_BFS: return 4.0 * (double)p.le[i];
    case K_GATHER: return 8.0 * (double)p.lc[i];   // (+8 B per packed vertex when it sums degrees)
    case K_DEGSUM: return 12.0 * (double)p.ln[i];
    default: return 0.0;
  }
}
static void prof_flush(Workspace* w, const QState* q, const PState* ps = nullptr) {
  // (a host woken by the end kernel's flag may be ahead of the last events)
  if (!w->prof.pending.empty()) (void)hipEventSynchronize(w->prof.pending.back().b);
  for (auto& r : w->prof.pending) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
      w->prof.launches[r.kid]++;
      w->prof.ms[r.kid] += ms;
      if (r.path) {
        if (ps) w->prof.bytes[r.kid] += prof_bytes_path(r, *ps);
      } else if (q) {
        w->prof.bytes[r.kid] += prof_bytes(w, r, *q);
      }
    }
    w->prof.pool.push_back(r.a);
    w->prof.pool.push_back(r.b);
  }
  w->prof.pending.clear();
}

void ws_profile(Workspace* w, int mode) {
  if (!w) return;
  prof_flush(w, nullptr);
  w->prof.on = mode != 0;
  w->prof.mask = mode == 2 ? ((1u << K_EXPAND_FINAL) | (1u << K_BFS)) : ~0u;
  const bool on = w->prof.on;
  if (on) {
    for (int k = 0; k < K_COUNT; ++k) { w->prof.launches[k] = 0; w->prof.ms[k] = 0; w->prof.bytes[k] = 0; }
  }
}

void ws_profile_inherit(Workspace* to, Workspace* from) {
  if (!to || !from) return;
  prof_flush(from, nullptr);
  to->prof.on = from->prof.on;
  to->prof.mask = from->prof.mask;
  for (int k = 0; k < K_COUNT; ++k) {
    to->prof.launches[k] = from->prof.launches[k];
    to->prof.ms[k] = from->prof.ms[k];
    to->prof.bytes[k] = from->prof.bytes[k];
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

Workspace* ws_create(uint64_t max_frontier, uint64_t nv, uint64_t e_max, hipStream_t s, std::string* err) {
  auto* w = new Workspace();
  w->stream = s;
  w->nv = nv;
  w->cap_frontier = max_frontier < 1024 ? 1024 : max_frontier;
  w->flag_bytes = cdiv(nv + 1, FLAG_ALIGN) * FLAG_ALIGN;
  hipError_t e = hipSuccess;
  auto M = [&](void** p, size_t b) { if (e == hipSuccess) e = hipMalloc(p, b); };
  M((void**)&w->frontier[0], w->cap_frontier * 4);
  M((void**)&w->frontier[1], w->cap_frontier * 4);
  M((void**)&w->seg_end, w->cap_frontier * 4);
  M((void**)&w->seg_rs, w->cap_frontier * 4);
  M((void**)&w->seg_end1, w->cap_frontier * 4);
  M((void**)&w->seg_rs1, w->cap_frontier * 4);
  M((void**)&w->rlist, w->cap_frontier * 4);
  M((void**)&w->flags, w->flag_bytes);
  M((void**)&w->seen, (nv + 1) * 4);
  w->e_max = e_max;
  w->cap_tiles = cdiv(w->cap_frontier + e_max + 1, TILE) + 2;
  M((void**)&w->tsplit, w->cap_tiles * 4);
  M((void**)&w->tsplit1, w->cap_tiles * 4);
  w->env_flags = getenv("NBG_MARK_FLAGS") && atoi(getenv("NBG_MARK_FLAGS")) != 0;
  w->mark_flags = w->env_flags;
  // QState and the per-workgroup row counts are one allocation: one copy ends a query
  M((void**)&w->q, sizeof(QState) + (size_t)MAX_TYPES_Q * EXPAND_GRID * 4);
  M((void**)&w->d_prog, (size_t)MAX_TYPES_Q * MAX_PROGRAM * sizeof(Ins));
  M((void**)&w->d_row_cols, MAX_YIELDS * sizeof(int64_t*));
  if (e == hipSuccess)
    e = hipHostMalloc((void**)&w->h_q, sizeof(QState) + (size_t)MAX_TYPES_Q * EXPAND_GRID * 4,
                      hipHostMallocMapped | hipHostMallocCoherent);
  if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&w->d_hq, w->h_q, 0);
  if (e == hipSuccess)
    e = hipHostMalloc((void**)&w->h_small, (SMALL_ROWS_WORDS + 1) * 8, hipHostMallocMapped | hipHostMallocCoherent);
  if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&w->d_small, w->h_small, 0);
  if (e == hipSuccess) w->h_small[0] = 0;
  if (e == hipSuccess) e = hipHostMalloc((void**)&w->h_wake, 64, hipHostMallocMapped | hipHostMallocCoherent);
  if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&w->d_wake, w->h_wake, 0);
  if (e == hipSuccess) w->h_wake[0] = 0;
  if (e == hipSuccess) e = hipMalloc((void**)&w->d_ticket, 64);
  if (e == hipSuccess) e = hipMemsetAsync(w->d_ticket, 0, 64, s);
  if (e == hipSuccess) {
    w->blk_rows = reinterpret_cast<uint32_t*>(w->q + 1);
    w->h_blk_rows = reinterpret_cast<uint32_t*>(w->h_q + 1);
    e = hipMemsetAsync(w->q, 0, sizeof(QState), s);
  }
  if (e == hipSuccess) e = hipHostMalloc((void**)&w->h_prog, (size_t)MAX_TYPES_Q * MAX_PROGRAM * sizeof(Ins),
                                         hipHostMallocDefault);
  if (e == hipSuccess) e = hipMemsetAsync(w->flags, 0, w->flag_bytes, s);
  if (e == hipSuccess) e = hipMemsetAsync(w->seen, 0, (nv + 1) * 4, s);
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
                  (void*)w->seg_end1, (void*)w->seg_rs1, (void*)w->tsplit1, (void*)w->seen,
                  (void*)w->rlist, (void*)w->flags, (void*)w->tsplit,
                  (void*)w->q, (void*)w->rows,
                  (void*)w->d_row_cols, (void*)w->d_prog, (void*)w->dtab, (void*)w->dkeep, (void*)w->dseg,
                  (void*)w->dcnt, (void*)w->dkinds, (void*)w->bt, (void*)w->walk_arena, (void*)w->sarena, (void*)w->xown,
                  (void*)w->xcnt, (void*)w->xsend, (void*)w->xrecv, (void*)w->bt_out, (void*)w->bt_recv,
                  (void*)w->bt_pack, (void*)w->bt_pre, (void*)w->bt_boff, (void*)w->bt_disp, (void*)w->d_ticket})
    if (p) (void)hipFree(p);
  for (void* p : {(void*)w->h_q, (void*)w->h_starts, (void*)w->h_prog, (void*)w->h_ps, (void*)w->h_path,
                  (void*)w->h_stage, (void*)w->h_small, (void*)w->h_wake})
    if (p) (void)hipHostFree(p);
  if (w->h_pgst) (void)hipHostFree(w->h_pgst);
  if (w->done_ev) (void)hipEventDestroy(w->done_ev);
  for (void* p : {(void*)w->sendbits, (void*)w->recvbits, (void*)w->gst, (void*)w->pgst, w->g_part, (void*)w->g_rec,
                  (void*)w->g_all, (void*)w->g_path, (void*)w->g_cur, (void*)w->ar_buf, (void*)w->fetch_meta,
                  (void*)w->fetch_out})
    if (p) (void)hipFree(p);
  if (w->h_gpath) (void)hipHostFree(w->h_gpath);
  if (w->h_gst) (void)hipHostFree(w->h_gst);
  if (w->h_btc) (void)hipHostFree(w->h_btc);
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

uint64_t ws_cap_frontier(Workspace* w) { return w ? w->cap_frontier : 0; }

static int lds_per_block() {
  static const int v = [] {
    int dev = 0, x = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&x, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) !=
                                                hipSuccess)
      x = 64 * 1024;
    return x;
  }();
  return v;
}
// (static LDS: k_expand ~10.7 KB, k_go_tiny ~25.1 KB, rounded up)
int interp_max_regs() { return std::max(1, std::min(MAX_REGS, (lds_per_block() - 12 * 1024) / (BLOCK * 8))); }
int tiny_max_regs() { return std::max(0, std::min(MAX_REGS, (lds_per_block() - 26 * 1024) / (BLOCK * 8))); }
uint64_t ws_cap_items(Workspace* w) { return w->cap_frontier + w->e_max; }
unsigned ws_final_grid_of(Workspace* w, int tix) { return w->final_grid[tix]; }
const uint32_t* ws_host_blk_rows(Workspace* w, int tix) { return w->h_blk_rows + (size_t)tix * EXPAND_GRID; }
int64_t* ws_row_col(Workspace* w, int c) { return w->rows + (uint64_t)c * w->cap_rows; }
const QState* ws_host_state(Workspace* w) { return w->h_q; }
const uint32_t* ws_current_frontier(Workspace* w) { return w->frontier[w->cur]; }

// The derived-string arena (OP_SOUT): at least `bytes`, grow-only.
hipError_t ws_reserve_arena(Workspace* w, uint64_t bytes) {
  if (bytes <= w->sarena_cap) return hipSuccess;
  HIP_TRY(ws_sync(w));
  if (w->sarena) HIP_TRY(hipFree(w->sarena));
  w->sarena = nullptr;
  w->sarena_cap = 0;
  HIP_TRY(hipMalloc((void**)&w->sarena, bytes));
  w->sarena_cap = bytes;
  return hipSuccess;
}

// The arena entries the finished query stored (QState::arena_used, read from the host copy).
hipError_t ws_read_arena(Workspace* w, uint64_t used, std::vector<char>* out) {
  if (used > w->sarena_cap) return hipErrorInvalidValue;
  out->resize(used);
  if (!used) return hipSuccess;
  HIP_TRY(hipMemcpyAsync(out->data(), w->sarena, used, hipMemcpyDeviceToHost, w->stream));
  return hipStreamSynchronize(w->stream);
}

const char* ws_arena(Workspace* w, uint64_t* cap) {
  *cap = w->sarena_cap;
  return w->sarena;
}

hipError_t ws_reserve_rows(Workspace* w, uint64_t rows, int ncols) {
  if (rows <= w->cap_rows && ncols <= w->ncols_alloc) return hipSuccess;
  HIP_TRY(ws_sync(w));
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

// The device QState is already zero (reset behind the previous query's final copy).  A short
// start list travels inside the first kernel's arguments: a query then begins with a launch, not
// a copy.  Programs are uploaded when the statement changes.
// Wait for the engine's stream.  A query's latency ends with this wait, so it polls an event
// (a host core spins for the few tens of microseconds a query takes) instead of the blocking
// hipStreamSynchronize; NBG_BLOCKING_SYNC=1 restores the blocking wait.
hipError_t ws_wait(Workspace* w) {
  static const bool blocking = getenv("NBG_BLOCKING_SYNC") != nullptr;
  if (blocking || w->comm) return ws_sync(w);
  if (!w->done_ev) HIP_TRY(hipEventCreateWithFlags(&w->done_ev, hipEventDisableTiming));
  HIP_TRY(hipEventRecord(w->done_ev, w->stream));
  hipError_t e;
  while ((e = hipEventQuery(w->done_ev)) == hipErrorNotReady) {
  }
  return e;
}

hipError_t ws_begin_query(Workspace* w, const uint32_t* starts, uint64_t n, const std::vector<TypeProgram>* progs,
                          uint64_t stmt_id) {
  if (n > w->cap_frontier) return hipErrorInvalidValue;
  w->cur = 0;
  w->seg_ready = false;
  w->list_acc = nullptr;
  w->pr = w->pc = 0;
  for (auto& g : w->final_grid) g = 0;
  w->start_n = n;
  w->start_inline = n <= INLINE_STARTS;
  if (w->start_inline) {
    w->inl.n = (uint32_t)n;
    for (uint64_t i = 0; i < n; ++i) w->inl.id[i] = starts[i];
  } else {
    if (n > w->cap_starts) {
      if (w->h_starts) HIP_TRY(hipHostFree(w->h_starts));
      w->cap_starts = n + n / 2 + 1024;
      HIP_TRY(hipHostMalloc((void**)&w->h_starts, w->cap_starts * 4, hipHostMallocDefault));
    }
    // the previous query on this workspace has completed (its end synchronised the stream)
    memcpy(w->h_starts, starts, n * 4);
    HIP_TRY(hipMemcpyAsync(w->frontier[0], w->h_starts, n * 4, hipMemcpyHostToDevice, w->stream));
  }
  if (progs && !progs->empty() && stmt_id != w->prog_stmt) {
    w->prog_stmt = stmt_id;
    // the programs' words in upload order; a statement whose programs equal the resident ones
    // (repeated requests of one shape, e.g. getBound) skips the upload
    std::vector<Ins> img;
    std::vector<uint32_t> lens;
    for (auto& p : *progs) {
      if (p.code.size() + p.data.size() > (size_t)MAX_PROGRAM) return hipErrorInvalidValue;
      img.insert(img.end(), p.code.begin(), p.code.end());
      img.insert(img.end(), p.data.begin(), p.data.end());   // (piece lists right after the code)
      lens.push_back((uint32_t)(p.code.size() + p.data.size()));
    }
    const bool same = lens == w->prog_lens && img.size() == w->prog_img.size() &&
                      (img.empty() || memcmp(img.data(), w->prog_img.data(), img.size() * sizeof(Ins)) == 0);
    if (!same) {
      size_t k = 0, off = 0;
      for (uint32_t n : lens) {
        memcpy(w->h_prog + k * MAX_PROGRAM, img.data() + off, n * sizeof(Ins));
        off += n;
        ++k;
      }
      HIP_TRY(hipMemcpyAsync(w->d_prog, w->h_prog, k * MAX_PROGRAM * sizeof(Ins), hipMemcpyHostToDevice, w->stream));
      w->prog_img.swap(img);
      w->prog_lens.swap(lens);
    }
  }
  return hipSuccess;
}

// The list one expansion consumes: the compaction's list when it already carries this (first)
// type's edge space, otherwise a k_relist of the current frontier over this type's CSR.
struct ListRef {
  const uint32_t* ids;
  const unsigned long long* acc;
  unsigned long long* stat_n;      // the expansion records |F_s| (its list is the whole frontier)
  int set;                         // edge-space set the list's seg_end / seg_rs / tsplit live in
};

static uint32_t* set_end(Workspace* w, int set) { return set ? w->seg_end1 : w->seg_end; }
static uint32_t* set_rs(Workspace* w, int set) { return set ? w->seg_rs1 : w->seg_rs; }
static uint32_t* set_split(Workspace* w, int set) { return set ? w->tsplit1 : w->tsplit; }

static DegSrc deg_of(const ExpandArgs& a) {
  DegSrc ds{};
  ds.row_ptr = a.row_ptr;
  ds.visible = a.visible;
  ds.cap = a.cap;
  return ds;
}

static ListOut list_out(Workspace* w, uint32_t* ids, unsigned long long* acc, unsigned long long* zero_next,
                        unsigned long long* stat_n, int set = 0) {
  ListOut o{};
  o.ids = ids;
  o.seg_end = set_end(w, set);
  o.seg_rs = set_rs(w, set);
  o.tsplit = set_split(w, set);
  o.acc = acc;
  o.zero_next = zero_next;
  o.stat_n = stat_n;
  return o;
}

static ListRef prepare_list(Workspace* w, const ExpandArgs& a, uint64_t n_bound, int step, int tix) {
  if (tix == 0 && w->seg_ready) {
    w->seg_ready = false;
    return ListRef{w->frontier[w->cur], w->list_acc, &w->q->step_n[step], w->cur};
  }
  unsigned long long* acc = &w->q->acc[w->pr];
  unsigned long long* other = &w->q->acc[w->pr ^ 1];
  w->pr ^= 1;
  const bool first = w->list_acc == nullptr;   // the start list
  const uint32_t* in = first && w->start_inline ? nullptr : w->frontier[w->cur];
  hipEvent_t p = prof_begin(w, K_RELIST);
  hipLaunchKernelGGL(k_relist, dim3((unsigned)cdiv(n_bound ? n_bound : 1, RL_TILE)), dim3(BLOCK), 0, w->stream, in,
                     w->list_acc, 1, (uint32_t)w->start_n, w->inl, deg_of(a),
                     list_out(w, w->rlist, acc, other, &w->q->step_n[step], w->cur), (unsigned long long*)nullptr);
  prof_end(w, p, K_RELIST, step, tix);
  return ListRef{w->rlist, acc, nullptr, w->cur};
}

// workgroups of a k_expand launch: one wave per tile up to EXPAND_GRID workgroups (persistent)
static unsigned expand_grid(uint64_t n_bound, uint64_t e_bound) {
  const uint64_t blocks = cdiv(cdiv(n_bound + e_bound + 1, TILE), WAVES);
  return (unsigned)(blocks < EXPAND_GRID ? (blocks ? blocks : 1) : EXPAND_GRID);
}

// intermediate GO steps' grid (NBG_MARK_GRID caps it, an A/B switch; default: the expansion grid)
static unsigned mark_grid(uint64_t n_bound, uint64_t e_bound) {
  static const unsigned cap = getenv("NBG_MARK_GRID") ? (unsigned)atoi(getenv("NBG_MARK_GRID")) : 0u;
  const unsigned g = expand_grid(n_bound, e_bound);
  return cap && cap < g ? cap : g;
}

// The expansion's list is the query's start list, available in inline form.
static bool inline_start_list(const Workspace* w, int tix, const InlineList* il) {
  return il && !(tix == 0 && w->seg_ready) && w->list_acc == nullptr && w->start_inline;
}

static DegSrc deg_src(const ExpandArgs* next0) { return next0 ? deg_of(*next0) : DegSrc{}; }

hipError_t ws_compact(Workspace* w, int step, const ExpandArgs* next0);

// NBG_PART_SPARSE=0: partitioned FIND PATH levels always exchange bitmaps (the A/B baseline)
static bool sparse_on() {
  static const bool on = !(getenv("NBG_PART_SPARSE") && atoi(getenv("NBG_PART_SPARSE")) == 0);
  return on;
}

// NBG_PART_FLAGS=1: partitioned MARK keeps byte flags + k_pack_bits (the A/B baseline)
static bool bits_off() {
  static const bool off = getenv("NBG_PART_FLAGS") && atoi(getenv("NBG_PART_FLAGS")) != 0;
  return off;
}

hipError_t ws_expand_mark(Workspace* w, const ExpandArgs& a0, uint64_t n_bound, uint64_t e_bound, int step, int tix,
                          const InlineList* il, const ExpandArgs* next0) {
  if (step > MAX_STEPS || tix >= MAX_TYPES_Q) return hipErrorInvalidValue;
  // claim mode (single engine): the step's dst SET is claimed against a per-step stamp and the
  // winners are appended, with their edge space over next0, straight to the next list (set
  // cur ^ 1, accumulator slot 2 + (step + 1) % 3; this step's first launch zeroes the slot of
  // step + 2, whose list (step - 1) nobody reads any more)
  BfsParams bp{};
  if (!w->comm && !w->mark_flags) {
    if (tix == 0) {
      if (++w->seen_stamp == 0) {   // wrap: clear the stamps once
        HIP_TRY(hipMemsetAsync(w->seen, 0, (w->nv + 1) * 4, w->stream));
        w->seen_stamp = 1;
      }
      w->step_stamp = w->seen_stamp;
    }
    bp.lab = w->seen;
    bp.stamp = w->step_stamp;
    const int nset = w->cur ^ 1;
    bp.nds = deg_src(next0);
    bp.nlist = list_out(w, w->frontier[nset], &w->q->acc[2 + (step + 1) % 3],
                        tix == 0 ? &w->q->acc[2 + (step + 2) % 3] : nullptr, nullptr, nset);
  }
  // partitioned MARK (not MARKB, whose roots ride with the byte flags): straight into the hop's
  // send bitmap, which ws_exchange then sends without a pack pass
  if (w->comm && !a0.bt && !bits_off()) {
    if (w->hop_slots) {   // a small hop: edge e's neighbour into slot e of its owner's segment (NO_ROW-filled)
      bp.sparse = reinterpret_cast<uint32_t*>(w->sendbits);
      bp.sp_stride = (uint32_t)w->hop_slots;
      bp.sp_npad = (uint32_t)w->npad;
    } else {
      bp.bits = w->sendbits;
    }
    w->hop_bits = true;
  }
  if (inline_start_list(w, tix, il)) {   // no k_relist: the list travels in the kernel arguments
    ExpandArgs a = a0;
    a.frontier = nullptr;
    a.tsplit = nullptr;
    hipEvent_t p = prof_begin(w, K_EXPAND_MARK);
    if (a.bt)
      hipLaunchKernelGGL((k_expand<MARKB, true>), dim3(mark_grid(il->n, il->total)), dim3(BLOCK), 0, w->stream, a,
                         (const unsigned long long*)nullptr, w->seg_end, w->seg_rs, w->flags, FinalParams{},
                         bp, &w->q->e_st[step][tix], &w->q->step_n[step], *il);
    else
      hipLaunchKernelGGL((k_expand<MARK, true>), dim3(mark_grid(il->n, il->total)), dim3(BLOCK), 0, w->stream, a,
                         (const unsigned long long*)nullptr, w->seg_end, w->seg_rs, w->flags, FinalParams{},
                         bp, &w->q->e_st[step][tix], &w->q->step_n[step], *il);
    prof_end(w, p, K_EXPAND_MARK, step, tix);
    return hipGetLastError();
  }
  const ListRef L = prepare_list(w, a0, n_bound, step, tix);
  ExpandArgs a = a0;
  a.frontier = L.ids;
  a.tsplit = set_split(w, L.set);
  FinalParams fp{};
  fp.err_flag = &w->q->err;   // (SPLIT_BAD)
  hipEvent_t p = prof_begin(w, K_EXPAND_MARK);
  if (a.bt)
    hipLaunchKernelGGL(k_expand<MARKB>, dim3(mark_grid(n_bound, e_bound)), dim3(BLOCK), 0, w->stream, a, L.acc,
                       set_end(w, L.set), set_rs(w, L.set), w->flags, fp, bp, &w->q->e_st[step][tix], L.stat_n,
                       NoInline{});
  else
    hipLaunchKernelGGL(k_expand<MARK>, dim3(mark_grid(n_bound, e_bound)), dim3(BLOCK), 0, w->stream, a, L.acc,
                       set_end(w, L.set), set_rs(w, L.set), w->flags, fp, bp, &w->q->e_st[step][tix], L.stat_n,
                       NoInline{});
  prof_end(w, p, K_EXPAND_MARK, step, tix);
  return hipGetLastError();
}

// Claims suit one OVER type (one claim per distinct neighbour); with several types the same
// vertices are reached through each, and the claim CAS on hot vertices costs more than plain
// byte flags plus one compaction (C5's knows + likes: 61.9 vs 126.8 G edges/s).
// The two modes keep different accumulator-slot invariants (claims: slot 2 + (step + 1) % 3, its
// successor zeroed by the step's first launch; flags: a ping-pong pair zeroed by k_compact), so a
// switch clears the slots first.
void ws_set_wake(Workspace* w, bool flag) { w->wake_flag = flag; }

void ws_set_mark_claims(Workspace* w, bool claims) {
  const bool flags = w->env_flags || !claims;
  if (flags != w->mark_flags) (void)hipMemsetAsync(&w->q->acc[2], 0, 3 * sizeof(unsigned long long), w->stream);
  w->mark_flags = flags;
}

hipError_t ws_finish_step(Workspace* w, int step, const ExpandArgs* next0) {
  if (w->mark_flags) return ws_compact(w, step, next0);
  w->cur ^= 1;
  w->list_acc = &w->q->acc[2 + (step + 1) % 3];
  w->seg_ready = next0 != nullptr;
  return hipSuccess;
}

hipError_t ws_compact(Workspace* w, int step, const ExpandArgs* next0) {
  unsigned long long* acc = &w->q->acc[2 + w->pc];
  unsigned long long* other = &w->q->acc[2 + (w->pc ^ 1)];
  w->pc ^= 1;
  uint32_t* next = w->frontier[w->cur ^ 1];
  hipEvent_t p = prof_begin(w, K_COMPACT);
  hipLaunchKernelGGL(k_compact, dim3((unsigned)(w->flag_bytes / CP_BYTES)), dim3(CP_THREADS), 0, w->stream, w->flags,
                     deg_src(next0), list_out(w, next, acc, other, nullptr, w->cur ^ 1));
  prof_end(w, p, K_COMPACT, step, 0);
  w->cur ^= 1;
  w->list_acc = acc;
  w->seg_ready = next0 != nullptr;
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
// A column as the fast path reads it: the narrow copy when the loader made one.
static const void* col_ptr(const ExpandArgs& a, int c, int* bytes) {
  if (a.hnarrow && a.hnarrow[c]) {
    *bytes = a.hnarrow_bytes[c];
    return a.hnarrow[c];
  }
  *bytes = 8;
  return a.hprops[c];
}

static FastProg detect_fast(const TypeProgram& prog, const ExpandArgs& a) {
  FastProg f{};
  f.enabled = 0;
  auto leaf_col = [&](const Ins& i) {
    return (i.op == OP_COL || (i.op == OP_COLV && a.valid == nullptr)) && a.hprops != nullptr;
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
    if (c.a == colI->d && c.b == constI->d) {
    } else if (c.a == constI->d && c.b == colI->d) {
      op = kSwap[op];
    } else {
      return f;
    }
    // col <op> k  as the range test lo <= x <= hi (negated for !=)
    const int64_t k = constI->imm;
    f.lo = INT64_MIN;
    f.hi = INT64_MAX;
    switch (op) {
      case 0: if (k == INT64_MIN) { f.lo = 1; f.hi = 0; } else f.hi = k - 1; break;   // <
      case 1: f.hi = k; break;                                                        // <=
      case 2: if (k == INT64_MAX) { f.lo = 1; f.hi = 0; } else f.lo = k + 1; break;   // >
      case 3: f.lo = k; break;                                                        // >=
      case 4: f.lo = f.hi = k; break;                                                 // ==
      default: f.lo = f.hi = k; f.where_neg = 1; break;                               // !=
    }
    f.has_where = 1;
    f.wcol = col_ptr(a, colI->aux, &f.wbytes);
  }
  const int ny = (int)prog.yield_reg.size();
  int pc = prog.where_len;
  for (int y = 0; y < ny; ++y) {
    if (prog.yield_reg[y] < 0) { f.ykind[y] = 4; continue; }
    if (pc >= (int)prog.code.size()) return f;
    const Ins& i = prog.code[pc++];
    if (i.d != prog.yield_reg[y]) return f;
    if (i.op == OP_DST) { f.ykind[y] = 0; f.dst_yield = 1; }
    else if (i.op == OP_SRC) f.ykind[y] = 1;
    else if (i.op == OP_RANK) f.ykind[y] = 2;
    else if (i.op == OP_EIDX) f.ykind[y] = 5;
    else if (leaf_col(i)) { f.ykind[y] = 3; f.ycol[y] = col_ptr(a, i.aux, &f.ybytes[y]); }
    else return f;
  }
  if (pc != (int)prog.code.size()) return f;
  f.enabled = 1;
  return f;
}

// The final step's grid: the expansion grid (8 workgroups per CU).  Round 2 capped it at 1920
// (7.5 per CU) for the FINALD kernel (profiles/r02_t_final_grid_ab.json: 280-282 -> 289-290 G
// edges/s); with k_final_dst a grid that is not a multiple of the CU count loses instead: half the
// CUs hold one workgroup more and set the launch's time (r05_i_final_grid_sweep.txt: 1920 -> 210 us,
// 1536 / 2048 / 2560 -> 202 us; GO 362-364 at 1920 and 2048).  NBG_FINAL_GRID caps it (0 = no cap).
static unsigned final_grid(uint64_t n_bound, uint64_t e_bound) {
  // (read per call: a statement's row regions are sized with the grid its launches use, and
  // both read it within one query)
  const char* ev = getenv("NBG_FINAL_GRID");
  const unsigned cap = ev ? (unsigned)atoi(ev) : 0u;
  const unsigned g = expand_grid(n_bound, e_bound);
  return cap && cap < g ? cap : g;
}

unsigned ws_final_grid(uint64_t n_bound, uint64_t e_bound) { return final_grid(n_bound, e_bound); }

uint64_t ws_final_blk_cap(uint64_t n_bound, uint64_t e_bound) {
  // a workgroup's waves each take tiles w, w + g, ... (g = grid * WAVES waves); a kernel
  // instantiated with V != VT needs its own tile size here
  const uint64_t tiles = cdiv(n_bound + e_bound + 1, TILE);
  const uint64_t waves = (uint64_t)final_grid(n_bound, e_bound) * WAVES;
  return cdiv(tiles, waves) * WAVES * TILE;
}

uint64_t ws_shard_cap(uint64_t n_bound, uint64_t e_bound) {
  uint64_t tiles = cdiv(n_bound + e_bound + 1, TILE);
  return cdiv(tiles, NSHARD) * TILE;
}

// NBG_FINAL_LEAN=0: the final step of a FINALD-shaped statement runs k_expand<FINALD> instead of
// final.hip's k_final_dst (A/B)
static bool lean_final() {
  static const bool on = !getenv("NBG_FINAL_LEAN") || atoi(getenv("NBG_FINAL_LEAN")) != 0;
  return on;
}

hipError_t ws_expand_final(Workspace* w, const ExpandArgs& a0, uint64_t n_bound, uint64_t e_bound, int step, int tix,
                           const TypeProgram& prog, uint64_t region_base, uint64_t blk_cap, const InlineList* il) {
  if (step > MAX_STEPS || tix >= MAX_TYPES_Q) return hipErrorInvalidValue;
  const bool inl = inline_start_list(w, tix, il);
  const ListRef L = inl ? ListRef{nullptr, nullptr, &w->q->step_n[step], 0} : prepare_list(w, a0, n_bound, step, tix);
  ExpandArgs a = a0;
  a.frontier = L.ids;
  a.tsplit = inl ? nullptr : set_split(w, L.set);
  uint32_t* const l_end = set_end(w, L.set);
  uint32_t* const l_rs = set_rs(w, L.set);
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
  for (int y = 0; y < MAX_YIELDS; ++y) fp.out_cols[y] = ws_row_col(w, y < w->ncols_alloc ? y : 0);
  fp.region_base = region_base;
  fp.blk_cap = blk_cap;
  fp.blk_rows = w->blk_rows + (size_t)tix * EXPAND_GRID;
  fp.err_flag = &w->q->err;
  fp.probe_mask = prog.probe_mask;
  fp.keep_on_error = prog.keep_on_error ? 1 : 0;
  fp.tag_bits = &w->q->tagbits;
  a.str.arena = w->sarena;
  a.str.arena_cap = w->sarena_cap;
  a.str.arena_used = &w->q->arena_used;
  a.str.err_flag = &w->q->err;
  fp.fast = detect_fast(prog, a);
  size_t lds = fp.fast.enabled ? 0 : (size_t)(prog.nregs > 0 ? prog.nregs : 1) * BLOCK * sizeof(int64_t);
  bool dst_only = fp.fast.enabled;   // YIELDs are _dst / constants: the deferred-store instantiation
  for (int y = 0; y < fp.nyields; ++y) dst_only = dst_only && (fp.fast.ykind[y] == 0 || fp.fast.ykind[y] == 4);
  // FINALY: many YIELD columns over a small expansion (getBound-sized: latency-bound, where four
  // columns' loads in flight beat the 8-wave occupancy FINALF keeps for bandwidth-bound steps)
  const bool wide = fp.fast.enabled && !dst_only && fp.nyields >= 4 && e_bound <= (1ull << 20);
  hipEvent_t p = prof_begin(w, K_EXPAND_FINAL);
  const dim3 grid(final_grid(n_bound, e_bound));
  unsigned long long* e_st = &w->q->e_st[step][tix];
  if (inl) {
    if (dst_only)
      hipLaunchKernelGGL((k_expand<FINALD, true>), grid, dim3(BLOCK), 0, w->stream, a, L.acc, l_end, l_rs,
                         w->flags, fp, BfsParams{}, e_st, L.stat_n, *il);
    else if (wide)
      hipLaunchKernelGGL((k_expand<FINALY, true>), grid, dim3(BLOCK), 0, w->stream, a, L.acc, l_end, l_rs,
                         w->flags, fp, BfsParams{}, e_st, L.stat_n, *il);
    else if (fp.fast.enabled)
      hipLaunchKernelGGL((k_expand<FINALF, true>), grid, dim3(BLOCK), 0, w->stream, a, L.acc, l_end, l_rs,
                         w->flags, fp, BfsParams{}, e_st, L.stat_n, *il);
    else
      hipLaunchKernelGGL((k_expand<FINAL, true>), grid, dim3(BLOCK), lds, w->stream, a, L.acc, l_end, l_rs,
                         w->flags, fp, BfsParams{}, e_st, L.stat_n, *il);
  } else if (dst_only && lean_final() && fp.fast.dst_yield && a.dst_vid && (!fp.fast.has_where || fp.fast.wcol)) {
    FinalDstArgs fa{};
    fa.acc = L.acc;
    fa.seg_end = l_end;
    fa.seg_rs = l_rs;
    fa.tsplit = a.tsplit;
    fa.tsplit_n = w->cap_tiles;
    fa.dst_vid = a.dst_vid;
    fa.wcol = fp.fast.wcol;
    fa.lo = fp.fast.lo;
    fa.hi = fp.fast.hi;
    fa.where_neg = fp.fast.where_neg;
    fa.nyields = fp.nyields;
    for (int y = 0; y < fp.nyields; ++y) {
      if (fp.fast.ykind[y] != 0) fa.const_mask |= 1ull << y;
      fa.yconst[y] = fp.yield_const[y];
      fa.out[y] = fp.out_cols[y];
    }
    fa.region_base = region_base;
    fa.blk_cap = blk_cap;
    fa.blk_rows = fp.blk_rows;
    fa.stat_e = e_st;
    fa.stat_n = L.stat_n;
    fa.err_flag = &w->q->err;
    const bool one = fp.nyields == 1 && fa.const_mask == 0;
    const hipError_t le = launch_final_dst(fa, fp.fast.has_where ? fp.fast.wbytes : 0, one, grid.x, w->stream);
    if (le != hipSuccess) {
      prof_end(w, p, K_EXPAND_FINAL, step, tix, 0.0, 0.0);   // (the profile's open event closed)
      return le;
    }
  } else if (dst_only) {
    hipLaunchKernelGGL(k_expand<FINALD>, grid, dim3(BLOCK), 0, w->stream, a, L.acc, l_end, l_rs, w->flags,
                       fp, BfsParams{}, e_st, L.stat_n, NoInline{});
  } else if (wide) {
    hipLaunchKernelGGL(k_expand<FINALY>, grid, dim3(BLOCK), 0, w->stream, a, L.acc, l_end, l_rs, w->flags,
                       fp, BfsParams{}, e_st, L.stat_n, NoInline{});
  } else if (fp.fast.enabled) {
    hipLaunchKernelGGL(k_expand<FINALF>, grid, dim3(BLOCK), 0, w->stream, a, L.acc, l_end, l_rs, w->flags,
                       fp, BfsParams{}, e_st, L.stat_n, NoInline{});
  } else {
    hipLaunchKernelGGL(k_expand<FINAL>, grid, dim3(BLOCK), lds, w->stream, a, L.acc, l_end, l_rs, w->flags,
                       fp, BfsParams{}, e_st, L.stat_n, NoInline{});
  }
  prof_end(w, p, K_EXPAND_FINAL, step, tix, (double)edge_columns_read(prog), (double)fp.nyields);
  w->final_grid[tix] = final_grid(n_bound, e_bound);
  return hipGetLastError();
}



hipError_t ws_backtracker(Workspace* w, int64_t** out, int64_t** in) {
  if (!w->bt) HIP_TRY(hipMalloc((void**)&w->bt, (w->nv + 1) * 8));
  if (w->comm && !w->h_btc) {
    const uint64_t G = (uint64_t)w->comm->world, nwords = G * w->npad / 64;
    if (!w->bt_out) HIP_TRY(hipMalloc((void**)&w->bt_out, G * w->npad * 8));
    if (!w->bt_pack) HIP_TRY(hipMalloc((void**)&w->bt_pack, G * w->npad * 8));
    if (!w->bt_recv) HIP_TRY(hipMalloc((void**)&w->bt_recv, G * w->npad * 8));
    if (!w->bt_pre) HIP_TRY(hipMalloc((void**)&w->bt_pre, 2 * nwords * 4));
    if (!w->bt_boff) HIP_TRY(hipMalloc((void**)&w->bt_boff, 2 * (nwords / RW_BLOCK) * 4));
    if (!w->bt_disp) HIP_TRY(hipMalloc((void**)&w->bt_disp, 2 * G * 8));
    HIP_TRY(hipHostMalloc((void**)&w->h_btc, 2 * G * 8, hipHostMallocMapped | hipHostMallocCoherent));
    HIP_TRY(hipHostGetDevicePointer((void**)&w->d_btc, w->h_btc, 0));
  }
  w->bt_active = true;
  *in = w->bt;
  *out = w->comm ? w->bt_out : w->bt;
  return hipSuccess;
}

void ws_backtracker_off(Workspace* w) { w->bt_active = false; }

// Scan-only expansion (final step whose WHERE folded to false still counts E_N).
hipError_t ws_scan_only(Workspace* w, const ExpandArgs& a, uint64_t n_bound, int step, int tix) {
  const ListRef L = prepare_list(w, a, n_bound, step, tix);
  hipLaunchKernelGGL(k_note, dim3(1), dim3(1), 0, w->stream, L.acc, &w->q->e_st[step][tix], L.stat_n);
  return hipGetLastError();
}




// QState + row counts -> the mapped host mirror with a kernel's stores: a hipMemcpyAsync of these
// ~13 KB took the copy engine's path, ~130 us against ~3 us (profiles/r03_l_d2h_probe.json).
// The host's wake-up at the end of a query's last kernel (called by every thread): each thread's
// stores are released to system scope, then the last workgroup to get here (a ticket, reset for
// the next query) stores seq into the mapped wake word the host polls.  The host so reads the
// results as soon as they are visible, not after the kernel has retired and an event behind it
// has been signalled.
struct Wake {
  unsigned long long* word;   // nullptr: the host waits on an event (NBG_WAKE=event)
  unsigned int* ticket;
  unsigned long long seq;
};
__device__ void wake_host(const Wake& wk) {
  if (!wk.word) return;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // (release only, at system scope: no cache invalidation)
  __syncthreads();
  if (threadIdx.x != 0) return;
  if (gridDim.x > 1) {
    const unsigned got = __hip_atomic_fetch_add(wk.ticket, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    if (got != gridDim.x - 1) return;
    // the last workgroup acquires what the others released with their tickets, so its system-scope
    // release of the wake word below covers every workgroup's host stores (cumulativity); one
    // acquire per launch, not one per workgroup
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    __hip_atomic_store(wk.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __hip_atomic_store(wk.word, wk.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// (the QState words, the first nq8, are zeroed behind the copy for the next query: no host
// memset call after the wait)
__global__ void __launch_bounds__(BLOCK) k_q_out(unsigned long long* __restrict__ src, unsigned long long* dst,
                                                 uint32_t n8, uint32_t nq8, Wake wk) {
  for (uint32_t i = threadIdx.x; i < n8; i += BLOCK) {
    dst[i] = src[i];
    if (i < nq8) src[i] = 0;
  }
  wake_host(wk);
}

static bool wake_by_flag() {   // (NBG_BLOCKING_SYNC: blocking waits, no polling)
  static const bool on = !(getenv("NBG_WAKE") && strcmp(getenv("NBG_WAKE"), "event") == 0) &&
                         getenv("NBG_BLOCKING_SYNC") == nullptr;
  return on;
}

// the Wake of the end kernel being enqueued (arms the host's poll)
static Wake arm_wake(Workspace* w) {
  w->wake_armed = wake_by_flag() && w->wake_flag && !w->comm;
  if (!w->wake_armed) return Wake{nullptr, nullptr, 0};
  return Wake{w->d_wake, w->d_ticket, ++w->wake_seq};
}

// Poll the wake word; the event behind the end kernel is looked at now and then, so a failed
// launch or a faulted kernel still ends the wait with its error.
static hipError_t wait_wake(Workspace* w) {
  const unsigned long long want = w->wake_seq;
  for (unsigned k = 1;; ++k) {
    if (__atomic_load_n(w->h_wake, __ATOMIC_ACQUIRE) == want) {
      (void)hipEventQuery(w->done_ev);   // (lets the runtime retire what it has finished: without
      return hipSuccess;                 // it, six queries in flight ran ~1.5 % slower)
    }
    if ((k & 255) == 0) {
      const hipError_t e = hipEventQuery(w->done_ev);
      if (e == hipErrorNotReady) continue;
      if (__atomic_load_n(w->h_wake, __ATOMIC_ACQUIRE) == want) return hipSuccess;
      return e == hipSuccess ? hipErrorLaunchFailure : e;   // (completed without the store: a bug)
    }
  }
}

// The end of a query in two halves: the QState / row-count store into host memory and an event
// behind it (async), then the wait for that event and the reset of QState for the next query.
hipError_t ws_end_query_async(Workspace* w) {
  int nt = 0;
  for (int t = 0; t < MAX_TYPES_Q; ++t)
    if (w->final_grid[t]) nt = t + 1;
  static_assert(sizeof(QState) % 8 == 0 && EXPAND_GRID % 2 == 0, "k_q_out copies 8-byte words");
  const size_t bytes = sizeof(QState) + (size_t)nt * EXPAND_GRID * 4;
  const Wake wk = arm_wake(w);
  hipLaunchKernelGGL(k_q_out, dim3(1), dim3(BLOCK), 0, w->stream, reinterpret_cast<unsigned long long*>(w->q),
                     reinterpret_cast<unsigned long long*>(w->d_hq), (uint32_t)(bytes / 8),
                     (uint32_t)(sizeof(QState) / 8), wk);
  w->q_reset = true;
  HIP_TRY(hipGetLastError());
  if (w->h_small) w->h_small[0] = 0;   // (this query's rows are not packed: the device does not run
                                       // ahead of this host write, the stream is idle on this slot)
  if (!w->done_ev) HIP_TRY(hipEventCreateWithFlags(&w->done_ev, hipEventDisableTiming));
  return hipEventRecord(w->done_ev, w->stream);
}

hipError_t ws_end_query_wait(Workspace* w) {
  static const bool blocking = getenv("NBG_BLOCKING_SYNC") != nullptr;
  if (w->comm) {
    HIP_TRY(ws_sync(w));   // bounded: a peer that never arrives aborts the communicator
  } else if (w->wake_armed) {
    w->wake_armed = false;
    HIP_TRY(wait_wake(w));
  } else if (blocking) {
    HIP_TRY(hipEventSynchronize(w->done_ev));
  } else {
    hipError_t e;
    while ((e = hipEventQuery(w->done_ev)) == hipErrorNotReady) {
    }
    HIP_TRY(e);
  }
  // reset for the next query (done by the end kernel itself, unless this query had none)
  if (!w->q_reset) HIP_TRY(hipMemsetAsync(w->q, 0, sizeof(QState), w->stream));
  w->q_reset = false;
  prof_flush(w, w->h_q);
  return hipSuccess;
}

// k_q_out, then (one workgroup) the result's rows into the mapped small-rows buffer when they fit:
// segment (type t, block b) = rows [region_t + b * blk_cap_t, + count) of every column, packed in
// (t, b) order at column-major offsets, as nbg_rows / ws_fetch_rows lay them out.  The non-empty
// segments are listed first (block scans over the row counts, in order), then each is copied by
// the whole workgroup, one cell per thread (column-major within the segment); a result with more
// than SMALL_SEGS non-empty segments is left to the host fetch like a large one.
constexpr int SMALL_SEGS = 2048;
constexpr int SMALL_WGS = 16;
__global__ void __launch_bounds__(BLOCK) k_q_out_small(unsigned long long* __restrict__ src, unsigned long long* dst,
                                                       uint32_t n8, uint32_t nq8, const uint32_t* __restrict__ blk_rows, SmallPack sp,
                                                       int64_t* const* __restrict__ cols, int64_t* small, Wake wk) {
  // (every workgroup lists the segments; workgroup b copies segments b, b + grid, ... and a share
  // of the state words: more stores over the host link in flight than one workgroup issues)
  // (the QState words, the first nq8, zeroed behind the copy as in k_q_out; the row counts after
  // them are read below and rewritten by the next final step)
  for (uint32_t i = blockIdx.x * BLOCK + threadIdx.x; i < n8; i += gridDim.x * BLOCK) {
    dst[i] = src[i];
    if (i < nq8) src[i] = 0;
  }
  __shared__ uint32_t s_seg[SMALL_SEGS];        // t << 16 | b of the non-empty segments, in order
  __shared__ uint32_t s_off[SMALL_SEGS + 1];    // their first row in the packed result
  __shared__ uint32_t s_lds[WAVES];
  __shared__ uint32_t s_n, s_rows;
  if (threadIdx.x == 0) s_n = s_rows = 0;
  __syncthreads();
  // thread k takes the SMALL_PER consecutive segments [k * SMALL_PER, ...) of each type: one
  // pair of block scans per type lists them in order
  constexpr int SMALL_PER = EXPAND_GRID / BLOCK;
  static_assert(EXPAND_GRID % BLOCK == 0, "segments split evenly over the threads");
  bool over = false;
  for (int t = 0; t < sp.ntypes && !over; ++t) {
    uint32_t nn[SMALL_PER], cn = 0, cr = 0;
    const uint32_t b0 = threadIdx.x * SMALL_PER;
#pragma unroll
    for (int k = 0; k < SMALL_PER; ++k) {
      nn[k] = b0 + k < sp.grid[t] ? blk_rows[(size_t)t * EXPAND_GRID + b0 + k] : 0u;
      cn += nn[k] ? 1u : 0u;
      cr += nn[k];
    }
    uint32_t tn = 0, tr = 0;
    uint32_t xn = block_excl_scan<BLOCK>(cn, &tn, s_lds);
    uint32_t xr = block_excl_scan<BLOCK>(cr, &tr, s_lds);
    const uint32_t base_n = s_n, base_r = s_rows;
    if (base_n + tn > SMALL_SEGS) {   // (uniform)
      over = true;
      break;
    }
#pragma unroll
    for (int k = 0; k < SMALL_PER; ++k) {
      if (!nn[k]) continue;
      s_seg[base_n + xn] = ((uint32_t)t << 16) | (b0 + k);
      s_off[base_n + xn] = base_r + xr;
      ++xn;
      xr += nn[k];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      s_n = base_n + tn;
      s_rows = base_r + tr;
    }
    __syncthreads();
  }
  const uint64_t total = s_rows;
  if (over || total * (uint64_t)sp.ncols > SMALL_ROWS_WORDS) {
    if (blockIdx.x == 0 && threadIdx.x == 0) small[0] = 0;
    wake_host(wk);
    return;
  }
  const uint32_t nseg = s_n;
  if (threadIdx.x == 0) s_off[nseg] = (uint32_t)total;
  __syncthreads();
  // the packed cells split evenly over every workgroup's threads (a small result has few
  // segments: a workgroup per segment left most of the grid idle and each thread a long chain of
  // reads); cell k = column c, packed row r, found in the segment list by a binary search in LDS
  const uint32_t rows = (uint32_t)total, cells = rows * (uint32_t)sp.ncols;
  for (uint32_t k = blockIdx.x * BLOCK + threadIdx.x; k < cells; k += gridDim.x * BLOCK) {
    const uint32_t c = k / rows, r = k - c * rows;
    uint32_t lo = 0, hi = nseg;   // the last segment whose first packed row is <= r
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (s_off[mid] <= r) lo = mid;
      else hi = mid;
    }
    const uint32_t t = s_seg[lo] >> 16, b = s_seg[lo] & 0xFFFFu;
    small[1 + (uint64_t)k] = cols[c][sp.region[t] + (uint64_t)b * sp.blk_cap[t] + (r - s_off[lo])];
  }
  // (the host reads the block after the wake or the kernel's completion: any workgroup may mark it)
  if (blockIdx.x == 0 && threadIdx.x == 0) small[0] = (int64_t)total + 1;
  wake_host(wk);
}

hipError_t ws_end_query_async_small(Workspace* w, const SmallPack& sp) {
  if (sp.ntypes > MAX_TYPES_Q || sp.ncols > MAX_YIELDS) return hipErrorInvalidValue;
  int nt = 0;
  for (int t = 0; t < MAX_TYPES_Q; ++t)
    if (w->final_grid[t]) nt = t + 1;
  const size_t bytes = sizeof(QState) + (size_t)nt * EXPAND_GRID * 4;
  const Wake wk = arm_wake(w);
  hipLaunchKernelGGL(k_q_out_small, dim3(SMALL_WGS), dim3(BLOCK), 0, w->stream, reinterpret_cast<unsigned long long*>(w->q),
                     reinterpret_cast<unsigned long long*>(w->d_hq), (uint32_t)(bytes / 8),
                     (uint32_t)(sizeof(QState) / 8), w->blk_rows, sp, (int64_t* const*)w->d_row_cols, w->d_small, wk);
  w->q_reset = true;
  HIP_TRY(hipGetLastError());
  if (!w->done_ev) HIP_TRY(hipEventCreateWithFlags(&w->done_ev, hipEventDisableTiming));
  return hipEventRecord(w->done_ev, w->stream);
}

const int64_t* ws_host_small_rows(Workspace* w, uint64_t count) {
  if (!w->h_small || w->h_small[0] != (int64_t)count + 1) return nullptr;
  return w->h_small + 1;
}

hipError_t ws_end_query(Workspace* w) {
  HIP_TRY(ws_end_query_async(w));
  return ws_end_query_wait(w);
}

// ----------------------------------------------------------------------------- tiny GO queries
// A GO N STEPS whose whole expansion is small (the host bounds it before launching: at most
// TINY_EDGES edge visits over all steps, nbg::tiny_bound) runs as ONE workgroup in ONE launch:
// the per-step sets in LDS (an open-addressing table), the final step's WHERE / YIELD through the
// interpreter, and the QState, row count and rows stored straight into the mapped host block the
// multi-launch path's k_q_out_small fills — the same host code reads them (go_collect,
// materialize_rows).  A query that small spends its time on launches and round trips
// (GoExecutor.cpp:410-474 per hop), so one launch and one wait are the whole query.
struct TinyParams {
  ExpandArgs a;
  const Ins* prog;
  int where_len, where_reg, prog_len, nyields;
  int yield_reg[MAX_YIELDS];
  int64_t yield_const[MAX_YIELDS];
  uint32_t probe_mask;
  uint32_t steps, n0;
  uint32_t start[INLINE_STARTS];
  int64_t* const* cols;            // the workspace's row columns (device)
  unsigned long long* hq;          // mapped: QState, then the per-workgroup row counts
  int64_t* small;                  // mapped: [0] = rows + 1, then the cells column by column
  Wake wk;
};

constexpr uint32_t TINY_HASH = 2 * TINY_EDGES;   // set slots (power of two, half full at most)

__global__ void __launch_bounds__(BLOCK) k_go_tiny(TinyParams t) {
  __shared__ uint32_t sF[2][TINY_EDGES + INLINE_STARTS];   // frontier (entry ids) of this / the next step
  __shared__ uint32_t sEnd[TINY_EDGES + INLINE_STARTS];    // inclusive prefix of the capped degrees
  __shared__ uint32_t sRs[TINY_EDGES + INLINE_STARTS];
  __shared__ uint32_t sSet[TINY_HASH];
  __shared__ uint32_t sScan[BLOCK / 64];
  __shared__ uint32_t sNext, sRows;
  __shared__ unsigned long long sStepN[MAX_STEPS + 2], sStepE[MAX_STEPS + 2];
  __shared__ uint32_t sErr, sTags;
  extern __shared__ int64_t regs[];   // [nregs][BLOCK], run_program's registers
  const ExpandArgs& a = t.a;
  const DegSrc ds{a.row_ptr, a.visible, a.cap};
  const int tid = threadIdx.x;
  uint32_t n = t.n0, cur = 0;
  for (uint32_t i = tid; i < n; i += BLOCK) sF[0][i] = t.start[i];
  if (tid == 0) {
    sErr = 0;
    sTags = 0;
    sRows = 0;
  }
  for (int s = tid; s < MAX_STEPS + 2; s += BLOCK) sStepN[s] = sStepE[s] = 0;
  __syncthreads();
  bool anyErr = false;
  uint32_t tbits = 0;
  for (uint32_t step = 1; step <= t.steps; ++step) {
    const bool final = step == t.steps;
    // the frontier's edge space: capped degrees, prefix, row starts (entries in chunks of BLOCK)
    uint32_t total = 0;
    for (uint32_t b = 0; b < n; b += BLOCK) {
      uint32_t rs = 0, d = 0;
      if (b + tid < n) d = vdeg(ds, sF[cur][b + tid], &rs);
      uint32_t tot = 0;
      const uint32_t x = block_excl_scan(d, &tot, sScan);
      if (b + tid < n) {
        sEnd[b + tid] = total + x + d;
        sRs[b + tid] = rs;
      }
      total += tot;
    }
    if (tid == 0) {
      sStepN[step] = n;
      sStepE[step] = total;
      sNext = 0;
    }
    if (!final)
      for (uint32_t k = tid; k < TINY_HASH; k += BLOCK) sSet[k] = 0;
    __syncthreads();
    // every edge of the frontier: its entry by binary search over the prefix
    for (uint32_t e0 = 0; e0 < total; e0 += BLOCK) {
      const uint32_t e = e0 + tid;
      const bool act = e < total;
      uint32_t lo = 0, hi = n;
      while (act && lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (sEnd[mid] <= e) lo = mid + 1;
        else hi = mid;
      }
      const uint32_t ent = act ? lo : 0;
      const uint32_t v = act ? sF[cur][ent] : 0;
      const uint32_t start = (act && ent) ? sEnd[ent - 1] : 0;
      const uint64_t j = act ? (uint64_t)sRs[ent] + (e - start) : 0;
      if (!final) {
        // the per-step SET of destinations (GoExecutor::getDstIdsFromResp)
        const uint32_t u = act ? a.col[j] : NO_ROW;
        if (u != NO_ROW) {
          uint32_t h = (u * 2654435761u) & (TINY_HASH - 1);
          for (uint32_t probe = 0; probe < TINY_HASH; ++probe) {   // (at most half full: the host's bound)
            const uint32_t old = atomicCAS(&sSet[h], 0u, u + 1);
            if (old == 0) {
              const uint32_t at = atomicAdd(&sNext, 1u);
              if (at < TINY_EDGES + INLINE_STARTS) sF[cur ^ 1][at] = u;   // (the host's bound: always)
              break;
            }
            if (old == u + 1) break;
            h = (h + 1) & (TINY_HASH - 1);
          }
        }
        continue;
      }
      // the final step: the holder's tags, WHERE, YIELD (as k_expand<FINAL>)
      if (act && t.probe_mask) {
        const uint32_t d = a.col[j];
        if (d != NO_ROW)
          for (uint32_t m = t.probe_mask; m; m &= m - 1) {
            const int tg = __builtin_ctz(m);
            if (a.tpres[tg][d]) tbits |= 1u << tg;
          }
      }
      const EdgeCtx c{j, v};
      bool pass = act;
      if (t.where_reg >= 0) {
        bool werr = false;
        run_program(t.prog, t.prog + t.prog_len, 0, t.where_len, c, a, regs, act, werr, tbits);
        pass = act && !werr && regs[t.where_reg * BLOCK + tid] != 0;
        if (act && werr) anyErr = true;
      }
      bool yerr = false;
      run_program(t.prog, t.prog + t.prog_len, t.where_len, t.prog_len, c, a, regs, pass, yerr, tbits);
      if (pass && yerr) anyErr = true;
      if (pass) {
        const uint32_t row = atomicAdd(&sRows, 1u);
        if (row >= TINY_EDGES) continue;   // (the host's bound: never)
        for (int y = 0; y < t.nyields; ++y) {
          const int r = t.yield_reg[y];
          t.cols[y][row] = r >= 0 ? regs[r * BLOCK + tid] : t.yield_const[y];
        }
      }
    }
    __syncthreads();
    n = min(sNext, TINY_EDGES + INLINE_STARTS);
    cur ^= 1;
  }
  if (anyErr) atomicOr(&sErr, 1u);
  if (tbits) atomicOr(&sTags, tbits);
  __syncthreads();
  // QState (every word: the fields go_collect reads, the rest zero), then one workgroup's row count
  const uint32_t nrows = min(sRows, TINY_EDGES);
  constexpr uint32_t NQ = sizeof(QState) / 8;
  for (uint32_t k = tid; k < NQ; k += BLOCK) {
    unsigned long long x = 0;
    if (k == offsetof(QState, err) / 8) x = sErr;
    else if (k == offsetof(QState, tagbits) / 8) x = sTags;
    else if (k >= offsetof(QState, step_n) / 8 && k < offsetof(QState, step_n) / 8 + MAX_STEPS + 2)
      x = sStepN[k - offsetof(QState, step_n) / 8];
    else if (k >= offsetof(QState, e_st) / 8 && k < offsetof(QState, e_st) / 8 + (MAX_STEPS + 2) * MAX_TYPES_Q) {
      const uint32_t o = k - (uint32_t)(offsetof(QState, e_st) / 8);
      x = o % MAX_TYPES_Q == 0 ? sStepE[o / MAX_TYPES_Q] : 0ull;
    }
    t.hq[k] = x;
  }
  if (tid == 0) reinterpret_cast<uint32_t*>(t.hq + NQ)[0] = nrows;
  // the rows, column by column, then the count that makes them valid
  const bool fits = (uint64_t)nrows * t.nyields <= SMALL_ROWS_WORDS;
  for (int y = 0; fits && y < t.nyields; ++y)
    for (uint32_t i = tid; i < nrows; i += BLOCK) t.small[1 + (uint64_t)y * nrows + i] = t.cols[y][i];
  __syncthreads();
  if (tid == 0) t.small[0] = fits ? (int64_t)nrows + 1 : 0;
  wake_host(t.wk);
}

// Walk bounds of one CSR for the tiny path: W_k(v) = deg(v) + sum over v's (capped) edges of
// W_{k-1}(neighbour), W_1 = deg (capped, 0 when invisible), saturated at TINY_EDGES + 1 (a vertex
// past it is not tiny, so a row longer than that is not read).
__global__ void __launch_bounds__(BLOCK) k_walk_bound(const uint32_t* __restrict__ row_ptr, const uint32_t* __restrict__ col,
                                                      const uint8_t* __restrict__ visible, uint32_t cap, uint64_t nv,
                                                      const uint16_t* __restrict__ prev, uint16_t* __restrict__ out) {
  const uint64_t v = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (v >= nv) return;
  constexpr uint32_t SAT = TINY_EDGES + 1;
  uint32_t deg = 0;
  if (!visible || visible[v]) {
    deg = row_ptr[v + 1] - row_ptr[v];
    deg = deg < cap ? deg : cap;
  }
  uint32_t w = deg < SAT ? deg : SAT;
  if (prev && w < SAT) {
    const uint32_t rs = row_ptr[v];
    for (uint32_t k = 0; k < deg && w < SAT; ++k) {
      const uint32_t u = col[rs + k];
      if (u != NO_ROW) w += prev[u];
    }
  }
  out[v] = (uint16_t)(w < SAT ? w : SAT);
}

hipError_t tiny_bounds(const uint32_t* row_ptr, const uint32_t* col, const uint8_t* visible, uint32_t cap, uint64_t nv,
                       std::vector<uint16_t>* w2, std::vector<uint16_t>* w3, hipStream_t s) {
  w2->clear();
  w3->clear();
  if (!nv) return hipSuccess;
  uint16_t* d = nullptr;
  HIP_TRY(hipMalloc((void**)&d, nv * 3 * sizeof(uint16_t)));
  const dim3 g((unsigned)((nv + BLOCK - 1) / BLOCK));
  hipLaunchKernelGGL(k_walk_bound, g, dim3(BLOCK), 0, s, row_ptr, col, visible, cap, nv, (const uint16_t*)nullptr, d);
  hipLaunchKernelGGL(k_walk_bound, g, dim3(BLOCK), 0, s, row_ptr, col, visible, cap, nv, (const uint16_t*)d, d + nv);
  hipLaunchKernelGGL(k_walk_bound, g, dim3(BLOCK), 0, s, row_ptr, col, visible, cap, nv, (const uint16_t*)(d + nv),
                     d + 2 * nv);
  hipError_t e = hipGetLastError();
  w2->resize(nv);
  w3->resize(nv);
  if (e == hipSuccess) e = hipMemcpyAsync(w2->data(), d + nv, nv * 2, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipMemcpyAsync(w3->data(), d + 2 * nv, nv * 2, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  (void)hipFree(d);
  if (e != hipSuccess) {
    w2->clear();
    w3->clear();
  }
  return e;
}

hipError_t ws_go_tiny(Workspace* w, const ExpandArgs& a, const uint32_t* starts, uint32_t n, uint32_t steps,
                      const TypeProgram& prog, int ncols) {
  if (n > INLINE_STARTS || steps < 1 || steps > MAX_STEPS || ncols > MAX_YIELDS || ncols < 1) return hipErrorInvalidValue;
  HIP_TRY(ws_reserve_rows(w, TINY_EDGES, ncols));
  TinyParams t{};
  t.a = a;
  t.prog = w->d_prog;
  t.where_len = prog.where_len;
  t.where_reg = prog.where_reg;
  t.prog_len = (int)prog.code.size();
  t.nyields = (int)prog.yield_reg.size();
  for (int y = 0; y < t.nyields; ++y) {
    t.yield_reg[y] = prog.yield_reg[y];
    t.yield_const[y] = prog.yield_const[y];
  }
  t.probe_mask = prog.probe_mask;
  t.steps = steps;
  t.n0 = n;
  for (uint32_t i = 0; i < n; ++i) t.start[i] = starts[i];
  t.cols = (int64_t* const*)w->d_row_cols;
  t.hq = reinterpret_cast<unsigned long long*>(w->d_hq);
  t.small = w->d_small;
  t.wk = arm_wake(w);
  for (auto& g : w->final_grid) g = 0;
  w->final_grid[0] = 1;   // (one workgroup's rows: go_collect reads one count)
  const size_t lds = (size_t)(prog.nregs > 0 ? prog.nregs : 1) * BLOCK * sizeof(int64_t);
  hipLaunchKernelGGL(k_go_tiny, dim3(1), dim3(BLOCK), lds, w->stream, t);
  HIP_TRY(hipGetLastError());
  if (!w->done_ev) HIP_TRY(hipEventCreateWithFlags(&w->done_ev, hipEventDisableTiming));
  return hipEventRecord(w->done_ev, w->stream);
}

// ----------------------------------------------------------------------------- partitioned mode
hipError_t ws_set_partition(Workspace* w, Comm* comm, uint64_t npad) {
  if (!comm || npad % PART_ALIGN || PART_ALIGN % BITS_BLOCK || PART_ALIGN % FLAG_ALIGN) return hipErrorInvalidValue;
  const uint64_t G = (uint64_t)comm->world;
  HIP_TRY(ws_sync(w));
  w->comm = comm;
  w->npad = npad;
  if (w->flags) HIP_TRY(hipFree(w->flags));
  w->flags = nullptr;
  w->flag_bytes = G * npad;                     // multiple of FLAG_ALIGN (PART_ALIGN is)
  HIP_TRY(hipMalloc((void**)&w->flags, w->flag_bytes));
  HIP_TRY(hipMemsetAsync(w->flags, 0, w->flag_bytes, w->stream));
  HIP_TRY(hipMalloc((void**)&w->sendbits, G * npad / 8));
  HIP_TRY(hipMemsetAsync(w->sendbits, 0, G * npad / 8, w->stream));   // all-zero between hops
  HIP_TRY(hipMalloc((void**)&w->recvbits, G * npad / 8));
  HIP_TRY(hipMalloc((void**)&w->gst, (GST_N + G) * sizeof(unsigned long long)));
  HIP_TRY(hipHostMalloc((void**)&w->h_gst, (GST_N + G) * sizeof(unsigned long long), hipHostMallocDefault));
  return ws_sync(w);
}

// A rank whose preparation of a query failed still takes part in the query's collectives (the
// fast path of a partitioned GO, engine.cpp go_launch): `hops` all-to-alls of the zero bitmap
// `send0` (G segments of seg_bytes; received into `recv`, never read), then the statistics
// all-reduce with zero statistics and its status word.  Synchronous; *agreed = the first failing
// rank's status.
hipError_t part_empty_query(Comm* c, hipStream_t s, int hops, const void* send0, void* recv, size_t seg_bytes,
                            size_t first_bytes, unsigned long long* gst, unsigned long long* h_gst, int32_t status,
                            int32_t* agreed) {
  const int G = c->world;
  for (int h = 0; h < hops; ++h)   // (the first hop may be a slot exchange: first_bytes per peer)
    if (c->alltoall(send0, recv, h == 0 && first_bytes ? first_bytes : seg_bytes, s)) return hipErrorUnknown;
  HIP_TRY(hipMemsetAsync(gst, 0, GST_N * sizeof(unsigned long long), s));
  hipLaunchKernelGGL(k_gst_status, dim3(1), dim3(64), 0, s, gst, G, c->rank, (long long)status);
  HIP_TRY(hipGetLastError());
  if (c->allreduce_sum_u64(gst, GST_N + G, s)) return hipErrorUnknown;
  HIP_TRY(hipMemcpyAsync(h_gst, gst, (GST_N + G) * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
  if (c->wait(s)) return hipErrorUnknown;
  *agreed = NBG_OK;
  for (int r = 0; r < G; ++r)
    if (h_gst[GST_N + r]) {
      *agreed = (int32_t)(long long)h_gst[GST_N + r];
      break;
    }
  return hipSuccess;
}
size_t part_gst_words(int world) { return (size_t)GST_N + (size_t)world; }

// After all OVER types of a non-final step marked their candidates (global ids) in the flags:
// pack -> all-to-all of npad-bit segments -> owner OR + compaction into the next local frontier.
Comm* ws_get_comm(const Workspace* w) { return w ? w->comm : nullptr; }
hipStream_t ws_stream(const Workspace* w) { return w->stream; }

// The hop's roots: only those of the vertices whose bits this rank sends, packed per destination
// in bit order, so a hop moves 8 bytes per sent vertex beside the bitmap instead of npad * 8 per
// peer.  RCCL's send/recv counts are host values: the per-rank counts (popcounts of the send and
// received bitmaps) come back through mapped memory with one host wait per hop — such queries
// already agree on their inputs before the first hop, so their hops are host-paced anyway.
static hipError_t ws_roots(Workspace* w, int step) {
  const int G = w->comm->world;
  const uint64_t nwords = (uint64_t)G * w->npad / 64, seg_words = w->npad / 64;
  const uint64_t nb = nwords / RW_BLOCK, spb = seg_words / RW_BLOCK;
  hipEvent_t p = prof_begin(w, K_ROOTS);
  hipLaunchKernelGGL(k_rt_prefix, dim3((unsigned)(2 * nb)), dim3(BLOCK), 0, w->stream, w->sendbits, w->recvbits, nb,
                     w->bt_pre, w->bt_boff);
  hipLaunchKernelGGL(k_rt_offsets, dim3(1), dim3(BLOCK), 0, w->stream, w->bt_boff, spb, G, w->bt_disp, w->d_btc);
  HIP_TRY(hipGetLastError());
  HIP_TRY(ws_sync(w));
  std::vector<uint64_t> sc(w->h_btc, w->h_btc + G), rc(w->h_btc + G, w->h_btc + 2 * G), sd(G), rd(G);
  uint64_t ts = 0, tr = 0, moved = 0;
  for (int q = 0; q < G; ++q) {
    sd[q] = ts;
    rd[q] = tr;
    ts += sc[q];
    tr += rc[q];
    if (q != w->comm->rank) moved += sc[q] * 8;
  }
  hipLaunchKernelGGL(k_rt_pack, dim3((unsigned)cdiv(nwords, BLOCK)), dim3(BLOCK), 0, w->stream, w->sendbits, nwords,
                     seg_words, w->bt_pre, w->bt_boff, w->bt_disp, w->bt_out, w->bt_pack);
  HIP_TRY(hipGetLastError());
  if (w->comm->alltoallv(w->bt_pack, sc.data(), sd.data(), w->bt_recv, rc.data(), rd.data(), 8, w->stream))
    return hipErrorUnknown;
  prof_end(w, p, K_ROOTS, step, 0, (double)moved);
  return hipSuccess;
}

// Every rank calls it before the hop's MARKs, a rank without edges of the OVER type (no MARK)
// too: its slots are empty (NO_ROW) and ws_exchange takes the slot format on every rank.  (Round 6
// first set the format and the NO_ROW fill inside the MARK: a part-less rank then sent its
// all-zero bitmap, which the owners read as local id 0 — an extra vertex on every rank — and
// exchanged bitmap-sized segments while its peers exchanged slots.)
hipError_t ws_set_hop_slots(Workspace* w, uint64_t stride) {
  if (!w) return hipErrorInvalidValue;
  w->hop_slots = stride && w->comm && stride * 4 * 2 <= w->npad / 8 ? stride : 0;
  if (!w->hop_slots) return hipSuccess;
  return hipMemsetAsync(w->sendbits, 0xFF, (uint64_t)w->comm->world * w->hop_slots * 4, w->stream);
}

hipError_t ws_exchange(Workspace* w, int step, const ExpandArgs* next0) {
  if (!w->comm) return hipErrorInvalidValue;
  const uint64_t G = (uint64_t)w->comm->world;
  const uint64_t nwords = G * w->npad / 64, seg_words = w->npad / 64, nb = w->npad / BITS_BLOCK;
  hipEvent_t p = nullptr;
  if (w->hop_slots && !w->bt_active) {
    // a small hop's slot arrays: stride ids per peer instead of npad / 8 bytes; the owner claims
    // the arrivals against the step's stamp (a vertex may arrive from several edges and ranks)
    const uint64_t stride = w->hop_slots;
    w->hop_slots = 0;
    w->hop_bits = false;
    p = prof_begin(w, K_ALLTOALL);
    if (w->comm->alltoall(w->sendbits, w->recvbits, stride * 4, w->stream)) return hipErrorUnknown;
    prof_end(w, p, K_ALLTOALL, step, 0, (double)((G - 1) * stride * 4));
    HIP_TRY(hipMemsetAsync(w->sendbits, 0, G * stride * 4, w->stream));   // (all-zero between hops)
    if (++w->seen_stamp == 0) {   // wrap: clear the stamps once
      HIP_TRY(hipMemsetAsync(w->seen, 0, (w->nv + 1) * 4, w->stream));
      w->seen_stamp = 1;
    }
    unsigned long long* acc = &w->q->acc[2 + w->pc];
    unsigned long long* other = &w->q->acc[2 + (w->pc ^ 1)];
    w->pc ^= 1;
    p = prof_begin(w, K_BITS_COMPACT);
    hipLaunchKernelGGL(k_slots_compact, dim3((unsigned)cdiv(G * stride, (uint64_t)BLOCK * SC_ITEMS)), dim3(BLOCK), 0,
                       w->stream, reinterpret_cast<const uint32_t*>(w->recvbits), G * stride, w->seen, w->seen_stamp,
                       w->nv, deg_src(next0), list_out(w, w->frontier[w->cur ^ 1], acc, other, nullptr, w->cur ^ 1));
    prof_end(w, p, K_BITS_COMPACT, step, 0);
    w->cur ^= 1;
    w->list_acc = acc;
    w->seg_ready = next0 != nullptr;
    return hipGetLastError();
  }
  w->hop_slots = 0;
  if (!w->hop_bits) {   // byte flags (MARKB): pack them into the send bitmap
    p = prof_begin(w, K_PACK);
    hipLaunchKernelGGL(k_pack_bits, dim3((unsigned)cdiv(nwords, BLOCK)), dim3(BLOCK), 0, w->stream, w->flags, nwords,
                       w->sendbits);
    prof_end(w, p, K_PACK, step, 0, (double)(G * w->npad) + (double)(G * w->npad / 8));
    HIP_TRY(hipGetLastError());
  }
  w->hop_bits = false;
  p = prof_begin(w, K_ALLTOALL);
  if (w->comm->alltoall(w->sendbits, w->recvbits, w->npad / 8, w->stream)) return hipErrorUnknown;
  prof_end(w, p, K_ALLTOALL, step, 0, (double)((G - 1) * w->npad / 8));
  RootsIn rt{};
  if (w->bt_active) {
    HIP_TRY(ws_roots(w, step));
    rt = RootsIn{w->bt_recv, w->bt_pre, w->bt_boff, w->bt_disp, nwords};
  }
  // the send bitmap is all-zero between hops (the next hop's MARKs OR into it)
  HIP_TRY(hipMemsetAsync(w->sendbits, 0, G * w->npad / 8, w->stream));
  unsigned long long* acc = &w->q->acc[2 + w->pc];
  unsigned long long* other = &w->q->acc[2 + (w->pc ^ 1)];
  w->pc ^= 1;
  p = prof_begin(w, K_BITS_COMPACT);
  hipLaunchKernelGGL(k_bits_compact, dim3((unsigned)nb), dim3(BLOCK), 0, w->stream, w->recvbits, (int)G, seg_words,
                     w->nv, deg_src(next0), list_out(w, w->frontier[w->cur ^ 1], acc, other, nullptr, w->cur ^ 1),
                     rt, w->bt);
  prof_end(w, p, K_BITS_COMPACT, step, 0);
  w->cur ^= 1;
  w->list_acc = acc;
  w->seg_ready = next0 != nullptr;
  return hipGetLastError();
}

// Global query statistics (err flag, |F_s|, E_s summed over ranks), synchronised with the query
// end; valid in ws_host_gstats() after ws_end_query.
hipError_t ws_global_stats(Workspace* w, int ntypes) {
  if (!w->comm) return hipErrorInvalidValue;
  const int G = w->comm->world;
  hipLaunchKernelGGL(k_gstats, dim3(1), dim3(64), 0, w->stream, w->q, ntypes, w->gst);
  HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL(k_gst_status, dim3(1), dim3(64), 0, w->stream, w->gst, G, w->comm->rank, 0ll);
  HIP_TRY(hipGetLastError());
  if (w->comm->allreduce_sum_u64(w->gst, GST_N + G, w->stream)) return hipErrorUnknown;
  return hipMemcpyAsync(w->h_gst, w->gst, (GST_N + G) * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                        w->stream);
}

// the first failing rank's status word of the last query's statistics (NBG_OK: none failed)
int32_t ws_host_gstatus(Workspace* w) {
  if (!w->comm) return NBG_OK;
  for (int r = 0; r < w->comm->world; ++r)
    if (w->h_gst[GST_N + r]) return (int32_t)(long long)w->h_gst[GST_N + r];
  return NBG_OK;
}

void ws_host_gstats(Workspace* w, unsigned long long* err, unsigned long long* step_n, unsigned long long* esum,
                    unsigned long long* tagbits) {
  *err = w->h_gst[0];
  *tagbits = 0;
  for (int b = 0; b < 2 * MAX_TAG_BITS; ++b)
    if (w->h_gst[GST_N0 + b]) *tagbits |= 1ull << b;
  for (int s = 0; s < MAX_STEPS + 2; ++s) {
    step_n[s] = w->h_gst[1 + s];
    esum[s] = w->h_gst[1 + (MAX_STEPS + 2) + s];
  }
}


// ============================================================================= FIND SHORTEST PATH
// Bidirectional BFS over epoch-stamped labels (path.cpp drives it level by level):
//   k_expand<BFS>  claims neighbours (CAS on the label), detects meets, appends to claim shards
//   (claims append straight to the next frontier slot, one atomic per wave tile)
//   k_degsum       degree sum of a frontier (which side to expand next)
//   k_stamp        label a list (sources, targets, level-0 vertices)
//   k_greedy_start / k_greedy_hop  lexicographically smallest shortest path through the B-sets
//                  (one launch per hop; a hop's adjacency is scanned by GREEDY_HOP_BLOCKS workgroups)

__global__ void __launch_bounds__(BLOCK) k_stamp(const uint32_t* __restrict__ ids,
                                                 const unsigned long long* __restrict__ np,
                                                 uint32_t* __restrict__ lab, uint32_t stamp) {
  const uint64_t n = *np;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (uint64_t)gridDim.x * BLOCK) {
    uint32_t v = ids[i];
    if (v != NO_ROW) lab[v] = stamp;
  }
}

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
  unsigned long long* gticket;  // PState::gticket / gv / gpart
  unsigned long long* gv;
  unsigned long long* gpart;
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
constexpr int GH_THREADS = 256;
constexpr int GH_U = 4;          // neighbours per thread per pass (loads issued back to back)
static_assert(sizeof(Cand) == 32, "Cand travels through PState::gpart as 4 words");

// Block-wide minimum; every thread gets the result.  INT64_MAX type marks "no candidate".
template <int NT>
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
    for (int i = 1; i < NT / 64; ++i)
      if (cand_less(lds[i], b)) b = lds[i];
    lds[NT / 64] = b;
  }
  __syncthreads();
  Cand r = lds[NT / 64];
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

__device__ __forceinline__ uint64_t ld_agent(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Greedy reconstruction, step 0 (one workgroup): v0 = the smallest vid among the start
// candidates (dense ids are in vid order).
__global__ void __launch_bounds__(GH_THREADS) k_greedy_start(GreedyArgs g) {
  __shared__ Cand lds[GH_THREADS / 64 + 1];
  const Cand none{INT64_MAX, INT64_MAX, INT64_MAX, NO_ROW};
  Cand c = none;
  const uint64_t ns = *g.nstarts;
  for (uint64_t i = threadIdx.x; i < ns; i += GH_THREADS) {
    const uint32_t d = g.starts[i];
    if (d != NO_ROW && (int64_t)d < c.t) c = Cand{(int64_t)d, 0, 0, d};
  }
  c = block_min<GH_THREADS>(c, lds);
  if (threadIdx.x != 0) return;
  *g.gticket = 0;
  *g.gv = c.d;
  if (c.d == NO_ROW)
    *g.err = 1;
  else
    g.out[0] = g.vids[c.d];
}

// Greedy reconstruction, hop pos (GREEDY_HOP_BLOCKS workgroups): the minimum (type, rank, dst)
// edge from the current vertex into B[pos + 1].  The current vertex may be a hub, so its
// adjacency is scanned by many CUs; each workgroup leaves its minimum in PState::gpart and the
// last one to finish (ticket) reduces them, records the hop and moves the current vertex.
__global__ void __launch_bounds__(GH_THREADS) k_greedy_hop(GreedyArgs g, int pos) {
  __shared__ Cand lds[GH_THREADS / 64 + 1];
  __shared__ int s_last;
  const Cand none{INT64_MAX, INT64_MAX, INT64_MAX, NO_ROW};
  const uint32_t v = (uint32_t)*g.gv;
  if (v == NO_ROW) return;   // an earlier step failed (err is set)
  Cand best = none;
  if (!g.visible || g.visible[v]) {
    for (int t = 0; t < g.ntypes; ++t) {
      const uint32_t rs = g.row_ptr[t][v];
      uint32_t deg = g.row_ptr[t][v + 1] - rs;
      deg = deg < g.cap ? deg : g.cap;
      const uint32_t stride = gridDim.x * GH_THREADS * GH_U;
      for (uint32_t k0 = blockIdx.x * GH_THREADS * GH_U; k0 < deg; k0 += stride) {
        uint32_t wv[GH_U];
#pragma unroll
        for (int u = 0; u < GH_U; ++u) {
          const uint32_t k = k0 + (uint32_t)u * GH_THREADS + threadIdx.x;
          wv[u] = k < deg ? g.col[t][(uint64_t)rs + k] : NO_ROW;
        }
        bool ok[GH_U];
#pragma unroll
        for (int u = 0; u < GH_U; ++u) ok[u] = greedy_valid(g, wv[u], pos + 1);
#pragma unroll
        for (int u = 0; u < GH_U; ++u) {
          if (!ok[u]) continue;
          const uint64_t j = (uint64_t)rs + k0 + (uint32_t)u * GH_THREADS + threadIdx.x;
          Cand x{(int64_t)g.type[t], g.rank[t] ? g.rank[t][j] : 0, g.dst_vid[t][j], wv[u]};
          if (cand_less(x, best)) best = x;
        }
      }
    }
  }
  best = block_min<GH_THREADS>(best, lds);
  unsigned long long* part = g.gpart + 4 * blockIdx.x;
  if (threadIdx.x == 0) {
    part[0] = (unsigned long long)best.t;
    part[1] = (unsigned long long)best.r;
    part[2] = (unsigned long long)best.v;
    part[3] = best.d;
    __threadfence();
    s_last = atomicAdd(g.gticket, 1ull) == gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last) return;
  __threadfence();
  Cand c = none;
  if (threadIdx.x < gridDim.x) {
    const unsigned long long* q = g.gpart + 4 * threadIdx.x;
    c = Cand{(int64_t)ld_agent(q), (int64_t)ld_agent(q + 1), (int64_t)ld_agent(q + 2), (uint32_t)ld_agent(q + 3)};
  }
  c = block_min<GH_THREADS>(c, lds);
  if (threadIdx.x != 0) return;
  *g.gticket = 0;
  if (c.d == NO_ROW) {
    *g.err = 1;
    *g.gv = NO_ROW;
    return;
  }
  g.out[1 + 3 * pos] = c.t;
  g.out[2 + 3 * pos] = c.r;
  g.out[3 + 3 * pos] = c.v;
  *g.gv = c.d;
}

// ----------------------------------------------------------------------------- path host side
constexpr uint64_t STAGE = 4096;
static hipEvent_t prof_begin_p(Workspace* w, int kid) { return prof_begin(w, kid); }
static void prof_end_p(Workspace* w, hipEvent_t a, int kid, int rec) {
  if (!a) return;
  hipEvent_t b = w->prof.get();
  (void)hipEventRecord(b, w->stream);
  w->prof.pending.push_back({kid, rec, 0, a, b, 0, 0, true});
}

static DegsumArgs degsum_args(const PathTypes& pt) {
  DegsumArgs d{};
  d.ntypes = pt.n;
  for (int t = 0; t < pt.n; ++t) d.row_ptr[t] = pt.a[t].row_ptr;
  d.visible = pt.n ? pt.a[0].visible : nullptr;
  d.cap = pt.n ? pt.a[0].cap : 0xFFFFFFFFu;
  return d;
}

hipError_t ws_path_begin(Workspace* w, uint64_t scratch_entries, uint64_t list_entries, bool zero_state) {
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
    HIP_TRY(ws_sync(w));
    for (auto*& p : w->slot) {
      if (p) HIP_TRY(hipFree(p));
      p = nullptr;
    }
    w->slot_cap = list_entries;
    for (auto*& p : w->slot) HIP_TRY(hipMalloc((void**)&p, w->slot_cap * sizeof(uint32_t)));
  }
  if (scratch_entries > w->pscratch_cap) {
    HIP_TRY(ws_sync(w));
    if (w->pscratch) HIP_TRY(hipFree(w->pscratch));
    w->pscratch = nullptr;
    w->pscratch_cap = scratch_entries;
    HIP_TRY(hipMalloc((void**)&w->pscratch, w->pscratch_cap * sizeof(uint32_t)));
  }
  w->rec = 0;
  w->ppr = 0;
  return zero_state ? hipMemsetAsync(w->ps, 0, sizeof(PState), w->stream) : hipSuccess;
}

struct PairSetup {
  uint32_t s, t;
  uint32_t *slot_f, *slot_b, *slot_start;
  int sf, sb, sst;
  uint32_t *lab_f, *lab_b;
  uint32_t stamp_f, stamp_b;
  DegsumArgs df, db;
  PState* ps;
};

__global__ void __launch_bounds__(BLOCK) k_path_setup(PairSetup a) {
  unsigned long long* p = reinterpret_cast<unsigned long long*>(a.ps);
  for (unsigned i = threadIdx.x; i < sizeof(PState) / 8; i += BLOCK) p[i] = 0;
  __syncthreads();
  if (threadIdx.x != 0) return;
  const bool hs = a.s != NO_ROW, ht = a.t != NO_ROW;
  a.slot_f[0] = a.s;
  a.slot_start[0] = a.s;
  a.slot_b[0] = a.t;
  a.ps->n[a.sf] = hs;
  a.ps->n[a.sst] = hs;
  a.ps->n[a.sb] = ht;
  if (hs) a.lab_f[a.s] = a.stamp_f;
  if (ht) a.lab_b[a.t] = a.stamp_b;
  a.ps->dsum[0] = degree_of(a.df, a.s);
  a.ps->dsum[1] = degree_of(a.db, a.t);
}

hipError_t ws_path_setup_pair(Workspace* w, const PathTypes& fwd, const PathTypes& bwd, uint32_t s, uint32_t t,
                              int slot_f, int slot_b, int slot_start, int lab_f, uint32_t stamp_f, int lab_b,
                              uint32_t stamp_b) {
  static_assert(sizeof(PState) % 8 == 0, "PState is cleared in 8-byte words");
  if (w->slot_cap < 1) return hipErrorInvalidValue;
  PairSetup a{};
  a.s = s;
  a.t = t;
  a.slot_f = w->slot[slot_f];
  a.slot_b = w->slot[slot_b];
  a.slot_start = w->slot[slot_start];
  a.sf = slot_f;
  a.sb = slot_b;
  a.sst = slot_start;
  a.lab_f = w->lab[lab_f];
  a.lab_b = w->lab[lab_b];
  a.stamp_f = stamp_f;
  a.stamp_b = stamp_b;
  a.df = degsum_args(fwd);
  a.db = degsum_args(bwd);
  a.ps = w->ps;
  hipLaunchKernelGGL(k_path_setup, dim3(1), dim3(BLOCK), 0, w->stream, a);
  return hipGetLastError();
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
    HIP_TRY(ws_sync(w));
    if (w->h_starts) HIP_TRY(hipHostFree(w->h_starts));
    w->cap_starts = n + n / 2 + 1024;
    HIP_TRY(hipHostMalloc((void**)&w->h_starts, w->cap_starts * 4, hipHostMallocDefault));
  }
  // the staging buffer may still feed an earlier copy of this query
  HIP_TRY(ws_sync(w));
  memcpy(w->h_starts, ids, n * 4);
  w->h_ps->n[s] = n;
  HIP_TRY(hipMemcpyAsync(w->slot[s], w->h_starts, n * 4, hipMemcpyHostToDevice, w->stream));
  return hipMemcpyAsync(&w->ps->n[s], &w->h_ps->n[s], sizeof(unsigned long long), hipMemcpyHostToDevice,
                        w->stream);
}

hipError_t ws_path_stamp(Workspace* w, int s, uint64_t n_bound, int l, uint32_t stamp) {
  unsigned nb = (unsigned)cdiv(n_bound ? n_bound : 1, BLOCK);
  if (nb > 1024) nb = 1024;
  hipEvent_t p = prof_begin_p(w, K_STAMP);
  hipLaunchKernelGGL(k_stamp, dim3(nb), dim3(BLOCK), 0, w->stream, w->slot[s], &w->ps->n[s], w->lab[l], stamp);
  prof_end_p(w, p, K_STAMP, 0);
  return hipGetLastError();
}

hipError_t ws_path_degsum(Workspace* w, int s, uint64_t n_bound, const PathTypes& pt, int side) {
  const DegsumArgs d = degsum_args(pt);
  unsigned nb = (unsigned)cdiv(n_bound ? n_bound : 1, BLOCK);
  if (nb > 2048) nb = 2048;
  const int rec = w->rec < PATH_REC ? w->rec++ : PATH_REC - 1;
  HIP_TRY(hipMemsetAsync(&w->ps->dsum[side], 0, sizeof(unsigned long long), w->stream));
  hipEvent_t p = prof_begin_p(w, K_DEGSUM);
  hipLaunchKernelGGL(k_degsum, dim3(nb), dim3(BLOCK), 0, w->stream, w->slot[s], &w->ps->n[s], d,
                     &w->ps->dsum[side], &w->ps->ln[rec]);
  prof_end_p(w, p, K_DEGSUM, rec);
  return hipGetLastError();
}

hipError_t ws_path_meet_degsum(Workspace* w, int s, const PathTypes& pt, bool out_edges) {
  const DegsumArgs d = degsum_args(pt);
  unsigned long long* o = out_edges ? &w->ps->mdsum_out : &w->ps->mdsum;
  HIP_TRY(hipMemsetAsync(o, 0, sizeof(unsigned long long), w->stream));
  hipLaunchKernelGGL(k_degsum, dim3(64), dim3(BLOCK), 0, w->stream, w->slot[s], &w->ps->n[s], d, o,
                     (unsigned long long*)nullptr);
  return hipGetLastError();
}

hipError_t ws_path_level(Workspace* w, const PathTypes& pt, int src, uint64_t n_bound, uint64_t e_bound, int dst,
                         const PathLevel& lv) {
  // claims append straight to slot dst (a level claims each vertex at most once: <= nv entries)
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
  const int rec = w->rec < PATH_REC ? w->rec++ : PATH_REC - 1;
  bp.out = w->slot[dst];
  bp.out_n = &w->ps->n[dst];
  // a clamped record (rec == PATH_REC - 1 reused) accumulates: the degree sum then only over-bounds
  if (lv.deg) { bp.deg = degsum_args(*lv.deg); bp.dsum = &w->ps->ld[rec]; }
  for (int t = 0; t < pt.n; ++t) {
    ExpandArgs a = pt.a[t];
    unsigned long long* acc = &w->ps->acc[w->ppr];
    unsigned long long* other = &w->ps->acc[w->ppr ^ 1];
    w->ppr ^= 1;
    hipEvent_t p = prof_begin_p(w, K_RELIST);
    hipLaunchKernelGGL(k_relist, dim3((unsigned)cdiv(n_bound ? n_bound : 1, RL_TILE)), dim3(BLOCK), 0, w->stream,
                       w->slot[src], &w->ps->n[src], 0, 0u, InlineIds{}, deg_of(a),
                       list_out(w, w->rlist, acc, other, t == 0 ? &w->ps->ln[rec] : nullptr),
                       t == 0 ? &w->ps->n[dst] : (unsigned long long*)nullptr);   // zeroed before the claims
    prof_end_p(w, p, K_RELIST, rec);
    a.frontier = w->rlist;
    a.tsplit = w->tsplit;
    p = prof_begin_p(w, K_BFS);
    hipLaunchKernelGGL(k_expand<BFS>, dim3(expand_grid(n_bound, e_bound)), dim3(BLOCK), 0, w->stream, a, acc,
                       w->seg_end, w->seg_rs, (uint8_t*)nullptr, FinalParams{}, bp, &w->ps->le[rec],
                       (unsigned long long*)nullptr, NoInline{});
    prof_end_p(w, p, K_BFS, rec);
  }
  return hipGetLastError();
}

int ws_path_last_rec(Workspace* w) { return w->rec - 1; }

hipError_t ws_path_read_label(Workspace* w, int l, uint32_t v, uint32_t* out) {
  HIP_TRY(hipMemcpyAsync(w->h_stage, w->lab[l] + v, sizeof(uint32_t), hipMemcpyDeviceToHost, w->stream));
  HIP_TRY(ws_wait(w));
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
  g.gticket = &w->ps->gticket;
  g.gv = &w->ps->gv;
  g.gpart = w->ps->gpart;
  hipEvent_t p = prof_begin_p(w, K_GREEDY);
  hipLaunchKernelGGL(k_greedy_start, dim3(1), dim3(GH_THREADS), 0, w->stream, g);
  for (int pos = 0; pos < pg.L; ++pos)
    hipLaunchKernelGGL(k_greedy_hop, dim3(GREEDY_HOP_BLOCKS), dim3(GH_THREADS), 0, w->stream, g, pos);
  prof_end_p(w, p, K_GREEDY, 0);
  return hipGetLastError();
}

hipError_t ws_path_sync(Workspace* w, PState* out, int64_t* path, int path_len) {
  HIP_TRY(hipMemcpyAsync(w->h_ps, w->ps, sizeof(PState), hipMemcpyDeviceToHost, w->stream));
  if (path && path_len > 0)
    HIP_TRY(hipMemcpyAsync(w->h_path, w->d_path, (size_t)path_len * sizeof(int64_t), hipMemcpyDeviceToHost,
                           w->stream));
  HIP_TRY(ws_wait(w));
  if (out) *out = *w->h_ps;
  if (path && path_len > 0) memcpy(path, w->h_path, (size_t)path_len * sizeof(int64_t));
  // resolve timing of the launches since the last sync (record indices stay valid per query)
  prof_flush(w, nullptr, w->h_ps);
  return hipSuccess;
}

// ============================================================================= partitioned FIND PATH
// The BFS of a partitioned engine: a level expands the rank's own frontier
// over its CSRs into byte flags over the global id space (k_expand<MARK>), the flags travel to
// their owners in the per-hop bitmap all-to-all, and the OWNER claims its vertices (label test
// and set — each vertex is handled by exactly one thread, no CAS), detects meets against its
// own labels of the other side and counts reached targets.  Sizes every rank needs (frontier
// sizes, degree sums, meets, targets found) are summed over ranks at each synchronisation.
struct ClaimParams {
  uint32_t* lab;                  // claim labels
  uint32_t stamp;
  uint32_t epoch;
  const uint32_t* rlab;           // restriction (nullable): claim v only if rlab[v] == rstamp
  uint32_t rstamp;
  const uint32_t* mlab;           // meet test (nullable)
  uint32_t mepoch;
  uint32_t* mout;
  uint32_t mstamp;
  uint32_t* meet_list;
  unsigned long long* meet_n;
  const uint32_t* tlab;           // targets (nullable)
  uint32_t tstamp;
  unsigned long long* found;
  uint32_t* out;                  // claimed vertices (next frontier, local ids)
  unsigned long long* out_n;
};

// Block-wide append of c items per thread to a list with counter *n: returns this thread's slot.
__device__ __forceinline__ uint32_t block_append(uint32_t c, unsigned long long* n) {
  __shared__ uint32_t lds[WAVES];
  __shared__ unsigned long long s_base;
  uint32_t tot;
  const uint32_t x = block_excl_scan(c, &tot, lds);
  if (threadIdx.x == 0) s_base = tot ? atomicAdd(n, (unsigned long long)tot) : 0ull;
  __syncthreads();
  return (uint32_t)s_base + x;
}

__global__ void __launch_bounds__(BLOCK) k_bits_claim(const unsigned long long* __restrict__ recv, int world,
                                                      uint64_t seg_words, uint64_t nv, ClaimParams cp) {
  const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;   // 16-bit slice index
  const uint64_t word = i >> 2;
  const int sh = (int)(i & 3) * 16;
  unsigned long long m64 = 0;
  for (int q = 0; q < world; ++q) m64 |= recv[(uint64_t)q * seg_words + word];
  uint32_t m = (uint32_t)(m64 >> sh) & 0xFFFFu;
  const uint64_t lo = i * 16;
  if (lo >= nv) m = 0;
  else if (nv - lo < 16) m &= (1u << (nv - lo)) - 1u;
  uint32_t cm = 0, mm = 0;
  for (uint32_t x = m; x; x &= x - 1) {
    const int b = __ffs(x) - 1;
    const uint32_t v = (uint32_t)(lo + b);
    if (cp.rlab && cp.rlab[v] != cp.rstamp) continue;
    if ((cp.lab[v] >> LVL_BITS) == cp.epoch) continue;
    cp.lab[v] = cp.stamp;
    cm |= 1u << b;
    if (cp.mlab && (cp.mlab[v] >> LVL_BITS) == cp.mepoch) mm |= 1u << b;
    if (cp.tlab && cp.tlab[v] == cp.tstamp) atomicAdd(cp.found, 1ull);
  }
  uint32_t pos = block_append((uint32_t)__popc(cm), cp.out_n);
  for (uint32_t x = cm; x; x &= x - 1) cp.out[pos++] = (uint32_t)(lo + __ffs(x) - 1);
  if (cp.meet_list) {
    uint32_t mp = block_append((uint32_t)__popc(mm), cp.meet_n);
    for (uint32_t x = mm; x; x &= x - 1) {
      const uint32_t v = (uint32_t)(lo + __ffs(x) - 1);
      cp.meet_list[mp++] = v;
      cp.mout[v] = cp.mstamp;
    }
  }
}

// The owner's claim over the sparse exchange: recv = world segments of `stride` slots (local ids
// or NO_ROW; a vertex may arrive several times, so the claim is a CAS on its label).
__global__ void __launch_bounds__(BLOCK) k_list_claim(const uint32_t* __restrict__ recv, uint64_t slots, ClaimParams cp) {
  const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  const uint32_t v = i < slots ? recv[i] : NO_ROW;
  bool claimed = false, met = false;
  if (v != NO_ROW && !(cp.rlab && cp.rlab[v] != cp.rstamp)) {
    const uint32_t old = cp.lab[v];
    if ((old >> LVL_BITS) != cp.epoch && atomicCAS(cp.lab + v, old, cp.stamp) == old) {
      claimed = true;
      met = cp.mlab && (cp.mlab[v] >> LVL_BITS) == cp.mepoch;
      if (cp.tlab && cp.tlab[v] == cp.tstamp) atomicAdd(cp.found, 1ull);
    }
  }
  const uint32_t pos = block_append(claimed ? 1u : 0u, cp.out_n);
  if (claimed) cp.out[pos] = v;
  if (cp.meet_list) {
    __syncthreads();   // block_append's shared scratch is reused
    const uint32_t mp = block_append(met ? 1u : 0u, cp.meet_n);
    if (met) {
      cp.meet_list[mp] = v;
      cp.mout[v] = cp.mstamp;
    }
  }
}

// Greedy reconstruction, one hop of a partitioned engine: among this rank's vertices u in the
// next B-set, the minimum (type, rank, vid) in-edge u <- v (the out-edge v -> u) from the current
// vertex v (global id); per-block minima, then one block reduces them to this rank's candidate.
struct GreedyPart {
  int ntypes;
  int32_t type[MAX_TYPES_Q];            // OVER types (positive)
  const uint32_t* row_ptr[MAX_TYPES_Q]; // in-edge CSRs (-type)
  const uint32_t* col[MAX_TYPES_Q];     // global id of the in-edge's source
  const int64_t* rank[MAX_TYPES_Q];
  const uint8_t* visible;               // reported per candidate: an invisible vertex has no out-edges
  const int64_t* vids;
  uint64_t nv;
  uint32_t gbase;                       // this rank's first global id
  uint32_t v;                           // current vertex (global id) ...
  const unsigned long long* vp;         // ... or read here ({gid, err}: nothing to do after an error)
  int pos;                              // B-set position of the candidates
  int L, kf;
  const uint32_t* lab_m;
  uint32_t em;
  const uint32_t* lab_b;
  uint32_t eb;
  Cand* part;                           // [2 * gridDim.x] per-block minima (row scan, hub scan)
  uint32_t* hubs;                       // B-set members whose in-edge rows the whole grid scans ...
  uint32_t* nhub;                       // ... and their count (reset by k_greedy_part_reduce)
  uint32_t hub_base;                    // k_greedy_hub's minima start at part[hub_base]
};
constexpr int GREC = 6;
constexpr uint32_t GP_HUB_ROW = 4096;   // a longer in-edge row is a hub's: scanned grid-wide
constexpr uint32_t GP_HUB_CAP = 1024;   // hubs listed per hop (more: scanned wave-wide in place)                 // rank record: type, rank, vid, global id (-1: none), visible, 0

__device__ __forceinline__ bool part_valid(const GreedyPart& g, uint32_t u) {
  if (g.pos <= g.kf) return g.lab_m[u] == ((g.em << LVL_BITS) | (uint32_t)g.pos);
  return g.lab_b[u] == ((g.eb << LVL_BITS) | (uint32_t)(g.L - g.pos));
}

__global__ void __launch_bounds__(BLOCK) k_greedy_part(GreedyPart g) {
  __shared__ Cand lds[WAVES + 1];
  Cand best{INT64_MAX, INT64_MAX, INT64_MAX, NO_ROW};
  // (locals, not writes into the by-value argument: a written kernel argument is copied to scratch)
  uint64_t nv = g.nv;
  uint32_t v = g.v;
  if (g.vp) {
    if (g.vp[1]) nv = 0;   // an earlier hop failed: no candidates
    v = (uint32_t)g.vp[0];
  }
  // a wave tests 64 consecutive vertices, then scans each B-set member's in-edge row together
  // (lane-strided, coalesced): a hub's row is not left to one thread
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (uint64_t base = ((uint64_t)blockIdx.x * WAVES + w) * 64; base < nv; base += (uint64_t)gridDim.x * BLOCK) {
    const uint64_t mine = base + lane;
    unsigned long long m = __ballot(mine < nv && part_valid(g, (uint32_t)mine));
    while (m) {
      const uint32_t u = (uint32_t)(base + __builtin_ctzll(m));
      m &= m - 1;
      uint32_t len = 0;
      for (int t = 0; t < g.ntypes; ++t) len += g.row_ptr[t][u + 1] - g.row_ptr[t][u];
      if (len > GP_HUB_ROW) {   // wave-uniform: left to k_greedy_hub unless the list is full
        uint32_t k = 0;
        if (lane == 0) k = atomicAdd(g.nhub, 1u);
        k = __shfl(k, 0, 64);
        if (k < GP_HUB_CAP) {
          if (lane == 0) g.hubs[k] = u;
          continue;
        }
      }
      const int64_t uvid = g.vids[u];
      for (int t = 0; t < g.ntypes; ++t) {
        const uint32_t rs = g.row_ptr[t][u], re = g.row_ptr[t][u + 1];
        for (uint32_t j = rs + lane; j < re; j += 64) {
          if (g.col[t][j] != v) continue;
          Cand x{(int64_t)g.type[t], g.rank[t] ? g.rank[t][j] : 0, uvid, u};
          if (cand_less(x, best)) best = x;
        }
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    Cand x = shfl_cand(best, o);
    if (cand_less(x, best)) best = x;
  }
  if (lane == 0) lds[w] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    Cand b = lds[0];
    for (int k = 1; k < WAVES; ++k)
      if (cand_less(lds[k], b)) b = lds[k];
    g.part[blockIdx.x] = b;
  }
}

// The hubs k_greedy_part listed: each in-edge row is scanned by the whole grid (thread-strided,
// coalesced); per-block minima go to part[hub_base + block].
__global__ void __launch_bounds__(BLOCK) k_greedy_hub(GreedyPart g) {
  __shared__ Cand lds[WAVES];
  Cand best{INT64_MAX, INT64_MAX, INT64_MAX, NO_ROW};
  uint32_t nh = *g.nhub;
  if (nh > GP_HUB_CAP) nh = GP_HUB_CAP;
  uint32_t v = g.v;
  if (g.vp) {
    if (g.vp[1]) nh = 0;
    v = (uint32_t)g.vp[0];
  }
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint32_t h = 0; h < nh; ++h) {
    const uint32_t u = g.hubs[h];
    const int64_t uvid = g.vids[u];
    for (int t = 0; t < g.ntypes; ++t) {
      const uint64_t rs = g.row_ptr[t][u], re = g.row_ptr[t][u + 1];
      for (uint64_t j = rs + (uint64_t)blockIdx.x * BLOCK + threadIdx.x; j < re; j += stride) {
        if (g.col[t][j] != v) continue;
        Cand x{(int64_t)g.type[t], g.rank[t] ? g.rank[t][j] : 0, uvid, u};
        if (cand_less(x, best)) best = x;
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    Cand x = shfl_cand(best, o);
    if (cand_less(x, best)) best = x;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) lds[w] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    Cand b = lds[0];
    for (int k = 1; k < WAVES; ++k)
      if (cand_less(lds[k], b)) b = lds[k];
    g.part[g.hub_base + blockIdx.x] = b;
  }
}

__device__ __forceinline__ void put_record(const Cand& b, uint32_t gbase, const uint8_t* visible, int64_t* out) {
  out[0] = b.t;
  out[1] = b.r;
  out[2] = b.v;
  out[3] = b.d == NO_ROW ? -1 : (int64_t)(gbase + b.d);
  out[4] = b.d == NO_ROW ? 0 : (visible ? visible[b.d] : 1);
  out[5] = 0;
}

__global__ void k_greedy_part_reduce(const Cand* __restrict__ part, int nparts, uint32_t gbase,
                                     const uint8_t* __restrict__ visible, int64_t* out, uint32_t* nhub) {
  if (nhub && threadIdx.x == 0) *nhub = 0;   // the next hop's hub list starts empty
  // one wave (launched with 64 threads): lane-strided minima, then a wave reduction
  Cand b{INT64_MAX, INT64_MAX, INT64_MAX, NO_ROW};
  for (int k = threadIdx.x; k < nparts; k += 64)
    if (cand_less(part[k], b)) b = part[k];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    Cand x = shfl_cand(b, o);
    if (cand_less(x, b)) b = x;
  }
  if (threadIdx.x == 0) put_record(b, gbase, visible, out);
}

// Minimum vid among a list's entries (B[0] of the greedy) as a rank record (type = rank = 0).
__global__ void k_min_vid(const uint32_t* __restrict__ ids, const unsigned long long* __restrict__ np,
                          const int64_t* __restrict__ vids, uint32_t gbase, const uint8_t* __restrict__ visible,
                          int64_t* out) {
  if (threadIdx.x != 0) return;
  Cand b{0, 0, INT64_MAX, NO_ROW};
  const uint64_t n = *np;
  for (uint64_t k = 0; k < n; ++k) {
    const uint32_t d = ids[k];
    if (d != NO_ROW && vids[d] < b.v) b = Cand{0, 0, vids[d], d};
  }
  put_record(b, gbase, visible, out);
}

// Every rank's record (after the all-gather) -> the global minimum (type, rank, vid): path entry
// `pos` (0: v0 alone) and the next hop's vertex in cur[0]; cur[1] = error (no candidate, or an
// invisible vertex that a further hop would have to leave).  Every rank computes the same.
__global__ void k_greedy_pick(const int64_t* __restrict__ all, int G, int pos, int L, int64_t* __restrict__ path,
                              unsigned long long* __restrict__ cur) {
  if (threadIdx.x != 0 || cur[1]) return;
  const int64_t* b = nullptr;
  for (int q = 0; q < G; ++q) {   // distinct ranks never tie (vids are unique)
    const int64_t* x = all + (size_t)q * GREC;
    if (x[3] < 0) continue;
    if (!b || x[0] < b[0] || (x[0] == b[0] && (x[1] < b[1] || (x[1] == b[1] && x[2] < b[2])))) b = x;
  }
  if (!b || (pos < L && !b[4])) {
    cur[1] = 1;
    return;
  }
  if (pos == 0) {
    path[0] = b[2];
  } else {
    path[1 + 3 * (pos - 1)] = b[0];
    path[2 + 3 * (pos - 1)] = b[1];
    path[3 + 3 * (pos - 1)] = b[2];
  }
  cur[0] = (unsigned long long)b[3];
}

// the greedy's start when it is known on every rank
__global__ void k_greedy_v0(int64_t vid, unsigned long long gid, int64_t* __restrict__ path,
                            unsigned long long* __restrict__ cur) {
  if (threadIdx.x != 0) return;
  path[0] = vid;
  cur[0] = gid;
  cur[1] = 0;
}

hipError_t ws_path_level_part(Workspace* w, const PathTypes& pt, int src, uint64_t n_bound, uint64_t e_bound, int dst,
                              const PathLevel& lv) {
  if (!w->comm) return hipErrorInvalidValue;
  const int rec = w->rec < PATH_REC ? w->rec++ : PATH_REC - 1;
  const uint64_t G = (uint64_t)w->comm->world;
  // exchange format: a level of one OVER type whose edge total (e_bound: the frontier's degree
  // sum over every rank, so a bound on each rank's edges) is small sends per-owner slot arrays
  // of e_bound ids instead of the npad-bit bitmap segments — the same choice on every rank
  const uint64_t stride = (e_bound + 63) / 64 * 64;
  const bool sparse = lv.global_bound && pt.n == 1 && e_bound && stride * 4 * 2 <= w->npad / 8 && !bits_off() &&
                      sparse_on();
  HIP_TRY(hipMemsetAsync(&w->ps->n[dst], 0, sizeof(unsigned long long), w->stream));
  if (sparse) HIP_TRY(hipMemsetAsync(w->sendbits, 0xFF, G * stride * 4, w->stream));
  for (int t = 0; t < pt.n; ++t) {
    ExpandArgs a = pt.a[t];
    unsigned long long* acc = &w->ps->acc[w->ppr];
    unsigned long long* other = &w->ps->acc[w->ppr ^ 1];
    w->ppr ^= 1;
    hipEvent_t p = prof_begin_p(w, K_RELIST);
    hipLaunchKernelGGL(k_relist, dim3((unsigned)cdiv(n_bound ? n_bound : 1, RL_TILE)), dim3(BLOCK), 0, w->stream,
                       w->slot[src], &w->ps->n[src], 0, 0u, InlineIds{}, deg_of(a),
                       list_out(w, w->rlist, acc, other, t == 0 ? &w->ps->ln[rec] : nullptr),
                       (unsigned long long*)nullptr);
    prof_end_p(w, p, K_RELIST, rec);
    a.frontier = w->rlist;
    a.tsplit = w->tsplit;
    BfsParams mb{};
    if (sparse) {
      mb.sparse = reinterpret_cast<uint32_t*>(w->sendbits);
      mb.sp_stride = (uint32_t)stride;
      mb.sp_npad = (uint32_t)w->npad;
    } else if (!bits_off()) {
      mb.bits = w->sendbits;   // the level's candidates straight into the send bitmap
    }
    p = prof_begin_p(w, K_EXPAND_MARK);
    hipLaunchKernelGGL(k_expand<MARK>, dim3(expand_grid(n_bound, e_bound)), dim3(BLOCK), 0, w->stream, a, acc,
                       w->seg_end, w->seg_rs, w->flags, FinalParams{}, mb, &w->ps->le[rec],
                       (unsigned long long*)nullptr, NoInline{});
    prof_end_p(w, p, K_EXPAND_MARK, rec);
  }
  const uint64_t nwords = G * w->npad / 64, seg_words = w->npad / 64, nb = w->npad / BITS_BLOCK;
  hipEvent_t p = nullptr;
  if (bits_off()) {
    p = prof_begin_p(w, K_PACK);
    hipLaunchKernelGGL(k_pack_bits, dim3((unsigned)cdiv(nwords, BLOCK)), dim3(BLOCK), 0, w->stream, w->flags, nwords,
                       w->sendbits);
    prof_end_p(w, p, K_PACK, rec);
    HIP_TRY(hipGetLastError());
  }
  const uint64_t xbytes = sparse ? stride * 4 : w->npad / 8;   // per peer
  if (w->comm->alltoall(w->sendbits, w->recvbits, xbytes, w->stream)) return hipErrorUnknown;
  HIP_TRY(hipMemsetAsync(w->sendbits, 0, G * xbytes, w->stream));   // all-zero between hops (GO ORs into it)
  ClaimParams cp{};
  cp.lab = w->lab[lv.lab];
  cp.stamp = lv.stamp;
  cp.epoch = lv.stamp >> LVL_BITS;
  if (lv.rlab >= 0) { cp.rlab = w->lab[lv.rlab]; cp.rstamp = lv.rstamp; }
  if (lv.mlab >= 0) {
    cp.mlab = w->lab[lv.mlab];
    cp.mepoch = lv.mepoch;
    cp.mout = w->lab[LAB_M];
    cp.mstamp = lv.mstamp;
    cp.meet_list = w->slot[lv.meet_slot];
    cp.meet_n = &w->ps->n[lv.meet_slot];
  }
  if (lv.tlab >= 0) { cp.tlab = w->lab[lv.tlab]; cp.tstamp = lv.tstamp; cp.found = &w->ps->found; }
  cp.out = w->slot[dst];
  cp.out_n = &w->ps->n[dst];
  p = prof_begin_p(w, K_BITS_COMPACT);
  if (sparse)
    hipLaunchKernelGGL(k_list_claim, dim3((unsigned)cdiv(G * stride, BLOCK)), dim3(BLOCK), 0, w->stream,
                       reinterpret_cast<const uint32_t*>(w->recvbits), G * stride, cp);
  else
    hipLaunchKernelGGL(k_bits_claim, dim3((unsigned)nb), dim3(BLOCK), 0, w->stream, w->recvbits, (int)G, seg_words,
                       w->nv, cp);
  prof_end_p(w, p, K_BITS_COMPACT, rec);
  return hipGetLastError();
}

// The PState fields every rank needs, summed over ranks (n[], dsum[], found, err, le[]).
constexpr int PG_N = PSLOTS + 2 + 2 + PATH_REC + 2;
__global__ void k_pgstats(const PState* __restrict__ ps, unsigned long long* __restrict__ g) {
  const int k = threadIdx.x;
  if (k < PSLOTS) g[k] = ps->n[k];
  if (k < 2) g[PSLOTS + k] = ps->dsum[k];
  if (k == 0) {
    g[PSLOTS + 2] = ps->found;
    g[PSLOTS + 3] = ps->err;
  }
  if (k < PATH_REC) g[PSLOTS + 4 + k] = ps->le[k];
  if (k == 0) g[PSLOTS + 4 + PATH_REC] = ps->mdsum;
  if (k == 1) g[PSLOTS + 5 + PATH_REC] = ps->mdsum_out;
}

// Synchronous: like ws_path_sync, with the per-rank sizes summed over ranks.
hipError_t ws_path_sync_part(Workspace* w, PState* out) {
  if (!w->comm) return hipErrorInvalidValue;
  if (!w->pgst) {
    HIP_TRY(hipMalloc((void**)&w->pgst, PG_N * sizeof(unsigned long long)));
    HIP_TRY(hipHostMalloc((void**)&w->h_pgst, PG_N * sizeof(unsigned long long), hipHostMallocDefault));
  }
  hipLaunchKernelGGL(k_pgstats, dim3(1), dim3(64), 0, w->stream, w->ps, w->pgst);
  HIP_TRY(hipGetLastError());
  if (w->comm->allreduce_sum_u64(w->pgst, PG_N, w->stream)) return hipErrorUnknown;
  HIP_TRY(hipMemcpyAsync(w->h_pgst, w->pgst, PG_N * sizeof(unsigned long long), hipMemcpyDeviceToHost, w->stream));
  // the rank's own PState only feeds the profiler's byte counts (every field the callers read is
  // in the reduced block): no second copy per level when nothing is being profiled
  if (!w->prof.pending.empty())
    HIP_TRY(hipMemcpyAsync(w->h_ps, w->ps, sizeof(PState), hipMemcpyDeviceToHost, w->stream));
  HIP_TRY(ws_wait(w));
  PState g = *w->h_ps;
  for (int k = 0; k < PSLOTS; ++k) g.n[k] = w->h_pgst[k];
  for (int k = 0; k < 2; ++k) g.dsum[k] = w->h_pgst[PSLOTS + k];
  g.found = w->h_pgst[PSLOTS + 2];
  g.err = w->h_pgst[PSLOTS + 3];
  for (int k = 0; k < PATH_REC; ++k) g.le[k] = w->h_pgst[PSLOTS + 4 + k];
  g.mdsum = w->h_pgst[PSLOTS + 4 + PATH_REC];
  g.mdsum_out = w->h_pgst[PSLOTS + 5 + PATH_REC];
  if (out) *out = g;
  prof_flush(w, nullptr, w->h_ps);
  return hipSuccess;
}

// Sum a host vector over ranks (small control data: label values, presence flags).
hipError_t ws_allreduce_host(Workspace* w, std::vector<unsigned long long>& v) {
  if (!w->comm || v.empty()) return hipSuccess;
  if (v.size() > w->ar_cap) {   // grow-only scratch (no allocation per query)
    if (w->ar_buf) {
      HIP_TRY(ws_sync(w));
      (void)hipFree(w->ar_buf);
      w->ar_buf = nullptr;
      w->ar_cap = 0;
    }
    const uint64_t cap = std::max<uint64_t>(v.size(), 256);
    HIP_TRY(hipMalloc((void**)&w->ar_buf, cap * 8));
    w->ar_cap = cap;
  }
  unsigned long long* d = w->ar_buf;
  hipError_t e = hipMemcpyAsync(d, v.data(), v.size() * 8, hipMemcpyHostToDevice, w->stream);
  if (e == hipSuccess && w->comm->allreduce_sum_u64(d, v.size(), w->stream)) e = hipErrorUnknown;
  if (e == hipSuccess) e = hipMemcpyAsync(v.data(), d, v.size() * 8, hipMemcpyDeviceToHost, w->stream);
  if (e == hipSuccess) e = ws_sync(w);
  return e;
}

// Lexicographically smallest shortest path through the B-sets on a partitioned engine; the path
// entries are written to `path` (1 + 3L).  Returns hipErrorNotFound when a hop has no candidate.
// The hops run back to back on the device: each rank's candidate record, one all-gather, and
// k_greedy_pick (the same on every rank) hands the next hop its vertex in device memory; the
// host waits once, for the path.
hipError_t ws_path_greedy_part(Workspace* w, const PathTypes& bwd, const PathGreedy& pg, const int64_t* vids,
                               const uint8_t* visible, int64_t* path) {
  if (!w->comm) return hipErrorInvalidValue;
  if (pg.L < 1 || pg.L > (int)MAX_PATH_LEN) return hipErrorInvalidValue;
  const int G = w->comm->world;
  const uint32_t gbase = (uint32_t)((uint64_t)w->comm->rank * w->npad);
  const uint64_t nblk = cdiv(w->nv ? w->nv : 1, BLOCK);
  constexpr unsigned kGrid = 1024;
  const unsigned grid = (unsigned)(nblk < kGrid ? nblk : kGrid);
  constexpr unsigned kHubGrid = 256;
  const size_t hub_off = ((size_t)kGrid + kHubGrid) * sizeof(Cand);
  if (!w->g_part) {
    HIP_TRY(hipMalloc(&w->g_part, hub_off + (GP_HUB_CAP + 1) * sizeof(uint32_t)));
    HIP_TRY(hipMemsetAsync(static_cast<char*>(w->g_part) + hub_off, 0, (GP_HUB_CAP + 1) * sizeof(uint32_t),
                           w->stream));
    HIP_TRY(hipMalloc((void**)&w->g_rec, GREC * 8));
    HIP_TRY(hipMalloc((void**)&w->g_all, (size_t)G * GREC * 8));
    HIP_TRY(hipMalloc((void**)&w->g_path, (1 + 3 * (size_t)MAX_PATH_LEN) * 8));
    HIP_TRY(hipMalloc((void**)&w->g_cur, 2 * 8));
    HIP_TRY(hipHostMalloc((void**)&w->h_gpath, (3 + 3 * (size_t)MAX_PATH_LEN) * 8, hipHostMallocDefault));
  }
  Cand* d_part = static_cast<Cand*>(w->g_part);
  if (pg.v0_gid >= 0) {
    // v0 known on every rank (one source): no exchange
    hipLaunchKernelGGL(k_greedy_v0, dim3(1), dim3(64), 0, w->stream, pg.v0_vid, (unsigned long long)pg.v0_gid,
                       w->g_path, w->g_cur);
  } else {
    HIP_TRY(hipMemsetAsync(w->g_cur, 0, 2 * 8, w->stream));
    // v0: the smallest vid of B[0]
    hipLaunchKernelGGL(k_min_vid, dim3(1), dim3(64), 0, w->stream, w->slot[pg.start_slot], &w->ps->n[pg.start_slot],
                       vids, gbase, visible, w->g_rec);
    HIP_TRY(hipGetLastError());
    if (w->comm->allgather(w->g_rec, w->g_all, GREC * 8, w->stream)) return hipErrorUnknown;
    hipLaunchKernelGGL(k_greedy_pick, dim3(1), dim3(64), 0, w->stream, w->g_all, G, 0, pg.L, w->g_path, w->g_cur);
  }
  HIP_TRY(hipGetLastError());
  GreedyPart g{};
  g.ntypes = bwd.n;
  for (int t = 0; t < bwd.n; ++t) {
    g.type[t] = -bwd.type[t];
    g.row_ptr[t] = bwd.a[t].row_ptr;
    g.col[t] = bwd.a[t].col;
    g.rank[t] = bwd.a[t].rank;
  }
  g.visible = visible;
  g.vids = vids;
  g.nv = w->nv;
  g.gbase = gbase;
  g.vp = w->g_cur;
  g.L = pg.L;
  g.kf = pg.kf;
  g.lab_m = w->lab[LAB_M];
  g.em = pg.em;
  g.lab_b = w->lab[LAB_B];
  g.eb = pg.eb;
  g.part = d_part;
  g.hubs = reinterpret_cast<uint32_t*>(static_cast<char*>(w->g_part) + hub_off);
  g.nhub = g.hubs + GP_HUB_CAP;
  g.hub_base = grid;
  for (int pos = 1; pos <= pg.L; ++pos) {
    g.pos = pos;
    hipEvent_t p = prof_begin_p(w, K_GREEDY);
    hipLaunchKernelGGL(k_greedy_part, dim3(grid), dim3(BLOCK), 0, w->stream, g);
    hipLaunchKernelGGL(k_greedy_hub, dim3(kHubGrid), dim3(BLOCK), 0, w->stream, g);
    hipLaunchKernelGGL(k_greedy_part_reduce, dim3(1), dim3(64), 0, w->stream, d_part, (int)(grid + kHubGrid), gbase,
                       visible, w->g_rec, g.nhub);
    prof_end_p(w, p, K_GREEDY, 0);
    HIP_TRY(hipGetLastError());
    if (w->comm->allgather(w->g_rec, w->g_all, GREC * 8, w->stream)) return hipErrorUnknown;
    hipLaunchKernelGGL(k_greedy_pick, dim3(1), dim3(64), 0, w->stream, w->g_all, G, pos, pg.L, w->g_path, w->g_cur);
    HIP_TRY(hipGetLastError());
  }
  const size_t np = 1 + 3 * (size_t)pg.L;
  HIP_TRY(hipMemcpyAsync(w->h_gpath, w->g_path, np * 8, hipMemcpyDeviceToHost, w->stream));
  HIP_TRY(hipMemcpyAsync(w->h_gpath + np, w->g_cur, 2 * 8, hipMemcpyDeviceToHost, w->stream));
  HIP_TRY(ws_sync(w));
  if (w->h_gpath[np + 1]) return hipErrorNotFound;
  memcpy(path, w->h_gpath, np * 8);
  return hipSuccess;
}

}  // namespace nbg
