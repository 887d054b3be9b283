// C ABI implementation (include/nbg.h) and the GO N STEPS driver.
//
// GO N STEPS follows GoExecutor (src/graph/GoExecutor.cpp):
//   * starts keep duplicates (prepareFrom :136-195); unknown vids contribute nothing;
//   * steps 1..N-1: frontier_{s+1} = SET of _dst over every live edge of every OVER type
//     (getDstIdsFromResp :501-541) — no global visited set; empty frontier -> empty result
//     (onEmptyInputs :791-800);
//   * step N: one row per (frontier entry, live edge) passing WHERE; WHERE/YIELD evaluation
//     errors fail the query (processFinalResult :948-969).
// Each hop runs on the device: degree scan -> merge-path partition -> expand (+ byte-flag
// dedup and compaction, or the final-step bytecode + row compaction).
#include <chrono>
#include <algorithm>
#include <atomic>
#include <cstring>
#include <ctime>
#include <set>
#include <iterator>
#include <unordered_map>

#include "engine.h"

static_assert(NBG_MAX_YIELDS == nbg::MAX_YIELDS && NBG_MAX_OVER == nbg::MAX_TYPES_Q,
              "include/nbg.h device limits match the engine's");

// a fresh seed for each query's rand32 / rand64 stream
static uint64_t query_rand_seed() {
  static std::atomic<uint64_t> ctr{(uint64_t)std::chrono::steady_clock::now().time_since_epoch().count() * 0x9e3779b97f4a7c15ull};
  return ctr.fetch_add(0x9e3779b97f4a7c15ull, std::memory_order_relaxed);
}

using namespace nbg;

namespace nbg {

static void free_edge_type(DevEdgeType& d) {
  for (void* p : {(void*)d.row_ptr, (void*)d.col, (void*)d.dst_vid, (void*)d.rank, (void*)d.valid, (void*)d.d_props})
    if (p) (void)hipFree(p);
  for (auto* p : d.props)
    if (p) (void)hipFree(p);
  for (auto* p : d.narrow)
    if (p) (void)hipFree(p);
  if (d.old) {
    free_edge_type(*d.old);
    delete d.old;
    d.old = nullptr;
  }
}

void Engine::free_snapshot() {
  for (auto& kv : snap.types) free_edge_type(kv.second);
  for (auto& kv : snap.tags) {
    if (kv.second.present) (void)hipFree(kv.second.present);
    for (auto* p : kv.second.cols)
      if (p) (void)hipFree(p);
  }
  for (void* p : {(void*)snap.d_tcols, (void*)snap.d_tpres, (void*)snap.d_vids, (void*)snap.d_visible, (void*)snap.d_zero_rows,
                  (void*)snap.d_soff, (void*)snap.d_sbytes, (void*)snap.d_s2i, (void*)snap.d_s2f, (void*)snap.d_s2ok})
    if (p) (void)hipFree(p);
  snap = Snapshot();
}

// The dictionary's device tables: its bytes (piece lists of derived strings read them) and what
// Expression::toInt / toDouble make of every string (Expressions.h:294-321; a string that is not
// a whole number fails the cast, as the host's constant folding and the oracle decide it).
int32_t Engine::upload_strings() {
  const auto& d = snap.strings;
  if (d.empty()) return NBG_OK;
  const size_t n = d.size();
  std::vector<uint32_t> off(n + 1, 0);
  for (size_t i = 0; i < n; ++i) {
    if ((uint64_t)off[i] + d[i].size() > 0xFFFFFFFFull) return fail(NBG_E_UNSUPPORTED, "string dictionary over 4 GB");
    off[i + 1] = off[i] + (uint32_t)d[i].size();
  }
  std::vector<char> bytes(std::max<size_t>(off[n], 1));
  std::vector<int64_t> s2i(n), s2f(n);
  std::vector<uint8_t> ok(n);
  for (size_t i = 0; i < n; ++i) {
    memcpy(bytes.data() + off[i], d[i].data(), d[i].size());
    CVal vi, vf;
    uint8_t b = 0;
    if (evalCast(0, CVal(d[i]), &vi)) { s2i[i] = std::get<int64_t>(vi); b |= 1; }
    if (evalCast(2, CVal(d[i]), &vf)) { const double x = std::get<double>(vf); memcpy(&s2f[i], &x, 8); b |= 2; }
    ok[i] = b;
  }
  hipError_t e = hipMalloc((void**)&snap.d_soff, (n + 1) * 4);
  if (e == hipSuccess) e = hipMalloc((void**)&snap.d_sbytes, bytes.size());
  if (e == hipSuccess) e = hipMalloc((void**)&snap.d_s2i, n * 8);
  if (e == hipSuccess) e = hipMalloc((void**)&snap.d_s2f, n * 8);
  if (e == hipSuccess) e = hipMalloc((void**)&snap.d_s2ok, n);
  if (e == hipSuccess) e = hipMemcpy(snap.d_soff, off.data(), (n + 1) * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(snap.d_sbytes, bytes.data(), bytes.size(), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(snap.d_s2i, s2i.data(), n * 8, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(snap.d_s2f, s2f.data(), n * 8, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(snap.d_s2ok, ok.data(), n, hipMemcpyHostToDevice);
  if (e != hipSuccess) return fail(NBG_E_OUT_OF_MEMORY, std::string("string tables: ") + hipGetErrorString(e));
  snap.device_bytes += (n + 1) * 4 + bytes.size() + n * 17;
  return NBG_OK;
}

DevStrings Engine::dev_strings() const {
  DevStrings s;
  s.off = snap.d_soff;
  s.bytes = snap.d_sbytes;
  s.s2i = snap.d_s2i;
  s.s2f = snap.d_s2f;
  s.s2ok = snap.d_s2ok;
  s.n = snap.strings.size();
  return s;
}

uint64_t Engine::sp_item_cap() const {
  // a level claims each vertex once; its items are its 64-entry runs over the side's types
  uint64_t pos_types = 0, e_out = 0, e_in = 0;
  for (auto& kv : snap.types) {
    if (kv.first > 0) { ++pos_types; e_out += kv.second.num_edges; }
    else e_in += kv.second.num_edges;
  }
  return snap.nv * std::max<uint64_t>(pos_types, 1) + std::max(e_out, e_in) / 64 + 1024;
}

uint64_t Engine::sp_edge_cap() const {
  uint64_t e_out = 0, e_in = 0;
  for (auto& kv : snap.types) (kv.first > 0 ? e_out : e_in) += kv.second.num_edges;
  return std::max(e_out, e_in) + 1;
}

SpCtx* Engine::new_sp(hipStream_t s, std::string* err) {
  SpCtx* c = sp_create(snap.nv, sp_item_cap(), sp_edge_cap(), s, err);
  if (c && prof_mode) sp_profile(c, prof_mode);
  return c;
}

uint32_t Engine::dense(int64_t vid) const {
  auto& v = snap.h_vids;
  auto it = std::lower_bound(v.begin(), v.end(), vid);
  return (it != v.end() && *it == vid) ? (uint32_t)(it - v.begin()) : NO_ROW;
}

}  // namespace nbg

// ============================================================================= result objects
struct nbg_rows {
  struct Seg {
    uint64_t begin = 0, end = 0;
    int type = 0;                          // index into kinds / const_str (OVER position)
  };
  std::vector<std::vector<VKind>> kinds;              // per OVER type: value kind of each column
  std::vector<std::vector<std::string>> const_str;    // per OVER type: string constants absent from the dictionary
  Engine* eng = nullptr;
  Workspace* ws = nullptr;               // the workspace holding the rows (device results)
  Workspace* owned_ws = nullptr;         // set when the engine handed that workspace over (ws_release)
  int ncols = 0;
  uint64_t count = 0;
  bool on_device = false;
  bool fetched = false;
  std::vector<int64_t*> dcols;           // column bases; rows live in segs (disjoint regions)
  // host copy (nbg_rows_fetch): column c at hbits + c * count, in pinned memory from the engine's
  // pool (DMA straight from the packed device copy, no staging and no zero-fill)
  int64_t* hbits = nullptr;
  size_t hbytes = 0;
  std::vector<std::vector<uint8_t>> tags;   // per-cell kinds, built on the first nbg_rows_col_tags
  std::vector<std::string> strings;
  std::unordered_map<int64_t, std::string> derived;   // STR_DERIVED codes -> their text
  std::vector<Seg> segs;                 // built on first use from the per-workgroup counts
  struct TypeBlocks {
    uint64_t region = 0, blk_cap = 0;
    std::vector<uint32_t> counts;        // rows per workgroup of the final expansion
  };
  std::vector<TypeBlocks> blocks;
  bool segs_built = false;
  void build_segs() {
    if (segs_built) return;
    segs_built = true;
    size_t n = 0;
    for (auto& tb : blocks)
      for (uint32_t c : tb.counts) n += c != 0;
    segs.reserve(n);
    for (size_t i = 0; i < blocks.size(); ++i) {
      const TypeBlocks& tb = blocks[i];
      for (size_t b = 0; b < tb.counts.size(); ++b) {
        if (!tb.counts[b]) continue;
        Seg seg;
        seg.begin = tb.region + (uint64_t)b * tb.blk_cap;
        seg.end = seg.begin + tb.counts[b];
        seg.type = (int)i;
        segs.push_back(seg);
      }
    }
  }
  int64_t* col(int c) const { return hbits + (uint64_t)c * count; }
  // the kind of column c when every OVER type gives it the same one (else -1: per-cell tags)
  int col_kind(int c) const {
    int k = -1;
    for (auto& kv : kinds) {
      if ((int)kv.size() <= c) continue;
      if (k < 0) k = kv[c];
      else if (k != kv[c]) return -1;
    }
    return k < 0 ? VK_INT : k;
  }
  uint64_t scanned = 0;
  std::vector<uint64_t> step_frontier, step_edges;
  // the result schema (GoExecutor::setupInterimResult): NBG_T_* per column, what RowWriter wrote
  // per (OVER type, column), and the read-back hazards it implies (see go_prepare)
  std::vector<int32_t> col_types;
  std::vector<std::vector<uint8_t>> wclass;
  bool small_ok = false;     // the end-of-query kernel may have packed these rows (ws_host_small_rows)
  bool misaligned = false;   // some column's written bytes differ in length from what its reader takes
  bool float_col = false;    // a FLOAT column: InterimResult::getRows fails on it
};

namespace nbg {

// Pinned host blocks for fetched rows, reused across queries (a fresh pinned allocation per fetch
// would cost more than the copy itself); at most kPinnedIdle blocks are kept idle.
constexpr size_t kPinnedIdle = 4;

void* Engine::pinned_get(size_t bytes, size_t* got) {
  std::lock_guard<std::mutex> lg(pinned_mu);
  size_t best = pinned_free.size();
  for (size_t i = 0; i < pinned_free.size(); ++i)
    if (pinned_free[i].first >= bytes && (best == pinned_free.size() || pinned_free[i].first < pinned_free[best].first))
      best = i;
  if (best < pinned_free.size()) {
    void* p = pinned_free[best].second;
    *got = pinned_free[best].first;
    pinned_free.erase(pinned_free.begin() + (ptrdiff_t)best);
    return p;
  }
  const size_t cap = std::max<size_t>(bytes + bytes / 8, 1 << 20);   // a little room to grow into
  void* p = nullptr;
  if (hipHostMalloc(&p, cap, hipHostMallocDefault) != hipSuccess) return nullptr;
  *got = cap;
  return p;
}

void Engine::pinned_put(void* p, size_t bytes) {
  if (!p) return;
  std::lock_guard<std::mutex> lg(pinned_mu);
  pinned_free.emplace_back(bytes, p);
  if (pinned_free.size() > kPinnedIdle) {   // drop the smallest idle block
    size_t small = 0;
    for (size_t i = 1; i < pinned_free.size(); ++i)
      if (pinned_free[i].first < pinned_free[small].first) small = i;
    (void)hipHostFree(pinned_free[small].second);
    pinned_free.erase(pinned_free.begin() + (ptrdiff_t)small);
  }
}

void Engine::pinned_release() {
  std::lock_guard<std::mutex> lg(pinned_mu);
  for (auto& b : pinned_free) (void)hipHostFree(b.second);
  pinned_free.clear();
}

}  // namespace nbg

namespace {

// The rows of a result into host memory: the device packs the segments into contiguous columns
// and DMAs them into a pinned block (nbg.h nbg_rows_fetch).  Only STRING columns are touched per
// cell on the host (dictionary code -> the result's string table).
// RowWriter's written form of one value (RowWriter.cpp:103-186, RowWriter.inl:9-33): the value
// itself (ID), or the default it falls back to for an incompatible column type — varint 0 / a
// false byte (ONE zero byte) or a 0.0 double (EIGHT zero bytes).
enum WClass : uint8_t { W_ID = 0, W_ONE = 1, W_EIGHT = 2 };
WClass written_class(VKind k, int32_t t) {
  switch (k) {
    case VK_INT: return (t == NBG_T_INT || t == NBG_T_TIMESTAMP || t == NBG_T_VID) ? W_ID : W_ONE;
    case VK_DOUBLE: return (t == NBG_T_DOUBLE || t == NBG_T_FLOAT) ? W_ID : W_EIGHT;
    case VK_BOOL: return t == NBG_T_BOOL ? W_ID : W_ONE;
    default: return t == NBG_T_STRING ? W_ID : W_ONE;
  }
}
// does the reader of a `t` column take exactly the bytes written? (else the row's later columns
// are read at shifted positions)
bool read_aligned(WClass w, int32_t t) {
  if (w == W_ID) return true;
  if (w == W_ONE) return t == NBG_T_INT || t == NBG_T_TIMESTAMP || t == NBG_T_BOOL || t == NBG_T_STRING;
  return t == NBG_T_VID;
}
VKind read_kind(int32_t t) {   // the value InterimResult::getRows reads from a `t` column
  switch (t) {
    case NBG_T_BOOL: return VK_BOOL;
    case NBG_T_FLOAT: case NBG_T_DOUBLE: return VK_DOUBLE;
    case NBG_T_STRING: return VK_STRING;
    default: return VK_INT;
  }
}

// Rows whose schema makes RowReader read columns at shifted positions: the reference's bytes are
// rebuilt per row (RowWriter with the result schema) and read back column by column as
// InterimResult::getRows does (InterimResult.cpp:74-153); a read past the row's end fails the
// query.  Runs on the fetched host copy (strings already dictionary-decoded).
int32_t reread_rows(nbg_rows* r) {
  Engine& E = *r->eng;
  const int nc = r->ncols;
  std::vector<uint8_t> b;
  uint64_t o = 0;
  for (auto& s : r->segs) {
    const uint64_t len = s.end - s.begin;
    const std::vector<uint8_t>& wc = r->wclass[s.type];
    for (uint64_t i = o; i < o + len; ++i) {
      b.clear();
      for (int c = 0; c < nc; ++c) {
        const int64_t v = r->col(c)[i];
        const int32_t t = r->col_types[c];
        if (wc[c] == W_ONE) { b.push_back(0); continue; }
        if (wc[c] == W_EIGHT) { b.insert(b.end(), 8, 0); continue; }
        switch (t) {
          case NBG_T_BOOL: b.push_back(v != 0); break;
          case NBG_T_VID: case NBG_T_DOUBLE:
            for (int k = 0; k < 8; ++k) b.push_back((uint8_t)((uint64_t)v >> (8 * k)));
            break;
          case NBG_T_STRING: {
            const std::string& str = r->strings[(size_t)v];
            for (uint64_t n = str.size();; n >>= 7) {
              b.push_back((uint8_t)((n & 0x7f) | (n > 0x7f ? 0x80 : 0)));
              if (n <= 0x7f) break;
            }
            b.insert(b.end(), str.begin(), str.end());
            break;
          }
          default:   // INT / TIMESTAMP: varint of the two's-complement bits
            for (uint64_t n = (uint64_t)v;; n >>= 7) {
              b.push_back((uint8_t)((n & 0x7f) | (n > 0x7f ? 0x80 : 0)));
              if (n <= 0x7f) break;
            }
        }
      }
      size_t p = 0;
      for (int c = 0; c < nc; ++c) {
        const int32_t t = r->col_types[c];
        int64_t out = 0;
        bool ok = true;
        auto varint = [&](uint64_t* x) {
          *x = 0;
          for (int sh = 0; sh < 64; sh += 7) {
            if (p >= b.size()) return false;
            const uint8_t y = b[p++];
            *x |= (uint64_t)(y & 0x7f) << sh;
            if (!(y & 0x80)) return true;
          }
          return false;
        };
        switch (t) {
          case NBG_T_BOOL:
            ok = p < b.size();
            if (ok) out = b[p++] != 0;
            break;
          case NBG_T_VID: case NBG_T_DOUBLE:
            ok = p + 8 <= b.size();
            if (ok) {
              uint64_t x = 0;
              for (int k = 0; k < 8; ++k) x |= (uint64_t)b[p + k] << (8 * k);
              p += 8;
              out = (int64_t)x;
            }
            break;
          case NBG_T_STRING: {
            uint64_t n = 0;
            ok = varint(&n) && n <= b.size() - p;
            if (ok) {
              out = (int64_t)r->strings.size();
              r->strings.emplace_back(reinterpret_cast<const char*>(b.data() + p), (size_t)n);
              p += n;
            }
            break;
          }
          default: {
            uint64_t x = 0;
            ok = varint(&x);
            out = (int64_t)x;
          }
        }
        if (!ok) return E.fail(NBG_E_EXECUTION_ERROR, "Get value from interim failed (column " + std::to_string(c) + ")");
        r->col(c)[i] = out;
      }
    }
    o += len;
  }
  return NBG_OK;
}

int32_t materialize_rows(nbg_rows* r) {
  if (r->fetched) return NBG_OK;
  r->build_segs();
  Engine& E = *r->eng;
  // InterimResult::getRows has no case for a FLOAT column: "Unknown Type: 4" (InterimResult.cpp:142-146)
  if (r->float_col && r->count) return E.fail(NBG_E_EXECUTION_ERROR, "Unknown Type: 4");
  const auto& dict = E.snap.strings;
  const size_t bytes = std::max<size_t>((size_t)r->count * (size_t)r->ncols * 8, 8);
  r->hbits = static_cast<int64_t*>(E.pinned_get(bytes, &r->hbytes));
  if (!r->hbits) return NBG_E_OUT_OF_MEMORY;
  // packed at the query's end already (a small result, go_launch): the segments' cells in this order
  const int64_t* pre = r->count && r->ws && r->small_ok ? ws_host_small_rows(r->ws, r->count) : nullptr;
  if (pre) {
    memcpy(r->hbits, pre, (size_t)r->count * (size_t)r->ncols * 8);
  } else if (r->count) {
    std::vector<std::pair<uint64_t, uint64_t>> segs;
    segs.reserve(r->segs.size());
    for (auto& s : r->segs) segs.emplace_back(s.begin, s.end - s.begin);
    const hipError_t he = ws_fetch_rows_pinned(r->ws ? r->ws : E.ws, segs, r->ncols, r->count, r->hbits);
    if (he != hipSuccess)   // (named: round 4's one "row fetch failed" left no trace of the failing call)
      return E.fail(NBG_E_DEVICE, std::string("row fetch failed: ") + hipGetErrorName(he) + " (" +
                                      hipGetErrorString(he) + "), " + std::to_string(segs.size()) + " segments, " +
                                      std::to_string(r->count) + " rows");
  }
  bool any_string = false;
  for (auto& kv : r->kinds)
    for (VKind k : kv) any_string = any_string || k == VK_STRING;
  if (any_string) {
    std::unordered_map<int64_t, int64_t> sidx;
    uint64_t o = 0;
    for (auto& s : r->segs) {
      const uint64_t len = s.end - s.begin;
      for (int c = 0; c < r->ncols; ++c) {
        if (r->kinds[s.type][c] != VK_STRING) continue;   // payloads are final as copied
        int64_t* col = r->col(c);
        for (uint64_t i = o; i < o + len; ++i) {
          const int64_t code = col[i];
          auto it = sidx.find(code);
          if (it == sidx.end()) {
            std::string txt;
            if (is_derived_code(code)) {
              auto d = r->derived.find(code);
              if (d == r->derived.end()) return E.fail(NBG_E_DEVICE, "a derived string's text is missing");
              txt = d->second;
            } else {
              txt = (code >= 0 && (code & 1) == 0 && (uint64_t)(code / 2) < dict.size()) ? dict[code / 2]
                                                                                          : r->const_str[s.type][c];
            }
            it = sidx.emplace(code, (int64_t)r->strings.size()).first;
            r->strings.push_back(txt);
          }
          col[i] = it->second;
        }
      }
      o += len;
    }
  }
  if (r->misaligned && r->count) {
    const int32_t rc = reread_rows(r);
    if (rc) return rc;
  }
  r->fetched = true;
  return NBG_OK;
}

// per-cell kinds of column c (nbg_rows_col_tags), built on first use
const uint8_t* cell_tags(nbg_rows* r, int c) {
  if (r->tags.empty()) r->tags.resize(r->ncols);
  std::vector<uint8_t>& t = r->tags[c];
  if (t.size() != r->count) {
    t.resize(r->count);
    uint64_t o = 0;
    for (auto& s : r->segs) {
      const uint64_t len = s.end - s.begin;
      std::fill(t.begin() + (ptrdiff_t)o, t.begin() + (ptrdiff_t)(o + len), (uint8_t)r->kinds[s.type][c]);
      o += len;
    }
  }
  return t.data();
}

}  // namespace

// ============================================================================= GO driver
// A prepared GO statement: GoExecutor::prepare() (OVER / WHERE / YIELD validated, compiled once
// per OVER type, GoExecutor.cpp:136-263); execute() runs it from a start list.
struct nbg_go_stmt {
  Engine* eng = nullptr;
  uint64_t id = 0;                   // device program cache key
  std::vector<int32_t> over;
  std::vector<TypeProgram> plist;    // OVER order (default program where compilation deferred)
  int ncols = 0;
  uint32_t steps = 1;
  int32_t deferred = NBG_OK;         // name-resolution error, reported only if the final step runs
  std::string deferred_msg;
  std::string dst_unknown;           // a $$ tag name is unknown: fails once the final step has edges
  bool distinct = false;             // YIELD DISTINCT: distinct starts and rows
  std::vector<int32_t> col_types;    // the result schema (NBG_T_* per column)
  std::vector<std::vector<uint8_t>> wclass;   // per OVER position: WClass of each column
  bool misaligned = false, float_col = false;
  // $- / $var input: index rows (the FROM vid, ascending; last row per vid) and their columns,
  // uploaded on first execution (the same index on every rank of a partitioned engine)
  bool derived = false;              // some YIELD stores derived strings (OP_SOUT: the string arena)
  uint64_t sout_row_bytes = 0;       // arena bytes one final edge may store (the largest type's bound)
  uint64_t arena_bytes = 0;          // the arena a query reserves
  bool uses_input = false;
  std::vector<int64_t> in_ids;
  std::vector<std::vector<int64_t>> in_cols;
  int64_t* d_in_ids = nullptr;
  int64_t** d_in_cols = nullptr;
  std::vector<int64_t*> d_in_col_ptrs;
  // input strings absent from the snapshot's dictionary (codes STR_INPUT | index), their bytes
  // uploaded with the index
  std::vector<std::string> in_xstr;
  uint32_t* d_xoff = nullptr;
  char* d_xbytes = nullptr;
  ~nbg_go_stmt() {
    if (d_in_ids) (void)hipFree(d_in_ids);
    if (d_xoff) (void)hipFree(d_xoff);
    if (d_xbytes) (void)hipFree(d_xbytes);
    for (auto* p : d_in_col_ptrs)
      if (p) (void)hipFree(p);
    if (d_in_cols) (void)hipFree(d_in_cols);
  }
};

static bool has_input_prop(const Node* n) {
  if (!n) return false;
  if (n->kind == EK_INPUT || n->kind == EK_VAR) return true;
  for (auto& k : n->kids)
    if (has_input_prop(k.get())) return true;
  return false;
}

// Props a query names on each edge alias (Expression::prepare's alias set, Expressions.cpp:314-400)
static void alias_props(const Node* n, std::map<std::string, std::set<std::string>>& out) {
  if (!n) return;
  switch (n->kind) {
    case EK_ALIAS: case EK_DST: case EK_SRCID: case EK_RANK: case EK_TYPE:
      out[n->alias].insert(n->prop);
      break;
    default: break;
  }
  for (auto& k : n->kids) alias_props(k.get(), out);
}

// OVER * without YIELD: GoExecutor::finishExecution names one `<edge>._dst` column per entry of
// the first response's edge_schema, in that map's iteration order (GoExecutor.cpp:481-499,
// 546-561).  The order is libstdc++'s: storaged fills edgeContexts_ (an unordered_map, from the
// request's edge types, QueryBaseProcessor.inl:46-57, QueryBaseProcessor.h:114), copies it into
// the response's edge_schema (an unordered_map, QueryBoundProcessor.cpp:139-158), and graphd
// decodes that into another unordered_map (storage.thrift:104).  The same three containers, keyed
// the same way, reproduce it.
// the iteration order of storaged's edgeContexts_ for a request's edge types: the order
// processVertex emits a vertex's edge data in (QueryBaseProcessor.inl:46-57, QueryBoundProcessor.cpp:120-167)
static std::vector<int32_t> edge_context_order(const std::vector<int32_t>& req) {
  std::unordered_map<int32_t, int> contexts;
  std::transform(req.begin(), req.end(), std::inserter(contexts, contexts.end()),
                 [](int32_t t) { return std::make_pair(t, 0); });
  std::vector<int32_t> order;
  for (const auto& kv : contexts) order.push_back(kv.first);
  return order;
}

static std::vector<int32_t> response_schema_order(const std::vector<int32_t>& req) {
  std::unordered_map<int32_t, int> contexts;
  std::transform(req.begin(), req.end(), std::inserter(contexts, contexts.end()),
                 [](int32_t t) { return std::make_pair(t, 0); });
  std::unordered_map<int32_t, int> schema;
  for (const auto& kv : contexts)
    if (schema.find(kv.first) == schema.end()) schema.emplace(kv.first, 0);
  std::unordered_map<int32_t, int> decoded;
  for (const auto& kv : schema) decoded.emplace(kv.first, 0);
  std::vector<int32_t> order;
  for (const auto& kv : decoded) order.push_back(kv.first);
  return order;
}

static int32_t go_prepare(Engine& E, const nbg_go_request* rq, nbg_go_stmt** out) {
  if (!rq || !out) return E.fail(NBG_E_INVALID_ARGUMENT, "null argument");
  *out = nullptr;
  if (!E.finalized) return E.fail(NBG_E_STATE, "engine not finalized");
  if (rq->steps < 1) return E.fail(NBG_E_INVALID_ARGUMENT, "steps must be >= 1");
  // OVER (prepareOver / prepareOverAll, GoExecutor.cpp:197-263)
  std::vector<int32_t> over;
  if (rq->over_all) {
    for (auto& kv : E.edges) over.push_back(kv.first);
  } else {
    for (int32_t i = 0; i < rq->num_edge_types; ++i) {
      int32_t t = rq->edge_types[i];
      if (t <= 0) return E.fail(NBG_E_EXECUTION_ERROR, "`REVERSELY' not supported yet");
      if (!E.edges.count(t)) return E.fail(NBG_E_EXECUTION_ERROR, "edge type not found");
      over.push_back(t);
    }
  }
  if (over.empty()) return E.fail(NBG_E_EXECUTION_ERROR, "empty OVER clause");
  // WHERE / YIELD
  std::string err;
  std::unique_ptr<Node> where;
  if (rq->where && rq->where_len) {
    where = decode_expr(rq->where, rq->where_len, &err);
    if (!where) return E.fail(NBG_E_INVALID_ARGUMENT, "WHERE: " + err);
  }
  std::vector<std::unique_ptr<Node>> yields;
  for (int32_t i = 0; i < rq->num_yields; ++i) {
    auto y = decode_expr(rq->yields[i], rq->yield_lens[i], &err);
    if (!y) return E.fail(NBG_E_INVALID_ARGUMENT, "YIELD: " + err);
    yields.push_back(std::move(y));
  }
  if (yields.empty()) {   // default YIELD <edge>._dst per OVER edge (parser.yy:518-531)
    for (int32_t t : rq->over_all ? response_schema_order(over) : over) {
      auto n = std::make_unique<Node>();
      n->kind = EK_DST;
      n->alias = E.edges[t].name;
      n->prop = "_dst";
      yields.push_back(std::move(n));
    }
  }
  if ((int)yields.size() > MAX_YIELDS) return E.fail(NBG_E_UNSUPPORTED, "too many YIELD columns");
  const int ncols = (int)yields.size();
  // $- / $var input: the index GoExecutor::setupStarts builds on the FROM column
  bool uses_input = has_input_prop(where.get());
  for (auto& y : yields) uses_input = uses_input || has_input_prop(y.get());
  std::vector<std::string> in_names;
  std::vector<VKind> in_kinds;
  std::vector<int64_t> in_ids;
  std::vector<std::vector<int64_t>> in_cols;
  std::vector<std::string> in_xstr;   // input strings absent from the dictionary (sorted, unique)
  if (uses_input && rq->num_input_cols > 0) {
    if (rq->num_input_cols > MAX_INPUT_COLS)
      return E.fail(NBG_E_UNSUPPORTED, "more than " + std::to_string(MAX_INPUT_COLS) + " input columns");
    if (!rq->input_names || !rq->input_kinds || !rq->input_cols ||
        rq->input_vid_col < 0 || rq->input_vid_col >= rq->num_input_cols)
      return E.fail(NBG_E_INVALID_ARGUMENT, "input table");
    const uint64_t n = rq->num_input_rows;
    for (int32_t c = 0; c < rq->num_input_cols; ++c) {
      in_names.emplace_back(rq->input_names[c] ? rq->input_names[c] : "");
      in_kinds.push_back((VKind)rq->input_kinds[c]);
    }
    const int64_t* vidc = static_cast<const int64_t*>(rq->input_cols[rq->input_vid_col]);
    std::vector<std::pair<int64_t, uint64_t>> rowof;   // (vid, last row)
    {
      std::unordered_map<int64_t, uint64_t> last;
      for (uint64_t r = 0; r < n; ++r) last[vidc[r]] = r;   // vidToRowIndex_[v] = row: the last wins
      for (auto& kv : last) rowof.emplace_back(kv.first, kv.second);
      std::sort(rowof.begin(), rowof.end());
    }
    in_cols.assign(rq->num_input_cols, std::vector<int64_t>(rowof.size()));
    for (auto& pr : rowof) in_ids.push_back(pr.first);
    // strings the dictionary lacks (a string derived by an earlier statement of the pipe): a table of
    // their own, so they keep their bytes (a dictionary code between neighbours would not)
    for (int32_t c = 0; c < rq->num_input_cols; ++c)
      if (in_kinds[c] == VK_STRING)
        for (auto& pr : rowof) {
          const char* str = static_cast<const char* const*>(rq->input_cols[c])[pr.second];
          if (string_code(E.snap.strings, str ? str : "") & 1) in_xstr.emplace_back(str ? str : "");
        }
    std::sort(in_xstr.begin(), in_xstr.end());
    in_xstr.erase(std::unique(in_xstr.begin(), in_xstr.end()), in_xstr.end());
    for (int32_t c = 0; c < rq->num_input_cols; ++c) {
      for (size_t k = 0; k < rowof.size(); ++k) {
        const uint64_t r = rowof[k].second;
        if (in_kinds[c] == VK_STRING) {
          const char* str = static_cast<const char* const*>(rq->input_cols[c])[r];
          int64_t code = string_code(E.snap.strings, str ? str : "");
          if (code & 1)
            code = STR_INPUT |
                   (int64_t)(std::lower_bound(in_xstr.begin(), in_xstr.end(), std::string(str ? str : "")) - in_xstr.begin());
          in_cols[c][k] = code;
        } else {
          in_cols[c][k] = static_cast<const int64_t*>(rq->input_cols[c])[r];
        }
      }
    }
  } else if (uses_input) {
    return E.fail(NBG_E_EXECUTION_ERROR, "$- / $var props need the piped or variable input");
  }
  // compile per OVER type; name-resolution errors are reported only if the final step runs
  std::map<int32_t, TypeProgram> progs;
  int32_t deferred = NBG_OK;
  std::string deferred_msg, dst_unknown;
  std::map<std::string, std::set<std::string>> named;
  alias_props(where.get(), named);
  for (auto& y : yields) alias_props(y.get(), named);
  if (E.max_dict_len_of != E.snap.strings.size()) {   // (cached: the dictionary is fixed after finalize)
    E.max_dict_len = 0;
    for (const std::string& x : E.snap.strings) E.max_dict_len = std::max<uint64_t>(E.max_dict_len, x.size());
    E.max_dict_len_of = E.snap.strings.size();
  }
  for (int32_t t : over) {
    auto it = E.snap.types.find(t);
    CompileEnv env{t, &over, &E.edges, &E.snap.strings,
                   it != E.snap.types.end() && it->second.valid != nullptr,
                   it != E.snap.types.end() && it->second.rank != nullptr};
    env.max_dict_len = E.max_dict_len;
    // the response edge row schema of type t: _dst, then the props named on t (getStepOutProps,
    // GoExecutor.cpp:587-630)
    std::map<std::string, VKind> row_cols{{"_dst", VK_INT}};
    const SchemaSet& es = E.edges[t];
    for (auto& p : named[es.name]) {
      if (p == "_src" || p == "_dst" || p == "_type" || p == "_rank") { row_cols.emplace(p, VK_INT); continue; }
      const Schema* sc = es.latest();
      const int c = sc ? sc->find(p) : -1;
      if (c >= 0) row_cols.emplace(p, kindOfType(sc->cols[c].type));
    }
    uint32_t probe = 0;
    env.tags = &E.tags;
    env.dtags = &E.snap.tags;
    env.row_cols = &row_cols;
    env.partitioned = E.partitioned();
    env.dst_unknown = &dst_unknown;
    env.probe_mask = &probe;
    if (uses_input) {
      env.input_names = &in_names;
      env.input_kinds = &in_kinds;
      env.input_derived = !in_xstr.empty();
      for (const std::string& x : in_xstr) env.max_dict_len = std::max<uint64_t>(env.max_dict_len, x.size());
    }
    ProgramBuilder pb;
    TypeProgram tp;
    tp.etype = t;
    int32_t rc = NBG_OK;
    if (where) {
      Compiled c;
      rc = compile_expr(*where, env, pb, &c, &err);
      if (rc == NBG_OK) {
        tp.where_len = (int)pb.code.size();
        if (c.is_const) {
          bool tv;
          switch (c.kind) {
            case VK_STRING: tv = c.const_str.empty(); break;
            case VK_DOUBLE: { double d; memcpy(&d, &c.const_bits, 8); tv = d != 0.0; break; }
            default: tv = c.const_bits != 0;
          }
          tp.where_const = true;
          tp.where_const_val = tv;
          tp.where_len = 0;
          pb.code.clear();
        } else {
          // asBool of the WHERE value (GoExecutor.cpp:954)
          int r = c.reg;
          if (c.kind == VK_INT) pb.code.push_back(Ins{OP_TRUTHY_I, (uint8_t)r, (uint8_t)r, 0, 0, 0});
          else if (c.kind == VK_DOUBLE) pb.code.push_back(Ins{OP_TRUTHY_F, (uint8_t)r, (uint8_t)r, 0, 0, 0});
          else if (c.kind == VK_STRING)
            pb.code.push_back(Ins{OP_TRUTHY_S, (uint8_t)r, (uint8_t)r, 0, 0, string_code(E.snap.strings, "")});
          tp.where_len = (int)pb.code.size();
          tp.where_reg = r;
          tp.where_always_error = c.always_error;
        }
        pb.next_reg = 0;   // WHERE registers are dead once its value is read
      }
    }
    for (int y = 0; rc == NBG_OK && y < ncols; ++y) {
      Compiled c;
      rc = compile_expr(*yields[y], env, pb, &c, &err, true);
      if (rc) break;
      tp.yield_kind.push_back(c.kind);
      if (c.is_const) {
        tp.yield_reg.push_back(-1);
        tp.yield_const.push_back(c.const_bits);
        tp.yield_const_str.push_back(c.const_str);
      } else {
        tp.yield_const_str.push_back(std::string());
        tp.yield_reg.push_back(c.reg);
        tp.yield_const.push_back(0);
      }
    }
    if (rc == NBG_E_UNSUPPORTED || rc == NBG_E_INVALID_ARGUMENT) return E.fail(rc, err);
    if (rc) {
      if (!deferred) { deferred = rc; deferred_msg = err; }
      continue;
    }
    tp.code = pb.code;
    tp.data = pb.data;
    for (const Ins& i : tp.code) tp.sout = tp.sout || i.op == OP_SOUT || i.op == OP_SMAT;   // (the arena)
    tp.sout_bytes = pb.sout_bytes;
    tp.probe_mask = probe;
    tp.nregs = std::max(1, pb.max_reg);
    if ((int)(tp.code.size() + tp.data.size()) > MAX_PROGRAM) return E.fail(NBG_E_UNSUPPORTED, "program too long");
    if (tp.nregs > interp_max_regs())
      return E.fail(NBG_E_UNSUPPORTED, "expression too deep for the device register file (" + std::to_string(tp.nregs) +
                                           " registers, " + std::to_string(interp_max_regs()) + " fit the LDS)");
    progs[t] = std::move(tp);
  }
  if ((int)over.size() > MAX_TYPES_Q || rq->steps > (uint32_t)MAX_STEPS)
    return E.fail(NBG_E_UNSUPPORTED, "too many OVER types or steps");
  // ---- the result schema and what RowWriter makes of each value (GoExecutor::setupInterimResult,
  // GoExecutor.cpp:707-788).  The reference types every column from the FIRST row it evaluates
  // (yield_column_type) and writes every row through that schema: a value of another kind becomes
  // the writer's default (RowWriter.cpp:103-186), and a default of another length shifts the
  // columns after it when InterimResult::getRows reads the row back.  Which row is first follows
  // hash-map order; the canonical row here is an edge of the first type in the request's
  // edge-context order (QueryBaseProcessor.inl:46-57, the order processVertex emits edge data in)
  // whose source has the $^ tags the columns read.  Aligned defaults become constants of the
  // compiled programs (the expression still runs, so its errors still fail the query); shifted
  // rows are re-read on the host copy (reread_rows); a FLOAT column fails the fetch.
  std::vector<int32_t> ctype(ncols, NBG_T_INT);
  std::vector<std::vector<uint8_t>> wclass(over.size(), std::vector<uint8_t>(ncols, W_ID));
  bool misaligned = false, float_col = false;
  {
    const int32_t t0 = edge_context_order(over)[0];
    std::map<std::string, int32_t> row_types{{"_dst", NBG_T_VID}};
    for (auto& p : named[E.edges[t0].name]) {
      if (p == "_src" || p == "_dst") { row_types[p] = NBG_T_VID; continue; }
      if (p == "_rank" || p == "_type") { row_types[p] = NBG_T_INT; continue; }
      const Schema* sc = E.edges[t0].latest();
      const int c = sc ? sc->find(p) : -1;
      if (c >= 0) row_types[p] = sc->cols[c].type;
    }
    ColTypeEnv cenv;
    cenv.row_type = t0;
    cenv.edges = &E.edges;
    cenv.tags = &E.tags;
    cenv.row_types = &row_types;
    if (uses_input) {
      cenv.input_names = &in_names;
      cenv.input_kinds = &in_kinds;
    }
    auto p0 = progs.find(t0);
    if (p0 == progs.end()) p0 = progs.begin();
    for (int y = 0; y < ncols; ++y) {
      ctype[y] = yield_column_type(*yields[y], cenv);
      if (!ctype[y] && p0 != progs.end()) {
        const VKind k = p0->second.yield_kind[y];
        ctype[y] = k == VK_DOUBLE ? NBG_T_DOUBLE : k == VK_BOOL ? NBG_T_BOOL : k == VK_STRING ? NBG_T_STRING : NBG_T_INT;
      }
      if (!ctype[y]) ctype[y] = NBG_T_INT;
      float_col = float_col || ctype[y] == NBG_T_FLOAT;
    }
    for (size_t i = 0; i < over.size(); ++i) {
      auto it = progs.find(over[i]);
      if (it == progs.end()) continue;
      TypeProgram& tp = it->second;
      for (int y = 0; y < ncols; ++y) {
        const WClass w = written_class(tp.yield_kind[y], ctype[y]);
        wclass[i][y] = w;
        if (w == W_ID) continue;
        misaligned = misaligned || !read_aligned(w, ctype[y]);
        const VKind rk = read_kind(ctype[y]);
        tp.yield_reg[y] = -1;
        tp.yield_kind[y] = rk;
        tp.yield_const[y] = rk == VK_STRING ? string_code(E.snap.strings, "") : 0;
        tp.yield_const_str[y] = std::string();
      }
    }
  }
  // Derived strings (concatenation, casts to string): a YIELD column's string has ONE code
  // whatever produced it — the dictionary's, else STR_DERIVED | its content hash — so constant
  // strings absent from the dictionary take the hash code too (YIELD DISTINCT compares codes).
  bool derived = false;
  uint64_t sout_row = 0;
  for (auto& kv : progs) {
    derived = derived || kv.second.sout;
    sout_row = std::max(sout_row, kv.second.sout_bytes);
  }
  if (derived)
    for (auto& kv : progs)
      for (int y = 0; y < ncols; ++y) {
        TypeProgram& tp = kv.second;
        if (tp.yield_reg[y] >= 0 || tp.yield_kind[y] != VK_STRING || !(tp.yield_const[y] & 1)) continue;
        uint64_t h = STR_HASH_INIT;
        for (char ch : tp.yield_const_str[y]) h = str_hash_step(h, (uint8_t)ch);
        tp.yield_const[y] = str_derived_code(h, tp.yield_const_str[y].size());
      }
  static std::atomic<uint64_t> next_id{1};
  auto* st = new nbg_go_stmt();
  st->derived = derived;
  st->sout_row_bytes = sout_row;
  st->eng = &E;
  st->id = next_id++;
  st->over = over;
  st->plist.resize(over.size());
  for (size_t i = 0; i < over.size(); ++i) {
    auto it = progs.find(over[i]);
    if (it != progs.end()) st->plist[i] = std::move(it->second);
  }
  st->ncols = ncols;
  st->steps = rq->steps;
  st->deferred = deferred;
  st->deferred_msg = deferred_msg;
  st->dst_unknown = dst_unknown;
  st->distinct = rq->distinct != 0;
  st->col_types = std::move(ctype);
  st->wclass = std::move(wclass);
  st->misaligned = misaligned;
  st->float_col = float_col;
  st->uses_input = uses_input;
  st->in_ids = std::move(in_ids);
  st->in_cols = std::move(in_cols);
  st->in_xstr = std::move(in_xstr);
  *out = st;
  return NBG_OK;
}

// A GO query enqueued on a workspace, completed by go_collect.
struct GoPending {
  nbg_rows* rows = nullptr;
  Workspace* ws = nullptr;
  bool device = false;
  bool finished = false;                 // nothing was enqueued (no start has rows)
  // partitioned, in band: this rank's preparation failed but it took part in the query's
  // collectives; nbg_go_submit keeps the ticket in its slot (so every rank's slot sequence stays
  // the same) and nbg_go_wait reports the code
  int32_t failed_rc = NBG_OK;
  std::string failed_msg;
  std::vector<uint64_t> region, blk_cap;
};

// Enqueue the whole query (every step, the final-step rows and the end-of-query copy) on the
// workspace *wsp (its stream `stream`); no host synchronisation.  *wsp may be null (created here)
// or hold an earlier device result's rows (handed to it first, ws_release).
//
// Partitioned (every rank runs the same call): everything that can fail on one rank alone —
// workspace (re)creation, the input index, the back tracker, the start list's edge space, the
// row buffers — happens BEFORE the query's first collective and is agreed there (Comm::agree,
// one small all-reduce): either every rank enqueues the query or every rank returns the same
// code.  A device error after that point aborts the communicator (the peers' collectives fail).
// pre_rc: a failure the caller already had on this rank (nbg_go_submit's slot stream); it is
// reported through the same agreement as the preparation failures below, so the peers' collective
// sequence for the query still matches.
// sync: the caller waits for this query next (nbg_go_execute): its end kernel wakes the host by
// the mapped flag.  A submitted query is waited for by its event: the other slots' queries hide
// the wake-up, and the event lets the runtime retire finished work (six in flight ran ~1 %
// slower on the flag, profiles/r04_w/x_go_wake_ab*.txt).
static int32_t go_launch(Engine& E, const nbg_go_stmt* st, const int64_t* starts, uint64_t num_starts, bool device,
                         Workspace** wsp, hipStream_t stream, Comm* qcomm, GoPending* p, bool sync,
                         int32_t pre_rc = NBG_OK, const char* pre_msg = nullptr) {
  if (num_starts && !starts) return E.fail(NBG_E_INVALID_ARGUMENT, "null argument");
  if (hipSetDevice(E.cfg.device) != hipSuccess) return E.fail(NBG_E_DEVICE, "hipSetDevice failed");
  const bool part = E.partitioned();
  if (part && !qcomm) return E.fail(NBG_E_STATE, "partitioned engine without a communicator");
  const std::vector<int32_t>& over = st->over;
  const std::vector<TypeProgram>& plist = st->plist;
  const int ncols = st->ncols;
  const uint32_t steps = st->steps;
  const int32_t deferred = st->deferred;
  std::string err;
  // starts -> dense ids (duplicates kept)
  std::vector<uint32_t> f0;
  f0.reserve(num_starts);
  for (uint64_t i = 0; i < num_starts; ++i) {
    uint32_t d = E.dense(starts[i]);
    if (d != NO_ROW) f0.push_back(d);
  }
  if (st->distinct) {   // DISTINCT de-duplicates the starts too (GoExecutor.cpp:101-107)
    std::sort(f0.begin(), f0.end());
    f0.erase(std::unique(f0.begin(), f0.end()), f0.end());
  }
  std::unique_ptr<nbg_rows> rows(new nbg_rows());
  rows->eng = &E;
  rows->ncols = ncols;
  rows->on_device = device;
  p->device = device;
  // (partitioned: every rank runs the same collective sequence, even with no local start)
  if (f0.empty() && !part) {
    p->finished = true;
    p->rows = rows.release();
    return NBG_OK;
  }
  // ---- rank-local preparation: the first failure is kept and agreed below
  int32_t lrc = NBG_OK;
  std::string lmsg;
  auto local_fail = [&](int32_t code, const std::string& msg) {
    if (!lrc) { lrc = code; lmsg = msg; }
  };
  if (pre_rc) local_fail(pre_rc, pre_msg ? pre_msg : "query set-up failed");
  if (E.fault(NBG_FAULT_ALLOC)) local_fail(NBG_E_OUT_OF_MEMORY, "query workspace allocation failed (injected)");
  const uint32_t cap = (uint32_t)(E.cfg.max_edge_returned_per_vertex <= 0 ? 0x7fffffff
                                                                          : E.cfg.max_edge_returned_per_vertex);
  // The start list keeps duplicates, so its edge space is the one list not bounded by a type's
  // edge count: the device lists carry it in 32 bits, and the workspace's merge-path tile splits
  // must cover it (on a partitioned engine each rank checks its own share).
  uint64_t start_edges = 0;
  for (int32_t t : over) {
    auto it = E.snap.types.find(t);
    if (it == E.snap.types.end()) continue;
    uint64_t sum = 0;
    for (uint32_t d : f0) sum += std::min<uint64_t>(it->second.h_row_ptr[d + 1] - it->second.h_row_ptr[d], cap);
    start_edges = std::max(start_edges, sum);
  }
  if (f0.size() + start_edges >= 0xFFFFFFFFull)   // merge-path items (entries + edges) are 32-bit too
    local_fail(NBG_E_UNSUPPORTED, "the start list's edges exceed 2^32-1 (duplicated hub starts)");
  if (!lrc && *wsp) {   // rows of an earlier device result still there: hand the workspace to them
    const int32_t rrc = ws_release(E, wsp, stream);
    if (rrc) local_fail(rrc, E.last_error);
  }
  // room for a duplicated start list: the decision comes from the whole start list, the same on
  // every rank of a partitioned engine (its own share, f0, is at most that)
  const uint64_t need = part ? std::max<uint64_t>(num_starts, 1) : f0.size();
  const uint64_t e_need = std::max<uint64_t>(E.snap.max_edges(), start_edges);
  if (!lrc && (!*wsp || need > ws_cap_frontier(*wsp) || f0.size() + start_edges > ws_cap_items(*wsp))) {
    const uint64_t fcap = std::max<uint64_t>({need, E.snap.nv + 1024, ws_cap_frontier(*wsp ? *wsp : nullptr)});
    Workspace* fresh = ws_create(fcap, E.snap.nv, e_need, stream, &err);
    if (fresh && part && ws_set_partition(fresh, qcomm, E.npad) != hipSuccess) {
      ws_destroy(fresh);
      fresh = nullptr;
      err = "partition buffers";
    }
    if (fresh && E.row_reserve && ws_reserve_rows(fresh, E.row_reserve, E.col_reserve) != hipSuccess) {
      ws_destroy(fresh);
      fresh = nullptr;
      err = "result rows";
    }
    if (!fresh) {
      local_fail(NBG_E_OUT_OF_MEMORY, err);
    } else {
      if (*wsp) {
        ws_profile_inherit(fresh, *wsp);
        ws_destroy(*wsp);
      }
      *wsp = fresh;
    }
  }
  Workspace* ws = *wsp;
  if (ws) ws_set_wake(ws, sync);
  int64_t *bt = nullptr, *bt_in = nullptr;   // VertexBackTracker roots ($- / $var props after >= 2 steps)
  if (ws) ws_backtracker_off(ws);
  if (!lrc && st->uses_input) {
    auto* ms = const_cast<nbg_go_stmt*>(st);
    if (!ms->d_in_ids) {
      const size_t n = std::max<size_t>(ms->in_ids.size(), 1);
      bool ok = hipMalloc((void**)&ms->d_in_ids, n * 8) == hipSuccess &&
                hipMemcpy(ms->d_in_ids, ms->in_ids.data(), ms->in_ids.size() * 8, hipMemcpyHostToDevice) == hipSuccess;
      ms->d_in_col_ptrs.assign(ms->in_cols.size(), nullptr);
      for (size_t c = 0; ok && c < ms->in_cols.size(); ++c)
        ok = hipMalloc((void**)&ms->d_in_col_ptrs[c], n * 8) == hipSuccess &&
             hipMemcpy(ms->d_in_col_ptrs[c], ms->in_cols[c].data(), ms->in_cols[c].size() * 8, hipMemcpyHostToDevice) ==
                 hipSuccess;
      ok = ok && hipMalloc((void**)&ms->d_in_cols, std::max<size_t>(ms->in_cols.size(), 1) * 8) == hipSuccess &&
           hipMemcpy(ms->d_in_cols, ms->d_in_col_ptrs.data(), ms->in_cols.size() * 8, hipMemcpyHostToDevice) ==
               hipSuccess;
      if (ok && !ms->in_xstr.empty()) {   // the input-string table (DevStrings::x*)
        std::vector<uint32_t> off{0};
        std::string bytes;
        for (const std::string& x : ms->in_xstr) {
          bytes += x;
          off.push_back((uint32_t)bytes.size());
        }
        ok = bytes.size() < 0xFFFFFFFFull && hipMalloc((void**)&ms->d_xoff, off.size() * 4) == hipSuccess &&
             hipMemcpy(ms->d_xoff, off.data(), off.size() * 4, hipMemcpyHostToDevice) == hipSuccess &&
             hipMalloc((void**)&ms->d_xbytes, std::max<size_t>(bytes.size(), 1)) == hipSuccess &&
             hipMemcpy(ms->d_xbytes, bytes.data(), bytes.size(), hipMemcpyHostToDevice) == hipSuccess;
      }
      if (!ok) {
        // a later execution retries the upload from scratch
        if (ms->d_in_ids) (void)hipFree(ms->d_in_ids);
        for (auto*& q : ms->d_in_col_ptrs)
          if (q) (void)hipFree(q);
        if (ms->d_in_cols) (void)hipFree(ms->d_in_cols);
        if (ms->d_xoff) (void)hipFree(ms->d_xoff);
        if (ms->d_xbytes) (void)hipFree(ms->d_xbytes);
        ms->d_in_ids = nullptr;
        ms->d_in_cols = nullptr;
        ms->d_xoff = nullptr;
        ms->d_xbytes = nullptr;
        ms->d_in_col_ptrs.clear();
        local_fail(NBG_E_OUT_OF_MEMORY, "input index upload");
      }
    }
    if (!lrc && steps > 1 && ws_backtracker(ws, &bt, &bt_in) != hipSuccess)
      local_fail(NBG_E_OUT_OF_MEMORY, "backtracker");
  }
  // now() is the query's wall-clock second (WallClock::fastNowInSec); rand32 / rand64 draw from a
  // stream of the query's own
  const int64_t query_now = (int64_t)time(nullptr);
  const uint64_t query_seed = query_rand_seed();
  auto args_for = [&](const DevEdgeType& dt) {
    ExpandArgs a{};
    a.now_sec = query_now;
    a.rand_seed = query_seed;
    a.row_ptr = dt.row_ptr;
    a.col = dt.col;
    a.dst_vid = dt.dst_vid;
    a.rank = dt.rank;
    a.valid = dt.valid;
    a.visible = E.snap.d_visible;
    a.vids = E.snap.d_vids;
    a.props = dt.d_props;
    a.hprops = dt.props.data();
    a.hnarrow = dt.narrow.empty() ? nullptr : dt.narrow.data();
    a.hnarrow_bytes = dt.narrow_bytes.empty() ? nullptr : dt.narrow_bytes.data();
    a.cap = cap;
    a.tcols = E.snap.d_tcols;
    a.tpres = E.snap.d_tpres;
    a.gbase = E.partitioned() ? (uint32_t)((uint64_t)E.cfg.rank * E.npad) : 0u;
    a.bt = bt;
    a.bt_in = bt_in;
    a.str = E.dev_strings();
    if (st->uses_input) {
      a.in_ids = st->d_in_ids;
      a.in_n = st->in_ids.size();
      a.in_cols = st->d_in_cols;
      a.str.xoff = st->d_xoff;
      a.str.xbytes = st->d_xbytes;
      a.str.xn = st->in_xstr.size();
    }
    return a;
  };
  // final-step row regions: the frontier entering step N is a set (N >= 2) or the start list
  // (N == 1, exact edge count known on the host)
  const uint64_t n_final = steps == 1 ? f0.size() : E.snap.nv;
  std::vector<uint64_t> region(over.size()), blk_cap(over.size()), ebound(over.size());
  uint64_t cap_rows = 0;
  for (size_t i = 0; i < over.size(); ++i) {
    auto it = E.snap.types.find(over[i]);
    uint64_t eb = 0;
    if (it != E.snap.types.end()) {
      if (steps == 1) {
        for (uint32_t d : f0) eb += std::min<uint64_t>(it->second.h_row_ptr[d + 1] - it->second.h_row_ptr[d], cap);
      } else {
        eb = it->second.num_edges;
      }
    }
    ebound[i] = eb;
    blk_cap[i] = ws_final_blk_cap(n_final, eb);
    region[i] = cap_rows;
    cap_rows += blk_cap[i] * ws_final_grid(n_final, eb);
  }
  if (!lrc && ws_reserve_rows(ws, cap_rows, ncols) != hipSuccess) local_fail(NBG_E_OUT_OF_MEMORY, "result rows");
  if (!lrc && st->derived) {
    // derived strings: every final edge's OP_SOUTs may store up to the program's bound (the
    // longest text its piece lists can spell, plus each entry's header; ProgramBuilder::sout_bytes)
    // up to NBG_STR_ARENA_KB (default 2 GB); a query whose strings need more fails with
    // E_OUT_OF_MEMORY.  The bound covers every row the result can hold, so below the cap the
    // arena never overflows.
    static const uint64_t cap_kb =
        getenv("NBG_STR_ARENA_KB") ? strtoull(getenv("NBG_STR_ARENA_KB"), nullptr, 10) : (2ull << 20);
    // (a pad length read per edge leaves the bound unknown — ProgramBuilder::value_reg's 2^40 — so
    // such a statement reserves 256 bytes per row instead of the whole cap on every workspace, and a
    // query whose strings outgrow that fails with E_OUT_OF_MEMORY through the arena's overflow
    // flag, never truncates)
    const uint64_t per_row =
        st->sout_row_bytes >= (1ull << 40) ? 256 : std::max<uint64_t>(st->sout_row_bytes, 32);
    const uint64_t need = cap_rows > UINT64_MAX / per_row ? UINT64_MAX : cap_rows * per_row;
    const uint64_t want = std::min<uint64_t>(std::max<uint64_t>(need, 1ull << 20), std::max<uint64_t>(cap_kb, 1) << 10);
    if (ws_reserve_arena(ws, want) != hipSuccess) local_fail(NBG_E_OUT_OF_MEMORY, "derived-string arena");
  }
  // ---- agreement: the query runs on every rank or on none.  A statement whose only collectives
  // are the hop bitmaps and the statistics (no YIELD DISTINCT owner exchange, no $- / $var roots)
  // needs no host round trip for it: a rank whose preparation failed still takes part in those
  // collectives, with zero bitmaps and its status word in the statistics, and every rank fails the
  // query when it reads them (go_collect).  Other statements agree first (Comm::agree).
  static const bool force_agree = getenv("NBG_GO_AGREE") && atoi(getenv("NBG_GO_AGREE")) != 0;
  // A small first hop travels as per-owner slot arrays instead of npad-bit bitmaps (ws_set_hop_slots:
  // the single-root hop is one row on one rank, and sent 3.6 MB per rank at RMAT-26 / G = 8).  Its
  // bound comes from the degrees every rank holds (Engine::first_hop_bound), so every rank — a
  // failing one too — picks the same format.  NBG_GO_SLOTS=0 keeps bitmaps (read per query).
  uint64_t hop1_slots = 0;
  if (part && steps >= 2 && over.size() == 1 && !(st->uses_input && steps > 1) &&
      !(getenv("NBG_GO_SLOTS") && atoi(getenv("NBG_GO_SLOTS")) == 0)) {
    const uint64_t b = E.first_hop_bound(over[0], starts, num_starts, cap);
    const uint64_t stride = b == UINT64_MAX ? 0 : std::max<uint64_t>(64, (b + 63) / 64 * 64);
    if (stride && stride * 4 * 2 <= E.npad / 8) hop1_slots = stride;
  }
  // (YIELD DISTINCT too: its owner exchange runs in go_collect, which every rank leaves at the
  // in-band status before reaching it)
  const bool in_band = part && !st->uses_input && !force_agree;
  if (in_band) {
    if (lrc) {
      int32_t agreed = NBG_OK;
      const hipError_t he = part_empty_query(qcomm, stream, (int)steps - 1, E.fb_send, E.fb_recv, E.npad / 8,
                                             hop1_slots * 4, E.fb_gst, E.fb_hgst, lrc, &agreed);
      if (he != hipSuccess) {
        qcomm->abort();
        return E.fail(NBG_E_DEVICE, "query statistics exchange: " + qcomm->last);
      }
      p->finished = true;
      p->failed_rc = lrc;
      p->failed_msg = lmsg;
      return E.fail(lrc, lmsg);
    }
  } else if (part) {
    int32_t agreed = NBG_OK;
    ++E.host_agreements;
    if (qcomm->agree(stream, lrc, &agreed)) return E.fail(NBG_E_DEVICE, "query agreement: " + qcomm->last);
    if (agreed) {
      if (lrc) return E.fail(lrc, lmsg);
      return E.fail(agreed, "the query failed on another rank (code " + std::to_string(agreed) + ")");
    }
  } else if (lrc) {
    return E.fail(lrc, lmsg);
  }
  p->ws = ws;
  rows->ws = ws;
  // a short start list travels to the first expansion in its kernel arguments, with its edge
  // space over each OVER type computed here from the host CSR offsets (no k_relist launch)
  std::vector<InlineList> inl;
  if (f0.size() <= (size_t)INLINE_STARTS) {
    inl.resize(over.size());
    for (size_t i = 0; i < over.size(); ++i) {
      InlineList& il = inl[i];
      il = InlineList{};
      il.n_in = (uint32_t)f0.size();
      auto it = E.snap.types.find(over[i]);
      if (it == E.snap.types.end()) continue;
      const std::vector<uint32_t>& rp = it->second.h_row_ptr;
      for (uint32_t d : f0) {
        if (!E.snap.h_visible.empty() && !E.snap.h_visible[d]) continue;
        const uint32_t deg = std::min<uint32_t>(rp[d + 1] - rp[d], cap);
        if (!deg) continue;
        il.total += deg;
        il.id[il.n] = d;
        il.end[il.n] = il.total;
        il.rs[il.n] = rp[d];
        ++il.n;
      }
    }
  }
  auto inl_of = [&](size_t i, uint32_t s) -> const InlineList* { return s == 1 && !inl.empty() ? &inl[i] : nullptr; };
  hipError_t he = ws_begin_query(ws, f0.data(), f0.size(), &plist, st->id);
  // A tiny query — its walk bound (DevEdgeType::h_w2 / h_w3) keeps every step within one
  // workgroup — runs as one launch (ws_go_tiny); NBG_TINY=0 turns it off.
  static const bool tiny_on = !getenv("NBG_TINY") || atoi(getenv("NBG_TINY")) != 0;
  bool tiny = tiny_on && he == hipSuccess && !part && !device && !st->distinct && !st->uses_input && !st->derived &&
              over.size() == 1 && ncols > 0 && !deferred && !(plist[0].where_const && !plist[0].where_const_val) &&
              f0.size() <= (size_t)INLINE_STARTS && steps <= 3 && plist[0].nregs <= tiny_max_regs();
  const DevEdgeType* tdt = nullptr;
  if (tiny) {
    auto it = E.snap.types.find(over[0]);
    tdt = it == E.snap.types.end() ? nullptr : &it->second;
    tiny = tdt && (steps == 1 || (tdt->h_w2.size() == E.snap.nv && tdt->h_w3.size() == E.snap.nv));
  }
  if (tiny) {
    uint64_t bound = 0;
    for (uint32_t d : f0) {
      if (steps == 1) {
        const bool vis = E.snap.h_visible.empty() || E.snap.h_visible[d];
        bound += vis ? std::min<uint64_t>(tdt->h_row_ptr[d + 1] - tdt->h_row_ptr[d], cap) : 0;
      } else {
        bound += steps == 2 ? tdt->h_w2[d] : tdt->h_w3[d];
      }
    }
    tiny = bound <= TINY_EDGES;
  }
  if (tiny) {
    he = ws_go_tiny(ws, args_for(*tdt), f0.data(), (uint32_t)f0.size(), steps, plist[0], ncols);
    if (he != hipSuccess) return E.fail(NBG_E_DEVICE, std::string("HIP: ") + hipGetErrorString(he));
    ++E.tiny_queries;
    p->region.assign(1, 0);
    p->blk_cap.assign(1, TINY_EDGES);
    p->rows = rows.release();
    return NBG_OK;
  }
  uint64_t n_bound = f0.size();
  ws_set_mark_claims(ws, over.size() == 1);
  const bool inject = part && E.fault(NBG_FAULT_DEVICE);
  for (uint32_t s = 1; he == hipSuccess && s <= steps; ++s) {
    const bool final = s == steps;
    // the next step's first OVER type: the next frontier list carries its edge space
    ExpandArgs next0{};
    const ExpandArgs* np0 = nullptr;
    if (!final) {
      auto it0 = E.snap.types.find(over[0]);
      if (it0 != E.snap.types.end()) {
        next0 = args_for(it0->second);
        np0 = &next0;
      }
    }
    // (before the MARKs, on every rank: one without edges of the type runs none)
    if (s == 1 && !final && hop1_slots) he = ws_set_hop_slots(ws, hop1_slots);
    for (size_t i = 0; he == hipSuccess && i < over.size(); ++i) {
      auto it = E.snap.types.find(over[i]);
      if (it == E.snap.types.end()) continue;
      ExpandArgs a = args_for(it->second);
      a.bt_first = s == 1;
      if (!final) {
        he = ws_expand_mark(ws, a, n_bound, it->second.num_edges, (int)s, (int)i, inl_of(i, s), np0);
      } else if (deferred || (plist[i].where_const && !plist[i].where_const_val)) {
        he = ws_scan_only(ws, a, n_bound, (int)s, (int)i);
      } else {
        he = ws_expand_final(ws, a, n_bound, ebound[i], (int)s, (int)i, plist[i], region[i], blk_cap[i],
                             inl_of(i, s));
      }
    }
    if (inject) he = hipErrorLaunchFailure;   // NBG_FAULT_DEVICE: a device error between collectives
    if (!final && he == hipSuccess) {
      he = part ? ws_exchange(ws, (int)s, np0) : ws_finish_step(ws, (int)s, np0);
      n_bound = E.snap.nv;
    }
  }
  if (he == hipSuccess && part) he = ws_global_stats(ws, (int)over.size());
  // a single engine's result that will be fetched to the host is packed there by the end-of-query
  // kernel when it is small (one host round trip less for it; YIELD DISTINCT compacts the rows
  // after this point, so it fetches them the usual way).  A device result (rows left in HBM) is
  // not: its end kernel is the one-workgroup state copy, a later nbg_rows_fetch copies the rows.
  if (he == hipSuccess && !part && !st->distinct && ncols > 0 && !device) {
    SmallPack sp{};
    sp.ntypes = (int)over.size();
    sp.ncols = ncols;
    for (size_t i = 0; i < over.size(); ++i) {
      sp.region[i] = region[i];
      sp.blk_cap[i] = blk_cap[i];
      sp.grid[i] = ws_final_grid_of(ws, (int)i);
    }
    he = ws_end_query_async_small(ws, sp);
  } else if (he == hipSuccess) {
    he = ws_end_query_async(ws);
  }
  if (he != hipSuccess) {
    // the peers may already wait in this query's next collective: release them
    if (part) qcomm->abort();
    const std::string cm = part && !qcomm->last.empty() ? " (" + qcomm->last + ")" : "";
    return E.fail(NBG_E_DEVICE, std::string("HIP: ") + hipGetErrorString(he) + cm);
  }
  p->region = std::move(region);
  p->blk_cap = std::move(blk_cap);
  p->rows = rows.release();
  return NBG_OK;
}

// Wait for a launched query and build its result.
// The text of every derived-string code in a result (nbg_rows::derived): the arena entries the
// query's OP_SOUT stored, and the statement's constants that carry the hash code.  Partitioned
// with YIELD DISTINCT, rows have moved between ranks, so every rank's entries are all-gathered
// (each rank runs this for the same query, in submission order).
static int32_t derived_strings(Engine& E, const nbg_go_stmt* st, Workspace* ws, uint64_t used, bool gather,
                               nbg_rows* rows) {
  std::vector<char> buf;
  std::vector<std::pair<uint64_t, uint64_t>> parts;   // (offset, bytes) per rank in buf
  if (!gather) {
    if (ws_read_arena(ws, used, &buf) != hipSuccess) return E.fail(NBG_E_DEVICE, "derived-string arena read");
    parts.emplace_back(0, used);
  } else {
    Comm* cm = ws_get_comm(ws);
    hipStream_t s = ws_stream(ws);
    std::vector<uint64_t> sizes;
    const uint64_t u = used;
    if (cm->gather_u64(s, &u, 1, &sizes)) return E.fail(NBG_E_DEVICE, "derived strings: " + cm->last);
    uint64_t mx = 8;
    for (uint64_t x : sizes) mx = std::max(mx, x);
    uint64_t cap = 0;
    const char* arena = ws_arena(ws, &cap);
    char *send = nullptr, *recv = nullptr;
    bool ok = hipMalloc((void**)&recv, mx * sizes.size()) == hipSuccess;
    if (ok && cap < mx) ok = hipMalloc((void**)&send, mx) == hipSuccess &&
                             (!used || hipMemcpyAsync(send, arena, used, hipMemcpyDeviceToDevice, s) == hipSuccess);
    // (a rank that cannot allocate cannot take part: the communicator is aborted, as for any
    // device failure between collectives)
    ok = ok && cm->allgather(send ? send : arena, recv, mx, s) == 0;
    buf.resize(mx * sizes.size());
    ok = ok && hipMemcpyAsync(buf.data(), recv, buf.size(), hipMemcpyDeviceToHost, s) == hipSuccess &&
         hipStreamSynchronize(s) == hipSuccess;
    if (send) (void)hipFree(send);
    if (recv) (void)hipFree(recv);
    if (!ok) {
      cm->abort();
      return E.fail(NBG_E_DEVICE, "derived strings all-gather");
    }
    for (size_t q = 0; q < sizes.size(); ++q) parts.emplace_back(q * mx, sizes[q]);
  }
  auto add = [&](int64_t code, std::string text) {
    auto it = rows->derived.find(code);
    if (it == rows->derived.end()) rows->derived.emplace(code, std::move(text));
    else if (it->second != text) return false;   // two strings with one 62-bit hash
    return true;
  };
  for (auto& pr : parts) {
    for (uint64_t o = pr.first; o + 16 <= pr.first + pr.second;) {
      int64_t code;
      uint64_t len;
      memcpy(&code, buf.data() + o, 8);
      memcpy(&len, buf.data() + o + 8, 8);
      if (o + 16 + len > pr.first + pr.second) return E.fail(NBG_E_DEVICE, "derived-string arena entry");
      // (an OP_SMAT entry, code 0, is a nested function's inner string: no result cell holds it)
      if (is_derived_code(code) && !add(code, std::string(buf.data() + o + 16, len)))
        return E.fail(NBG_E_EXECUTION_ERROR, "derived-string hash collision");
      o += 16 + ((len + 7) & ~7ull);
    }
  }
  for (const TypeProgram& tp : st->plist)
    for (size_t y = 0; y < tp.yield_const.size(); ++y)
      if (tp.yield_reg[y] < 0 && tp.yield_kind[y] == VK_STRING && is_derived_code(tp.yield_const[y]) &&
          !add(tp.yield_const[y], tp.yield_const_str[y]))
        return E.fail(NBG_E_EXECUTION_ERROR, "derived-string hash collision");
  return NBG_OK;
}

static int32_t go_collect(Engine& E, const nbg_go_stmt* st, GoPending* p, nbg_rows** out) {
  nbg_rows* rows = p->rows;
  p->rows = nullptr;
  if (p->failed_rc) {
    delete rows;
    return E.fail(p->failed_rc, p->failed_msg);
  }
  if (p->finished) { *out = rows; return NBG_OK; }
  Workspace* ws = p->ws;
  const std::vector<int32_t>& over = st->over;
  const std::vector<TypeProgram>& plist = st->plist;
  const int ncols = st->ncols;
  const uint32_t steps = st->steps;
  const int32_t deferred = st->deferred;
  const std::vector<uint64_t>& region = p->region;
  const std::vector<uint64_t>& blk_cap = p->blk_cap;
  const bool device = p->device;
  hipError_t he = ws_end_query_wait(ws);
  if (he != hipSuccess) {
    delete rows;
    return E.fail(NBG_E_DEVICE, std::string("HIP: ") + hipGetErrorString(he));
  }
  if (E.partitioned()) {   // a rank whose preparation failed (go_launch, in-band statuses)
    const int32_t code = ws_host_gstatus(ws);
    if (code) {
      delete rows;
      return E.fail(code, "the query failed on another rank (code " + std::to_string(code) + ")");
    }
  }
  const QState& q = *ws_host_state(ws);
  // statistics of the whole query: this engine's, or summed over all ranks when partitioned
  unsigned long long g_err = q.err, g_n[MAX_STEPS + 2], g_e[MAX_STEPS + 2], g_tb = q.tagbits;
  if (E.partitioned()) {
    ws_host_gstats(ws, &g_err, g_n, g_e, &g_tb);
  } else {
    for (int s = 0; s < MAX_STEPS + 2; ++s) {
      g_n[s] = q.step_n[s];
      g_e[s] = 0;
      for (size_t i = 0; i < over.size(); ++i) g_e[s] += q.e_st[s][i];
    }
  }
  for (uint32_t s = 1; s <= steps; ++s) {
    rows->step_frontier.push_back(g_n[s]);
    rows->step_edges.push_back(g_e[s]);
    rows->scanned += g_e[s];
  }
  const bool reached_final = g_n[steps] > 0;
  if (reached_final && deferred) { delete rows; return E.fail(deferred, st->deferred_msg); }
  if (reached_final && g_e[steps] > 0 && !st->dst_unknown.empty()) {
    delete rows;
    return E.fail(NBG_E_EXECUTION_ERROR, st->dst_unknown);
  }
  if (g_err >= SPLIT_BAD) {
    delete rows;
    return E.fail(NBG_E_DEVICE, "internal: a frontier list's merge-path split did not describe its tile");
  }
  if (g_err >= ARENA_OVERFLOW) {
    delete rows;
    return E.fail(NBG_E_OUT_OF_MEMORY, "the derived strings of the result need " + std::to_string(q.arena_used >> 10) +
                                       " KB, more than the string arena's cap (NBG_STR_ARENA_KB)");
  }
  if (g_err) { delete rows; return E.fail(NBG_E_EXECUTION_ERROR, "WHERE/YIELD evaluation error"); }
  // a $$ default read for a tag no final destination has: VertexHolder::defaultFor fails
  if ((g_tb >> MAX_TAG_BITS) & ~g_tb & ((1ull << MAX_TAG_BITS) - 1)) {
    delete rows;
    return E.fail(NBG_E_EXECUTION_ERROR, "Unknown Vertex");
  }
  rows->col_types = st->col_types;
  rows->wclass = st->wclass;
  rows->misaligned = st->misaligned;
  rows->float_col = st->float_col;
  for (size_t i = 0; i < over.size(); ++i) {
    rows->kinds.push_back(plist[i].yield_kind);
    rows->const_str.push_back(plist[i].yield_const_str);
    const unsigned grid = ws_final_grid_of(ws, (int)i);   // 0: the final expansion did not run
    const uint32_t* per_block = ws_host_blk_rows(ws, (int)i);
    nbg_rows::TypeBlocks tb;
    tb.region = region[i];
    tb.blk_cap = blk_cap[i];
    tb.counts.assign(per_block, per_block + grid);
    uint64_t c = 0;
    for (uint32_t x : tb.counts) c += x;
    rows->count += c;
    rows->blocks.push_back(std::move(tb));
  }
  if (st->distinct && (rows->count || E.partitioned())) {
    // YIELD DISTINCT on the device: segments deduplicated and compacted in place; partitioned,
    // the survivors then travel to the rank their identity hashes to, which deduplicates again
    // (every rank takes part: the exchange is collective)
    auto segments = [&](std::vector<std::pair<size_t, size_t>>* where) {
      std::vector<std::array<uint64_t, 3>> segs;
      for (size_t i = 0; i < rows->blocks.size(); ++i) {
        const auto& tb = rows->blocks[i];
        for (size_t b = 0; b < tb.counts.size(); ++b) {
          if (!tb.counts[b]) continue;
          segs.push_back({tb.region + (uint64_t)b * tb.blk_cap, tb.counts[b], (uint64_t)i});
          if (where) where->emplace_back(i, b);
        }
      }
      return segs;
    };
    std::vector<std::pair<size_t, size_t>> where;   // (type, block) of each segment
    std::vector<std::array<uint64_t, 3>> segs = segments(&where);
    std::vector<uint32_t> kept;
    hipError_t de = ws_distinct(ws, segs, ncols, rows->kinds, &kept);
    rows->count = 0;
    for (size_t k = 0; de == hipSuccess && k < segs.size(); ++k) {
      rows->blocks[where[k].first].counts[where[k].second] = kept[k];
      rows->count += kept[k];
    }
    if (E.partitioned()) {
      // the exchange is collective: every rank takes part, a rank whose dedup pass failed with no
      // rows and its status, which travels with the exchange's counts (no agreement of its own)
      std::vector<DistinctBlock> db;
      int32_t gstatus = NBG_OK;
      const int32_t mine = de == hipSuccess ? NBG_OK : NBG_E_DEVICE;
      de = ws_distinct_exchange(ws, mine ? std::vector<std::array<uint64_t, 3>>{} : segments(nullptr), ncols,
                                rows->kinds, &db, mine, &gstatus);
      if (de == hipSuccess && gstatus) {
        delete rows;
        return E.fail(gstatus, mine ? std::string("YIELD DISTINCT: the dedup pass failed")
                                    : "YIELD DISTINCT failed on another rank (code " + std::to_string(gstatus) + ")");
      }
      rows->count = 0;
      for (size_t i = 0; de == hipSuccess && i < rows->blocks.size() && i < db.size(); ++i) {
        rows->blocks[i].region = db[i].region;
        rows->blocks[i].blk_cap = db[i].blk_cap;
        rows->blocks[i].counts = db[i].counts;
        for (uint32_t c : db[i].counts) rows->count += c;
      }
    }
    if (de != hipSuccess) {
      // a failure inside the owner exchange (after its first collective) leaves the peers in the
      // later collectives of this query: abort the communicator, as for any device failure
      // between collectives, so they fail at once instead of at NBG_COMM_TIMEOUT_S
      if (E.partitioned()) ws_get_comm(ws)->abort();
      delete rows;
      return E.fail(NBG_E_DEVICE, std::string("HIP (distinct): ") + hipGetErrorString(de));
    }
  }
  if (st->derived) {
    const int32_t rc = derived_strings(E, st, ws, q.arena_used, E.partitioned() && st->distinct, rows);
    if (rc) {
      delete rows;
      return rc;
    }
  }
  for (int c = 0; c < ncols; ++c) rows->dcols.push_back(ws_row_col(ws, c));
  rows->small_ok = !E.partitioned() && !st->distinct && !device;   // (go_launch packed a small result)
  if (!device) {
    int32_t rc = materialize_rows(rows);
    if (rc) {
      delete rows;
      return rc == NBG_E_EXECUTION_ERROR || rc == NBG_E_DEVICE ? rc : E.fail(rc, "row fetch failed");
    }
  } else if (rows->count) {
    E.holders[ws] = rows;   // the rows stay valid until nbg_rows_free (ws_release)
  }
  *out = rows;
  return NBG_OK;
}

static int32_t go_execute(Engine& E, const nbg_go_stmt* st, const int64_t* starts, uint64_t num_starts, bool device,
                          nbg_rows** out) {
  if (!out) return E.fail(NBG_E_INVALID_ARGUMENT, "null argument");
  *out = nullptr;
  GoPending p;
  int32_t rc = go_launch(E, st, starts, num_starts, device, &E.ws, E.stream, E.comm.get(), &p, true);
  if (rc) return rc;
  return go_collect(E, st, &p, out);
}

static int32_t go_impl(Engine& E, const nbg_go_request* rq, bool device, nbg_rows** out) {
  std::lock_guard<std::mutex> lg(E.mu);
  nbg_go_stmt* st = nullptr;
  int32_t rc = go_prepare(E, rq, &st);
  if (rc) return rc;
  rc = go_execute(E, st, rq->starts, rq->num_starts, device, out);
  delete st;
  return rc;
}

// ============================================================================= asynchronous GO
// Up to NBG_QUERY_SLOTS queries of one engine in flight: each on its own workspace and HIP
// stream, so the device overlaps one query's latency-bound small launches with another's
// expansion (graphd serves concurrent queries the same way, one executor per query).
struct nbg_go_ticket {
  nbg_go_stmt* st = nullptr;
  int slot = -1;
  GoPending p;
  bool done = false;
  int32_t rc = NBG_OK;
  nbg_rows* result = nullptr;
};

static int query_slots() {
  static const int n = [] {
    const char* v = getenv("NBG_QUERY_SLOTS");
    const int k = v ? atoi(v) : 6;
    return k < 1 ? 1 : (k > 16 ? 16 : k);
  }();
  return n;
}

// complete the oldest submitted ticket (its result stays in the ticket until nbg_go_wait)
static void complete_oldest(Engine& E) {
  auto* t = static_cast<nbg_go_ticket*>(E.inflight.front());
  E.inflight.erase(E.inflight.begin());
  t->rc = go_collect(E, t->st, &t->p, &t->result);
  t->done = true;
  E.slots[t->slot].ticket = nullptr;
}

int32_t nbg::ws_release(Engine& E, Workspace** wsp, hipStream_t stream) {
  auto it = E.holders.find(*wsp);
  if (it == E.holders.end()) return NBG_OK;
  // the fresh workspace first: on failure nothing changes (the rows keep their workspace, which
  // stays busy until they are freed)
  Comm* cm = ws_get_comm(*wsp);   // (the fresh workspace keeps the slot's communicator)
  std::string err;
  Workspace* fresh = ws_create(E.snap.nv + 1024, E.snap.nv, E.snap.max_edges(), stream, &err);
  if (fresh && E.partitioned() && ws_set_partition(fresh, cm ? cm : E.comm.get(), E.npad) != hipSuccess) {
    ws_destroy(fresh);
    fresh = nullptr;
    err = "partition buffers";
  }
  if (fresh && E.row_reserve && ws_reserve_rows(fresh, E.row_reserve, E.col_reserve) != hipSuccess) {
    ws_destroy(fresh);
    fresh = nullptr;
    err = "result rows";
  }
  if (!fresh)
    return E.fail(NBG_E_OUT_OF_MEMORY, "a held device result occupies the query workspace and a new one could not be "
                                       "allocated (" + err + "); free device results first");
  nbg_rows* r = it->second;
  E.holders.erase(it);
  r->owned_ws = *wsp;
  ws_profile_inherit(fresh, *wsp);
  *wsp = fresh;
  return NBG_OK;
}

// The query workspace of a finalized (or snapshot-loaded) engine.
int32_t nbg::engine_ready(Engine& E) {
  if (int32_t rc = E.upload_strings()) return rc;
  if (E.partitioned() && !E.snap.d_zero_rows) {   // (path.cpp: OVER types this rank has no edges of)
    const size_t zb = ((size_t)E.snap.nv + 1) * 4;
    if (hipMalloc((void**)&E.snap.d_zero_rows, zb) != hipSuccess || hipMemset(E.snap.d_zero_rows, 0, zb) != hipSuccess)
      return E.fail(NBG_E_OUT_OF_MEMORY, "empty CSR rows");
  }
  static const bool tiny_on = !getenv("NBG_TINY") || atoi(getenv("NBG_TINY")) != 0;
  if (!E.partitioned() && tiny_on) {   // walk bounds of the tiny GO path (a failure only disables it)
    const uint32_t cap = (uint32_t)(E.cfg.max_edge_returned_per_vertex <= 0 ? 0x7fffffff
                                                                            : E.cfg.max_edge_returned_per_vertex);
    for (auto& kv : E.snap.types)
      if (kv.first > 0)
        (void)tiny_bounds(kv.second.row_ptr, kv.second.col, E.snap.d_visible, cap, E.snap.nv, &kv.second.h_w2,
                          &kv.second.h_w3, E.stream);
  }
  std::string err;
  E.ws = ws_create(E.snap.nv + 1024, E.snap.nv, E.snap.max_edges(), E.stream, &err);
  if (!E.ws) return E.fail(NBG_E_OUT_OF_MEMORY, err);
  if (E.partitioned()) {
    hipError_t he = ws_set_partition(E.ws, E.comm.get(), E.npad);
    const size_t G = (size_t)E.cfg.num_gpus, seg = E.npad / 8, gw = part_gst_words((int)G);
    if (he == hipSuccess) he = hipMalloc(&E.fb_send, G * seg);
    if (he == hipSuccess) he = hipMemset(E.fb_send, 0, G * seg);
    if (he == hipSuccess) he = hipMalloc(&E.fb_recv, G * seg);
    if (he == hipSuccess) he = hipMalloc((void**)&E.fb_gst, gw * 8);
    if (he == hipSuccess) he = hipHostMalloc((void**)&E.fb_hgst, gw * 8, hipHostMallocDefault);
    if (he != hipSuccess) return E.fail(NBG_E_OUT_OF_MEMORY, std::string("partition buffers: ") + hipGetErrorString(he));
    return build_path_replica(E);   // collective: every rank finalizes together
  }
  return NBG_OK;
}

// ============================================================================= C ABI
extern "C" {

int32_t nbg_go_submit(nbg_go_stmt* st, const int64_t* starts, uint64_t num_starts, int32_t device,
                      nbg_go_ticket** out) {
  if (!st || !st->eng || !out) return NBG_E_INVALID_ARGUMENT;
  Engine& E = *st->eng;
  std::lock_guard<std::mutex> lg(E.mu);
  *out = nullptr;
  if (hipSetDevice(E.cfg.device) != hipSuccess) return E.fail(NBG_E_DEVICE, "hipSetDevice failed");
  if (E.slots.empty()) E.slots.resize(query_slots());
  int slot = -1;
  for (size_t i = 0; i < E.slots.size() && slot < 0; ++i)
    if (!E.slots[i].ticket) slot = (int)i;
  if (slot < 0) {   // every slot busy: finish the oldest query first
    const int s0 = static_cast<nbg_go_ticket*>(E.inflight.front())->slot;
    complete_oldest(E);
    slot = s0;
  }
  Engine::QuerySlot& q = E.slots[slot];
  // A partitioned engine's queries are collectives.  Each slot gets its own communicator (a
  // split of the engine's, made collectively the first time the slot is used: every rank submits
  // the same queries in the same order, so it picks the same slot at the same call), and so its
  // own stream: the ranks issue every communicator's collectives in one order, and queries of
  // different slots overlap on the device.  Without a split (in-process transport, or
  // NBG_SLOT_COMMS=0) the slots share the engine's stream and communicator, one query after
  // another on the device.
  if (E.partitioned() && !q.comm_tried) {
    q.comm_tried = true;
    static const bool split_ok = !getenv("NBG_SLOT_COMMS") || atoi(getenv("NBG_SLOT_COMMS")) != 0;
    if (split_ok) {
      std::string err;
      q.comm.reset(E.comm->split(&err));
      // the split is collective: keep it only if every rank got one (else all share the engine's)
      if (E.comm->kind() != std::string("local")) {
        int32_t agreed = NBG_OK;
        if (E.comm->agree(E.stream, q.comm ? NBG_OK : NBG_E_DEVICE, &agreed))
          return E.fail(NBG_E_DEVICE, "slot communicator agreement: " + E.comm->last);
        if (agreed) q.comm.reset();
      }
    }
  }
  const bool own_stream = !E.partitioned() || q.comm != nullptr;
  Comm* const qcomm = q.comm ? q.comm.get() : E.comm.get();
  hipStream_t qstream = own_stream ? q.stream : E.stream;
  int32_t pre_rc = NBG_OK;
  const bool stream_fault = own_stream && E.fault(NBG_FAULT_STREAM);
  if (own_stream && (!q.stream || stream_fault)) {
    if (stream_fault || hipStreamCreateWithFlags(&q.stream, hipStreamNonBlocking) != hipSuccess) {
      if (!stream_fault) q.stream = nullptr;
      if (!E.partitioned()) return E.fail(NBG_E_DEVICE, "hipStreamCreate failed");
      // the peers run this query's collectives (in band or an agreement, per statement): fail it
      // with them through go_launch, on the engine's stream
      pre_rc = NBG_E_DEVICE;
      qstream = E.stream;
    } else {
      qstream = q.stream;
    }
  }
  auto* t = new nbg_go_ticket();
  t->st = st;
  t->slot = slot;
  int32_t rc = go_launch(E, st, starts, num_starts, device != 0, &q.ws, qstream, qcomm, &t->p, false, pre_rc,
                         "hipStreamCreate failed");
  // an in-band failure keeps its slot like any submitted query (the peers' slot holds theirs);
  // nbg_go_wait returns the code
  if (rc && !t->p.failed_rc) { delete t; return rc; }
  q.ticket = t;
  E.inflight.push_back(t);
  *out = t;
  return NBG_OK;
}

int32_t nbg_go_wait(nbg_go_ticket* t, nbg_rows** out) {
  if (!t || !out) return NBG_E_INVALID_ARGUMENT;
  Engine& E = *t->st->eng;
  std::lock_guard<std::mutex> lg(E.mu);
  *out = nullptr;
  if (!t->done) {
    // complete every older ticket first (their results stay in their tickets)
    while (!E.inflight.empty() && E.inflight.front() != t) complete_oldest(E);
    complete_oldest(E);
  }
  const int32_t rc = t->rc;
  *out = t->result;
  delete t;
  return rc;
}


int32_t nbg_create(const nbg_config* cfg, nbg_engine** out) {
  if (!cfg || !out) return NBG_E_INVALID_ARGUMENT;
  if (cfg->num_parts <= 0 || cfg->num_gpus <= 0 || cfg->rank < 0 || cfg->rank >= cfg->num_gpus)
    return NBG_E_INVALID_ARGUMENT;
  auto* h = new nbg_engine();
  h->e.cfg = *cfg;
  if (h->e.cfg.max_edge_returned_per_vertex <= 0) h->e.cfg.max_edge_returned_per_vertex = 0x7fffffff;
  *out = h;
  return NBG_OK;
}

void nbg_destroy(nbg_engine* h) {
  if (!h) return;
  Engine& E = h->e;
  while (!E.inflight.empty()) {   // tickets never waited for
    auto* t = static_cast<nbg_go_ticket*>(E.inflight.front());
    complete_oldest(E);
    if (t->result) nbg_rows_free(t->result);
    t->result = nullptr;
    delete t;
  }
  E.holders.clear();   // results must be freed before nbg_destroy (nbg.h)
  for (auto& q : E.slots) {
    if (q.stream) (void)hipStreamSynchronize(q.stream);
    if (q.ws) ws_destroy(q.ws);
    q.comm.reset();
    if (q.stream) (void)hipStreamDestroy(q.stream);
  }
  path_slots_release(E);
  destroy_path_replica(E);
  if (E.stream) (void)hipStreamSynchronize(E.stream);
  for (void* p : {E.fb_send, E.fb_recv, (void*)E.fb_gst})
    if (p) (void)hipFree(p);
  if (E.fb_hgst) (void)hipHostFree(E.fb_hgst);
  E.pinned_release();
  if (E.ws) ws_destroy(E.ws);
  if (E.sp) sp_destroy(E.sp);
  E.free_snapshot();
  if (E.stream) (void)hipStreamDestroy(E.stream);
  delete h;
}

int32_t nbg_inject_fault(nbg_engine* h, int32_t site, int32_t count) {
  if (!h || site < 0 || count < 0) return NBG_E_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lg(h->e.mu);
  h->e.fault_site = count ? site : 0;
  h->e.fault_count = count;
  return NBG_OK;
}

int32_t nbg_staged_edges(const nbg_engine* h, int32_t type, int64_t* src, int64_t* dst, int64_t* rank, uint64_t cap,
                         uint64_t* n) {
  if (!h || !n || type == 0) return NBG_E_INVALID_ARGUMENT;
  const Engine& E = h->e;
  std::lock_guard<std::mutex> lg(const_cast<Engine&>(E).mu);
  if (E.finalized) return NBG_E_STATE;
  *n = 0;
  auto it = E.stage.find(type);
  if (it == E.stage.end()) return NBG_OK;
  const EdgeStage& st = it->second;
  *n = st.size();
  const uint64_t m = std::min<uint64_t>(cap, st.size());
  for (uint64_t i = 0; i < m; ++i) {
    if (src) src[i] = st.src[i];
    if (dst) dst[i] = st.dst[i];
    if (rank) rank[i] = st.rank.empty() ? 0 : st.rank[i];
  }
  return NBG_OK;
}

const char* nbg_last_error(const nbg_engine* h) { return h ? h->e.last_error.c_str() : "null engine"; }

static int32_t reg_schema(std::map<int32_t, SchemaSet>& m, int32_t id, const char* name, int64_t ver,
                          const nbg_column_def* cols, int32_t ncols) {
  if (!name || ncols < 0 || (ncols && !cols)) return NBG_E_INVALID_ARGUMENT;
  SchemaSet& ss = m[id];
  ss.name = name;
  Schema s;
  s.version = ver;
  for (int32_t i = 0; i < ncols; ++i) {
    if (!cols[i].name) return NBG_E_INVALID_ARGUMENT;
    s.cols.push_back(Column{cols[i].name, cols[i].type});
  }
  ss.versions[ver] = s;
  return NBG_OK;
}

int32_t nbg_register_tag(nbg_engine* h, int32_t tag_id, const char* name, int64_t ver, const nbg_column_def* cols,
                         int32_t ncols) {
  if (!h) return NBG_E_INVALID_ARGUMENT;
  if (h->e.finalized) return h->e.fail(NBG_E_STATE, "engine already finalized");
  return reg_schema(h->e.tags, tag_id, name, ver, cols, ncols);
}

int32_t nbg_register_edge(nbg_engine* h, int32_t edge_type, const char* name, int64_t ver,
                          const nbg_column_def* cols, int32_t ncols) {
  if (!h) return NBG_E_INVALID_ARGUMENT;
  if (h->e.finalized) return h->e.fail(NBG_E_STATE, "engine already finalized");
  if (edge_type <= 0) return h->e.fail(NBG_E_INVALID_ARGUMENT, "edge types are positive");
  return reg_schema(h->e.edges, edge_type, name, ver, cols, ncols);
}

int32_t nbg_load_part_kv(nbg_engine* h, int32_t part, const uint8_t* kd, const uint64_t* ko, const uint8_t* vd,
                         const uint64_t* vo, uint64_t n) {
  if (!h || (n && (!kd || !ko || !vd || !vo))) return NBG_E_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lg(h->e.mu);
  return h->e.load_part_kv(part, kd, ko, vd, vo, n);
}

int32_t nbg_load_edges(nbg_engine* h, int32_t edge_type, const int64_t* src, const int64_t* dst, const int64_t* rank,
                       uint64_t n, const void* const* prop_cols, int32_t ncols) {
  if (!h || (n && (!src || !dst)) || (ncols && !prop_cols)) return NBG_E_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lg(h->e.mu);
  return h->e.load_edges(edge_type, src, dst, rank, n, prop_cols, ncols);
}

int32_t nbg_finalize(nbg_engine* h) {
  if (!h) return NBG_E_INVALID_ARGUMENT;
  Engine& E = h->e;
  std::lock_guard<std::mutex> lg(E.mu);
  if (hipSetDevice(E.cfg.device) != hipSuccess) return E.fail(NBG_E_DEVICE, "hipSetDevice failed");
  if (!E.stream && hipStreamCreateWithFlags(&E.stream, hipStreamNonBlocking) != hipSuccess)
    return E.fail(NBG_E_DEVICE, "hipStreamCreate failed");
  int32_t rc = E.finalize();
  if (rc) return rc;
  return engine_ready(E);
}

int32_t nbg_get_stats(const nbg_engine* h, nbg_stats* out) {
  if (!h || !out) return NBG_E_INVALID_ARGUMENT;
  const Engine& E = h->e;
  memset(out, 0, sizeof(*out));
  out->num_vertices = E.snap.nv;
  for (auto& kv : E.snap.types) out->num_edges += kv.second.num_edges;
  out->device_bytes = E.snap.device_bytes;
  out->num_edge_types = (int32_t)E.snap.types.size();
  out->tiny_queries = E.tiny_queries;
  out->host_agreements = E.host_agreements;
  out->path_batch_contexts = E.batch_sp.size();
  out->path_batch_reruns = E.batch_reruns;
  uint64_t hb = 0;
  for (const std::string& x : E.snap.strings) hb += x.size() + sizeof(std::string);
  for (auto& kv : E.snap.types)
    hb += (kv.second.h_row_ptr.size() + kv.second.h_w2.size() / 2 + kv.second.h_w3.size() / 2) * 4;
  hb += E.snap.h_visible.size();
  out->host_bytes = hb;
  return NBG_OK;
}

int32_t nbg_go(nbg_engine* h, const nbg_go_request* req, nbg_rows** out) {
  if (!h) return NBG_E_INVALID_ARGUMENT;
  return go_impl(h->e, req, false, out);
}

int32_t nbg_go_device(nbg_engine* h, const nbg_go_request* req, nbg_rows** out) {
  if (!h) return NBG_E_INVALID_ARGUMENT;
  return go_impl(h->e, req, true, out);
}

int32_t nbg_go_default_columns(nbg_engine* h, const int32_t* over, int32_t n, int32_t over_all, int32_t* out,
                               int32_t cap) {
  if (!h || n < 0 || (n && !over) || (cap && !out)) return NBG_E_INVALID_ARGUMENT;
  std::vector<int32_t> req(over, over + n);
  if (over_all) req = response_schema_order(req);
  for (int32_t i = 0; i < cap && i < (int32_t)req.size(); ++i) out[i] = req[i];
  return (int32_t)req.size();
}

// Result rows of a statement whose final frontier is a step's SET (N >= 2): the same bound
// go_launch computes per query, so a prepared statement's first execution allocates nothing.
static uint64_t stmt_row_bound(const Engine& E, const nbg_go_stmt* st) {
  uint64_t cap_rows = 0;
  for (int32_t t : st->over) {
    auto it = E.snap.types.find(t);
    const uint64_t eb = it == E.snap.types.end() ? 0 : it->second.num_edges;
    cap_rows += ws_final_blk_cap(E.snap.nv, eb) * ws_final_grid(E.snap.nv, eb);
  }
  return cap_rows;
}

int32_t nbg_go_prepare(nbg_engine* h, const nbg_go_request* req, nbg_go_stmt** out) {
  if (!h) return NBG_E_INVALID_ARGUMENT;
  Engine& E = h->e;
  std::lock_guard<std::mutex> lg(E.mu);
  const int32_t rc = go_prepare(E, req, out);
  if (rc || (*out)->steps < 2) return rc;
  // GoExecutor::prepare() validates once and execute() then only runs: size the row buffers of
  // the engine's workspace and of every query slot's now (growing a multi-GB buffer inside the
  // first execution cost that query ~0.2 s at RMAT-26).  A failure here is not an error: the
  // query grows (or fails) on its own.
  if (hipSetDevice(E.cfg.device) != hipSuccess) return NBG_OK;
  const uint64_t rows = stmt_row_bound(E, *out);
  auto reserve = [&](Workspace* w) {
    if (w && !E.holders.count(w)) (void)ws_reserve_rows(w, rows, (*out)->ncols);
  };
  reserve(E.ws);
  for (auto& q : E.slots) reserve(q.ws);
  E.row_reserve = std::max(E.row_reserve, rows);
  E.col_reserve = std::max(E.col_reserve, (*out)->ncols);
  return NBG_OK;
}

int32_t nbg_go_execute(nbg_go_stmt* st, const int64_t* starts, uint64_t num_starts, int32_t device, nbg_rows** out) {
  if (!st || !st->eng) return NBG_E_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lg(st->eng->mu);
  return go_execute(*st->eng, st, starts, num_starts, device != 0, out);
}

void nbg_go_stmt_free(nbg_go_stmt* st) { delete st; }

int64_t nbg_rows_count(const nbg_rows* r) { return r ? (int64_t)r->count : -1; }
int32_t nbg_rows_num_cols(const nbg_rows* r) { return r ? r->ncols : -1; }
uint64_t nbg_rows_edges_scanned(const nbg_rows* r) { return r ? r->scanned : 0; }

int32_t nbg_rows_step_stats(const nbg_rows* r, uint64_t* frontier, uint64_t* edges, int32_t cap) {
  if (!r) return NBG_E_INVALID_ARGUMENT;
  int32_t k = 0;
  for (; k < cap && k < (int32_t)r->step_frontier.size(); ++k) {
    if (frontier) frontier[k] = r->step_frontier[k];
    if (edges) edges[k] = k < (int32_t)r->step_edges.size() ? r->step_edges[k] : 0;
  }
  return k;
}

int32_t nbg_rows_fetch(nbg_rows* r) {
  if (!r) return NBG_E_INVALID_ARGUMENT;
  if (r->fetched) return NBG_OK;
  std::lock_guard<std::mutex> lg(r->eng->mu);   // the fetch runs on the result's workspace stream
  if (hipSetDevice(r->eng->cfg.device) != hipSuccess) return NBG_E_DEVICE;
  return materialize_rows(r);
}

const int64_t* nbg_rows_col_bits(const nbg_rows* r, int32_t col) {
  if (!r || !r->fetched || col < 0 || col >= r->ncols) return nullptr;
  return r->col(col);
}
const uint8_t* nbg_rows_col_tags(const nbg_rows* r, int32_t col) {
  if (!r || !r->fetched || col < 0 || col >= r->ncols) return nullptr;
  return cell_tags(const_cast<nbg_rows*>(r), col);
}
int32_t nbg_rows_col_kind(const nbg_rows* r, int32_t col) {
  if (!r || col < 0 || col >= r->ncols) return -1;
  return r->col_kind(col);
}
const char* nbg_rows_string(const nbg_rows* r, int64_t id) {
  if (!r || id < 0 || id >= (int64_t)r->strings.size()) return nullptr;
  return r->strings[id].c_str();
}
int64_t nbg_rows_num_segments(const nbg_rows* r) {
  if (!r) return -1;
  const_cast<nbg_rows*>(r)->build_segs();
  return (int64_t)r->segs.size();
}
int32_t nbg_rows_segment(const nbg_rows* r, int64_t i, uint64_t* begin, uint64_t* end) {
  if (r) const_cast<nbg_rows*>(r)->build_segs();
  if (!r || i < 0 || i >= (int64_t)r->segs.size() || !begin || !end) return NBG_E_INVALID_ARGUMENT;
  *begin = r->segs[i].begin;
  *end = r->segs[i].end;
  return NBG_OK;
}
const void* nbg_rows_device_col(const nbg_rows* r, int32_t col) {
  if (!r || col < 0 || col >= (int32_t)r->dcols.size()) return nullptr;
  return r->dcols[col];
}
int32_t nbg_rows_digest(const nbg_rows* r, uint64_t* out) {
  if (!r || !out) return NBG_E_INVALID_ARGUMENT;
  out[0] = out[1] = out[2] = 0;
  if (!r->count) return NBG_OK;
  if (r->fetched && !r->on_device) {   // host rows: the same chain on the host
    for (uint64_t i = 0; i < r->count; ++i) {
      uint64_t h = 0;
      for (int c = 0; c < r->ncols; ++c) {
        uint64_t z = (h ^ (uint64_t)r->col(c)[i]) + 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        h = z ^ (z >> 31);
      }
      ++out[0];
      out[1] ^= h;
      out[2] += h;
    }
    return NBG_OK;
  }
  Engine& E = *r->eng;
  std::lock_guard<std::mutex> lg(E.mu);
  if (hipSetDevice(E.cfg.device) != hipSuccess) return E.fail(NBG_E_DEVICE, "hipSetDevice failed");
  auto* m = const_cast<nbg_rows*>(r);
  m->build_segs();
  std::vector<std::pair<uint64_t, uint64_t>> segs;
  for (auto& sg : m->segs) segs.emplace_back(sg.begin, sg.end - sg.begin);
  const hipError_t he = ws_rows_digest(r->owned_ws ? r->owned_ws : r->ws, segs, r->ncols, out);
  return he == hipSuccess ? NBG_OK : E.fail(NBG_E_DEVICE, std::string("digest: ") + hipGetErrorString(he));
}

void nbg_rows_free(nbg_rows* r) {
  if (!r) return;
  if (r->eng && r->hbits) r->eng->pinned_put(r->hbits, r->hbytes);
  if (r->eng && (r->owned_ws || r->ws)) {
    Engine& E = *r->eng;
    std::lock_guard<std::mutex> lg(E.mu);
    auto it = E.holders.find(r->ws);
    if (it != E.holders.end() && it->second == r) E.holders.erase(it);
    if (r->owned_ws) {
      (void)hipSetDevice(E.cfg.device);
      ws_destroy(r->owned_ws);
    }
  }
  delete r;
}

int32_t nbg_set_path_replica(nbg_engine* h, int32_t mode) {
  if (!h || mode < 0 || mode > 1) return NBG_E_INVALID_ARGUMENT;
  Engine& E = h->e;
  std::lock_guard<std::mutex> lg(E.mu);
  if (!E.finalized) {   // before finalize: whether to build it
    E.path_replica_mode = mode;
    return NBG_OK;
  }
  if (mode && !E.rep) return E.fail(NBG_E_STATE, "this engine has no FIND PATH replica");
  E.path_replica_use = mode != 0;   // after: whether FIND PATH uses it
  return NBG_OK;
}

int32_t nbg_path_replica_active(const nbg_engine* h) { return h && h->e.rep && h->e.path_replica_use ? 1 : 0; }

int32_t nbg_profile(nbg_engine* h, int32_t enable) {
  if (!h) return NBG_E_INVALID_ARGUMENT;
  Engine& E = h->e;
  std::lock_guard<std::mutex> lg(E.mu);
  if (!E.ws) return E.fail(NBG_E_STATE, "engine not finalized");
  const int mode = enable == 2 ? 2 : (enable != 0 ? 1 : 0);
  ws_profile(E.ws, mode);
  // the one-pair SHORTEST contexts (device-driven chains): their launches and algorithmic bytes
  for (Engine* P : {&E, E.rep.get()}) {   // (and the FIND PATH replica's)
    if (!P) continue;
    P->prof_mode = mode;
    sp_profile(P->sp, mode);
    for (auto& ps : P->path_slots) sp_profile(ps.sp, mode);
    for (SpCtx* c : P->batch_sp) sp_profile(c, mode);
  }
  return NBG_OK;
}

int32_t nbg_profile_read(const nbg_engine* h, nbg_kernel_stat* out, int32_t cap) {
  if (!h || !out || !h->e.ws) return 0;
  const Engine& E = h->e;
  int n = ws_profile_read(E.ws, out, cap);
  double launches[CHAIN_KINDS] = {}, ms[CHAIN_KINDS] = {}, bytes[CHAIN_KINDS] = {};
  for (const Engine* P : {&E, (const Engine*)E.rep.get()}) {
    if (!P) continue;
    sp_profile_accum(P->sp, launches, ms, bytes);
    for (auto& ps : P->path_slots) sp_profile_accum(ps.sp, launches, ms, bytes);
    for (SpCtx* c : P->batch_sp) sp_profile_accum(c, launches, ms, bytes);
  }
  for (int k = 0; k < CHAIN_KINDS && n < cap; ++k, ++n) {
    out[n].name = kChainKernelNames[k];
    out[n].launches = (uint64_t)launches[k];
    out[n].total_ms = ms[k];
    out[n].algo_bytes = bytes[k];
  }
  return n;
}

int32_t nbg_find_path(nbg_engine* h, const nbg_path_request* req, nbg_paths** out);

int64_t nbg_paths_count(const nbg_paths* p) { return p ? (int64_t)p->paths.size() : -1; }
int64_t nbg_path_len(const nbg_paths* p, int64_t i) {
  return (p && i >= 0 && i < (int64_t)p->paths.size()) ? (int64_t)p->paths[i].size() : -1;
}
const int64_t* nbg_path_entries(const nbg_paths* p, int64_t i) {
  return (p && i >= 0 && i < (int64_t)p->paths.size()) ? p->paths[i].data() : nullptr;
}
uint64_t nbg_paths_edges_scanned(const nbg_paths* p) { return p ? p->edges : 0; }
uint32_t nbg_paths_chain_batches(const nbg_paths* p) { return p ? p->batches : 0; }
void nbg_paths_free(nbg_paths* p) { delete p; }

}  // extern "C"
