// SPDX: test infrastructure — NOT product code.
//
// CSR ORACLE: a second CPU restatement of the same semantics, over an in-memory CSR instead of
// the storaged-faithful KV store (storage.cpp / graph.cpp).  Two jobs:
//   * the checker at sizes the faithful restatement cannot reach in seconds (RMAT-22 full row
//     compares, RMAT-26 order-independent digests);
//   * CPU baseline mode (ii) of SURVEY.md §8(d): an OpenMP CSR GO / bidirectional BFS, the
//     honest "good CPU" denominator next to the storaged-faithful mode (i).
// It is pinned to the faithful restatement on RMAT <= 12 (tests/test_oracle_csr.py).  Only
// tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.
//
// Semantics restated (paths relative to the reference checkout):
//   * one live edge per (src, dst) — rank 0, the last sample wins (AddEdgesProcessor.cpp:15-37
//     same-key overwrite); in-edges mirror out-edges (InsertEdgeExecutor.cpp:180-196);
//   * GO N STEPS: starts keep duplicates; frontier_{s+1} = SET of _dst over the step's edges, no
//     global visited set (GoExecutor.cpp:501-541); final step: one row per (frontier entry, live
//     edge) passing WHERE (GoExecutor.cpp:803-984);
//   * FIND SHORTEST PATH s -> t UPTO n: minimal hop count, one path, ties broken by the
//     lexicographically smallest vid sequence (the build's canonical rule), length
//     >= 1 (s == t asks for the shortest cycle through s, FindPathExecutor.cpp:218-290).
#include <omp.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <numeric>
#include <vector>

namespace {

inline uint64_t mix64(uint64_t z) {   // splitmix64 finaliser
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
inline uint64_t splitmix64(uint64_t x) { return mix64(x + 0x9E3779B97F4A7C15ull); }

// per-query labels of one FIND SHORTEST PATH search (epoch-stamped: no clearing between queries);
// one per concurrent search (orc_csr_shortest_many runs one per thread)
struct SpCtx {
  std::vector<uint32_t> labf, labb, mark;   // mark: B-set position, epoch-stamped like the labels
  uint32_t epoch = 0;
  void init(uint64_t nv) {
    if (labf.size() == nv) return;
    labf.assign(nv, 0);
    labb.assign(nv, 0);
    mark.assign(nv, 0);
    epoch = 0;
  }
};

struct Csr {
  uint64_t nv = 0, ne = 0;
  std::vector<int64_t> vid;                 // dense id -> vid (bucket-major; not sorted)
  std::vector<uint64_t> off, ioff;          // out / in row offsets [nv + 1]
  std::vector<uint32_t> nbr, inbr;          // out / in neighbour dense ids
  std::vector<int64_t> w;                   // out-edge weight column
  // vid -> dense id: hash bucket, then binary search inside the bucket's sorted vids
  SpCtx sp;                                 // the single-query search's labels
  int bbits = 0;
  std::vector<uint64_t> bstart;             // [B + 1] first dense id of each bucket
  int threads = 1;

  uint64_t bucket_of(int64_t v) const { return mix64((uint64_t)v) >> (64 - bbits); }
  int64_t dense(int64_t v) const {
    const uint64_t b = bucket_of(v);
    auto lo = vid.begin() + bstart[b], hi = vid.begin() + bstart[b + 1];
    auto it = std::lower_bound(lo, hi, v);
    return (it != hi && *it == v) ? (int64_t)(it - vid.begin()) : -1;
  }
};

// Stable bucketing of `keys` by key -> bucket id (parallel counting sort); returns the bucket
// offsets and the permutation (order[i] = index into keys).
template <typename BucketFn>
void bucket_sort(uint64_t n, uint64_t nb, BucketFn bucket, int T, std::vector<uint64_t>& start,
                 std::vector<uint64_t>& order) {
  std::vector<uint64_t> cnt((uint64_t)T * nb, 0);
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num();
    const uint64_t b = n * t / T, e = n * (t + 1) / T;
    uint64_t* c = cnt.data() + (uint64_t)t * nb;
    for (uint64_t i = b; i < e; ++i) ++c[bucket(i)];
  }
  start.assign(nb + 1, 0);
  // bucket-major, thread-minor prefix: stable
  uint64_t run = 0;
  for (uint64_t k = 0; k < nb; ++k) {
    start[k] = run;
    for (int t = 0; t < T; ++t) {
      const uint64_t x = cnt[(uint64_t)t * nb + k];
      cnt[(uint64_t)t * nb + k] = run;
      run += x;
    }
  }
  start[nb] = run;
  order.resize(n);
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num();
    const uint64_t b = n * t / T, e = n * (t + 1) / T;
    uint64_t* c = cnt.data() + (uint64_t)t * nb;
    for (uint64_t i = b; i < e; ++i) order[c[bucket(i)]++] = i;
  }
}

Csr* build(const int64_t* src, const int64_t* dst, const int64_t* w, uint64_t n, int T) {
  const bool verbose = getenv("ORC_CSR_VERBOSE") != nullptr;
  auto t_last = std::chrono::steady_clock::now();
  auto phase = [&](const char* what) {
    auto now = std::chrono::steady_clock::now();
    if (verbose) fprintf(stderr, "csr build %s %.3fs\n", what, std::chrono::duration<double>(now - t_last).count());
    t_last = now;
  };
  auto* g = new Csr();
  g->threads = T;
  // ---- vertex dictionary: every endpoint, hashed into buckets, sorted and de-duplicated
  g->bbits = 8;
  while (g->bbits < 24 && (1ull << g->bbits) * 4096 < 2 * n) ++g->bbits;
  const uint64_t B = 1ull << g->bbits;
  std::vector<uint64_t> bst, order;
  bucket_sort(2 * n, B, [&](uint64_t i) { return g->bucket_of(i < n ? src[i] : dst[i - n]); }, T, bst, order);
  phase("bucket");
  std::vector<uint32_t> dense_of(2 * n);
  std::vector<uint64_t> bu(B + 1, 0);   // unique vids per bucket
  std::vector<std::vector<int64_t>> uniq(B);
#pragma omp parallel for schedule(dynamic, 64) num_threads(T)
  for (int64_t b = 0; b < (int64_t)B; ++b) {
    std::vector<int64_t>& u = uniq[b];
    for (uint64_t k = bst[b]; k < bst[b + 1]; ++k) {
      const uint64_t i = order[k];
      u.push_back(i < n ? src[i] : dst[i - n]);
    }
    std::sort(u.begin(), u.end());
    u.erase(std::unique(u.begin(), u.end()), u.end());
    bu[b + 1] = u.size();
  }
  for (uint64_t b = 0; b < B; ++b) bu[b + 1] += bu[b];
  g->nv = bu[B];
  g->bstart = bu;
  g->vid.resize(g->nv);
#pragma omp parallel for schedule(dynamic, 64) num_threads(T)
  for (int64_t b = 0; b < (int64_t)B; ++b) {
    std::copy(uniq[b].begin(), uniq[b].end(), g->vid.begin() + bu[b]);
    const std::vector<int64_t>& u = uniq[b];
    for (uint64_t k = bst[b]; k < bst[b + 1]; ++k) {
      const uint64_t i = order[k];
      const int64_t v = i < n ? src[i] : dst[i - n];
      dense_of[i] = (uint32_t)(bu[b] + (std::lower_bound(u.begin(), u.end(), v) - u.begin()));
    }
    std::vector<int64_t>().swap(uniq[b]);
  }
  std::vector<uint64_t>().swap(order);
  phase("dictionary");
  const uint64_t nv = g->nv;
  // ---- out CSR: edges grouped by dense source (atomic counting scatter), then per row sorted by
  // (dst, load order descending) — the first of each dst is the live edge (last sample wins)
  std::vector<uint64_t> rs(nv + 1, 0), eo(n);
  {
    std::vector<uint64_t> cnt(nv + 1, 0);
#pragma omp parallel for schedule(static) num_threads(T)
    for (int64_t i = 0; i < (int64_t)n; ++i) __atomic_fetch_add(&cnt[dense_of[i] + 1], 1ull, __ATOMIC_RELAXED);
    for (uint64_t d = 0; d < nv; ++d) cnt[d + 1] += cnt[d];
    rs = cnt;
#pragma omp parallel for schedule(static) num_threads(T)
    for (int64_t i = 0; i < (int64_t)n; ++i) eo[__atomic_fetch_add(&cnt[dense_of[i]], 1ull, __ATOMIC_RELAXED)] = i;
  }
  phase("group");
  std::vector<uint32_t> live_cnt(nv, 0);
#pragma omp parallel for schedule(dynamic, 1024) num_threads(T)
  for (int64_t d = 0; d < (int64_t)nv; ++d) {
    auto b = eo.begin() + rs[d], e = eo.begin() + rs[d + 1];
    std::sort(b, e, [&](uint64_t x, uint64_t y) {
      const uint32_t dx = dense_of[n + x], dy = dense_of[n + y];
      return dx != dy ? dx < dy : x > y;
    });
    uint64_t m = 0;
    for (auto it = b; it != e; ++it)
      if (it == b || dense_of[n + *it] != dense_of[n + *(it - 1)]) b[m++] = *it;
    live_cnt[d] = (uint32_t)m;
  }
  phase("row sort");
  g->off.assign(nv + 1, 0);
  for (uint64_t d = 0; d < nv; ++d) g->off[d + 1] = g->off[d] + live_cnt[d];
  g->ne = g->off[nv];
  g->nbr.resize(g->ne);
  g->w.resize(g->ne);
#pragma omp parallel for schedule(dynamic, 1024) num_threads(T)
  for (int64_t d = 0; d < (int64_t)nv; ++d) {
    for (uint32_t k = 0; k < live_cnt[d]; ++k) {
      const uint64_t i = eo[rs[d] + k];
      g->nbr[g->off[d] + k] = dense_of[n + i];
      g->w[g->off[d] + k] = w ? w[i] : 0;
    }
  }
  // ---- in CSR: the mirror of every live out-edge, grouped by destination
  std::vector<uint64_t> icnt(nv + 1, 0);
#pragma omp parallel for schedule(static) num_threads(T)
  for (int64_t j = 0; j < (int64_t)g->ne; ++j) __atomic_fetch_add(&icnt[g->nbr[j] + 1], 1ull, __ATOMIC_RELAXED);
  for (uint64_t d = 0; d < nv; ++d) icnt[d + 1] += icnt[d];
  g->ioff = icnt;
  g->inbr.resize(g->ne);
#pragma omp parallel for schedule(dynamic, 1024) num_threads(T)
  for (int64_t d = 0; d < (int64_t)nv; ++d)
    for (uint64_t j = g->off[d]; j < g->off[d + 1]; ++j)
      g->inbr[__atomic_fetch_add(&icnt[g->nbr[j]], 1ull, __ATOMIC_RELAXED)] = (uint32_t)d;
  g->sp.init(nv);
  phase("csr");
  return g;
}

// ---------------------------------------------------------------- GO N STEPS
struct GoOut {
  uint64_t rows = 0, x = 0, sum = 0, scanned = 0;
};

enum { Y_DST = 1, Y_SRC = 2, Y_W = 4 };

inline bool where_ok(int op, int64_t w, int64_t c) {
  switch (op) {
    case 0: return true;
    case 1: return w < c;
    case 2: return w <= c;
    case 3: return w > c;
    case 4: return w >= c;
    case 5: return w == c;
    default: return w != c;
  }
}

// rows_out (nullable, cap rows x ncols int64, row-major): the first `cap` rows, any order
GoOut go(Csr& g, const int64_t* starts, uint64_t ns, uint32_t steps, int op, int64_t c, int ymask, int64_t* rows_out,
         uint64_t cap) {
  GoOut out;
  const int T = g.threads;
  std::vector<uint32_t> f;
  for (uint64_t i = 0; i < ns; ++i) {
    const int64_t d = g.dense(starts[i]);
    if (d >= 0) f.push_back((uint32_t)d);
  }
  std::vector<uint64_t> bits;
  for (uint32_t s = 1; s < steps && !f.empty(); ++s) {
    bits.assign((g.nv + 63) / 64, 0);
    uint64_t sc = 0;
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : sc) num_threads(T)
    for (int64_t k = 0; k < (int64_t)f.size(); ++k) {
      const uint32_t v = f[k];
      sc += g.off[v + 1] - g.off[v];
      for (uint64_t j = g.off[v]; j < g.off[v + 1]; ++j) {
        const uint32_t u = g.nbr[j];
        const uint64_t m = 1ull << (u & 63);
        if (!(__atomic_load_n(&bits[u >> 6], __ATOMIC_RELAXED) & m)) __atomic_fetch_or(&bits[u >> 6], m, __ATOMIC_RELAXED);
      }
    }
    out.scanned += sc;
    f.clear();
    for (uint64_t wd = 0; wd < bits.size(); ++wd)
      for (uint64_t b = bits[wd]; b; b &= b - 1) f.push_back((uint32_t)(wd * 64 + __builtin_ctzll(b)));
  }
  if (f.empty()) return out;
  const int ncols = __builtin_popcount(ymask);
  std::atomic<uint64_t> wr{0};
  uint64_t rows = 0, x = 0, sum = 0, sc = 0;
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : rows, sum, sc) reduction(^ : x) num_threads(T)
  for (int64_t k = 0; k < (int64_t)f.size(); ++k) {
    const uint32_t v = f[k];
    sc += g.off[v + 1] - g.off[v];
    for (uint64_t j = g.off[v]; j < g.off[v + 1]; ++j) {
      if (!where_ok(op, g.w[j], c)) continue;
      int64_t cols[3];
      int n = 0;
      if (ymask & Y_DST) cols[n++] = g.vid[g.nbr[j]];
      if (ymask & Y_SRC) cols[n++] = g.vid[v];
      if (ymask & Y_W) cols[n++] = g.w[j];
      uint64_t h = 0;
      for (int q = 0; q < n; ++q) h = splitmix64(h ^ (uint64_t)cols[q]);
      ++rows;
      x ^= h;
      sum += h;
      if (rows_out) {
        const uint64_t r = wr.fetch_add(1, std::memory_order_relaxed);
        if (r < cap)
          for (int q = 0; q < ncols; ++q) rows_out[r * ncols + q] = cols[q];
      }
    }
  }
  out.rows = rows;
  out.x = x;
  out.sum = sum;
  out.scanned += sc;
  return out;
}

// ---------------------------------------------------------------- FIND SHORTEST PATH
// Labels: epoch << 6 | level, live when the epoch matches.
constexpr int LB = 6;

struct Level {
  std::vector<uint32_t> v;
};

// Expands `f` over (off, nbr) claiming unlabelled neighbours at `level` in `lab`; returns the
// new frontier and the edges scanned; `meet` collects claimed (or already-claimed) vertices
// carrying a live label of the other side.
uint64_t expand(const Csr& g, const std::vector<uint64_t>& off, const std::vector<uint32_t>& nbr,
                const std::vector<uint32_t>& f, std::vector<uint32_t>& lab, const std::vector<uint32_t>& other,
                uint32_t ep, uint32_t level, std::vector<uint32_t>& next, std::vector<uint32_t>& meet, int T) {
  uint64_t sc = 0;
  uint64_t work = 0;
  for (size_t k = 0; k < f.size() && work < 65536; ++k) work += off[f[k] + 1] - off[f[k]] + 1;
  if (work < 65536) T = 1;   // a small level: no thread fan-out
  std::vector<std::vector<uint32_t>> nx(T), mt(T);
  const uint32_t stamp = ep << LB | level;
#pragma omp parallel num_threads(T) reduction(+ : sc)
  {
    const int t = omp_get_thread_num();
#pragma omp for schedule(dynamic, 64)
    for (int64_t k = 0; k < (int64_t)f.size(); ++k) {
      const uint32_t v = f[k];
      sc += off[v + 1] - off[v];
      for (uint64_t j = off[v]; j < off[v + 1]; ++j) {
        const uint32_t u = nbr[j];
        uint32_t cur = __atomic_load_n(&lab[u], __ATOMIC_RELAXED);
        if ((cur >> LB) == ep) continue;
        if (__atomic_compare_exchange_n(&lab[u], &cur, stamp, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
          nx[t].push_back(u);
          if ((other[u] >> LB) == ep) mt[t].push_back(u);
        }
      }
    }
  }
  next.clear();
  meet.clear();
  for (int t = 0; t < T; ++t) {
    next.insert(next.end(), nx[t].begin(), nx[t].end());
    meet.insert(meet.end(), mt[t].begin(), mt[t].end());
  }
  return sc;
}

// returns the path length L (0: none within upto); path = [vid0, vid1, ..., vidL]
int shortest(const Csr& g, SpCtx& x, int T, int64_t sv, int64_t tv, uint32_t upto, std::vector<int64_t>& path,
             uint64_t* scanned) {
  path.clear();
  *scanned = 0;
  const int64_t s64 = g.dense(sv), t64 = g.dense(tv);
  if (s64 < 0 || t64 < 0 || upto == 0) return 0;
  const uint32_t s = (uint32_t)s64, t = (uint32_t)t64;
  if (++x.epoch >= (1u << (32 - LB))) {
    std::fill(x.labf.begin(), x.labf.end(), 0);
    std::fill(x.labb.begin(), x.labb.end(), 0);
    std::fill(x.mark.begin(), x.mark.end(), 0);
    x.epoch = 1;
  }
  const uint32_t ep = x.epoch;
  auto lev = [&](const std::vector<uint32_t>& lab, uint32_t v) -> int {
    return (lab[v] >> LB) == ep ? (int)(lab[v] & ((1u << LB) - 1)) : -1;
  };
  std::vector<std::vector<uint32_t>> F{{s}}, Bk{{t}};
  x.labf[s] = ep << LB;
  uint32_t kf = 0, kb = 0, L = 0;
  std::vector<uint32_t> meet, next;
  if (s == t) {
    // shortest cycle through s: forward BFS; position L = the first level whose frontier has an
    // edge into s.  dist_t(v) = distance from v to s over out-edges = backward BFS from s.
    for (kf = 0; kf < upto && !F[kf].empty(); ++kf) {
      bool hit = false;
      for (uint32_t v : F[kf]) {
        *scanned += 0;
        for (uint64_t j = g.off[v]; j < g.off[v + 1] && !hit; ++j) hit = g.nbr[j] == s;
      }
      if (hit) { L = kf + 1; break; }
      std::vector<uint32_t> m;
      *scanned += expand(g, g.off, g.nbr, F[kf], x.labf, x.labb, ep, kf + 1, next, m, T);
      F.push_back(next);
    }
    if (!L) return 0;
    // backward levels from t over in-edges up to L - 1 (t = s stamped at 0 on the b side)
    x.labb[t] = ep << LB;
    for (kb = 0; kb + 1 < L; ++kb) {
      std::vector<uint32_t> m;
      *scanned += expand(g, g.ioff, g.inbr, Bk[kb], x.labb, x.labf, ep, kb + 1, next, m, T);
      Bk.push_back(next);
    }
    path.push_back(g.vid[s]);
    uint32_t c = s;
    for (uint32_t i = 0; i + 1 < L; ++i) {
      int64_t best = -1;
      uint32_t bu = 0;
      for (uint64_t j = g.off[c]; j < g.off[c + 1]; ++j) {
        const uint32_t u = g.nbr[j];
        if (u == s || lev(x.labf, u) != (int)(i + 1) || lev(x.labb, u) != (int)(L - i - 1)) continue;
        if (best < 0 || g.vid[u] < best) { best = g.vid[u]; bu = u; }
      }
      if (best < 0) return 0;
      path.push_back(best);
      c = bu;
    }
    path.push_back(g.vid[s]);
    return (int)L;
  }
  x.labb[t] = ep << LB;
  // bidirectional level-synchronous BFS: expand the side whose frontier has the smaller degree
  // sum; the first level that claims a vertex labelled by the other side fixes L = kf + kb
  auto dsum = [&](const std::vector<uint32_t>& fr, const std::vector<uint64_t>& off) {
    uint64_t x = 0;
    for (uint32_t v : fr) x += off[v + 1] - off[v];
    return x;
  };
  bool fwd_last = true;
  while (kf + kb < upto) {
    if (F[kf].empty() || Bk[kb].empty()) return 0;
    const bool fwd = dsum(F[kf], g.off) <= dsum(Bk[kb], g.ioff);
    if (fwd) {
      *scanned += expand(g, g.off, g.nbr, F[kf], x.labf, x.labb, ep, kf + 1, next, meet, T);
      F.push_back(next);
      ++kf;
    } else {
      *scanned += expand(g, g.ioff, g.inbr, Bk[kb], x.labb, x.labf, ep, kb + 1, next, meet, T);
      Bk.push_back(next);
      ++kb;
    }
    fwd_last = fwd;
    if (!meet.empty()) break;
  }
  if (meet.empty()) return 0;
  L = kf + kb;
  // positions: the meet set sits at forward position kf; B[i] for i < kf = vertices of forward
  // level i with an out-edge into B[i + 1]; positions > kf are backward levels L - i
  (void)fwd_last;
  std::vector<uint32_t> cur(meet);
  std::vector<uint32_t>& mark = x.mark;    // ep << LB | position, for B-set members at positions <= kf
  for (uint32_t v : cur) mark[v] = ep << LB | kf;
  for (int i = (int)kf - 1; i >= 0; --i) {
    std::vector<uint32_t> prev;
    const uint32_t st = ep << LB | (uint32_t)i;
    for (uint32_t v : cur)
      for (uint64_t j = g.ioff[v]; j < g.ioff[v + 1]; ++j) {
        const uint32_t u = g.inbr[j];
        if (lev(x.labf, u) == i && mark[u] != st) {
          mark[u] = st;
          prev.push_back(u);
        }
      }
    cur.swap(prev);
  }
  path.push_back(g.vid[s]);
  uint32_t c = s;
  for (uint32_t i = 0; i < L; ++i) {
    int64_t best = -1;
    uint32_t bu = 0;
    for (uint64_t j = g.off[c]; j < g.off[c + 1]; ++j) {
      const uint32_t u = g.nbr[j];
      const bool ok = (i + 1 <= kf) ? mark[u] == (ep << LB | (i + 1)) : lev(x.labb, u) == (int)(L - i - 1);
      if (!ok) continue;
      if (best < 0 || g.vid[u] < best) { best = g.vid[u]; bu = u; }
    }
    if (best < 0) return 0;
    path.push_back(best);
    c = bu;
  }
  return (int)L;
}

// ---------------------------------------------------------------- several OVER types (C5)
// GO N STEPS FROM starts OVER t_0, .., t_{k-1} with the default YIELD (one `<t_i>._dst` column per
// OVER type, parser.yy:518-531): a row of a t_i edge holds its dst in column i and the other edge
// types' default 0 (GoExecutor.cpp:863-869).  Each type is its own Csr (own dense ids), so the
// frontier travels as sorted unique vids; the per-step SET is the union over the types.
GoOut go_multi(Csr* const* gs, int nt, const int64_t* starts, uint64_t ns, uint32_t steps) {
  GoOut out;
  const int T = gs[0]->threads;
  std::vector<int64_t> f(starts, starts + ns);   // duplicates kept at step 1
  for (uint32_t s = 1; s < steps && !f.empty(); ++s) {
    std::vector<std::vector<int64_t>> nx(T);
    uint64_t sc = 0;
    for (int k = 0; k < nt; ++k) {
      const Csr& g = *gs[k];
#pragma omp parallel num_threads(T) reduction(+ : sc)
      {
        std::vector<int64_t>& mine = nx[omp_get_thread_num()];
#pragma omp for schedule(dynamic, 64)
        for (int64_t i = 0; i < (int64_t)f.size(); ++i) {
          const int64_t d = g.dense(f[i]);
          if (d < 0) continue;
          sc += g.off[d + 1] - g.off[d];
          for (uint64_t j = g.off[d]; j < g.off[d + 1]; ++j) mine.push_back(g.vid[g.nbr[j]]);
        }
      }
    }
    out.scanned += sc;
    f.clear();
    for (auto& v : nx) f.insert(f.end(), v.begin(), v.end());
    std::sort(f.begin(), f.end());
    f.erase(std::unique(f.begin(), f.end()), f.end());
  }
  uint64_t rows = 0, x = 0, sum = 0, sc = 0;
  for (int k = 0; k < nt; ++k) {
    const Csr& g = *gs[k];
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : rows, sum, sc) reduction(^ : x) num_threads(T)
    for (int64_t i = 0; i < (int64_t)f.size(); ++i) {
      const int64_t d = g.dense(f[i]);
      if (d < 0) continue;
      sc += g.off[d + 1] - g.off[d];
      for (uint64_t j = g.off[d]; j < g.off[d + 1]; ++j) {
        uint64_t h = 0;
        for (int q = 0; q < nt; ++q) h = splitmix64(h ^ (uint64_t)(q == k ? g.vid[g.nbr[j]] : 0));
        ++rows;
        x ^= h;
        sum += h;
      }
    }
  }
  out.rows = rows;
  out.x = x;
  out.sum = sum;
  out.scanned += sc;
  return out;
}

// ---------------------------------------------------------------- FIND ALL PATH (walks)
// FIND ALL PATH s -> t UPTO n over one type returns every walk of 1..n edges (cycles included,
// FindPathExecutor.cpp:292-411).  Counted per length by dynamic programming over walk counts,
// meeting in the middle: f_a[v] = walks s -> v of a edges (out-edges), b_c[v] = walks v -> t of c
// edges (in-edges), count[L] = (A^L)[s, t] = sum_v f_a[v] * b_(L-a)[v] with a = ceil(L / 2) — two
// half-length expansions instead of L full ones (a 4-step count on RMAT-24 scanned most of the
// graph per pair); enumerated by a depth-first search pruned with the backward BFS distance to t.
namespace {
using WalkLevel = std::vector<std::pair<uint32_t, uint64_t>>;   // (dense id, walks), sorted by id

WalkLevel walk_expand(const std::vector<uint64_t>& off, const std::vector<uint32_t>& nbr, const WalkLevel& cur,
                      std::vector<uint64_t>& acc, std::vector<uint32_t>& touched) {
  touched.clear();
  for (const auto& e : cur)
    for (uint64_t j = off[e.first]; j < off[e.first + 1]; ++j) {
      const uint32_t u = nbr[j];
      if (!acc[u]) touched.push_back(u);
      acc[u] += e.second;
    }
  std::sort(touched.begin(), touched.end());
  WalkLevel out;
  out.reserve(touched.size());
  for (uint32_t u : touched) {
    out.emplace_back(u, acc[u]);
    acc[u] = 0;
  }
  return out;
}

uint64_t walk_dot(const WalkLevel& x, const WalkLevel& y) {
  uint64_t sum = 0;
  for (size_t i = 0, j = 0; i < x.size() && j < y.size();) {
    if (x[i].first < y[j].first) {
      ++i;
    } else if (y[j].first < x[i].first) {
      ++j;
    } else {
      sum += x[i++].second * y[j++].second;
    }
  }
  return sum;
}
}  // namespace

void walk_counts(const Csr& g, int64_t sv, int64_t tv, uint32_t upto, uint64_t* cnt) {
  for (uint32_t L = 0; L <= upto; ++L) cnt[L] = 0;
  const int64_t s = g.dense(sv), t = g.dense(tv);
  if (s < 0 || t < 0) return;
  std::vector<uint64_t> acc(g.nv, 0);
  std::vector<uint32_t> touched;
  const uint32_t A = (upto + 1) / 2, Bc = upto / 2;
  std::vector<WalkLevel> f(A + 1), b(Bc + 1);
  f[0] = {{(uint32_t)s, 1}};
  b[0] = {{(uint32_t)t, 1}};
  for (uint32_t a = 1; a <= A; ++a) f[a] = walk_expand(g.off, g.nbr, f[a - 1], acc, touched);
  for (uint32_t c = 1; c <= Bc; ++c) b[c] = walk_expand(g.ioff, g.inbr, b[c - 1], acc, touched);
  for (uint32_t L = 1; L <= upto; ++L) {
    const uint32_t a = (L + 1) / 2;
    cnt[L] = walk_dot(f[a], b[L - a]);
  }
}

uint64_t all_walks(const Csr& g, int64_t sv, int64_t tv, uint32_t upto, int64_t* out, uint64_t cap) {
  const int64_t s = g.dense(sv), t = g.dense(tv);
  if (s < 0 || t < 0) return 0;
  // distance to t over out-edges (backward BFS over in-edges), capped at upto
  std::vector<uint32_t> dist(g.nv, 0xFFFFFFFFu);
  std::vector<uint32_t> fr{(uint32_t)t}, nx;
  dist[t] = 0;
  for (uint32_t d = 1; d <= upto && !fr.empty(); ++d) {
    nx.clear();
    for (uint32_t v : fr)
      for (uint64_t j = g.ioff[v]; j < g.ioff[v + 1]; ++j)
        if (dist[g.inbr[j]] == 0xFFFFFFFFu) { dist[g.inbr[j]] = d; nx.push_back(g.inbr[j]); }
    fr.swap(nx);
  }
  uint64_t n = 0;
  std::vector<uint32_t> walk{(uint32_t)s};
  const uint64_t width = 1 + (uint64_t)upto;   // vids of one walk, padded with -1
  std::function<void()> dfs = [&]() {
    const uint32_t v = walk.back();
    const uint32_t len = (uint32_t)walk.size() - 1;
    if (len >= upto) return;
    for (uint64_t j = g.off[v]; j < g.off[v + 1]; ++j) {
      const uint32_t u = g.nbr[j];
      if (dist[u] == 0xFFFFFFFFu || len + 1 + dist[u] > upto) continue;
      walk.push_back(u);
      if (u == (uint32_t)t) {
        if (n < cap)
          for (uint64_t k = 0; k < width; ++k) out[n * width + k] = k < walk.size() ? g.vid[walk[k]] : -1;
        ++n;
      }
      dfs();
      walk.pop_back();
    }
  };
  dfs();
  return n;
}

// Per-rank load of GO `steps` STEPS from each start (one query per start), for the partition
// part = (uint64)vid % parts + 1 (NebulaKeyUtils / StorageClient::partId), rank = part % G
// (CreateSpaceProcessor.cpp:84-95 with GPUs as hosts).  A step's edges are scanned at the frontier
// vertex's part, so out[((q * steps) + s) * G + r] = edges that rank r scans in step s of query q.
void rank_edges(const Csr& g, const int64_t* starts, uint64_t ns, uint32_t steps, uint32_t parts, uint32_t G,
                uint64_t* out) {
  std::vector<uint8_t> owner(g.nv);
#pragma omp parallel for schedule(static) num_threads(g.threads)
  for (int64_t d = 0; d < (int64_t)g.nv; ++d) owner[d] = (uint8_t)(((uint64_t)g.vid[d] % parts + 1) % G);
  std::vector<uint64_t> bits((g.nv + 63) / 64);
  for (uint64_t q = 0; q < ns; ++q) {
    uint64_t* o = out + q * steps * G;
    std::fill(o, o + (uint64_t)steps * G, 0);
    std::vector<uint32_t> f;
    const int64_t d0 = g.dense(starts[q]);
    if (d0 >= 0) f.push_back((uint32_t)d0);
    for (uint32_t s = 0; s < steps && !f.empty(); ++s) {
      std::vector<uint64_t> per(G, 0);
      for (uint32_t v : f) per[owner[v]] += g.off[v + 1] - g.off[v];
      for (uint32_t r = 0; r < G; ++r) o[s * G + r] = per[r];
      if (s + 1 == steps) break;
      std::fill(bits.begin(), bits.end(), 0);
#pragma omp parallel for schedule(dynamic, 64) num_threads(g.threads)
      for (int64_t k = 0; k < (int64_t)f.size(); ++k)
        for (uint64_t j = g.off[f[k]]; j < g.off[f[k] + 1]; ++j) {
          const uint32_t u = g.nbr[j];
          __atomic_fetch_or(&bits[u >> 6], 1ull << (u & 63), __ATOMIC_RELAXED);
        }
      f.clear();
      for (uint64_t wd = 0; wd < bits.size(); ++wd)
        for (uint64_t b = bits[wd]; b; b &= b - 1) f.push_back((uint32_t)(wd * 64 + __builtin_ctzll(b)));
    }
  }
}

}  // namespace

extern "C" {

void orc_csr_rank_edges(void* h, const int64_t* starts, uint64_t ns, uint32_t steps, uint32_t parts, uint32_t G,
                        uint64_t* out) {
  rank_edges(*static_cast<Csr*>(h), starts, ns, steps, parts, G, out);
}

// GO steps STEPS FROM starts OVER the nt types (one Csr each), default YIELD: out4 as orc_csr_go
double orc_csr_go_multi(void* const* hs, int32_t nt, const int64_t* starts, uint64_t ns, uint32_t steps,
                        uint64_t* out4) {
  auto t0 = std::chrono::steady_clock::now();
  GoOut r = go_multi(reinterpret_cast<Csr* const*>(hs), nt, starts, ns, steps);
  out4[0] = r.rows;
  out4[1] = r.x;
  out4[2] = r.sum;
  out4[3] = r.scanned;
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

// walks s -> t of exactly L edges, for L = 0..upto, into cnt[0..upto]
void orc_csr_walk_counts(void* h, int64_t s, int64_t t, uint32_t upto, uint64_t* cnt) {
  walk_counts(*static_cast<Csr*>(h), s, t, upto, cnt);
}

// every walk s -> t of 1..upto edges as upto + 1 vids (-1 padded), the first `cap` of them;
// returns how many there are
uint64_t orc_csr_all_walks(void* h, int64_t s, int64_t t, uint32_t upto, int64_t* out, uint64_t cap) {
  return all_walks(*static_cast<Csr*>(h), s, t, upto, out, cap);
}

void* orc_csr_build(const int64_t* src, const int64_t* dst, const int64_t* w, uint64_t n, int32_t threads) {
  return build(src, dst, w, n, threads > 0 ? threads : omp_get_max_threads());
}
void orc_csr_free(void* h) { delete static_cast<Csr*>(h); }
uint64_t orc_csr_nv(void* h) { return static_cast<Csr*>(h)->nv; }
uint64_t orc_csr_ne(void* h) { return static_cast<Csr*>(h)->ne; }
void orc_csr_threads(void* h, int32_t threads) { static_cast<Csr*>(h)->threads = threads > 0 ? threads : 1; }

// GO `steps` STEPS FROM starts OVER e [WHERE e.w <op> c] YIELD (e._dst | e._src | e.w per ymask
// bit, in that order).  out4 = {rows, xor of row hashes, sum of row hashes, edges scanned}.
// op: 0 none, 1 <, 2 <=, 3 >, 4 >=, 5 ==, 6 !=.  Returns seconds (steady clock).
double orc_csr_go(void* h, const int64_t* starts, uint64_t ns, uint32_t steps, int32_t op, int64_t c, int32_t ymask,
                  uint64_t* out4, int64_t* rows_out, uint64_t cap) {
  auto t0 = std::chrono::steady_clock::now();
  GoOut r = go(*static_cast<Csr*>(h), starts, ns, steps, op, c, ymask, rows_out, cap);
  auto t1 = std::chrono::steady_clock::now();
  out4[0] = r.rows;
  out4[1] = r.x;
  out4[2] = r.sum;
  out4[3] = r.scanned;
  return std::chrono::duration<double>(t1 - t0).count();
}

// FIND SHORTEST PATH s -> t UPTO upto over e: writes L + 1 vids into path (cap >= upto + 1);
// returns L (0: no path); *scanned = adjacency entries scanned (both directions).
int32_t orc_csr_shortest(void* h, int64_t s, int64_t t, uint32_t upto, int64_t* path, uint64_t* scanned) {
  std::vector<int64_t> p;
  Csr& g = *static_cast<Csr*>(h);
  const int L = shortest(g, g.sp, g.threads, s, t, upto, p, scanned);
  for (size_t i = 0; L && i < p.size(); ++i) path[i] = p[i];
  return L;
}

// n independent searches, one per thread (each serial, with its own labels): path i's L + 1
// vids at paths[i * (upto + 1)], len[i] = L (0: no path), scanned[i] its edges scanned
void orc_csr_shortest_many(void* h, const int64_t* s, const int64_t* t, uint64_t n, uint32_t upto, int64_t* paths,
                           int32_t* len, uint64_t* scanned) {
  Csr& g = *static_cast<Csr*>(h);
  const int T = g.threads;
  std::vector<SpCtx> ctx(T);
#pragma omp parallel num_threads(T)
  {
    SpCtx& c = ctx[omp_get_thread_num()];
    c.init(g.nv);
    std::vector<int64_t> p;
#pragma omp for schedule(dynamic, 4)
    for (int64_t i = 0; i < (int64_t)n; ++i) {
      uint64_t sc = 0;
      const int L = shortest(g, c, 1, s[i], t[i], upto, p, &sc);
      len[i] = L;
      scanned[i] = sc;
      for (size_t k = 0; L && k < p.size(); ++k) paths[i * (upto + 1) + k] = p[k];
    }
  }
}

}  // extern "C"
