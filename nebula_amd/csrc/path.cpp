// FIND SHORTEST PATH driver (FindPathExecutor result semantics) over the device snapshot.
//
// Reference: src/graph/FindPathExecutor.cpp — rounds of from-side expansion over the OVER types
// and to-side expansion over their in-edges (-type) (:145-216), odd/even meets (:218-290), one
// path per target across all sources, minimum hop count (:292-382), UPTO N steps (parser.yy
// :858-861, default 5), from/to de-duplicated (VerticesClause).  The reference breaks ties
// between equal-length paths by hash-map iteration order; this engine (and the oracle,
// oracle/graph.cpp runShortestBfs) returns the lexicographically smallest entry list
// [v0, t0, r0, v1, ...] instead — a deterministic member of the reference's answer set.
//
// Two device strategies, identical results:
//   * one source, one target (s != t): bidirectional BFS.  Each level expands the side whose
//     frontier has the smaller degree sum; labels are epoch-stamped (no clearing).  The first
//     level that claims a vertex labelled by the other side fixes L = kf + kb, and every vertex
//     met in that level sits at forward position kf (no shorter meet existed).  B-sets over
//     the forward levels are then recovered backwards from the meet set through in-edges,
//     restricted to forward level i; positions past kf are the backward BFS levels.
//   * otherwise: one-sided BFS from all sources (walk length >= 1, as the reference's rounds
//     never revisit a source at depth 0), stopping once every target is labelled; per target
//     the B-sets are recovered from the target through in-edges restricted to forward levels.
// The path is then built greedily (k_path_greedy): v0 = min B[0], each hop the minimum
// (type, rank, dst) edge into the next B-set.  Lexicographic minimality follows because every
// B-set member extends to a shortest path.
//
// Partitioned engine: every rank runs the same sequence collectively.  A level
// marks next-frontier candidates by global id, the bitmap all-to-all hands them to their owners,
// and the owner claims them against its own labels (ws_path_level_part) — the meet test and the
// target count are local at the owner; sizes and "all targets found" are summed over ranks at
// each synchronisation.  The greedy walks the in-edges of each rank's B-set members (the
// out-edge v -> u is stored at v's owner, its mirror at u's owner where u's labels are) and
// takes the minimum of the ranks' candidates, one small all-gather per hop.
//
// In-edge records mirror out-edges (InsertEdgeExecutor.cpp:180-196 writes both), so the to-side
// sees exactly the reverse of the from-side.  With a non-default max_edge_returned_per_vertex the
// two sides see different capped graphs and the search follows the reference's rounds instead
// (pathcap.hip).
#include <algorithm>
#include <chrono>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_set>

#include "engine.h"

using namespace nbg;

namespace {

constexpr int S_F0 = 0, S_B0 = 2, S_MEET = 4, S_START = 5, S_SET0 = 6;

inline uint32_t stamp(uint32_t epoch, uint32_t level) { return (epoch << LVL_BITS) | level; }

struct PathCtx {
  Engine& E;
  Workspace* ws;
  PathTypes fwd, bwd;
  uint64_t bwd_edges = 0;   // in-edges over the OVER types (B-set pass bound)
  uint64_t edges = 0;       // BFS edges scanned (both sides)
  bool part = false;        // partitioned engine: collective levels and greedy
};

// A device error in the middle of a partitioned search leaves the peers in (or on their way to) the
// next collective: abort the communicator so that they fail too instead of waiting.
int32_t dev_fail(Engine& E, hipError_t e, const char* what) {
  std::string msg = std::string(what) + ": " + hipGetErrorString(e);
  if (E.partitioned() && E.comm) {
    if (!E.comm->last.empty()) msg += " (" + E.comm->last + ")";
    E.comm->abort();
  }
  return E.fail(NBG_E_DEVICE, msg);
}

hipError_t level(PathCtx& c, const PathTypes& pt, int src, uint64_t n_bound, uint64_t e_bound, int dst,
                 const PathLevel& lv) {
  return c.part ? ws_path_level_part(c.ws, pt, src, n_bound, e_bound, dst, lv)
                : ws_path_level(c.ws, pt, src, n_bound, e_bound, dst, lv);
}

// One level plus the degree sum of its output list over the same CSRs (the next level's bound
// and, bidirectionally, its direction).  Single engine: summed by the level's k_expand<BFS> into
// PState.ld[rec]; partitioned: a collective k_degsum into PState.dsum[side].  *rec = the level's
// PState record.
// out_bound: a bound on the output list's length for the partitioned degree sum (0: e_bound).
hipError_t level_ds(PathCtx& c, const PathTypes& pt, int src, uint64_t n_bound, uint64_t e_bound, int dst,
                    PathLevel lv, int side, int* rec) {
  if (!c.part) lv.deg = &pt;
  lv.global_bound = true;   // e_bound: the frontier's degree sum over every rank
  hipError_t he = level(c, pt, src, n_bound, e_bound, dst, lv);
  *rec = ws_path_last_rec(c.ws);
  if (he == hipSuccess && c.part) he = ws_path_degsum(c.ws, dst, e_bound ? e_bound : 1, pt, side);
  return he;
}

uint64_t level_dsum(const PathCtx& c, const PState& ps, int rec, int side) {
  return c.part ? ps.dsum[side] : ps.ld[rec >= 0 && rec < PATH_REC ? rec : PATH_REC - 1];
}

// Degree of local vertex v over a direction's CSRs, from the host copy of the offsets (single
// engine), capped like k_degsum.
uint64_t host_degree(const PathCtx& c, const PathTypes& pt, uint32_t v) {
  if (v == NO_ROW || (!c.E.snap.h_visible.empty() && !c.E.snap.h_visible[v])) return 0;
  uint64_t sum = 0;
  for (int k = 0; k < pt.n; ++k) {
    auto it = c.E.snap.types.find(pt.type[k]);
    if (it == c.E.snap.types.end() || it->second.h_row_ptr.size() <= (size_t)v + 1) continue;
    const std::vector<uint32_t>& rp = it->second.h_row_ptr;
    sum += std::min<uint64_t>(rp[v + 1] - rp[v], pt.a[k].cap);
  }
  return sum;
}

// sizes of the whole graph (summed over ranks when partitioned)
hipError_t sync(PathCtx& c, PState* ps) {
  return c.part ? ws_path_sync_part(c.ws, ps) : ws_path_sync(c.ws, ps, nullptr, 0);
}

// one id (or none: NO_ROW, a vertex owned by another rank) into a slot
hipError_t upload1(Workspace* ws, int slot, uint32_t id) { return ws_path_upload(ws, slot, &id, id != NO_ROW); }

// Recover B[i] for i = top-1 .. lo from B[top] (slot `cur`, <= n_top entries) through in-edges:
// B[i] = { u : u -> B[i+1], forward label of u == i } (i >= 1) or u in S (i == 0).
// first_bound (partitioned): the top list's in-degree sum over every rank (0: unknown), so the
// first step may exchange slot arrays
hipError_t bsets(PathCtx& c, int cur, uint64_t n_top, int top, int lo, uint32_t ef, uint32_t em, uint32_t es,
                 const std::vector<uint64_t>& level_n, int* out_slot, uint64_t first_bound = 0) {
  hipError_t he = hipSuccess;
  uint64_t nb = n_top;
  for (int i = top - 1; i >= lo && he == hipSuccess; --i) {
    PathLevel lv;
    const bool first = i == top - 1 && first_bound;
    lv.global_bound = first;
    lv.lab = LAB_M;
    lv.stamp = stamp(em, (uint32_t)i);
    if (i >= 1) {
      lv.rlab = LAB_F;
      lv.rstamp = stamp(ef, (uint32_t)i);
    } else {
      // B[0] (sources) is only the greedy's start list; claim it in a fresh LAB_B epoch, as a
      // source may also be the target itself, already in B[L] under this LAB_M epoch
      lv.lab = LAB_B;
      lv.stamp = stamp(ws_path_epoch(c.ws, LAB_B), 0);
      lv.rlab = LAB_S;
      lv.rstamp = stamp(es, 0);
    }
    const int dst = cur == S_SET0 ? S_SET0 + 1 : S_SET0;
    he = level(c, c.bwd, cur, nb, first ? first_bound : c.bwd_edges, dst, lv);
    cur = dst;
    nb = (size_t)i < level_n.size() ? level_n[i] : c.E.snap.nv;
  }
  *out_slot = cur;
  return he;
}

// Greedy reconstruction of one path of length L and its readback.
int32_t greedy_path(PathCtx& c, const PathGreedy& g, std::vector<int64_t>* path) {
  const int L = g.L;
  std::vector<int64_t> p(1 + 3 * (size_t)L);
  if (c.part) {
    hipError_t he = ws_path_greedy_part(c.ws, c.bwd, g, c.E.snap.d_vids, c.E.snap.d_visible, p.data());
    if (he == hipErrorNotFound)
      return c.E.fail(NBG_E_UNKNOWN, "shortest-path reconstruction failed (in/out edges disagree)");
    if (he != hipSuccess) return dev_fail(c.E, he, "path reconstruction");
    *path = std::move(p);
    return NBG_OK;
  }
  hipError_t he = ws_path_greedy(c.ws, c.fwd, g);
  if (he != hipSuccess) return dev_fail(c.E, he, "path reconstruction");
  PState ps;
  he = ws_path_sync(c.ws, &ps, p.data(), (int)p.size());
  if (he != hipSuccess) return dev_fail(c.E, he, "path readback");
  if (ps.err) return c.E.fail(NBG_E_UNKNOWN, "shortest-path reconstruction failed (in/out edges disagree)");
  *path = std::move(p);
  return NBG_OK;
}

// s, t: local ids (NO_ROW on a rank that does not own them); partitioned: s_gid / s_vid = the
// source's global id and vid on every rank (the greedy's v0 without an exchange), deg = deg(s),
// deg(t) over ranks when known (null: a set-up exchange)
int32_t bidirectional(PathCtx& c, uint32_t s, uint32_t t, uint32_t upto, nbg_paths* out, int64_t s_gid = -1,
                      int64_t s_vid = 0, const unsigned long long* deg = nullptr) {
  Workspace* ws = c.ws;
  const uint32_t ef = ws_path_epoch(ws, LAB_F), eb = ws_path_epoch(ws, LAB_B), em = ws_path_epoch(ws, LAB_M);
  hipError_t he = hipSuccess;
  auto T = [&](hipError_t e) { if (he == hipSuccess) he = e; };
  PState ps;
  uint64_t dsf = 0, dsb = 0;
  // NBG_PATH_TRACE=1: one stderr line per pair with the host-side phase times (microseconds)
  static const bool trace = getenv("NBG_PATH_TRACE") != nullptr;
  std::string tr;
  auto t_last = std::chrono::steady_clock::now();
  auto mark = [&](const char* what) {
    if (!trace) return;
    const auto now = std::chrono::steady_clock::now();
    tr += std::string(" ") + what + "=" +
          std::to_string(std::chrono::duration_cast<std::chrono::microseconds>(now - t_last).count());
    t_last = now;
  };
  struct Flush {
    const std::string& s;
    ~Flush() {
      if (trace && !s.empty()) fprintf(stderr, "nbg path trace:%s\n", s.c_str());
    }
  } flush{tr};
  if (!c.part) {
    // the first level's bounds and direction come from the host copy of the CSR offsets, so the
    // set-up needs no round trip; an endpoint without edges has no path at all
    dsf = host_degree(c, c.fwd, s);
    dsb = host_degree(c, c.bwd, t);
    if (!dsf || !dsb) return NBG_OK;
    // the PState clear was left to this launch (ws_path_begin zero_state=false)
    T(ws_path_setup_pair(ws, c.fwd, c.bwd, s, t, S_F0, S_B0, S_START, LAB_F, stamp(ef, 0), LAB_B, stamp(eb, 0)));
    if (he != hipSuccess) return dev_fail(c.E, he, "path setup");
  } else {
    T(upload1(ws, S_F0, s));
    T(upload1(ws, S_B0, t));
    T(upload1(ws, S_START, s));
    T(ws_path_stamp(ws, S_F0, 1, LAB_F, stamp(ef, 0)));
    T(ws_path_stamp(ws, S_B0, 1, LAB_B, stamp(eb, 0)));
    if (deg) {
      // deg(s), deg(t) came with the request's presence exchange: no set-up round trip
      if (he != hipSuccess) return dev_fail(c.E, he, "path setup");
      dsf = deg[0];
      dsb = deg[1];
      if (!dsf || !dsb) return NBG_OK;
    } else {
      T(ws_path_degsum(ws, S_F0, 1, c.fwd, 0));
      T(ws_path_degsum(ws, S_B0, 1, c.bwd, 1));
      T(sync(c, &ps));
      if (he != hipSuccess) return dev_fail(c.E, he, "path setup");
      dsf = ps.dsum[0];
      dsb = ps.dsum[1];
    }
  }
  mark("setup");
  int fcur = S_F0, bcur = S_B0, kf = 0, kb = 0;
  uint64_t nf = 1, nbk = 1;
  std::vector<uint64_t> fn(1, 1);   // forward level sizes
  std::vector<uint64_t> bn(1, 1);   // backward level sizes
  bool met = false;
  while ((uint32_t)(kf + kb) < upto) {
    const bool forward = dsf <= dsb;
    PathLevel lv;
    lv.mlab = forward ? LAB_B : LAB_F;
    lv.mepoch = forward ? eb : ef;
    lv.meet_slot = S_MEET;
    int rec = -1;
    if (forward) {
      lv.lab = LAB_F;
      lv.stamp = stamp(ef, (uint32_t)kf + 1);
      lv.mstamp = stamp(em, (uint32_t)kf + 1);
      T(level_ds(c, c.fwd, fcur, nf, dsf, fcur ^ 1, lv, 0, &rec));
      fcur ^= 1;
      ++kf;
    } else {
      lv.lab = LAB_B;
      lv.stamp = stamp(eb, (uint32_t)kb + 1);
      lv.mstamp = stamp(em, (uint32_t)kf);
      T(level_ds(c, c.bwd, bcur, nbk, dsb, bcur ^ 1, lv, 1, &rec));
      bcur ^= 1;
      ++kb;
    }
    if (c.part) {   // the first B-set steps' bounds (backward, and forward past kf)
      T(ws_path_meet_degsum(ws, S_MEET, c.bwd));
    }
    mark(forward ? "fwd_enq" : "bwd_enq");
    T(sync(c, &ps));
    mark("sync");
    if (he != hipSuccess) return dev_fail(c.E, he, "path level");
    if (rec >= 0 && rec < PATH_REC) c.edges += ps.le[rec];
    nf = ps.n[fcur];
    nbk = ps.n[bcur];
    if (forward)
      dsf = level_dsum(c, ps, rec, 0);
    else
      dsb = level_dsum(c, ps, rec, 1);
    if (forward) fn.push_back(nf);
    else bn.push_back(nbk);
    if (ps.n[S_MEET]) { met = true; break; }
    if (nf == 0 || nbk == 0) break;
  }
  if (!met) return NBG_OK;
  const int L = kf + kb;
  int start_slot = S_START;
  if (kf >= 1) {
    // B[kf] = the meet list; B[kf-1] .. B[1] through in-edges; B[0] = {s}
    int slot = S_MEET;
    T(bsets(c, S_MEET, ps.n[S_MEET], kf, 1, ef, em, 0, fn, &slot, c.part ? ps.mdsum : 0));
  }
  if (he != hipSuccess) return dev_fail(c.E, he, "path B-sets");
  mark("bsets_enq");
  PathGreedy g{L, kf, em, eb, start_slot};
  g.v0_gid = s_gid;   // B[0] = {s}
  g.v0_vid = s_vid;
  std::vector<int64_t> p;
  int32_t rc = greedy_path(c, g, &p);
  mark("greedy");
  if (rc) return rc;
  out->paths.push_back(std::move(p));
  return NBG_OK;
}

// One (s, t) pair on a single engine: the persistent device search (sp.hip) — one launch, one
// result copy, one host wait.
SpTypes sp_types(const Engine& E, const PathTypes& pt) {
  SpTypes T{};
  T.n = pt.n;
  for (int k = 0; k < pt.n; ++k) {
    T.type[k] = pt.type[k];
    T.ne[k] = E.snap.types.at(pt.type[k]).num_edges;
    T.row_ptr[k] = pt.a[k].row_ptr;
    T.col[k] = pt.a[k].col;
    T.dst_vid[k] = pt.a[k].dst_vid;
    T.rank[k] = pt.a[k].rank;
  }
  return T;
}

int32_t device_pair(PathCtx& c, int mode, uint32_t s, uint32_t t, uint32_t upto, nbg_paths* out) {
  Engine& E = c.E;
  if (!E.sp) {
    std::string err;
    E.sp = E.new_sp(E.stream, &err);
    if (!E.sp) return E.fail(NBG_E_OUT_OF_MEMORY, err);
  }
  const uint64_t ds = host_degree(c, c.fwd, s), dt = host_degree(c, c.bwd, t);
  if (!ds || !dt) return NBG_OK;   // an endpoint without edges
  hipError_t he = sp_launch(E.sp, sp_types(c.E, c.fwd), sp_types(c.E, c.bwd), E.snap.d_visible, E.snap.d_vids, s, t, upto,
                            std::min(ds, dt));
  SpResult r;
  if (he == hipSuccess) he = sp_wait(E.sp, &r);
  if (he != hipSuccess) return dev_fail(E, he, "shortest path");
  if (r.err == 1) return E.fail(NBG_E_UNKNOWN, "shortest-path reconstruction failed (in/out edges disagree)");
  if (r.err) return E.fail(NBG_E_DEVICE, "shortest path: " + sp_err_text(r.err));
  c.edges += r.edges;
  out->batches += (uint32_t)r.batches;
  if (r.L) out->paths.emplace_back(r.path, r.path + 1 + 3 * r.L);
  return NBG_OK;
}

// One-pair SHORTEST on a single engine.  NBG_SP_MODE (read per query: tests switch it):
//   chain (default) - the device-driven level loop (spchain.hip): one host round trip per pair;
//                     one OVER type per direction, other requests take the host loop
//   host            - the host-driven level loop (bidirectional above), one round trip per level
constexpr int PM_HOST = -1;
int sp_mode(const PathCtx& c) {
  const char* m = getenv("NBG_SP_MODE");
  if (m && !strcmp(m, "host")) return PM_HOST;
  return c.fwd.n == 1 && c.bwd.n == 1 ? (int)SP_CHAIN : PM_HOST;
}

// S: this rank's sources (local ids); Tg: every target, by global position, as a local id
// (NO_ROW where another rank owns it); nS: the number of sources over all ranks.
int32_t one_sided(PathCtx& c, const std::vector<uint32_t>& S, const std::vector<uint32_t>& Tg, uint64_t nS,
                  uint32_t upto, nbg_paths* out) {
  Workspace* ws = c.ws;
  const uint32_t ef = ws_path_epoch(ws, LAB_F), es = ws_path_epoch(ws, LAB_S), et = ws_path_epoch(ws, LAB_B);
  hipError_t he = hipSuccess;
  auto T = [&](hipError_t e) { if (he == hipSuccess) he = e; };
  std::vector<uint32_t> Tl;
  for (uint32_t d : Tg)
    if (d != NO_ROW) Tl.push_back(d);
  T(ws_path_upload(ws, S_START, S.data(), S.size()));
  T(ws_path_stamp(ws, S_START, S.size(), LAB_S, stamp(es, 0)));
  T(ws_path_upload(ws, S_MEET, Tl.data(), Tl.size()));
  T(ws_path_stamp(ws, S_MEET, Tl.size(), LAB_B, stamp(et, 0)));
  T(ws_path_upload(ws, S_F0, S.data(), S.size()));
  T(ws_path_degsum(ws, S_F0, S.size(), c.fwd, 0));
  PState ps;
  T(sync(c, &ps));
  if (he != hipSuccess) return dev_fail(c.E, he, "path setup");
  std::vector<uint64_t> level_n(1, nS);
  int cur = S_F0;
  uint64_t n = nS, ds = ps.dsum[0];
  for (uint32_t l = 1; l <= upto; ++l) {
    PathLevel lv;
    lv.lab = LAB_F;
    lv.stamp = stamp(ef, l);
    lv.tlab = LAB_B;
    lv.tstamp = stamp(et, 0);
    int rec = -1;
    T(level_ds(c, c.fwd, cur, n, ds, cur ^ 1, lv, 0, &rec));
    cur ^= 1;
    T(sync(c, &ps));
    if (he != hipSuccess) return dev_fail(c.E, he, "path level");
    if (rec >= 0 && rec < PATH_REC) c.edges += ps.le[rec];
    n = ps.n[cur];
    ds = level_dsum(c, ps, rec, 0);
    level_n.push_back(n);
    if (n == 0 || ps.found >= Tg.size()) break;
  }
  // per target: its forward level is its distance (read at the owner, summed over ranks)
  std::vector<unsigned long long> labels(Tg.size(), 0);
  for (size_t i = 0; i < Tg.size(); ++i) {
    if (Tg[i] == NO_ROW) continue;
    uint32_t x = 0;
    he = ws_path_read_label(ws, LAB_F, Tg[i], &x);
    if (he != hipSuccess) return dev_fail(c.E, he, "label readback");
    labels[i] = x;
  }
  if (c.part) {
    he = ws_allreduce_host(ws, labels);
    if (he != hipSuccess) return dev_fail(c.E, he, "label exchange");
  }
  for (size_t i = 0; i < Tg.size(); ++i) {
    if ((uint32_t)(labels[i] >> LVL_BITS) != ef) continue;
    const int L = (int)(labels[i] & MAX_PATH_LEN);
    const uint32_t em = ws_path_epoch(ws, LAB_M);
    T(upload1(ws, S_SET0, Tg[i]));
    T(ws_path_stamp(ws, S_SET0, 1, LAB_M, stamp(em, (uint32_t)L)));
    int slot = S_SET0;
    T(bsets(c, S_SET0, 1, L, 0, ef, em, es, level_n, &slot));
    if (he != hipSuccess) return dev_fail(c.E, he, "path B-sets");
    PathGreedy g{L, L, em, 0, slot};
    std::vector<int64_t> p;
    int32_t rc = greedy_path(c, g, &p);
    if (rc) return rc;
    out->paths.push_back(std::move(p));
  }
  return NBG_OK;
}

// NBG_MAX_WALKS: partial walks FIND ALL PATH may store before it reports "too many paths"
uint64_t max_walks() {
  static const uint64_t n = getenv("NBG_MAX_WALKS") ? strtoull(getenv("NBG_MAX_WALKS"), nullptr, 10) : (1ull << 28);
  return n;
}

// FIND ALL PATH: backward BFS distances from the targets over in-edges (LAB_B, levels
// 0..upto-1), then the pruned forward walk enumeration (ws_all_paths; partitioned:
// ws_all_paths_part, walks extended at their last vertex's owner, levels all-gathered).
// Partitioned: Sgid / Svid are every source (global id, vid), the same on every rank.
int32_t all_paths(PathCtx& c, const std::vector<uint32_t>& S, const std::vector<uint32_t>& T, uint32_t upto,
                  const std::vector<uint32_t>& Sgid, const std::vector<int64_t>& Svid, nbg_paths* out) {
  Workspace* ws = c.ws;
  const uint32_t eb = ws_path_epoch(ws, LAB_B);
  hipError_t he = hipSuccess;
  auto Tr = [&](hipError_t e) { if (he == hipSuccess) he = e; };
  Tr(ws_path_upload(ws, S_B0, T.data(), T.size()));
  Tr(ws_path_stamp(ws, S_B0, T.size(), LAB_B, stamp(eb, 0)));
  Tr(ws_path_degsum(ws, S_B0, T.size(), c.bwd, 1));
  PState ps;
  Tr(sync(c, &ps));
  if (he != hipSuccess) return dev_fail(c.E, he, "path setup");
  int cur = S_B0;
  // partitioned: the targets over all ranks (every rank must run the same levels)
  uint64_t n = c.part ? ps.n[S_B0] : T.size(), ds = ps.dsum[1];
  for (uint32_t l = 1; l < upto && n; ++l) {
    PathLevel lv;
    lv.lab = LAB_B;
    lv.stamp = stamp(eb, l);
    int rec = -1;
    Tr(level_ds(c, c.bwd, cur, n, ds, cur ^ 1, lv, 1, &rec));
    cur ^= 1;
    Tr(sync(c, &ps));
    if (he != hipSuccess) return dev_fail(c.E, he, "path level");
    n = ps.n[cur];
    ds = level_dsum(c, ps, rec, 1);
  }
  uint64_t scanned = 0;
  if (c.part)
    he = ws_all_paths_part(ws, c.fwd, LAB_B, eb, Sgid.data(), Svid.data(), Sgid.size(), upto, c.E.snap.nv,
                           c.E.snap.d_visible, max_walks(), &out->paths, &scanned);
  else
    he = ws_all_paths(ws, c.fwd, LAB_B, eb, S.data(), S.size(), upto, c.E.snap.d_vids, c.E.snap.d_visible,
                      max_walks(), &out->paths, &scanned);
  if (he == hipErrorOutOfMemory) return c.E.fail(NBG_E_OUT_OF_MEMORY, "FIND ALL PATH: too many paths");
  if (he != hipSuccess) return dev_fail(c.E, he, "path enumeration");
  c.edges += scanned;
  return NBG_OK;
}


// A one-pair SHORTEST request handed to a query slot instead of being run here.
struct PairLaunch {
  int mode = SP_CHAIN;
  SpTypes fwd, bwd;
  uint32_t s = NO_ROW, t = NO_ROW, upto = 0;
  uint64_t dmin = 0;   // min(out-degree of s, in-degree of t): the chain's length hint (sp_launch)
};
constexpr int32_t PAIR_DEFERRED = 1;

// nbg_find_path under the engine lock.  With `pl`, a single-engine one-pair SHORTEST request
// whose endpoints have edges is not run: *pl describes it and PAIR_DEFERRED is returned.
int32_t find_path_locked(Engine& E, const nbg_path_request* rq, nbg_paths** out, PairLaunch* pl) {
  if (!E.finalized) return E.fail(NBG_E_STATE, "engine not finalized");
  if (hipSetDevice(E.cfg.device) != hipSuccess) return E.fail(NBG_E_DEVICE, "hipSetDevice failed");
  if (!rq->shortest && rq->upto > 32) return E.fail(NBG_E_UNSUPPORTED, "FIND ALL PATH UPTO exceeds 32");
  if (rq->upto > MAX_PATH_LEN) return E.fail(NBG_E_UNSUPPORTED, "UPTO exceeds the device path limit (63)");
  // OVER (FindPathExecutor::prepareOver)
  std::vector<int32_t> over;
  if (rq->over_all) {
    for (auto& kv : E.edges) over.push_back(kv.first);
  } else {
    for (int32_t i = 0; i < rq->num_edge_types; ++i) {
      int32_t t = rq->edge_types[i];
      if (t <= 0 || !E.edges.count(t)) return E.fail(NBG_E_EXECUTION_ERROR, "edge type not found");
      if (std::find(over.begin(), over.end(), t) == over.end()) over.push_back(t);
    }
  }
  if (over.empty()) return E.fail(NBG_E_EXECUTION_ERROR, "empty OVER clause");
  if ((int)over.size() > MAX_TYPES_Q) return E.fail(NBG_E_UNSUPPORTED, "too many OVER types");
  auto* res = new nbg_paths();
  // from / to: de-duplicated; vertices without rows have no edges on either side.  Partitioned:
  // each rank resolves the ids it owns, and presence is summed over ranks so that every rank
  // takes the same branches (all collective calls below happen in the same order everywhere).
  std::vector<int64_t> fv, tv;
  {
    std::unordered_set<int64_t> seen;
    for (uint64_t i = 0; i < rq->num_from; ++i)
      if (seen.insert(rq->from[i]).second) fv.push_back(rq->from[i]);
    seen.clear();
    for (uint64_t i = 0; i < rq->num_to; ++i)
      if (seen.insert(rq->to[i]).second) tv.push_back(rq->to[i]);
  }
  std::vector<uint32_t> fd(fv.size()), td(tv.size());
  for (size_t i = 0; i < fv.size(); ++i) fd[i] = E.dense(fv[i]);
  for (size_t i = 0; i < tv.size(); ++i) td[i] = E.dense(tv[i]);
  // presence per from / to id, then: rank has OVER out-edges, rank lacks an OVER type's in-edges.
  // Partitioned, a present id's entry is its global id + 1 (owner * npad + local id + 1; only the
  // owner contributes), so the sum also tells every rank where each endpoint lives.  Next: the
  // OVER out-degree of the first source and in-degree of the first target (a pair's first
  // direction, summed like the rest: no set-up exchange later).
  const bool partd = E.partitioned();
  const size_t G = partd ? (size_t)E.cfg.num_gpus : 0;
  std::vector<unsigned long long> pres(fv.size() + tv.size() + 4 + G, 0);
  const size_t P_DEG = fv.size() + tv.size();
  const size_t P_ERR = P_DEG + 2;   // partitioned: one status word per rank (before the last two flags)
  auto presence = [&](uint32_t d) -> unsigned long long {
    if (d == NO_ROW) return 0;
    return partd ? (unsigned long long)E.cfg.rank * E.npad + d + 1 : 1;
  };
  for (size_t i = 0; i < fv.size(); ++i) pres[i] = presence(fd[i]);
  for (size_t i = 0; i < tv.size(); ++i) pres[fv.size() + i] = presence(td[i]);
  auto degree = [&](uint32_t v, int sign) {   // as host_degree over the OVER types (uncapped)
    unsigned long long sum = 0;
    if (v == NO_ROW || (!E.snap.h_visible.empty() && !E.snap.h_visible[v])) return sum;
    for (int32_t t : over) {
      auto it = E.snap.types.find(sign * t);
      if (it == E.snap.types.end() || it->second.h_row_ptr.size() <= (size_t)v + 1) continue;
      sum += it->second.h_row_ptr[v + 1] - it->second.h_row_ptr[v];
    }
    return sum;
  };
  const bool one_one = fv.size() == 1 && tv.size() == 1;
  if (one_one) {
    pres[P_DEG] = degree(fd[0], 1);
    pres[P_DEG + 1] = degree(td[0], -1);
  }
  for (int32_t t : over) {
    const bool out_edges = E.snap.types.count(t) > 0, in_edges = E.snap.types.count(-t) > 0;
    if (out_edges) pres[pres.size() - 2] = 1;
    if (out_edges && !in_edges) pres[pres.size() - 1] = 1;
  }
  if (partd) {
    // Everything that can fail on this rank alone happens before the request's first collective
    // and travels with it (one status word per rank): every rank then fails with the same code.
    int32_t lrc = ws_release(E, &E.ws, E.stream);   // a held device GO result keeps its rows
    std::string lmsg = lrc ? E.last_error : std::string();
    if (!lrc) {
      const hipError_t he = E.fault(NBG_FAULT_ALLOC)
                                ? hipErrorOutOfMemory
                                : ws_path_begin(E.ws, 0, E.snap.nv + fv.size() + tv.size() + 1024, true);
      if (he != hipSuccess) {
        lrc = NBG_E_OUT_OF_MEMORY;
        lmsg = std::string("path workspace: ") + hipGetErrorString(he);
      }
    }
    pres[P_ERR + (size_t)E.cfg.rank] = (unsigned long long)(int64_t)lrc;
    hipError_t he = ws_allreduce_host(E.ws, pres);
    if (he != hipSuccess) { delete res; return dev_fail(E, he, "path request exchange"); }
    for (size_t q = 0; q < G; ++q) {
      const int32_t code = (int32_t)(int64_t)pres[P_ERR + q];
      if (!code) continue;
      delete res;
      if (lrc) return E.fail(lrc, lmsg);
      return E.fail(code, "FIND PATH failed on rank " + std::to_string(q) + " (code " + std::to_string(code) + ")");
    }
  }
  if (pres[pres.size() - 1]) {
    delete res;
    return E.fail(NBG_E_UNSUPPORTED, "FIND PATH needs the in-edge records of every OVER type");
  }
  std::vector<uint32_t> S, Tg;        // local sources; targets by global position (NO_ROW: not here)
  std::vector<int64_t> Sv, Tv;        // their vids
  std::vector<uint32_t> Sgid, Tgid;   // partitioned: every source's / target's global id
  for (size_t i = 0; i < fv.size(); ++i)
    if (pres[i]) {
      Sv.push_back(fv[i]);
      if (partd) Sgid.push_back((uint32_t)(pres[i] - 1));
      if (fd[i] != NO_ROW) S.push_back(fd[i]);
    }
  for (size_t i = 0; i < tv.size(); ++i)
    if (pres[fv.size() + i]) {
      Tv.push_back(tv[i]);
      Tg.push_back(td[i]);
      if (partd) Tgid.push_back((uint32_t)(pres[fv.size() + i] - 1));
    }
  if (Sv.empty() || Tv.empty() || rq->upto == 0 || !pres[pres.size() - 2]) { *out = res; return NBG_OK; }
  if (!partd) {
    const int32_t rrc = ws_release(E, &E.ws, E.stream);   // a held device GO result keeps its rows
    if (rrc) { delete res; return rrc; }
  }
  PathCtx c{E, E.ws, {}, {}, 0, 0, E.partitioned()};
  const uint32_t cap = 0x7fffffff;
  // Partitioned, every rank lists every OVER type in the same order: lists, walk records and
  // greedy candidates name a type by its position, and a rank without edges of a type (a rank
  // with few or no parts) must not shift the others.  Such a type gets an empty CSR.
  bool zero_fail = false;
  auto add = [&](PathTypes& pt, int32_t signed_type) {
    auto it = E.snap.types.find(signed_type);
    if (it == E.snap.types.end()) {
      if (!partd) return;
      if (!E.snap.d_zero_rows) {
        void* z = nullptr;
        if (hipMalloc(&z, ((size_t)E.snap.nv + 1) * 4) != hipSuccess || hipMemset(z, 0, ((size_t)E.snap.nv + 1) * 4) != hipSuccess) {
          if (z) (void)hipFree(z);
          zero_fail = true;
          return;
        }
        E.snap.d_zero_rows = static_cast<uint32_t*>(z);
      }
      ExpandArgs a{};
      a.row_ptr = E.snap.d_zero_rows;
      a.visible = E.snap.d_visible;
      a.vids = E.snap.d_vids;
      a.cap = cap;
      pt.type[pt.n] = signed_type;
      pt.a[pt.n++] = a;
      return;
    }
    const DevEdgeType& dt = it->second;
    ExpandArgs a{};
    a.row_ptr = dt.row_ptr;
    a.col = dt.col;
    a.dst_vid = dt.dst_vid;
    a.rank = dt.rank;
    a.valid = dt.valid;
    a.visible = E.snap.d_visible;
    a.vids = E.snap.d_vids;
    a.props = dt.d_props;
    a.cap = cap;
    pt.type[pt.n] = signed_type;
    pt.a[pt.n++] = a;
    if (signed_type < 0) c.bwd_edges += dt.num_edges;
  };
  for (int32_t t : over) {
    add(c.fwd, t);
    add(c.bwd, -t);
  }
  if (zero_fail) {   // (after the request exchange: the collectives below would run without this rank)
    if (E.comm) E.comm->abort();
    delete res;
    return E.fail(NBG_E_OUT_OF_MEMORY, "empty CSR of an absent OVER type");
  }
  if (E.cfg.max_edge_returned_per_vertex != INT_MAX) {
    // capped rows: the reference's rounds over the two capped graphs (pathcap.hip); every
    // endpoint by global id (single engine: its dense id)
    CapEnv env;
    env.stream = ws_stream(E.ws);
    env.comm = partd ? ws_get_comm(E.ws) : nullptr;
    env.world = partd ? (int)G : 1;
    env.rank = partd ? E.cfg.rank : 0;
    env.nv = E.snap.nv;
    env.npad = E.npad;
    env.visible = E.snap.d_visible;
    env.vids = E.snap.d_vids;
    env.K = (uint32_t)E.cfg.max_edge_returned_per_vertex;
    const std::vector<uint32_t>& sg = partd ? Sgid : S;
    const std::vector<uint32_t>& tg = partd ? Tgid : Tg;
    uint64_t scanned = 0;
    const hipError_t he = rq->shortest
                              ? cap_shortest(env, c.fwd, c.bwd, sg, Sv, tg, rq->upto, &res->paths, &scanned)
                              : cap_all(env, c.fwd, c.bwd, sg, Sv, tg, Tv, rq->upto, max_walks(), &res->paths, &scanned);
    int32_t rc = NBG_OK;
    if (he == hipErrorNotFound)
      rc = E.fail(NBG_E_UNKNOWN, "shortest-path reconstruction failed (capped rows)");
    else if (he == hipErrorOutOfMemory)
      rc = E.fail(NBG_E_OUT_OF_MEMORY, "FIND PATH: too many paths or out of device memory");
    else if (he != hipSuccess)
      rc = dev_fail(E, he, "capped FIND PATH");
    if (rc) { delete res; return rc; }
    std::sort(res->paths.begin(), res->paths.end());
    res->edges = scanned;
    *out = res;
    return NBG_OK;
  }
  const bool pair = rq->shortest && Sv.size() == 1 && Tv.size() == 1 && Sv[0] != Tv[0];
  const int pmode = pair && !c.part ? sp_mode(c) : PM_HOST;
  if (pmode != PM_HOST) {
    const uint32_t s0 = S.empty() ? NO_ROW : S[0];
    const uint64_t ds0 = host_degree(c, c.fwd, s0), dt0 = host_degree(c, c.bwd, Tg[0]);
    if (pl && ds0 && dt0) {
      pl->dmin = std::min(ds0, dt0);
      pl->mode = pmode;
      pl->fwd = sp_types(c.E, c.fwd);
      pl->bwd = sp_types(c.E, c.bwd);
      pl->s = s0;
      pl->t = Tg[0];
      pl->upto = rq->upto;
      delete res;
      return PAIR_DEFERRED;
    }
    int32_t rc = device_pair(c, pmode, s0, Tg[0], rq->upto, res);
    if (rc) { delete res; return rc; }
    res->edges = c.edges;
    *out = res;
    return NBG_OK;
  }
  if (!partd) {   // (partitioned: begun before the request exchange)
    hipError_t he = ws_path_begin(c.ws, 0, E.snap.nv + S.size() + Tg.size() + 1024, !pair);
    if (he != hipSuccess) { delete res; return dev_fail(E, he, "path workspace"); }
  }
  int32_t rc;
  if (!rq->shortest) {
    std::vector<uint32_t> Tl;
    for (uint32_t d : Tg)
      if (d != NO_ROW) Tl.push_back(d);
    // partitioned: every source's global id (from the presence exchange) and vid
    std::vector<int64_t> Svid;
    if (c.part) Svid = Sv;
    rc = all_paths(c, S, Tl, rq->upto, Sgid, Svid, res);
  } else if (pair)
    rc = bidirectional(c, S.empty() ? NO_ROW : S[0], Tg[0], rq->upto, res, c.part ? (int64_t)Sgid[0] : -1, Sv[0],
                       c.part && one_one ? &pres[P_DEG] : nullptr);
  else
    rc = one_sided(c, S, Tg, Sv.size(), rq->upto, res);
  if (rc) { delete res; return rc; }
  std::sort(res->paths.begin(), res->paths.end());
  res->edges = c.edges;
  *out = res;
  return NBG_OK;
}

int sp_query_slots() {
  static const int n = [] {
    const char* v = getenv("NBG_QUERY_SLOTS");
    const int k = v ? atoi(v) : 6;
    return k < 1 ? 1 : (k > 16 ? 16 : k);
  }();
  return n;
}

}  // namespace

// ============================================================================= asynchronous FIND PATH
// Up to NBG_QUERY_SLOTS one-pair SHORTEST queries in flight, each on its own shortest-path
// workspace and HIP stream (the way graphd runs concurrent FindPathExecutors); every other request
// runs at submission.
struct nbg_path_ticket {
  Engine* eng = nullptr;
  int slot = -1;
  bool done = false;
  int32_t rc = NBG_OK;
  nbg_paths* result = nullptr;
};

namespace {

void path_complete_oldest(Engine& E) {
  auto* t = static_cast<nbg_path_ticket*>(E.path_inflight.front());
  E.path_inflight.erase(E.path_inflight.begin());
  Engine::PathSlot& ps = E.path_slots[t->slot];
  SpResult r;
  hipError_t he = sp_wait(ps.sp, &r);
  if (he != hipSuccess) {
    t->rc = E.fail(NBG_E_DEVICE, std::string("shortest path: ") + hipGetErrorString(he));
  } else if (r.err == 1) {
    t->rc = E.fail(NBG_E_UNKNOWN, "shortest-path reconstruction failed (in/out edges disagree)");
  } else if (r.err) {
    t->rc = E.fail(NBG_E_DEVICE, "shortest path: " + sp_err_text(r.err));
  } else {
    auto* res = new nbg_paths();
    res->edges = r.edges;
    res->batches = (uint32_t)r.batches;
    if (r.L) res->paths.emplace_back(r.path, r.path + 1 + 3 * r.L);
    t->result = res;
  }
  t->done = true;
  ps.ticket = nullptr;
}

}  // namespace

namespace {
nbg_paths* paths_of(const SpResult& r) {
  auto* res = new nbg_paths();
  res->edges = r.edges;
  res->batches = (uint32_t)r.batches;
  if (r.L) res->paths.emplace_back(r.path, r.path + 1 + 3 * r.L);
  return res;
}

int sp_batch_size() {
  static const int n = [] {
    const char* v = getenv("NBG_SP_BATCH");
    // RMAT-22 fixed batches: 16 -> 35.6 k, 32 -> 44.8 k pairs/s; RMAT-26 rolling runs: 32 -> 55.9 k,
    // 48 -> 60.3 k (profiles/r06_y_sp_slots_ab.txt; 64 contexts of ~3.2 GB do not fit beside the graph)
    // (64 with quarter-size lists, batch_list_cap: 61.4-62.0 k -> 63.4-64.2 k pairs/s, 87 GB of HBM
    // left free against 42 GB with 48 full-size contexts, profiles/r06_ap_sp_batch_lists_ab.txt)
    const int k = v ? atoi(v) : 64;
    return k < 1 ? 1 : (k > CH_ROLL_SLOTS ? CH_ROLL_SLOTS : k);
  }();
  return n;
}
}  // namespace

void nbg::path_slots_release(Engine& E) {
  while (!E.path_inflight.empty()) {
    auto* t = static_cast<nbg_path_ticket*>(E.path_inflight.front());
    path_complete_oldest(E);
    if (t->result) delete t->result;
    delete t;
  }
  for (auto& ps : E.path_slots) {
    if (ps.sp) sp_destroy(ps.sp);
    if (ps.stream) (void)hipStreamDestroy(ps.stream);
  }
  E.path_slots.clear();
  for (SpCtx* c : E.batch_sp) sp_destroy(c);
  E.batch_sp.clear();
  if (E.batch_stream) (void)hipStreamDestroy(E.batch_stream);
  E.batch_stream = nullptr;
}

extern "C" {

int32_t nbg_find_path(nbg_engine* h, const nbg_path_request* rq, nbg_paths** out) {
  if (!h || !rq || !out) return NBG_E_INVALID_ARGUMENT;
  *out = nullptr;
  Engine& E = *h->e.path_engine();   // a partitioned engine's replica runs it rank-locally
  std::lock_guard<std::mutex> lg(E.mu);
  static const bool trace = getenv("NBG_PATH_TRACE") != nullptr;
  if (!trace) return find_path_locked(E, rq, out, nullptr);
  const auto t0 = std::chrono::steady_clock::now();
  const int32_t rc = find_path_locked(E, rq, out, nullptr);
  fprintf(stderr, "nbg path total=%lld\n",
          (long long)std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0)
              .count());
  return rc;
}

int32_t nbg_find_path_submit(nbg_engine* h, const nbg_path_request* rq, nbg_path_ticket** out) {
  if (!h || !rq || !out) return NBG_E_INVALID_ARGUMENT;
  *out = nullptr;
  Engine& E = *h->e.path_engine();   // a partitioned engine's replica runs it rank-locally
  std::lock_guard<std::mutex> lg(E.mu);
  auto* t = new nbg_path_ticket();
  t->eng = &E;
  PairLaunch pl;
  nbg_paths* res = nullptr;
  const int32_t rc = find_path_locked(E, rq, &res, E.partitioned() ? nullptr : &pl);
  if (rc != PAIR_DEFERRED) {   // ran here (or failed): the ticket carries the outcome
    t->done = true;
    t->rc = rc;
    t->result = res;
    *out = t;
    return NBG_OK;
  }
  if (E.path_slots.empty()) E.path_slots.resize(sp_query_slots());
  int slot = -1;
  for (size_t i = 0; i < E.path_slots.size() && slot < 0; ++i)
    if (!E.path_slots[i].ticket) slot = (int)i;
  if (slot < 0) {   // every slot busy: finish the oldest query first
    slot = static_cast<nbg_path_ticket*>(E.path_inflight.front())->slot;
    path_complete_oldest(E);
  }
  Engine::PathSlot& ps = E.path_slots[slot];
  if (!ps.stream && hipStreamCreateWithFlags(&ps.stream, hipStreamNonBlocking) != hipSuccess) {
    delete t;
    return E.fail(NBG_E_DEVICE, "hipStreamCreate failed");
  }
  if (!ps.sp) {
    std::string err;
    ps.sp = E.new_sp(ps.stream, &err);
    if (!ps.sp) { delete t; return E.fail(NBG_E_OUT_OF_MEMORY, err); }
  }
  hipError_t he = sp_launch(ps.sp, pl.fwd, pl.bwd, E.snap.d_visible, E.snap.d_vids, pl.s, pl.t, pl.upto, pl.dmin);
  if (he != hipSuccess) { delete t; return dev_fail(E, he, "shortest path"); }
  t->slot = slot;
  ps.ticket = t;
  E.path_inflight.push_back(t);
  *out = t;
  return NBG_OK;
}

// A batch context's list capacity: NBG_SP_BATCH_LIST (default 1/4, read when contexts are made) of
// the vertices, at least 64 entries.  A pair whose search would outgrow it fails in the run with a
// list overflow and is rerun on the engine's full-size context; the lists are most of a context's
// memory (RMAT-26: 3.2 -> 1.2 GB per context), so 64 contexts take less HBM than 48 did.
static uint64_t batch_list_cap(const Engine& E) {
  const double frac = getenv("NBG_SP_BATCH_LIST") ? atof(getenv("NBG_SP_BATCH_LIST")) : 0.25;
  const uint64_t nv = E.snap.nv;
  return frac >= 1.0 || frac <= 0.0 ? 0 : std::max<uint64_t>(64, (uint64_t)((double)nv * frac) + 1);
}

// Batch contexts (with their level-loop buffers: a run allocates nothing) up to `want`, as HBM
// allows while leaving NBG_SP_BATCH_RESERVE_GB (default 8) free for the engine's other queries: a
// context that does not fit only makes the rolling runs narrower.  A growth that stopped short is
// retried by nbg_path_reserve only, not by every batch (each try allocates and frees gigabytes).
static void grow_batch_contexts(Engine& E, int want, std::string* err, bool retry) {
  if (E.batch_sp_full && !retry) return;   // (not every batch: a failed growth allocates and frees GBs)
  E.batch_sp_full = false;
  static const double reserve_gb = getenv("NBG_SP_BATCH_RESERVE_GB") ? atof(getenv("NBG_SP_BATCH_RESERVE_GB")) : -1.0;
  while ((int)E.batch_sp.size() < want) {
    SpCtx* c = E.new_sp(E.batch_stream, err);
    if (!c) {
      E.batch_sp_full = true;
      break;
    }
    sp_set_list_cap(c, batch_list_cap(E));
    size_t free_b = 0, total_b = 0;
    const bool ok = sp_reserve_chain(c) == hipSuccess && hipMemGetInfo(&free_b, &total_b) == hipSuccess;
    const double reserve = (reserve_gb >= 0 ? reserve_gb : 8.0) * (1ull << 30);
    if (!ok || (!E.batch_sp.empty() && (double)free_b < reserve)) {
      sp_destroy(c);
      if (!ok && err) *err = "shortest-path chain buffers";
      E.batch_sp_full = true;
      break;
    }
    E.batch_sp.push_back(c);
  }
  if (getenv("NBG_SP_TRACE")) {
    size_t free_b = 0, total_b = 0;
    (void)hipMemGetInfo(&free_b, &total_b);
    fprintf(stderr, "[sp batch] %zu contexts (wanted %d, lists of %llu entries), %.1f GB of HBM free; %llu pairs rerun so far\n",
            E.batch_sp.size(), want, (unsigned long long)batch_list_cap(E), free_b / 1073741824.0,
            (unsigned long long)E.batch_reruns);
  }
}

int32_t nbg_find_path_batch(nbg_engine* h, const nbg_path_request* reqs, uint64_t n, nbg_paths** out, int32_t* rcs) {
  if (!h || (n && (!reqs || !out || !rcs))) return NBG_E_INVALID_ARGUMENT;
  Engine& E = *h->e.path_engine();
  std::lock_guard<std::mutex> lg(E.mu);
  for (uint64_t i = 0; i < n; ++i) {
    out[i] = nullptr;
    rcs[i] = NBG_OK;
  }
  // every request is classified as nbg_find_path_submit would; the one-pair SHORTEST ones of the
  // device level loop are deferred and run as batched chains, the rest run here
  std::vector<PairLaunch> pl;
  std::vector<uint64_t> at;
  for (uint64_t i = 0; i < n; ++i) {
    PairLaunch x;
    nbg_paths* res = nullptr;
    const int32_t rc = find_path_locked(E, &reqs[i], &res, E.partitioned() ? nullptr : &x);
    if (rc == PAIR_DEFERRED && x.mode == SP_CHAIN) {
      pl.push_back(x);
      at.push_back(i);
      continue;
    }
    if (rc == PAIR_DEFERRED) {   // another device mode: one pair at a time on the engine's workspace
      res = new nbg_paths();
      if (!E.sp) {
        std::string err;
        E.sp = E.new_sp(E.stream, &err);
        if (!E.sp) {
          delete res;
          rcs[i] = E.fail(NBG_E_OUT_OF_MEMORY, err);
          continue;
        }
      }
      SpResult r;
      hipError_t he = sp_launch(E.sp, x.fwd, x.bwd, E.snap.d_visible, E.snap.d_vids, x.s, x.t, x.upto, x.dmin);
      if (he == hipSuccess) he = sp_wait(E.sp, &r);
      delete res;
      if (he != hipSuccess) {
        rcs[i] = dev_fail(E, he, "shortest path");
        continue;
      }
      if (r.err) {
        rcs[i] = E.fail(r.err == 1 ? NBG_E_UNKNOWN : NBG_E_DEVICE, "shortest path: " + sp_err_text(r.err));
        continue;
      }
      out[i] = paths_of(r);
      continue;
    }
    rcs[i] = rc;
    out[i] = res;
  }
  if (pl.empty()) return NBG_OK;
  // From here on every deferred request gets its own status: a batch-level failure marks the
  // requests that did not run (out[i] stays NULL only where rcs[i] != NBG_OK, nbg.h)
  std::vector<char> ran(pl.size(), 0);
  auto fail_rest = [&](int32_t code) {
    for (size_t k = 0; k < pl.size(); ++k)
      if (!ran[k]) rcs[at[k]] = code;
    return code;
  };
  if (!E.batch_stream && hipStreamCreateWithFlags(&E.batch_stream, hipStreamNonBlocking) != hipSuccess)
    return fail_rest(E.fail(NBG_E_DEVICE, "hipStreamCreate failed"));
  // batch contexts (each holds ~72 B per vertex): as many as NBG_SP_BATCH asks for and HBM
  // allows — a context that cannot be allocated only makes the batches smaller
  const int want = std::min<int>(sp_batch_size(), (int)pl.size());
  std::string cerr;
  grow_batch_contexts(E, want, &cerr, false);
  if (E.batch_sp.empty()) return fail_rest(E.fail(NBG_E_OUT_OF_MEMORY, cerr));
  const int B = std::min<int>(want, (int)E.batch_sp.size());
  // a pair whose search outgrew its batch context's lists (err bit 2: list overflow; batch_list_cap)
  // runs again on the engine's own full-size context
  auto finish = [&](size_t k, SpResult r) -> hipError_t {
    const uint64_t i = at[k];
    if (r.err & 2) {
      const PairLaunch& x = pl[k];
      std::string err;
      if (!E.sp) E.sp = E.new_sp(E.stream, &err);
      if (!E.sp) return hipErrorOutOfMemory;
      hipError_t he = sp_launch(E.sp, x.fwd, x.bwd, E.snap.d_visible, E.snap.d_vids, x.s, x.t, x.upto, x.dmin);
      if (he == hipSuccess) he = sp_wait(E.sp, &r);
      if (he != hipSuccess) return he;
      ++E.batch_reruns;
    }
    ran[k] = 1;
    if (r.err == 1) {
      rcs[i] = E.fail(NBG_E_UNKNOWN, "shortest-path reconstruction failed (in/out edges disagree)");
    } else if (r.err) {
      rcs[i] = E.fail(NBG_E_DEVICE, "shortest path: " + sp_err_text(r.err));
    } else {
      out[i] = paths_of(r);
    }
    return hipSuccess;
  };
  // (read per call: the tests run both paths and small runs in one process)
  auto env_int = [](const char* k, int dflt) { return getenv(k) ? atoi(getenv(k)) : dflt; };
  const bool roll = env_int("NBG_SP_ROLL", 1) != 0;
  const size_t chunk = (size_t)std::max(1, env_int("NBG_SP_ROLL_CHUNK", 4096));
  const int roll_slots = std::max(1, std::min(B, env_int("NBG_SP_ROLL_SLOTS", B)));
  // pairs [k0, k1) of one query shape as rolling runs (a slot takes the next pair as soon as its
  // pair is done; spchain.hip k_ch_roll) of at most NBG_SP_ROLL_CHUNK (4096) pairs over
  // NBG_SP_ROLL_SLOTS (NBG_SP_BATCH) slots
  auto run_roll = [&](size_t k0, size_t k1) -> hipError_t {
    std::vector<uint32_t> ss, ts;
    std::vector<SpResult> res;
    for (size_t c0 = k0; c0 < k1; c0 += chunk) {
      const size_t c1 = std::min(k1, c0 + chunk), m = c1 - c0;
      ss.resize(m);
      ts.resize(m);
      res.resize(m);
      for (size_t k = 0; k < m; ++k) {
        ss[k] = pl[c0 + k].s;
        ts[k] = pl[c0 + k].t;
      }
      const int slots = (int)std::min<size_t>((size_t)roll_slots, m);
      const PairLaunch& x = pl[c0];
      if (hipError_t he = sp_roll(E.batch_sp.data(), slots, x.fwd, x.bwd, E.snap.d_visible, E.snap.d_vids, ss.data(),
                                  ts.data(), (uint32_t)m, x.upto, res.data()))
        return he;
      for (size_t k = 0; k < m; ++k)
        if (hipError_t he = finish(c0 + k, res[k])) return he;
    }
    return hipSuccess;
  };
  // ... or as batches of B pairs, each running the whole chain UPTO allows (UPTO over
  // CH_ROLL_UPTO, or NBG_SP_ROLL=0)
  auto run_fixed = [&](size_t k0, size_t k1) -> hipError_t {
    const int Bf = std::min(B, 32);
    for (size_t b0 = k0; b0 < k1; b0 += (size_t)Bf) {
      const int nb = (int)std::min<size_t>((size_t)Bf, k1 - b0);
      std::vector<SpPair> sp(nb);
      for (int p = 0; p < nb; ++p) {
        const PairLaunch& x = pl[b0 + p];
        sp[p] = SpPair{&x.fwd, &x.bwd, E.snap.d_visible, E.snap.d_vids, x.s, x.t, x.upto};
      }
      hipError_t he = sp_launch_batch(E.batch_sp.data(), nb, sp.data());
      for (int p = 0; p < nb && he == hipSuccess; ++p) {
        SpResult r;
        he = sp_wait(E.batch_sp[p], &r);
        if (he == hipSuccess) he = finish(b0 + p, r);
      }
      if (he != hipSuccess) return he;
    }
    return hipSuccess;
  };
  auto same_shape = [&](const PairLaunch& a, const PairLaunch& b) {
    return a.upto == b.upto && a.fwd.row_ptr[0] == b.fwd.row_ptr[0] && a.fwd.col[0] == b.fwd.col[0] &&
           a.bwd.row_ptr[0] == b.bwd.row_ptr[0] && a.bwd.col[0] == b.bwd.col[0] && a.fwd.type[0] == b.fwd.type[0] &&
           a.fwd.dst_vid[0] == b.fwd.dst_vid[0] && a.fwd.rank[0] == b.fwd.rank[0] && a.fwd.ne[0] == b.fwd.ne[0] &&
           a.bwd.ne[0] == b.bwd.ne[0];
  };
  for (size_t k0 = 0; k0 < pl.size();) {
    size_t k1 = k0 + 1;
    while (k1 < pl.size() && same_shape(pl[k0], pl[k1])) ++k1;
    const hipError_t he = roll && pl[k0].upto <= CH_ROLL_UPTO ? run_roll(k0, k1) : run_fixed(k0, k1);
    if (he != hipSuccess) return fail_rest(dev_fail(E, he, "shortest path batch"));
    k0 = k1;
  }
  return NBG_OK;
}

int32_t nbg_path_reserve(nbg_engine* h, int32_t slots, int32_t batch) {
  if (!h || slots < 0 || batch < 0) return NBG_E_INVALID_ARGUMENT;
  Engine& E = *h->e.path_engine();
  std::lock_guard<std::mutex> lg(E.mu);
  if (!E.finalized) return E.fail(NBG_E_STATE, "engine not finalized");
  if (E.partitioned()) return NBG_OK;   // partitioned searches run on the engine's workspace
  if (hipSetDevice(E.cfg.device) != hipSuccess) return E.fail(NBG_E_DEVICE, "hipSetDevice failed");
  std::string err;
  auto ready = [&](SpCtx*& c, hipStream_t s) -> int32_t {
    if (!c) c = E.new_sp(s, &err);
    if (!c) return E.fail(NBG_E_OUT_OF_MEMORY, err);
    return sp_reserve_chain(c) == hipSuccess ? NBG_OK : E.fail(NBG_E_OUT_OF_MEMORY, "shortest-path chain buffers");
  };
  if (int32_t rc = ready(E.sp, E.stream)) return rc;
  if (E.path_slots.empty()) E.path_slots.resize(sp_query_slots());
  for (int i = 0; i < slots && i < (int)E.path_slots.size(); ++i) {
    Engine::PathSlot& ps = E.path_slots[i];
    if (!ps.stream && hipStreamCreateWithFlags(&ps.stream, hipStreamNonBlocking) != hipSuccess)
      return E.fail(NBG_E_DEVICE, "hipStreamCreate failed");
    if (int32_t rc = ready(ps.sp, ps.stream)) return rc;
  }
  const int want = std::min(batch, sp_batch_size());
  if (want > 0 && !E.batch_stream && hipStreamCreateWithFlags(&E.batch_stream, hipStreamNonBlocking) != hipSuccess)
    return E.fail(NBG_E_DEVICE, "hipStreamCreate failed");
  // (batch contexts as HBM allows, as nbg_find_path_batch allocates them: one that does not fit
  // only makes the rolling runs narrower)
  grow_batch_contexts(E, want, &err, true);
  if (want > 0 && E.batch_sp.empty()) return E.fail(NBG_E_OUT_OF_MEMORY, "shortest-path batch contexts");
  return NBG_OK;
}

int32_t nbg_find_path_wait(nbg_path_ticket* t, nbg_paths** out) {
  if (!t || !out) return NBG_E_INVALID_ARGUMENT;
  Engine& E = *t->eng;
  std::lock_guard<std::mutex> lg(E.mu);
  *out = nullptr;
  if (!t->done) {
    while (!E.path_inflight.empty() && E.path_inflight.front() != t) path_complete_oldest(E);
    path_complete_oldest(E);
  }
  const int32_t rc = t->rc;
  *out = t->result;
  delete t;
  return rc;
}

}  // extern "C"
