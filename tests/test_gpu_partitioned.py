"""Partitioned GO N STEPS on the MI355X: G engines, each holding the parts
p % G == rank, exchange each hop's candidate set with a bitmap all-to-all.  The union of the
ranks' rows must equal the single-engine result bit-exactly (sorted row multisets), and the
whole-query statistics (|F_s|, E_s) must equal the single engine's.

The ranks run as an in-process group on one GPU (nbg_comm_init_local: one host thread per rank,
the same engine code as one RCCL rank per process; only the transport differs)."""
import numpy as np
import pytest

from nebula_amd import LocalCluster, NbgError, _lib, expr as E, kvgen
from tests.support import golden, graphs
from tests.support.oracle import nba_oracle

pytestmark = pytest.mark.gpu

WHERES = {
    "none": None,
    "w<50": E.binop("<", E.edge_prop("e", "w"), E.const(50)),
    "w%7==3||w>=90": E.binop("||", E.binop("==", E.binop("%", E.edge_prop("e", "w"), E.const(7)), E.const(3)),
                             E.binop(">=", E.edge_prop("e", "w"), E.const(90))),
}


def cluster_for(src, dst, w, world, parts=100, max_edge=0x7FFFFFFF, replica=False):
    """A partitioned cluster.  FIND PATH here tests the COLLECTIVE search over the partitioned
    snapshot, so the path replica is off unless asked for (test_gpu_replica.py covers it)."""
    c = LocalCluster(parts, world, max_edge_returned_per_vertex=max_edge)
    c.set_path_replica(1 if replica else 0)
    c.register_edge(graphs.E_TYPE, "e", graphs.E_SCHEMA)
    c.load_edges(graphs.E_TYPE, src, dst, [w])
    c.finalize()
    return c


@pytest.fixture(scope="module")
def rmat11():
    src, dst, w = graphs.rmat_graph(11)
    single = graphs.one_sided_engine(src, dst, w)
    orc = graphs.rmat_oracle(src, dst, w)
    clusters = {g: cluster_for(src, dst, w, g) for g in (2, 3, 4)}
    yield src, single, orc, clusters
    for c in clusters.values():
        c.close()
    single.close()
    orc.close()


@pytest.mark.parametrize("world", [2, 3, 4])
@pytest.mark.parametrize("steps", [1, 2, 3])
@pytest.mark.parametrize("where", list(WHERES))
def test_partitioned_go_matches_single_and_oracle(rmat11, world, steps, where):
    src, single, orc, clusters = rmat11
    c = clusters[world]
    wb = WHERES[where].encode() if WHERES[where] is not None else b""
    yields = [E.edge_prop("e", "_src").encode(), E.edge_prop("e", "_dst").encode(), E.edge_prop("e", "w").encode()]
    for r in graphs.roots(src, 3, seed=5):
        got = graphs.sorted_rows(c.go([r], [1], steps, wb, yields))
        ref = graphs.sorted_rows(single.go([r], [1], steps, wb, yields))
        assert got == ref, f"G={world} root {r}: {len(got)} vs {len(ref)} rows"
        # the whole-query statistics are global on every rank
        assert c.last_step_stats == single.last_step_stats
        exp = graphs.sorted_rows(orc.go([r], [1], steps, wb, yields))
        assert got == exp


def test_partitioned_multi_start_duplicates(rmat11):
    src, single, orc, clusters = rmat11
    rs = graphs.roots(src, 6, seed=9)
    starts = rs + rs[:2] + [123456789]          # duplicates kept, unknown vid ignored
    for world, c in clusters.items():
        got = graphs.sorted_rows(c.go(starts, [1], 2))
        assert got == graphs.sorted_rows(orc.go(starts, [1], 2)), world


def test_partitioned_eval_error_is_global(rmat11):
    # WHERE e.w / 0 fails the whole query wherever the failing edge lives
    src, single, orc, clusters = rmat11
    bad = E.binop("==", E.binop("/", E.edge_prop("e", "w"), E.const(0)), E.const(1)).encode()
    r = graphs.roots(src, 1, seed=3)[0]
    for c in clusters.values():
        errs = c.each(lambda e: _code_of(lambda: e.go([r], [1], 2, bad)))
        assert errs == [_lib.E_EXECUTION_ERROR] * len(errs)


def _code_of(fn):
    try:
        fn()
        return 0
    except NbgError as ex:
        return ex.code


def test_partitioned_edge_cap():
    src, dst, w = graphs.rmat_graph(10)
    c = cluster_for(src, dst, w, 2, max_edge=3)
    orc = graphs.rmat_oracle(src, dst, w, max_edge=3)
    try:
        for r in graphs.roots(src, 3, seed=11):
            assert graphs.sorted_rows(c.go([r], [1], 3)) == graphs.sorted_rows(orc.go([r], [1], 3))
    finally:
        c.close()
        orc.close()


def test_partitioned_nba_golden(nba_data):
    """The reference's GoTest golden cases through the KV path on 3 ranks (7 parts)."""
    parts = 7
    c = LocalCluster(parts, 3)
    for (kind, name), cols in kvgen.NBA_SCHEMAS.items():
        if kind == "edge":
            c.register_edge(kvgen.NBA_EDGES[name], name, cols)
        else:
            c.register_tag(kvgen.NBA_TAGS[name], name, cols)
    c.load_builder(kvgen.nba_kv(nba_data, parts))
    orc = nba_oracle(nba_data, parts)
    try:
        checked = 0
        for case in golden.load("go_golden.json"):
            if golden.unsupported_reason(case):
                continue
            try:
                ok, msg = golden.run_go_case(c, case)
            except NbgError as ex:
                if ex.code == _lib.E_UNSUPPORTED:   # same cases the single-engine test skips
                    continue
                raise
            assert ok, msg
            checked += 1
        assert checked > 0
    finally:
        c.close()
        orc.close()


# --------------------------------------------------------------------------- FIND SHORTEST PATH
# The partitioned BFS claims at the owner after the bitmap all-to-all; B-sets and the greedy are
# collective.  Every rank returns the same paths, equal to the single engine's and the oracle's.
@pytest.mark.parametrize("world", [2, 3, 4])
def test_partitioned_shortest_single_pairs(rmat11, world):
    from nebula_amd import rmat
    src, single, orc, clusters = rmat11
    c = clusters[world]
    found = 0
    for s, t in rmat.pick_pairs(src, _dst_of(src), 24, seed=world):
        for upto in (2, 5):
            st, st1 = {}, {}
            got = c.find_path([s], [t], [1], upto, stats=st)
            ref = single.find_path([s], [t], [1], upto, stats=st1)
            assert got == ref, (world, s, t, upto)
            assert st["edges"] == st1["edges"]
            assert got == sorted(orc.find_path([s], [t], [1], upto, True, mode=1))
            found += len(got)
    assert found > 0


@pytest.mark.parametrize("world", [2, 3])
def test_partitioned_shortest_sparse_and_bitmap_levels(world):
    """RMAT-16: a level whose edge total is at most 1/16 of a bitmap segment's bits exchanges
    per-owner slot arrays (k_list_claim), a larger one the bitmap (k_bits_claim); the greedy
    scans hub rows wave-wide.  Paths and scanned-edge counts equal the single engine's, which
    the oracle pins at RMAT-11 above."""
    from nebula_amd import rmat
    src, dst, w = graphs.rmat_graph(16)
    single = graphs.one_sided_engine(src, dst, w)
    c = cluster_for(src, dst, w, world)
    try:
        found = 0
        for s, t in rmat.pick_pairs(src, dst, 40, seed=31 + world):
            st, st1 = {}, {}
            got = c.find_path([s], [t], [1], 5, stats=st)
            assert got == single.find_path([s], [t], [1], 5, stats=st1), (world, s, t)
            assert st["edges"] == st1["edges"]
            found += len(got)
        assert found > 0
        ps = rmat.pick_pairs(src, dst, 8, seed=7)
        frm, to = [p[0] for p in ps[:3]], [p[1] for p in ps]
        assert c.find_path(frm, to, [1], 4) == single.find_path(frm, to, [1], 4)
    finally:
        c.close()
        single.close()


@pytest.mark.parametrize("world", [2, 4])
def test_partitioned_shortest_multi_and_self(rmat11, world):
    from nebula_amd import rmat
    src, single, orc, clusters = rmat11
    c = clusters[world]
    ps = rmat.pick_pairs(src, _dst_of(src), 18, seed=13)
    for k in range(0, 18, 6):
        frm = [p[0] for p in ps[k:k + 3]]
        to = [p[1] for p in ps[k:k + 6]] + [frm[0], 123456789]
        got = c.find_path(frm + frm[:1], to, [1], 4)
        assert got == single.find_path(frm + frm[:1], to, [1], 4), (frm, to)
        assert got == sorted(orc.find_path(frm, to, [1], 4, True, mode=1))
    s = ps[0][0]
    assert c.find_path([s], [s], [1], 5) == single.find_path([s], [s], [1], 5)
    assert c.find_path([s], [123456789], [1], 5) == []
    assert c.find_path([123456789], [s], [1], 5) == []


# --------------------------------------------------------------------------- FIND ALL PATH
# A walk is extended by the owner of its last vertex; each level is all-gathered, so every rank
# holds every walk and returns the same entry lists (the single engine's, the oracle's).
@pytest.mark.parametrize("world", [2, 3, 4])
@pytest.mark.parametrize("upto", [1, 2, 3, 4])
def test_partitioned_all_paths_single_pairs(rmat11, world, upto):
    from nebula_amd import rmat
    src, single, orc, clusters = rmat11
    c = clusters[world]
    total = 0
    for s, t in rmat.pick_pairs(src, _dst_of(src), 6, seed=10 * world + upto):
        st, st1 = {}, {}
        got = c.find_path([s], [t], [1], upto, shortest=False, stats=st)
        ref = single.find_path([s], [t], [1], upto, shortest=False, stats=st1)
        assert got == ref, (world, s, t, upto, len(got), len(ref))
        assert st["edges"] == st1["edges"]
        if upto <= 3:
            assert got == sorted(orc.find_path([s], [t], [1], upto, False))
        total += len(got)
    if upto >= 3:
        assert total > 0


@pytest.mark.parametrize("world", [2, 3])
def test_partitioned_all_paths_sets(rmat11, world):
    """Several sources and targets, a source that is also a target (cycles back to it), duplicate
    and unknown vids."""
    from nebula_amd import rmat
    src, single, orc, clusters = rmat11
    c = clusters[world]
    ps = rmat.pick_pairs(src, _dst_of(src), 12, seed=21)
    frm = [p[0] for p in ps[:3]]
    to = [p[1] for p in ps[:5]] + [frm[0], 123456789]
    got = c.find_path(frm + frm[:1], to, [1], 3, shortest=False)
    assert got == single.find_path(frm + frm[:1], to, [1], 3, shortest=False) and got
    assert got == sorted(orc.find_path(frm, to, [1], 3, False))
    assert c.find_path([123456789], to, [1], 3, shortest=False) == []


def test_partitioned_all_paths_multi_edge_ranks():
    """Two OVER types with ranks on 3 ranks: multi-edges between the same pair are distinct walks,
    each carrying its own type and rank through the level exchange."""
    from nebula_amd import rmat
    src, persons, single, orc = graphs.tagged_pair(9)
    c = graphs.tagged_pair_cluster(9, 3)
    try:
        for s, t in rmat.pick_pairs(src, src[::-1].copy(), 8, seed=2):
            got = c.find_path([s], [t], [graphs.E_TYPE, graphs.E_F], 3, shortest=False)
            assert got == single.find_path([s], [t], [graphs.E_TYPE, graphs.E_F], 3, shortest=False), (s, t)
            assert got == sorted(orc.find_path([s], [t], [graphs.E_TYPE, graphs.E_F], 3, False))
    finally:
        c.close()
        single.close()
        orc.close()


def test_partitioned_shortest_nba_golden(nba_data):
    """The reference's FindPathTest golden cases on 3 ranks (7 parts)."""
    c = LocalCluster(7, 3)
    c.set_path_replica(0)   # the collective search
    for (kind, name), cols in kvgen.NBA_SCHEMAS.items():
        if kind == "edge":
            c.register_edge(kvgen.NBA_EDGES[name], name, cols)
        else:
            c.register_tag(kvgen.NBA_TAGS[name], name, cols)
    c.load_builder(kvgen.nba_kv(nba_data, 7))
    try:
        checked = 0
        for case in golden.load("findpath_golden.json"):
            if golden.unsupported_reason(case):
                continue
            ok, msg = golden.run_path_case(c, case)   # SHORTEST and ALL: nothing unsupported
            assert ok, msg
            checked += 1
        assert checked > 0
    finally:
        c.close()


_DST = {}


def _dst_of(src):
    """The dst array of the module's RMAT-11 graph (pick_pairs draws from both ends)."""
    if "d" not in _DST:
        _DST["d"] = graphs.rmat_graph(11)[1]
    return _DST["d"]


@pytest.mark.parametrize("world", [2, 3])
def test_partitioned_async_slots(rmat11, world):
    """nbg_go_submit on a partitioned engine: more queries than slots in flight per rank (the
    slots share the rank's stream, so the collectives stay in submission order); the union of
    the ranks' rows equals the single engine's for every query."""
    src, single, orc, clusters = rmat11
    c = clusters[world]
    wb = WHERES["w<50"].encode()
    roots = graphs.roots(src, 9, seed=13)

    def run(e):
        stmt = e.prepare_go([graphs.E_TYPE], 3, wb)
        try:
            tickets = [stmt.submit([r], device=False) for r in roots]
            out = []
            for t in tickets:
                res = stmt.wait(t)
                out.append((res.fetch(), res.edges_scanned))
                res.free()
            return out
        finally:
            stmt.free()

    per_rank = c.each(run)
    for i, r in enumerate(roots):
        rows = []
        for rk in per_rank:
            rows += rk[i][0]
        exp = single.go([r], [graphs.E_TYPE], 3, wb)
        assert graphs.sorted_rows(rows) == graphs.sorted_rows(exp), r
        assert all(rk[i][1] == per_rank[0][i][1] for rk in per_rank)


@pytest.mark.parametrize("world", [2, 3, 4])
@pytest.mark.parametrize("steps", [1, 2, 3])
def test_partitioned_distinct_matches_single(rmat11, world, steps):
    """YIELD DISTINCT on a partitioned engine: each rank deduplicates its rows, the survivors go to
    the rank their identity hashes to (all-to-all) and are deduplicated there, so the union of the
    ranks' rows has every distinct row exactly once — the single engine's DISTINCT result."""
    src, single, orc, clusters = rmat11
    c = clusters[world]
    wb = WHERES["w<50"].encode()
    for yields in ([E.edge_prop("e", "_dst").encode()],
                   [E.edge_prop("e", "w").encode(), E.binop("%", E.edge_prop("e", "_dst"), E.const(7)).encode()]):
        for r in graphs.roots(src, 2, seed=steps):
            got = graphs.sorted_rows(c.go([r], [1], steps, wb, yields, distinct=True))
            ref = graphs.sorted_rows(single.go([r], [1], steps, wb, yields, distinct=True))
            assert got == ref, (world, steps, r, len(got), len(ref))
            assert len(set(map(tuple, got))) == len(got)
            assert got == graphs.sorted_rows(orc.go([r], [1], steps, wb, yields, distinct=True))


def test_partitioned_nba_golden_needs_no_skips(nba_data):
    """Every GO golden case the single engine runs also runs on 3 ranks (DISTINCT, $$ STRING,
    $- / $var props): no NBG_E_UNSUPPORTED left on the partitioned path."""
    c = LocalCluster(7, 3)
    for (kind, name), cols in kvgen.NBA_SCHEMAS.items():
        if kind == "edge":
            c.register_edge(kvgen.NBA_EDGES[name], name, cols)
        else:
            c.register_tag(kvgen.NBA_TAGS[name], name, cols)
    c.load_builder(kvgen.nba_kv(nba_data, 7))
    try:
        skipped = []
        for case in golden.load("go_golden.json"):
            if golden.unsupported_reason(case):
                continue
            try:
                ok, msg = golden.run_go_case(c, case)
            except NbgError as ex:
                if ex.code == _lib.E_UNSUPPORTED:
                    skipped.append((case["query"], str(ex)))
                    continue
                raise
            assert ok, msg
        assert not skipped, skipped
    finally:
        c.close()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("steps", [1, 2, 3])
def test_partitioned_input_props_backtracker(world, steps):
    """$-.col in YIELD / WHERE after N steps on a partitioned engine: the roots travel with each
    hop's exchange (as vids, to the neighbour's owner) — vs the oracle, on the forest whose roots
    reach disjoint vertex sets (so the reference's last-write-wins back tracker is unambiguous)."""
    from tests.test_gpu_go import _forest
    roots, src, dst, w = _forest()
    c = LocalCluster(7, world)
    c.register_edge(graphs.E_TYPE, "e", graphs.E_SCHEMA)
    c.load_edges(graphs.E_TYPE, src, dst, [w])
    c.finalize()
    orc = graphs.rmat_oracle(src, dst, w, parts=7)
    try:
        rows = [[r, 1000 + i, 0.5 * i] for i, r in enumerate(roots)] + [[roots[0], 7, 9.25]]
        inputs = (["id", "tag", "score"], rows, "id")
        yields = [E.input_prop("tag").encode(), E.input_prop("score").encode(), E.edge_prop("e", "_dst").encode()]
        where = E.binop(">", E.input_prop("tag"), E.const(1001)).encode()
        for wb in (b"", where):
            got = c.go(roots, [1], steps, wb, yields, inputs=inputs)
            exp = orc.go(roots, [1], steps, wb, yields, inputs=inputs)
            assert graphs.sorted_rows(got) == graphs.sorted_rows(exp) and got
    finally:
        c.close()
        orc.close()


def test_partitioned_shortest_forward_bsets_switch():
    """NBG_PART_FWD_BSETS=1 (off by default): the forward B-set recovery past kf gives
    the single engine's paths and scanned-edge counts.  The switch is read once per process, so
    the check runs in a child process started with it set."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, NBG_PART_FWD_BSETS="1", NBG_COMM_TIMEOUT_S="60")
    p = subprocess.run([sys.executable, os.path.join(root, "tests", "support", "fwd_bsets_probe.py")], cwd=root,
                       env=env, capture_output=True, text=True, timeout=180)
    assert p.returncode == 0 and "PASS" in p.stdout, p.stdout[-3000:] + p.stderr[-3000:]
