"""The 8-way partition (BASELINE configs[2]: 100 parts over 8 GPUs) as a tested path.

G = 8 reaches code that G = 2/3/4 does not: ranks holding 12 or 13 of the 100 parts
(`CreateSpaceProcessor.cpp:84-95`, GPU = part % G), `npad` rounding over 8 dictionaries, 7 peers
per all-to-all, 7 split communicators per rank for the query slots, the FIND PATH replica
all-gathered over 8 ranks, and — with the 7-part nba space — a rank that serves no part at all.

Every check compares the 8-rank result with the single engine (which the oracle pins at every
size the other test files cover) and, where the faithful oracle finishes in seconds, with the
oracle directly.  The ranks are an in-process group on one GPU (nbg_comm_init_local); the
8-process RCCL rehearsal is `tools/rccl_probe.py --same-device` (profiles/r04_*)."""
import numpy as np
import pytest

from nebula_amd import LocalCluster, NbgError, _lib as L, expr as E, kvgen, rmat
from tests.support import golden, graphs
from tests.support.oracle import nba_oracle

pytestmark = pytest.mark.gpu

G = 8
WHERE = E.binop("<", E.edge_prop("e", "w"), E.const(50))
WHERE2 = E.binop("||", E.binop("==", E.binop("%", E.edge_prop("e", "w"), E.const(7)), E.const(3)),
                 E.binop(">=", E.edge_prop("e", "w"), E.const(90)))
YIELDS = [E.edge_prop("e", "_src"), E.edge_prop("e", "_dst"), E.edge_prop("e", "w")]


def _cluster(src, dst, w, parts=100, max_edge=0x7FFFFFFF, replica=False):
    c = LocalCluster(parts, G, max_edge_returned_per_vertex=max_edge)
    c.set_path_replica(1 if replica else 0)
    c.register_edge(graphs.E_TYPE, "e", graphs.E_SCHEMA)
    c.load_edges(graphs.E_TYPE, src, dst, [w])
    c.finalize()
    return c


def _codes(c, fn):
    def one(e):
        try:
            fn(e)
            return 0
        except NbgError as ex:
            return ex.code
    return c.each(one)


@pytest.fixture(scope="module")
def rmat14():
    src, dst, w = graphs.rmat_graph(14)
    single = graphs.one_sided_engine(src, dst, w)
    orc = graphs.rmat_oracle(src, dst, w)
    c = _cluster(src, dst, w)
    yield src, dst, w, single, orc, c
    c.close()
    single.close()
    orc.close()


def test_every_rank_serves_its_parts(rmat14):
    """part % 8: ranks hold 12 or 13 of the 100 parts; every vertex is owned by exactly one rank,
    so the ranks' vertex counts add up to the single engine's."""
    src, dst, w, single, orc, c = rmat14
    per = [e.stats() for e in c.engines]
    owned = [sum(1 for p in range(1, 101) if p % G == r) for r in range(G)]
    assert sorted(set(owned)) == [12, 13]
    assert sum(s["num_vertices"] for s in per) == single.stats()["num_vertices"]
    assert all(s["num_vertices"] > 0 for s in per)


@pytest.mark.parametrize("steps", [1, 2, 3])
@pytest.mark.parametrize("where", ["none", "w<50", "w%7==3||w>=90"])
def test_go_matches_single_and_oracle(rmat14, steps, where):
    src, dst, w, single, orc, c = rmat14
    wx = {"none": None, "w<50": WHERE, "w%7==3||w>=90": WHERE2}[where]
    wb = wx.encode() if wx is not None else b""
    yb = [y.encode() for y in YIELDS]
    for i, r in enumerate(graphs.roots(src, 3, seed=41 + steps)):
        got = graphs.sorted_rows(c.go([r], [1], steps, wb, yb))
        ref = graphs.sorted_rows(single.go([r], [1], steps, wb, yb))
        assert got == ref, (steps, where, r, len(got), len(ref))
        assert c.last_step_stats == single.last_step_stats
        if i == 0:
            assert got == graphs.sorted_rows(orc.go([r], [1], steps, wb, yb))


def test_go_first_hop_slot_exchange(rmat14, monkeypatch):
    """A small first hop (its per-owner edge bound from the degrees every rank holds) is exchanged
    as slot arrays of local ids instead of npad-bit bitmap segments: the rows equal the bitmap
    exchange's (NBG_GO_SLOTS=0) and the single engine's, for single roots (slots), a start list
    with hubs whose bound passes the threshold (bitmaps) and duplicated starts; and a single root's
    first hop moves (G - 1) x 4 x stride bytes per rank instead of (G - 1) x npad / 8."""
    src, dst, w, single, orc, c = rmat14
    wb = WHERE.encode()
    yb = [y.encode() for y in YIELDS]

    def run(starts, steps, slots):
        monkeypatch.setenv("NBG_GO_SLOTS", slots)
        c.each(lambda e: e.profile(True))
        rows = graphs.sorted_rows(c.go(starts, [1], steps, wb, yb))
        prof = c.each(lambda e: e.profile_read())
        c.each(lambda e: e.profile(False))
        return rows, prof[0].get("alltoall(xGMI)", {}).get("algo_bytes", 0)

    small = graphs.roots(src, 6, seed=5)
    cases = [[r] for r in small] + [graphs.roots(src, 200, seed=6), small + small[:2] + [987654321]]
    fewer = 0
    for starts in cases:
        for steps in (2, 3):
            ref = graphs.sorted_rows(single.go(starts, [1], steps, wb, yb))
            bits, bb = run(starts, steps, "0")
            slots, sb = run(starts, steps, "1")
            assert slots == bits == ref, (starts[:3], steps)
            assert sb <= bb
            fewer += sb < bb
    assert fewer >= 6   # (the single roots: their first hop is a slot exchange)


def test_go_multi_start_duplicates_and_unknown(rmat14):
    src, dst, w, single, orc, c = rmat14
    rs = graphs.roots(src, 12, seed=9)
    starts = rs + rs[:3] + [123456789]
    for steps in (1, 3):
        got = graphs.sorted_rows(c.go(starts, [1], steps, WHERE.encode()))
        assert got == graphs.sorted_rows(single.go(starts, [1], steps, WHERE.encode()))


@pytest.mark.parametrize("steps", [1, 2, 3])
def test_go_distinct(rmat14, steps):
    src, dst, w, single, orc, c = rmat14
    wb = WHERE.encode()
    agreed = [e.stats()["host_agreements"] for e in c.engines]
    for yields in ([E.edge_prop("e", "_dst")],
                   [E.edge_prop("e", "w"), E.binop("%", E.edge_prop("e", "_dst"), E.const(7))]):
        yb = [y.encode() for y in yields]
        for r in graphs.roots(src, 2, seed=steps + 70):
            got = graphs.sorted_rows(c.go([r], [1], steps, wb, yb, distinct=True))
            assert got == graphs.sorted_rows(single.go([r], [1], steps, wb, yb, distinct=True)), (steps, r)
            assert len(set(got)) == len(got)
    # statuses in band: no host agreement before a DISTINCT query's first collective
    assert [e.stats()["host_agreements"] for e in c.engines] == agreed


@pytest.mark.parametrize("steps", [1, 2, 3])
def test_go_input_props_backtracker(steps):
    """$-.col after N steps: the roots travel with each hop's exchange over 8 ranks."""
    from tests.test_gpu_go import _forest
    roots, src, dst, w = _forest(seed=11, roots=10)
    c = LocalCluster(100, G)
    c.register_edge(graphs.E_TYPE, "e", graphs.E_SCHEMA)
    c.load_edges(graphs.E_TYPE, src, dst, [w])
    c.finalize()
    orc = graphs.rmat_oracle(src, dst, w)
    try:
        rows = [[r, 1000 + i, 0.5 * i] for i, r in enumerate(roots)]
        inputs = (["id", "tag", "score"], rows, "id")
        yields = [E.input_prop("tag").encode(), E.input_prop("score").encode(), E.edge_prop("e", "_dst").encode()]
        where = E.binop(">", E.input_prop("tag"), E.const(1003)).encode()
        for wb in (b"", where):
            got = c.go(roots, [1], steps, wb, yields, inputs=inputs)
            exp = orc.go(roots, [1], steps, wb, yields, inputs=inputs)
            assert graphs.sorted_rows(got) == graphs.sorted_rows(exp) and got
    finally:
        c.close()
        orc.close()


def test_input_props_roots_travel_packed():
    """The `$-` roots of a hop travel only for the vertices whose bits the hop sends, packed in
    bit order per destination rank: at most twice the bitmap's bytes for these frontiers (they
    were npad * 8 bytes per peer, 64x the bitmap), and the rows equal the oracle's.  (A forest:
    each vertex has one root, so the reference's last-write-wins backtracker has one answer.)"""
    from tests.test_gpu_go import _forest
    roots, src, dst, w = _forest(seed=11, roots=10)
    c = LocalCluster(100, G)
    c.register_edge(graphs.E_TYPE, "e", graphs.E_SCHEMA)
    c.load_edges(graphs.E_TYPE, src, dst, [w])
    c.finalize()
    orc = graphs.rmat_oracle(src, dst, w)
    try:
        inputs = (["id", "tag"], [[r, 7000 + i] for i, r in enumerate(roots)], "id")
        yields = [E.input_prop("tag").encode(), E.edge_prop("e", "_dst").encode()]
        agreed = [e.stats()["host_agreements"] for e in c.engines]
        c.each(lambda e: e.profile(True))
        try:
            got = graphs.sorted_rows(c.go(roots, [1], 3, b"", yields, inputs=inputs))
            profs = c.each(lambda e: e.profile_read())
        finally:
            c.each(lambda e: e.profile(False))
        exp = graphs.sorted_rows(orc.go(roots, [1], 3, b"", yields, inputs=inputs))
        assert len(got) == len(exp) and got, (len(got), len(exp))
        assert got == exp
        bits = sum(p["alltoall(xGMI)"]["algo_bytes"] for p in profs)
        sent = sum(p["alltoallv(roots)"]["algo_bytes"] for p in profs)
        assert all(p["alltoallv(roots)"]["launches"] == 2 for p in profs)   # one per hop
        assert 0 < sent <= 2 * bits, (sent, bits)
        assert [e.stats()["host_agreements"] for e in c.engines] == [a + 1 for a in agreed]   # ($- inputs agree)
    finally:
        c.close()
        orc.close()


def test_go_async_slots_split_communicators(rmat14):
    """More queries in flight than slots on every rank: each slot's collectives run on its own
    communicator (7 peers each); the union of the ranks' rows equals the single engine's."""
    src, dst, w, single, orc, c = rmat14
    wb = WHERE.encode()
    roots = graphs.roots(src, 14, seed=13)

    def run(e):
        stmt = e.prepare_go([graphs.E_TYPE], 3, wb)
        try:
            out = []
            for device in (False, True):
                tickets = [stmt.submit([r], device=device) for r in roots]
                for t in tickets:
                    res = stmt.wait(t)
                    out.append(res.fetch())
                    res.free()
            return out
        finally:
            stmt.free()

    per_rank = c.each(run)
    for i, r in enumerate(roots + roots):
        rows = [row for rk in per_rank for row in rk[i]]
        assert graphs.sorted_rows(rows) == graphs.sorted_rows(single.go([r], [graphs.E_TYPE], 3, wb)), r


def test_go_eval_error_is_global(rmat14):
    src, dst, w, single, orc, c = rmat14
    bad = E.binop("==", E.binop("/", E.edge_prop("e", "w"), E.const(0)), E.const(1)).encode()
    r = graphs.roots(src, 1, seed=3)[0]
    assert _codes(c, lambda e: e.go([r], [1], 2, bad)) == [L.E_EXECUTION_ERROR] * G
    assert graphs.sorted_rows(c.go([r], [1], 2)) == graphs.sorted_rows(single.go([r], [1], 2))


# --------------------------------------------------------------------------- FIND PATH
def test_collective_shortest(rmat14):
    src, dst, w, single, orc, c = rmat14
    assert not c.path_replica_active
    found = 0
    for k, (s, t) in enumerate(rmat.pick_pairs(src, dst, 24, seed=8)):
        for upto in (2, 5):
            st, st1 = {}, {}
            got = c.find_path([s], [t], [1], upto, stats=st)
            assert got == single.find_path([s], [t], [1], upto, stats=st1), (s, t, upto)
            assert st["edges"] == st1["edges"]
            if k < 6:
                assert got == sorted(orc.find_path([s], [t], [1], upto, True, mode=1))
            found += len(got)
    assert found > 0
    ps = rmat.pick_pairs(src, dst, 8, seed=19)
    frm, to = [p[0] for p in ps[:3]], [p[1] for p in ps] + [ps[0][0], 123456789]
    assert c.find_path(frm, to, [1], 4) == single.find_path(frm, to, [1], 4)
    assert c.find_path([123456789], [ps[0][1]], [1], 5) == []


def test_collective_all_paths(rmat14):
    src, dst, w, single, orc, c = rmat14
    total = 0
    for upto in (1, 2, 3):
        for s, t in rmat.pick_pairs(src, dst, 5, seed=30 + upto):
            st, st1 = {}, {}
            got = c.find_path([s], [t], [1], upto, shortest=False, stats=st)
            assert got == single.find_path([s], [t], [1], upto, shortest=False, stats=st1), (s, t, upto)
            assert st["edges"] == st1["edges"]
            total += len(got)
    assert total > 0


def test_replica_over_eight_ranks(rmat14):
    """The replica all-gathered over 8 ranks: every rank answers its own pairs alone, SHORTEST,
    ALL and batched, with the single engine's paths and scanned-edge counts."""
    src, dst, w, single, orc, _ = rmat14
    c = _cluster(src, dst, w, replica=True)
    try:
        assert c.path_replica_active
        pairs = rmat.pick_pairs(src, dst, 48, seed=12)
        res = c.each_indexed(lambda r, e: [(e.find_path([s], [t], [1], 5), e.find_path([s], [t], [1], 3, shortest=False))
                                           for s, t in pairs[r::G]])
        for r in range(G):
            for (s, t), (sp, ap) in zip(pairs[r::G], res[r]):
                assert sp == single.find_path([s], [t], [1], 5), (r, s, t)
                assert ap == single.find_path([s], [t], [1], 3, shortest=False), (r, s, t)
        reqs = [([s], [t], [1], 5, True) for s, t in pairs]
        assert c.engines[G - 1].find_path_batch(reqs) == single.find_path_batch(reqs)
    finally:
        c.close()


@pytest.mark.parametrize("k", [1, 3])
def test_capped_paths(k):
    """FIND PATH under max_edge_returned_per_vertex on 8 ranks (collective capped search) vs the
    faithful oracle, which applies the cap in its storage restatement."""
    from tests.test_gpu_path_capped import mixed_pairs
    src, dst, w = graphs.rmat_graph(11)
    c = _cluster(src, dst, w, max_edge=k)
    orc = graphs.rmat_oracle(src, dst, w, max_edge=k)
    try:
        found = 0
        for s, t in mixed_pairs(orc, src, dst, 8, 5, seed=50 + k):
            got = c.find_path([s], [t], [1], 5)
            assert got == sorted(orc.find_path([s], [t], [1], 5, True, mode=0)), (k, s, t)
            found += len(got)
            got = c.find_path([s], [t], [1], 4, shortest=False)
            assert got == sorted(orc.find_path([s], [t], [1], 4, False, mode=0)), (k, s, t)
        assert found > 0
    finally:
        c.close()
        orc.close()


# --------------------------------------------------------------------------- failing together
def test_failures_agreed_over_eight_ranks(rmat14):
    src, dst, w, single, orc, c = rmat14
    r0 = graphs.roots(src, 1, seed=5)[0]
    wb = WHERE.encode()
    exp = graphs.sorted_rows(single.go([r0], [1], 3, wb))
    for rank in (0, 5, G - 1):
        c.inject_fault(rank, L.FAULT_ALLOC)
        assert _codes(c, lambda e: e.go([r0], [1], 3, wb)) == [L.E_OUT_OF_MEMORY] * G
        assert graphs.sorted_rows(c.go([r0], [1], 3, wb)) == exp
    yd = [E.edge_prop("e", "_dst").encode()]
    c.inject_fault(3, L.FAULT_ALLOC)
    assert _codes(c, lambda e: e.go([r0], [1], 2, wb, yd, distinct=True)) == [L.E_OUT_OF_MEMORY] * G
    assert graphs.sorted_rows(c.go([r0], [1], 2, wb, yd, distinct=True)) == \
        graphs.sorted_rows(single.go([r0], [1], 2, wb, yd, distinct=True))
    s, t = rmat.pick_pairs(src, dst, 1, seed=17)[0]
    c.inject_fault(6, L.FAULT_ALLOC)
    assert _codes(c, lambda e: e.find_path([s], [t], [1], 5)) == [L.E_OUT_OF_MEMORY] * G
    assert c.find_path([s], [t], [1], 5) == single.find_path([s], [t], [1], 5)


def test_device_error_aborts_all_eight():
    src, dst, w = graphs.rmat_graph(11)
    c = _cluster(src, dst, w)
    try:
        r0 = graphs.roots(src, 1, seed=5)[0]
        c.inject_fault(4, L.FAULT_DEVICE)
        assert _codes(c, lambda e: e.go([r0], [1], 3, WHERE.encode())) == [L.E_DEVICE] * G
        assert all(e.lib.nbg_comm_aborted(e.h) == 1 for e in c.engines)
    finally:
        c.close()


# --------------------------------------------------------------------------- a rank with no parts
def test_nba_golden_with_an_empty_rank(nba_data):
    """The 7-part nba space over 8 ranks: rank 0 serves no part (p % 8 for p in 1..7), yet takes
    part in every collective; GoTest and FindPathTest golden cases still pass, and the rank's own
    result share is empty."""
    c = LocalCluster(7, G)
    for (kind, name), cols in kvgen.NBA_SCHEMAS.items():
        if kind == "edge":
            c.register_edge(kvgen.NBA_EDGES[name], name, cols)
        else:
            c.register_tag(kvgen.NBA_TAGS[name], name, cols)
    c.load_builder(kvgen.nba_kv(nba_data, 7))
    orc = nba_oracle(nba_data, 7)
    try:
        assert c.engines[0].stats()["num_vertices"] == 0
        checked = 0
        for case in golden.load("go_golden.json"):
            if golden.unsupported_reason(case):
                continue
            try:
                ok, msg = golden.run_go_case(c, case)
            except NbgError as ex:
                if ex.code == L.E_UNSUPPORTED:
                    continue
                raise
            assert ok, msg
            checked += 1
        assert checked > 0
        for replica in (0, 1):
            c.set_path_replica(replica)
            for case in golden.load("findpath_golden.json"):
                if golden.unsupported_reason(case):
                    continue
                ok, msg = golden.run_path_case(c, case)
                assert ok, (replica, msg)
    finally:
        c.close()
        orc.close()


def test_rmat16_go_and_shortest_digests():
    """RMAT-16 (65 k vertices, 1 M samples): larger frontiers, hub rows spanning many tiles, and
    SHORTEST levels that switch between slot arrays and bitmaps on 8 ranks."""
    src, dst, w = graphs.rmat_graph(16)
    single = graphs.one_sided_engine(src, dst, w)
    c = _cluster(src, dst, w)
    try:
        wb = WHERE.encode()
        for r in graphs.roots(src, 6, seed=2):
            got = graphs.sorted_rows(c.go([r], [1], 3, wb))
            assert got == graphs.sorted_rows(single.go([r], [1], 3, wb)), r
            assert c.last_step_stats == single.last_step_stats
        for s, t in rmat.pick_pairs(src, dst, 24, seed=3):
            st, st1 = {}, {}
            assert c.find_path([s], [t], [1], 5, stats=st) == single.find_path([s], [t], [1], 5, stats=st1)
            assert st["edges"] == st1["edges"]
    finally:
        c.close()
        single.close()


def test_first_hop_slots_with_an_empty_rank(nba_data, monkeypatch):
    """The first-hop slot exchange where rank 0 serves no part (7 parts over 8 ranks): that rank
    runs no MARK, yet sends empty slots in the slot format.  (Round 6's first version set the
    format and the NO_ROW fill inside the MARK: the part-less rank sent its all-zero bitmap, which
    every owner read as its local vertex 0, and 2- and 3-step rows gained those vertices' edges.)
    Rows equal the oracle's with slots and with bitmaps (NBG_GO_SLOTS=0)."""
    from tests.support import ngql
    c = LocalCluster(7, G)
    for (kind, name), cols in kvgen.NBA_SCHEMAS.items():
        if kind == "edge":
            c.register_edge(kvgen.NBA_EDGES[name], name, cols)
        else:
            c.register_tag(kvgen.NBA_TAGS[name], name, cols)
    c.load_builder(kvgen.nba_kv(nba_data, 7))
    orc = nba_oracle(nba_data, 7)
    td, tp = 'hash("Tim Duncan")', 'hash("Tony Parker")'
    qs = [f'GO 2 STEPS FROM {td} OVER like YIELD like._dst',
          f'GO 2 STEPS FROM {td} OVER like YIELD $$.player.name, like._src',
          f'GO 2 STEPS FROM {td} OVER like YIELD DISTINCT left(right($$.player.name, 4), 2) AS f',
          f'GO 3 STEPS FROM {tp} OVER like YIELD like._dst',
          f'GO 2 STEPS FROM {td}, {tp} OVER like WHERE like.likeness > 80 YIELD like._dst, like.likeness']
    try:
        for q in qs:
            want = sorted(tuple(r) for r in ngql.Session(orc).execute(q).rows)
            assert want, q
            for slots in ("1", "0"):
                monkeypatch.setenv("NBG_GO_SLOTS", slots)
                got = sorted(tuple(r) for r in ngql.Session(c).execute(q).rows)
                assert got == want, (slots, q)
    finally:
        c.close()
        orc.close()
