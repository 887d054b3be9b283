"""GO N STEPS parity on the MI355X: nebula_amd (libnbg.so, gfx950 kernels) vs the CPU oracle
on the same inputs — reference golden cases (nba dataset) and seeded RMAT graphs.  Bit-exact:
rows are compared as sorted multisets (TestBase::verifyResult semantics)."""
import numpy as np
import pytest

from nebula_amd import NbgError, expr as E, kvgen, nba_engine
from nebula_amd import _lib
from tests.support import golden, graphs
from tests.support.oracle import nba_oracle

pytestmark = pytest.mark.gpu

GO = golden.load("go_golden.json")


@pytest.fixture(scope="module")
def nba(nba_data):
    eng = nba_engine(nba_data)
    yield eng
    eng.close()


@pytest.mark.parametrize("case", GO, ids=[f"{c['test']}-{i}" for i, c in enumerate(GO)])
def test_go_golden_on_gpu(nba, case):
    why = golden.unsupported_reason(case)
    if why:
        pytest.skip(why)
    try:
        ok, msg = golden.run_go_case(nba, case)
    except NbgError as ex:
        if ex.code == _lib.E_UNSUPPORTED:
            pytest.skip(f"not on the device path yet: {ex}")
        raise
    assert ok, msg


@pytest.fixture(scope="module")
def rmat12():
    src, dst, w = graphs.rmat_graph(12)
    eng = graphs.rmat_engine(src, dst, w)
    orc = graphs.rmat_oracle(src, dst, w)
    yield src, eng, orc
    eng.close()
    orc.close()


WHERES = {
    "none": None,
    "w<50": E.binop("<", E.edge_prop("e", "w"), E.const(50)),
    "w%7==3||w>=90": E.binop("||", E.binop("==", E.binop("%", E.edge_prop("e", "w"), E.const(7)), E.const(3)),
                             E.binop(">=", E.edge_prop("e", "w"), E.const(90))),
    "w*1.5>=60.0": E.binop(">=", E.binop("*", E.edge_prop("e", "w"), E.const(1.5)), E.const(60.0)),
}


@pytest.mark.parametrize("steps", [1, 2, 3])
@pytest.mark.parametrize("where", list(WHERES))
def test_rmat_go_parity(rmat12, steps, where):
    src, eng, orc = rmat12
    starts = graphs.roots(src, 4, seed=steps)
    w = WHERES[where]
    wb = w.encode() if w is not None else b""
    yields = [E.edge_prop("e", "_dst").encode(), E.edge_prop("e", "w").encode(),
              E.edge_prop("e", "_src").encode()]
    got = eng.go(starts, [1], steps, wb, yields)
    exp = orc.go(starts, [1], steps, wb, yields)
    assert len(got) == len(exp)
    assert graphs.sorted_rows(got) == graphs.sorted_rows(exp)


def test_small_results_packed_at_query_end(rmat12):
    """Results of at most 32 k cells are packed into host memory by the end-of-query kernel (one
    round trip), larger ones are fetched after it: rows from both sides of the bound equal the
    oracle's, through nbg_go (host rows) and through a device result fetched later."""
    src, eng, orc = rmat12
    yields = [E.edge_prop("e", "_dst").encode(), E.edge_prop("e", "w").encode(),
              E.edge_prop("e", "_src").encode()]
    wb = WHERES["w<50"].encode()
    small = big = 0
    stmt = eng.prepare_go([1], 2, wb, yields)
    try:
        for r in graphs.roots(src, 24, seed=11):
            exp = graphs.sorted_rows(orc.go([r], [1], 2, wb, yields))
            assert graphs.sorted_rows(eng.go([r], [1], 2, wb, yields)) == exp, r
            res = stmt.run_device([r])
            try:
                assert graphs.sorted_rows(res.fetch()) == exp, r
            finally:
                res.free()
            if len(exp) * len(yields) <= 32768:
                small += 1
            else:
                big += 1
    finally:
        stmt.free()
    assert small and big, (small, big)


def test_rmat_go_each_root(rmat12):
    """GO 3 STEPS with WHERE from 16 single roots (one query each), default YIELD."""
    src, eng, orc = rmat12
    wb = WHERES["w<50"].encode()
    for r in graphs.roots(src, 16, seed=42):
        got = eng.go([r], [1], 3, wb)
        exp = orc.go([r], [1], 3, wb)
        assert graphs.sorted_rows(got) == graphs.sorted_rows(exp), r


def test_duplicate_and_unknown_starts(rmat12):
    src, eng, orc = rmat12
    r = graphs.roots(src, 2, seed=5)
    starts = [r[0], r[0], 123456789, r[1]]
    for steps in (1, 2):
        assert graphs.sorted_rows(eng.go(starts, [1], steps)) == graphs.sorted_rows(orc.go(starts, [1], steps))
    assert eng.go([], [1], 2) == []
    assert eng.go([987654321], [1], 3) == []


def test_kv_and_bulk_loaders_agree():
    src, dst, w = graphs.rmat_graph(9)
    a = graphs.rmat_engine(src, dst, w, parts=7)
    b = graphs.rmat_engine(src, dst, w, parts=7, via_kv=True)
    assert a.stats()["num_edges"] == b.stats()["num_edges"]
    for r in graphs.roots(src, 6):
        assert graphs.sorted_rows(a.go([r], [1], 2, yields=[E.edge_prop("e", "w").encode()])) == \
               graphs.sorted_rows(b.go([r], [1], 2, yields=[E.edge_prop("e", "w").encode()]))


def test_max_edge_returned_per_vertex():
    src, dst, w = graphs.rmat_graph(10)
    eng = graphs.rmat_engine(src, dst, w, max_edge=3)
    orc = graphs.rmat_oracle(src, dst, w, max_edge=3)
    for r in graphs.roots(src, 5):
        for steps in (1, 2, 3):
            assert graphs.sorted_rows(eng.go([r], [1], steps)) == graphs.sorted_rows(orc.go([r], [1], steps))


def test_eval_error_fails_query(rmat12):
    """Integer division by zero in WHERE fails the whole query (GoExecutor.cpp:950-953)."""
    src, eng, orc = rmat12
    bad = E.binop(">", E.binop("/", E.const(10), E.binop("-", E.edge_prop("e", "w"), E.edge_prop("e", "w"))),
                  E.const(1))
    r = graphs.roots(src, 1)
    with pytest.raises(NbgError) as ex:
        eng.go(r, [1], 1, bad.encode())
    assert ex.value.code == _lib.E_EXECUTION_ERROR


def test_device_rows_stay_in_hbm(rmat12):
    src, eng, orc = rmat12
    r = graphs.roots(src, 3)
    dev = eng.go_device(r, [1], 3, WHERES["w<50"].encode())
    n = dev.count
    assert dev.device_col(0) != 0 or n == 0
    rows = dev.fetch()
    assert len(rows) == n
    assert graphs.sorted_rows(rows) == graphs.sorted_rows(orc.go(r, [1], 3, WHERES["w<50"].encode()))
    dev.free()


def test_prepared_statements_interleaved(rmat12):
    """GoExecutor prepare/execute split: two prepared statements with interpreter (generic)
    programs run alternately from inline (<= 32) and long start lists; rows equal the oracle's."""
    src, eng, orc = rmat12
    w1 = WHERES["w*1.5>=60.0"].encode()
    w2 = WHERES["w%7==3||w>=90"].encode()
    ys = [E.edge_prop("e", "_src").encode(), E.binop("+", E.edge_prop("e", "w"), E.const(1)).encode()]
    s1 = eng.prepare_go([1], 2, w1, ys)
    s2 = eng.prepare_go([1], 3, w2)
    roots = graphs.roots(src, 40, seed=21)
    for k in range(3):
        starts = roots[: 1 + 19 * k]          # 1, 20, 39 starts: inline and copied start lists
        got1 = graphs.sorted_rows(s1.run(starts))
        got2 = graphs.sorted_rows(s2.run(starts))
        assert got1 == graphs.sorted_rows(orc.go(starts, [1], 2, w1, ys))
        assert got2 == graphs.sorted_rows(orc.go(starts, [1], 3, w2))
    s1.free()
    s2.free()


def test_device_rows_segments_cover_count(rmat12):
    src, eng, orc = rmat12
    stmt = eng.prepare_go([1], 3, WHERES["w<50"].encode())
    r = graphs.roots(src, 1, seed=2)[0]
    res = stmt.run_device([r])
    n = eng.lib.nbg_rows_num_segments(res.h)
    spans = []
    for i in range(n):
        b, e = _lib.u64(), _lib.u64()
        assert eng.lib.nbg_rows_segment(res.h, i, b, e) == 0
        spans.append((b.value, e.value))
    spans.sort()
    assert sum(e - b for b, e in spans) == res.count
    assert all(spans[i][1] <= spans[i + 1][0] for i in range(len(spans) - 1))
    assert len(res.fetch()) == res.count
    res.free()
    stmt.free()


@pytest.mark.parametrize("scale_w", [(-1, -50), (300, 0), (70000, 0), (10 ** 12, -7)])
def test_narrow_int_columns(scale_w):
    """The final-step fast path reads INT columns at their narrowest width (1/2/4/8 bytes,
    sign-extended): values spanning each width, WHERE range tests and YIELD of the column."""
    mul, add = scale_w
    src, dst, w = graphs.rmat_graph(10)
    w2 = w * mul + add
    eng = graphs.rmat_engine(src, dst, w2)
    orc = graphs.rmat_oracle(src, dst, w2)
    try:
        mid = int(np.median(w2))
        ys = [E.edge_prop("e", "_dst").encode(), E.edge_prop("e", "w").encode()]
        for op in ("<", "<=", ">", ">=", "==", "!="):
            wh = E.binop(op, E.edge_prop("e", "w"), E.const(mid)).encode()
            for r in graphs.roots(src, 2, seed=13):
                got = graphs.sorted_rows(eng.go([r], [1], 2, wh, ys))
                assert got == graphs.sorted_rows(orc.go([r], [1], 2, wh, ys)), (op, mul, add)
    finally:
        eng.close()
        orc.close()


def test_async_submit_wait_parity(rmat12):
    """nbg_go_submit / nbg_go_wait: queries in flight on the query slots (more than there are
    slots, waited for out of order) return exactly the synchronous results."""
    src, eng, orc = rmat12
    wb = WHERES["w<50"].encode()
    stmt = eng.prepare_go([1], 3, wb)
    roots = graphs.roots(src, 11, seed=9)
    try:
        tickets = [stmt.submit([r], device=False) for r in roots]
        order = list(range(len(roots)))[::-1]   # newest first: older tickets complete inside
        got = {}
        for i in order:
            res = stmt.wait(tickets[i])
            got[i] = (res.count, res.edges_scanned, graphs.sorted_rows(res.fetch()))
            res.free()
        for i, r in enumerate(roots):
            exp = graphs.sorted_rows(orc.go([r], [1], 3, wb))
            assert got[i][2] == exp, r
            assert got[i][0] == len(exp)
    finally:
        stmt.free()


def test_async_device_rows_outlive_slot_reuse(rmat12):
    """Device tickets: more submissions than query slots, every result held (not freed) while
    later queries reuse the slots; each result's rows stay intact (the slot's workspace is handed
    to the live result) and equal the oracle's.  Also the synchronous device path: a held
    nbg_go_device result survives later queries on the engine's own workspace."""
    src, eng, orc = rmat12
    wb = WHERES["w<50"].encode()
    stmt = eng.prepare_go([1], 2, wb)
    roots = graphs.roots(src, 14, seed=19)
    held = []
    try:
        tickets = [stmt.submit([r], device=True) for r in roots]
        held = [stmt.wait(t) for t in tickets]
        sync = [stmt.run_device([r]) for r in roots[:3]]
        for r, res in zip(roots, held):
            exp = graphs.sorted_rows(orc.go([r], [1], 2, wb))
            assert res.count == len(exp)
            assert graphs.sorted_rows(res.fetch()) == exp, r
        for r, res in zip(roots[:3], sync):
            assert graphs.sorted_rows(res.fetch()) == graphs.sorted_rows(orc.go([r], [1], 2, wb)), r
        held += sync
    finally:
        for res in held:
            res.free()
        stmt.free()


def test_c1_go_2_steps_nba(nba, nba_data):
    """BASELINE configs[0] (C1): GO 2 STEPS FROM "Tim Duncan" OVER like (the `follow` edge of
    later releases is this reference's `like`) — device vs the oracle, plus
    YIELD variants on the same hop pattern."""
    from tests.support import ngql
    from nebula_amd.vidhash import std_hash
    orc = nba_oracle(nba_data)
    try:
        tim = std_hash("Tim Duncan")
        for q in (f"GO 2 STEPS FROM {tim} OVER like",
                  f"GO 2 STEPS FROM {tim} OVER like YIELD like._dst, like.likeness, $$.player.name",
                  f"GO 2 STEPS FROM {tim} OVER like WHERE like.likeness >= 90 YIELD like._src, like._dst",
                  f"GO 2 STEPS FROM {tim} OVER *"):
            got = ngql.Session(nba).execute(q)
            exp = ngql.Session(orc).execute(q)
            assert got.columns == exp.columns, q
            assert golden.rows_match(got.rows, exp.rows), q
            assert got.rows, q
    finally:
        orc.close()


def _forest(seed=3, roots=6, depth=4, fan=4):
    """A forest (every vertex has one parent): a final row's root is unique, so the reference's
    VertexBackTracker (last write wins over unordered responses) is deterministic on it."""
    rng = np.random.default_rng(seed)
    src, dst = [], []
    level = [int(x) for x in rng.choice(1 << 40, roots, replace=False)]
    all_roots = list(level)
    nxt = 1 << 41
    for _ in range(depth):
        new = []
        for v in level:
            for _ in range(int(rng.integers(1, fan + 1))):
                nxt += int(rng.integers(1, 1000))
                src.append(v)
                dst.append(nxt)
                new.append(nxt)
        level = new
    w = rng.integers(0, 100, len(src))
    return all_roots, np.array(src, np.int64), np.array(dst, np.int64), w.astype(np.int64)


@pytest.mark.parametrize("steps", [1, 2, 3])
def test_input_props_backtracker(steps):
    """$-.col in YIELD / WHERE after N steps: the root's input row (GoExecutor::getPropFromInterim,
    VertexBackTracker) — device MARKB roots vs the oracle."""
    roots, src, dst, w = _forest()
    eng = graphs.rmat_engine(src, dst, w, parts=7)
    orc = graphs.rmat_oracle(src, dst, w, parts=7)
    try:
        # input rows: (id, name-like int, score) with a duplicated id (the last row wins)
        rows = [[r, 1000 + i, 0.5 * i] for i, r in enumerate(roots)] + [[roots[0], 7, 9.25]]
        inputs = (["id", "tag", "score"], rows, "id")
        yields = [E.input_prop("tag").encode(), E.input_prop("score").encode(), E.edge_prop("e", "_dst").encode()]
        where = E.binop(">", E.input_prop("tag"), E.const(1001)).encode()
        for wb in (b"", where):
            got = eng.go(roots, [1], steps, wb, yields, inputs=inputs)
            exp = orc.go(roots, [1], steps, wb, yields, inputs=inputs)
            assert graphs.sorted_rows(got) == graphs.sorted_rows(exp) and got
        bad = [E.input_prop("nosuch").encode()]
        with pytest.raises(NbgError):
            eng.go(roots, [1], steps, b"", bad, inputs=inputs)
    finally:
        eng.close()
        orc.close()


def test_snapshot_save_load_roundtrip(tmp_path):
    """nbg_snapshot_save / nbg_snapshot_load: a reloaded engine answers GO (tag props, ranks,
    two types), GetNeighbors and FIND PATH exactly like the engine that built the snapshot."""
    from nebula_amd import Engine
    src, persons, eng, orc = graphs.tagged_pair(9)
    path = str(tmp_path / "snap.nbg")
    try:
        eng.snapshot_save(path)
        re = Engine(7)
        re.snapshot_load(path)
        ps = set(persons)
        starts = [r for r in graphs.roots(src, 40, seed=2) if r in ps][:5]
        ys = [E.edge_prop("e", "_dst").encode(), E.dst_prop("person", "name").encode(),
              E.edge_prop("f", "_rank").encode()]
        for steps in (1, 2, 3):
            if steps == 1:   # the starts are persons: $^ is defined
                ys = ys + [E.src_prop("person", "age").encode()]
            a = graphs.sorted_rows(eng.go(starts, [1, 2], steps, b"", ys))
            b = graphs.sorted_rows(re.go(starts, [1, 2], steps, b"", ys))
            assert a == b and a
            ys = ys[:3]
        assert eng.find_path(starts[:2], starts[2:], [1, 2], 4) == re.find_path(starts[:2], starts[2:], [1, 2], 4)
        pvs = [(kvgen.part_of(v, 7), v) for v in starts]
        rets = [(3, 1, "_dst"), (3, 1, "w"), (1, graphs.T_PERSON, "name")]
        assert eng.get_neighbors(pvs, [1, 2], b"", rets) == re.get_neighbors(pvs, [1, 2], b"", rets)
        assert eng.stats()["num_edges"] == re.stats()["num_edges"]
        re.close()
        # a snapshot of another partitioning is rejected
        other = Engine(5)
        with pytest.raises(NbgError):
            other.snapshot_load(path)
        other.close()
    finally:
        eng.close()
        orc.close()
