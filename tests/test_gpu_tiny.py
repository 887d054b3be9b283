"""The single-launch path for tiny GO queries (kernels.hip k_go_tiny, engine.cpp go_launch).

A GO N STEPS (N <= 3, one OVER type, rows fetched to the host) whose walk bound — W_N of its
starts, DevEdgeType::h_w2 / h_w3 — fits one workgroup runs as ONE launch: per-step sets in LDS,
WHERE / YIELD through the interpreter, results stored straight into mapped host memory.  It must
return what the multi-launch path returns: the same rows as the oracle (GoExecutor semantics,
GoExecutor.cpp:410-474, 501-541) and the same per-step statistics as the same query left in HBM
(nbg_go_device, which never takes the tiny path)."""
import pytest

from nebula_amd import expr as E, rmat
from tests.support import golden, graphs
from tests.support.oracle import nba_oracle

pytestmark = pytest.mark.gpu


def _tiny_count(eng):
    return eng.stats()["tiny_queries"]


@pytest.fixture(scope="module")
def rmat12():
    src, dst, w = graphs.rmat_graph(12)
    eng = graphs.rmat_engine(src, dst, w)
    orc = graphs.rmat_oracle(src, dst, w)
    yield src, eng, orc
    eng.close()
    orc.close()


WHERES = {
    "none": b"",
    "w<50": E.binop("<", E.edge_prop("e", "w"), E.const(50)).encode(),
    "w/0": E.binop("==", E.binop("/", E.edge_prop("e", "w"), E.const(0)), E.const(1)).encode(),   # eval error
}
YIELDS = [E.edge_prop("e", "_src").encode(), E.edge_prop("e", "_dst").encode(), E.edge_prop("e", "w").encode(),
          E.binop("+", E.edge_prop("e", "w"), E.edge_prop("e", "_rank")).encode()]


@pytest.mark.parametrize("steps", [1, 2, 3])
@pytest.mark.parametrize("where", list(WHERES))
def test_tiny_matches_oracle_and_device_path(rmat12, steps, where):
    src, eng, orc = rmat12
    wb = WHERES[where]
    tried = tiny = 0
    for r in graphs.roots(src, 200, seed=steps):
        before = _tiny_count(eng)
        try:
            got = graphs.sorted_rows(eng.go([r], [1], steps, wb, YIELDS))
            err = None
        except Exception as ex:   # the eval-error case: both paths and the oracle fail
            got, err = None, ex
        if _tiny_count(eng) == before:
            continue   # not tiny: covered by every other GO test
        tiny += 1
        stats = eng.last_step_stats
        try:
            exp = graphs.sorted_rows(orc.go([r], [1], steps, wb, YIELDS))
        except Exception:
            exp = None
        assert (got is None) == (exp is None), (r, steps, where, err)
        assert got == exp, (r, steps, where)
        if got is not None:
            dev = eng.go_device([r], [1], steps, wb, YIELDS)
            try:
                assert graphs.sorted_rows(dev.fetch()) == got
                assert dev.step_stats() == tuple(stats[:2]), (r, steps)
                assert dev.edges_scanned == stats[2]
            finally:
                dev.free()
        tried += 1
        if tried >= 12:
            break
    assert tiny > 0


def test_tiny_multi_start_duplicates(rmat12):
    src, eng, orc = rmat12
    rs = [r for r in graphs.roots(src, 400, seed=9)]
    small = []
    for r in rs:
        before = _tiny_count(eng)
        eng.go([r], [1], 2)
        if _tiny_count(eng) > before:
            small.append(r)
        if len(small) == 4:
            break
    starts = small + small[:2] + [123456789]
    before = _tiny_count(eng)
    got = graphs.sorted_rows(eng.go(starts, [1], 2, WHERES["w<50"], YIELDS))
    assert got == graphs.sorted_rows(orc.go(starts, [1], 2, WHERES["w<50"], YIELDS))
    assert _tiny_count(eng) >= before   # (the summed bound decides)


def test_tiny_tag_props(nba_data):
    """$^ / $$ props, the holder's "Unknown Vertex" rule and string columns on the nba space: the
    reference's GoTest golden cases, most of them tiny, vs their expected rows."""
    from nebula_amd.engine import nba_engine
    eng = nba_engine(nba_data)
    orc = nba_oracle(nba_data)
    try:
        before = _tiny_count(eng)
        for case in golden.load("go_golden.json"):
            if golden.unsupported_reason(case):
                continue
            ok, msg = golden.run_go_case(eng, case)
            assert ok, (case["query"], msg)
        assert _tiny_count(eng) > before
    finally:
        eng.close()
        orc.close()


def test_tiny_c1_query(nba_data):
    """BASELINE configs[0]: GO 2 STEPS FROM "Tim Duncan" OVER like, one launch."""
    from nebula_amd import kvgen
    from nebula_amd.engine import nba_engine
    from nebula_amd.vidhash import std_hash
    eng = nba_engine(nba_data)
    orc = nba_oracle(nba_data)
    try:
        like = kvgen.NBA_EDGES["like"]
        tim = std_hash("Tim Duncan")
        stmt = eng.prepare_go([like], 2)
        before = _tiny_count(eng)
        rows = stmt.run([tim])
        stmt.free()
        assert _tiny_count(eng) == before + 1
        assert graphs.sorted_rows(rows) == graphs.sorted_rows(orc.go([tim], [like], 2)) and rows
    finally:
        eng.close()
        orc.close()
