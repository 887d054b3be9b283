"""The host's wake-up at the end of a query (DESIGN.md §5 "Host wake-up"): by default a
synchronous GO query, getNeighbors and a SHORTEST chain end with the end kernel storing a sequence
number into a mapped word the host polls; NBG_WAKE=event restores the wait on the event behind
the end kernel.  Both must return the same results: the same queries run here (the mapped word)
and in a child process with NBG_WAKE=event (the setting is read once per process), and on the
wake-word side also against the CPU oracle; NBG_BLOCKING_SYNC=1 (blocking waits) likewise."""
import json
import os
import subprocess
import sys

import pytest

from nebula_amd import expr as E
from tests.support import graphs

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WB = E.binop("<", E.edge_prop("e", "w"), E.const(50)).encode()
YIELDS = [E.edge_prop("e", "_dst").encode(), E.edge_prop("e", "w").encode()]


def run_queries(eng, src, orc=None):
    """GO through nbg_go (host rows: the small-row pack), a device result fetched later (the
    one-workgroup end kernel), submitted queries (the event wait) and SHORTEST pairs (the chain's
    wake word, continuation batches included): results as comparable strings."""
    out = {"go": [], "dev": [], "sub": [], "sp": []}
    rs = graphs.roots(src, 12, seed=3)
    for r in rs:
        rows = graphs.sorted_rows(eng.go([r], [1], 2, WB, YIELDS))
        if orc is not None:
            assert rows == graphs.sorted_rows(orc.go([r], [1], 2, WB, YIELDS)), r
        out["go"].append(repr(rows))
    stmt = eng.prepare_go([1], 3, WB, YIELDS)
    try:
        for r in rs[:6]:
            res = stmt.run_device([r])
            try:
                out["dev"].append(repr(graphs.sorted_rows(res.fetch())))
            finally:
                res.free()
        tickets = [stmt.submit([r]) for r in rs[6:]]
        for tk in tickets:
            res = stmt.wait(tk)
            try:
                out["sub"].append(repr(graphs.sorted_rows(res.fetch())))
            finally:
                res.free()
    finally:
        stmt.free()
    for i in range(0, len(rs) - 1, 2):
        out["sp"].append(repr(eng.find_path([rs[i]], [rs[i + 1]], [1], 5)))
    return out


def _child():
    src, dst, w = graphs.rmat_graph(12)
    eng = graphs.rmat_engine(src, dst, w)
    try:
        print(json.dumps(run_queries(eng, src)))
    finally:
        eng.close()


@pytest.mark.parametrize("var,val", [("NBG_WAKE", "event"), ("NBG_BLOCKING_SYNC", "1")])
def test_event_wait_matches_wake_word(var, val):
    """The child waits on events (polled, or blocking with NBG_BLOCKING_SYNC)."""
    src, dst, w = graphs.rmat_graph(12)
    eng = graphs.rmat_engine(src, dst, w)
    orc = graphs.rmat_oracle(src, dst, w)
    try:
        mine = run_queries(eng, src, orc)
    finally:
        eng.close()
        orc.close()
    env = dict(os.environ, **{var: val})
    p = subprocess.run([sys.executable, "-c", "from tests.test_gpu_wake import _child; _child()"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    theirs = json.loads(p.stdout.strip().splitlines()[-1])
    assert sum(len(v) for v in mine.values()) > 20
    for k in mine:
        assert mine[k] == theirs[k], k
