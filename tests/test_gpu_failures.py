"""Failure semantics of the partitioned engine (include/nbg.h, "Failure semantics").

The reference keeps a GO / FIND PATH alive when some storaged parts fail and reports the failed
parts (StorageClient.inl:112-136, GoExecutor.cpp:424-442).  A collective engine cannot run a hop
without one of its ranks, so here a failure on ONE rank must fail the query on EVERY rank with
the same code — never leave a peer blocked in a collective — and the engines must keep answering:

  * rank-local failures before the first collective (allocation, a start list over one rank's
    2^32 edge limit) are agreed: same code everywhere, engines still usable;
  * a device error between collectives aborts the communicator: every rank fails (no hang) and
    later queries fail fast.

The ranks are an in-process group on one GPU (nbg_comm_init_local); the 2-process RCCL variant
is tests/test_gpu_rccl.py.  Also: the held-result hand-over (ws_release) keeps the rows and the
workspace when its allocation fails."""
import numpy as np
import pytest

from nebula_amd import LocalCluster, NbgError, _lib as L, expr as E, rmat
from tests.support import graphs

pytestmark = pytest.mark.gpu

WHERE = E.binop("<", E.edge_prop("e", "w"), E.const(50)).encode()


def _codes(c, fn):
    def one(e):
        try:
            fn(e)
            return 0
        except NbgError as ex:
            return ex.code
    return c.each(one)


@pytest.fixture(scope="module")
def graph():
    src, dst, w = graphs.rmat_graph(11)
    single = graphs.rmat_engine(src, dst, w)
    yield src, dst, w, single
    single.close()


def _hub(src, dst):
    """The vertex with the most distinct out-neighbours and that CSR degree (samples repeat)."""
    pairs = np.unique(np.stack([src, dst], axis=1), axis=0)
    ids, deg = np.unique(pairs[:, 0], return_counts=True)
    return int(ids[np.argmax(deg)]), int(deg.max())


def _cluster(src, dst, w, world):
    c = LocalCluster(100, world)
    c.set_path_replica(0)   # FIND PATH failures of the collective search
    c.register_edge(graphs.E_TYPE, "e", graphs.E_SCHEMA)
    c.load_edges(graphs.E_TYPE, src, dst, [w])
    c.finalize()
    return c


@pytest.mark.parametrize("world", [2, 3])
def test_agreed_failures_leave_engines_usable(graph, world):
    src, dst, w, single = graph
    c = _cluster(src, dst, w, world)
    try:
        r0 = graphs.roots(src, 1, seed=5)[0]
        exp = graphs.sorted_rows(single.go([r0], [1], 3, WHERE))
        # (1) an allocation failure on the last rank only, GO
        c.inject_fault(world - 1, L.FAULT_ALLOC)
        assert _codes(c, lambda e: e.go([r0], [1], 3, WHERE)) == [L.E_OUT_OF_MEMORY] * world
        assert graphs.sorted_rows(c.go([r0], [1], 3, WHERE)) == exp
        # (2) a duplicated-hub start list over the owner's 2^32 edge limit: only the hub's owner
        #     sees it, every rank returns E_UNSUPPORTED
        hub, hdeg = _hub(src, dst)
        starts = np.full((1 << 32) // hdeg + 1, hub, dtype=np.int64)
        assert _codes(c, lambda e: e.go(starts, [1], 2)) == [L.E_UNSUPPORTED] * world
        assert graphs.sorted_rows(c.go([r0], [1], 3, WHERE)) == exp
        # (3) asynchronous submission: the failing rank's submit fails; its peers' statuses arrive
        #     with the query's statistics, so their wait fails with the same code; the next runs
        c.inject_fault(0, L.FAULT_ALLOC)

        def submit_twice(e):
            st = e.prepare_go([1], 3, WHERE)
            try:
                try:
                    st.wait(st.submit([r0], device=False)).free()
                    first = 0
                except NbgError as ex:
                    first = ex.code
                res = st.wait(st.submit([r0], device=False))
                rows = res.fetch()
                res.free()
                return first, rows
            finally:
                st.free()
        out = c.each(submit_twice)
        assert [o[0] for o in out] == [L.E_OUT_OF_MEMORY] * world
        assert graphs.sorted_rows([r for o in out for r in o[1]]) == exp
        # (3b) YIELD DISTINCT: its failures travel in band too (the statistics, then the owner
        #      exchange's counts), with no agreement round trip of their own
        yd = [E.edge_prop("e", "_dst").encode()]
        exp_d = graphs.sorted_rows(single.go([r0], [1], 2, WHERE, yd, distinct=True))
        c.inject_fault(world - 1, L.FAULT_ALLOC)
        assert _codes(c, lambda e: e.go([r0], [1], 2, WHERE, yd, distinct=True)) == [L.E_OUT_OF_MEMORY] * world
        assert graphs.sorted_rows(c.go([r0], [1], 2, WHERE, yd, distinct=True)) == exp_d
        # (4) FIND PATH: an allocation failure on rank 0, then a normal request
        s, t = rmat.pick_pairs(src, dst, 1, seed=17)[0]
        c.inject_fault(0, L.FAULT_ALLOC)
        assert _codes(c, lambda e: e.find_path([s], [t], [1], 5)) == [L.E_OUT_OF_MEMORY] * world
        assert c.find_path([s], [t], [1], 5) == single.find_path([s], [t], [1], 5)
    finally:
        c.close()


def test_device_error_between_collectives_aborts_every_rank(graph):
    """A device error after the query's first collective on rank 1: rank 1 aborts the group, rank
    0's next collective fails at once (no wait for the timeout), both report E_DEVICE, and the
    aborted engines fail later queries fast instead of hanging."""
    src, dst, w, single = graph
    c = _cluster(src, dst, w, 2)
    try:
        r0 = graphs.roots(src, 1, seed=5)[0]
        c.inject_fault(1, L.FAULT_DEVICE)
        assert _codes(c, lambda e: e.go([r0], [1], 3, WHERE)) == [L.E_DEVICE] * 2
        assert all(e.lib.nbg_comm_aborted(e.h) == 1 for e in c.engines)
        assert _codes(c, lambda e: e.go([r0], [1], 3, WHERE)) == [L.E_DEVICE] * 2
    finally:
        c.close()


def test_host_exception_on_one_rank_releases_its_peers(graph):
    """A host-side exception on one rank (not an engine status) while its peer is already inside
    a collective: LocalCluster aborts the group, so the peer returns instead of blocking forever
    (the r02_h session that never printed its summary)."""
    src, dst, w, single = graph
    c = _cluster(src, dst, w, 2)
    try:
        r0 = graphs.roots(src, 1, seed=5)[0]

        def fn(i, e):
            if i == 0:
                raise RuntimeError("host-side failure on rank 0")
            return e.go([r0], [1], 3, WHERE)
        with pytest.raises(RuntimeError):
            c.each_indexed(fn)
        assert c.engines[1].lib.nbg_comm_aborted(c.engines[1].h) == 1
    finally:
        c.close()


def test_duplicated_start_list_longer_than_the_graph(graph):
    """GO keeps duplicated starts (GoExecutor.cpp:101-107): a start list whose edge space exceeds
    every CSR's edge count (but not 2^32) runs — the workspace's merge-path tiles grow to cover
    it — and its rows are the hub's rows repeated."""
    src, dst, w, single = graph
    hub, hdeg = _hub(src, dst)
    reps = 3 * len(src) // hdeg
    assert reps * hdeg > len(src)
    eng = graphs.rmat_engine(src, dst, w)
    try:
        one = graphs.sorted_rows(eng.go([hub], [1], 1, WHERE))
        got = graphs.sorted_rows(eng.go([hub] * reps, [1], 1, WHERE))
        assert got == graphs.sorted_rows(one * reps)
        # two steps: the per-step SET makes the duplicates irrelevant after step 1
        assert graphs.sorted_rows(eng.go([hub] * reps, [1], 2)) == graphs.sorted_rows(single.go([hub], [1], 2))
    finally:
        eng.close()


def test_held_result_handover_failure_keeps_rows_and_workspace(graph):
    """ws_release: when the fresh workspace for the next query cannot be allocated, the held
    device rows stay valid, the query fails with E_OUT_OF_MEMORY, and once the rows are freed the
    engine answers again (no null workspace left behind)."""
    src, dst, w, single = graph
    eng = graphs.rmat_engine(src, dst, w)
    try:
        r0 = graphs.roots(src, 1, seed=5)[0]
        exp = graphs.sorted_rows(single.go([r0], [1], 3, WHERE))
        held = eng.go_device([r0], [1], 3, WHERE)
        assert held.count == len(exp)
        eng._check(eng.lib.nbg_inject_fault(eng.h, L.FAULT_ALLOC, 1), "inject")
        with pytest.raises(NbgError) as ex:
            eng.go([r0], [1], 3, WHERE)
        assert ex.value.code == L.E_OUT_OF_MEMORY
        assert graphs.sorted_rows(held.fetch()) == exp   # the held rows are intact
        assert graphs.sorted_rows(eng.go([r0], [1], 3, WHERE)) == exp
        held.free()
        s, t = rmat.pick_pairs(src, dst, 1, seed=17)[0]
        assert eng.find_path([s], [t], [1], 5) == single.find_path([s], [t], [1], 5)
    finally:
        eng.close()
