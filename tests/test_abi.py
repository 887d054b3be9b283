"""CPU-side checks of the C ABI: the library loads, exports every symbol include/nbg.h declares,
and the host-only calls (schemas, loading) behave without a GPU."""
import os
import re

import numpy as np
import pytest

from nebula_amd import _lib, kvgen
from nebula_amd.engine import Engine, NbgError

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    with open(os.path.join(ROOT, "include", "nbg.h")) as f:
        src = f.read()
    return sorted(set(re.findall(r"\b(nbg_[a-z_]+)\s*\(", src)))


def test_header_symbols_exported():
    L = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 25
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing


def test_signatures_cover_header():
    declared = {n for n, _, _ in _lib.SIGNATURES}
    assert set(header_symbols()) == declared


def test_create_register_load_without_gpu():
    e = Engine(num_parts=3)
    e.register_edge(1, "e", [("w", kvgen.INT)])
    e.register_tag(2, "t", [("name", kvgen.STRING)])
    kb = kvgen.KVBuilder(3)
    kb.insert_edge(1, 2, 1, 0, [("w", kvgen.INT)], [5], 1)
    for p in sorted(kb.recs):
        e.load_part(p, *kb.flat(p))
    e.load_edges(1, np.array([3, 4]), np.array([4, 5]), [np.array([1, 2])])
    # querying before finalize is a state error, not a crash
    with pytest.raises(NbgError) as ex:
        e.go([1], [1], 1)
    assert ex.value.code == _lib.E_STATE
    e.close()


def test_invalid_config_rejected():
    with pytest.raises(NbgError):
        Engine(num_parts=0)
    with pytest.raises(NbgError):
        Engine(num_parts=4, num_gpus=2, rank=2)


def test_bulk_load_rejects_unknown_type():
    e = Engine(num_parts=1)
    with pytest.raises(NbgError) as ex:
        e.load_edges(9, np.array([1]), np.array([2]))
    assert ex.value.code == _lib.E_EDGE_PROP_NOT_FOUND


def test_over_all_default_column_order():
    """OVER * without YIELD: columns follow the response edge_schema map's iteration order
    (GoExecutor.cpp:481-499); for the nba types serve=4, like=5 that is like, serve — what
    GoTest.cpp:437-448 expects ({0, team} rows).  Engine (host-only ABI) and oracle agree."""
    from tests.support.oracle import Oracle
    e = Engine(num_parts=1)
    o = Oracle(1)
    try:
        assert e.default_columns([4, 5], over_all=True) == [5, 4]
        assert e.default_columns([4, 5], over_all=False) == [4, 5]
        for types in ([1], [1, 2, 3], [2, 7, 9, 30], list(range(1, 20))):
            assert e.default_columns(types, True) == o.default_columns(types, True), types
    finally:
        e.close()
        o.close()


def test_find_path_batch_arguments_without_gpu():
    """nbg_find_path_batch: an empty batch is a no-op; missing arrays are invalid arguments; every
    request of a batch on an engine that is not finalized fails with NBG_E_STATE in its own status."""
    import ctypes as C
    e = Engine(num_parts=3)
    e.register_edge(1, "e", [("w", kvgen.INT)])
    try:
        assert e.find_path_batch([]) == []
        assert e.lib.nbg_find_path_batch(e.h, None, 2, None, None) == _lib.E_INVALID_ARGUMENT
        res = e.find_path_batch([([1], [2], [1], 5, True), ([1], [3], [1], 3, False)])
        assert [r.code for r in res] == [_lib.E_STATE, _lib.E_STATE]
    finally:
        e.close()
