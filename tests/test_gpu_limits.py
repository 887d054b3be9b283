"""The device limits at the C ABI (include/nbg.h "Device limits"), on the MI355X.

Round 6 lifted three shapes the reference answers and the engine used to refuse with
NBG_E_UNSUPPORTED (-1002):
  * `$-` / `$var` input strings absent from the snapshot's dictionary (a string derived by the
    previous statement of a pipe): the statement keeps them in a table of its own (STR_INPUT codes)
    and reads its input string columns as derived strings;
  * YIELD columns and OVER types up to 32 each (16 before);
  * a window / trim / pad over another one's per-edge result, or a pad drawn from one: the inner
    view is materialised into the query's string arena (OP_SMAT) and read back as one piece.
Each lifted shape is compared with the oracle's rows on one engine and on 8 in-process ranks.

What stays is listed in include/nbg.h; every such statement returns NBG_E_UNSUPPORTED, never
rows, so a binding can hand it to the reference's own GoExecutor / FindPathExecutor
(INTEGRATION.md §2).  References: GoExecutor.cpp:197-221 (OVER *), :803-984 (the YIELD loop),
FunctionManager.cpp:249-409 (the string bodies), InterimResult.cpp:158-250 (the input index)."""
import numpy as np
import pytest

from nebula_amd import Engine, LocalCluster, NbgError, _lib as L, kvgen
from nebula_amd.engine import nba_engine
from tests.support import graphs, ngql
from tests.support.oracle import Oracle, OracleError, nba_oracle

pytestmark = pytest.mark.gpu

TD = 'hash("Tim Duncan")'
TP = 'hash("Tony Parker")'


def _run(backend, q):
    try:
        res = ngql.Session(backend).execute(q)
        return sorted(tuple(r) for r in res.rows), None
    except (NbgError, OracleError, ngql.ExecError) as ex:
        return None, ex


def _nba_cluster(nba_data, world, parts=7):
    c = LocalCluster(parts, world)
    for (kind, name), cols in kvgen.NBA_SCHEMAS.items():
        if kind == "edge":
            c.register_edge(kvgen.NBA_EDGES[name], name, cols)
        else:
            c.register_tag(kvgen.NBA_TAGS[name], name, cols)
    c.load_builder(kvgen.nba_kv(nba_data, parts))
    return c


@pytest.fixture(scope="module")
def nba(nba_data):
    eng = nba_engine(nba_data)
    orc = nba_oracle(nba_data)
    c8 = _nba_cluster(nba_data, 8)
    orc7 = nba_oracle(nba_data, 7)
    yield eng, orc, c8, orc7
    eng.close()
    orc.close()
    c8.close()
    orc7.close()


def _parity(nba, q, want_rows=True):
    eng, orc, c8, orc7 = nba
    (rg, eg), (ro, eo) = _run(eng, q), _run(orc, q)
    assert eg is None and eo is None, (q, eg, eo)
    assert rg == ro, (q, rg, ro)
    if want_rows:
        assert rg, q
    (r8, e8), (r7, e7) = _run(c8, q), _run(orc7, q)
    assert e8 is None and e7 is None, (q, e8, e7)
    assert r8 == r7, (q, r8, r7)
    return rg


# ---------------------------------------------------------------- lifted: nested string functions
NESTED = [
    f'GO FROM {TD} OVER like YIELD trim(left($$.player.name, 4)) AS a, ltrim(right(" " + $$.player.name, 5)) AS b',
    f'GO FROM {TD} OVER like YIELD substr(lpad($$.player.name, 20, "-"), 2, 5) AS a',
    f'GO FROM {TD} OVER like YIELD lpad($$.player.name, 20, right($^.player.name, 2)) AS a',
    f'GO FROM {TD}, {TP} OVER like YIELD upper(trim(rpad(left($$.player.name, 3), 6, " b"))) AS a, '
    f'rpad(substr(lower($$.player.name), 2, like.likeness / 20), like.likeness / 8, left($^.player.name, 3)) AS b',
    f'GO FROM {TD}, {TP} OVER like YIELD length(substr(trim(lpad($$.player.name, 25, " ")), 1, 4)) AS n, '
    f'hash(right(left($$.player.name, 6), 2)) AS h, strcasecmp(left(right($$.player.name, 5), 3), "ARK") AS c',
    f'GO FROM {TD}, {TP} OVER like WHERE left(trim("  " + $$.player.name), 3) == "Tim" YIELD $$.player.name',
    f'GO 2 STEPS FROM {TD} OVER like YIELD DISTINCT left(right($$.player.name, 4), 2) AS f',
    f'GO FROM {TD}, {TP} OVER like YIELD left(left(left(left($$.player.name, 9), 7), 5), 3) AS deep, '
    f'(int)substr(rpad((string)like.likeness, 5, "7"), 2, 3) AS k',
]


@pytest.mark.parametrize("q", NESTED)
def test_nested_string_functions_lifted(nba, q):
    _parity(nba, q)


def test_nested_string_function_failures_match(nba):
    """The bodies' own failures under nesting fail on both sides (an inner lpad to a negative
    length, an empty pad drawn from a window)."""
    eng, orc, _, _ = nba
    for q in (f'GO FROM {TD} OVER like YIELD left(lpad($$.player.name, 0 - like.likeness, "x"), 3)',
              f'GO FROM {TD} OVER like YIELD rpad($$.player.name, 40, left($^.player.name, 0))'):
        (rg, eg), (ro, eo) = _run(eng, q), _run(orc, q)
        assert eg is not None and eo is not None, (q, rg, ro)


# ---------------------------------------------------------------- lifted: input strings absent from the dictionary
PIPES = [
    # a derived string piped on: the next statement's $-.nm is not in the dictionary
    f'GO FROM {TD} OVER like YIELD like._dst AS id, $$.player.name + "_x" AS nm | '
    f'GO FROM $-.id OVER like YIELD $-.nm, $-.nm + "!", like._dst',
    f'GO FROM {TD}, {TP} OVER like YIELD like._dst AS id, lower($$.player.name) AS nm, $$.player.name AS pn | '
    f'GO FROM $-.id OVER like WHERE $-.nm > "m" YIELD $-.nm AS a, $-.pn AS b, length($-.nm) AS n, hash($-.nm) AS h',
    f'GO FROM {TD}, {TP} OVER like YIELD like._dst AS id, upper($$.player.name) AS nm | '
    f'GO FROM $-.id OVER like WHERE strcasecmp($-.nm, $$.player.name) != 0 YIELD $-.nm, $$.player.name, '
    f'upper($$.player.name) == $-.nm AS same',
    f'GO FROM {TD} OVER like YIELD like._dst AS id, left($$.player.name, 0) AS e, (string)like.likeness AS s | '
    f'GO FROM $-.id OVER like YIELD $-.e AS e, (int)$-.s + 1 AS k, $-.s + $-.e AS c',
    f'$a = GO FROM {TD}, {TP} OVER like YIELD like._dst AS id, right($$.player.name, 3) AS nm; '
    f'GO FROM $a.id OVER like YIELD DISTINCT $a.nm AS nm, like._dst AS d',
]


@pytest.mark.parametrize("q", PIPES)
def test_input_strings_absent_from_dictionary(nba, q):
    _parity(nba, q)


# ---------------------------------------------------------------- lifted: 32 YIELD columns / OVER types
def test_32_yield_columns(nba):
    cols = ["like._dst", "like.likeness", "$$.player.name", "$^.player.age", "$$.player.age + like.likeness",
            'left($$.player.name, 2)', "like._src", "$$.player.age * 2"]
    q = f'GO FROM {TD}, {TP} OVER like YIELD ' + ", ".join(f"{cols[i % len(cols)]} AS c{i}" for i in range(32))
    rows = _parity(nba, q)
    assert all(len(r) == 32 for r in rows)


def _many_types(nt, parts=7, seed=3):
    """nt edge types e1..e<nt> over 400 vertices, 120 edges each, w in [0, 100)."""
    rng = np.random.default_rng(seed)
    kb = kvgen.KVBuilder(parts)
    verts = [int(v) for v in rng.choice(1 << 30, 400, replace=False)]
    ts = 1_600_000_000_000_000
    for t in range(1, nt + 1):
        for _ in range(120):
            s, d = rng.choice(len(verts), 2)
            kb.insert_edge(verts[s], verts[d], t, 0, graphs.E_SCHEMA, [int(rng.integers(0, 100))], ts)
    return verts, kb


def _register_types(be, nt, is_engine):
    for t in range(1, nt + 1):
        if is_engine:
            be.register_edge(t, f"e{t}", graphs.E_SCHEMA)
        else:
            be.register(True, t, f"e{t}", graphs.E_SCHEMA)


@pytest.fixture(scope="module")
def types24():
    verts, kb = _many_types(24)
    eng = Engine(7)
    _register_types(eng, 24, True)
    eng.load_builder(kb)
    orc = Oracle(7)
    _register_types(orc, 24, False)
    orc.load_builder(kb)
    c8 = LocalCluster(7, 8)
    _register_types(c8, 24, True)
    c8.load_builder(kb)
    yield verts, eng, orc, c8
    eng.close()
    orc.close()
    c8.close()


def test_over_24_types(types24):
    """GO over 24 edge types (OVER * and an explicit list): the default YIELD is one _dst column
    per OVER type (24 columns), a WHERE per type, 2 and 3 steps; FIND SHORTEST PATH OVER *."""
    verts, eng, orc, c8 = types24
    over = ", ".join(f"e{t}" for t in range(1, 25))
    starts = ", ".join(str(v) for v in verts[:6])
    qs = [f"GO FROM {starts} OVER *",
          f"GO 2 STEPS FROM {starts} OVER {over}",
          f"GO 3 STEPS FROM {starts} OVER * WHERE e3.w > 20 || e17.w < 50 YIELD e3._dst, e17._dst, e24.w",
          f"GO 2 STEPS FROM {starts} OVER {over} YIELD DISTINCT e1._dst, e20._dst"]
    total = 0
    for q in qs:
        (rg, eg), (ro, eo) = _run(eng, q), _run(orc, q)
        assert eg is None and eo is None, (q, eg, eo)
        assert rg == ro, q
        (r8, e8) = _run(c8, q)
        assert e8 is None and r8 == ro, (q, e8)
        total += len(rg)
    assert total > 100
    for s, t in zip(verts[:12], verts[12:24]):
        q = f"FIND SHORTEST PATH FROM {s} TO {t} OVER * UPTO 5 STEPS"
        (rg, eg), (ro, eo) = _run(eng, q), _run(orc, q)
        assert eg is None and eo is None and rg == ro, (q, eg, eo)


# ---------------------------------------------------------------- what stays: -1002, never rows
def _unsupported(backend, q):
    rows, ex = _run(backend, q)
    assert rows is None, (q, "returned rows")
    assert isinstance(ex, NbgError) and ex.code == L.E_UNSUPPORTED, (q, ex)


def test_limit_yield_columns(nba):
    eng, _, c8, _ = nba
    q = f'GO FROM {TD} OVER like YIELD ' + ", ".join(f"like._dst AS c{i}" for i in range(33))
    _unsupported(eng, q)
    _unsupported(c8, q)


def test_limit_over_types():
    verts, kb = _many_types(33, seed=4)
    eng = Engine(7)
    _register_types(eng, 33, True)
    eng.load_builder(kb)
    try:
        _unsupported(eng, f"GO FROM {verts[0]} OVER *")
        _unsupported(eng, f"FIND SHORTEST PATH FROM {verts[0]} TO {verts[1]} OVER * UPTO 3 STEPS")
        over = ", ".join(f"e{t}" for t in range(1, 33))   # 32 types: answered
        assert _run(eng, f"GO FROM {verts[0]} OVER {over}")[1] is None
    finally:
        eng.close()


def _balanced_sum(terms):
    while len(terms) > 1:
        terms = [f"({a} + {b})" if b else a for a, b in zip(terms[0::2], terms[1::2] + [None])]
    return terms[0]


def test_limit_program_length_and_registers(nba):
    eng, _, _, _ = nba
    # > 256 instructions (a balanced tree: shallow enough for the expression decoder)
    _unsupported(eng, f'GO FROM {TD} OVER like YIELD ' + _balanced_sum([f"like.likeness * {k}" for k in range(100)]))
    assert _run(eng, f'GO FROM {TD} OVER like YIELD ' + _balanced_sum([f"like.likeness * {k}" for k in range(20)]))[0]
    # more live registers than the device register file holds: 32 columns, the last one deep (a
    # right-leaning tree keeps one more register live per level)
    deep = "like.likeness"
    for k in range(24):
        deep = f"(like.likeness + {k} * ({deep}))"
    cols = ", ".join(f"like.likeness + {i} AS c{i}" for i in range(31))
    _unsupported(eng, f'GO FROM {TD} OVER like YIELD {cols}, {deep} AS last')


def test_limit_steps_and_upto(nba):
    eng, _, _, _ = nba
    _unsupported(eng, f'GO 33 STEPS FROM {TD} OVER like')
    _unsupported(eng, f'FIND SHORTEST PATH FROM {TD} TO {TP} OVER like UPTO 64 STEPS')
    _unsupported(eng, f'FIND ALL PATH FROM {TD} TO {TP} OVER like UPTO 33 STEPS')
    assert _run(eng, f'GO 32 STEPS FROM {TD} OVER like')[1] is None
    assert _run(eng, f'FIND SHORTEST PATH FROM {TD} TO {TP} OVER like UPTO 63 STEPS')[1] is None


def test_limit_dst_tag_index():
    """$$ of a tag registered 17th or later (the per-query holder bits cover 16 tags)."""
    rng = np.random.default_rng(9)
    kb = kvgen.KVBuilder(7)
    ts = 1_600_000_000_000_000
    eng = Engine(7)
    eng.register_edge(1, "e", graphs.E_SCHEMA)
    for k in range(17):
        eng.register_tag(100 + k, f"t{k}", [("x", kvgen.INT)])
    verts = [int(v) for v in rng.choice(1 << 20, 50, replace=False)]
    for v in verts:
        kb.insert_vertex(v, 116, [("x", kvgen.INT)], [v % 7], ts)
        kb.insert_vertex(v, 100, [("x", kvgen.INT)], [v % 5], ts)
    for a, b in zip(verts, verts[1:]):
        kb.insert_edge(a, b, 1, 0, graphs.E_SCHEMA, [1], ts)
    eng.load_builder(kb)
    try:
        _unsupported(eng, f"GO FROM {verts[0]} OVER e YIELD $$.t16.x")
        assert _run(eng, f"GO FROM {verts[0]} OVER e YIELD $$.t0.x")[0] == [(verts[1] % 5,)]
    finally:
        eng.close()


def test_limit_input_columns(nba):
    eng, _, _, _ = nba
    src = ", ".join(f"like._dst AS c{i}" for i in range(33))
    _unsupported(eng, f'GO FROM {TD} OVER like YIELD {src} | GO FROM $-.c0 OVER like YIELD $-.c32')
