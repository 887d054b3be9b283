"""The rest of FunctionManager (src/common/filter/FunctionManager.cpp:20-437) over per-edge values
on the MI355X, against the oracle's restatement (oracle/expr.cpp callFunction).

Constant calls fold on the host with the reference's bodies (ExpressionTest's FunctionCall /
StringFunctionCall vectors: tests/test_gpu_expr.py).  Here the arguments are columns, so the
device ops run: the double math (OP_MATH1_F / OP_MATH2_F), hash over ints, doubles, bools and
strings (libstdc++'s _Hash_bytes restated on the device), length and strcasecmp over dictionary
strings and derived piece lists, rand32 / rand64 and now, and the string-valued bodies (lower,
upper, trim, ltrim, rtrim, left, right, lpad, rpad, substr) as views over piece lists.

Tolerance: integer, string and hash results must be equal; the exactly rounded functions (sqrt,
abs, floor, ceil, round) bit-exact; the transcendental ones (cbrt, exp, exp2, log*, trig, pow,
hypot) within 4 ulps of glibc's value — gtest's ASSERT_DOUBLE_EQ, the tolerance the reference's
own ExpressionTest applies to them.  rand32 / rand64 are random in the reference too: checked by
their ranges; now() by the wall clock."""
import math
import time

import pytest

from nebula_amd import LocalCluster, NbgError, _lib as L, kvgen
from tests.support import ngql
from nebula_amd.engine import nba_engine
from tests.support.golden import _ulps_equal
from tests.support.oracle import OracleError, nba_oracle

pytestmark = pytest.mark.gpu

TD = 'hash("Tim Duncan")'
TP = 'hash("Tony Parker")'

EXACT = [
    f'GO FROM {TD}, {TP} OVER like YIELD hash(like.likeness) AS h, hash(like.likeness * 1.5) AS d, '
    f'hash(like.likeness > 90) AS b, hash(like.likeness * 0.0) AS z',
    f'GO FROM {TD}, {TP} OVER like YIELD hash($$.player.name) AS h, hash($^.player.name + "/" + $$.player.name) AS j',
    f'GO 2 STEPS FROM {TD} OVER like YIELD hash((string)like.likeness) AS h, hash($$.player.name + "") AS e',
    f'GO FROM {TD}, {TP} OVER like YIELD length($$.player.name) AS n, length($^.player.name + $$.player.name) AS m, '
    f'length((string)like.likeness) AS k',
    f'GO FROM {TD}, {TP} OVER like YIELD strcasecmp($$.player.name, "tony parker") AS a, '
    f'strcasecmp($$.player.name, $^.player.name) AS b, strcasecmp("MANU GINOBILI", $$.player.name + "") AS c',
    f'GO FROM {TD} OVER serve YIELD strcasecmp($$.team.name, "spurs") AS a, length($$.team.name) AS n',
    f'GO FROM {TD}, {TP} OVER like WHERE length($$.player.name) > 11 YIELD $$.player.name',
    f'GO FROM {TD}, {TP} OVER like WHERE strcasecmp($$.player.name, "TONY PARKER") == 0 YIELD like._dst',
    f'GO FROM {TD}, {TP} OVER like WHERE hash($$.player.name) == {TP} YIELD $$.player.name',
    f'GO FROM {TD}, {TP} OVER like YIELD sqrt(like.likeness) AS s, abs(0 - like.likeness) AS a, '
    f'floor(like.likeness / 7.0) AS f, ceil(like.likeness / 7.0) AS c, round(like.likeness / 8.0) AS r',
    # kinds the bodies reject (boost::bad_get): the query fails on both
    f'GO FROM {TD} OVER like YIELD length(like.likeness)',
    f'GO FROM {TD} OVER like YIELD strcasecmp($$.player.name, 3)',
    f'GO FROM {TD} OVER like YIELD cbrt($$.player.name)',
    f'GO FROM {TD} OVER like YIELD pow(like.likeness, $$.player.name)',
    f'GO FROM {TD} OVER like YIELD rand32(1.5 * like.likeness)',
]

APPROX = [
    f'GO FROM {TD}, {TP} OVER like YIELD cbrt(like.likeness) AS a, exp(like.likeness / 50.0) AS b, '
    f'exp2(like.likeness / 10.0) AS c, log(like.likeness) AS d, log2(like.likeness) AS e, log10(like.likeness) AS f',
    f'GO FROM {TD}, {TP} OVER like YIELD sin(like.likeness) AS a, asin(like.likeness / 100.0) AS b, '
    f'cos(like.likeness) AS c, acos(like.likeness / 100.0) AS d, tan(like.likeness) AS e, atan(like.likeness) AS f',
    f'GO FROM {TD}, {TP} OVER like YIELD pow(like.likeness, 2) AS a, pow(1.5, like.likeness / 10.0) AS b, '
    f'hypot(like.likeness, 3) AS c, hypot(sin(like.likeness), cos(like.likeness)) AS d',
    f'GO 2 STEPS FROM {TD} OVER like WHERE sqrt(pow(like.likeness, 2)) >= 90 YIELD like.likeness AS l, '
    f'log(like.likeness) AS g',
]


def _run(backend, q):
    try:
        res = ngql.Session(backend).execute(q)
        return sorted(tuple(r) for r in res.rows), None
    except (NbgError, OracleError, ngql.ExecError) as ex:
        return None, ex


@pytest.fixture(scope="module")
def nba(nba_data):
    eng = nba_engine(nba_data)
    orc = nba_oracle(nba_data)
    yield eng, orc
    eng.close()
    orc.close()


@pytest.mark.parametrize("q", EXACT)
def test_functions_exact(nba, q):
    eng, orc = nba
    (rg, eg), (ro, eo) = _run(eng, q), _run(orc, q)
    assert (eg is None) == (eo is None), (q, eg, eo)
    assert rg == ro, (q, rg, ro)
    if eg is None:
        assert rg, q


@pytest.mark.parametrize("q", APPROX)
def test_functions_within_4_ulps(nba, q):
    eng, orc = nba
    (rg, eg), (ro, eo) = _run(eng, q), _run(orc, q)
    assert eg is None and eo is None, (q, eg, eo)
    assert len(rg) == len(ro) > 0, q
    # rows sorted by their values; a value differs by a few ulps at most, so pair rows by order
    for a, b in zip(rg, ro):
        for x, y in zip(a, b):
            if isinstance(x, float):
                assert (math.isnan(x) and math.isnan(y)) or _ulps_equal(x, y), (q, a, b)
            else:
                assert x == y, (q, a, b)


def test_rand_ranges_and_now(nba):
    """rand32(max) in [0, max), rand32(min, max) in [min, max), rand64 likewise, per row; now() is
    the query's wall-clock second."""
    eng, _ = nba
    s = ngql.Session(eng)
    q = (f'GO 2 STEPS FROM {TD} OVER like WHERE like.likeness > 20 YIELD like.likeness AS l, rand32(like.likeness) AS a, '
         f'rand32(10, like.likeness) AS b, rand64(like.likeness) AS c, rand64(-5, like.likeness) AS d, '
         f'rand32() AS e, now() AS t')
    t0 = int(time.time())
    rows = s.execute(q).rows
    t1 = int(time.time())
    assert rows
    for l, a, b, c, d, e, t in rows:
        assert 0 <= a < l and 10 <= b < l and 0 <= c < l and -5 <= d < l, (l, a, b, c, d)
        assert -2**31 <= e < 2**31
        assert t0 <= t <= t1
    assert len({r[1] for r in rows}) > 1   # a value per row
    kept = s.execute(f'GO FROM {TD} OVER like WHERE now() > 1554716753 YIELD like._dst').rows
    assert len(kept) == len(s.execute(f'GO FROM {TD} OVER like').rows)


# the string-valued bodies over per-edge values (FunctionManager.cpp:249-409): PC_VIEW pieces of a
# derived string, in WHERE, YIELD and under other string ops (length, hash, strcasecmp, compare,
# concatenation, DISTINCT); the bodies' failures (asInt / asString of the wrong kind, a negative
# or pad-less padding) fail the query on both sides
STRING_FNS = [
    f'GO FROM {TD}, {TP} OVER like YIELD lower($$.player.name) AS a, upper($^.player.name) AS b, '
    f'(string)upper((string)like.likeness) AS c',
    f'GO FROM {TD}, {TP} OVER like YIELD left($$.player.name, 3) AS a, (string)right($$.player.name, like.likeness / 10) AS b, '
    f'left($$.player.name, 0) AS c, right($$.player.name, 100) AS d, left($^.player.name, -2) AS e',
    f'GO FROM {TD}, {TP} OVER like YIELD substr($$.player.name, 2, 4) AS a, substr($$.player.name, -3, 2) AS b, '
    f'substr($$.player.name, 0, 1) AS c, substr($$.player.name, 100, 1) AS d, substr($$.player.name, 1, -1) AS e, '
    f'substr($$.player.name, -100, 3) AS f, (string)substr($$.player.name, like.likeness / 20, like.likeness / 30) AS g',
    f'GO FROM {TD}, {TP} OVER like YIELD lpad($$.player.name, 20, "*-") AS a, (string)rpad($$.player.name, like.likeness / 5, "ab") AS b, '
    f'lpad($$.player.name, 3, "x") AS c, rpad($^.player.name, 0, "") AS d, lpad($$.player.name, like.likeness / 4, $^.player.name) AS e',
    f'GO FROM {TD}, {TP} OVER like YIELD trim("  " + $$.player.name + "   ") AS a, ltrim(" " + $$.player.name + " ") AS b, '
    f'rtrim(" " + $$.player.name + " ") AS c, trim("   ") AS d, trim(lower(" a B ")) AS e, '
    f'ltrim("  " + $^.player.name) AS f',
    f'GO FROM {TD}, {TP} OVER like YIELD (int)length(upper($$.player.name)) AS a, (int)hash(lower($$.player.name)) AS b, '
    f'(int)strcasecmp(upper($$.player.name), lower($$.player.name)) AS c, lower($^.player.name) + "->" + upper($$.player.name) AS d',
    f'GO FROM {TD}, {TP} OVER like WHERE lower($$.player.name) == "tony parker" YIELD $$.player.name',
    f'GO FROM {TD}, {TP} OVER like WHERE left($$.player.name, 1) < "M" YIELD $$.player.name, left($$.player.name, 1) AS f',
    f'GO 2 STEPS FROM {TD} OVER like YIELD DISTINCT left($$.player.name, 1) AS f, upper(right($^.player.name, 2)) AS g',
    f'GO FROM {TD}, {TP} OVER like YIELD (int)substr((string)like.likeness, 1, 1) AS a, '
    f'(double)rpad((string)like.likeness, 4, "5") AS b',
    f'GO FROM {TD} OVER serve YIELD upper($$.team.name) AS a, (string)lpad((string)serve.start_year, 6, "#") AS b',
    # case maps composed with the other functions (a case map commutes with windows and trims)
    f'GO FROM {TD}, {TP} OVER like YIELD lower(upper($$.player.name) + "X") AS a, trim(lower(" " + $$.player.name + " ")) AS b, '
    f'lpad(upper($$.player.name), 15, "ab") AS c, upper(lpad($$.player.name, 15, "ab")) AS d, '
    f'lower(left($^.player.name, 4) + right($$.player.name, 4)) AS e',
    # the bodies' failures
    f'GO FROM {TD} OVER like YIELD lpad($$.player.name, 0 - like.likeness, "x")',
    f'GO FROM {TD} OVER like YIELD rpad($$.player.name, 40, "")',
    f'GO FROM {TD} OVER like YIELD left($$.player.name, "3")',
    f'GO FROM {TD} OVER like YIELD lower(like.likeness)',
    f'GO FROM {TD} OVER like YIELD substr($$.player.name, 1.5, 2)',
    f'GO FROM {TD} OVER like YIELD lpad($$.player.name, 12, 7)',
]


@pytest.mark.parametrize("q", STRING_FNS)
def test_string_functions_on_columns(nba, q):
    eng, orc = nba
    (rg, eg), (ro, eo) = _run(eng, q), _run(orc, q)
    assert (eg is None) == (eo is None), (q, eg, eo)
    assert rg == ro, (q, rg, ro)


def test_string_functions_on_columns_return_rows(nba):
    """Guard against the comparison passing because both sides failed: the first 12 return rows."""
    eng, _ = nba
    assert all(_run(eng, q)[0] for q in STRING_FNS[:12])


def test_string_functions_partitioned(nba_data):
    """Three ranks: the views travel with their rows (and through YIELD DISTINCT's exchange)."""
    c = LocalCluster(7, 3)
    for (kind, name), cols in kvgen.NBA_SCHEMAS.items():
        if kind == "edge":
            c.register_edge(kvgen.NBA_EDGES[name], name, cols)
        else:
            c.register_tag(kvgen.NBA_TAGS[name], name, cols)
    c.load_builder(kvgen.nba_kv(nba_data, 7))
    orc = nba_oracle(nba_data, 7)
    try:
        for q in STRING_FNS[:12]:
            (rg, eg), (ro, eo) = _run(c, q), _run(orc, q)
            assert eg is None and eo is None and rg == ro, (q, eg, eo)
    finally:
        c.close()
        orc.close()


def test_nested_string_functions_on_columns(nba):
    """A window, trim or pad over another window, trim or pad of a per-edge string (round 6: the
    inner view is materialised into the arena, OP_SMAT) equals the oracle; over constants any
    nesting folds.  tests/test_gpu_limits.py covers more shapes, on 8 ranks too."""
    eng, orc = nba
    for q in (f'GO FROM {TD} OVER like YIELD trim(left($$.player.name, 4))',
              f'GO FROM {TD} OVER like YIELD substr(lpad($$.player.name, 20, "-"), 2, 5)',
              f'GO FROM {TD} OVER like YIELD lpad($$.player.name, 20, right($^.player.name, 2))',
              f'GO FROM {TD} OVER like YIELD trim(left(" Abc ", 3)) AS a, $$.player.name'):
        (rg, eg), (ro, eo) = _run(eng, q), _run(orc, q)
        assert eg is None and eo is None and rg == ro and rg, (q, eg, eo)
