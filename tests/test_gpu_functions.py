"""The rest of FunctionManager (src/common/filter/FunctionManager.cpp:20-437) over per-edge values
on the MI355X, against the oracle's restatement (oracle/expr.cpp callFunction).

Constant calls fold on the host with the reference's bodies (ExpressionTest's FunctionCall /
StringFunctionCall vectors: tests/test_gpu_expr.py).  Here the arguments are columns, so the
device ops run: the double math (OP_MATH1_F / OP_MATH2_F), hash over ints, doubles, bools and
strings (libstdc++'s _Hash_bytes restated on the device), length and strcasecmp over dictionary
strings and derived piece lists, rand32 / rand64 and now.

Tolerance: integer, string and hash results must be equal; the exactly rounded functions (sqrt,
abs, floor, ceil, round) bit-exact; the transcendental ones (cbrt, exp, exp2, log*, trig, pow,
hypot) within 4 ulps of glibc's value — gtest's ASSERT_DOUBLE_EQ, the tolerance the reference's
own ExpressionTest applies to them.  rand32 / rand64 are random in the reference too: checked by
their ranges; now() by the wall clock."""
import math
import time

import pytest

from nebula_amd import NbgError, _lib as L, ngql
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


def test_string_valued_functions_on_columns_unsupported(nba):
    """lower / upper / trim / left / right / lpad / rpad / substr fold over constants; over
    per-edge strings the engine says so (NBG_E_UNSUPPORTED) rather than return other values."""
    eng, _ = nba
    with pytest.raises(NbgError) as ei:
        ngql.Session(eng).execute(f'GO FROM {TD} OVER like YIELD lower($$.player.name)')
    assert ei.value.code == L.E_UNSUPPORTED
