"""String semantics of WHERE / YIELD on columns on the MI355X vs the oracle.

The reference evaluates `string + string` (Expressions.cpp:858-860) and TypeCasting between
strings and numbers (Expressions.cpp:773-793, Expression::toInt / toDouble / toString,
Expressions.h:274-321) on any value, columns included; FunctionCallExpression runs
FunctionManager's bodies (udf_is_in, FunctionManager.cpp:440-486; abs/floor/ceil/round/sqrt).
The device evaluates them with dictionary-backed piece lists (exprc.cpp emit_pieces,
kernels.hip run_program), per-string toInt/toDouble tables, and a content-hashed string arena
for derived YIELD values; the oracle (oracle/expr.cpp) with real strings.  Every query is run on
both through the nGQL front end; rows are compared as sorted multisets, and a query that fails
must fail on both."""
import pytest

from nebula_amd import Engine, LocalCluster, NbgError, kvgen
from tests.support import ngql
from nebula_amd.engine import nba_engine
from tests.support.oracle import Oracle, OracleError, nba_oracle

pytestmark = pytest.mark.gpu

TD = 'hash("Tim Duncan")'
NBA_QUERIES = [
    # concatenation in YIELD: constant + column, column + column, nested, with ints cast to string
    f'GO FROM {TD} OVER like YIELD $^.player.name + "!" AS a',
    f'GO FROM {TD} OVER like YIELD $^.player.name + " likes " + $$.player.name AS a, like.likeness',
    f'GO FROM {TD} OVER like YIELD $$.player.name + (string)$$.player.age AS a',
    f'GO FROM {TD} OVER like YIELD (string)like.likeness + "%" AS a, (string)($$.player.age > 40) AS b',
    f'GO FROM {TD} OVER serve YIELD $$.team.name + "@" + (string)serve.start_year AS a',
    f'GO 2 STEPS FROM {TD} OVER like YIELD $^.player.name + "->" + $$.player.name AS a',
    # concatenation in WHERE: equality, ordering, asBool (empty()) of a derived string
    f'GO FROM {TD} OVER like WHERE $$.player.name + "" == "Tony Parker" YIELD like._dst',
    f'GO FROM {TD} OVER like WHERE $^.player.name + $$.player.name == "Tim DuncanManu Ginobili" '
    f'YIELD $$.player.name',
    f'GO 2 STEPS FROM {TD} OVER like WHERE $$.player.name + "z" > "Tony" YIELD $$.player.name',
    f'GO 2 STEPS FROM {TD} OVER like WHERE $$.player.name + "" <= "Manu Ginobili" YIELD $$.player.name',
    f'GO FROM {TD} OVER like WHERE $$.player.name + "" YIELD like._dst',
    f'GO FROM {TD} OVER like WHERE !($$.player.name + "") YIELD like._dst',
    f'GO FROM {TD} OVER like WHERE (string)like.likeness == "95" YIELD $$.player.name',
    f'GO FROM {TD} OVER like WHERE (string)like.likeness + "0" > "900" YIELD $$.player.name',
    # casts of strings to numbers
    f'GO FROM {TD} OVER like YIELD (int)((string)like.likeness + "1") AS a, '
    f'(double)((string)$$.player.age + ".5") AS b',
    f'GO FROM {TD} OVER like YIELD (int)$$.player.name',                       # not a number: fails
    f'GO FROM {TD} OVER like YIELD (double)($$.player.name + "1")',            # fails
    f'GO FROM {TD} OVER like YIELD (bool)($$.player.name + "")',
    # YIELD DISTINCT over derived strings (one code per string, whatever made it)
    f'GO 2 STEPS FROM {TD} OVER like YIELD DISTINCT $$.player.name + "!" AS a',
    f'GO 2 STEPS FROM {TD} OVER like, serve YIELD DISTINCT like._dst + 0 AS d, '
    f'(string)serve.start_year + "" AS y',
    # FunctionManager: udf_is_in over every comparand kind, the exact math functions
    f'GO FROM {TD} OVER like WHERE udf_is_in(like.likeness, 90, 95.0, "80") YIELD $$.player.name',
    f'GO FROM {TD} OVER serve WHERE udf_is_in($$.team.name, "Hawks", "Spurs", 7) YIELD $$.team.name',
    f'GO FROM {TD} OVER like WHERE udf_is_in($$.player.name + "", "Tony Parker") YIELD $$.player.name',
    f'GO FROM {TD} OVER like WHERE udf_is_in((string)like.likeness, 95, "96") YIELD like.likeness',
    f'GO FROM {TD} OVER like WHERE udf_is_in($$.player.age > 30, true) YIELD $$.player.age',
    f'GO FROM {TD} OVER like WHERE udf_is_in(1.0 * $$.player.age, 36, $$.player.age) YIELD $$.player.age',
    f'GO FROM {TD} OVER like YIELD udf_is_in(like.likeness, $$.player.age, 95) AS i',
    f'GO FROM {TD} OVER like YIELD abs(like.likeness - 100) AS a, floor(like.likeness / 7.0) AS f, '
    f'ceil(like.likeness / 7.0) AS c, round(like.likeness / 2.0) AS r, sqrt(like.likeness) AS s',
    f'GO FROM {TD} OVER like YIELD abs($$.player.name)',                        # asDouble of a string
]


def _run(backend, q):
    try:
        res = ngql.Session(backend).execute(q)
        return sorted(tuple(r) for r in res.rows), None
    except (NbgError, OracleError, ngql.ExecError) as ex:
        return None, ex


def _same(got, exp, q):
    (rg, eg), (ro, eo) = got, exp
    assert (eg is None) == (eo is None), (q, eg, eo)
    assert rg == ro, (q, rg, ro)


@pytest.fixture(scope="module")
def nba(nba_data):
    eng = nba_engine(nba_data)
    orc = nba_oracle(nba_data)
    yield eng, orc
    eng.close()
    orc.close()


@pytest.mark.parametrize("q", NBA_QUERIES)
def test_nba_string_semantics(nba, q):
    eng, orc = nba
    _same(_run(eng, q), _run(orc, q), q)


def test_nba_string_semantics_return_rows(nba):
    """Guard against the comparison passing because both sides failed: most queries return rows."""
    eng, orc = nba
    ok = sum(1 for q in NBA_QUERIES if _run(eng, q)[0])
    assert ok >= len(NBA_QUERIES) - 6   # (3 fail on purpose, 2 select no row)


def test_partitioned_string_semantics(nba_data):
    """The same queries on 3 ranks: derived strings stay with their rows, and YIELD DISTINCT
    (rows exchanged between ranks) all-gathers the arenas' texts."""
    c = LocalCluster(7, 3)
    for (kind, name), cols in kvgen.NBA_SCHEMAS.items():
        if kind == "edge":
            c.register_edge(kvgen.NBA_EDGES[name], name, cols)
        else:
            c.register_tag(kvgen.NBA_TAGS[name], name, cols)
    c.load_builder(kvgen.nba_kv(nba_data, 7))
    orc = nba_oracle(nba_data, 7)
    try:
        for q in NBA_QUERIES:
            _same(_run(c, q), _run(orc, q), q)
    finally:
        c.close()
        orc.close()


# --------------------------------------------------------------------------- numbers in strings
ITEM, REL = 21, 22
ITEM_S = [("code", kvgen.STRING), ("f", kvgen.DOUBLE)]
REL_S = [("s", kvgen.STRING), ("n", kvgen.INT)]
TEXTS = ["12", "-7", " 42", "3.5", "1e3", "abc", "", "+8", "99999999999999999999", "0x10", "7 ", "-0", ".5",
         "5.", "1e", "-2.25e-2", "  -9.75", "9223372036854775807", "-9223372036854775808", "1.0e22", "12e21"]


SLOW_DOUBLE = {"99999999999999999999", "0x10", "9223372036854775807", "-9223372036854775808", "-2.25e-2",
               "1.0e22", "12e21", "1e3"}


def _numbers_kv(parts):
    kb = kvgen.KVBuilder(parts)
    now = 1_600_000_000_000_000
    for i, t in enumerate(TEXTS):
        kb.insert_vertex(100 + i, ITEM, ITEM_S, [t, 0.25 * i], now)
        kb.insert_edge(1, 100 + i, REL, 0, REL_S, [t, i], now)
    return kb


def _numbers(parts, cluster=None):
    if cluster:
        be = LocalCluster(parts, cluster)
    else:
        be = Engine(parts)
    be.register_tag(ITEM, "item", ITEM_S)
    be.register_edge(REL, "rel", REL_S)
    be.load_builder(_numbers_kv(parts))
    orc = Oracle(parts)
    orc.register(False, ITEM, "item", ITEM_S)
    orc.register(True, REL, "rel", REL_S)
    orc.load_builder(_numbers_kv(parts))
    return be, orc


@pytest.mark.parametrize("expr", ["(int)rel.s", "(double)rel.s", "(int)$$.item.code", "(double)$$.item.code",
                                  "(int)(rel.s + \"\")", "(double)(\"\" + rel.s)", "(int)(rel.s + \"0\")",
                                  "(double)(rel.s + \"5\")", "rel.s + $$.item.code", "(bool)(rel.s + \"\")",
                                  "udf_is_in(rel.n, rel.s, \"3\")"])
def test_string_number_casts_per_row(expr):
    """One row at a time (WHERE rel.n == i), so each text's conversion is compared on its own:
    the value, or an evaluation error on both sides.  A DERIVED string cast to DOUBLE is parsed
    on the device by the exact fast path only (at most 19 significant digits, the
    value m * 10^e with m < 2^53 and |e| <= 22); texts outside it (longer mantissas, hex) are
    left out of that comparison — a dictionary string's cast reads the host's strtod table."""
    eng, orc = _numbers(3)
    derived_double = expr.startswith("(double)(")
    try:
        for i in range(len(TEXTS)):
            if derived_double and TEXTS[i] in SLOW_DOUBLE:
                continue
            q = f"GO FROM 1 OVER rel WHERE rel.n == {i} YIELD {expr} AS v"
            _same(_run(eng, q), _run(orc, q), q)
    finally:
        eng.close()
        orc.close()


def test_string_number_casts_partitioned():
    c, orc = _numbers(5, cluster=2)
    try:
        for expr in ("(int)rel.s", "(double)rel.s", "rel.s + \"|\" + $$.item.code"):
            for i in range(len(TEXTS)):
                q = f"GO FROM 1 OVER rel WHERE rel.n == {i} YIELD {expr} AS v"
                _same(_run(c, q), _run(orc, q), q)
    finally:
        c.close()
        orc.close()


def test_arena_overflow_fails_cleanly(monkeypatch):
    """A result whose derived strings exceed the arena fails with E_OUT_OF_MEMORY (nothing is
    truncated), and the engine answers the next query."""
    import subprocess
    import sys
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = (
        "import sys; sys.path.insert(0, %r)\n"
        "from tests.test_gpu_strings import _numbers, _run\n"
        "from nebula_amd import NbgError, _lib\n"
        "eng, orc = _numbers(3)\n"
        "big = ' + '.join(['rel.s'] * 8)\n"
        "q = 'GO FROM 1 OVER rel YIELD ' + ' , '.join([big] * 4)\n"
        "from tests.support import ngql\n"
        "try:\n"
        "    ngql.Session(eng).execute(q)\n"
        "    print('NO-ERROR')\n"
        "except NbgError as ex:\n"
        "    print('CODE', ex.code)\n"
        "r, e = _run(eng, 'GO FROM 1 OVER rel WHERE rel.n == 0 YIELD rel.s + \"x\"')\n"
        "print('NEXT', r)\n" % root)
    env = dict(os.environ, NBG_STR_ARENA_KB="4")
    p = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True, text=True, timeout=120)
    assert "CODE -1004" in p.stdout and "NEXT [('12x',)]" in p.stdout, p.stdout + p.stderr


def test_long_derived_strings_of_a_large_result():
    """Derived strings longer than 16 bytes over a result far above 1 MB: the arena is
    sized from each program's bound on its pieces' text (ProgramBuilder::sout_bytes), so a hub's
    40,000 rows of ~60-byte concatenations fit, equal to the oracle's."""
    parts = 3
    kb = kvgen.KVBuilder(parts)
    now = 1_600_000_000_000_000
    n = 40000
    for i in range(n):
        kb.insert_edge(1, 1000 + i, REL, 0, REL_S, ["x" * 24 + str(i), i], now)
    eng = Engine(parts)
    eng.register_edge(REL, "rel", REL_S)
    eng.load_builder(kb)
    orc = Oracle(parts)
    orc.register(True, REL, "rel", REL_S)
    orc.load_builder(kb)
    try:
        q = 'GO FROM 1 OVER rel YIELD rel.s + "/" + rel.s AS a, (string)rel.n + rel.s AS b'
        got, exp = _run(eng, q), _run(orc, q)
        _same(got, exp, q)
        assert len(got[0]) == n and sum(len(a) + len(b) for a, b in got[0]) > (3 << 20)
    finally:
        eng.close()
        orc.close()
