"""Helpers to run the reference's golden GO / FIND PATH cases against a backend."""
from __future__ import annotations

import json
import os

from tests.support import ngql

GOLDEN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "golden")

# Cases whose features are outside the hot path this build covers (documented in DESIGN.md).
UNSUPPORTED = (
    ("REVERSELY", "REVERSELY is rejected by the reference GoExecutor (GoExecutor.cpp:243-246)"),
)


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def unsupported_reason(case):
    q = case["query"]
    for pat, why in UNSUPPORTED:
        if pat == "$-." and "$-." in q:
            # `FROM $-.id` is supported; only $- in YIELD/WHERE is not
            tail = q.split("|")[-1]
            after_from = tail.split("OVER", 1)[-1]
            if "$-." in after_from:
                return why
            continue
        if pat in q:
            return why
    if case.get("test", "").startswith("DISABLED_"):
        return "disabled in the reference test suite"
    return None


def norm(v):
    if isinstance(v, bool):
        return int(v)
    return v


def rows_match(got, expected):
    """TestBase::verifyResult (src/graph/test/TestBase.h:182-223): the rows as a sorted multiset,
    every column in its own position."""
    g = sorted((tuple(norm(x) for x in r) for r in got), key=repr)
    e = sorted((tuple(norm(x) for x in r) for r in expected), key=repr)
    return g == e


def run_go_case(backend, case):
    s = ngql.Session(backend)
    if case.get("expect_error"):
        try:
            s.execute(case["query"])
        except Exception:
            return True, "failed as expected"
        return False, "expected an error"
    res = s.execute(case["query"])
    if "col_names" in case and res.columns != case["col_names"]:
        return False, f"columns {res.columns} != {case['col_names']}"
    ok = rows_match(res.rows, case.get("expected", []))
    return ok, "" if ok else f"rows {res.rows} != {case.get('expected')}"


def run_path_case(backend, case):
    s = ngql.Session(backend)
    res = s.execute(case["query"])
    names = backend.edge_names
    got = sorted(ngql.path_string(r[0], names) for r in res.rows)
    exp = sorted(case["expected"])
    return got == exp, "" if got == exp else f"{got} != {exp}"


# ------------------------------------------------------------------- ExpressionTest.cpp vectors
EXPR_ROOT = 'hash("Tim Duncan")'   # two `like` edges: every case yields two equal rows


def expr_queries(case):
    """The GO statements one ExpressionTest vector runs as (WHERE and YIELD)."""
    e = case["expr"]
    return (f"GO FROM {EXPR_ROOT} OVER like WHERE {e} YIELD like._dst AS d",
            f"GO FROM {EXPR_ROOT} OVER like YIELD {e} AS v")


def run_expr_case(backend, case):
    """(ok, message): the WHERE keeps both edges iff the value is true; the YIELD value equals
    the test's expected value (ASSERT_DOUBLE_EQ: within 4 ulps); invalid expressions fail."""
    import math
    s = ngql.Session(backend)
    where_q, yield_q = expr_queries(case)
    if case.get("error"):
        for q in (where_q, yield_q):
            try:
                s.execute(q)
            except Exception:
                continue
            return False, f"{q!r} did not fail"
        return True, "failed as expected"
    rows = s.execute(where_q).rows
    exp = case["expect"]
    # Expression::asBool (Expressions.h:228-242): a string is "true" when it is EMPTY
    truthy = bool(exp) if case["kind"] != "String" else exp == ""
    if len(rows) != (2 if truthy else 0):
        return False, f"WHERE kept {len(rows)} rows"
    vals = [r[0] for r in s.execute(yield_q).rows]
    if len(vals) != 2:
        return False, f"YIELD gave {vals}"
    for v in vals:
        if case["kind"] == "Double":
            if not isinstance(v, float) or not math.isclose(v, exp, rel_tol=4 * 2.0 ** -52, abs_tol=0.0):
                return False, f"YIELD {v!r} != {exp!r}"
        elif case["kind"] == "Bool":
            if not isinstance(v, bool) or v != exp:
                return False, f"YIELD {v!r} != {exp!r}"
        elif case["kind"] == "Int":
            if isinstance(v, bool) or not isinstance(v, int) or v != exp:
                return False, f"YIELD {v!r} != {exp!r}"
        elif v != exp:
            return False, f"YIELD {v!r} != {exp!r}"
    return True, "ok"


def _ulps_equal(a: float, b: float, ulps: int = 4) -> bool:
    """gtest's ASSERT_DOUBLE_EQ: within 4 units in the last place."""
    import struct
    if a == b:
        return True
    ia = struct.unpack("<q", struct.pack("<d", a))[0]
    ib = struct.unpack("<q", struct.pack("<d", b))[0]
    # biased representation: negative doubles ordered below the positive ones
    ia = -(ia & 0x7FFFFFFFFFFFFFFF) if ia < 0 else ia
    ib = -(ib & 0x7FFFFFFFFFFFFFFF) if ib < 0 else ib
    return abs(ia - ib) <= ulps


def run_func_case(backend, case):
    """(ok, message) for a FunctionCall / StringFunctionCall vector of ExpressionTest.cpp:585-745:
    TEST_EXPR(expected, op, expr, type) asserts is<type>(v) and ASSERT_<op>(expected, v)
    (ASSERT_DOUBLE_EQ for Double EQ: within 4 ulps).  The YIELD form gives the value; the WHERE form
    keeps both edges iff asBool(value) (not checked for rand32 / rand64, a value per row)."""
    import operator
    s = ngql.Session(backend)
    where_q, yield_q = expr_queries(case)
    kind, op, exp = case["kind"], case["op"], case["expect"]
    if kind == "Double":
        exp = 2.7182818284590451 if exp == "euler" else float(exp)
    elif kind == "Int":
        exp = int(exp)
    vals = [r[0] for r in s.execute(yield_q).rows]
    if len(vals) != 2:
        return False, f"YIELD gave {vals}"
    cmp = {"EQ": operator.eq, "NE": operator.ne, "LT": operator.lt, "LE": operator.le, "GT": operator.gt,
           "GE": operator.ge}[op]
    for v in vals:
        want = {"Double": float, "Int": int, "String": str}[kind]
        if isinstance(v, bool) or not isinstance(v, want):
            return False, f"YIELD {v!r} is not {kind}"
        good = _ulps_equal(exp, v) if (kind == "Double" and op == "EQ") else cmp(exp, v)
        if not good:
            return False, f"ASSERT_{op}({exp!r}, {v!r}) fails"
    if not case["expr"].startswith("rand"):
        truthy = (vals[0] != 0) if kind != "String" else vals[0] == ""
        rows = s.execute(where_q).rows
        if len(rows) != (2 if truthy else 0):
            return False, f"WHERE kept {len(rows)} rows"
    return True, "ok"
