#!/usr/bin/env python3
"""Generate tests/golden/expression_cases.json from the reference's expression unit test
(src/common/filter/test/ExpressionTest.cpp, read as text).

Every ``TEST_EXPR(...)`` vector of the literal blocks becomes one case: the WHERE expression
text, the value kind the test asserts (Bool / Int / Double / String) and the expected value.
  * LiteralConstants            TEST_EXPR(expr, type): the expected value is the C++ value of
                                the literal expression itself (restated below);
  * LiteralContantsArithmetic   TEST_EXPR(expr, expected, type);
  * LiteralConstantsRelational,
    LiteralConstantsLogical     TEST_EXPR(expr, expected)  (Bool);
  * FunctionCall, StringFunctionCall
                                TEST_EXPR(expected, op, expr, type)  (kept, marked "function");
  * InvalidExpressionTest       TEST_EXPR(expr): evaluation must fail.
The string-literal case of LiteralConstants and the explicit `16 + 8 / 4 - 2` case are added
as written in the test.  Usage: make_golden_expr.py [reference root] > expression_cases.json
"""
import json
import re
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
SRC = f"{REF}/src/common/filter/test/ExpressionTest.cpp"


def split_args(s):
    """Top-level comma split of a macro argument list."""
    out, depth, cur, q = [], 0, "", None
    for ch in s:
        if q:
            cur += ch
            if ch == q:
                q = None
            continue
        if ch in "\"'":
            q = ch
        elif ch == "(":
            depth += 1
        elif ch == ")":
            depth -= 1
        elif ch == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
            continue
        cur += ch
    out.append(cur.strip())
    return out


def cpp_value(expr):
    """The C++ value of a literal expression of LiteralConstants (bools, ints, hex, doubles)."""
    py = expr.replace("&&", " and ").replace("||", " or ").replace("true", "True").replace("false", "False")
    py = re.sub(r"!(?!=)", " not ", py)
    v = eval(py, {}, {})   # noqa: S307 - literal constants only
    return v


def cases():
    text = open(SRC).read()
    blocks = re.split(r"\nTEST_F\(ExpressionTest, (\w+)\)", text)
    out = []
    for name, body in zip(blocks[1::2], blocks[2::2]):
        for m in re.finditer(r"^\s*TEST_EXPR\((.*)\);", body, re.M):
            args = split_args(m.group(1))
            case = {"test": name}
            if name == "LiteralConstants":
                expr, kind = args
                v = cpp_value(expr)
                case.update(expr=expr, kind=kind, expect=bool(v) if kind == "Bool" else v)
            elif name == "LiteralContantsArithmetic":
                expr, exp, kind = args
                case.update(expr=expr, kind=kind, expect=float(exp) if kind == "Double" else int(exp))
            elif name in ("LiteralConstantsRelational", "LiteralConstantsLogical"):
                expr, exp = args
                case.update(expr=expr, kind="Bool", expect=exp == "true")
            elif name in ("FunctionCall", "StringFunctionCall"):
                exp, op, expr, kind = args
                case.update(expr=expr, kind=kind, op=op, expect=exp.strip('"') if kind == "String" else exp,
                            function=True)
            elif name == "InvalidExpressionTest":
                case.update(expr=args[0], error=True)
            else:
                continue
            out.append(case)
    out.append({"test": "LiteralConstants", "expr": '"string_literal"', "kind": "String", "expect": "string_literal"})
    out.append({"test": "LiteralContantsArithmetic", "expr": "16 + 8 / 4 - 2", "kind": "Int", "expect": 16})
    return out


if __name__ == "__main__":
    json.dump(cases(), sys.stdout, indent=1)
    sys.stdout.write("\n")
