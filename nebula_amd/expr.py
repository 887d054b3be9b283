"""Expression AST + the reference's binary wire codec (``Expression::encode``).

The C ABI (``include/nbg.h``) takes WHERE / YIELD expressions as the bytes
``Expression::encode`` produces (``src/common/filter/Expressions.cpp:93-116`` and the
per-class ``encode`` methods).  One extension, specified in ``include/nbg.h`` ("Expression
wire"): the reference cannot encode a ``TypeCastingExpression`` (its ``encode`` is empty,
Expressions.cpp:801-802), so nebula_amd encodes it as ``kind=4, uint8 ColumnType, operand``
(the graphd-side encoder body is in INTEGRATION.md §2; ``tests/support/wire.py`` produces the
unpatched bytes).

``to_string`` follows each class's ``toString`` (used for default YIELD column names).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import List, Optional, Union

# Expression::Kind (src/common/filter/Expressions.h:326-347)
K_PRIMARY, K_FUNC, K_UNARY, K_CAST, K_ARITH, K_REL, K_LOGIC = 1, 2, 3, 4, 5, 6, 7
K_SRC, K_RANK, K_DST, K_SRCID, K_TYPE, K_ALIAS, K_VAR, K_DESTP, K_INPUT = range(8, 17)

UNARY = {"+": 0, "-": 1, "!": 2}
ARITH = {"+": 0, "-": 1, "*": 2, "/": 3, "%": 4, "^": 5}
REL = {"<": 0, "<=": 1, ">": 2, ">=": 3, "==": 4, "!=": 5}
LOGIC = {"&&": 0, "||": 1, "XOR": 2}
# ColumnType (Expressions.h:21-23)
CAST = {"int": 0, "string": 1, "double": 2, "bigint": 3, "bool": 4, "timestamp": 5}

Value = Union[int, float, bool, str]


@dataclass
class Expr:
    kind: int
    op: str = ""
    value: Optional[Value] = None
    alias: str = ""
    prop: str = ""
    ref: str = ""
    args: List["Expr"] = field(default_factory=list)

    # ------------------------------------------------------------------ encode
    def encode(self) -> bytes:
        k = self.kind
        out = bytearray([k])

        def s16(s: str):
            b = s.encode()
            out.extend(struct.pack("<H", len(b)))
            out.extend(b)

        if k == K_PRIMARY:
            v = self.value
            if isinstance(v, bool):
                out += bytes([2, 1 if v else 0])
            elif isinstance(v, int):
                out += bytes([0]) + struct.pack("<q", v)
            elif isinstance(v, float):
                out += bytes([1]) + struct.pack("<d", v)
            else:
                out += bytes([3])
                s16(v)
        elif k == K_FUNC:
            s16(self.alias)
            out.extend(struct.pack("<H", len(self.args)))
            for a in self.args:
                out += a.encode()
        elif k == K_UNARY:
            out += bytes([UNARY[self.op]]) + self.args[0].encode()
        elif k == K_CAST:
            out += bytes([CAST[self.op]]) + self.args[0].encode()
        elif k in (K_ARITH, K_REL, K_LOGIC):
            table = {K_ARITH: ARITH, K_REL: REL, K_LOGIC: LOGIC}[k]
            out += bytes([table[self.op]]) + self.args[0].encode() + self.args[1].encode()
        elif k in (K_SRC, K_ALIAS, K_VAR, K_DESTP):
            s16(self.alias)
            s16(self.prop)
        elif k == K_INPUT:
            s16(self.prop)
        elif k in (K_RANK, K_DST, K_SRCID, K_TYPE):
            s16(self.alias)
        else:
            raise ValueError(f"cannot encode kind {k}")
        return bytes(out)

    # ------------------------------------------------------------------ toString
    def to_string(self) -> str:
        k = self.kind
        if k == K_PRIMARY:
            v = self.value
            if isinstance(v, bool):
                return "true" if v else "false"
            if isinstance(v, float):
                return "%f" % v
            return str(v)
        if k in (K_SRC, K_DESTP, K_ALIAS, K_VAR, K_INPUT, K_RANK, K_DST, K_SRCID, K_TYPE):
            buf = self.ref
            if self.ref not in ("", "$"):
                buf += "."
            buf += self.alias
            if self.alias:
                buf += "."
            return buf + self.prop
        if k == K_UNARY:
            return self.op + "(" + self.args[0].to_string() + ")"
        if k == K_CAST:
            return "(" + self.op + ")" + self.args[0].to_string()
        if k == K_FUNC:
            return self.alias + "(" + ",".join(a.to_string() for a in self.args) + ")"
        op = self.op
        return "(" + self.args[0].to_string() + op + self.args[1].to_string() + ")"

    def walk(self):
        yield self
        for a in self.args:
            yield from a.walk()


# ---------------------------------------------------------------- builders
def const(v: Value) -> Expr:
    return Expr(K_PRIMARY, value=v)


def edge_prop(edge: str, prop: str) -> Expr:
    if prop == "_dst":
        return Expr(K_DST, alias=edge, prop="_dst")
    if prop == "_src":
        return Expr(K_SRCID, alias=edge, prop="_src")
    if prop == "_rank":
        return Expr(K_RANK, alias=edge, prop="_rank")
    if prop == "_type":
        return Expr(K_TYPE, alias=edge, prop="_type")
    return Expr(K_ALIAS, alias=edge, prop=prop)


def src_prop(tag: str, prop: str) -> Expr:
    return Expr(K_SRC, alias=tag, prop=prop, ref="$^")


def dst_prop(tag: str, prop: str) -> Expr:
    return Expr(K_DESTP, alias=tag, prop=prop, ref="$$")


def input_prop(prop: str) -> Expr:
    return Expr(K_INPUT, prop=prop, ref="$-")


def var_prop(var: str, prop: str) -> Expr:
    return Expr(K_VAR, alias=var, prop=prop, ref="$")


def binop(op: str, a: Expr, b: Expr) -> Expr:
    if op in REL:
        return Expr(K_REL, op=op, args=[a, b])
    if op in LOGIC:
        return Expr(K_LOGIC, op=op, args=[a, b])
    return Expr(K_ARITH, op=op, args=[a, b])


def unary(op: str, a: Expr) -> Expr:
    return Expr(K_UNARY, op=op, args=[a])


def cast(ctype: str, a: Expr) -> Expr:
    return Expr(K_CAST, op=ctype, args=[a])
