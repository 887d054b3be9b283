"""The bytes an UNPATCHED reference graphd sends for an expression.

`Expression::encode` (`src/common/filter/Expressions.cpp:93-98`) calls each node's `encode`,
and `TypeCastingExpression::encode` (`:801-802`) writes nothing at all: not its kind byte, not
its ColumnType, not its operand.  So a cast and its whole subtree vanish from the wire, and the
parent's remaining bytes are a prefix-coded tree with one subtree missing.  The reference's own
`Expression::decode` (`:102-116`) then runs out of bytes (THROW_IF_NO_SPACE) and fails; a root
cast encodes to zero bytes.

nebula_amd's wire extension (`include/nbg.h`, "Expression wire") encodes the cast as
`kind = 4, uint8 ColumnType, operand`; `reference_encode` below is the unpatched encoder, used by
the tests that check the engine rejects these bytes cleanly instead of misparsing them."""
from __future__ import annotations

import dataclasses

from nebula_amd import expr as E


class _Raw:
    """A child whose bytes are already encoded (duck-types Expr.encode)."""

    def __init__(self, b: bytes):
        self.b = b

    def encode(self) -> bytes:
        return self.b


def reference_encode(e: E.Expr) -> bytes:
    if e.kind == E.K_CAST:
        return b""   # TypeCastingExpression::encode(Cord&) const {}
    if not e.args:
        return e.encode()
    return dataclasses.replace(e, args=[_Raw(reference_encode(a)) for a in e.args]).encode()


def cast_shapes():
    """(name, WHERE expr or None, YIELD exprs): the three cast shapes of VERDICT r04 item 4 over
    the nba `like` edge (likeness INT) and `player` tag (name STRING, age INT)."""
    likeness = E.edge_prop("like", "likeness")
    return [
        ("(int)a > 1", E.binop(">", E.cast("int", likeness), E.const(1)), []),
        ("(int)a + (int)b", None, [E.binop("+", E.cast("int", likeness), E.cast("int", E.edge_prop("like", "_dst")))]),
        ('(string)a + "x"', None, [E.binop("+", E.cast("string", likeness), E.const("x"))]),
        ("(int)a > 1 && a <= 100", E.binop("&&", E.binop(">", E.cast("int", likeness), E.const(1)),
                                         E.binop("<=", likeness, E.const(100))), []),
        ("YIELD (int)a", None, [E.cast("int", likeness)]),
    ]
