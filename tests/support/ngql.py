"""TEST HARNESS (not product code; SURVEY.md §2 puts the nGQL front end out of scope): a small
nGQL front end for the traversal statements (GO / FIND PATH), pipes and
variables — enough to drive the engine the way graphd does, so parity tests read like the
reference's GoTest / FindPathTest.

Grammar follows ``src/parser/parser.yy`` (go_sentence :513-537, find_path_sentence
:835-861, expression precedence :400-512).  Execution follows graphd:
  * ``GO ... FROM $-.col`` takes the column's values with duplicates
    (``InterimResult::getVIDs``, src/graph/InterimResult.cpp:29-49);
  * FIND PATH ``FROM/TO`` lists are de-duplicated (``VerticesClause::prepare``,
    src/parser/Clauses.cpp:51-92; ``getDistinctVIDs``);
  * default YIELD is ``<edge>._dst`` per OVER edge (parser.yy:518-531).
The backend (``nebula_amd.Engine`` on the GPU, or the test oracle) executes each sentence.
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import List, Optional

from nebula_amd import expr as E
from nebula_amd.vidhash import std_hash

_TOK = re.compile(r"""\s*(?:
    (?P<double>\d+\.\d*(?:[eE][+-]?\d+)?|\.\d+(?:[eE][+-]?\d+)?)
   |(?P<int>0[xX][0-9a-fA-F]+|\d+)
   |(?P<str>"(?:[^"\\]|\\.)*"|'(?:[^'\\]|\\.)*')
   |(?P<var>\$[A-Za-z_]\w*)
   |(?P<sym>\$\^|\$\$|\$-|<=|>=|==|!=|&&|\|\||[<>+\-*/%^!(),.;|=])
   |(?P<name>[A-Za-z_]\w*)
)""", re.X)


class ParseError(Exception):
    pass


def int_literal(text: str) -> int:
    """An INTEGER token as scanner.lex:328-368 reads it.  Flex takes the longest match, first rule
    on a tie: `0[Xx]{HEX}+` (sscanf %lx), `0{OCT}+` (%lo), `{DEC}+` (folly::to<int64_t>) — so
    "0777" is octal but "09" and "0789" are decimal (the decimal match is longer).  Hex with more
    than 16 significant digits and octal with more than 22 (or 22 not starting with 1) stop the
    scan; the sscanf conversions wrap into int64, the decimal one rejects out-of-range values."""
    if text[:2] in ("0x", "0X"):
        if len(text[2:].lstrip("0")) > 16:
            raise ParseError(f"hex literal out of range: {text}")
        v = int(text, 16)
        return v - (1 << 64) if v >= 1 << 63 else v
    if len(text) > 1 and text[0] == "0" and all(c in "01234567" for c in text):
        sig = text[1:].lstrip("0")
        if len(sig) > 22 or (len(sig) == 22 and sig[0] != "1"):
            raise ParseError(f"octal literal out of range: {text}")
        v = int(text, 8)
        return v - (1 << 64) if v >= 1 << 63 else v
    v = int(text, 10)
    if v >= 1 << 63:
        raise ParseError(f"integer out of range: {text}")
    return v


def tokenize(s: str):
    pos, out = 0, []
    s = s.rstrip()
    while pos < len(s):
        m = _TOK.match(s, pos)
        if not m or m.end() == pos:
            raise ParseError(f"bad token at {s[pos:pos + 20]!r}")
        pos = m.end()
        kind = m.lastgroup
        text = m.group(kind)
        out.append((kind, text))
    out.append(("eof", ""))
    return out


@dataclass
class YieldCol:
    expr: E.Expr
    alias: Optional[str] = None

    def name(self):
        return self.alias if self.alias else self.expr.to_string()


@dataclass
class GoSentence:
    steps: int = 1
    upto: bool = False
    from_vids: List[int] = field(default_factory=list)
    from_ref: Optional[tuple] = None          # ("$-", col) or ("$var", col)
    over: List[str] = field(default_factory=list)
    over_all: bool = False
    reversely: bool = False
    where: Optional[E.Expr] = None
    yields: Optional[List[YieldCol]] = None
    distinct: bool = False


@dataclass
class FindPathSentence:
    shortest: bool
    from_vids: List[int] = field(default_factory=list)
    from_ref: Optional[tuple] = None
    to_vids: List[int] = field(default_factory=list)
    to_ref: Optional[tuple] = None
    over: List[str] = field(default_factory=list)
    over_all: bool = False
    upto: int = 5


@dataclass
class Pipe:
    left: object
    right: object


@dataclass
class Assign:
    var: str
    stmt: object


class Parser:
    def __init__(self, text):
        self.t = tokenize(text)
        self.i = 0

    # ---------------------------------------------------------------- helpers
    def peek(self, k=0):
        return self.t[self.i + k]

    def kw(self, *words):
        kind, text = self.peek()
        return kind == "name" and text.upper() in words

    def take(self):
        tok = self.t[self.i]
        self.i += 1
        return tok

    def expect_kw(self, w):
        if not self.kw(w):
            raise ParseError(f"expected {w} near {self.peek()[1]!r}")
        self.take()

    def expect_sym(self, s):
        kind, text = self.take()
        if text != s:
            raise ParseError(f"expected {s!r}, got {text!r}")

    def sym(self, s):
        kind, text = self.peek()
        return kind == "sym" and text == s

    # ---------------------------------------------------------------- statements
    def parse(self):
        stmts = [self.statement()]
        while self.sym(";"):
            self.take()
            if self.peek()[0] == "eof":
                break
            stmts.append(self.statement())
        if self.peek()[0] != "eof":
            raise ParseError(f"trailing input near {self.peek()[1]!r}")
        return stmts

    def statement(self):
        if self.peek()[0] == "var" and self.peek(1) == ("sym", "="):
            var = self.take()[1][1:]
            self.take()
            return Assign(var, self.piped())
        return self.piped()

    def piped(self):
        left = self.primary_sentence()
        while self.sym("|"):
            self.take()
            left = Pipe(left, self.primary_sentence())
        return left

    def primary_sentence(self):
        if self.sym("("):
            self.take()
            s = self.piped()
            self.expect_sym(")")
            return s
        if self.kw("GO"):
            return self.go()
        if self.kw("FIND"):
            return self.find_path()
        raise ParseError(f"unsupported sentence near {self.peek()[1]!r}")

    def vid_list_or_ref(self):
        kind, text = self.peek()
        if kind == "sym" and text == "$-":
            self.take()
            col = "id"
            if self.sym("."):
                self.take()
                col = self.take()[1]
            return [], ("$-", col)
        if kind == "var":
            self.take()
            col = "id"
            if self.sym("."):
                self.take()
                col = self.take()[1]
            return [], (text[1:], col)
        vids = [self.const_int()]
        while self.sym(","):
            self.take()
            vids.append(self.const_int())
        return vids, None

    def const_int(self):
        e = self.expression()
        v = fold_const(e)
        if not isinstance(v, int) or isinstance(v, bool):
            raise ParseError("Vertex ID should be of type integer")
        return v

    def over_clause(self):
        edges, over_all, rev = [], False, False
        while True:
            if self.sym("*"):
                self.take()
                over_all = True
            else:
                edges.append(self.take()[1])
                if self.kw("AS"):
                    self.take()
                    self.take()
                if self.kw("REVERSELY"):
                    self.take()
                    rev = True
            if not self.sym(","):
                break
            self.take()
        return edges, over_all, rev

    def go(self):
        self.expect_kw("GO")
        g = GoSentence()
        if self.kw("UPTO"):
            self.take()
            g.steps = int(self.take()[1])
            g.upto = True
            self.expect_kw("STEPS")
        elif self.peek()[0] == "int":
            g.steps = int(self.take()[1])
            self.expect_kw("STEPS")
        self.expect_kw("FROM")
        g.from_vids, g.from_ref = self.vid_list_or_ref()
        self.expect_kw("OVER")
        g.over, g.over_all, g.reversely = self.over_clause()
        if self.kw("WHERE"):
            self.take()
            g.where = self.expression()
        if self.kw("YIELD"):
            self.take()
            if self.kw("DISTINCT"):
                self.take()
                g.distinct = True
            g.yields = [self.yield_col()]
            while self.sym(","):
                self.take()
                g.yields.append(self.yield_col())
        return g

    def yield_col(self):
        e = self.expression()
        alias = None
        if self.kw("AS"):
            self.take()
            alias = self.take()[1]
        return YieldCol(e, alias)

    def find_path(self):
        self.expect_kw("FIND")
        shortest = self.kw("SHORTEST")
        if not (shortest or self.kw("ALL")):
            raise ParseError("expected SHORTEST or ALL")
        self.take()
        self.expect_kw("PATH")
        s = FindPathSentence(shortest=shortest)
        self.expect_kw("FROM")
        s.from_vids, s.from_ref = self.vid_list_or_ref()
        self.expect_kw("TO")
        s.to_vids, s.to_ref = self.vid_list_or_ref()
        self.expect_kw("OVER")
        s.over, s.over_all, _ = self.over_clause()
        if self.kw("UPTO"):
            self.take()
            s.upto = int(self.take()[1])
            self.expect_kw("STEPS")
        return s

    # ---------------------------------------------------------------- expressions
    def expression(self):
        left = self.logic_or()
        while self.kw("XOR"):
            self.take()
            left = E.binop("XOR", left, self.logic_or())
        return left

    def logic_or(self):
        left = self.logic_and()
        while self.sym("||") or self.kw("OR"):
            self.take()
            left = E.binop("||", left, self.logic_and())
        return left

    def logic_and(self):
        left = self.equality()
        while self.sym("&&") or self.kw("AND"):
            self.take()
            left = E.binop("&&", left, self.equality())
        return left

    def equality(self):
        left = self.relational()
        while self.sym("==") or self.sym("!="):
            op = self.take()[1]
            left = E.binop(op, left, self.relational())
        return left

    def relational(self):
        left = self.additive()
        while any(self.sym(s) for s in ("<", ">", "<=", ">=")):
            op = self.take()[1]
            left = E.binop(op, left, self.additive())
        return left

    def additive(self):
        left = self.multiplicative()
        while self.sym("+") or self.sym("-"):
            op = self.take()[1]
            left = E.binop(op, left, self.multiplicative())
        return left

    def multiplicative(self):
        left = self.xor_arith()
        while self.sym("*") or self.sym("/") or self.sym("%"):
            op = self.take()[1]
            left = E.binop(op, left, self.xor_arith())
        return left

    def xor_arith(self):
        left = self.unary()
        while self.sym("^"):
            self.take()
            left = E.binop("^", left, self.unary())
        return left

    def unary(self):
        if self.sym("+") or self.sym("-") or self.sym("!"):
            op = self.take()[1]
            return E.unary(op, self.unary())
        if self.kw("NOT"):
            self.take()
            return E.unary("!", self.unary())
        if self.sym("(") and self.peek(1)[0] == "name" and self.peek(1)[1].lower() in E.CAST \
                and self.peek(2) == ("sym", ")"):
            self.take()
            ctype = self.take()[1].lower()
            self.take()
            return E.cast(ctype, self.unary())
        return self.primary()

    def primary(self):
        kind, text = self.take()
        if kind == "int":
            return E.const(int_literal(text))
        if kind == "double":
            return E.const(float(text))
        if kind == "str":
            return E.const(bytes(text[1:-1], "utf-8").decode("unicode_escape"))
        if kind == "sym" and text == "(":
            e = self.expression()
            self.expect_sym(")")
            return e
        if kind == "sym" and text in ("$^", "$$"):
            self.expect_sym(".")
            tag = self.take()[1]
            self.expect_sym(".")
            prop = self.take()[1]
            return E.src_prop(tag, prop) if text == "$^" else E.dst_prop(tag, prop)
        if kind == "sym" and text == "$-":
            prop = "id"
            if self.sym("."):
                self.take()
                prop = self.take()[1]
            return E.input_prop(prop)
        if kind == "var":
            prop = "id"
            if self.sym("."):
                self.take()
                prop = self.take()[1]
            return E.var_prop(text[1:], prop)
        if kind == "name":
            if text.lower() in ("true", "false"):
                return E.const(text.lower() == "true")
            if self.sym("("):
                self.take()
                args = []
                if not self.sym(")"):
                    args.append(self.expression())
                    while self.sym(","):
                        self.take()
                        args.append(self.expression())
                self.expect_sym(")")
                return E.Expr(E.K_FUNC, alias=text, args=args)
            if self.sym("."):
                self.take()
                prop = self.take()[1]
                return E.edge_prop(text, prop)
            return E.const(text)     # bare name_label -> PrimaryExpression(string)
        raise ParseError(f"unexpected {text!r}")


def parse(text: str):
    return Parser(text).parse()


def fold_const(e: E.Expr):
    """Evaluate a constant vid expression (integers, unary minus, hash('...'))."""
    if e.kind == E.K_PRIMARY:
        return e.value
    if e.kind == E.K_UNARY and e.op == "-":
        v = fold_const(e.args[0])
        return -v
    if e.kind == E.K_UNARY and e.op == "+":
        return fold_const(e.args[0])
    if e.kind == E.K_FUNC and e.alias.lower() == "hash" and len(e.args) == 1:
        v = fold_const(e.args[0])
        return std_hash(str(v))
    raise ParseError("vid expression is not constant")


# ------------------------------------------------------------------------------- execution
class ExecError(Exception):
    def __init__(self, msg, code=-8):
        super().__init__(msg)
        self.code = code


@dataclass
class Interim:
    columns: List[str]
    rows: List[list]

    def col(self, name):
        if name not in self.columns:
            raise ExecError(f"column `{name}' not found")
        i = self.columns.index(name)
        return [r[i] for r in self.rows]


class Session:
    """Executes parsed statements against a backend with
    ``go(**kw) -> (rows)`` and ``find_path(**kw) -> [entry lists]`` plus schema maps
    ``edge_types`` (name -> type) / ``edge_names`` (type -> name)."""

    def __init__(self, backend):
        self.b = backend
        self.vars = {}

    def execute(self, text: str) -> Interim:
        result = Interim([], [])
        for st in parse(text):
            result = self._run(st, None)
        return result

    def _run(self, st, inp: Optional[Interim]):
        if isinstance(st, Assign):
            r = self._run(st.stmt, inp)
            self.vars[st.var] = r
            return r
        if isinstance(st, Pipe):
            return self._run(st.right, self._run(st.left, inp))
        if isinstance(st, GoSentence):
            return self._go(st, inp)
        if isinstance(st, FindPathSentence):
            return self._find(st, inp)
        raise ExecError("unsupported statement")

    def _source(self, ref, inp):
        if ref[0] == "$-":
            return inp
        if ref[0] not in self.vars:
            raise ExecError(f"Variable `{ref[0]}' not defined")
        return self.vars[ref[0]]

    def _edge_types(self, names, over_all):
        if over_all:
            return sorted(t for t in self.b.edge_names if t > 0)
        out = []
        for n in names:
            if n not in self.b.edge_types:
                raise ExecError(f"edge `{n}' not found")
            out.append(self.b.edge_types[n])
        return out

    def _go(self, g: GoSentence, inp):
        if g.upto:
            raise ExecError("`UPTO' not supported yet")
        if g.reversely:
            raise ExecError("`REVERSELY' not supported yet")
        etypes = self._edge_types(g.over, g.over_all)
        if g.yields is None:
            cols = [] if g.over_all else [YieldCol(E.edge_prop(n, "_dst")) for n in g.over]
        else:
            cols = g.yields
        if g.over_all and not cols:
            # one `<edge>._dst` column per entry of the response's edge_schema, in that map's
            # order (GoExecutor::finishExecution, GoExecutor.cpp:546-561)
            cols = [YieldCol(E.edge_prop(self.b.edge_names[t], "_dst"))
                    for t in self.b.default_columns(etypes, over_all=True)]
        # `$-.*` / `$var.*`: every column of the input (YieldClause expansion)
        if any(c.expr.kind in (E.K_INPUT, E.K_VAR) and c.expr.prop == "*" for c in cols):
            if g.from_ref is None:
                raise ExecError("`*' input props need a piped or variable FROM")
            src = self._source(g.from_ref, inp)
            expanded = []
            for c in cols:
                if c.expr.kind in (E.K_INPUT, E.K_VAR) and c.expr.prop == "*":
                    for n in (src.columns if src is not None else []):
                        expanded.append(YieldCol(E.input_prop(n) if c.expr.kind == E.K_INPUT
                                                 else E.var_prop(c.expr.alias, n)))
                else:
                    expanded.append(c)
            cols = expanded
        names = [c.name() for c in cols]
        if g.from_ref is not None:
            src = self._source(g.from_ref, inp)
            if src is None or not src.rows:
                return Interim(names, [])
            starts = [int(v) for v in src.col(g.from_ref[1])]
        else:
            starts = list(g.from_vids)
        uses_input = any(n.kind in (E.K_INPUT, E.K_VAR)
                         for c in cols + ([YieldCol(g.where)] if g.where else []) for n in c.expr.walk())
        kw = {}
        if uses_input:
            # $-.x / $var.x read the FROM source's rows (GoExecutor::setupStarts index)
            if g.from_ref is None:
                raise ExecError("input/variable props need a piped or variable FROM")
            src = self._source(g.from_ref, inp)
            kw["inputs"] = (src.columns, src.rows, g.from_ref[1])
        rows = self.b.go(starts=starts, etypes=etypes, steps=g.steps,
                         where=g.where.encode() if g.where else b"",
                         yields=[c.expr.encode() for c in cols], distinct=g.distinct, **kw)
        return Interim(names, rows)

    def _find(self, s: FindPathSentence, inp):
        def vids(lst, ref):
            if ref is None:
                out, seen = [], set()
                for v in lst:
                    if v not in seen:
                        seen.add(v)
                        out.append(v)
                return out
            src = self._source(ref, inp)
            if src is None or not src.rows:
                return []
            return list(dict.fromkeys(int(v) for v in src.col(ref[1])))
        frm, to = vids(s.from_vids, s.from_ref), vids(s.to_vids, s.to_ref)
        etypes = self._edge_types(s.over, s.over_all)
        paths = self.b.find_path(frm=frm, to=to, etypes=etypes, upto=s.upto, shortest=s.shortest)
        return Interim(["_path_"], [[p] for p in paths])


def path_string(entry: List[int], edge_names) -> str:
    """TraverseTestBase::buildPathString (src/graph/test/TraverseTestBase.h:78-98)."""
    out = []
    i = 0
    while i + 3 < len(entry) + 1 and i + 1 < len(entry):
        out.append(f"{entry[i]}<{edge_names[entry[i + 1]]},{entry[i + 2]}>")
        i += 3
    out.append(str(entry[i]))
    return "".join(out)
