#!/usr/bin/env python3
"""Regenerate tests/golden/*.json from the reference's own test files (run in the build
container only; /root/reference does not exist on the GPU box).

What it extracts (data only — inputs and expected outputs):
  * nba.json            the TraverseTestBase dataset (players/ages, teams, serve/like edges
                        in listed order) from src/graph/test/TraverseTestBase.h:260-915.
                        The uuid() copy of the data is dropped (time-dependent vids).
  * findpath_golden.json every FIND PATH case of src/graph/test/FindPathTest.cpp: the query
                        text with vids substituted and the expected path strings.
  * go_golden.json      every GO case of src/graph/test/GoTest.cpp: the query text with vids
                        substituted, expected rows / column names / expected-failure flag.

VIDs are std::hash<std::string>(name) (nebula_amd.vidhash.std_hash, pinned against
SURVEY.md §0 values).
"""
import json
import os
import re
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from nebula_amd.vidhash import std_hash  # noqa: E402

REF = os.environ.get("NEBULA_REF", "/root/reference")
OUT = os.path.join(os.path.dirname(__file__), "..", "tests", "golden")


def read(p):
    with open(os.path.join(REF, p)) as f:
        return f.read()


# ----------------------------------------------------------------------------- dataset
def parse_dataset():
    src = read("src/graph/test/TraverseTestBase.h")
    players = [(m.group(1), int(m.group(2)))
               for m in re.finditer(r'Player\{"([^"]+)",\s*(-?\d+)', src)]
    teams = [m.group(1) for m in re.finditer(r'Team\{"([^"]+)"\}', src)]
    body = src[src.index("AssertionResult TraverseTestBase::prepareData()"):]
    body = body[:body.index('std::string query = "USE nba"')]
    serves, likes = [], []
    for stmt in re.finditer(r'players_\["([^"]+)"\]((?:\s*\.\w+\([^)]*\))+)\s*;', body):
        who = stmt.group(1)
        for call in re.finditer(r'\.(serve|like)\(([^)]*)\)', stmt.group(2)):
            args = [a.strip() for a in call.group(2).split(",")]
            if call.group(1) == "serve":
                serves.append([who, args[0].strip('"'), int(args[1]), int(args[2])])
            else:
                likes.append([who, args[0].strip('"'), int(args[1])])
    return {
        "source": "src/graph/test/TraverseTestBase.h (uuid copy dropped)",
        "players": [{"name": n, "age": a, "vid": std_hash(n)} for n, a in players],
        "teams": [{"name": n, "vid": std_hash(n)} for n in teams],
        "serve": serves,
        "like": likes,
    }


# ----------------------------------------------------------------------------- C++ literal scanner
TOK = re.compile(r'''\s*(?:(?P<str>"(?:[^"\\]|\\.)*")|(?P<num>-?\d+)|(?P<open>\{)|(?P<close>\})|(?P<comma>,)
                     |(?P<ref>(?:players_|teams_)\["[^"]+"\]\.(?:vid|name)\(\))
                     |(?P<var>[A-Za-z_]\w*\.(?:vid|name)\(\))
                     |(?P<hash>std::hash<std::string>\(\)\("[^"]*"\))
                     |(?P<ident>[A-Za-z_]\w*))''', re.X)


class Ctx:
    def __init__(self, data):
        self.vars = {}
        self.pv = {p["name"]: p["vid"] for p in data["players"]}
        self.tv = {t["name"]: t["vid"] for t in data["teams"]}

    def value(self, kind, text):
        if kind == "str":
            return bytes(text[1:-1], "utf-8").decode("unicode_escape")
        if kind == "num":
            return int(text)
        if kind == "hash":
            return std_hash(re.search(r'\("([^"]*)"\)$', text).group(1))
        if kind == "ref":
            m = re.match(r'(players_|teams_)\["([^"]+)"\]\.(vid|name)\(\)', text)
            name = m.group(2)
            return name if m.group(3) == "name" else std_hash(name)
        if kind == "var":
            v, acc = text.split(".")
            name = self.vars[v]
            return name if acc.startswith("name") else std_hash(name)
        if kind == "ident" and text == "nonExistPlayerID":
            # GoTest.cpp:301-311: hash("NON EXIST VERTEX ID"), bumped past any player vid
            v = std_hash("NON EXIST VERTEX ID")
            while v in self.pv.values():
                v += 1
            return v
        raise ValueError(kind + ":" + text)


def scan_init(ctx, text):
    """Parse a C++ brace initializer of tuples/strings into Python lists."""
    pos, stack, cur = 0, [], None
    root = []
    cur = root
    pending_str = None
    while pos < len(text):
        m = TOK.match(text, pos)
        if not m:
            pos += 1
            continue
        pos = m.end()
        kind = m.lastgroup
        if kind == "open":
            new = []
            cur.append(new)
            stack.append(cur)
            cur = new
        elif kind == "close":
            cur = stack.pop()
        elif kind == "comma":
            pending_str = None
            continue
        elif kind == "str" and cur and isinstance(cur[-1], str) and pending_str is not None:
            cur[-1] += ctx.value("str", m.group(kind))   # adjacent literal concatenation
        else:
            cur.append(ctx.value(kind, m.group(kind)))
        pending_str = True if kind == "str" else None
    return root


def cpp_strings(text):
    """Concatenate adjacent C string literals."""
    return "".join(bytes(s[1:-1], "utf-8").decode("unicode_escape")
                   for s in re.findall(r'"(?:[^"\\]|\\.)*"', text))


def printf_ld(fmt, args):
    out, it = [], iter(args)
    parts = fmt.split("%ld")
    for i, p in enumerate(parts):
        out.append(p)
        if i < len(parts) - 1:
            out.append(str(next(it)))
    return "".join(out)


def blocks(src, cls):
    """Yield (test_name, block_text) for each `{ cpp2::ExecutionResponse resp; ... }` block."""
    for t in re.finditer(r"TEST_F\(%s, (\w+)\)\s*\{" % cls, src):
        start = t.end()
        depth, i = 1, start
        while depth:
            c = src[i]
            depth += (c == "{") - (c == "}")
            i += 1
        body = src[start:i - 1]
        for b in re.split(r"\n\s*\{\s*\n\s*cpp2::ExecutionResponse resp;", body)[1:]:
            yield t.group(1), b


def parse_block(ctx, b):
    ctx.vars = {}
    for m in re.finditer(r'auto\s*&\s*(\w+)\s*=\s*(?:players_|teams_)\["([^"]+)"\]\s*;', b):
        ctx.vars[m.group(1)] = m.group(2)
    q = None
    m = re.search(r'auto\s*\*\s*fmt\s*=\s*((?:"(?:[^"\\]|\\.)*"\s*)+);', b)
    if m:
        fmt = cpp_strings(m.group(1))
        a = re.search(r"folly::stringPrintf\(\s*fmt\s*,(.*?)\);", b, re.S)
        args = scan_init(ctx, a.group(1)) if a else []
        q = printf_ld(fmt, args)
    m2 = re.search(r'(?:std::string|auto\s*\*?)\s*query\s*=\s*((?:"(?:[^"\\]|\\.)*"\s*)+);', b)
    if q is None and m2:
        q = cpp_strings(m2.group(1))
    case = {"query": q}
    if re.search(r"ASSERT_NE\(cpp2::ErrorCode::SUCCEEDED, code\)", b):
        case["expect_error"] = True
        return case
    if "ASSERT_EQ(nullptr, resp.get_rows())" in b:
        case["expected"] = []
    m = re.search(r"expectedColNames\{(.*?)\};", b, re.S)
    if m:
        case["col_names"] = [c[0] if isinstance(c, list) else c for c in scan_init(ctx, m.group(1))]
    m = re.search(r"expected\s*=\s*\{(.*?)\};", b, re.S)
    if m:
        rows = scan_init(ctx, m.group(1))
        # path cases are flat lists of strings; GO cases are lists of tuples
        case["expected"] = rows if all(isinstance(r, str) for r in rows) else \
            [r if isinstance(r, list) else [r] for r in rows]
    elif re.search(r"std::vector<std::string> expected;", b):
        case["expected"] = []
    return case


def main():
    os.makedirs(OUT, exist_ok=True)
    data = parse_dataset()
    ctx = Ctx(data)
    with open(os.path.join(OUT, "nba.json"), "w") as f:
        json.dump(data, f, indent=1)
    fp = []
    for name, b in blocks(read("src/graph/test/FindPathTest.cpp"), "FindPathTest"):
        c = parse_block(ctx, b)
        c["test"] = name
        c["source"] = "src/graph/test/FindPathTest.cpp"
        fp.append(c)
    with open(os.path.join(OUT, "findpath_golden.json"), "w") as f:
        json.dump(fp, f, indent=1)
    go = []
    for name, b in blocks(read("src/graph/test/GoTest.cpp"), "GoTest"):
        c = parse_block(ctx, b)
        c["test"] = name
        c["source"] = "src/graph/test/GoTest.cpp"
        go.append(c)
    with open(os.path.join(OUT, "go_golden.json"), "w") as f:
        json.dump(go, f, indent=1)
    print(f"players={len(data['players'])} teams={len(data['teams'])} serve={len(data['serve'])} "
          f"like={len(data['like'])} findpath_cases={len(fp)} go_cases={len(go)}")


if __name__ == "__main__":
    main()
