#!/usr/bin/env python3
"""8-rank GO first-hop slot exchange against the oracle (GPU box): NBA data over 8 in-process
ranks, 2-step statements with slots on / off (NBG_GO_SLOTS, read per query), run on a fresh
cluster and again after other 8-rank clusters have run and been closed (device memory reused).
Prints every mismatch.  Usage: diag_slots8.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nebula_amd import LocalCluster, kvgen  # noqa: E402
from tests.support import ngql  # noqa: E402
from tests.support.oracle import nba_oracle  # noqa: E402

with open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "nba.json")) as f:
    data = json.load(f)


def cluster(world, parts=7):
    c = LocalCluster(parts, world)
    for (kind, name), cols in kvgen.NBA_SCHEMAS.items():
        if kind == "edge":
            c.register_edge(kvgen.NBA_EDGES[name], name, cols)
        else:
            c.register_tag(kvgen.NBA_TAGS[name], name, cols)
    c.load_builder(kvgen.nba_kv(data, parts))
    return c


def rows(b, q):
    try:
        return sorted(tuple(r) for r in ngql.Session(b).execute(q).rows)
    except Exception as ex:   # noqa: BLE001
        return f"error {ex}"


TD, TP = 'hash("Tim Duncan")', 'hash("Tony Parker")'
QS = [f'GO 2 STEPS FROM {TD} OVER like YIELD DISTINCT left(right($$.player.name, 4), 2) AS f',
      f'GO 2 STEPS FROM {TD} OVER like YIELD like._dst',
      f'GO 2 STEPS FROM {TD} OVER like YIELD DISTINCT $$.player.name',
      f'GO 2 STEPS FROM {TD} OVER like YIELD $$.player.name, like._src',
      f'GO 3 STEPS FROM {TP} OVER like YIELD like._dst']
orc = nba_oracle(data, 7)
want = {q: rows(orc, q) for q in QS}


def check(tag, c):
    bad = 0
    for slots in ("1", "0"):
        os.environ["NBG_GO_SLOTS"] = slots
        for q in QS:
            got = rows(c, q)
            if got != want[q]:
                bad += 1
                print(f"{tag} slots={slots} MISMATCH {q}\n   got  {got}\n   want {want[q]}", flush=True)
    print(f"{tag}: {bad} mismatches", flush=True)


for world, parts in ((8, 7), (8, 100), (2, 7), (4, 7)):
    orc = nba_oracle(data, parts)
    want = {q: rows(orc, q) for q in QS}
    c = cluster(world, parts)
    check(f"fresh world {world} parts {parts}", c)
    c.close()
orc = nba_oracle(data, 7)
want = {q: rows(orc, q) for q in QS}
# other clusters: many 2- and 3-step statements from every player, then closed
players = [p for p in data.get("players", [])][:40] if isinstance(data, dict) else []
for k in range(3):
    d = cluster(8)
    for q in QS:
        rows(d, q)
    for name in ["Steve Nash", "Ray Allen", "Kobe Bryant", "LeBron James", "Dwyane Wade", "Yao Ming"]:
        for st in (2, 3):
            rows(d, f'GO {st} STEPS FROM hash("{name}") OVER like YIELD DISTINCT left(right($$.player.name, 4), 2) AS f')
            rows(d, f'GO {st} STEPS FROM hash("{name}") OVER like, serve YIELD like._dst, serve._dst')
    d.close()
    print(f"dirty cluster {k} closed", flush=True)
c = cluster(8)
check("after", c)
for name in ["Steve Nash", "Ray Allen", "Kobe Bryant"]:
    rows(c, f'GO 2 STEPS FROM hash("{name}") OVER like YIELD DISTINCT left(right($$.player.name, 4), 2) AS f')
check("same cluster after other roots", c)
c.close()
