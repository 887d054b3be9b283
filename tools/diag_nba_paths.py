#!/usr/bin/env python3
"""Diagnosis: FindPathTest golden cases on the nba space over G in-process ranks (G = 8 leaves
rank 0 without a part), collective search and replica, one line per case and mode."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import json
    from nebula_amd import LocalCluster, NbgError, kvgen
    from tests.support import golden
    data = json.load(open(os.path.join(ROOT, "tests", "golden", "nba.json")))
    for world in [int(x) for x in (sys.argv[1:] or ["8", "7"])]:
        c = LocalCluster(7, world)
        for (kind, name), cols in kvgen.NBA_SCHEMAS.items():
            if kind == "edge":
                c.register_edge(kvgen.NBA_EDGES[name], name, cols)
            else:
                c.register_tag(kvgen.NBA_TAGS[name], name, cols)
        c.load_builder(kvgen.nba_kv(data, 7))
        print(f"world {world}: vertices per rank {[e.stats()['num_vertices'] for e in c.engines]}", flush=True)
        for replica in (0, 1):
            c.set_path_replica(replica)
            for case in golden.load("findpath_golden.json"):
                if golden.unsupported_reason(case):
                    continue
                try:
                    ok, msg = golden.run_path_case(c, case)
                    res = "OK" if ok else "MISMATCH " + msg[:200]
                except NbgError as ex:
                    res = f"ERROR {ex.code}: {ex}"
                print(f"  G={world} replica={replica} {case['query'][:90]}: {res}", flush=True)
        c.close()


if __name__ == "__main__":
    main()
