#!/usr/bin/env python3
"""The final GO step's launch (k_final_dst) at one RMAT scale under environment settings (GPU
box): per setting a fresh statement, the bench's roots one at a time with HIP events around every
FINAL launch (profile mode 2), the average launch, its algorithmic bytes and fraction of 8 TB/s,
and the digest of every root checked against the first setting's.
Usage: go_final_probe.py <scale> <roots> <setting>...   setting = VAR=VALUE[,VAR=VALUE] or "default"."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nebula_amd import Engine, expr as E, rmat  # noqa: E402

scale, nroots = int(sys.argv[1]), int(sys.argv[2])
settings = sys.argv[3:] or ["default"]
src, dst, w = rmat.rmat_edges_fast(scale)
eng = Engine(100)
eng.register_edge(1, "e", [("w", 2)])
eng.load_edges(1, src, dst, [w])
eng.finalize()
sv, _ = rmat.vertex_sets(scale)
roots = [int(x) for x in rmat.pick_roots(src, nroots, 42, verts=sv)]
del src, dst, w
where = E.binop("<", E.edge_prop("e", "w"), E.const(50)).encode()
base = None
for rnd in range(2):
    for spec in settings:
        env = {} if spec == "default" else dict(kv.split("=", 1) for kv in spec.split(","))
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            stmt = eng.prepare_go([1], 3, where)
            for r in roots[:8]:
                stmt.run_device([r]).free()
            digs = []
            eng.profile(2)
            t0 = time.perf_counter()
            for r in roots:
                res = stmt.run_device([r])
                digs.append(res.digest())
                res.free()
            el = time.perf_counter() - t0
            ks = eng.profile_read()
            eng.profile(False)
            stmt.free()
            if base is None:
                base = digs
            name, v = max(ks.items(), key=lambda kv: kv[1]["ms"])
            us = v["ms"] * 1e3 / max(1, v["launches"])
            gbs = v["algo_bytes"] / (v["ms"] * 1e-3) / 1e9 if v["ms"] else 0
            print(f"r{rnd} {spec:36s} {name} {v['launches']} launches avg {us:8.2f} us  {gbs:7.1f} GB/s "
                  f"frac {gbs / 8000:.4f}  MB/launch {v['algo_bytes'] / max(1, v['launches']) / 1e6:.1f}  "
                  f"wall {el * 1e3:.1f} ms  same {sum(a == b for a, b in zip(digs, base))}/{len(digs)}", flush=True)
        finally:
            for k, val in old.items():
                if val is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = val
eng.close()
