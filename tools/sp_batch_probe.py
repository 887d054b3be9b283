#!/usr/bin/env python3
"""Batched FIND SHORTEST PATH A/B on one loaded graph (GPU box): the bench's pairs through
nbg_find_path_batch under each setting (environment variables the library reads per batch),
every result compared with the first setting's, plus the one-pair latency of a sample.
Usage: sp_batch_probe.py <scale> <pairs> <setting>...   setting = VAR=VALUE[,VAR=VALUE] or "default"."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nebula_amd import Engine, rmat  # noqa: E402

scale, npairs = int(sys.argv[1]), int(sys.argv[2])
settings = sys.argv[3:] or ["default"]
src, dst, w = rmat.rmat_edges_fast(scale)
eng = Engine(100)
eng.register_edge(1, "e", [("w", 2)])
eng.load_edges(1, src, dst, [w])
eng.finalize()
_, av = rmat.vertex_sets(scale)
pairs = rmat.pick_pairs(src, dst, 10000, 7, verts=av)[:npairs]
del src, dst, w
eng.path_reserve(6, 64)   # (the library's NBG_SP_BATCH contexts)
reqs = [([s], [t], [1], 5, True) for s, t in pairs]
chunk = 2000
preps = [eng.path_batch_prepare(reqs[k:k + chunk]) for k in range(0, len(reqs), chunk)]
base = None
print(f"RMAT-{scale}, {len(pairs)} pairs", flush=True)
for rnd in range(int(os.environ.get('PROBE_ROUNDS', '2'))):
    for spec in settings:
        env = {} if spec == "default" else dict(kv.split("=", 1) for kv in spec.split(","))
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            eng.find_path_batch(reqs[:64])   # warm
            t0 = time.perf_counter()
            results = [eng.path_batch_run(p) for p in preps]
            el = time.perf_counter() - t0
            got, fails = [], []
            for k, ((outs, rcs), p) in enumerate(zip(results, preps)):
                for i in range(p[1]):
                    if rcs[i]:
                        fails.append((k * chunk + i, rcs[i]))
                        got.append(None)
                        continue
                    got.append(eng._paths(outs[i], None))
            msg = eng.lib.nbg_last_error(eng.h)
            if fails:
                print(f"   {len(fails)} failed; last error: {msg.decode() if msg else ''}; codes "
                      f"{sorted(set(rc for _, rc in fails))}; first indices {[i for i, _ in fails[:12]]}", flush=True)
            for idx, rc in fails[:3]:
                s_, t_ = pairs[idx]
                one = eng.find_path([s_], [t_], [1], 5)
                print(f"   FAILED pair {idx} ({s_}, {t_}) rc {rc}; batch slot {idx % 32}; one-pair: {one}", flush=True)
            if base is None:
                base = got
            same = sum(a == b for a, b in zip(got, base))
            lat = []
            for s, t in pairs[:1000]:
                q0 = time.perf_counter()
                eng.find_path([s], [t], [1], 5)
                lat.append((time.perf_counter() - q0) * 1e3)
            lat = np.array(lat)
            print(f"r{rnd} {spec:40s} failed {len(fails)} batched {len(pairs) / el:9.0f} pairs/s  same-as-first {same}/{len(got)}  "
                  f"one-pair p50 {np.percentile(lat, 50):.4f} p99 {np.percentile(lat, 99):.4f} ms", flush=True)
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
eng.close()
