"""Partitioned SHORTEST with NBG_PART_FWD_BSETS=1 (true B-sets past kf, forward from the meet
set, before the greedy): paths and scanned-edge counts equal the single engine's.  The switch is
read once per process, so tests/test_gpu_partitioned.py runs this file in a child process with the
variable set before any GPU call."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    assert os.environ.get("NBG_PART_FWD_BSETS") == "1"
    from nebula_amd import LocalCluster, rmat
    from tests.support import graphs
    ok, found = True, 0
    for scale, world, npairs in ((11, 2, 24), (16, 2, 24), (16, 3, 12)):
        src, dst, w = graphs.rmat_graph(scale)
        single = graphs.one_sided_engine(src, dst, w)
        c = LocalCluster(100, world)
        c.set_path_replica(0)
        c.register_edge(graphs.E_TYPE, "e", graphs.E_SCHEMA)
        c.load_edges(graphs.E_TYPE, src, dst, [w])
        c.finalize()
        try:
            for s, t in rmat.pick_pairs(src, dst, npairs, seed=40 + scale):
                for upto in (3, 5):
                    st, st1 = {}, {}
                    got = c.find_path([s], [t], [1], upto, stats=st)
                    ref = single.find_path([s], [t], [1], upto, stats=st1)
                    good = got == ref and st["edges"] == st1["edges"]
                    ok &= good
                    found += len(got)
                    if not good:
                        print(f"MISMATCH scale {scale} G={world} {s}->{t} upto {upto}: {got} vs {ref}", flush=True)
        finally:
            c.close()
            single.close()
    print(f"fwd B-sets probe: {found} paths,", "PASS" if ok and found else "FAIL", flush=True)
    sys.exit(0 if ok and found else 1)


if __name__ == "__main__":
    main()
