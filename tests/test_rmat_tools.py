"""The bench's synthetic-graph tooling (CPU): the C++ RMAT generator equals the numpy one, and the
per-rank generator of a partitioned bench run keeps exactly the samples its rank's loader keeps
(source or destination in one of its parts), in sample order."""
import numpy as np
import pytest

from nebula_amd import rmat


def test_fast_generator_matches_numpy():
    a = rmat.rmat_edges(10)
    b = rmat.rmat_edges_fast(10)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("gpus", [2, 3, 8])
def test_owned_samples_per_rank(gpus):
    src, dst, w = rmat.rmat_edges_fast(12)
    parts = 100
    seen = np.zeros(len(src), np.int64)
    for r in range(gpus):
        s, d, x = rmat.rmat_edges_owned(12, parts, gpus, r)
        own = lambda v: ((v.astype(np.uint64) % np.uint64(parts) + np.uint64(1)) % np.uint64(gpus)) == r
        keep = own(src) | own(dst)
        assert np.array_equal(s, src[keep]) and np.array_equal(d, dst[keep]) and np.array_equal(x, w[keep])
        seen += own(src)
    assert (seen == 1).all()   # every out-edge is owned by exactly one rank
