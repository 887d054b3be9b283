"""Pin the CPU oracle against the reference's own known answers (FindPathTest.cpp, GoTest.cpp)
over the TraverseTestBase dataset.  CPU only."""
import pytest

from nebula_amd.vidhash import std_hash
from tests.support import golden
from tests.support.oracle import nba_oracle

FIND = golden.load("findpath_golden.json")
GO = golden.load("go_golden.json")


@pytest.fixture(scope="module")
def orc(nba_data):
    o = nba_oracle(nba_data)
    yield o
    o.close()


def test_vid_hash_pins():
    # std::hash<std::string> with libstdc++ (TraverseTestBase.h:111,233)
    assert std_hash("Tim Duncan") == 5662213458193308137
    assert std_hash("Tony Parker") == -7579316172763586624
    assert std_hash("Spurs") == 7193291116733635180


def test_dataset_counts(nba_data):
    # S19: 152 listed serve edges (146 unique) and 82 listed like edges (81 unique)
    assert len(nba_data["serve"]) == 152
    assert len(nba_data["like"]) == 82
    assert len({(a, b) for a, b, *_ in nba_data["serve"]}) == 146
    assert len({(a, b) for a, b, *_ in nba_data["like"]}) == 81


@pytest.mark.parametrize("case", FIND, ids=[f"{c['test']}-{i}" for i, c in enumerate(FIND)])
def test_findpath_faithful(orc, case):
    ok, msg = golden.run_path_case(orc, case)
    assert ok, msg


class _Bfs:
    """Backend adapter: the canonical-BFS SHORTEST restatement."""

    def __init__(self, o):
        self.o = o
        self.edge_types, self.edge_names = o.edge_types, o.edge_names

    def go(self, **kw):
        return self.o.go(**kw)

    def find_path(self, frm, to, etypes, upto=5, shortest=True):
        return self.o.find_path(frm, to, etypes, upto, shortest, mode=1)


@pytest.mark.parametrize("case", [c for c in FIND if "SHORTEST" in c["query"]],
                         ids=lambda c: c["query"][:60])
def test_findpath_canonical_bfs(orc, case):
    ok, msg = golden.run_path_case(_Bfs(orc), case)
    assert ok, msg


@pytest.mark.parametrize("case", GO, ids=[f"{c['test']}-{i}" for i, c in enumerate(GO)])
def test_go_golden(orc, case):
    why = golden.unsupported_reason(case)
    if why:
        pytest.skip(why)
    ok, msg = golden.run_go_case(orc, case)
    assert ok, msg
