"""SST-file ingest: RocksDB BlockBasedTable files as the reference's Spark
generator writes them (SstFileOutputFormat.scala:150-202) loaded through nbg_ingest_sst /
nbg_ingest_dir (NebulaStore::ingest, src/kvstore/NebulaStore.cpp:436-466).

The files come from tests/support/sstwriter.py (the published table format restated; no RocksDB
in this image, so parity against RocksDB-written bytes is unpinned).  The CPU tests check the
reader's acceptance and error codes through the C ABI (parsing, checksums and Snappy decoding
run before any device work); the GPU tests check that an ingested engine answers exactly like
one loaded with nbg_load_part_kv from the same records, and the reference's golden cases."""
import os

import numpy as np
import pytest

from nebula_amd import Engine, LocalCluster, NbgError, _lib, expr as E, kvgen
from tests.support import golden, graphs, sstwriter


def _kv(n=300, seed=3):
    kb = kvgen.KVBuilder(3)
    rng = np.random.default_rng(seed)
    now = 1_600_000_000_000_000
    for i in range(n):
        s, d = int(rng.integers(1, 50)), int(rng.integers(1, 50))
        kb.insert_edge(s, d, graphs.E_TYPE, 0, graphs.E_SCHEMA, [int(rng.integers(0, 100))], now + i)
    return kb


def _records(kb, part):
    return [(bytes(k), bytes(v)) for k, v in kb.recs[part]]


def _code(fn):
    try:
        fn()
        return 0
    except NbgError as ex:
        return ex.code


def _engine():
    e = Engine(3)
    e.register_edge(graphs.E_TYPE, "e", graphs.E_SCHEMA)
    return e


# --------------------------------------------------------------------------- CPU: format checks
def test_crc32c_known_answers():
    assert sstwriter.crc32c(b"123456789") == 0xE3069283          # the Castagnoli check value
    assert sstwriter.crc32c(b"\x00" * 32) == 0x8A9136AA             # RFC 3720 B.4 vectors
    assert sstwriter.crc32c(b"\xff" * 32) == 0x62A8AB43
    assert sstwriter.crc32c(bytes(range(32))) == 0x46DD794E


@pytest.mark.parametrize("kw", [dict(), dict(compression=None), dict(legacy_footer=True),
                                dict(block_size=256, restart_interval=4), dict(format_version=3)])
def test_valid_files_are_accepted(tmp_path, kw):
    kb = _kv()
    e = _engine()
    try:
        for part in kb.recs:
            p = sstwriter.write_sst(str(tmp_path / f"{part}.sst"), _records(kb, part), **kw)
            e.ingest_sst(part, p)
    finally:
        e.close()


def test_snappy_blocks_are_compressed(tmp_path):
    # the writer's Snappy path is taken (so the reader's decoder is exercised by the tests above)
    kb = _kv(2000)
    recs = _records(kb, 1)
    a = sstwriter.write_sst(str(tmp_path / "a.sst"), recs)
    b = sstwriter.write_sst(str(tmp_path / "b.sst"), recs, compression=None)
    assert os.path.getsize(a) < 0.8 * os.path.getsize(b)


@pytest.mark.parametrize("damage, code", [
    ("flip", _lib.E_INVALID_ARGUMENT),        # a data byte: block checksum mismatch
    ("truncate", _lib.E_INVALID_ARGUMENT),    # footer gone: not an SST file
    ("garbage", _lib.E_INVALID_ARGUMENT),
    ("codec", _lib.E_UNSUPPORTED),            # a block compressed with a codec other than Snappy
    ("delete", _lib.E_UNSUPPORTED),           # a Delete record (SstFileWriter::Delete)
    ("version", _lib.E_UNSUPPORTED),          # format_version 4 (delta-encoded index values)
    ("missing", _lib.E_INVALID_ARGUMENT),
])
def test_bad_files_fail(tmp_path, damage, code):
    kb = _kv()
    recs = _records(kb, 1)
    p = str(tmp_path / "x.sst")
    if damage == "codec":
        sstwriter.write_sst(p, recs, compression="zlib-marker")
    elif damage == "delete":
        sstwriter.write_sst(p, recs, value_type=0)
    elif damage == "version":
        sstwriter.write_sst(p, recs, format_version=4)
    elif damage != "missing":
        sstwriter.write_sst(p, recs, compression=None)
        raw = bytearray(open(p, "rb").read())
        if damage == "flip":
            raw[10] ^= 0x40
        elif damage == "truncate":
            raw = raw[:-20]
        else:
            raw = bytearray(os.urandom(len(raw)))
        open(p, "wb").write(bytes(raw))
    e = _engine()
    try:
        with pytest.raises(NbgError) as ex:
            e.ingest_sst(1, p)
        assert ex.value.code == code and "x.sst" in str(ex.value)
    finally:
        e.close()


def test_ingest_dir_layout_and_part_range(tmp_path):
    kb = _kv()
    sstwriter.write_download_dir(str(tmp_path), kb, files_per_part=3)
    os.makedirs(tmp_path / "9" / "nested")   # a part this space does not have: never visited
    e = _engine()
    try:
        e.ingest_dir(str(tmp_path))
        e.ingest_dir(str(tmp_path / "absent"))   # no download dir: nothing to ingest
        assert _code(lambda: e.ingest_sst(4, str(tmp_path / "1" / "x.sst"))) == _lib.E_PART_NOT_FOUND
    finally:
        e.close()


# --------------------------------------------------------------------------- GPU: loaded == ingested
def _tagged_from_sst(root, scale=9, parts=7, world=1):
    _, _, kb = graphs.tagged_kv(scale, parts)
    sstwriter.write_download_dir(root, kb, files_per_part=2)
    if world == 1:
        e = Engine(parts)
        graphs.tagged_register(e, True)
        e.ingest_dir(root)
        e.finalize()
        return e
    c = LocalCluster(parts, world)
    graphs.tagged_register(c, True)
    c.ingest_dir(root)
    c.finalize()
    return c


@pytest.mark.gpu
def test_ingested_engine_equals_kv_loaded(tmp_path):
    src, persons, loaded, orc = graphs.tagged_pair(9)
    ing = _tagged_from_sst(str(tmp_path))
    try:
        yields = [E.edge_prop("e", "_dst").encode(), E.edge_prop("e", "w").encode(),
                  E.src_prop("person", "name").encode(), E.dst_prop("person", "age").encode()]
        where = E.binop("<", E.edge_prop("e", "w"), E.const(60)).encode()
        checked = 0
        for r in graphs.roots(src, 6, seed=8):
            for steps in (1, 2, 3):
                for wb in (b"", where):
                    try:
                        exp = graphs.sorted_rows(loaded.go([r], [graphs.E_TYPE], steps, wb, yields))
                    except NbgError as ex:
                        assert _code(lambda: ing.go([r], [graphs.E_TYPE], steps, wb, yields)) == ex.code
                        continue
                    got = graphs.sorted_rows(ing.go([r], [graphs.E_TYPE], steps, wb, yields))
                    assert got == exp, (r, steps)
                    checked += 1
        assert checked > 0
        for s, t in zip(graphs.roots(src, 6, seed=1), graphs.roots(src, 6, seed=2)):
            for shortest in (True, False):
                assert ing.find_path([s], [t], [graphs.E_TYPE, graphs.E_F], 3, shortest=shortest) == \
                    loaded.find_path([s], [t], [graphs.E_TYPE, graphs.E_F], 3, shortest=shortest)
    finally:
        ing.close()
        loaded.close()
        orc.close()


@pytest.mark.gpu
def test_ingested_partitioned_cluster_equals_single(tmp_path):
    src, persons, loaded, orc = graphs.tagged_pair(9)
    c = _tagged_from_sst(str(tmp_path), world=3)
    try:
        for r in graphs.roots(src, 4, seed=4):
            for steps in (1, 3):
                got = graphs.sorted_rows(c.go([r], [graphs.E_TYPE, graphs.E_F], steps))
                assert got == graphs.sorted_rows(loaded.go([r], [graphs.E_TYPE, graphs.E_F], steps)), r
    finally:
        c.close()
        loaded.close()
        orc.close()


@pytest.mark.gpu
def test_ingested_nba_golden(tmp_path, nba_data):
    """The reference's GoTest / FindPathTest golden cases on the nba space ingested from SST files."""
    parts = 7
    sstwriter.write_download_dir(str(tmp_path), kvgen.nba_kv(nba_data, parts), files_per_part=2)
    e = Engine(parts)
    for (kind, name), cols in kvgen.NBA_SCHEMAS.items():
        if kind == "edge":
            e.register_edge(kvgen.NBA_EDGES[name], name, cols)
        else:
            e.register_tag(kvgen.NBA_TAGS[name], name, cols)
    e.ingest_dir(str(tmp_path))
    e.finalize()
    try:
        checked = 0
        for fname, run in (("go_golden.json", golden.run_go_case), ("findpath_golden.json", golden.run_path_case)):
            for case in golden.load(fname):
                if golden.unsupported_reason(case):
                    continue
                ok, msg = run(e, case)
                assert ok, msg
                checked += 1
        assert checked > 20
    finally:
        e.close()
