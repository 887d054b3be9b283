"""Build storaged-format KV records (NebulaKeyUtils keys + RowWriter values) for fixtures.

These are exactly the bytes the reference's write path leaves in RocksDB:
  * ``InsertEdgeExecutor`` writes an out-edge ``(src, +type, rank, dst)`` carrying the row and
    an in-edge ``(dst, -type, rank, src)`` with an EMPTY value
    (src/graph/InsertEdgeExecutor.cpp:180-196);
  * ``AddEdgesProcessor`` keys them with ``version = bigEndian(INT64_MAX - now_us)``
    (src/storage/AddEdgesProcessor.cpp:15-37);
  * keys live in the partition of their first vid: ``part = uint64(vid) % parts + 1``
    (src/storage/client/StorageClient.cpp:10-11,402-407).
Used by tests (nba fixture, QueryBoundTest-style mock data) and small examples; large
synthetic graphs come from the C++ generator (nebula_amd.tools).
"""
from __future__ import annotations

import struct
from collections import defaultdict
from typing import Dict, List, Sequence, Tuple

import numpy as np

from .vidhash import std_hash

# common.thrift SupportedType
BOOL, INT, VID, FLOAT, DOUBLE, STRING, TIMESTAMP = 1, 2, 3, 4, 5, 6, 7
INT64_MAX = (1 << 63) - 1


def part_of(vid: int, parts: int) -> int:
    return (vid & ((1 << 64) - 1)) % parts + 1


def version_of(now_us: int) -> int:
    """bigEndian(INT64_MAX - now_us) as the raw int64 stored in the key."""
    v = INT64_MAX - now_us
    return struct.unpack("<q", struct.pack(">q", v))[0]


def edge_key(part: int, src: int, etype: int, rank: int, dst: int, ver: int) -> bytes:
    return struct.pack("<iqIqqq", (part << 8) | 1, src, (etype & 0xFFFFFFFF) | 0x40000000,
                       rank, dst, ver)


def vertex_key(part: int, vid: int, tag: int, ver: int) -> bytes:
    return struct.pack("<iqIq", (part << 8) | 1, vid, tag & 0xBFFFFFFF, ver)


def _varint(v: int) -> bytes:
    v &= (1 << 64) - 1
    out = bytearray()
    while v >= 0x80:
        out.append(0x80 | (v & 0x7F))
        v >>= 7
    out.append(v)
    return bytes(out)


def encode_row(schema: Sequence[Tuple[str, int]], values: Sequence, schema_ver: int = 0) -> bytes:
    """RowWriter(schema) << values...; encode() (src/dataman/RowWriter.cpp:49-75)."""
    cord = bytearray()
    offsets = []
    for i, ((_, t), v) in enumerate(zip(schema, values)):
        if t in (INT, TIMESTAMP):
            cord += _varint(int(v))
        elif t == VID:
            cord += struct.pack("<q", int(v))
        elif t == BOOL:
            cord += b"\x01" if v else b"\x00"
        elif t == FLOAT:
            cord += struct.pack("<f", float(v))
        elif t == DOUBLE:
            cord += struct.pack("<d", float(v))
        elif t == STRING:
            b = v.encode() if isinstance(v, str) else bytes(v)
            cord += _varint(len(b)) + b
        else:
            raise ValueError(t)
        n = i + 1
        if n % 16 == 0:
            offsets.append(len(cord))
    ob = max(1, (len(cord).bit_length() + 7) // 8)
    header = ob - 1
    out = bytearray()
    if schema_ver > 0:
        vb = max(1, (schema_ver.bit_length() + 7) // 8)
        out.append(header | (vb << 5))
        out += schema_ver.to_bytes(vb, "little")
    else:
        out.append(header)
    for o in offsets:
        out += o.to_bytes(ob, "little")
    return bytes(out + cord)


class KVBuilder:
    """Accumulates KV records per part, in write order."""

    def __init__(self, parts: int):
        self.parts = parts
        self.recs: Dict[int, List[Tuple[bytes, bytes]]] = defaultdict(list)

    def put(self, part: int, key: bytes, val: bytes):
        self.recs[part].append((key, val))

    def insert_vertex(self, vid: int, tag: int, schema, values, now_us: int):
        p = part_of(vid, self.parts)
        self.put(p, vertex_key(p, vid, tag, version_of(now_us)), encode_row(schema, values))

    def insert_edge(self, src: int, dst: int, etype: int, rank: int, schema, values, now_us: int):
        ver = version_of(now_us)
        ps = part_of(src, self.parts)
        self.put(ps, edge_key(ps, src, etype, rank, dst, ver), encode_row(schema, values))
        pd = part_of(dst, self.parts)
        self.put(pd, edge_key(pd, dst, -etype, rank, src, ver), b"")

    def flat(self, part: int):
        """(key_data u8, key_offs u64[n+1], val_data u8, val_offs u64[n+1], n)"""
        recs = self.recs.get(part, [])
        kd = b"".join(k for k, _ in recs)
        vd = b"".join(v for _, v in recs)
        ko = np.zeros(len(recs) + 1, np.uint64)
        vo = np.zeros(len(recs) + 1, np.uint64)
        if recs:
            ko[1:] = np.cumsum([len(k) for k, _ in recs])
            vo[1:] = np.cumsum([len(v) for _, v in recs])
        return (np.frombuffer(kd, np.uint8).copy() if kd else np.zeros(1, np.uint8), ko,
                np.frombuffer(vd, np.uint8).copy() if vd else np.zeros(1, np.uint8), vo, len(recs))


# ------------------------------------------------------------------------------ nba fixture
NBA_SPACE = 1
NBA_TAGS = {"player": 2, "team": 3}
NBA_EDGES = {"serve": 4, "like": 5}
NBA_SCHEMAS = {
    ("tag", "player"): [("name", STRING), ("age", INT)],
    ("tag", "team"): [("name", STRING)],
    ("edge", "serve"): [("start_year", INT), ("end_year", INT)],
    ("edge", "like"): [("likeness", INT)],
}


def nba_kv(data: dict, parts: int = 1, now_us: int = 1_600_000_000_000_000) -> KVBuilder:
    """TraverseTestBase::prepareData as KV records (one INSERT per statement → one version)."""
    kb = KVBuilder(parts)
    pv = {p["name"]: std_hash(p["name"]) for p in data["players"]}
    tv = {t["name"]: std_hash(t["name"]) for t in data["teams"]}
    for p in data["players"]:
        kb.insert_vertex(pv[p["name"]], NBA_TAGS["player"], NBA_SCHEMAS[("tag", "player")],
                         [p["name"], p["age"]], now_us)
    for t in data["teams"]:
        kb.insert_vertex(tv[t["name"]], NBA_TAGS["team"], NBA_SCHEMAS[("tag", "team")],
                         [t["name"]], now_us + 1)
    for who, team, a, b in data["serve"]:
        kb.insert_edge(pv[who], tv[team], NBA_EDGES["serve"], 0, NBA_SCHEMAS[("edge", "serve")],
                       [a, b], now_us + 2)
    for who, other, n in data["like"]:
        kb.insert_edge(pv[who], pv[other], NBA_EDGES["like"], 0, NBA_SCHEMAS[("edge", "like")],
                       [n], now_us + 3)
    return kb
