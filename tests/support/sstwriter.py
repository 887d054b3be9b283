"""Test infrastructure: a writer of RocksDB BlockBasedTable SST files, as rocksdb::SstFileWriter
(5.x, default Options: 4 KiB blocks, restart interval 16, format_version 2, crc32c checksums,
Snappy block compression when it saves at least 1/8) writes them for the reference's Spark
generator (src/tools/spark-sstfile-generator/.../SstFileOutputFormat.scala:150-202).

RocksDB is not in this image, so this restates the published table format (see the header of
nebula_amd/csrc/sst.cpp for the layout); the ingest tests write KV records with it and check that
nbg_ingest_* loads exactly what nbg_load_part_kv loads.  Parity against bytes written by a real
RocksDB is unpinned (no SST fixture exists in the reference).  Also a Snappy block encoder
(greedy, 4-byte hash matches) and the crc32c the format uses.
"""
from __future__ import annotations

import os
import struct

MAGIC = 0x88E241B785F4CFF7
LEGACY_MAGIC = 0xDB4775248B80FB57


def _crc_table():
    t = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ (0x82F63B78 if c & 1 else 0)
        t.append(c)
    return t


_T = _crc_table()


def crc32c(data: bytes, crc: int = 0) -> int:
    crc ^= 0xFFFFFFFF
    for b in data:
        crc = _T[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def crc_mask(c: int) -> int:
    return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


def varint(v: int) -> bytes:
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def snappy_compress(data: bytes) -> bytes:
    """Snappy block format: literals and 2-byte-offset copies found through a 4-byte hash."""
    out = bytearray(varint(len(data)))
    n, i, lit = len(data), 0, 0
    table = {}

    def literal(a, b):
        while a < b:
            k = min(b - a, 65536)
            if k <= 60:
                out.append((k - 1) << 2)
            elif k <= 256:
                out.extend(bytes([60 << 2, k - 1]))
            else:
                out.extend(bytes([61 << 2]) + struct.pack("<H", k - 1))
            out.extend(data[a:a + k])
            a += k

    while i + 4 <= n:
        key = data[i:i + 4]
        j = table.get(key)
        table[key] = i
        if j is not None and i - j < 65536:
            m = 4
            while i + m < n and data[j + m] == data[i + m] and m < 64:
                m += 1
            literal(lit, i)
            out.append(((m - 1) << 2) | 2)
            out += struct.pack("<H", i - j)
            i += m
            lit = i
        else:
            i += 1
    literal(lit, n)
    return bytes(out)


def _block(entries, restart_interval):
    """entries: [(key, value)] in order -> prefix-compressed block contents."""
    buf, restarts, prev = bytearray(), [], b""
    for k, (key, val) in enumerate(entries):
        if k % restart_interval == 0:
            restarts.append(len(buf))
            shared = 0
        else:
            shared = 0
            while shared < min(len(prev), len(key)) and prev[shared] == key[shared]:
                shared += 1
        buf += varint(shared) + varint(len(key) - shared) + varint(len(val)) + key[shared:] + val
        prev = key
    if not restarts:
        restarts = [0]
    for r in restarts:
        buf += struct.pack("<I", r)
    buf += struct.pack("<I", len(restarts))
    return bytes(buf)


class SstWriter:
    def __init__(self, path, compression="snappy", block_size=4096, restart_interval=16, format_version=2,
                 legacy_footer=False, value_type=1):
        self.path = path
        self.compression = compression
        self.block_size = block_size
        self.restart_interval = restart_interval
        self.format_version = format_version
        self.legacy_footer = legacy_footer
        self.value_type = value_type
        self.out = bytearray()
        self.pending = []
        self.pending_bytes = 0
        self.index = []
        self.last = None

    def _write_block(self, contents, compress):
        ctype, body = 0, contents
        if compress == "snappy":
            c = snappy_compress(contents)
            if len(c) < len(contents) - len(contents) // 8:   # GoodCompressionRatio
                ctype, body = 1, c
        elif compress == "zlib-marker":   # an unsupported codec tag (the reader must refuse it)
            ctype = 2
        off = len(self.out)
        crc = crc_mask(crc32c(body + bytes([ctype])))
        self.out += body + bytes([ctype]) + struct.pack("<I", crc)
        return off, len(body)

    def _flush(self):
        if not self.pending:
            return
        off, size = self._write_block(_block(self.pending, self.restart_interval), self.compression)
        self.index.append((self.pending[-1][0], varint(off) + varint(size)))
        self.pending, self.pending_bytes = [], 0

    def put(self, key: bytes, value: bytes):
        if self.last is not None and key <= self.last:
            raise ValueError("keys must be strictly increasing (SstFileWriter)")
        self.last = key
        ikey = key + struct.pack("<Q", (0 << 8) | self.value_type)
        self.pending.append((ikey, value))
        self.pending_bytes += len(ikey) + len(value) + 8
        if self.pending_bytes >= self.block_size:
            self._flush()

    def finish(self):
        self._flush()
        meta_off, meta_size = self._write_block(_block([], 1), None)
        idx_off, idx_size = self._write_block(_block(self.index, 1), None)
        handles = varint(meta_off) + varint(meta_size) + varint(idx_off) + varint(idx_size)
        if self.legacy_footer:
            self.out += handles.ljust(40, b"\0") + struct.pack("<Q", LEGACY_MAGIC)
        else:
            self.out += bytes([1]) + handles.ljust(40, b"\0") + struct.pack("<I", self.format_version)
            self.out += struct.pack("<Q", MAGIC)
        with open(self.path, "wb") as f:
            f.write(self.out)
        return self.path


def write_sst(path, records, **kw):
    """records: (key, value) pairs; sorted and de-duplicated (last wins) as the generator's
    partition sort leaves them, then written as one file."""
    d = {}
    for k, v in records:
        d[bytes(k)] = bytes(v)
    w = SstWriter(path, **kw)
    for k in sorted(d):
        w.put(k, d[k])
    return w.finish()


def write_download_dir(root, kb, files_per_part=2, **kw):
    """A KVBuilder's records as the generator lays them out: <root>/<part>/vertex-*.sst and
    edge-*.sst (24-byte keys are vertices, 40-byte keys edges), each kind split over
    `files_per_part` files of disjoint key ranges."""
    for part, recs in kb.recs.items():
        pdir = os.path.join(root, str(part))
        os.makedirs(pdir, exist_ok=True)
        for kind, klen in (("vertex", 24), ("edge", 40)):
            rs = {}
            for k, v in recs:
                if len(k) == klen:
                    rs[bytes(k)] = bytes(v)
            keys = sorted(rs)
            if not keys:
                continue
            step = max(1, -(-len(keys) // files_per_part))
            for i in range(0, len(keys), step):
                chunk = keys[i:i + step]
                write_sst(os.path.join(pdir, f"{kind}-{chunk[0].hex()}.sst"), [(k, rs[k]) for k in chunk], **kw)
