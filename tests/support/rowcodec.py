"""RowReader / RowSetReader restated for test assertions (src/dataman/RowReader.cpp:140-420,
RowSetReader.cpp:20-80): decode a row of a known column-type list, and split a RowSet.
Test infrastructure only (the product encodes rows in getneighbors.cpp)."""
import struct

from nebula_amd.kvgen import BOOL, DOUBLE, FLOAT, INT, STRING, TIMESTAMP, VID


def _varint(b, pos):
    v, shift = 0, 0
    while True:
        c = b[pos]
        pos += 1
        v |= (c & 0x7F) << shift
        shift += 7
        if not c & 0x80:
            break
    if v >= 1 << 63:
        v -= 1 << 64
    return v, pos


def header(row: bytes, ncols: int):
    """(schema version, block offsets, header length): byte 0 = (offset width - 1) | (version
    bytes << 5), then the version, then one offset per 16 fields."""
    h = row[0]
    ob, vb = (h & 0x07) + 1, h >> 5
    pos = 1
    ver = int.from_bytes(row[pos:pos + vb], "little") if vb else 0
    pos += vb
    offs = []
    for _ in range(ncols // 16):
        offs.append(int.from_bytes(row[pos:pos + ob], "little"))
        pos += ob
    return ver, offs, pos


def decode_row(row: bytes, types):
    """Field values of one row, per the column types (INT/TIMESTAMP varint, VID 8 bytes, BOOL one
    byte, FLOAT 4, DOUBLE 8, STRING varint length + bytes)."""
    _, _, pos = header(row, len(types))
    out = []
    for t in types:
        if t in (INT, TIMESTAMP):
            v, pos = _varint(row, pos)
        elif t == VID:
            v = struct.unpack_from("<q", row, pos)[0]
            pos += 8
        elif t == BOOL:
            v = row[pos] != 0
            pos += 1
        elif t == FLOAT:
            v = struct.unpack_from("<f", row, pos)[0]
            pos += 4
        elif t == DOUBLE:
            v = struct.unpack_from("<d", row, pos)[0]
            pos += 8
        elif t == STRING:
            n, pos = _varint(row, pos)
            v = row[pos:pos + n].decode()
            pos += n
        else:
            raise ValueError(t)
        out.append(v)
    return out


def split_rowset(rs: bytes):
    """The rows of a RowSet (each prefixed by its varint length)."""
    rows, pos = [], 0
    while pos < len(rs):
        n, pos = _varint(rs, pos)
        rows.append(rs[pos:pos + n])
        pos += n
    return rows


def value_kinds(types):
    """The column types a schema-less RowWriter uses for values decoded from these types
    (RowReader::getPropByName -> VariantType -> PropsCollector, QueryBaseProcessor.inl:300-350):
    int64 for INT / VID / TIMESTAMP, double for FLOAT / DOUBLE."""
    m = {VID: INT, TIMESTAMP: INT, FLOAT: DOUBLE}
    return [m.get(t, t) for t in types]
