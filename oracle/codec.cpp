// Test infrastructure (oracle) — key and row codecs restated from the reference.
#include <algorithm>
#include <cmath>
#include "orc.h"

namespace orc {

// ---------------------------------------------------------------- K1
// NebulaKeyUtils::edgeKey (src/common/base/NebulaKeyUtils.cpp:28-47): item = (part<<8)|kData,
// src LE, type|0x40000000 LE, rank LE, dst LE, version (raw 8 bytes, written as given).
std::string edgeKey(int32_t part, int64_t src, int32_t type, int64_t rank, int64_t dst, int64_t ver) {
  std::string k(40, '\0');
  int32_t item = (part << 8) | 1;
  uint32_t t = static_cast<uint32_t>(type) | 0x40000000u;
  memcpy(&k[0], &item, 4);
  memcpy(&k[4], &src, 8);
  memcpy(&k[12], &t, 4);
  memcpy(&k[16], &rank, 8);
  memcpy(&k[24], &dst, 8);
  memcpy(&k[32], &ver, 8);
  return k;
}
// NebulaKeyUtils::edgePrefix (NebulaKeyUtils.cpp:106-117)
std::string edgePrefix(int32_t part, int64_t src, int32_t type) {
  return edgeKey(part, src, type, 0, 0, 0).substr(0, 16);
}
// NebulaKeyUtils::vertexKey (NebulaKeyUtils.cpp:12-26): tag & 0xBFFFFFFF
std::string vertexKey(int32_t part, int64_t vid, int32_t tag, int64_t ver) {
  std::string k(24, '\0');
  int32_t item = (part << 8) | 1;
  uint32_t t = static_cast<uint32_t>(tag) & 0xBFFFFFFFu;
  memcpy(&k[0], &item, 4);
  memcpy(&k[4], &vid, 8);
  memcpy(&k[12], &t, 4);
  memcpy(&k[16], &ver, 8);
  return k;
}
std::string vertexPrefix(int32_t part, int64_t vid, int32_t tag) {
  return vertexKey(part, vid, tag, 0).substr(0, 16);
}
int64_t keySrc(const char* k) { int64_t v; memcpy(&v, k + 4, 8); return v; }
int64_t keyRank(const char* k) { int64_t v; memcpy(&v, k + 16, 8); return v; }
int64_t keyDst(const char* k) { int64_t v; memcpy(&v, k + 24, 8); return v; }
// NebulaKeyUtils::getEdgeType (NebulaKeyUtils.h:146-152): positive types lose bit 30.
int32_t keyType(const char* k) {
  int32_t t; memcpy(&t, k + 12, 4);
  return t > 0 ? (t & static_cast<int32_t>(0xBFFFFFFF)) : t;
}
int32_t keyPart(const char* k) { int32_t v; memcpy(&v, k, 4); return v >> 8; }

// ---------------------------------------------------------------- varint (folly LEB128)
static int encodeVarint(uint64_t v, uint8_t* buf) {
  int n = 0;
  while (v >= 0x80) { buf[n++] = static_cast<uint8_t>(0x80 | (v & 0x7f)); v >>= 7; }
  buf[n++] = static_cast<uint8_t>(v);
  return n;
}
bool decodeVarint(const uint8_t* p, size_t avail, uint64_t& v, int& len) {
  v = 0; len = 0;
  for (int shift = 0; shift < 64 && static_cast<size_t>(len) < avail; shift += 7) {
    uint8_t b = p[len++];
    v |= static_cast<uint64_t>(b & 0x7f) << shift;
    if (!(b & 0x80)) return true;
  }
  return false;
}

// ---------------------------------------------------------------- RowWriter
static int occupiedBytes(uint64_t v) { int b = 0; do { b++; v >>= 8; } while (v); return b; }

void RowWriter::afterWrite() {   // RW_CLEAN_UP_WRITE (RowWriter.h:143-160)
  colNum++;
  if (colNum != 0 && (colNum >> 4 << 4) == colNum) blockOffsets.push_back((int64_t)cord.size());
}
void RowWriter::writeVarint(int64_t v) {
  uint8_t b[10]; int n = encodeVarint(static_cast<uint64_t>(v), b);
  cord.append(reinterpret_cast<char*>(b), n);
}
static SType colTypeAt(RowWriter& w, SType dflt, const char* name) {
  if (w.schema) return w.colNum < (int64_t)w.schema->cols.size() ? w.schema->cols[w.colNum].type : ST_UNKNOWN;
  w.own.cols.push_back({name ? name : ("Column" + std::to_string(w.colNum + 1)), dflt});
  return dflt;
}
RowWriter& RowWriter::putInt(int64_t v, const char* name) {
  SType t = colTypeAt(*this, ST_INT, name);
  if (t == ST_VID) cord.append(reinterpret_cast<char*>(&v), 8);
  else writeVarint((t == ST_INT || t == ST_TIMESTAMP) ? v : 0);
  afterWrite(); return *this;
}
RowWriter& RowWriter::putVid(int64_t v, const char* name) {
  SType t = colTypeAt(*this, ST_VID, name);
  if (t == ST_VID) cord.append(reinterpret_cast<char*>(&v), 8);
  else writeVarint((t == ST_INT || t == ST_TIMESTAMP) ? v : 0);
  afterWrite(); return *this;
}
RowWriter& RowWriter::putBool(bool v, const char* name) {
  SType t = colTypeAt(*this, ST_BOOL, name);
  char c = (t == ST_BOOL) ? (v ? 1 : 0) : 0;
  cord.append(&c, 1);
  afterWrite(); return *this;
}
RowWriter& RowWriter::putDouble(double v, const char* name) {
  SType t = colTypeAt(*this, ST_DOUBLE, name);
  if (t == ST_FLOAT) { float f = static_cast<float>(v); cord.append(reinterpret_cast<char*>(&f), 4); }
  else { double d = (t == ST_DOUBLE) ? v : 0.0; cord.append(reinterpret_cast<char*>(&d), 8); }
  afterWrite(); return *this;
}
RowWriter& RowWriter::putString(const std::string& v, const char* name) {
  SType t = colTypeAt(*this, ST_STRING, name);
  if (t == ST_STRING) { writeVarint((int64_t)v.size()); cord += v; } else writeVarint(0);
  afterWrite(); return *this;
}
RowWriter& RowWriter::putValue(const Value& v, SType t, const char* name) {
  switch (v.index()) {
    case 0: return t == ST_VID ? putVid(std::get<0>(v), name) : putInt(std::get<0>(v), name);
    case 1: return putDouble(std::get<1>(v), name);
    case 2: return putBool(std::get<2>(v), name);
    default: return putString(std::get<3>(v), name);
  }
}
// RowWriter::encodeTo (RowWriter.cpp:49-75); with a schema, missing trailing columns are
// written as defaults (Skip, RowWriter.cpp:202-262).
std::string RowWriter::encode() {
  if (schema) {
    while (colNum < (int64_t)schema->cols.size()) {
      switch (schema->cols[colNum].type) {
        case ST_BOOL: cord.push_back('\0'); break;
        case ST_INT: case ST_TIMESTAMP: writeVarint(0); break;
        case ST_FLOAT: { float f = 0; cord.append(reinterpret_cast<char*>(&f), 4); break; }
        case ST_DOUBLE: { double d = 0; cord.append(reinterpret_cast<char*>(&d), 8); break; }
        case ST_STRING: writeVarint(0); break;
        case ST_VID: { int64_t z = 0; cord.append(reinterpret_cast<char*>(&z), 8); break; }
        default: break;
      }
      colNum++;
      if (colNum != 0 && (colNum >> 4 << 4) == colNum) blockOffsets.push_back((int64_t)cord.size());
    }
  }
  std::string out;
  int offBytes = occupiedBytes(cord.size());
  char header = static_cast<char>(offBytes - 1);
  int64_t ver = sch().version;
  if (ver > 0) {
    int vb = occupiedBytes(static_cast<uint64_t>(ver));
    header |= static_cast<char>(vb << 5);
    out.append(&header, 1);
    out.append(reinterpret_cast<char*>(&ver), vb);
  } else {
    out.append(&header, 1);
  }
  for (auto o : blockOffsets) out.append(reinterpret_cast<char*>(&o), offBytes);
  out += cord;
  return out;
}

// ---------------------------------------------------------------- RowReader
// RowReader::getSchemaVer (RowReader.cpp:172-200)
int32_t rowSchemaVer(std::string_view row) {
  if (row.empty()) return 0;
  const uint8_t* it = reinterpret_cast<const uint8_t*>(row.data());
  size_t vb = it[0] >> 5;
  int32_t ver = 0;
  if (vb > 0) {
    if (vb + 1 > row.size()) return 0;
    for (size_t i = 0; i < vb; ++i) ver |= (uint32_t(it[1 + i]) << (8 * i));
  }
  return ver;
}

// RowReader::processHeader (RowReader.cpp:217-258)
RowReader::RowReader(std::string_view row, const Schema* s) : schema(s) {
  if (row.empty() || !s) return;
  const uint8_t* it = reinterpret_cast<const uint8_t*>(row.data());
  int offBytes = (it[0] & 0x07) + 1;
  int vb = it[0] >> 5;
  size_t numOffsets = s->cols.size() >> 4;
  if (offBytes * numOffsets + vb + 1 > row.size()) return;
  size_t hdr = 1 + vb + offBytes * numOffsets;
  data = it + hdr;
  len = row.size() - hdr;
  offsets.assign(1, 0);
  valid = true;
}

static int fieldWidth(SType t, const uint8_t* p, size_t avail, bool& ok) {
  ok = true;
  switch (t) {
    case ST_BOOL: return 1;
    case ST_INT: case ST_TIMESTAMP: {
      uint64_t v; int n; ok = decodeVarint(p, avail, v, n); return n;
    }
    case ST_FLOAT: return 4;
    case ST_DOUBLE: return 8;
    case ST_VID: return 8;
    case ST_STRING: {
      uint64_t v; int n; ok = decodeVarint(p, avail, v, n); return n + (int)v;
    }
    default: ok = false; return 0;
  }
}

bool RowReader::fieldOffset(int idx, int64_t& off) {
  while ((int)offsets.size() <= idx) {
    int i = (int)offsets.size() - 1;
    int64_t o = offsets.back();
    if (o > (int64_t)len) return false;
    bool ok;
    int w = fieldWidth(schema->cols[i].type, data + o, len - o, ok);
    if (!ok || o + w > (int64_t)len) return false;
    offsets.push_back(o + w);
  }
  off = offsets[idx];
  return true;
}

OptValue RowReader::getIdx(int idx) {
  if (!valid || idx < 0 || idx >= (int)schema->cols.size()) return Status::Err("bad field");
  int64_t off;
  if (!fieldOffset(idx, off)) return Status::Err("E_DATA_INVALID");
  const uint8_t* p = data + off;
  size_t avail = len - off;
  switch (schema->cols[idx].type) {
    case ST_BOOL: if (avail < 1) break; return Value(p[0] != 0);
    case ST_INT: case ST_TIMESTAMP: {
      uint64_t v; int n; if (!decodeVarint(p, avail, v, n)) break;
      return Value(static_cast<int64_t>(v));
    }
    case ST_VID: { if (avail < 8) break; int64_t v; memcpy(&v, p, 8); return Value(v); }
    case ST_FLOAT: { if (avail < 4) break; float f; memcpy(&f, p, 4); return Value(static_cast<double>(f)); }
    case ST_DOUBLE: { if (avail < 8) break; double d; memcpy(&d, p, 8); return Value(d); }
    case ST_STRING: {
      uint64_t v; int n; if (!decodeVarint(p, avail, v, n)) break;
      if (n + v > avail) break;
      return Value(std::string(reinterpret_cast<const char*>(p + n), v));
    }
    default: break;
  }
  return Status::Err("E_DATA_INVALID");
}

OptValue RowReader::get(const std::string& name) {
  int i = schema ? schema->find(name) : -1;
  if (i < 0) return Status::Err("prop not found: " + name);
  return getIdx(i);
}

OptValue defaultProp(const Schema& s, const std::string& prop) {
  switch (s.typeOf(prop)) {
    case ST_BOOL: return Value(false);
    case ST_TIMESTAMP: case ST_INT: case ST_VID: return Value(int64_t(0));
    case ST_FLOAT: case ST_DOUBLE: return Value(0.0);
    case ST_STRING: return Value(std::string());
    default: return Status::Err("Unknown type");
  }
}

// RowSetWriter::addRow (RowSetWriter.cpp:21-43): varint(row length) + row
void rowSetAdd(std::string& rs, const std::string& row) {
  uint8_t b[10]; int n = encodeVarint(row.size(), b);
  rs.append(reinterpret_cast<char*>(b), n);
  rs += row;
}
std::vector<std::string> rowSetSplit(const std::string& rs) {
  std::vector<std::string> out;
  size_t off = 0;
  while (off < rs.size()) {
    uint64_t len; int n;
    if (!decodeVarint(reinterpret_cast<const uint8_t*>(rs.data()) + off, rs.size() - off, len, n)) break;
    out.emplace_back(rs.substr(off + n, len));
    off += n + len;
  }
  return out;
}

}  // namespace orc
