// SST-file ingest: the loader source behind the reference's bulk import.
//
// Reference path: the Spark generator writes one RocksDB SST file per (part, vertex|edge) with
// rocksdb::SstFileWriter and default Options (rocksdbjni 5.17.2;
// src/tools/spark-sstfile-generator/src/main/scala/com/vesoft/tools/SstFileOutputFormat.scala:150-202:
// keys are NebulaKeyUtils keys, values RowWriter rows, strictly increasing per file).  The files
// are downloaded to <data>/download/<part>/ and StorageHttpIngestHandler (src/storage/
// StorageHttpIngestHandler.cpp:45-100) calls NebulaStore::ingest (src/kvstore/NebulaStore.cpp:
// 436-466): for every part of the space, every "*.sst" under download/<part> goes through
// RocksEngine::ingest (src/kvstore/RocksEngine.cpp:360-370) = DB::IngestExternalFile, which gives
// the file a sequence number above everything already in the part (a later file's key wins).
//
// RocksDB itself is not part of this image, so the table is read here from its published on-disk
// format (BlockBasedTable, format_version 0-3 as written by 5.x):
//   [data blocks][meta blocks][metaindex block][index block][footer]
//   every block = contents + 1-byte compression type + fixed32 masked crc32c(contents ‖ type)
//   block contents = entries {varint32 shared, varint32 non_shared, varint32 value_len,
//                    key delta, value} + fixed32 restarts[] + fixed32 num_restarts
//   footer (53 B, format_version >= 1) = checksum type, metaindex handle, index handle, zero
//   padding to 41 B, fixed32 format_version, fixed64 magic 0x88e241b785f4cff7;
//   legacy footer (48 B) = two handles padded to 40 B, magic 0xdb4775248b80fb57
//   index block entries map a separator key to the BlockHandle {varint64 offset, varint64 size}
//   of one data block; data-block keys are internal keys: user key ‖ fixed64(seq << 8 | type).
// Compression: none and Snappy (rocksdb's default when built with it, as rocksdbjni is) are
// decoded here; other codecs fail the ingest with NBG_E_UNSUPPORTED.  Only Put records
// (type 1, all SstFileWriter::Put writes) are accepted.
//
// The decoded records are handed to Engine::load_part_kv in file order, files in name order, so
// ingesting is exactly loading the same KV records (an identical key in a later file overwrites).
#include <dirent.h>
#include <sys/stat.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "engine.h"

namespace nbg {
namespace {

constexpr uint64_t kMagic = 0x88e241b785f4cff7ull;
constexpr uint64_t kLegacyMagic = 0xdb4775248b80fb57ull;
constexpr size_t kTrailer = 5;

// ---------------------------------------------------------------------------- crc32c (Castagnoli)
struct Crc32c {
  uint32_t t[256];
  Crc32c() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
      t[i] = c;
    }
  }
  uint32_t operator()(const uint8_t* p, size_t n, uint32_t crc = 0) const {
    crc = ~crc;
    for (size_t i = 0; i < n; ++i) crc = t[(crc ^ p[i]) & 0xFF] ^ (crc >> 8);
    return ~crc;
  }
};
const Crc32c& crc32c() {
  static const Crc32c c;
  return c;
}
inline uint32_t crc_unmask(uint32_t m) {
  const uint32_t r = m - 0xa282ead8u;
  return (r >> 17) | (r << 15);
}

// ---------------------------------------------------------------------------- byte readers
struct Cur {
  const uint8_t* p;
  const uint8_t* e;
  bool ok = true;
  bool varint(uint64_t* out) {
    uint64_t v = 0;
    for (int shift = 0; shift <= 63 && p < e; shift += 7) {
      const uint8_t b = *p++;
      v |= (uint64_t)(b & 0x7F) << shift;
      if (!(b & 0x80)) {
        *out = v;
        return true;
      }
    }
    ok = false;
    return false;
  }
};
inline uint32_t fixed32(const uint8_t* p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}
inline uint64_t fixed64(const uint8_t* p) {
  uint64_t v;
  memcpy(&v, p, 8);
  return v;
}

// ---------------------------------------------------------------------------- snappy
// Snappy's published block format: varint32 uncompressed length, then elements whose tag's low
// two bits pick literal / copy with a 1-, 2- or 4-byte offset.
bool snappy_decode(const uint8_t* in, size_t n, std::string* out) {
  Cur c{in, in + n};
  uint64_t ulen = 0;
  // one element (at least 2 bytes, a 1-byte-offset copy) yields at most 64 bytes: a longer claimed
  // length is a corrupt header (and must not size an allocation)
  if (!c.varint(&ulen) || ulen > ((uint64_t)1 << 32) || ulen > 32 * (uint64_t)n + 64) return false;
  out->assign(ulen, '\0');
  uint8_t* o = reinterpret_cast<uint8_t*>(&(*out)[0]);
  size_t op = 0;
  const uint8_t* p = c.p;
  const uint8_t* e = c.e;
  while (p < e) {
    const uint8_t tag = *p++;
    size_t len = 0, off = 0;
    switch (tag & 3) {
      case 0: {   // literal
        len = tag >> 2;
        if (len >= 60) {
          const size_t nb = len - 59;
          if ((size_t)(e - p) < nb) return false;
          len = 0;
          for (size_t k = 0; k < nb; ++k) len |= (size_t)p[k] << (8 * k);
          p += nb;
        }
        ++len;
        if ((size_t)(e - p) < len || op + len > ulen) return false;
        memcpy(o + op, p, len);
        p += len;
        op += len;
        continue;
      }
      case 1:
        if (p >= e) return false;
        len = 4 + ((tag >> 2) & 7);
        off = ((size_t)(tag >> 5) << 8) | *p++;
        break;
      case 2:
        if (e - p < 2) return false;
        len = 1 + (tag >> 2);
        off = (size_t)p[0] | ((size_t)p[1] << 8);
        p += 2;
        break;
      default:
        if (e - p < 4) return false;
        len = 1 + (tag >> 2);
        off = fixed32(p);
        p += 4;
        break;
    }
    if (off == 0 || off > op || op + len > ulen) return false;
    for (size_t k = 0; k < len; ++k, ++op) o[op] = o[op - off];   // overlapping copies repeat
  }
  return op == ulen;
}

// ---------------------------------------------------------------------------- table
struct Handle {
  uint64_t off = 0, size = 0;
};

struct Table {
  std::vector<uint8_t> f;
  bool verify = true;   // checksum type 1 (crc32c); type 0 = none
  std::string err;
  int32_t code = NBG_OK;

  bool fail(int32_t c, const std::string& m) {
    code = c;
    err = m;
    return false;
  }
  // a block's contents, checksum-verified and decompressed
  bool block(const Handle& h, std::string* out) {
    if (h.off > f.size() || h.size > f.size() - h.off || f.size() - h.off - h.size < kTrailer)
      return fail(NBG_E_INVALID_ARGUMENT, "block handle outside the file");
    const uint8_t* b = f.data() + h.off;
    const uint8_t type = b[h.size];
    if (verify) {
      const uint32_t want = crc_unmask(fixed32(b + h.size + 1));
      const uint32_t got = crc32c()(b, h.size + 1);   // contents and the compression type byte
      if (want != got) return fail(NBG_E_INVALID_ARGUMENT, "block checksum mismatch");
    }
    if (type == 0) {
      out->assign(reinterpret_cast<const char*>(b), h.size);
      return true;
    }
    if (type == 1) {
      if (!snappy_decode(b, h.size, out)) return fail(NBG_E_INVALID_ARGUMENT, "corrupt snappy block");
      return true;
    }
    return fail(NBG_E_UNSUPPORTED, "block compression type " + std::to_string(type) + " (only none and snappy)");
  }
  // every entry of a block (prefix-compressed keys restored)
  template <class F>
  bool entries(const std::string& blk, F&& fn) {
    if (blk.size() < 4) return fail(NBG_E_INVALID_ARGUMENT, "short block");
    const uint8_t* b = reinterpret_cast<const uint8_t*>(blk.data());
    const uint32_t nr = fixed32(b + blk.size() - 4);
    if (nr & 0x80000000u) return fail(NBG_E_UNSUPPORTED, "data-block hash index");
    if ((uint64_t)nr * 4 + 4 > blk.size()) return fail(NBG_E_INVALID_ARGUMENT, "restart array");
    Cur c{b, b + blk.size() - 4 - (size_t)nr * 4};
    std::string key;
    while (c.p < c.e) {
      uint64_t shared = 0, nonshared = 0, vlen = 0;
      if (!c.varint(&shared) || !c.varint(&nonshared) || !c.varint(&vlen) || shared > key.size() ||
          nonshared > (uint64_t)(c.e - c.p) || vlen > (uint64_t)(c.e - c.p) - nonshared)
        return fail(NBG_E_INVALID_ARGUMENT, "block entry");
      key.resize(shared);
      key.append(reinterpret_cast<const char*>(c.p), nonshared);
      c.p += nonshared;
      if (!fn(key, c.p, vlen)) return false;
      c.p += vlen;
    }
    return true;
  }
  bool read(const std::string& path) {
    FILE* fp = fopen(path.c_str(), "rb");
    if (!fp) return fail(NBG_E_INVALID_ARGUMENT, "cannot open " + path);
    fseek(fp, 0, SEEK_END);
    const long n = ftell(fp);
    fseek(fp, 0, SEEK_SET);
    f.resize(n > 0 ? (size_t)n : 0);
    const bool got = f.empty() || fread(f.data(), 1, f.size(), fp) == f.size();
    fclose(fp);
    if (!got) return fail(NBG_E_INVALID_ARGUMENT, "cannot read " + path);
    return true;
  }
  // Put records in key order -> kd/ko/vd/vo
  bool records(std::vector<uint8_t>* kd, std::vector<uint64_t>* ko, std::vector<uint8_t>* vd, std::vector<uint64_t>* vo) {
    if (f.size() < 48) return fail(NBG_E_INVALID_ARGUMENT, "not an SST file (too short)");
    const uint64_t magic = fixed64(f.data() + f.size() - 8);
    Cur c{nullptr, nullptr};
    if (magic == kMagic) {
      if (f.size() < 53) return fail(NBG_E_INVALID_ARGUMENT, "not an SST file (footer)");
      const uint8_t* ft = f.data() + f.size() - 53;
      const uint32_t version = fixed32(f.data() + f.size() - 12);
      if (version > 3) return fail(NBG_E_UNSUPPORTED, "BlockBasedTable format_version " + std::to_string(version));
      if (ft[0] > 1) return fail(NBG_E_UNSUPPORTED, "checksum type " + std::to_string(ft[0]) + " (only crc32c)");
      verify = ft[0] == 1;
      c = Cur{ft + 1, ft + 41};
    } else if (magic == kLegacyMagic) {
      const uint8_t* ft = f.data() + f.size() - 48;
      verify = true;
      c = Cur{ft, ft + 40};
    } else {
      return fail(NBG_E_INVALID_ARGUMENT, "not a block-based SST file (magic)");
    }
    Handle meta, index;
    if (!c.varint(&meta.off) || !c.varint(&meta.size) || !c.varint(&index.off) || !c.varint(&index.size))
      return fail(NBG_E_INVALID_ARGUMENT, "footer handles");
    std::string iblk;
    if (!block(index, &iblk)) return false;
    std::vector<Handle> data;
    if (!entries(iblk, [&](const std::string&, const uint8_t* v, uint64_t n) {
          Cur h{v, v + n};
          Handle d;
          if (!h.varint(&d.off) || !h.varint(&d.size)) return fail(NBG_E_INVALID_ARGUMENT, "index entry");
          data.push_back(d);
          return true;
        }))
      return false;
    ko->push_back(kd->size());
    vo->push_back(vd->size());
    std::string blk;
    for (const Handle& d : data) {
      if (!block(d, &blk)) return false;
      if (!entries(blk, [&](const std::string& ikey, const uint8_t* v, uint64_t n) {
            if (ikey.size() < 8) return fail(NBG_E_INVALID_ARGUMENT, "internal key");
            const uint8_t vt = (uint8_t)ikey[ikey.size() - 8];   // low byte of seq << 8 | type
            if (vt != 1) return fail(NBG_E_UNSUPPORTED, "record type " + std::to_string(vt) + " (only Put)");
            kd->insert(kd->end(), ikey.begin(), ikey.end() - 8);
            vd->insert(vd->end(), v, v + n);
            ko->push_back(kd->size());
            vo->push_back(vd->size());
            return true;
          }))
        return false;
    }
    return true;
  }
};

bool is_dir(const std::string& p) {
  struct stat sb;
  return stat(p.c_str(), &sb) == 0 && S_ISDIR(sb.st_mode);
}

// "*.sst" files of a directory, recursively (FileUtils::listAllFilesInDir(path, true, "*.sst")),
// in name order
void list_sst(const std::string& dir, std::vector<std::string>* out) {
  DIR* d = opendir(dir.c_str());
  if (!d) return;
  std::vector<std::string> names;
  while (dirent* de = readdir(d)) {
    const std::string n = de->d_name;
    if (n != "." && n != "..") names.push_back(n);
  }
  closedir(d);
  std::sort(names.begin(), names.end());
  for (const std::string& n : names) {
    const std::string p = dir + "/" + n;
    if (is_dir(p))
      list_sst(p, out);
    else if (n.size() > 4 && n.compare(n.size() - 4, 4, ".sst") == 0)
      out->push_back(p);
  }
}

}  // namespace

int32_t Engine::ingest_sst(int32_t part, const std::string& path) {
  if (finalized) return fail(NBG_E_STATE, "engine already finalized");
  try {   // (no exception crosses the C ABI: an allocation failure is a status)
    Table t;
    std::vector<uint8_t> kd, vd;
    std::vector<uint64_t> ko, vo;
    if (!t.read(path) || !t.records(&kd, &ko, &vd, &vo)) return fail(t.code, path + ": " + t.err);
    const uint64_t n = ko.size() - 1;
    return load_part_kv(part, kd.data(), ko.data(), vd.data(), vo.data(), n);
  } catch (const std::bad_alloc&) {
    return fail(NBG_E_OUT_OF_MEMORY, path + ": out of host memory");
  }
}

// NebulaStore::ingest: every part this engine serves, every *.sst under download/<part>.
int32_t Engine::ingest_dir(const std::string& download) {
  if (finalized) return fail(NBG_E_STATE, "engine already finalized");
  for (int32_t part = 1; part <= cfg.num_parts; ++part) {
    if (cfg.num_gpus > 1 && part % cfg.num_gpus != cfg.rank) continue;
    const std::string dir = download + "/" + std::to_string(part);
    if (!is_dir(dir)) continue;   // "not existed": nothing to ingest for this part
    std::vector<std::string> files;
    list_sst(dir, &files);
    for (const std::string& p : files)
      if (int32_t rc = ingest_sst(part, p)) return rc;
  }
  return NBG_OK;
}

}  // namespace nbg

extern "C" {

int32_t nbg_ingest_sst(nbg_engine* h, int32_t part, const char* path) {
  if (!h || !path || part < 1) return NBG_E_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lg(h->e.mu);
  if (part > h->e.cfg.num_parts) return h->e.fail(NBG_E_PART_NOT_FOUND, "part out of range");
  return h->e.ingest_sst(part, path);
}

int32_t nbg_ingest_dir(nbg_engine* h, const char* download_dir) {
  if (!h || !download_dir) return NBG_E_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lg(h->e.mu);
  return h->e.ingest_dir(download_dir);
}

}  // extern "C"
