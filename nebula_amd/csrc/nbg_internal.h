// nebula_amd internal declarations (host side + kernel launch interface).
#pragma once
#include <hip/hip_runtime_api.h>

#include <array>
#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/nbg.h"

namespace nbg {

constexpr uint32_t NO_ROW = 0xFFFFFFFFu;   // dst vertex has no rows on this rank

// ----------------------------------------------------------------------------- schema
struct Column {
  std::string name;
  int32_t type;   // NBG_T_*
};
struct Schema {
  int64_t version = 0;
  std::vector<Column> cols;
  int find(const std::string& n) const {
    for (size_t i = 0; i < cols.size(); ++i)
      if (cols[i].name == n) return static_cast<int>(i);
    return -1;
  }
};
struct SchemaSet {   // all versions of one tag / edge type
  std::string name;
  std::map<int64_t, Schema> versions;
  const Schema* latest() const { return versions.empty() ? nullptr : &versions.rbegin()->second; }
  const Schema* at(int64_t v) const {
    auto it = versions.find(v);
    return it == versions.end() ? nullptr : &it->second;
  }
};

// Value kinds on the device (VariantType alternatives).
enum VKind : uint8_t { VK_INT = 0, VK_DOUBLE = 1, VK_BOOL = 2, VK_STRING = 3 };
inline VKind kindOfType(int32_t t) {
  switch (t) {
    case NBG_T_BOOL: return VK_BOOL;
    case NBG_T_FLOAT: case NBG_T_DOUBLE: return VK_DOUBLE;
    case NBG_T_STRING: return VK_STRING;
    default: return VK_INT;
  }
}

// ----------------------------------------------------------------------------- host staging
struct EdgeStage {              // one signed edge type, before finalize: records in load order
  std::vector<int64_t> src, dst;                 // (identical keys: the later record wins)
  std::vector<int64_t> rank;    // empty: every rank so far is 0
  std::vector<uint64_t> verkey; // version bytes read big-endian (memcmp order); empty: all == ver0
  uint64_t ver0 = 0;
  std::vector<int32_t> part;    // empty: every record so far sits in its source's hash part
  std::vector<std::vector<int64_t>> props;   // [col][i] 8-byte payload (positive types)
  std::vector<uint8_t> valid;   // value decoded (positive types); empty: all decoded
  uint64_t size() const { return src.size(); }
};

struct TagStage {               // one tag's vertex records, before finalize
  std::vector<int64_t> vid;
  std::vector<uint64_t> verkey; // version bytes read big-endian (memcmp order: newest first)
  std::vector<uint64_t> seq;
  std::vector<int32_t> part;
  std::vector<std::vector<int64_t>> props;   // [col][i] 8-byte payload (latest schema order)
  std::vector<uint8_t> valid;
};

// ----------------------------------------------------------------------------- device snapshot
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

struct DevEdgeType {            // CSR for one signed edge type over this rank's vertices
  int32_t type = 0;
  uint64_t num_edges = 0;
  uint32_t* row_ptr = nullptr;  // [nV + 1]
  uint32_t* col = nullptr;      // [E] dense id of dst, NO_ROW if the dst has no rows here
  int64_t* dst_vid = nullptr;   // [E]
  int64_t* rank = nullptr;      // [E] or nullptr when every rank is 0
  std::vector<int64_t*> props;  // [ncols][E] (positive types)
  int64_t** d_props = nullptr;  // device copy of `props`
  std::vector<void*> narrow;    // [ncols] INT column at narrow_bytes width (nullptr: none)
  std::vector<int> narrow_bytes;
  std::vector<VKind> prop_kind;
  uint8_t* valid = nullptr;     // [E] or nullptr when every value decoded
  int max_degree = 0;
  std::vector<uint32_t> h_row_ptr;   // host copy (path reconstruction, host planning)
  std::vector<uint16_t> h_w2, h_w3;  // tiny-path walk bounds (single engine, positive types; tiny_bounds)
  // Superseded versions (multi-version data only): a CSR of the older versions of every edge, in
  // key order, with h_grp[i] = the live edge (index into this CSR's parent) of version i.  Read
  // by GetNeighbors' filtered walk, which sees older versions until an edge is accepted
  // (QueryBaseProcessor.inl:394-456).  Owned by the parent; persisted by snapshot_save (format 2).
  DevEdgeType* old = nullptr;
  std::vector<uint32_t> h_grp;
};

// Tag properties of one tag, indexed by vertex id (single GPU: dense id; partitioned: global id,
// gathered from every rank at finalize so `$$` reads a remote destination's props locally).
struct DevTag {
  int32_t tag = 0;
  int index = 0;                // position in Snapshot::d_tpres
  int col_base = 0;             // first column in Snapshot::d_tcols
  uint8_t* present = nullptr;   // [tag_space] the vertex has a record of this tag
  std::vector<int64_t*> cols;   // [ncols][tag_space] latest-schema columns
  std::vector<VKind> kind;
  // host copies over this engine's local dense ids (GetNeighbors tag rows are built on the host)
  std::vector<uint8_t> h_present;   // 0 none, 1 decoded, 2 record present but undecodable
  std::vector<std::vector<int64_t>> h_cols;
};

struct Snapshot {
  uint64_t nv = 0;
  int64_t* d_vids = nullptr;            // dense id -> vid (sorted ascending, signed)
  std::vector<int64_t> h_vids;
  uint8_t* d_visible = nullptr;         // home part == hash part; nullptr when all visible
  uint32_t* d_zero_rows = nullptr;      // [nv + 1] zeros: the CSR of an OVER type this rank has no
                                        // edges of (partitioned FIND PATH, allocated on first use)
  std::vector<uint8_t> h_visible;       // host copy (empty when all visible)
  std::vector<int32_t> h_part;          // home part per dense id
  std::map<int32_t, DevEdgeType> types; // signed type -> CSR
  std::vector<std::string> strings;     // sorted dictionary; device code = 2 * index
  // its device tables (DevStrings): bytes, offsets, per-string toInt / toDouble (casts of columns)
  uint32_t* d_soff = nullptr;
  char* d_sbytes = nullptr;
  int64_t* d_s2i = nullptr;
  int64_t* d_s2f = nullptr;
  uint8_t* d_s2ok = nullptr;
  std::map<int32_t, DevTag> tags;       // tag id -> per-vertex columns
  int64_t** d_tcols = nullptr;          // device array: every tag column (DevTag::col_base + c)
  uint8_t** d_tpres = nullptr;          // device array: presence per tag (DevTag::index)
  uint64_t device_bytes = 0;
  uint64_t max_edges() const {   // the longest edge space of one CSR (superseded versions included)
    uint64_t m = 0;
    for (auto& kv : types) {
      m = kv.second.num_edges > m ? kv.second.num_edges : m;
      if (kv.second.old && kv.second.old->num_edges > m) m = kv.second.old->num_edges;
    }
    return m;
  }
};

// ----------------------------------------------------------------------------- bytecode
// One instruction of the per-edge program (WHERE / YIELD).  Registers are 8-byte slots.
enum Op : uint8_t {
  OP_END = 0,
  OP_CONST,      // r[d] = imm
  OP_COL,        // r[d] = props[aux][j]                (8-byte payload)
  OP_COLV,       // like OP_COL but sets the error flag when the edge value is missing
  OP_DST,        // r[d] = dst_vid[j]
  OP_SRC,        // r[d] = vid of the source vertex
  OP_RANK,       // r[d] = rank[j] (0 when no rank column)
  OP_ERR,        // error flag := 1 (statically ill-typed node, still evaluated)
  // tag props; aux = tag index << 16 | tag column (Snapshot::d_tpres / d_tcols)
  OP_TAGS,       // r[d] = $^ prop of the source vertex; imm when the vertex lacks the tag
  OP_TAGS_E,     // same, but a vertex without the tag is an evaluation error
  OP_TAGD,       // r[d] = $$ prop of the destination; imm (+ the tag's "default used" bit) when absent
  OP_EIDX,       // r[d] = the edge's CSR index (GetNeighbors: rows regrouped in key order on the host)
  OP_INPUT,      // r[d] = column aux of the input row of the source's root ($-.col / $var.col)
  // int64
  OP_ADD_I, OP_SUB_I, OP_MUL_I, OP_DIV_I, OP_MOD_I, OP_XOR_I, OP_NEG_I,
  OP_LT_I, OP_LE_I, OP_GT_I, OP_GE_I, OP_EQ_I, OP_NE_I,
  // double
  OP_ADD_F, OP_SUB_F, OP_MUL_F, OP_DIV_F, OP_MOD_F, OP_XOR_F, OP_NEG_F,
  OP_LT_F, OP_LE_F, OP_GT_F, OP_GE_F, OP_EQ_F, OP_NE_F,
  // conversions / bool
  OP_I2F, OP_B2I, OP_B2F, OP_F2I, OP_NOT,
  OP_TRUTHY_I, OP_TRUTHY_F, OP_TRUTHY_S,   // asBool (string: code == imm, the empty string)
  OP_AND, OP_OR, OP_XORB,
  // strings beyond dictionary codes (ExpandArgs::str; piece lists live in the program's data):
  OP_S2I,        // r[d] = toInt(dictionary string r[a]) (a per-string table; not a number: error)
  OP_S2F,        // r[d] = toDouble(dictionary string r[a])
  OP_SCMP,       // r[d] = piece list at data[aux] <rel a> piece list at data[imm] (bytes compared)
  OP_SPARSE_I,   // r[d] = toInt(piece list data[aux])
  OP_SPARSE_F,   // r[d] = toDouble(piece list data[aux])
  OP_SEMPTY,     // r[d] = piece list data[aux] is "" (asBool of a string)
  OP_SOUT,       // r[d] = the derived string of piece list data[aux], stored in the workspace's string
                 //        arena; its code is STR_DERIVED | content hash
  OP_ISIN_I,     // r[d] = r[b] || r[a] == imm   (udf_is_in over int64 / codes / bools)
  OP_ISIN_F,     // r[d] = r[b] || double(r[a]) == double(imm) (exact, as std::unordered_set<double>)
  OP_EQX_F,      // r[d] = double(r[a]) == double(r[b]) (exact)
  OP_ABS_F, OP_FLOOR_F, OP_CEIL_F, OP_ROUND_F, OP_SQRT_F,   // FunctionManager's exact math
  // the rest of FunctionManager (FunctionManager.cpp:20-437) over per-edge values
  OP_MATH1_F,    // r[d] = f(double(r[a])), aux: cbrt exp exp2 log log2 log10 sin asin cos acos tan atan
  OP_MATH2_F,    // r[d] = aux 0: pow(r[a], r[b]), 1: hypot(r[a], r[b]) (doubles)
  OP_HASH_F,     // r[d] = std::hash<double>(r[a]) (libstdc++ _Hash_bytes of the 8 bytes; 0.0 -> 0)
  OP_HASH_S,     // r[d] = std::hash<std::string> of the piece list data[aux]
  OP_SLEN,       // r[d] = the length of the piece list data[aux]
  OP_SCASE,      // r[d] = strcasecmp(piece list data[aux], piece list data[imm]) (glibc's difference)
  OP_RAND,       // r[d] = rand32 / rand64 (aux bit 2) over aux & 3 INT arguments r[a], r[b]
  OP_NOW,        // r[d] = WallClock::fastNowInSec() of the query (ExpandArgs::now_sec)
  OP_SMAT,       // r[d] = STR_ARENA | the arena offset of piece list data[aux], stored there: a string
                 //        function's per-edge result that another window / trim / pad reads (nesting)
  OP_COUNT_
};

struct Ins {
  uint8_t op, d, a, b;
  int32_t aux;
  int64_t imm;
};
static_assert(sizeof(Ins) == 16, "Ins layout");
// piece kinds of a derived string's piece list (exprc.cpp emit_pieces, kernels.hip piece_view)
enum PieceKind : uint8_t { PC_DICT = 1, PC_INT = 2, PC_BOOL = 3, PC_CONST = 4, PC_VIEW = 5 };
// PC_VIEW's function (FunctionManager.cpp:249-409): piece {op PC_VIEW, d = the first INT argument's
// register, a = ViewFn, b = the second's (substr's length), aux = the inner list's header, imm =
// the pad list's header (lpad / rpad)}
enum ViewFn : uint8_t { VF_LOWER = 0, VF_UPPER, VF_TRIM, VF_LTRIM, VF_RTRIM, VF_LEFT, VF_RIGHT, VF_LPAD, VF_RPAD,
                        VF_SUBSTR };

// A derived string's code in a result / register: the tag bit plus a 62-bit content hash, so
// equal strings have equal codes (YIELD DISTINCT, the partitioned owner exchange); its bytes are
// in the producing workspace's arena (nbg_rows_fetch decodes them).  Dictionary codes are < 2^33.
constexpr int64_t STR_DERIVED = (int64_t)1 << 62;
constexpr uint64_t STR_HASH_MASK = ((uint64_t)1 << 62) - 1;
// (negative codes are dictionary codes too: -1 is "" when the dictionary lacks it)
inline bool is_derived_code(int64_t c) { return ((uint64_t)c >> 62) == 1; }
// A $- / $var input string absent from the snapshot's dictionary: STR_INPUT | its index in the
// statement's input-string table (DevStrings::x*), the table sorted and unique.  Such a statement
// reads its input string columns as derived strings (piece lists), so every compare is on bytes and
// a YIELD stores the value into the arena (STR_DERIVED code).
constexpr int64_t STR_INPUT = (int64_t)1 << 61;
// A string materialised inside one edge's evaluation (OP_SMAT): STR_ARENA | its entry's offset in
// the workspace's arena.  Only a piece of a later view reads it; it never reaches a result column.
constexpr int64_t STR_ARENA = (int64_t)1 << 60;
inline bool is_input_code(int64_t c) { return ((uint64_t)c >> 61) == 1; }
constexpr uint64_t STR_HASH_INIT = 0xcbf29ce484222325ull;   // FNV-1a over the bytes, then mixed

#if defined(__HIPCC__)
#define NBG_HD __host__ __device__
#else
#define NBG_HD
#endif
NBG_HD inline uint64_t str_hash_step(uint64_t h, uint8_t b) { return (h ^ b) * 0x100000001b3ull; }
NBG_HD inline int64_t str_derived_code(uint64_t h, uint64_t len) {
  uint64_t z = h ^ (len * 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return STR_DERIVED | (int64_t)(z & STR_HASH_MASK);
}

// Device string tables of a snapshot (built at finalize when the dictionary is not empty): the
// dictionary's bytes and the per-string toInt / toDouble results the casts read
struct DevStrings {
  const uint32_t* off = nullptr;    // [n + 1] byte offsets into bytes
  const char* bytes = nullptr;
  const int64_t* s2i = nullptr;     // [n] toInt(string) payload
  const int64_t* s2f = nullptr;     // [n] toDouble(string) bits
  const uint8_t* s2ok = nullptr;    // [n] bit 0: toInt ok, bit 1: toDouble ok
  uint64_t n = 0;
  // the statement's input strings absent from the dictionary (codes STR_INPUT | index)
  const uint32_t* xoff = nullptr;   // [xn + 1]
  const char* xbytes = nullptr;
  uint64_t xn = 0;
  // the query's derived-string arena (OP_SOUT): entries [u64 hash][u32 len][u32 0][bytes, 8-aligned]
  char* arena = nullptr;
  unsigned long long* arena_used = nullptr;   // bytes claimed (may exceed arena_cap: overflow)
  uint64_t arena_cap = 0;
  unsigned long long* err_flag = nullptr;     // QState::err: an overflow ORs in ARENA_OVERFLOW
};
constexpr unsigned long long ARENA_OVERFLOW = 1ull << 32;   // (summed over ranks, still >= 2^32)
// QState::err: a merge-path split read from a list did not describe a tile (entries out of the list,
// out of order, or more than the tile holds); the tile is skipped, never read out of bounds, and
// the query fails with NBG_E_DEVICE (summed over ranks, still >= 2^48)
constexpr unsigned long long SPLIT_BAD = 1ull << 48;

constexpr int MAX_REGS = 48;       // the compiler's ceiling; the device's LDS sets the run-time one
// The interpreter's registers are [nregs][BLOCK] x 8 B of dynamic LDS beside each kernel's static
// LDS: the register counts a program may use on this device (k_expand / k_go_tiny), from the
// device's LDS per workgroup
int interp_max_regs();
int tiny_max_regs();
constexpr int MAX_PROGRAM = 256;   // instructions per query/type (WHERE + all YIELDs)
constexpr int MAX_YIELDS = 32;

// A compiled query for one OVER edge type.
struct TypeProgram {
  int32_t etype = 0;
  std::vector<Ins> code;           // WHERE first (if any), then each YIELD
  int where_len = 0;               // instructions of the WHERE part
  int where_reg = -1;              // register holding the WHERE value (-1: no WHERE)
  VKind where_kind = VK_BOOL;
  bool where_const = false;        // WHERE folded to a constant
  bool where_const_val = true;
  bool where_always_error = false;
  std::vector<int> yield_reg;      // register per YIELD column (-1 = constant)
  std::vector<VKind> yield_kind;
  std::vector<int64_t> yield_const;   // constant payload when yield_reg == -1
  std::vector<std::string> yield_const_str;   // string constants (may be absent from the dictionary)
  std::vector<Ins> data;           // piece lists and constant bytes of derived strings (after `code`)
  bool sout = false;               // some YIELD stores a derived string (OP_SOUT: the string arena)
  uint64_t sout_bytes = 0;         // arena bytes one row's OP_SOUTs may store (ProgramBuilder)
  bool needs_error_check = false;  // any op can raise an error
  uint32_t probe_mask = 0;         // tags read through $$: presence probed for every final edge
  bool keep_on_error = false;      // storage filter: an evaluation error keeps the edge (inl:444-448)
  int nregs = 0;
};

// ----------------------------------------------------------------------------- kernel interface
#ifndef NBG_VT
#define NBG_VT 4
#endif
constexpr int VT = NBG_VT;             // k_expand: path items per thread
constexpr int TILE = 64 * VT;          // path items (frontier entries + edges) per wave tile
constexpr int NSHARD = 64;             // row-output shards (one counter + region each)
constexpr int MAX_STEPS = 32;          // GO N STEPS upper bound
constexpr int MAX_TYPES_Q = 32;        // OVER types per query
constexpr int INLINE_STARTS = 32;      // start lists up to this size travel in kernel arguments
constexpr int MAX_TAG_BITS = 16;       // tags addressable by $$ (QState::tagbits: has | used << 16)
constexpr int MAX_INPUT_COLS = 32;     // columns of a piped / variable input

// A short start list with its edge space over one CSR, built on the host from the CSR offsets
// (the host copy of row_ptr) and passed by value to the first expansion: the query's first
// list needs no device pass (no k_relist launch).
struct InlineList {
  uint32_t n;                     // entries: the starts with edges
  uint32_t n_in;                  // starts given (|F_1|: duplicates and edgeless starts included)
  uint32_t total;                 // edges of the entries (capped degrees)
  uint32_t id[INLINE_STARTS];
  uint32_t end[INLINE_STARTS];    // inclusive prefix sums of the degrees
  uint32_t rs[INLINE_STARTS];     // row starts
};

// Device-resident state of one query: every size the kernels need, so a query is enqueued
// without host synchronisation; the host reads it back once at the end.
struct QState {
  unsigned long long n;                // current frontier size
  unsigned long long total;            // edges of the current (step, type) expansion
  unsigned long long err;              // WHERE/YIELD evaluation error
  unsigned long long acc[5];           // packed list sizes (entries << 32 | edges): relist 0/1,
                                       // step lists 2..4 (compaction ping-pong 2/3, claim lists rotate 2..4)
  unsigned long long step_n[MAX_STEPS + 2];              // frontier size entering step s
  unsigned long long e_st[MAX_STEPS + 2][MAX_TYPES_Q];   // edges per (step, type)
  // $$ holder semantics (GoExecutor::VertexHolder, GoExecutor.cpp:986-1064): bit t = some final
  // destination has tag t; bit 16 + t = a row read tag t's default for a destination without it
  unsigned long long tagbits;
  unsigned long long arena_used;       // bytes the query's OP_SOUT claimed in the string arena
};

struct ExpandArgs {                // one (step, edge type) expansion
  const uint32_t* frontier;        // filled in by the workspace (current buffer)
  const uint32_t* row_ptr;
  const uint32_t* col;
  const int64_t* dst_vid;
  const int64_t* rank;
  const uint8_t* valid;
  const uint8_t* visible;
  const int64_t* vids;             // dense id -> vid (for _src)
  const int64_t* const* props;     // device array of column pointers
  uint32_t cap;                    // max_edge_returned_per_vertex
  const uint32_t* tsplit;          // per-tile merge-path splits (set by the workspace)
  const int64_t* const* hprops;    // host array of the same column pointers (host-side planning)
  void* const* hnarrow;            // host array: narrow copies of INT columns (nullptr: none)
  const int* hnarrow_bytes;
  const int64_t* const* tcols;     // tag columns (Snapshot::d_tcols), indexed by vertex id
  const uint8_t* const* tpres;     // tag presence (Snapshot::d_tpres)
  uint32_t gbase;                  // id of local vertex 0 in the tag index space (rank * npad)
  // piped / variable input (GoExecutor::setupStarts index + VertexBackTracker, GoExecutor.h:169-188)
  // Roots travel as vids, so a root means the same on every rank.  MARKB writes bt[u] for each
  // neighbour u (single engine: dense ids; partitioned: global ids, exchanged to u's owner with
  // the hop) and reads bt_in[src] for a frontier vertex src (the owner's local view).
  int64_t* bt;                     // (nullptr: not tracked)
  const int64_t* bt_in;
  int bt_first;                    // MARK: this is step 1 (the root of a start is itself)
  const int64_t* in_ids;           // input index: the rows' vids, ascending (last row wins)
  uint64_t in_n;
  const int64_t* const* in_cols;   // [col][k] 8-byte payloads of the indexed rows
  DevStrings str;                  // strings beyond dictionary codes (casts, concatenation)
  int64_t now_sec;                 // now(): the query's wall-clock second (set per query)
  uint64_t rand_seed;              // rand32 / rand64: this query's stream (set per query)
};

// The lean final step (final.hip) for WHERE `col <cmp> const` (or none) with _dst / constant
// YIELDs: the final list (packed count, edge offsets, row starts, tile splits), the _dst column,
// the WHERE column at its stored width, and the rows' destination (as k_expand<FINALD>)
struct FinalDstArgs {
  const unsigned long long* acc;
  const uint32_t* seg_end;
  const uint32_t* seg_rs;
  const uint32_t* tsplit;
  uint64_t tsplit_n;               // entries tsplit holds (the first splits are read before the list's size)
  const int64_t* dst_vid;
  const void* wcol;
  int64_t lo, hi;                  // pass = (lo <= w && w <= hi) != where_neg
  int32_t where_neg;
  int32_t nyields;
  uint64_t const_mask;             // bit y: YIELD y is the constant yconst[y] (else _dst)
  int64_t yconst[MAX_YIELDS];
  int64_t* out[MAX_YIELDS];
  uint64_t region_base, blk_cap;   // rows of workgroup b at region_base + b * blk_cap
  uint32_t* blk_rows;
  unsigned long long* stat_e;
  unsigned long long* stat_n;
  unsigned long long* err_flag;    // QState::err (SPLIT_BAD)
};
hipError_t launch_final_dst(const FinalDstArgs& a, int wbytes, bool one, unsigned grid, hipStream_t s);

// ----------------------------------------------------------------------------- FIND PATH state
// Vertex labels are epoch-stamped so no per-query clearing is needed: label = epoch << LVL_BITS |
// level, live when its epoch is the current one.
constexpr int LVL_BITS = 6;
constexpr uint32_t MAX_PATH_LEN = (1u << LVL_BITS) - 1;   // UPTO bound
constexpr int PSLOTS = 8;           // 0,1 forward / 2,3 backward frontiers, 4 meets, 5 starts, 6,7 B-sets
enum PathLabel { LAB_F = 0, LAB_B = 1, LAB_S = 2, LAB_M = 3, NUM_LABS = 4 };
constexpr int GREEDY_HOP_BLOCKS = 64;   // workgroups scanning one reconstruction hop
constexpr int PATH_REC = 64;        // per-query expansion records (profiling byte counts)

struct PState {                      // device-resident sizes of one FIND PATH query
  unsigned long long n[PSLOTS];      // size of each frontier slot
  unsigned long long total;          // edges of the current expansion
  unsigned long long edges;          // BFS edges scanned (both sides)
  unsigned long long meets;          // meet-list length
  unsigned long long found;          // targets reached (one-sided search)
  unsigned long long err;            // reconstruction failure
  unsigned long long acc[2];         // packed relist sizes (ping-pong)
  unsigned long long dsum[2];        // degree sum of the current forward / backward frontier
  unsigned long long shard[NSHARD];  // claim counters
  unsigned long long ln[PATH_REC];   // per expansion record: frontier size, edges, claims
  unsigned long long le[PATH_REC];
  unsigned long long lc[PATH_REC];
  unsigned long long gticket;         // greedy hop: workgroups done (the last one reduces)
  unsigned long long gv;              // greedy hop: the current path vertex (dense id)
  unsigned long long gpart[4 * GREEDY_HOP_BLOCKS];   // greedy hop: per-workgroup minimum candidate
  unsigned long long ld[PATH_REC];   // degree sum of the level's output list (summed by k_expand<BFS>)
  unsigned long long mdsum;          // partitioned: in-degree sum of the meet list (its B-set step's bound)
  unsigned long long mdsum_out;      // partitioned: its out-degree sum (the forward B-set step's bound)
};

struct PathTypes {                   // the CSRs one search direction expands (one per OVER type)
  int n = 0;
  int32_t type[MAX_TYPES_Q];
  ExpandArgs a[MAX_TYPES_Q];
};

// ----------------------------------------------------------------------------- one-pair FIND SHORTEST PATH (sp.hip)
struct SpTypes {                     // the CSRs one search direction expands (OVER order)
  int n = 0;
  int32_t type[MAX_TYPES_Q];
  const uint32_t* row_ptr[MAX_TYPES_Q];
  const uint32_t* col[MAX_TYPES_Q];
  const int64_t* dst_vid[MAX_TYPES_Q];
  const int64_t* rank[MAX_TYPES_Q];
  uint64_t ne[MAX_TYPES_Q];          // edges of each CSR (bounds of the checked build)
};
struct SpResult {                    // one query's result (from the chain's ChOut)
  unsigned long long L;              // path length, 0 = no path within UPTO
  unsigned long long edges;          // BFS adjacency entries scanned (both sides)
  unsigned long long err;            // 1 reconstruction failure, 3 list overflow, 4 a bad tile split,
                                     // CH_ERR_WALK_CAP, 256 << site: CH_GUARD bounds violation
  unsigned long long levels;         // BFS levels run
  unsigned long long abytes;         // algorithmic bytes of its level / B-set launches (chain mode)
  unsigned long long launches;       // device launches of its chain (setup + steps + hops)
  unsigned long long batches;        // launch batches the host enqueued (1: no continuation)
  long long path[1 + 3 * MAX_PATH_LEN];   // [v0, t0, r0, v1, ...]
};
constexpr unsigned long long CH_ERR_WALK_CAP = 64;   // the greedy walk did not end within its launch cap
// the text of a failed search's SpResult::err (path.cpp's error messages)
inline std::string sp_err_text(unsigned long long err) {
  if (err == CH_ERR_WALK_CAP) return "greedy walk incomplete at the chain's launch cap";
  if (err & 4) return "a frontier list's merge-path split did not describe its tile (code " + std::to_string(err) + ")";
  return "device search aborted (code " + std::to_string(err) + ")";
}
// A vertex's forward, backward and B-set labels (epoch << LVL_BITS | level) are one 16-byte
// record: a BFS claim tests its own side's label and the other side's, a B-set step the forward
// label and LAB_M, so each item's label tests touch one line, not two or three (sp.hip allocates
// (nv + 1) records; SpCtx::lab[i] points at word i of record 0)
constexpr uint32_t CH_LAB_WORDS = 4;
struct SpCtx;                        // labels and level-loop buffers of one slot (sp.hip)
// item_cap: items a list may hold = sum over a side's types of (nv + E_t / 64), plus slack
// One query at a time per context; the level-loop buffers are allocated on its first use.
enum SpMode : int { SP_CHAIN = 1 };
SpCtx* sp_create(uint64_t nv, uint64_t item_cap, uint64_t edge_cap, hipStream_t s, std::string* err);
void sp_destroy(SpCtx* c);
// enqueue the search for s -> t (local dense ids, s != t): the device-driven level loop
// (spchain.hip, one OVER type per direction), its result stored into mapped host memory
hipError_t sp_launch(SpCtx* c, const SpTypes& fwd, const SpTypes& bwd, const uint8_t* visible, const int64_t* vids,
                     uint32_t s, uint32_t t, uint32_t upto, uint64_t dmin = 0);
bool sp_ready(SpCtx* c);
struct SpPair {                 // one query of sp_launch_batch
  const SpTypes* fwd;
  const SpTypes* bwd;
  const uint8_t* visible;
  const int64_t* vids;
  uint32_t s, t, upto;
};
hipError_t sp_launch_batch(SpCtx* const* cs, int n, const SpPair* pairs);
struct ChainCtx;
// list_cap: entries each frontier / meet list holds (0: nv + 1, every vertex); a search that
// would outgrow a smaller one fails with err 3 (list overflow) and its caller reruns it
ChainCtx* chain_create(uint64_t nv, uint64_t edge_cap, hipStream_t s, std::string* err, uint64_t list_cap = 0);
void sp_set_list_cap(SpCtx* c, uint64_t list_cap);   // before the level-loop buffers exist
void chain_destroy(ChainCtx* c);
hipError_t chain_launch(ChainCtx* c, const SpTypes& fwd, const SpTypes& bwd, const uint8_t* visible,
                        const int64_t* vids, uint32_t* const lab[3], uint32_t epoch, uint32_t s, uint32_t t,
                        uint32_t upto, uint64_t dmin = 0);
bool chain_more(ChainCtx* c, hipError_t* he);   // false: a continuation batch was enqueued
bool chain_woken(const ChainCtx* c);   // the current batch's last launch has stored the result
// one query of a batched chain (spchain.hip, chain_launch_batch)
struct ChainQuery {
  const SpTypes* fwd;
  const SpTypes* bwd;
  const uint8_t* visible;
  const int64_t* vids;
  uint32_t* const* lab;   // [3]
  uint32_t epoch, s, t, upto;
};
hipError_t chain_launch_batch(ChainCtx* const* cs, int n, const ChainQuery* qs);
// a rolling run (spchain.hip chain_roll): slot l = a context, its labels and its first epoch
struct ChainSlot {
  ChainCtx* c;
  uint32_t* const* lab;   // [3]
  uint32_t ebase;         // the run uses epochs ebase + 1 .. ebase + n + 1
};
constexpr uint32_t CH_ROLL_UPTO = 32;   // rolling runs: UPTO at most this (CH_MAXS launches per pair suffice)
constexpr int CH_ROLL_SLOTS = 64;       // slots of a rolling run, at most
hipError_t chain_roll(const ChainSlot* slots, int nslots, const SpTypes& fwd, const SpTypes& bwd,
                      const uint8_t* visible, const int64_t* vids, const uint32_t* s, const uint32_t* t, uint32_t n,
                      uint32_t upto, SpResult* results);
// n pairs on nslots slot contexts (one stream) as one rolling run (sp.hip)
hipError_t sp_roll(SpCtx* const* cs, int nslots, const SpTypes& fwd, const SpTypes& bwd, const uint8_t* visible,
                   const int64_t* vids, const uint32_t* s, const uint32_t* t, uint32_t n, uint32_t upto,
                   SpResult* results);
void chain_result(const ChainCtx* c, SpResult* out);
constexpr int CHAIN_KINDS = 4;                       // profiled chain launch kinds
extern const char* const kChainKernelNames[CHAIN_KINDS];
void chain_profile(ChainCtx* c, int mode);           // nbg_profile modes; resets the counters
void chain_profile_done(ChainCtx* c, const SpResult& r);
void chain_profile_accum(const ChainCtx* c, double* launches, double* ms, double* bytes);
void sp_profile(SpCtx* c, int mode);
hipError_t sp_reserve_chain(SpCtx* c);               // the level-loop buffers now, not at the first query
void sp_profile_accum(const SpCtx* c, double* launches, double* ms, double* bytes);
hipError_t sp_wait(SpCtx* c, SpResult* out);

// ----------------------------------------------------------------------------- collectives (comm.cpp)
// Transport of the partitioned engine.  Methods return 0 on success; `last` holds the error.
//
// Failure semantics (the reference keeps a query alive on partial failure and reports the
// failed parts, StorageClient.inl:112-136, GoExecutor.cpp:424-442; here every rank must instead
// leave a collective query TOGETHER, or its peers block in the next collective):
//   * rank-local failures before a query's first collective (allocation, a start list too large
//     for one rank, ...) are agreed with agree(): every rank learns every rank's code and returns
//     the same one (the first failing rank's);
//   * a failure after that point (a device error between collectives, a peer that never arrives)
//     aborts the communicator: abort() wakes the peers' pending collectives with an error, and a
//     host wait on a partitioned stream gives up after NBG_COMM_TIMEOUT_S (default 120) seconds
//     and aborts too.  An aborted communicator fails every later collective at once.
struct Comm {
  int world = 1, rank = 0;
  std::string last;
  virtual ~Comm();
  virtual const char* kind() const = 0;
  // Every rank passes its local status; *out = the status of the lowest-ranked rank that failed
  // (NBG_OK when none did), the same on every rank.  Returns 0, or -1 when the exchange itself
  // failed (the communicator is then aborted).  Synchronous (host round trip).
  int agree(hipStream_t s, int32_t local, int32_t* out);
  // out[q * k + i] = rank q's mine[i], on every rank (k equal on every rank, world * k <=
  // GATHER_WORDS); through the communicator's own scratch, so nothing is allocated per call.
  // Returns 0, or -1 when the exchange failed (the communicator is then aborted) or is too large.
  int gather_u64(hipStream_t s, const uint64_t* mine, size_t k, std::vector<uint64_t>* out);
  virtual void abort() { aborted = true; }
  bool is_aborted() const { return aborted; }
  // Wait for a stream that runs this communicator's collectives; gives up (aborting) after the
  // communicator timeout.  0 = done, -1 = failed or timed out (`last` says which).
  int wait(hipStream_t s);
  // recv[q * bytes ..] <- rank q's send[rank * bytes ..], for every q (stream-ordered)
  virtual int alltoall(const void* send, void* recv, size_t bytes, hipStream_t s) = 0;
  // recv[rdisp[q] * elem ..] <- rank q's send[sdisp[rank] * elem ..], rcount[q] elements of elem
  // bytes (rank q's scount[rank]); counts and displacements are host values on every rank
  virtual int alltoallv(const void* send, const uint64_t* scount, const uint64_t* sdisp, void* recv,
                        const uint64_t* rcount, const uint64_t* rdisp, size_t elem, hipStream_t s) = 0;
  // recv[q * bytes ..] <- rank q's send[0 .. bytes)
  virtual int allgather(const void* send, void* recv, size_t bytes, hipStream_t s) = 0;
  virtual int allreduce_sum_u64(unsigned long long* buf, size_t n, hipStream_t s) = 0;
  // A second communicator over the same ranks (collective: every rank calls it at the same
  // point), for collectives on another stream; nullptr when the transport has none.
  virtual Comm* split(std::string* err) {
    (void)err;
    return nullptr;
  }

 bool agree_ready(std::string* err);         // allocate agree()'s scratch (at communicator creation)

 protected:
  volatile bool aborted = false;
  unsigned long long* agree_dev = nullptr;    // [GATHER_WORDS] device scratch of agree() / gather_u64()
  unsigned long long* agree_host = nullptr;   // pinned mirror
};
constexpr int AGREE_WORDS = 256;            // agree(): one status word per rank (world <= 256)
constexpr size_t GATHER_WORDS = 8192;       // gather_u64(): world * k words (the scratch's size)
double comm_timeout_s();                    // NBG_COMM_TIMEOUT_S
Comm* comm_rccl(const uint8_t id[NBG_UNIQUE_ID_BYTES], int world, int rank, std::string* err);
std::vector<Comm*> comm_local_group(int world);

// ----------------------------------------------------------------------------- snapshot build (build.hip)
// Neighbour id of a vid: single GPU = its dense id in `dict`; partitioned = owner * npad + its
// index in the owner's dictionary (gdict = every rank's dictionary, npad apart).
struct GidMap {
  const int64_t* dict = nullptr;    // device, sorted local dictionary
  uint64_t nv = 0;
  const int64_t* gdict = nullptr;   // device [G * npad] (partitioned) or nullptr
  const uint64_t* gcount = nullptr; // device [G]
  uint64_t npad = 0;
  int32_t gpus = 1, parts = 1;
};
struct TypeBuildIn {                // one signed type's staged records, load order
  uint64_t n = 0;
  const int64_t* d_src = nullptr;   // device copy of the sources
  const int64_t* dst = nullptr;     // host arrays from here on
  const int64_t* rank = nullptr;    // nullptr: every rank is 0
  const uint64_t* verkey = nullptr; // nullptr: one version for every record
  int nprops = 0;
  const int64_t* const* props = nullptr;   // [nprops][n] (string ids already dictionary codes)
  const VKind* kinds = nullptr;
  const uint8_t* valid = nullptr;   // nullptr: every value decoded
};
// sorted unique values of n device int64s -> *out (hipMalloc'd, *n_out entries)
hipError_t bd_sort_unique(const int64_t* d_in, uint64_t n, int64_t** out, uint64_t* n_out, hipStream_t s);
// home part per dense id (d_home zeroed by the caller): part[i] or, when null, the source's hash part
hipError_t bd_home(int32_t* d_home, const int64_t* d_src, const int32_t* part, uint64_t n, const int64_t* d_dict,
                   uint64_t nv, int32_t parts, bool* split, hipStream_t s);
// CSR of one signed type over the dictionary's vertices (row_ptr, col, dst_vid, rank, props,
// narrow INT copies, valid, h_row_ptr, max_degree); *bytes = device bytes kept
hipError_t bd_build_type(const TypeBuildIn& in, const GidMap& gm, hipStream_t s, DevEdgeType* out, uint64_t* bytes,
                         std::string* err);

struct Workspace;   // kernels.hip

// e_max: the largest edge count of one signed type (sizes the per-tile split array)
Workspace* ws_create(uint64_t max_frontier, uint64_t nv, uint64_t e_max, hipStream_t s, std::string* err);
void ws_destroy(Workspace* w);
void ws_profile(Workspace* w, int mode);   // 0 off, 1 every launch, 2 final/BFS expansions only
int ws_profile_read(Workspace* w, nbg_kernel_stat* out, int cap);
void ws_profile_inherit(Workspace* to, Workspace* from);   // profiling mode and counters
uint64_t ws_cap_frontier(Workspace* w);
uint64_t ws_cap_items(Workspace* w);   // entries + edges of one list the merge-path tiles cover
hipError_t ws_reserve_arena(Workspace* w, uint64_t bytes);   // derived strings (OP_SOUT), grow-only
hipError_t ws_read_arena(Workspace* w, uint64_t used, std::vector<char>* out);
const char* ws_arena(Workspace* w, uint64_t* cap);           // device pointer + capacity
hipError_t ws_reserve_rows(Workspace* w, uint64_t rows, int ncols);
int64_t* ws_row_col(Workspace* w, int c);       // device pointer of output column c
uint64_t ws_shard_cap(uint64_t n_bound, uint64_t e_bound);
// final-step row layout: ws_final_grid workgroups, each appending to its own blk_cap rows
unsigned ws_final_grid(uint64_t n_bound, uint64_t e_bound);
uint64_t ws_final_blk_cap(uint64_t n_bound, uint64_t e_bound);
unsigned ws_final_grid_of(Workspace* w, int tix);          // grid of the last final expansion (0: none)
const uint32_t* ws_host_blk_rows(Workspace* w, int tix);    // rows per workgroup (after ws_end_query)
hipError_t ws_fetch_rows(Workspace* w, const std::vector<std::pair<uint64_t, uint64_t>>& segs, int ncols,
                         uint64_t total, int64_t* const* host_cols);
hipError_t ws_fetch_rows_pinned(Workspace* w, const std::vector<std::pair<uint64_t, uint64_t>>& segs, int ncols,
                                uint64_t total, int64_t* host_block);   // pinned, columns back to back
// order-independent digest {rows, xor, sum} of the rows in segs (splitmix64 chain per row)
hipError_t ws_rows_digest(Workspace* w, const std::vector<std::pair<uint64_t, uint64_t>>& segs, int ncols,
                          uint64_t out[3]);
const QState* ws_host_state(Workspace* w);       // valid after ws_end_query
// YIELD DISTINCT: dedup + in-place compaction of result segments (first row, rows, OVER index)
// Partitioned YIELD DISTINCT: rows hashed to their owner rank (all-to-all), deduplicated there.
// Collective: every rank calls it, with its own (already locally deduplicated) segments.  The
// rank's rows are then, per OVER type t, blocks r = 0..G-1 at out[t].region + r * out[t].blk_cap
// holding out[t].counts[r] rows (the rows received from rank r).
struct DistinctBlock {
  uint64_t region = 0, blk_cap = 0;
  std::vector<uint32_t> counts;
};
// status: this rank's local status (its dedup pass); *gstatus: the first failing rank's, the same on
// every rank (then nothing was exchanged and the query fails everywhere)
hipError_t ws_distinct_exchange(Workspace* w, const std::vector<std::array<uint64_t, 3>>& segs, int ncols,
                                const std::vector<std::vector<VKind>>& kinds, std::vector<DistinctBlock>* out,
                                int32_t status, int32_t* gstatus);
hipError_t ws_distinct(Workspace* w, const std::vector<std::array<uint64_t, 3>>& segs, int ncols,
                       const std::vector<std::vector<VKind>>& kinds, std::vector<uint32_t>* counts);
const uint32_t* ws_current_frontier(Workspace* w);

// Query pipeline (all asynchronous on the workspace stream until ws_end_query):
hipError_t ws_begin_query(Workspace* w, const uint32_t* starts, uint64_t n, const std::vector<TypeProgram>* progs,
                          uint64_t stmt_id);
// steps 1..N-1, per OVER type: scan + expand into the next frontier.  Single engine: every new
// neighbour is CLAIMED against a per-step stamp and appended to the next list (with its edge
// space over next0 = the first OVER type's CSR of step + 1); partitioned: byte flags over the
// global id space for ws_exchange.  il: the start list's inline form for this type.
hipError_t ws_expand_mark(Workspace* w, const ExpandArgs& a, uint64_t n_bound, uint64_t e_bound, int step, int tix,
                          const InlineList* il, const ExpandArgs* next0);
// after all types of a non-final step (single engine): the claimed list becomes the frontier
hipError_t ws_finish_step(Workspace* w, int step, const ExpandArgs* next0);
void ws_set_mark_claims(Workspace* w, bool claims);   // per query, before its first step
void ws_set_wake(Workspace* w, bool flag);   // the next end kernel wakes the host by its mapped flag
// step N, per OVER type: scan + WHERE/YIELD + sharded row emission into [region_base, +NSHARD*shard_cap)
hipError_t ws_expand_final(Workspace* w, const ExpandArgs& a, uint64_t n_bound, uint64_t e_bound, int step, int tix,
                           const TypeProgram& prog, uint64_t region_base, uint64_t blk_cap, const InlineList* il = nullptr);
hipError_t ws_scan_only(Workspace* w, const ExpandArgs& a, uint64_t n_bound, int step, int tix);
// roots (allocated on first use): *out written by MARKB, *in read (the same array on a single
// engine; partitioned, out spans the global id space and in is the owner's local view, merged by
// the hop exchange).  Enables the root exchange for the workspace's queries until reset.
hipError_t ws_backtracker(Workspace* w, int64_t** out, int64_t** in);
void ws_backtracker_off(Workspace* w);
hipError_t ws_end_query(Workspace* w);
hipError_t ws_end_query_async(Workspace* w);   // enqueue the end-of-query copy + event
// ... and, for a result small enough (SMALL_ROWS_WORDS cells), its rows packed into host memory
// by the same kernel (no second host round trip to fetch them): the final step's row segments per
// OVER type, in the order nbg_rows lays them out
struct SmallPack {
  int ntypes, ncols;
  uint64_t region[MAX_TYPES_Q], blk_cap[MAX_TYPES_Q];
  uint32_t grid[MAX_TYPES_Q];
};
constexpr uint64_t SMALL_ROWS_WORDS = 32768;   // 256 KB of 8-byte cells
hipError_t ws_end_query_async_small(Workspace* w, const SmallPack& sp);
// the rows ws_end_query_async_small packed (column c at c * count), or nullptr when the last
// query's result was not packed or has a count other than `count`
const int64_t* ws_host_small_rows(Workspace* w, uint64_t count);
hipError_t ws_end_query_wait(Workspace* w);    // wait for it (then as ws_end_query)
// A GO query bounded by TINY_EDGES edge visits over all its steps (one OVER type, inline starts,
// rows fetched to the host): the whole query in one single-workgroup launch whose results land
// where ws_end_query_async_small puts them; then ws_end_query_wait.
constexpr uint32_t TINY_EDGES = 1024;
// W_2 / W_3 of every vertex of one CSR (saturated at TINY_EDGES + 1): the edge visits GO 2 / 3
// STEPS from it can make at most (empty vectors on failure: no tiny path for that type)
hipError_t tiny_bounds(const uint32_t* row_ptr, const uint32_t* col, const uint8_t* visible, uint32_t cap, uint64_t nv,
                       std::vector<uint16_t>* w2, std::vector<uint16_t>* w3, hipStream_t s);
hipError_t ws_go_tiny(Workspace* w, const ExpandArgs& a, const uint32_t* starts, uint32_t n, uint32_t steps,
                      const TypeProgram& prog, int ncols);
// partitioned mode: flags over [world * npad) global ids, per-hop bitmap all-to-all
constexpr uint64_t PART_ALIGN = 16384 * 4;   // npad granularity (flag / bit workgroups divide it)
hipError_t ws_set_partition(Workspace* w, Comm* comm, uint64_t npad);
Comm* ws_get_comm(const Workspace* w);   // the communicator of a partitioned workspace (else nullptr)
hipStream_t ws_stream(const Workspace* w);
hipError_t ws_exchange(Workspace* w, int step, const ExpandArgs* next0);   // replaces ws_compact
// the next hop (its MARKs and ws_exchange) sends per-owner slot arrays of `stride` local ids
// instead of npad-bit bitmap segments; the caller guarantees the hop's edges on every rank fit
hipError_t ws_set_hop_slots(Workspace* w, uint64_t stride);
hipError_t ws_global_stats(Workspace* w, int ntypes);      // before ws_end_query
int32_t ws_host_gstatus(Workspace* w);                     // after it: the first failing rank's status
hipError_t part_empty_query(Comm* c, hipStream_t s, int hops, const void* send0, void* recv, size_t seg_bytes,
                            size_t first_bytes, unsigned long long* gst, unsigned long long* h_gst, int32_t status,
                            int32_t* agreed);
size_t part_gst_words(int world);
void ws_host_gstats(Workspace* w, unsigned long long* err, unsigned long long* step_n, unsigned long long* esum,
                    unsigned long long* tagbits);

// FIND SHORTEST PATH (kernels.hip).  Frontier lists live in numbered device slots; PState sizes
// are read back by ws_path_sync.  All calls enqueue on the workspace stream.
hipError_t ws_path_begin(Workspace* w, uint64_t scratch_entries, uint64_t list_entries, bool zero_state = true);
// One-pair set-up in one launch (replaces the PState clear, three single-id uploads, two stamps
// and two degree sums): slots f/b/start = {s}, {t}, {s}; labels lab_f[s], lab_b[t] stamped;
// PState.dsum[0] = out-degree of s over fwd, dsum[1] = in-degree of t over bwd.
hipError_t ws_path_setup_pair(Workspace* w, const PathTypes& fwd, const PathTypes& bwd, uint32_t s, uint32_t t,
                              int slot_f, int slot_b, int slot_start, int lab_f, uint32_t stamp_f, int lab_b,
                              uint32_t stamp_b);
uint32_t ws_path_epoch(Workspace* w, int lab);                    // fresh epoch for one label array
uint32_t* ws_path_slot(Workspace* w, int slot);
hipError_t ws_path_upload(Workspace* w, int slot, const uint32_t* ids, uint64_t n);
// lab[ids of slot] = stamp
hipError_t ws_path_stamp(Workspace* w, int slot, uint64_t n_bound, int lab, uint32_t stamp);
// degree sum of a slot's frontier over the given CSRs into PState.dsum[side]
hipError_t ws_path_degsum(Workspace* w, int slot, uint64_t n_bound, const PathTypes& pt, int side);
// partitioned: the degree sum of a slot's list over pt into PState::mdsum (summed over ranks by
// the next ws_path_sync_part); no expansion record
hipError_t ws_path_meet_degsum(Workspace* w, int slot, const PathTypes& pt, bool out_edges = false);
// one BFS level: expand slot `src` over pt, claim into lab `bp` fields, pack claims into `dst`
struct PathLevel {
  int lab;                 // label claimed
  uint32_t stamp;
  int rlab = -1;           // restriction label (-1 none)
  uint32_t rstamp = 0;
  int mlab = -1;           // meet-test label (-1 none)
  uint32_t mepoch = 0;
  uint32_t mstamp = 0;     // written into LAB_M for met vertices
  int meet_slot = -1;
  int tlab = -1;           // target label (-1 none)
  uint32_t tstamp = 0;
  const PathTypes* deg = nullptr;   // non-null: k_expand<BFS> also sums the output list's degrees over
                                    // these CSRs into PState.ld[rec] (replaces a k_degsum launch)
  bool global_bound = false;        // partitioned: e_bound is the same on every rank and bounds each
                                    // rank's edges (a degree sum over ranks), so the level may
                                    // exchange slot arrays instead of bitmaps
};
hipError_t ws_path_level(Workspace* w, const PathTypes& pt, int src, uint64_t n_bound, uint64_t e_bound, int dst,
                         const PathLevel& lv);
// greedy lexicographically smallest reconstruction of one path of length L (see path.cpp)
struct PathGreedy {
  int L, kf;
  uint32_t em, eb;         // epochs of LAB_M (positions <= kf) and LAB_B (positions > kf)
  int start_slot;          // B[0] candidates (minimum dense id starts the path)
  int64_t v0_gid = -1;     // partitioned, B[0] = {one source}: its global id and vid (no exchange)
  int64_t v0_vid = 0;
};
hipError_t ws_path_greedy(Workspace* w, const PathTypes& out_types, const PathGreedy& g);
int ws_path_last_rec(Workspace* w);                              // PState record of the last launch
hipError_t ws_path_read_label(Workspace* w, int lab, uint32_t v, uint32_t* out);   // synchronous
hipError_t ws_path_sync(Workspace* w, PState* out, int64_t* path, int path_len);
// FIND ALL PATH (single engine): every walk of 1..upto hops from the sources S (host, local ids)
// whose hops keep the label distance (lab, epoch: backward BFS level from the targets) within
// budget; entry lists appended to *out.  hipErrorOutOfMemory when more than max_walks partial
// walks would be stored.
hipError_t ws_all_paths(Workspace* w, const PathTypes& fwd, int lab, uint32_t epoch, const uint32_t* S, uint64_t nS,
                        uint32_t upto, const int64_t* d_vids, const uint8_t* visible, uint64_t max_walks,
                        std::vector<std::vector<int64_t>>* out, uint64_t* scanned);
// partitioned engine (collective: every rank calls these in the same order)
// FIND ALL PATH: the walks of a level are extended by the owner of their last vertex and the level
// is all-gathered (every rank holds every level); Sgid / Svid: every source (global id, vid), the
// same on every rank.  Every rank appends the same entry lists.
hipError_t ws_all_paths_part(Workspace* w, const PathTypes& fwd, int lab, uint32_t epoch, const uint32_t* Sgid,
                             const int64_t* Svid, uint64_t nS, uint32_t upto, uint64_t nv, const uint8_t* visible,
                             uint64_t max_walks, std::vector<std::vector<int64_t>>* out, uint64_t* scanned);
hipError_t ws_path_level_part(Workspace* w, const PathTypes& pt, int src, uint64_t n_bound, uint64_t e_bound, int dst,
                              const PathLevel& lv);
hipError_t ws_path_sync_part(Workspace* w, PState* out);                 // sizes summed over ranks
hipError_t ws_allreduce_host(Workspace* w, std::vector<unsigned long long>& v);
// greedy over the in-edges (bwd) of the rank's B-set members; writes the 1 + 3L path entries
hipError_t ws_path_greedy_part(Workspace* w, const PathTypes& bwd, const PathGreedy& pg, const int64_t* vids,
                               const uint8_t* visible, int64_t* path);

// FIND SHORTEST / ALL PATH under max_edge_returned_per_vertex (pathcap.hip): the from side walks
// the first K out-edges of each (vertex, type), the to side the first K in-edges, as
// FindPathExecutor sees them through getNeighbors.  Ids are global ids (single engine: dense ids);
// partitioned, every rank calls these collectively with the same endpoints.
struct CapEnv {
  hipStream_t stream = nullptr;
  Comm* comm = nullptr;          // partitioned: the communicator (nullptr: single engine)
  int world = 1, rank = 0;
  uint64_t nv = 0, npad = 0;     // local vertices; global id = rank * npad + local id
  const uint8_t* visible = nullptr;
  const int64_t* vids = nullptr; // local dense id -> vid
  uint32_t K = 0x7fffffff;
};
// one path per reachable target (lexicographically smallest entry list of minimum length);
// hipErrorNotFound: the reconstruction found no edge the B-sets promised
hipError_t cap_shortest(const CapEnv& env, const PathTypes& fwd, const PathTypes& bwd,
                        const std::vector<uint32_t>& Sgid, const std::vector<int64_t>& Svid,
                        const std::vector<uint32_t>& Tgid, uint32_t upto, std::vector<std::vector<int64_t>>* out,
                        uint64_t* scanned);
// every valid walk of 1..upto edges; hipErrorOutOfMemory past max_walks partial walks or paths
hipError_t cap_all(const CapEnv& env, const PathTypes& fwd, const PathTypes& bwd, const std::vector<uint32_t>& Sgid,
                   const std::vector<int64_t>& Svid, const std::vector<uint32_t>& Tgid,
                   const std::vector<int64_t>& Tvid, uint32_t upto, uint64_t max_walks,
                   std::vector<std::vector<int64_t>>* out, uint64_t* scanned);

}  // namespace nbg
