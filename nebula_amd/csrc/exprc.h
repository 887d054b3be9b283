// Expression wire decoding and compilation to the per-edge device bytecode.
#pragma once
#include <memory>
#include <string>
#include <variant>
#include <vector>

#include "nbg_internal.h"

namespace nbg {

// Expression::Kind (src/common/filter/Expressions.h:326-347)
enum EKind : uint8_t {
  EK_PRIMARY = 1, EK_FUNC, EK_UNARY, EK_CAST, EK_ARITH, EK_REL, EK_LOGIC, EK_SRCPROP,
  EK_RANK, EK_DST, EK_SRCID, EK_TYPE, EK_ALIAS, EK_VAR, EK_DSTPROP, EK_INPUT,
};

using CVal = std::variant<int64_t, double, bool, std::string>;   // VariantType

struct Node {
  EKind kind{};
  uint8_t op = 0;
  CVal prim;
  std::string alias, prop;
  std::vector<std::unique_ptr<Node>> kids;
};

// Decodes Expression::encode bytes; nullptr + *err on malformed input.
std::unique_ptr<Node> decode_expr(const uint8_t* p, size_t n, std::string* err);

struct CompileEnv {
  int32_t etype;                                   // edge type of the rows being evaluated
  const std::vector<int32_t>* over;                // OVER types
  const std::map<int32_t, SchemaSet>* edges;       // registered edge schemas
  const std::vector<std::string>* strings;         // sorted string dictionary
  bool has_valid;                                  // the type has edges without a decoded value
  bool has_rank;
  // tag props ($^ / $$)
  const std::map<int32_t, SchemaSet>* tags = nullptr;   // registered tag schemas
  const std::map<int32_t, DevTag>* dtags = nullptr;     // device tag tables (index, columns, kinds)
  // $^ of a source without the tag reads RowReader::getDefaultProp of the RESPONSE edge row
  // schema (GoExecutor.cpp:896-898): `_dst` plus every prop the query names on this edge type
  const std::map<std::string, VKind>* row_cols = nullptr;
  bool partitioned = false;
  std::string* dst_unknown = nullptr;   // set when a $$ tag name is unknown (fails iff E_N > 0)
  uint32_t* probe_mask = nullptr;       // tags read through $$
  // storage-side filter (QueryBaseProcessor.inl:580-606 getters): another edge's alias and the
  // key props `_src/_dst/_rank` read from the value row fail, $^ without the tag fails
  bool storage = false;
  // $-.col / $var.col: the input rows' columns (names, kinds); nullptr: the query has no input
  const std::vector<std::string>* input_names = nullptr;
  const std::vector<VKind>* input_kinds = nullptr;
  // the input holds strings absent from the dictionary (STR_INPUT codes): its string columns are
  // read as derived strings, so compares, casts and YIELDs work on their bytes
  bool input_derived = false;
  uint64_t max_dict_len = 0;   // the longest dictionary string (bounds a derived string's bytes)
};

// One piece of a derived string (a STRING value built on the device: concatenation, casts to
// string, string functions): its bytes are those of a dictionary string (register holding a
// code), of an INT register in decimal, of a BOOL register ("true" / "false"), of a constant, or
// (PC_VIEW) a FunctionManager string function over an inner piece list without views: a window of
// its bytes, case-mapped, between pad bytes drawn cyclically from a second list.
struct Piece {
  PieceKind kind;
  int reg = -1;
  std::string text;            // PC_CONST
  // PC_VIEW: the function (ViewFn), its INT arguments' registers (-1: none), the inner list and
  // the pad list (lpad / rpad)
  uint8_t fn = 0;
  uint8_t cs = 0;              // a case map of the inner bytes merged into a window function (1 lower, 2 upper)
  uint8_t oc = 0;              // a case map of every byte, pads included (an outer lower / upper)
  int reg_b = -1;
  std::vector<Piece> inner, pad;
  uint64_t bound = 0;          // the longest text it can spell (UINT64_MAX: unbounded)
  bool mat = false;            // PC_DICT over a string OP_SMAT materialised (its bound is `bound`)
};

// Result of compiling one expression for one edge type.
struct Compiled {
  VKind kind = VK_INT;
  bool is_const = false;
  int64_t const_bits = 0;     // payload when is_const (strings: dictionary code)
  std::string const_str;      // string constant text (may be absent from the dictionary)
  CVal cval;                  // the constant value when is_const
  bool always_error = false;
  int reg = -1;
  // a derived STRING (kind VK_STRING): its pieces, in order; the registers they read stay live
  // until a sink (compare, cast, truthiness, YIELD) consumes them
  bool derived = false;
  std::vector<Piece> pieces;
};

// Status codes: NBG_OK, NBG_E_UNSUPPORTED, NBG_E_IMPROPER_DATA_TYPE (deferred: the reference
// reports it only when the final step is reached), NBG_E_INVALID_ARGUMENT.
// `data` follows `code` in the device program slot: derived-string piece lists and constant
// bytes, addressed by instructions relative to the data's start (Ins-sized entries).
struct ProgramBuilder {
  std::vector<Ins> code;
  std::vector<Ins> data;
  int next_reg = 0;
  int max_reg = 0;
  // arena bytes one evaluation of every OP_SOUT may store (str_store: a 16-byte header plus the
  // string rounded up to 8), from each piece list's longest possible text
  uint64_t sout_bytes = 0;
};

// yield_value: the expression is a YIELD column (a derived string becomes its canonical code,
// OP_SOUT); otherwise a derived string at the top is a WHERE, read as asBool (empty()).
int32_t compile_expr(const Node& e, const CompileEnv& env, ProgramBuilder& pb, Compiled* out, std::string* err,
                     bool yield_value = false);

// Evaluate constant-only expressions on the host with the reference's exact rules
// (Expressions.cpp eval); returns false if the expression is not constant.
bool fold_constant(const Node& e, CVal* out, bool* error);

int64_t string_code(const std::vector<std::string>& dict, const std::string& s);

// TypeCastingExpression's conversions of one value (Expressions.cpp:773-793): cast type ct
// (ColumnType: 0 INT, 1 STRING, 2 DOUBLE, 3 BIGINT, 4 BOOL, 5 TIMESTAMP); false = evaluation error
bool evalCast(uint8_t ct, const CVal& v, CVal* out);

// ---- result column types (GoExecutor::setupInterimResult's schema, GoExecutor.cpp:707-748)
// The schema of a GO result comes from the first row the reference evaluates: a column's type is
// the type the LAST prop getter of its expression set while evaluating it (operands left before
// right, no short-circuit: Expressions.cpp:835-1131; getters GoExecutor.cpp:851-945), or the cast
// type of a root TypeCasting (:970-974), else (0 here) the value's own kind.  The row context is
// fixed statically (see go_prepare): an edge of `row_type` whose source carries the $^ tags read.
struct ColTypeEnv {
  int32_t row_type = 0;                                 // edge type of the first row
  const std::map<int32_t, SchemaSet>* edges = nullptr;  // registered edge schemas
  const std::map<int32_t, SchemaSet>* tags = nullptr;   // registered tag schemas
  // the response edge row schema of row_type: `_dst` plus every prop the query names on it
  const std::map<std::string, int32_t>* row_types = nullptr;
  const std::vector<std::string>* input_names = nullptr;   // $- / $var columns and their kinds
  const std::vector<VKind>* input_kinds = nullptr;
};
int32_t yield_column_type(const Node& e, const ColTypeEnv& env);   // NBG_T_* or 0 (the value's kind)

}  // namespace nbg
