// Expression wire decoding + static typing + constant folding + bytecode emission.
//
// The reference evaluates WHERE / YIELD by walking an Expression tree of VariantType values
// per edge (src/common/filter/Expressions.cpp:133-1131, GoExecutor.cpp:803-984).  On the
// device every leaf has a static type (schema column types, key props, literals), so each
// node's VariantType alternative is known per OVER edge type and the tree compiles to typed
// 3-address code.  Type errors the reference raises at run time become statically known
// "always error" nodes (OP_ERR): they still fail the query exactly when the reference would,
// i.e. when at least one row evaluates them.  Integer /0 and INT64_MIN/-1 (undefined
// behaviour in the reference) are defined as evaluation errors.
#include "exprc.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <functional>
#include <strings.h>

namespace nbg {

// ============================================================================= decode
namespace {
struct Rd {
  const uint8_t* p;
  const uint8_t* e;
  bool ok = true;
  bool need(size_t n) { if (p + n > e) ok = false; return ok; }
  uint8_t u8() { if (!need(1)) return 0; return *p++; }
  std::string s16() {
    if (!need(2)) return {};
    uint16_t n; memcpy(&n, p, 2); p += 2;
    if (!need(n)) return {};
    std::string s(reinterpret_cast<const char*>(p), n);
    p += n;
    return s;
  }
};

std::unique_ptr<Node> dec(Rd& r, int depth) {
  if (depth > 64) { r.ok = false; return nullptr; }
  uint8_t k = r.u8();
  if (!r.ok) return nullptr;
  auto n = std::make_unique<Node>();
  n->kind = static_cast<EKind>(k);
  switch (k) {
    case EK_PRIMARY: {
      uint8_t which = r.u8();
      if (which == 0) { if (!r.need(8)) return nullptr; int64_t v; memcpy(&v, r.p, 8); r.p += 8; n->prim = v; }
      else if (which == 1) { if (!r.need(8)) return nullptr; double v; memcpy(&v, r.p, 8); r.p += 8; n->prim = v; }
      else if (which == 2) { n->prim = r.u8() != 0; }
      else if (which == 3) { n->prim = r.s16(); }
      else return nullptr;
      break;
    }
    case EK_UNARY: case EK_CAST:
      n->op = r.u8();
      // the cast extension's ColumnType is one of INT, STRING, DOUBLE, BIGINT, BOOL, TIMESTAMP
      // (Expressions.h:21-23; the wire extension is specified in include/nbg.h)
      if (k == EK_CAST && n->op > 5) return nullptr;
      n->kids.push_back(dec(r, depth + 1));
      if (!n->kids[0]) return nullptr;
      break;
    case EK_ARITH: case EK_REL: case EK_LOGIC:
      n->op = r.u8();
      for (int i = 0; i < 2; ++i) {
        n->kids.push_back(dec(r, depth + 1));
        if (!n->kids.back()) return nullptr;
      }
      break;
    case EK_FUNC: {
      n->alias = r.s16();
      if (!r.need(2)) return nullptr;
      uint16_t c; memcpy(&c, r.p, 2); r.p += 2;
      for (uint16_t i = 0; i < c; ++i) {
        n->kids.push_back(dec(r, depth + 1));
        if (!n->kids.back()) return nullptr;
      }
      break;
    }
    case EK_SRCPROP: case EK_ALIAS: case EK_VAR: case EK_DSTPROP:
      n->alias = r.s16();
      n->prop = r.s16();
      break;
    case EK_INPUT:
      n->prop = r.s16();
      break;
    case EK_RANK: case EK_DST: case EK_SRCID: case EK_TYPE:
      n->alias = r.s16();
      n->prop = k == EK_RANK ? "_rank" : k == EK_DST ? "_dst" : k == EK_SRCID ? "_src" : "_type";
      break;
    default:
      return nullptr;
  }
  return r.ok ? std::move(n) : nullptr;
}
}  // namespace

std::unique_ptr<Node> decode_expr(const uint8_t* p, size_t n, std::string* err) {
  Rd r{p, p + n};
  auto e = dec(r, 0);
  if (!e || !r.ok || r.p != r.e) {
    if (err) *err = "malformed expression bytes";
    return nullptr;
  }
  return e;
}

int64_t string_code(const std::vector<std::string>& dict, const std::string& s) {
  auto it = std::lower_bound(dict.begin(), dict.end(), s);
  int64_t idx = it - dict.begin();
  return (it != dict.end() && *it == s) ? 2 * idx : 2 * idx - 1;
}

// ============================================================================= constant folding
namespace {

bool truthy(const CVal& v) {   // Expression::asBool (Expressions.h:228-241)
  switch (v.index()) {
    case 0: return std::get<0>(v) != 0;
    case 1: return std::get<1>(v) != 0.0;
    case 2: return std::get<2>(v);
    default: return std::get<3>(v).empty();
  }
}
double toD(const CVal& v) {
  switch (v.index()) {
    case 0: return (double)std::get<0>(v);
    case 1: return std::get<1>(v);
    case 2: return std::get<2>(v) ? 1.0 : 0.0;
    default: return 0.0;
  }
}
int64_t toI(const CVal& v) {
  switch (v.index()) {
    case 0: return std::get<0>(v);
    case 1: return (int64_t)std::get<1>(v);
    case 2: return std::get<2>(v) ? 1 : 0;
    default: return 0;
  }
}
bool isArith(const CVal& v) { return v.index() <= 1; }

// variant '<' on same alternatives
bool vless(const CVal& a, const CVal& b) {
  switch (a.index()) {
    case 0: return std::get<0>(a) < std::get<0>(b);
    case 1: return std::get<1>(a) < std::get<1>(b);
    case 2: return std::get<2>(a) < std::get<2>(b);
    default: return std::get<3>(a) < std::get<3>(b);
  }
}
bool veq(const CVal& a, const CVal& b) {
  switch (a.index()) {
    case 0: return std::get<0>(a) == std::get<0>(b);
    case 1: return std::get<1>(a) == std::get<1>(b);
    case 2: return std::get<2>(a) == std::get<2>(b);
    default: return std::get<3>(a) == std::get<3>(b);
  }
}

bool evalUnary(uint8_t op, const CVal& v, CVal* out) {      // Expressions.cpp:698-716
  if (op == 0) { *out = v; return true; }
  if (op == 1) {
    if (v.index() == 0) { *out = (int64_t)(0ull - (uint64_t)std::get<0>(v)); return true; }
    if (v.index() == 1) { *out = -std::get<1>(v); return true; }
    return false;
  }
  *out = !truthy(v);
  return true;
}

bool cast_value(uint8_t ct, const CVal& v, CVal* out) {     // Expressions.cpp:773-793
  switch (ct) {
    case 0: case 5:
      if (v.index() == 3) {
        const std::string& s = std::get<3>(v);
        char* end = nullptr; errno = 0;
        long long r = strtoll(s.c_str(), &end, 10);
        if (s.empty() || *end || errno) return false;
        *out = (int64_t)r; return true;
      }
      *out = toI(v); return true;
    case 1:
      if (v.index() == 0) { *out = std::to_string(std::get<0>(v)); return true; }
      if (v.index() == 2) { *out = std::string(std::get<2>(v) ? "true" : "false"); return true; }
      if (v.index() == 3) { *out = v; return true; }
      return false;   // folly::to<std::string>(double): not restated (unpinned)
    case 2:
      if (v.index() == 3) {
        const std::string& s = std::get<3>(v);
        char* end = nullptr;
        double r = strtod(s.c_str(), &end);
        if (s.empty() || *end) return false;
        *out = r; return true;
      }
      *out = toD(v); return true;
    case 4: *out = truthy(v); return true;
    default: return false;   // BIGINT
  }
}

bool evalArith(uint8_t op, const CVal& l, const CVal& r, CVal* out) {   // Expressions.cpp:835-909
  if (isArith(l) && isArith(r)) {
    bool dbl = l.index() == 1 || r.index() == 1;
    if (dbl) {
      double a = toD(l), b = toD(r);
      switch (op) {
        case 0: *out = a + b; return true;
        case 1: *out = a - b; return true;
        case 2: *out = a * b; return true;
        case 3: *out = a / b; return true;
        case 4: *out = std::fmod(a, b); return true;
        case 5: *out = (int64_t)std::llround(a) ^ (int64_t)std::llround(b); return true;
        default: return false;
      }
    }
    uint64_t a = (uint64_t)std::get<0>(l), b = (uint64_t)std::get<0>(r);
    int64_t sa = std::get<0>(l), sb = std::get<0>(r);
    switch (op) {
      case 0: *out = (int64_t)(a + b); return true;
      case 1: *out = (int64_t)(a - b); return true;
      case 2: *out = (int64_t)(a * b); return true;
      case 3: case 4:
        if (sb == 0 || (sa == INT64_MIN && sb == -1)) return false;
        *out = op == 3 ? sa / sb : sa % sb; return true;
      case 5: *out = sa ^ sb; return true;
      default: return false;
    }
  }
  if (op == 0 && l.index() == 3 && r.index() == 3) { *out = std::get<3>(l) + std::get<3>(r); return true; }
  return false;
}

bool evalRel(uint8_t op, CVal l, CVal r, CVal* out) {       // Expressions.cpp:976-1045
  if (l.index() != r.index()) {
    if (l.index() == 3 || r.index() == 3) return false;
    if (l.index() == 1 || r.index() == 1) { l = toD(l); r = toD(r); }
    else { l = toI(l); r = toI(r); }
  }
  if ((op == 4 || op == 5) && isArith(l) && isArith(r) && (l.index() == 1 || r.index() == 1)) {
    bool eq = std::fabs(toD(l) - toD(r)) < 1e-8;
    *out = op == 4 ? eq : !eq;
    return true;
  }
  switch (op) {
    case 0: *out = vless(l, r); return true;
    case 1: *out = !vless(r, l); return true;
    case 2: *out = vless(r, l); return true;
    case 3: *out = !vless(l, r); return true;
    case 4: *out = veq(l, r); return true;
    case 5: *out = !veq(l, r); return true;
    default: return false;
  }
}

bool evalLogic(uint8_t op, const CVal& l, const CVal& r, CVal* out) {   // Expressions.cpp:1103-1131
  bool a = truthy(l), b = truthy(r);
  *out = op == 0 ? (a && b) : op == 1 ? (a || b) : (a != b);
  return true;
}

// ---- FunctionManager (src/common/filter/FunctionManager.cpp:20-487): the table of functions
// with their arity bounds (FunctionManager::getInternal rejects other names and arities)
struct FnDef {
  const char* name;
  int lo, hi;
};
constexpr FnDef kFns[] = {
    {"abs", 1, 1},       {"floor", 1, 1},  {"ceil", 1, 1},     {"round", 1, 1},  {"sqrt", 1, 1},
    {"cbrt", 1, 1},      {"hypot", 2, 2},  {"pow", 2, 2},      {"exp", 1, 1},    {"exp2", 1, 1},
    {"log", 1, 1},       {"log2", 1, 1},   {"log10", 1, 1},    {"sin", 1, 1},    {"asin", 1, 1},
    {"cos", 1, 1},       {"acos", 1, 1},   {"tan", 1, 1},      {"atan", 1, 1},   {"rand32", 0, 2},
    {"rand64", 0, 2},    {"now", 0, 0},    {"strcasecmp", 2, 2}, {"lower", 1, 1}, {"upper", 1, 1},
    {"length", 1, 1},    {"trim", 1, 1},   {"ltrim", 1, 1},    {"rtrim", 1, 1},  {"left", 2, 2},
    {"right", 2, 2},     {"lpad", 3, 3},   {"rpad", 3, 3},     {"substr", 3, 3}, {"hash", 1, 1},
    {"udf_is_in", 2, 1 << 30}};

const FnDef* fn_def(const std::string& f) {
  for (const FnDef& d : kFns)
    if (f == d.name) return &d;
  return nullptr;
}

// the one-argument double functions beyond abs / floor / ceil / round / sqrt, in OP_MATH1_F's order
constexpr const char* kMath1[] = {"cbrt", "exp", "exp2", "log", "log2", "log10", "sin", "asin", "cos", "acos",
                                  "tan", "atan"};
int math1_id(const std::string& f) {
  for (int i = 0; i < (int)(sizeof(kMath1) / sizeof(kMath1[0])); ++i)
    if (f == kMath1[i]) return i;
  return -1;
}
double math1(int id, double x) {
  switch (id) {
    case 0: return std::cbrt(x);
    case 1: return std::exp(x);
    case 2: return std::exp2(x);
    case 3: return std::log(x);
    case 4: return std::log2(x);
    case 5: return std::log10(x);
    case 6: return std::sin(x);
    case 7: return std::asin(x);
    case 8: return std::cos(x);
    case 9: return std::acos(x);
    case 10: return std::tan(x);
    default: return std::atan(x);
  }
}

// Expression::asDouble / asInt / asString (Expressions.h:217-246): boost::get, so an argument of
// another kind throws (bad_get) — an evaluation error here
bool as_double(const CVal& v, double* d) {
  if (v.index() == 0) { *d = (double)std::get<0>(v); return true; }
  if (v.index() == 1) { *d = std::get<1>(v); return true; }
  return false;
}

// A function body of FunctionManager.cpp over constant arguments, as the reference runs it (on
// the host the compiler's own std::hash is libstdc++'s, as the reference's).  false: the body
// throws (an argument of another kind), or would not return (lpad / rpad with a negative size or,
// padding, an empty pad: their loop never ends) — an evaluation error here.  rand32 / rand64 /
// now are never folded (a value per evaluation / per query).
bool fm_eval(const std::string& f, const std::vector<CVal>& a, CVal* out) {
  double x = 0, y = 0;
  if (f == "abs" || f == "floor" || f == "ceil" || f == "round" || f == "sqrt" || math1_id(f) >= 0) {
    if (!as_double(a[0], &x)) return false;
    *out = f == "abs" ? std::fabs(x) : f == "floor" ? std::floor(x) : f == "ceil" ? std::ceil(x)
         : f == "round" ? std::round(x) : f == "sqrt" ? std::sqrt(x) : math1(math1_id(f), x);
    return true;
  }
  if (f == "hypot" || f == "pow") {
    if (!as_double(a[0], &x) || !as_double(a[1], &y)) return false;
    *out = f == "hypot" ? std::hypot(x, y) : std::pow(x, y);
    return true;
  }
  if (f == "hash") {
    switch (a[0].index()) {
      case 0: *out = (int64_t)std::hash<int64_t>{}(std::get<0>(a[0])); return true;
      case 1: *out = (int64_t)std::hash<double>{}(std::get<1>(a[0])); return true;
      case 2: *out = (int64_t)std::hash<bool>{}(std::get<2>(a[0])); return true;
      default: *out = (int64_t)std::hash<std::string>{}(std::get<3>(a[0])); return true;
    }
  }
  // string functions: asString of the first argument (and of strcasecmp's second / a pad)
  for (size_t i = 0; i < a.size(); ++i) {
    const bool str = i == 0 || (f == "strcasecmp") || ((f == "lpad" || f == "rpad") && i == 2);
    if (str ? a[i].index() != 3 : a[i].index() != 0) return false;   // the others: asInt
  }
  const std::string& v = std::get<3>(a[0]);
  if (f == "strcasecmp") {   // glibc's strcasecmp: the difference of the first differing lowered bytes
    *out = (int64_t)::strcasecmp(v.c_str(), std::get<3>(a[1]).c_str());
    return true;
  }
  if (f == "length") { *out = (int64_t)v.length(); return true; }
  if (f == "lower" || f == "upper") {
    std::string r = v;
    for (char& ch : r) {
      const unsigned char u = (unsigned char)ch;
      if (f == "lower" && u >= 'A' && u <= 'Z') ch = (char)(u + 32);
      if (f == "upper" && u >= 'a' && u <= 'z') ch = (char)(u - 32);
    }
    *out = r;
    return true;
  }
  if (f == "trim" || f == "ltrim" || f == "rtrim") {
    std::string r = v;
    if (f != "rtrim") r.erase(0, r.find_first_not_of(" "));
    if (f != "ltrim") r.erase(r.find_last_not_of(" ") + 1);
    *out = r;
    return true;
  }
  const int64_t n = std::get<0>(a[1]);
  if (f == "left") { *out = n <= 0 ? std::string() : v.substr(0, (size_t)n); return true; }
  if (f == "right") {
    if (n <= 0) { *out = std::string(); return true; }
    const size_t k = (uint64_t)n > v.size() ? v.size() : (size_t)n;
    *out = v.substr(v.size() - k);
    return true;
  }
  if (f == "lpad" || f == "rpad") {
    const std::string& pad = std::get<3>(a[2]);
    if (n < 0) return false;                       // size_t size: the padding loop never ends
    if ((uint64_t)n < v.size()) { *out = v.substr(0, (size_t)n); return true; }
    size_t need = (size_t)n - v.size();
    if (need && pad.empty()) return false;         // the loop never ends
    std::string p;
    while (need > pad.size()) { p += pad; need -= pad.size(); }
    p += pad.substr(0, need);
    *out = f == "lpad" ? p + v : v + p;
    return true;
  }
  if (f == "substr") {
    const int64_t start = n, len = std::get<0>(a[2]);
    const uint64_t ast = start == INT64_MIN ? (uint64_t)1 << 63 : (uint64_t)(start < 0 ? -start : start);
    if (ast > v.size() || len <= 0 || start == 0) { *out = std::string(); return true; }
    *out = start > 0 ? v.substr((size_t)start - 1, (size_t)len) : v.substr(v.size() - ast, (size_t)len);
    return true;
  }
  return false;
}

}  // namespace

bool evalCast(uint8_t ct, const CVal& v, CVal* out) { return cast_value(ct, v, out); }

bool fold_constant(const Node& e, CVal* out, bool* error) {
  *error = false;
  switch (e.kind) {
    case EK_PRIMARY: *out = e.prim; return true;
    case EK_UNARY: case EK_CAST: {
      CVal v; bool er;
      if (!fold_constant(*e.kids[0], &v, &er)) return false;
      if (er) { *error = true; return true; }
      bool ok = e.kind == EK_UNARY ? evalUnary(e.op, v, out) : cast_value(e.op, v, out);
      *error = !ok;
      return true;
    }
    case EK_ARITH: case EK_REL: case EK_LOGIC: {
      CVal a, b; bool ea, eb;
      if (!fold_constant(*e.kids[0], &a, &ea) || !fold_constant(*e.kids[1], &b, &eb)) return false;
      if (ea || eb) { *error = true; return true; }
      bool ok = e.kind == EK_ARITH ? evalArith(e.op, a, b, out)
              : e.kind == EK_REL ? evalRel(e.op, a, b, out) : evalLogic(e.op, a, b, out);
      *error = !ok;
      return true;
    }
    default: return false;   // props, EdgeType (validated against OVER first), functions
  }
}

// ============================================================================= emission
namespace {

struct Ctx {
  const CompileEnv& env;
  ProgramBuilder& pb;
  std::string* err;
  int max_reg = 0;
  int top = 0;               // stack discipline: next free register

  int push() {
    int r = top++;
    if (top > max_reg) max_reg = top;
    return r;
  }
  void emit(uint8_t op, int d, int a = 0, int b = 0, int32_t aux = 0, int64_t imm = 0) {
    pb.code.push_back(Ins{op, (uint8_t)d, (uint8_t)a, (uint8_t)b, aux, imm});
  }
  VKind kind_of(const CVal& v) { return static_cast<VKind>(v.index()); }
  int64_t bits_of(const CVal& v) {
    switch (v.index()) {
      case 0: return std::get<0>(v);
      case 1: { double d = std::get<1>(v); int64_t b; memcpy(&b, &d, 8); return b; }
      case 2: return std::get<2>(v) ? 1 : 0;
      default: return string_code(*env.strings, std::get<3>(v));
    }
  }
  Compiled make_const(const CVal& v) {
    Compiled c;
    c.kind = kind_of(v);
    c.is_const = true;
    c.const_bits = bits_of(v);
    c.cval = v;
    if (v.index() == 3) c.const_str = std::get<3>(v);
    return c;
  }
  Compiled make_error() {
    Compiled c;
    c.always_error = true;
    c.kind = VK_INT;
    c.reg = push();
    emit(OP_ERR, c.reg);
    return c;
  }
  // materialise a constant operand into the top register
  int materialize(Compiled& c) {
    if (!c.is_const) return c.reg;
    c.reg = push();
    emit(OP_CONST, c.reg, 0, 0, 0, c.const_bits);
    return c.reg;
  }
  // ---- derived strings: piece lists in the program's data
  std::vector<Piece> pieces_of(const Compiled& c) {
    if (c.derived) return c.pieces;
    if (c.is_const) return {Piece{PC_CONST, -1, c.const_str}};
    return {Piece{PC_DICT, c.reg, {}}};
  }
  // the lowest register the pieces read (views: their arguments' and inner lists' too)
  static int low_reg(const std::vector<Piece>& ps) {
    int r = -1;
    auto take = [&r](int q) {
      if (q >= 0 && (r < 0 || q < r)) r = q;
    };
    for (auto& p : ps) {
      take(p.reg);
      take(p.reg_b);
      take(low_reg(p.inner));
      take(low_reg(p.pad));
    }
    return r;
  }
  // the longest text a piece list can spell (UINT64_MAX: unbounded)
  uint64_t bound_of(const std::vector<Piece>& ps) const {
    uint64_t most = 0;
    for (const Piece& p : ps) {
      const uint64_t b = p.kind == PC_CONST ? p.text.size() : p.kind == PC_INT ? 20 : p.kind == PC_BOOL ? 5
                       : (p.kind == PC_VIEW || p.mat) ? p.bound : env.max_dict_len;
      most = b > UINT64_MAX - most ? UINT64_MAX : most + b;
    }
    return most;
  }
  // header entry {d = pieces, aux = first piece}, the pieces {op = kind, d = reg, aux = byte offset
  // of a constant's bytes from the data's start, imm = its length}, then the constants' bytes.  A
  // view's inner and pad lists are emitted first (flat lists: a view holds no view)
  int32_t emit_pieces(const std::vector<Piece>& ps) {
    auto& D = pb.data;
    std::vector<std::pair<int32_t, int32_t>> sub(ps.size(), {0, 0});
    for (size_t k = 0; k < ps.size(); ++k)
      if (ps[k].kind == PC_VIEW) sub[k] = {emit_pieces(ps[k].inner), ps[k].pad.empty() ? 0 : emit_pieces(ps[k].pad)};
    const int32_t hdr = (int32_t)D.size();
    D.push_back(Ins{0, (uint8_t)ps.size(), 0, 0, hdr + 1, 0});
    for (size_t k = 0; k < ps.size(); ++k) {
      const Piece& p = ps[k];
      if (p.kind == PC_VIEW)
        D.push_back(Ins{(uint8_t)PC_VIEW, (uint8_t)(p.reg < 0 ? 0 : p.reg), p.fn, (uint8_t)(p.reg_b < 0 ? 0 : p.reg_b),
                        sub[k].first, (int64_t)sub[k].second | (int64_t)p.cs << 32 | (int64_t)p.oc << 34});
      else
        D.push_back(Ins{(uint8_t)p.kind, (uint8_t)(p.reg < 0 ? 0 : p.reg), 0, 0, 0, (int64_t)p.text.size()});
    }
    for (size_t k = 0; k < ps.size(); ++k) {
      if (ps[k].kind != PC_CONST || ps[k].text.empty()) continue;
      const size_t at = D.size();
      D[hdr + 1 + k].aux = (int32_t)(at * sizeof(Ins));
      D.resize(at + (ps[k].text.size() + sizeof(Ins) - 1) / sizeof(Ins), Ins{});
      memcpy(reinterpret_cast<char*>(D.data() + at), ps[k].text.data(), ps[k].text.size());
    }
    return hdr;
  }
  // the register a sink over these pieces writes (the lowest one they read: all are read first)
  int sink_reg(const std::vector<Piece>& a, const std::vector<Piece>& b = {}) {
    int r = low_reg(a), q = low_reg(b);
    if (q >= 0 && (r < 0 || q < r)) r = q;
    if (r < 0) r = push();
    top = r + 1;
    if (top > max_reg) max_reg = top;
    return r;
  }
  Compiled derived_of(std::vector<Piece> ps) {
    Compiled c;
    c.kind = VK_STRING;
    c.derived = true;
    c.pieces = std::move(ps);
    c.reg = low_reg(c.pieces);
    return c;
  }
  // asBool of a derived string: empty() (Expressions.h:228-241)
  int empty_reg(const Compiled& c) {
    const int32_t h = emit_pieces(c.pieces);
    const int r = sink_reg(c.pieces);
    emit(OP_SEMPTY, r, 0, 0, h);
    return r;
  }
  // a derived string as a result value: its canonical code (OP_SOUT)
  int value_reg(const Compiled& c) {
    // the longest text the pieces can spell (an unbounded one, lpad / rpad to a per-edge length,
    // reserves the arena's cap: past it the query fails with E_OUT_OF_MEMORY)
    const uint64_t most = std::min<uint64_t>(bound_of(c.pieces), 1ull << 40);
    const uint64_t add = 16 + ((most + 7) & ~7ull);
    pb.sout_bytes = add > UINT64_MAX - pb.sout_bytes ? UINT64_MAX : pb.sout_bytes + add;
    const int32_t h = emit_pieces(c.pieces);
    const int r = sink_reg(c.pieces);
    emit(OP_SOUT, r, 0, 0, h);
    return r;
  }

  int truthy_reg(Compiled& c) {
    if (c.derived) return empty_reg(c);
    int r = materialize(c);
    switch (c.kind) {
      case VK_INT: emit(OP_TRUTHY_I, r, r); break;
      case VK_DOUBLE: emit(OP_TRUTHY_F, r, r); break;
      case VK_BOOL: break;
      case VK_STRING: emit(OP_TRUTHY_S, r, r, 0, 0, string_code(*env.strings, "")); break;
    }
    return r;
  }
  const SchemaSet* edge_by_name(const std::string& name, int32_t* type) {
    for (auto& kv : *env.edges) {
      if (kv.second.name == name) { *type = kv.first; return &kv.second; }
    }
    return nullptr;
  }

  int32_t leaf_alias(const Node& e, Compiled* out) {
    // GoExecutor::processFinalResult getAliasProp (GoExecutor.cpp:851-878)
    int32_t et;
    const SchemaSet* ss = edge_by_name(e.alias, &et);
    if (!ss || (!env.storage && std::find(env.over->begin(), env.over->end(), et) == env.over->end())) {
      *err = "the edge was not found '" + e.alias + "'";
      return NBG_E_EXECUTION_ERROR;   // deferred to the final step (getStepOutProps)
    }
    bool key = e.prop == "_dst" || e.prop == "_src" || e.prop == "_rank" || e.prop == "_type";
    if (env.storage && (et != env.etype || key)) {   // "ignore this edge" / "Invalid Prop"
      *out = make_error();
      return NBG_OK;
    }
    const Schema* sc = ss->latest();
    int col = (!key && sc) ? sc->find(e.prop) : -1;
    if (!key && col < 0) {
      *err = "prop `" + e.alias + "." + e.prop + "' not found";
      return NBG_E_IMPROPER_DATA_TYPE;   // storage rejects the request (inl:275-286); deferred
    }
    if (et != env.etype) {
      // another OVER edge: the schema default of its response column (RowReader::getDefaultProp)
      if (key) { *out = make_const(CVal(int64_t(0))); return NBG_OK; }
      switch (kindOfType(sc->cols[col].type)) {
        case VK_BOOL: *out = make_const(CVal(false)); break;
        case VK_DOUBLE: *out = make_const(CVal(0.0)); break;
        case VK_STRING: *out = make_const(CVal(std::string())); break;
        default: *out = make_const(CVal(int64_t(0))); break;
      }
      return NBG_OK;
    }
    Compiled c;
    c.kind = VK_INT;
    if (e.prop == "_type") { *out = make_const(CVal((int64_t)et)); return NBG_OK; }
    c.reg = push();
    if (e.prop == "_dst") emit(OP_DST, c.reg);
    else if (e.prop == "_src") emit(OP_SRC, c.reg);
    else if (e.prop == "_rank") emit(OP_RANK, c.reg);
    else {
      c.kind = kindOfType(sc->cols[col].type);
      emit(env.has_valid ? OP_COLV : OP_COL, c.reg, 0, 0, col);
    }
    *out = c;
    return NBG_OK;
  }

  const SchemaSet* tag_by_name(const std::string& name, int32_t* tag) {
    if (!env.tags) return nullptr;
    for (auto& kv : *env.tags) {
      if (kv.second.name == name) { *tag = kv.first; return &kv.second; }
    }
    return nullptr;
  }
  int64_t default_bits(VKind k) {   // RowReader::getDefaultProp: 0, 0.0, false, ""
    return k == VK_STRING ? string_code(*env.strings, "") : 0;
  }
  // the tag column `e.prop` of tag `e.alias`: NBG_OK with *col < 0 when the prop is unknown
  int32_t tag_column(const Node& e, const DevTag** dt, int* col) {
    int32_t tid;
    const SchemaSet* ts = tag_by_name(e.alias, &tid);
    *col = -1;
    *dt = nullptr;
    if (!ts) return NBG_E_TAG_PROP_NOT_FOUND;
    if (!env.dtags || !env.dtags->count(tid)) {
      *err = "tag tables missing";
      return NBG_E_UNSUPPORTED;
    }
    *dt = &env.dtags->at(tid);
    const Schema* sc = ts->latest();
    *col = sc ? sc->find(e.prop) : -1;
    return NBG_OK;
  }

  // $^.tag.prop: GoExecutor's source getter over the getNeighbors tag data
  // (GoExecutor.cpp:888-905); the tag / prop name checks are the storage request's
  // (getStepOutProps :603-612, QueryBaseProcessor.inl:77-100) and fail the final step.
  int32_t leaf_src_tag(const Node& e, Compiled* out) {
    const DevTag* dt;
    int col;
    int32_t rc = tag_column(e, &dt, &col);
    if (rc == NBG_E_TAG_PROP_NOT_FOUND) {
      *err = "No schema found for '" + e.alias + "'";
      return NBG_E_EXECUTION_ERROR;   // deferred to the final step
    }
    if (rc) return rc;
    if (col < 0) {
      *err = "Get neighbors failed: prop `" + e.alias + "." + e.prop + "' not found";
      return NBG_E_IMPROPER_DATA_TYPE;   // deferred to the final step
    }
    Compiled c;
    c.kind = dt->kind[col];
    const int32_t aux = (dt->index << 16) | (dt->col_base + col);
    const bool has_default = !env.storage && env.row_cols && env.row_cols->count(e.prop);
    c.reg = push();
    if (!has_default) {
      emit(OP_TAGS_E, c.reg, 0, 0, aux, 0);   // no such column in the row schema: "Unknown type"
    } else {
      if (env.row_cols->at(e.prop) != c.kind) {
        *err = "$^ prop whose missing-tag default has another type";
        return NBG_E_UNSUPPORTED;
      }
      emit(OP_TAGS, c.reg, 0, 0, aux, default_bits(c.kind));
    }
    *out = c;
    return NBG_OK;
  }

  // $$.tag.prop: VertexHolder::get over the final destinations' tag data (GoExecutor.cpp:986-1064)
  int32_t leaf_dst_tag(const Node& e, Compiled* out) {
    const DevTag* dt;
    int col;
    int32_t rc = tag_column(e, &dt, &col);
    if (rc == NBG_E_TAG_PROP_NOT_FOUND) {
      // fetchVertexProps fails the query once the final step returned edges (GoExecutor.cpp:652-690)
      if (env.dst_unknown && env.dst_unknown->empty()) *env.dst_unknown = "No schema found for '" + e.alias + "'";
      *out = make_error();
      return NBG_OK;
    }
    if (rc) return rc;
    if (col < 0) {   // getVertexProps rejects the request: the holder is empty -> "Unknown Vertex"
      *out = make_error();
      return NBG_OK;
    }
    if (dt->index >= MAX_TAG_BITS) {
      *err = "$$ over more than 16 tags";
      return NBG_E_UNSUPPORTED;
    }
    Compiled c;
    c.kind = dt->kind[col];
    c.reg = push();
    emit(OP_TAGD, c.reg, 0, 0, (dt->index << 16) | (dt->col_base + col), default_bits(c.kind));
    if (env.probe_mask) *env.probe_mask |= 1u << dt->index;
    *out = c;
    return NBG_OK;
  }

  int32_t compile(const Node& e, Compiled* out) {
    // constant subtrees fold on the host with the reference's exact rules
    {
      CVal v; bool error;
      if (fold_constant(e, &v, &error)) {
        *out = error ? make_error() : make_const(v);
        return NBG_OK;
      }
    }
    switch (e.kind) {
      case EK_ALIAS: case EK_DST: case EK_SRCID: case EK_RANK:
        return leaf_alias(e, out);
      case EK_TYPE: {
        int32_t et;
        const SchemaSet* ss = edge_by_name(e.alias, &et);
        if (!env.storage && (!ss || std::find(env.over->begin(), env.over->end(), et) == env.over->end())) {
          *err = "the edge was not found '" + e.alias + "'";
          return NBG_E_EXECUTION_ERROR;
        }
        *out = make_const(CVal(e.alias));
        return NBG_OK;
      }
      case EK_SRCPROP: return leaf_src_tag(e, out);
      case EK_DSTPROP: return leaf_dst_tag(e, out);
      case EK_INPUT: case EK_VAR: {
        // GoExecutor getInputProp / getVariableProp -> InterimResultIndex::getColumnWithVID
        // (GoExecutor.cpp:932-945, InterimResult.cpp:252-270): the column of the root's input row
        if (!env.input_names) {
          *err = "input/variable props without an input";
          return NBG_E_EXECUTION_ERROR;
        }
        auto it = std::find(env.input_names->begin(), env.input_names->end(), e.prop);
        if (it == env.input_names->end()) {   // "Prop `x' not found": an evaluation error
          *out = make_error();
          return NBG_OK;
        }
        const int col = (int)(it - env.input_names->begin());
        Compiled c;
        c.kind = (*env.input_kinds)[col];
        c.reg = push();
        emit(OP_INPUT, c.reg, 0, 0, col);
        if (c.kind == VK_STRING && env.input_derived) c = derived_of({Piece{PC_DICT, c.reg, {}}});
        *out = c;
        return NBG_OK;
      }
      case EK_FUNC: return function(e, out);
      case EK_UNARY: {
        Compiled a;
        int32_t rc = compile(*e.kids[0], &a);
        if (rc) return rc;
        if (a.always_error) { *out = a; return NBG_OK; }
        if (a.is_const) {
          CVal v;
          *out = evalUnary(e.op, a.cval, &v) ? make_const(v) : make_error();
          return NBG_OK;
        }
        if (e.op == 0) { *out = a; return NBG_OK; }
        if (e.op == 1) {
          if (!a.derived && (a.kind == VK_INT || a.kind == VK_DOUBLE)) {
            int r = materialize(a);
            emit(a.kind == VK_INT ? OP_NEG_I : OP_NEG_F, r, r);
            *out = a;
            return NBG_OK;
          }
          *out = make_error();
          return NBG_OK;
        }
        int r = truthy_reg(a);
        emit(OP_NOT, r, r);
        Compiled c; c.kind = VK_BOOL; c.reg = r;
        *out = c;
        return NBG_OK;
      }
      case EK_CAST: {
        Compiled a;
        int32_t rc = compile(*e.kids[0], &a);
        if (rc) return rc;
        if (a.always_error) { *out = a; return NBG_OK; }
        if (a.is_const) {
          CVal v;
          *out = cast_value(e.op, a.cval, &v) ? make_const(v) : make_error();
          return NBG_OK;
        }
        if (a.derived) {   // a concatenation / cast result: parsed from its bytes
          Compiled c;
          switch (e.op) {
            case 0: case 5: case 2: {
              const int32_t h = emit_pieces(a.pieces);
              c.reg = sink_reg(a.pieces);
              c.kind = e.op == 2 ? VK_DOUBLE : VK_INT;
              emit(e.op == 2 ? OP_SPARSE_F : OP_SPARSE_I, c.reg, 0, 0, h);
              break;
            }
            case 4: c.reg = empty_reg(a); c.kind = VK_BOOL; break;
            case 1: c = a; break;
            default: *out = make_error(); return NBG_OK;
          }
          *out = c;
          return NBG_OK;
        }
        if (e.op == 1) {   // to STRING (Expression::toString): a derived string of the value's text
          switch (a.kind) {
            case VK_STRING: *out = a; return NBG_OK;
            case VK_INT: *out = derived_of({Piece{PC_INT, a.reg, {}}}); return NBG_OK;
            case VK_BOOL: *out = derived_of({Piece{PC_BOOL, a.reg, {}}}); return NBG_OK;
            // folly::to<std::string>(double) is not restated (unpinned, as for constants)
            default: *out = make_error(); return NBG_OK;
          }
        }
        Compiled c; c.reg = materialize(a);
        switch (e.op) {
          case 0: case 5:
            c.kind = VK_INT;
            if (a.kind == VK_DOUBLE) emit(OP_F2I, c.reg, c.reg);
            else if (a.kind == VK_BOOL) emit(OP_B2I, c.reg, c.reg);
            else if (a.kind == VK_STRING) emit(OP_S2I, c.reg, c.reg);   // per-string table
            break;
          case 2:
            c.kind = VK_DOUBLE;
            if (a.kind == VK_INT) emit(OP_I2F, c.reg, c.reg);
            else if (a.kind == VK_BOOL) emit(OP_B2F, c.reg, c.reg);
            else if (a.kind == VK_STRING) emit(OP_S2F, c.reg, c.reg);
            break;
          case 4:
            c.reg = truthy_reg(a);
            c.kind = VK_BOOL;
            break;
          default:
            *out = make_error();
            return NBG_OK;
        }
        *out = c;
        return NBG_OK;
      }
      case EK_ARITH: case EK_REL: case EK_LOGIC: {
        Compiled a, b;
        int32_t rc = compile(*e.kids[0], &a);
        if (rc) return rc;
        rc = compile(*e.kids[1], &b);
        if (rc) return rc;
        if (a.always_error || b.always_error) {
          Compiled c = a.always_error ? a : b;
          c.always_error = true;
          *out = c;
          return NBG_OK;
        }
        return binary(e, a, b, out);
      }
      default:
        *err = "unsupported expression kind";
        return NBG_E_UNSUPPORTED;
    }
  }

  // FunctionCallExpression (Expressions.cpp:589-621) over FunctionManager's functions
  // (FunctionManager.cpp:20-487): a name the manager does not define, or the wrong arity, fails
  // the statement as FunctionManager::get does.  Arguments are evaluated left to right before the
  // call; an argument's error is the call's error.  Constant arguments fold on the host with the
  // reference's bodies (fm_eval); otherwise the call is a device op: the double math, hash,
  // length, strcasecmp, rand32 / rand64 and now; the string-valued functions (lower, upper, trim,
  // ltrim, rtrim, left, right, lpad, rpad, substr) become PC_VIEW pieces of a derived string (one
  // level: a string function over another's per-edge result is NBG_E_UNSUPPORTED).
  static int view_fn(const std::string& f) {
    static const char* const names[] = {"lower", "upper", "trim", "ltrim", "rtrim", "left", "right", "lpad", "rpad",
                                        "substr"};
    for (int i = 0; i < 10; ++i)
      if (f == names[i]) return i;
    return -1;
  }
  int32_t function(const Node& e, Compiled* out) {
    const std::string& f = e.alias;
    const size_t n = e.kids.size();
    const FnDef* def = fn_def(f);
    if (!def) {
      *err = "Function `" + f + "' not defined";
      return NBG_E_EXECUTION_ERROR;
    }
    if ((int)n < def->lo || (int)n > def->hi) {
      *err = "Arity not match for function `" + f + "'";
      return NBG_E_EXECUTION_ERROR;
    }
    if (f == "udf_is_in") return is_in(e, out);
    std::vector<Compiled> args(n);
    for (size_t i = 0; i < n; ++i) {
      const int32_t rc = compile(*e.kids[i], &args[i]);
      if (rc) return rc;
    }
    for (auto& x : args)
      if (x.always_error) { *out = make_error(); return NBG_OK; }
    const bool varying = f == "rand32" || f == "rand64" || f == "now";   // a value per evaluation / query
    bool all_const = true;
    for (auto& x : args) all_const = all_const && x.is_const && !x.derived;
    if (all_const && !varying) {
      std::vector<CVal> cv;
      for (auto& x : args) cv.push_back(x.cval);
      CVal r;
      *out = fm_eval(f, cv, &r) ? make_const(r) : make_error();
      return NBG_OK;
    }
    auto numeric = [](const Compiled& x) { return !x.derived && (x.kind == VK_INT || x.kind == VK_DOUBLE); };
    auto as_double_reg = [&](Compiled& x) {   // Expression::asDouble: an INT widens
      const int r = materialize(x);
      if (x.kind == VK_INT) emit(OP_I2F, r, r);
      return r;
    };
    Compiled c;
    static const char* exact[] = {"abs", "floor", "ceil", "round", "sqrt"};
    static const uint8_t exact_op[] = {OP_ABS_F, OP_FLOOR_F, OP_CEIL_F, OP_ROUND_F, OP_SQRT_F};
    int xi = -1;
    for (int i = 0; i < 5; ++i)
      if (f == exact[i]) xi = i;
    if (xi >= 0 || math1_id(f) >= 0) {
      if (!numeric(args[0])) { *out = make_error(); return NBG_OK; }   // boost::bad_get
      c.reg = as_double_reg(args[0]);
      if (xi >= 0) emit(exact_op[xi], c.reg, c.reg);
      else emit(OP_MATH1_F, c.reg, c.reg, 0, math1_id(f));
      c.kind = VK_DOUBLE;
    } else if (f == "pow" || f == "hypot") {
      if (!numeric(args[0]) || !numeric(args[1])) { *out = make_error(); return NBG_OK; }
      const int ra = as_double_reg(args[0]);
      const int rb = as_double_reg(args[1]);
      c.reg = std::min(ra, rb);
      emit(OP_MATH2_F, c.reg, ra, rb, f == "pow" ? 0 : 1);
      c.kind = VK_DOUBLE;
    } else if (f == "hash") {
      Compiled& x = args[0];
      c.kind = VK_INT;
      if (x.kind == VK_STRING) {   // std::hash<std::string>: the bytes, whatever made them
        const std::vector<Piece> ps = pieces_of(x);
        const int32_t h = emit_pieces(ps);
        c.reg = sink_reg(ps);
        emit(OP_HASH_S, c.reg, 0, 0, h);
      } else {
        c.reg = materialize(x);   // std::hash<int64_t> / <bool>: the value itself
        if (x.kind == VK_DOUBLE) emit(OP_HASH_F, c.reg, c.reg);
      }
    } else if (f == "length" || f == "strcasecmp") {
      for (auto& x : args)
        if (x.kind != VK_STRING) { *out = make_error(); return NBG_OK; }   // asString: bad_get
      const std::vector<Piece> pa = pieces_of(args[0]);
      const std::vector<Piece> pq = n > 1 ? pieces_of(args[1]) : std::vector<Piece>{};
      const int32_t ha = emit_pieces(pa);
      const int32_t hb = n > 1 ? emit_pieces(pq) : 0;
      c.reg = sink_reg(pa, pq);
      if (f == "length") emit(OP_SLEN, c.reg, 0, 0, ha);
      else emit(OP_SCASE, c.reg, 0, 0, ha, hb);
      c.kind = VK_INT;
    } else if (f == "rand32" || f == "rand64") {
      int r[2] = {0, 0};
      for (size_t i = 0; i < n; ++i) {
        if (args[i].derived || args[i].kind != VK_INT) { *out = make_error(); return NBG_OK; }   // asInt
        r[i] = materialize(args[i]);
      }
      c.reg = n ? std::min(r[0], n > 1 ? r[1] : r[0]) : push();
      emit(OP_RAND, c.reg, r[0], r[1], (int32_t)n | (f == "rand64" ? 4 : 0));
      c.kind = VK_INT;
    } else if (f == "now") {
      c.reg = push();
      emit(OP_NOW, c.reg);
      c.kind = VK_INT;
    } else if (view_fn(f) >= 0) {
      const uint8_t vf = (uint8_t)view_fn(f);
      const bool pads = vf == VF_LPAD || vf == VF_RPAD;
      const size_t nint = vf == VF_SUBSTR ? 2 : (vf == VF_LEFT || vf == VF_RIGHT || pads) ? 1 : 0;
      if (args[0].kind != VK_STRING || (pads && args[2].kind != VK_STRING)) { *out = make_error(); return NBG_OK; }
      for (size_t i = 1; i <= nint; ++i)
        if (args[i].derived || args[i].kind != VK_INT) { *out = make_error(); return NBG_OK; }   // asInt
      Piece v;
      v.kind = PC_VIEW;
      v.fn = vf;
      v.inner = pieces_of(args[0]);
      if (pads) v.pad = pieces_of(args[2]);
      bool nested = false;
      for (const auto* l : {&v.inner, &v.pad})
        for (const Piece& p : *l) nested = nested || p.kind == PC_VIEW;
      const bool casefn = vf == VF_LOWER || vf == VF_UPPER;
      if (nested && casefn) {
        // lower / upper over a list holding views: every byte mapped.  Runs of flat pieces become
        // case views; a view keeps its function and gets the map over all its bytes (pads too)
        std::vector<Piece> mapped, run;
        auto flush = [&] {
          if (run.empty()) return;
          Piece w;
          w.kind = PC_VIEW;
          w.fn = vf;
          w.inner = std::move(run);
          w.bound = bound_of(w.inner);
          mapped.push_back(std::move(w));
          run.clear();
        };
        for (Piece& p : v.inner) {
          if (p.kind != PC_VIEW) {
            run.push_back(std::move(p));
            continue;
          }
          flush();
          p.oc = vf == VF_LOWER ? 1 : 2;
          mapped.push_back(std::move(p));
        }
        flush();
        *out = derived_of(std::move(mapped));
        return NBG_OK;
      }
      bool pad_views = false;
      for (const Piece& p : v.pad) pad_views = pad_views || p.kind == PC_VIEW;
      if (nested && !pad_views && v.inner.size() == 1 && v.inner[0].kind == PC_VIEW && !v.inner[0].oc &&
          (v.inner[0].fn == VF_LOWER || v.inner[0].fn == VF_UPPER)) {
        // a window / trim / pad over lower(x) or upper(x): case maps keep lengths and spaces, so
        // the window is the same over x, its bytes mapped (cs); pads stay as they are
        Piece in = std::move(v.inner[0]);
        v.cs = in.fn == VF_LOWER ? 1 : 2;
        v.inner = std::move(in.inner);
        nested = false;
        for (const Piece& p : v.inner) nested = nested || p.kind == PC_VIEW;
      }
      if (nested && env.storage) {   // (a storage filter runs without a string arena)
        *err = "function `" + f + "' over another string function's per-edge result is not supported in a storage filter";
        return NBG_E_UNSUPPORTED;
      }
      if (nested) {
        // a window / trim / pad over another one's per-edge result, or a pad drawn from one: each
        // inner view is materialised into the arena (OP_SMAT) and read back as one flat piece, so
        // views compose to any depth.  Its registers stay live (a fresh one holds the entry)
        for (auto* l : {&v.inner, &v.pad})
          for (Piece& p : *l) {
            if (p.kind != PC_VIEW) continue;
            std::vector<Piece> one;
            one.push_back(std::move(p));
            const uint64_t most = std::min<uint64_t>(bound_of(one), 1ull << 40);
            const uint64_t add = 16 + ((most + 7) & ~7ull);
            pb.sout_bytes = add > UINT64_MAX - pb.sout_bytes ? UINT64_MAX : pb.sout_bytes + add;
            const int32_t h = emit_pieces(one);
            const int r = push();
            emit(OP_SMAT, r, 0, 0, h);
            Piece d;
            d.kind = PC_DICT;
            d.reg = r;
            d.mat = true;
            d.bound = most;
            p = std::move(d);
          }
        nested = false;
      }
      if (nint >= 1) v.reg = materialize(args[1]);
      if (nint >= 2) v.reg_b = materialize(args[2]);
      v.bound = bound_of(v.inner);
      if (pads) v.bound = args[1].is_const ? std::max<uint64_t>(v.bound, (uint64_t)std::max<int64_t>(args[1].const_bits, 0))
                                           : UINT64_MAX;
      *out = derived_of({std::move(v)});   // (its registers stay live until a sink reads it)
      return NBG_OK;
    } else {
      *err = "function `" + f + "' over per-edge values is not supported on the device";
      return NBG_E_UNSUPPORTED;
    }
    top = c.reg + 1;
    if (top > max_reg) max_reg = top;
    *out = c;
    return NBG_OK;
  }

  // udf_is_in(cmp, v1, ...) (FunctionManager.cpp:440-486): every vi converted to cmp's kind
  // (toInt / toDouble / toBool / toString), then set membership (exact equality).
  int32_t is_in(const Node& e, Compiled* out) {
    Compiled cmp;
    int32_t rc = compile(*e.kids[0], &cmp);
    if (rc) return rc;
    std::vector<Compiled> args(e.kids.size() - 1);
    bool any_error = cmp.always_error;
    for (size_t i = 1; i < e.kids.size(); ++i) {
      rc = compile(*e.kids[i], &args[i - 1]);
      if (rc) return rc;
      any_error = any_error || args[i - 1].always_error;
    }
    if (any_error) { *out = make_error(); return NBG_OK; }
    const VKind K = cmp.kind;
    if (K == VK_STRING) return is_in_string(cmp, args, out);
    // numeric / bool: the comparand in a register, the accumulator above everything compiled so far
    const int x = materialize(cmp);
    const int acc = push();
    emit(OP_CONST, acc, 0, 0, 0, 0);
    for (Compiled& a : args) {
      if (a.is_const && !a.derived) {
        CVal v;
        bool ok = true;
        if (K == VK_INT) ok = cast_value(0, a.cval, &v);
        else if (K == VK_DOUBLE) ok = cast_value(2, a.cval, &v);
        else v = CVal(truthy(a.cval));
        if (!ok) { *out = make_error(); return NBG_OK; }   // folly::to throws on the set's build
        const int64_t bits = bits_of(v);
        emit(K == VK_DOUBLE ? OP_ISIN_F : OP_ISIN_I, acc, x, acc, 0, bits);
        continue;
      }
      // a value computed per edge: converted into a register, compared, OR-ed in
      int r;
      if (K == VK_BOOL) {
        r = truthy_reg(a);
      } else if (a.derived) {
        const int32_t h = emit_pieces(a.pieces);
        r = sink_reg(a.pieces);
        emit(K == VK_DOUBLE ? OP_SPARSE_F : OP_SPARSE_I, r, 0, 0, h);
      } else {
        r = a.reg;
        const bool dbl = K == VK_DOUBLE;
        switch (a.kind) {
          case VK_INT: if (dbl) emit(OP_I2F, r, r); break;
          case VK_DOUBLE: if (!dbl) emit(OP_F2I, r, r); break;
          case VK_BOOL: emit(dbl ? OP_B2F : OP_B2I, r, r); break;
          case VK_STRING: emit(dbl ? OP_S2F : OP_S2I, r, r); break;
        }
      }
      emit(K == VK_DOUBLE ? OP_EQX_F : OP_EQ_I, r, x, r);
      emit(OP_OR, acc, acc, r);
      top = acc + 1;
    }
    // the result lands in the comparand's register (the lowest live one)
    emit(OP_B2I, x, acc);
    Compiled c;
    c.kind = VK_BOOL;
    c.reg = x;
    top = x + 1;
    *out = c;
    return NBG_OK;
  }

  int32_t is_in_string(const Compiled& cmp, std::vector<Compiled>& args, Compiled* out) {
    const std::vector<Piece> pc = pieces_of(cmp);
    int acc = -1;
    for (Compiled& a : args) {
      std::vector<Piece> pa;
      if (a.kind == VK_STRING) {
        pa = pieces_of(a);
      } else if (a.is_const) {   // Expression::toString of a constant
        CVal v;
        if (!cast_value(1, a.cval, &v)) { *out = make_error(); return NBG_OK; }
        pa = {Piece{PC_CONST, -1, std::get<3>(v)}};
      } else if (a.kind == VK_INT || a.kind == VK_BOOL) {
        pa = {Piece{a.kind == VK_INT ? PC_INT : PC_BOOL, a.reg, {}}};
      } else {   // folly's double formatting: unpinned
        *out = make_error();
        return NBG_OK;
      }
      const int32_t ha = emit_pieces(pc), hb = emit_pieces(pa);
      // the comparison writes above every live piece register; the accumulator sits below it
      int r = push();
      for (auto& p : pc) r = std::max(r, p.reg + 1);
      for (auto& p : pa) r = std::max(r, p.reg + 1);
      if (r >= top) { top = r + 1; if (top > max_reg) max_reg = top; }
      emit(OP_SCMP, r, 4, 0, ha, hb);
      if (acc < 0) {
        acc = r;
      } else {
        emit(OP_OR, acc, acc, r);
      }
    }
    Compiled c;
    c.kind = VK_BOOL;
    c.reg = acc;
    *out = c;
    return NBG_OK;
  }

  // Registers of a (left) and b (right): constants are materialised lazily so that the
  // result ends up in the lower slot.
  int32_t binary(const Node& e, Compiled& a, Compiled& b, Compiled* out) {
    Compiled c;
    if (a.is_const && b.is_const) {   // e.g. EdgeType constants once validated
      CVal v;
      bool ok = e.kind == EK_ARITH ? evalArith(e.op, a.cval, b.cval, &v)
              : e.kind == EK_REL ? evalRel(e.op, a.cval, b.cval, &v) : evalLogic(e.op, a.cval, b.cval, &v);
      *out = ok ? make_const(v) : make_error();
      return NBG_OK;
    }
    if (e.kind == EK_LOGIC) {
      // both operands are always evaluated; asBool on each
      int lr = truthy_reg(a);
      int rr = truthy_reg(b);
      emit(e.op == 0 ? OP_AND : e.op == 1 ? OP_OR : OP_XORB, std::min(lr, rr), lr, rr);
      c.kind = VK_BOOL;
      c.reg = std::min(lr, rr);
      top = c.reg + 1;
      *out = c;
      return NBG_OK;
    }
    if (e.kind == EK_ARITH) {
      bool arith = !a.derived && !b.derived && (a.kind == VK_INT || a.kind == VK_DOUBLE) &&
                   (b.kind == VK_INT || b.kind == VK_DOUBLE);
      if (!arith) {
        if (e.op == 0 && a.kind == VK_STRING && b.kind == VK_STRING) {   // Expressions.cpp:858-860
          std::vector<Piece> ps = pieces_of(a), pb2 = pieces_of(b);
          ps.insert(ps.end(), pb2.begin(), pb2.end());
          *out = derived_of(std::move(ps));
          return NBG_OK;
        }
        *out = make_error();
        return NBG_OK;
      }
      bool dbl = a.kind == VK_DOUBLE || b.kind == VK_DOUBLE;
      int lr = materialize(a);
      if (dbl && a.kind == VK_INT) emit(OP_I2F, lr, lr);
      int rr = materialize(b);
      if (dbl && b.kind == VK_INT) emit(OP_I2F, rr, rr);
      static const uint8_t iops[] = {OP_ADD_I, OP_SUB_I, OP_MUL_I, OP_DIV_I, OP_MOD_I, OP_XOR_I};
      static const uint8_t fops[] = {OP_ADD_F, OP_SUB_F, OP_MUL_F, OP_DIV_F, OP_MOD_F, OP_XOR_F};
      if (e.op > 5) { *out = make_error(); return NBG_OK; }
      int d = std::min(lr, rr);
      emit(dbl ? fops[e.op] : iops[e.op], d, lr, rr);
      c.kind = (dbl && e.op != 5) ? VK_DOUBLE : VK_INT;
      c.reg = d;
      top = d + 1;
      *out = c;
      return NBG_OK;
    }
    // relational with implicit casting bool -> int -> double (Expressions.cpp:1027-1045)
    if (e.op > 5) { *out = make_error(); return NBG_OK; }
    VKind ka = a.kind, kb = b.kind;
    if (ka != kb && (ka == VK_STRING || kb == VK_STRING)) { *out = make_error(); return NBG_OK; }
    if (a.derived || b.derived) {   // string bytes compared (std::string operators)
      const std::vector<Piece> pa = pieces_of(a), pbb = pieces_of(b);
      const int32_t ha = emit_pieces(pa), hb = emit_pieces(pbb);
      c.reg = sink_reg(pa, pbb);
      emit(OP_SCMP, c.reg, e.op, 0, ha, hb);
      c.kind = VK_BOOL;
      *out = c;
      return NBG_OK;
    }
    bool dbl = (ka != kb) ? (ka == VK_DOUBLE || kb == VK_DOUBLE) : ka == VK_DOUBLE;
    int lr = materialize(a);
    if (ka != kb) {
      if (dbl) { if (ka == VK_INT) emit(OP_I2F, lr, lr); else if (ka == VK_BOOL) emit(OP_B2F, lr, lr); }
      else if (ka == VK_BOOL) emit(OP_B2I, lr, lr);
    }
    int rr = materialize(b);
    if (ka != kb) {
      if (dbl) { if (kb == VK_INT) emit(OP_I2F, rr, rr); else if (kb == VK_BOOL) emit(OP_B2F, rr, rr); }
      else if (kb == VK_BOOL) emit(OP_B2I, rr, rr);
    }
    static const uint8_t iops[] = {OP_LT_I, OP_LE_I, OP_GT_I, OP_GE_I, OP_EQ_I, OP_NE_I};
    static const uint8_t fops[] = {OP_LT_F, OP_LE_F, OP_GT_F, OP_GE_F, OP_EQ_F, OP_NE_F};
    int d = std::min(lr, rr);
    emit(dbl ? fops[e.op] : iops[e.op], d, lr, rr);
    c.kind = VK_BOOL;
    c.reg = d;
    top = d + 1;
    *out = c;
    return NBG_OK;
  }
};

}  // namespace

int32_t compile_expr(const Node& e, const CompileEnv& env, ProgramBuilder& pb, Compiled* out, std::string* err,
                     bool yield_value) {
  Ctx c{env, pb, err};
  c.top = pb.next_reg;
  c.max_reg = pb.next_reg;
  int32_t rc = c.compile(e, out);
  if (rc) return rc;
  if (out->derived) {   // the sink of a derived string: a result value, or a WHERE's asBool
    Compiled v;
    v.kind = yield_value ? VK_STRING : VK_BOOL;
    v.reg = yield_value ? c.value_reg(*out) : c.empty_reg(*out);
    *out = v;
  }
  if ((int)(pb.code.size() + pb.data.size()) > MAX_PROGRAM) {
    *err = "program too long";
    return NBG_E_UNSUPPORTED;
  }
  if (!out->is_const && out->reg >= 0) pb.next_reg = out->reg + 1;
  if (c.max_reg > MAX_REGS) {
    *err = "expression too deep for the device register file";
    return NBG_E_UNSUPPORTED;
  }
  pb.max_reg = std::max(pb.max_reg, c.max_reg);
  return NBG_OK;
}

}  // namespace nbg

namespace nbg {

// ============================================================================= result column types
namespace {
int32_t natural_type(VKind k) {
  switch (k) {
    case VK_DOUBLE: return NBG_T_DOUBLE;
    case VK_BOOL: return NBG_T_BOOL;
    case VK_STRING: return NBG_T_STRING;
    default: return NBG_T_INT;
  }
}

const SchemaSet* by_name(const std::map<int32_t, SchemaSet>* m, const std::string& name) {
  if (!m) return nullptr;
  for (auto& kv : *m)
    if (kv.second.name == name) return &kv.second;
  return nullptr;
}

int32_t prop_type(const SchemaSet* ss, const std::string& prop) {   // getFieldType: 0 if absent
  const Schema* sc = ss ? ss->latest() : nullptr;
  const int c = sc ? sc->find(prop) : -1;
  return c < 0 ? 0 : sc->cols[c].type;
}

// post-order, left operand first: *t = the type set by the last getter evaluated
void last_getter(const Node& e, const ColTypeEnv& env, int32_t* t) {
  for (auto& k : e.kids)
    if (k) last_getter(*k, env, t);
  switch (e.kind) {
    case EK_ALIAS: case EK_DST: case EK_SRCID: case EK_RANK: {
      // getAliasProp: an unknown edge fails before the type is saved; else the type comes from the
      // ROW's schema (iter->getSchema()->getFieldType(prop)), whatever edge the alias names
      if (!by_name(env.edges, e.alias)) return;
      *t = 0;
      if (env.row_types) {
        auto it = env.row_types->find(e.prop);
        if (it != env.row_types->end()) *t = it->second;
      }
      return;
    }
    case EK_SRCPROP:   // getSrcTagProp: saved when the source has the tag (the fixed row context)
      if (const SchemaSet* ts = by_name(env.tags, e.alias)) *t = prop_type(ts, e.prop);
      return;
    case EK_DSTPROP:   // VertexHolder::getType: the tag schema's type of the prop
      if (const SchemaSet* ts = by_name(env.tags, e.alias)) *t = prop_type(ts, e.prop);
      return;
    case EK_INPUT: case EK_VAR: {   // getPropTypeFromInterim: the input column's type
      if (!env.input_names || !env.input_kinds) return;
      for (size_t c = 0; c < env.input_names->size(); ++c)
        if ((*env.input_names)[c] == e.prop) { *t = natural_type((*env.input_kinds)[c]); return; }
      *t = 0;
      return;
    }
    default: return;
  }
}
}  // namespace

int32_t yield_column_type(const Node& e, const ColTypeEnv& env) {
  if (e.kind == EK_CAST) {   // SchemaHelper::columnTypeToSupportedType of the cast's ColumnType
    static const int32_t m[6] = {NBG_T_INT, NBG_T_STRING, NBG_T_DOUBLE, NBG_T_INT, NBG_T_BOOL, NBG_T_TIMESTAMP};
    return e.op < 6 ? m[e.op] : 0;
  }
  int32_t t = 0;
  last_getter(e, env, &t);
  return t;
}

}  // namespace nbg
