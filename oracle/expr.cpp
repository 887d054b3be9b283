// Test infrastructure (oracle) — Expression wire decoder + tree-walking evaluator,
// restated from src/common/filter/Expressions.{h,cpp}.
#include <cmath>
#include <functional>
#include <strings.h>
#include <cctype>
#include <ctime>
#include "orc.h"

namespace orc {

namespace {

struct Dec {
  const uint8_t* p;
  const uint8_t* end;
  std::string err;
  bool need(size_t n) {
    if (p + n > end) { if (err.empty()) err = "Not enough space left"; return false; }
    return true;
  }
  bool str16(std::string& out) {      // uint16 length + bytes (e.g. Expressions.cpp:150-171)
    if (!need(2)) return false;
    uint16_t n; memcpy(&n, p, 2); p += 2;
    if (!need(n)) return false;
    out.assign(reinterpret_cast<const char*>(p), n); p += n;
    return true;
  }
  std::unique_ptr<Expr> expr();
};

// Expression::makeExpr + per-kind decode (Expressions.cpp:50-89, 150-1162).
std::unique_ptr<Expr> Dec::expr() {
  if (!need(1)) return nullptr;
  uint8_t kind = *p++;
  auto e = std::make_unique<Expr>();
  e->kind = static_cast<Kind>(kind);
  switch (kind) {
    case kPrimary: {   // PrimaryExpression::decode (:539-570)
      if (!need(1)) return nullptr;
      uint8_t which = *p++;
      switch (which) {
        case 0: { if (!need(8)) return nullptr; int64_t v; memcpy(&v, p, 8); p += 8; e->prim = v; break; }
        case 1: { if (!need(8)) return nullptr; double v; memcpy(&v, p, 8); p += 8; e->prim = v; break; }
        case 2: { if (!need(1)) return nullptr; e->prim = (*p++ != 0); break; }
        case 3: { std::string s; if (!str16(s)) return nullptr; e->prim = s; break; }
        default: err = "Unknown variant type"; return nullptr;
      }
      return e;
    }
    case kUnary: {     // UnaryExpression::decode (:730-737)
      if (!need(2)) return nullptr;
      e->op = *p++;
      e->a = expr();
      return e->a ? std::move(e) : nullptr;
    }
    case kTypeCasting: {
      // TypeCastingExpression::encode is empty in the reference (:801-802) and its decode
      // throws (Expressions.h:830-832).  nebula_amd wire extension (specified in include/nbg.h,
      // "Expression wire"; the graphd-side encoder is in INTEGRATION.md §2): kind, uint8
      // ColumnType, operand.  Bytes from an unpatched encoder lack the whole cast subtree and
      // fail below for want of bytes, as the reference's decode does.
      if (!need(2)) return nullptr;
      e->castType = *p++;
      e->a = expr();
      return e->a ? std::move(e) : nullptr;
    }
    case kArithmetic: case kRelational: case kLogical: {   // (:932-943, :1068-1079, :1151-1162)
      if (!need(2)) return nullptr;
      e->op = *p++;
      e->a = expr();
      if (!e->a) return nullptr;
      e->b = expr();
      return e->b ? std::move(e) : nullptr;
    }
    case kFunctionCall: {   // (:637-657)
      if (!str16(e->alias)) return nullptr;   // name
      if (!need(2)) return nullptr;
      uint16_t cnt; memcpy(&cnt, p, 2); p += 2;
      for (uint16_t i = 0; i < cnt; ++i) {
        auto a = expr();
        if (!a) return nullptr;
        e->args.push_back(std::move(a));
      }
      return e;
    }
    case kSourceProp: case kAliasProp: case kVariableProp: case kDestProp: {
      if (!str16(e->alias)) return nullptr;
      if (!str16(e->prop)) return nullptr;
      return e;
    }
    case kInputProp: {
      if (!str16(e->prop)) return nullptr;
      return e;
    }
    case kEdgeRank: case kEdgeDstId: case kEdgeSrcId: case kEdgeType: {
      if (!str16(e->alias)) return nullptr;
      // the reference decoder leaves prop_ unset; the constructor sets it (Expressions.h:499-587)
      e->prop = kind == kEdgeRank ? "_rank" : kind == kEdgeDstId ? "_dst"
              : kind == kEdgeSrcId ? "_src" : "_type";
      return e;
    }
    default:
      err = "Illegal expression kind";
      return nullptr;
  }
}

bool isInt(const Value& v) { return v.index() == 0; }
bool isDouble(const Value& v) { return v.index() == 1; }
bool isStr(const Value& v) { return v.index() == 3; }
bool isArith(const Value& v) { return v.index() <= 1; }
int64_t asInt(const Value& v) { return std::get<0>(v); }
double asDouble(const Value& v) { return v.index() == 0 ? static_cast<double>(std::get<0>(v)) : std::get<1>(v); }

// Expression::toInt/toDouble (Expressions.h:290-321)
int64_t toInt(const Value& v, bool& ok) {
  ok = true;
  switch (v.index()) {
    case 0: return std::get<0>(v);
    case 1: return static_cast<int64_t>(std::get<1>(v));
    case 2: return std::get<2>(v) ? 1 : 0;
    default: {
      const std::string& s = std::get<3>(v);
      char* endp = nullptr;
      errno = 0;
      long long r = strtoll(s.c_str(), &endp, 10);
      if (s.empty() || *endp != '\0' || errno) { ok = false; return 0; }
      return r;
    }
  }
}
double toDouble(const Value& v, bool& ok) {
  ok = true;
  switch (v.index()) {
    case 0: return static_cast<double>(std::get<0>(v));
    case 1: return std::get<1>(v);
    case 2: return std::get<2>(v) ? 1.0 : 0.0;
    default: {
      const std::string& s = std::get<3>(v);
      char* endp = nullptr;
      double r = strtod(s.c_str(), &endp);
      if (s.empty() || *endp != '\0') { ok = false; return 0; }
      return r;
    }
  }
}

bool almostEqual(double l, double r) { return std::abs(l - r) < 1e-8; }   // Expressions.h:268-271

// boost::variant operator< after implicit casting (same alternative on both sides)
int cmpSame(const Value& l, const Value& r) {
  switch (l.index()) {
    case 0: return asInt(l) < asInt(r) ? -1 : asInt(l) > asInt(r) ? 1 : 0;
    case 1: { double a = std::get<1>(l), b = std::get<1>(r); return a < b ? -1 : a > b ? 1 : (a == b ? 0 : 2); }
    case 2: return (int)std::get<2>(l) - (int)std::get<2>(r);
    default: { int c = std::get<3>(l).compare(std::get<3>(r)); return c < 0 ? -1 : c > 0 ? 1 : 0; }
  }
}

// Expression::toString (Expressions.h:274-288); folly's double formatting is not restated
bool toStr(const Value& v, std::string* out) {
  switch (v.index()) {
    case 0: *out = std::to_string(std::get<0>(v)); return true;
    case 2: *out = std::get<2>(v) ? "true" : "false"; return true;
    case 3: *out = std::get<3>(v); return true;
    default: return false;
  }
}

}  // namespace

// FunctionManager's bodies (src/common/filter/FunctionManager.cpp:20-487).  Arguments are read
// with Expression::asDouble / asInt / asString (Expressions.h:217-246), i.e. boost::get: an
// argument of another kind throws bad_get, an evaluation error here.  lpad / rpad with a negative
// size, or padding with an empty pad, never return in the reference (their loop does not end):
// an evaluation error here.  rand32 / rand64 / now are random / the clock: only their ranges are
// restated.  udf_is_in (:440-486): std::unordered_set membership after converting every
// candidate to the comparand's alternative.
namespace {
uint64_t splitmix(uint64_t x) {
  x += 0x9e3779b97f4a7c15ull;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}
uint64_t rand_bits() {
  static uint64_t state = (uint64_t)time(nullptr) * 0x9e3779b97f4a7c15ull;
  return splitmix(state += 0x9e3779b97f4a7c15ull);
}
}  // namespace

OptValue callFunction(const std::string& f, const std::vector<Value>& av) {
  static const char* math1[] = {"abs", "floor", "ceil", "round", "sqrt", "cbrt", "exp", "exp2", "log",
                                "log2", "log10", "sin", "asin", "cos", "acos", "tan", "atan"};
  for (int i = 0; i < 17; ++i) {
    if (f != math1[i]) continue;
    if (av.size() != 1) return Status::Err("Arity not match");
    if (!isArith(av[0])) return Status::Err("asDouble of a non-number");   // boost::bad_get
    const double x = asDouble(av[0]);
    double (*const fn[17])(double) = {std::fabs, std::floor, std::ceil, std::round, std::sqrt, std::cbrt,
                                      std::exp,  std::exp2,  std::log,  std::log2,  std::log10, std::sin,
                                      std::asin, std::cos,   std::acos, std::tan,   std::atan};
    return Value(fn[i](x));
  }
  if (f == "hypot" || f == "pow") {
    if (av.size() != 2) return Status::Err("Arity not match");
    if (!isArith(av[0]) || !isArith(av[1])) return Status::Err("asDouble of a non-number");
    const double x = asDouble(av[0]), y = asDouble(av[1]);
    return Value(f == "hypot" ? std::hypot(x, y) : std::pow(x, y));
  }
  if (f == "rand32" || f == "rand64") {   // folly::Random::rand32 / rand64 (max), (min, max)
    if (av.size() > 2) return Status::Err("Arity not match");
    for (auto& v : av)
      if (!isInt(v)) return Status::Err("asInt of a non-int");
    const uint64_t r = rand_bits();
    if (f == "rand32") {
      if (av.empty()) return Value((int64_t)(int32_t)(uint32_t)r);
      const uint32_t lo = av.size() == 2 ? (uint32_t)asInt(av[0]) : 0u, hi = (uint32_t)asInt(av.back());
      if (lo == hi) return Value((int64_t)0);
      const uint32_t got = lo + (uint32_t)(r % (uint32_t)(hi - lo));
      return Value(av.size() == 1 ? (int64_t)(int32_t)got : (int64_t)got);
    }
    if (av.empty()) return Value((int64_t)r);
    const uint64_t lo = av.size() == 2 ? (uint64_t)asInt(av[0]) : 0ull, hi = (uint64_t)asInt(av.back());
    if (lo == hi) return Value((int64_t)0);
    return Value((int64_t)(lo + r % (hi - lo)));
  }
  if (f == "now") {
    if (!av.empty()) return Status::Err("Arity not match");
    return Value((int64_t)time(nullptr));   // WallClock::fastNowInSec
  }
  if (f == "hash") {   // std::hash of the variant's alternative (libstdc++: identity for integers)
    if (av.size() != 1) return Status::Err("Arity not match");
    switch (av[0].index()) {
      case 0: return Value((int64_t)std::hash<int64_t>{}(std::get<0>(av[0])));
      case 1: return Value((int64_t)std::hash<double>{}(std::get<1>(av[0])));
      case 2: return Value((int64_t)std::hash<bool>{}(std::get<2>(av[0])));
      default: return Value((int64_t)std::hash<std::string>{}(std::get<3>(av[0])));
    }
  }
  struct Sig {
    const char* name;
    size_t n;
    const char* kinds;   // s: asString, i: asInt
  };
  static const Sig sigs[] = {{"strcasecmp", 2, "ss"}, {"lower", 1, "s"},  {"upper", 1, "s"},
                             {"length", 1, "s"},      {"trim", 1, "s"},   {"ltrim", 1, "s"},
                             {"rtrim", 1, "s"},       {"left", 2, "si"},  {"right", 2, "si"},
                             {"lpad", 3, "sis"},      {"rpad", 3, "sis"}, {"substr", 3, "sii"}};
  for (const Sig& g : sigs) {
    if (f != g.name) continue;
    if (av.size() != g.n) return Status::Err("Arity not match");
    for (size_t k = 0; k < g.n; ++k)
      if (g.kinds[k] == 's' ? !isStr(av[k]) : !isInt(av[k])) return Status::Err("bad_get");
    std::string v = std::get<3>(av[0]);
    if (f == "strcasecmp") return Value((int64_t)::strcasecmp(v.c_str(), std::get<3>(av[1]).c_str()));
    if (f == "length") return Value((int64_t)v.length());
    if (f == "lower" || f == "upper") {
      for (char& c : v) c = (char)(f == "lower" ? std::tolower((unsigned char)c) : std::toupper((unsigned char)c));
      return Value(v);
    }
    if (f == "trim" || f == "ltrim" || f == "rtrim") {
      if (f != "rtrim") v.erase(0, v.find_first_not_of(" "));
      if (f != "ltrim") v.erase(v.find_last_not_of(" ") + 1);
      return Value(v);
    }
    const int64_t n = asInt(av[1]);
    if (f == "left") return Value(n <= 0 ? std::string() : v.substr(0, (size_t)n));
    if (f == "right") {
      if (n <= 0) return Value(std::string());
      const size_t k = (uint64_t)n > v.size() ? v.size() : (size_t)n;
      return Value(v.substr(v.size() - k));
    }
    if (f == "lpad" || f == "rpad") {
      const std::string& extra = std::get<3>(av[2]);
      const size_t size = (size_t)n;
      if (size < v.size()) return Value(v.substr(0, size));
      if (n < 0 || (size > v.size() && extra.empty())) return Status::Err("padding never ends");
      size_t need = size - v.size();
      std::string pad;
      while (need > extra.size()) {
        pad += extra;
        need -= extra.size();
      }
      pad += extra.substr(0, need);
      return Value(f == "lpad" ? pad + v : v + pad);
    }
    // substr
    const int64_t start = n, len = asInt(av[2]);
    const uint64_t ast = start < 0 ? 0ull - (uint64_t)start : (uint64_t)start;
    if (ast > v.size() || len <= 0 || start == 0) return Value(std::string());
    return Value(start > 0 ? v.substr((size_t)start - 1, (size_t)len) : v.substr(v.size() - ast, (size_t)len));
  }
  if (f != "udf_is_in") return Status::Err("Function not defined");
  if (av.size() < 2) return Status::Err("Arity not match");
  const Value& cmp = av[0];
  bool found = false;
  for (size_t i = 1; i < av.size(); ++i) {
    bool ok = true;
    switch (cmp.index()) {
      case 0: { int64_t x = toInt(av[i], ok); found = found || (ok && x == std::get<0>(cmp)); break; }
      case 1: { double x = toDouble(av[i], ok); found = found || (ok && x == std::get<1>(cmp)); break; }
      case 2: found = found || asBool(av[i]) == std::get<2>(cmp); break;
      default: {
        std::string x;
        ok = toStr(av[i], &x);
        found = found || (ok && x == std::get<3>(cmp));
      }
    }
    if (!ok) return Status::Err("conversion failed");   // folly::to throws
  }
  return Value(found);
}

bool asBool(const Value& v) {   // Expressions.h:228-241 (string -> empty())
  switch (v.index()) {
    case 0: return std::get<0>(v) != 0;
    case 1: return std::get<1>(v) != 0.0;
    case 2: return std::get<2>(v);
    default: return std::get<3>(v).empty();
  }
}

std::unique_ptr<Expr> decodeExpr(const uint8_t* buf, size_t len, std::string* err) {
  Dec d{buf, buf + len, {}};
  auto e = d.expr();
  if (e && d.p != d.end) { d.err = "Buffer not consumed up"; e.reset(); }
  if (!e && err) *err = d.err.empty() ? "decode failed" : d.err;
  return e;
}

OptValue Expr::eval(Getters& g) const {
  switch (kind) {
    case kPrimary: return prim;
    case kAliasProp: case kEdgeRank: case kEdgeDstId: case kEdgeSrcId:
      return g.aliasProp(alias, prop);                          // Expressions.cpp:133-135,338-396
    case kEdgeType: return Value(alias);                        // Expressions.cpp:310-312
    case kSourceProp: return g.srcTagProp(alias, prop);         // :429-431
    case kDestProp: return g.dstTagProp(alias, prop);           // :217-219
    case kInputProp: case kVariableProp: return g.inputProp(prop);   // GoExecutor.cpp:932-945
    case kFunctionCall: {   // FunctionCallExpression::eval (:589-603): arguments first, then the body
      std::vector<Value> av;
      for (auto& x : args) {
        auto v = x->eval(g);
        if (!v.ok()) return v;
        av.push_back(v.v);
      }
      return callFunction(alias, av);
    }
    case kUnary: {        // UnaryExpression::eval (:698-716)
      auto v = a->eval(g);
      if (v.ok()) {
        if (op == 0) return v;
        if (op == 1) {
          if (isInt(v.v)) return Value(static_cast<int64_t>(0ULL - static_cast<uint64_t>(asInt(v.v))));
          if (isDouble(v.v)) return Value(-std::get<1>(v.v));
        } else {
          return Value(!asBool(v.v));
        }
      }
      return Status::Err("attempt to perform unary arithmetic");
    }
    case kTypeCasting: {  // TypeCastingExpression::eval (:773-793); ColumnType INT,STRING,DOUBLE,BIGINT,BOOL,TIMESTAMP
      auto v = a->eval(g);
      if (!v.ok()) return v;
      bool ok = true;
      switch (castType) {
        case 0: case 5: { int64_t r = toInt(v.v, ok); if (!ok) return Status::Err("bad cast"); return Value(r); }
        case 1: {
          switch (v.v.index()) {
            case 0: return Value(std::to_string(asInt(v.v)));
            case 2: return Value(std::string(std::get<2>(v.v) ? "true" : "false"));
            case 3: return v;
            default: return Status::Err("double->string cast is unpinned");
          }
        }
        case 2: { double r = toDouble(v.v, ok); if (!ok) return Status::Err("bad cast"); return Value(r); }
        case 4: return Value(asBool(v.v));
        default: return Status::Err("Type bigint not supported yet");
      }
    }
    case kArithmetic: {   // ArithmeticExpression::eval (:835-909)
      auto lv = a->eval(g);
      auto rv = b->eval(g);
      if (!lv.ok()) return lv;
      if (!rv.ok()) return rv;
      const Value& l = lv.v; const Value& r = rv.v;
      if (isArith(l) && isArith(r)) {
        bool dbl = isDouble(l) || isDouble(r);
        uint64_t ul = dbl ? 0 : static_cast<uint64_t>(asInt(l));
        uint64_t ur = dbl ? 0 : static_cast<uint64_t>(asInt(r));
        switch (op) {
          case 0: return dbl ? Value(asDouble(l) + asDouble(r)) : Value(static_cast<int64_t>(ul + ur));
          case 1: return dbl ? Value(asDouble(l) - asDouble(r)) : Value(static_cast<int64_t>(ul - ur));
          case 2: return dbl ? Value(asDouble(l) * asDouble(r)) : Value(static_cast<int64_t>(ul * ur));
          case 3: case 4: {
            if (dbl) return op == 3 ? Value(asDouble(l) / asDouble(r)) : Value(std::fmod(asDouble(l), asDouble(r)));
            // integer /0 and INT64_MIN/-1 trap in the reference; defined here as an eval error
            if (asInt(r) == 0 || (asInt(l) == INT64_MIN && asInt(r) == -1))
              return Status::Err("division by zero");
            return op == 3 ? Value(asInt(l) / asInt(r)) : Value(asInt(l) % asInt(r));
          }
          case 5: {
            if (dbl) return Value(static_cast<int64_t>(std::round(asDouble(l))) ^
                                  static_cast<int64_t>(std::round(asDouble(r))));
            return Value(asInt(l) ^ asInt(r));
          }
          default: break;
        }
      } else if (op == 0 && isStr(l) && isStr(r)) {
        return Value(std::get<3>(l) + std::get<3>(r));
      }
      return Status::Err("attempt to perform arithmetic on incompatible types");
    }
    case kRelational: {   // RelationalExpression::eval (:976-1045)
      auto lv = a->eval(g);
      auto rv = b->eval(g);
      if (!lv.ok()) return lv;
      if (!rv.ok()) return rv;
      Value l = lv.v, r = rv.v;
      if (l.index() != r.index()) {
        bool ok = true;
        if (isStr(l) || isStr(r)) return Status::Err("A string type can not be compared with a non-string type.");
        if (isDouble(l) || isDouble(r)) { l = toDouble(l, ok); r = toDouble(r, ok); }
        else if (isInt(l) || isInt(r)) { l = toInt(l, ok); r = toInt(r, ok); }
      }
      if ((op == 4 || op == 5) && isArith(l) && isArith(r) && (isDouble(l) || isDouble(r))) {
        bool eq = almostEqual(asDouble(l), asDouble(r));
        return Value(op == 4 ? eq : !eq);
      }
      // boost::variant defines only < and ==; >, <=, >= derive from < (so a NaN operand
      // makes <= and >= true), != is !(==).
      bool lt = cmpSame(l, r) == -1, gt = cmpSame(r, l) == -1;
      bool eq = cmpSame(l, r) == 0;
      switch (op) {
        case 0: return Value(lt);
        case 1: return Value(!gt);
        case 2: return Value(gt);
        case 3: return Value(!lt);
        case 4: return Value(eq);
        case 5: return Value(!eq);
        default: return Status::Err("Wrong operator");
      }
    }
    case kLogical: {      // LogicalExpression::eval (:1103-1131): both sides always evaluated
      auto lv = a->eval(g);
      auto rv = b->eval(g);
      if (!lv.ok()) return lv;
      if (!rv.ok()) return rv;
      bool l = asBool(lv.v), r = asBool(rv.v);
      if (op == 0) return Value(l && r);
      if (op == 1) return Value(l || r);
      return Value(l != r);
    }
    default:
      return Status::Err("unsupported expression kind");
  }
}

}  // namespace orc
