// json.hpp — minimal JSON value, reader and writer for the optflow CLI.
//
// Mirrors how the reference uses jsoncpp (/root/reference/src/optflow.cpp):
//   * Json::Reader::parse with comments allowed (docs/example.json is commented);
//   * objects keep their members in sorted key order (jsoncpp stores them in a
//     std::map, so getMemberNames() — the ROI loop at optflow.cpp:339 — is sorted);
//   * v.get(key, default) and asInt/asFloat/asDouble/asBool/asString conversions
//     (numbers convert freely; asInt truncates a double).
// Unlike the reference (which ignores parse's return value, optflow.cpp:51,56) a
// malformed file is reported with a line/column and the CLI exits non-zero.
#pragma once

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace ofjson {

class Value {
 public:
  enum Type { Null, Bool, Int, Real, String, Array, Object };

  Value() = default;
  Value(bool b) : t_(Bool), b_(b) {}
  Value(int v) : t_(Int), i_(v) {}
  Value(int64_t v) : t_(Int), i_(v) {}
  Value(double v) : t_(Real), d_(v) {}
  Value(const char *s) : t_(String), s_(s) {}
  Value(std::string s) : t_(String), s_(std::move(s)) {}

  Type type() const { return t_; }
  bool isNull() const { return t_ == Null; }
  bool isObject() const { return t_ == Object; }
  bool isArray() const { return t_ == Array; }
  bool isString() const { return t_ == String; }
  bool isNumeric() const { return t_ == Int || t_ == Real || t_ == Bool; }

  bool isMember(const std::string &k) const { return t_ == Object && o_.count(k) != 0; }
  const Value *find(const std::string &k) const {
    if (t_ != Object) return nullptr;
    auto it = o_.find(k);
    return it == o_.end() ? nullptr : &it->second;
  }
  // jsoncpp get(key, default): member if present, else the default.
  Value get(const std::string &k, const Value &dflt) const {
    const Value *v = find(k);
    return v ? *v : dflt;
  }
  Value &operator[](const std::string &k) {
    if (t_ == Null) t_ = Object;
    if (t_ != Object) throw std::runtime_error("json: not an object");
    return o_[k];
  }
  const Value &operator[](const std::string &k) const {
    static const Value null;
    const Value *v = find(k);
    return v ? *v : null;
  }
  Value &operator[](int i) { return (*this)[(size_t)i]; }
  const Value &operator[](int i) const { return (*this)[(size_t)i]; }
  Value &operator[](const char *k) { return (*this)[std::string(k)]; }
  const Value &operator[](const char *k) const { return (*this)[std::string(k)]; }
  Value &operator[](size_t i) {
    if (t_ == Null) t_ = Array;
    if (t_ != Array) throw std::runtime_error("json: not an array");
    if (i >= a_.size()) a_.resize(i + 1);
    return a_[i];
  }
  const Value &operator[](size_t i) const {
    static const Value null;
    return (t_ == Array && i < a_.size()) ? a_[i] : null;
  }
  void append(const Value &v) {
    if (t_ == Null) t_ = Array;
    if (t_ != Array) throw std::runtime_error("json: not an array");
    a_.push_back(v);
  }
  size_t size() const { return t_ == Array ? a_.size() : (t_ == Object ? o_.size() : 0); }
  std::vector<std::string> memberNames() const {
    std::vector<std::string> r;
    if (t_ == Object)
      for (auto &kv : o_) r.push_back(kv.first);
    return r;
  }
  void clear() {
    a_.clear();
    o_.clear();
  }

  bool asBool() const {
    switch (t_) {
      case Bool: return b_;
      case Int: return i_ != 0;
      case Real: return d_ != 0.0;
      case Null: return false;
      case String: return !s_.empty() && s_ != "false" && s_ != "0";
      default: throw std::runtime_error("json: value not convertible to bool");
    }
  }
  int64_t asInt64() const {
    switch (t_) {
      case Bool: return b_ ? 1 : 0;
      case Int: return i_;
      case Real: return (int64_t)d_;  // jsoncpp truncates
      case Null: return 0;
      case String: return std::stoll(s_);
      default: throw std::runtime_error("json: value not convertible to int");
    }
  }
  int asInt() const { return (int)asInt64(); }
  double asDouble() const {
    switch (t_) {
      case Bool: return b_ ? 1.0 : 0.0;
      case Int: return (double)i_;
      case Real: return d_;
      case Null: return 0.0;
      case String: return std::stod(s_);
      default: throw std::runtime_error("json: value not convertible to double");
    }
  }
  float asFloat() const { return (float)asDouble(); }
  std::string asString() const {
    switch (t_) {
      case String: return s_;
      case Null: return "";
      case Bool: return b_ ? "true" : "false";
      case Int: return std::to_string(i_);
      case Real: {
        char b[64];
        snprintf(b, sizeof b, "%.17g", d_);
        return b;
      }
      default: throw std::runtime_error("json: value not convertible to string");
    }
  }

  std::string dump(int indent = -1) const {
    std::string out;
    write(out, indent, 0);
    return out;
  }

 private:
  static void esc(std::string &out, const std::string &s) {
    out += '"';
    for (unsigned char c : s) {
      switch (c) {
        case '"': out += "\\\""; break;
        case '\\': out += "\\\\"; break;
        case '\n': out += "\\n"; break;
        case '\r': out += "\\r"; break;
        case '\t': out += "\\t"; break;
        default:
          if (c < 0x20) {
            char b[8];
            snprintf(b, sizeof b, "\\u%04x", c);
            out += b;
          } else {
            out += (char)c;
          }
      }
    }
    out += '"';
  }
  void write(std::string &out, int indent, int depth) const {
    auto nl = [&](int d) {
      if (indent >= 0) {
        out += '\n';
        out.append((size_t)(indent * d), ' ');
      }
    };
    switch (t_) {
      case Null: out += "null"; break;
      case Bool: out += b_ ? "true" : "false"; break;
      case Int: out += std::to_string(i_); break;
      case Real: {
        if (std::isfinite(d_)) {
          char b[64];
          snprintf(b, sizeof b, "%.17g", d_);
          std::string t(b);
          if (t.find_first_of(".eE") == std::string::npos) t += ".0";
          out += t;
        } else {
          out += "null";
        }
        break;
      }
      case String: esc(out, s_); break;
      case Array: {
        out += '[';
        for (size_t i = 0; i < a_.size(); ++i) {
          if (i) out += ',';
          nl(depth + 1);
          a_[i].write(out, indent, depth + 1);
        }
        if (!a_.empty()) nl(depth);
        out += ']';
        break;
      }
      case Object: {
        out += '{';
        bool first = true;
        for (auto &kv : o_) {
          if (!first) out += ',';
          first = false;
          nl(depth + 1);
          esc(out, kv.first);
          out += indent >= 0 ? ": " : ":";
          kv.second.write(out, indent, depth + 1);
        }
        if (!o_.empty()) nl(depth);
        out += '}';
        break;
      }
    }
  }

  Type t_ = Null;
  bool b_ = false;
  int64_t i_ = 0;
  double d_ = 0.0;
  std::string s_;
  std::vector<Value> a_;
  std::map<std::string, Value> o_;
  friend class Parser;
};

// Recursive-descent reader: strict JSON plus /* */ and // comments (jsoncpp's
// default Features::all()).
class Parser {
 public:
  explicit Parser(const std::string &text) : s_(text) {}

  Value parse() {
    Value v = value();
    ws();
    if (p_ != s_.size()) fail("trailing characters after the JSON value");
    return v;
  }

 private:
  [[noreturn]] void fail(const std::string &msg) const {
    size_t line = 1, col = 1;
    for (size_t i = 0; i < p_ && i < s_.size(); ++i) {
      if (s_[i] == '\n') {
        ++line;
        col = 1;
      } else {
        ++col;
      }
    }
    throw std::runtime_error("JSON parse error at line " + std::to_string(line) + ", column " +
                             std::to_string(col) + ": " + msg);
  }
  void ws() {
    for (;;) {
      while (p_ < s_.size() && (s_[p_] == ' ' || s_[p_] == '\t' || s_[p_] == '\n' || s_[p_] == '\r'))
        ++p_;
      if (p_ + 1 < s_.size() && s_[p_] == '/' && s_[p_ + 1] == '*') {
        const size_t e = s_.find("*/", p_ + 2);
        if (e == std::string::npos) fail("unterminated /* comment");
        p_ = e + 2;
        continue;
      }
      if (p_ + 1 < s_.size() && s_[p_] == '/' && s_[p_ + 1] == '/') {
        while (p_ < s_.size() && s_[p_] != '\n') ++p_;
        continue;
      }
      break;
    }
  }
  char peek() {
    ws();
    return p_ < s_.size() ? s_[p_] : '\0';
  }
  void expect(char c) {
    if (peek() != c) fail(std::string("expected '") + c + "'");
    ++p_;
  }
  // nesting bound: a config nested deeper than this is an error, not a stack overflow
  static constexpr int kMaxDepth = 256;
  struct Nest {
    Parser &p;
    explicit Nest(Parser &pp) : p(pp) {
      if (++p.depth_ > kMaxDepth) p.fail("nesting deeper than 256 levels");
    }
    ~Nest() { --p.depth_; }
  };
  Value value() {
    const char c = peek();
    if (c == '{') {
      Nest n(*this);
      return object();
    }
    if (c == '[') {
      Nest n(*this);
      return array();
    }
    if (c == '"') return Value(string());
    if (c == 't' && s_.compare(p_, 4, "true") == 0) { p_ += 4; return Value(true); }
    if (c == 'f' && s_.compare(p_, 5, "false") == 0) { p_ += 5; return Value(false); }
    if (c == 'n' && s_.compare(p_, 4, "null") == 0) { p_ += 4; return Value(); }
    if (c == '-' || (c >= '0' && c <= '9')) return number();
    fail("unexpected character");
  }
  Value object() {
    Value v;
    v.t_ = Value::Object;
    expect('{');
    if (peek() == '}') {
      ++p_;
      return v;
    }
    for (;;) {
      if (peek() != '"') fail("expected a string key");
      std::string k = string();
      expect(':');
      v.o_[k] = value();
      const char c = peek();
      if (c == ',') {
        ++p_;
        if (peek() == '}') fail("trailing comma in object");
        continue;
      }
      if (c == '}') {
        ++p_;
        return v;
      }
      fail("expected ',' or '}' (missing comma?)");
    }
  }
  Value array() {
    Value v;
    v.t_ = Value::Array;
    expect('[');
    if (peek() == ']') {
      ++p_;
      return v;
    }
    for (;;) {
      v.a_.push_back(value());
      const char c = peek();
      if (c == ',') {
        ++p_;
        continue;
      }
      if (c == ']') {
        ++p_;
        return v;
      }
      fail("expected ',' or ']'");
    }
  }
  static void utf8(std::string &o, unsigned cp) {
    if (cp < 0x80) {
      o += (char)cp;
    } else if (cp < 0x800) {
      o += (char)(0xC0 | (cp >> 6));
      o += (char)(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
      o += (char)(0xE0 | (cp >> 12));
      o += (char)(0x80 | ((cp >> 6) & 0x3F));
      o += (char)(0x80 | (cp & 0x3F));
    } else {
      o += (char)(0xF0 | (cp >> 18));
      o += (char)(0x80 | ((cp >> 12) & 0x3F));
      o += (char)(0x80 | ((cp >> 6) & 0x3F));
      o += (char)(0x80 | (cp & 0x3F));
    }
  }
  unsigned hex4(size_t at) const {
    if (at + 4 > s_.size()) fail("bad \\u escape");
    unsigned v = 0;
    for (size_t i = at; i < at + 4; ++i) {
      const char h = s_[i];
      const int d = h >= '0' && h <= '9' ? h - '0' : h >= 'a' && h <= 'f' ? h - 'a' + 10
                  : h >= 'A' && h <= 'F' ? h - 'A' + 10 : -1;
      if (d < 0) fail("bad \\u escape");
      v = v * 16 + (unsigned)d;
    }
    return v;
  }
  std::string string() {
    expect('"');
    std::string o;
    while (p_ < s_.size() && s_[p_] != '"') {
      char c = s_[p_++];
      if (c != '\\') {
        o += c;
        continue;
      }
      if (p_ >= s_.size()) fail("bad escape");
      c = s_[p_++];
      switch (c) {
        case '"': o += '"'; break;
        case '\\': o += '\\'; break;
        case '/': o += '/'; break;
        case 'b': o += '\b'; break;
        case 'f': o += '\f'; break;
        case 'n': o += '\n'; break;
        case 'r': o += '\r'; break;
        case 't': o += '\t'; break;
        case 'u': {
          unsigned cp = hex4(p_);
          p_ += 4;
          if (cp >= 0xD800 && cp < 0xDC00 && p_ + 6 <= s_.size() && s_[p_] == '\\' &&
              s_[p_ + 1] == 'u') {
            const unsigned lo = hex4(p_ + 2);
            if (lo < 0xDC00 || lo >= 0xE000) fail("bad \\u surrogate pair");
            p_ += 6;
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          utf8(o, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
    if (p_ >= s_.size()) fail("unterminated string");
    ++p_;
    return o;
  }
  Value number() {
    const size_t b = p_;
    if (s_[p_] == '-') ++p_;
    bool real = false;
    while (p_ < s_.size()) {
      const char c = s_[p_];
      if (c >= '0' && c <= '9') {
        ++p_;
      } else if (c == '.' || c == 'e' || c == 'E' || c == '+' || c == '-') {
        real = true;
        ++p_;
      } else {
        break;
      }
    }
    const std::string t = s_.substr(b, p_ - b);
    // the whole token must be the number ("-", "1e", "1-2" are errors, not exceptions)
    size_t used = 0;
    try {
      if (!real) {
        const long long i = std::stoll(t, &used);
        if (used == t.size()) return Value((int64_t)i);
      }
    } catch (const std::out_of_range &) {   // out of int64 range: a double
    } catch (const std::invalid_argument &) {
    }
    try {
      const double d = std::stod(t, &used);
      if (used == t.size()) return Value(d);
    } catch (const std::exception &) {
    }
    fail("bad number '" + t + "'");
  }

  const std::string &s_;
  size_t p_ = 0;
  int depth_ = 0;
};

inline Value parse(const std::string &text) { return Parser(text).parse(); }

}  // namespace ofjson
