// Minimal JSON value + parser/serializer for the dstack-amd native agents (C++17, header-only).
// Objects keep insertion order (small vectors), numbers are stored as double or int64.
#pragma once
#include <cmath>
#include <cstring>
#include <cstdint>
#include <cstdio>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace dsa {

class Json {
 public:
  enum Type { Null, Bool, Int, Double, String, Array, Object };

  Json() : t_(Null) {}
  Json(std::nullptr_t) : t_(Null) {}
  Json(bool b) : t_(Bool), b_(b) {}
  Json(int v) : t_(Int), i_(v) {}
  Json(long v) : t_(Int), i_(v) {}
  Json(long long v) : t_(Int), i_(v) {}
  Json(unsigned v) : t_(Int), i_(v) {}
  Json(unsigned long v) : t_(Int), i_((int64_t)v) {}
  Json(unsigned long long v) : t_(Int), i_((int64_t)v) {}
  Json(double v) : t_(Double), d_(v) {}
  Json(const char* s) : t_(String), s_(s) {}
  Json(std::string s) : t_(String), s_(std::move(s)) {}

  static Json array() { Json j; j.t_ = Array; return j; }
  static Json object() { Json j; j.t_ = Object; return j; }

  Type type() const { return t_; }
  bool is_null() const { return t_ == Null; }
  bool is_object() const { return t_ == Object; }
  bool is_array() const { return t_ == Array; }
  bool is_string() const { return t_ == String; }
  bool is_number() const { return t_ == Int || t_ == Double; }
  bool is_bool() const { return t_ == Bool; }

  // accessors with defaults (never throw on type mismatch)
  bool as_bool(bool def = false) const { return t_ == Bool ? b_ : def; }
  int64_t as_int(int64_t def = 0) const {
    return t_ == Int ? i_ : (t_ == Double ? (int64_t)d_ : def);
  }
  double as_double(double def = 0) const {
    return t_ == Double ? d_ : (t_ == Int ? (double)i_ : def);
  }
  const std::string& as_string() const {
    static const std::string empty;
    return t_ == String ? s_ : empty;
  }
  std::string str(const std::string& def = "") const { return t_ == String ? s_ : def; }

  // arrays
  size_t size() const { return t_ == Array ? a_.size() : (t_ == Object ? o_.size() : 0); }
  const Json& operator[](size_t i) const {
    static const Json null;
    return (t_ == Array && i < a_.size()) ? a_[i] : null;
  }
  void push_back(Json v) {
    if (t_ == Null) t_ = Array;
    a_.push_back(std::move(v));
  }
  const std::vector<Json>& items() const { return a_; }

  // objects
  bool has(const std::string& k) const {
    if (t_ != Object) return false;
    for (auto& kv : o_)
      if (kv.first == k) return true;
    return false;
  }
  const Json& get(const std::string& k) const {
    static const Json null;
    if (t_ != Object) return null;
    for (auto& kv : o_)
      if (kv.first == k) return kv.second;
    return null;
  }
  const Json& operator[](const std::string& k) const { return get(k); }
  const Json& operator[](const char* k) const { return get(k); }
  Json& set(const std::string& k, Json v) {
    if (t_ == Null) t_ = Object;
    for (auto& kv : o_)
      if (kv.first == k) {
        kv.second = std::move(v);
        return kv.second;
      }
    o_.emplace_back(k, std::move(v));
    return o_.back().second;
  }
  Json& operator()(const std::string& k) {  // mutable object access, creates null entry
    if (t_ == Null) t_ = Object;
    for (auto& kv : o_)
      if (kv.first == k) return kv.second;
    o_.emplace_back(k, Json());
    return o_.back().second;
  }
  const std::vector<std::pair<std::string, Json>>& members() const { return o_; }

  std::string dump() const {
    std::string out;
    dump_to(out);
    return out;
  }

  static Json parse(const std::string& s) {
    size_t i = 0;
    Json j = parse_value(s, i);
    skip_ws(s, i);
    if (i != s.size()) throw std::runtime_error("json: trailing characters");
    return j;
  }

 private:
  Type t_;
  bool b_ = false;
  int64_t i_ = 0;
  double d_ = 0;
  std::string s_;
  std::vector<Json> a_;
  std::vector<std::pair<std::string, Json>> o_;

  static void escape(const std::string& s, std::string& out) {
    out.push_back('"');
    for (unsigned char c : s) {
      switch (c) {
        case '"': out += "\\\""; break;
        case '\\': out += "\\\\"; break;
        case '\n': out += "\\n"; break;
        case '\r': out += "\\r"; break;
        case '\t': out += "\\t"; break;
        case '\b': out += "\\b"; break;
        case '\f': out += "\\f"; break;
        default:
          if (c < 0x20) {
            char buf[8];
            snprintf(buf, sizeof buf, "\\u%04x", c);
            out += buf;
          } else {
            out.push_back((char)c);
          }
      }
    }
    out.push_back('"');
  }

  void dump_to(std::string& out) const {
    switch (t_) {
      case Null: out += "null"; break;
      case Bool: out += b_ ? "true" : "false"; break;
      case Int: out += std::to_string(i_); break;
      case Double: {
        if (!std::isfinite(d_)) {
          out += "null";
          break;
        }
        char buf[40];
        snprintf(buf, sizeof buf, "%.17g", d_);
        out += buf;
        // keep it a double on re-parse ("-0" or "3" would come back as an integer)
        if (!strpbrk(buf, ".eE")) out += ".0";
        break;
      }
      case String: escape(s_, out); break;
      case Array: {
        out.push_back('[');
        for (size_t k = 0; k < a_.size(); ++k) {
          if (k) out.push_back(',');
          a_[k].dump_to(out);
        }
        out.push_back(']');
        break;
      }
      case Object: {
        out.push_back('{');
        for (size_t k = 0; k < o_.size(); ++k) {
          if (k) out.push_back(',');
          escape(o_[k].first, out);
          out.push_back(':');
          o_[k].second.dump_to(out);
        }
        out.push_back('}');
        break;
      }
    }
  }

  static void skip_ws(const std::string& s, size_t& i) {
    while (i < s.size() && (s[i] == ' ' || s[i] == '\n' || s[i] == '\r' || s[i] == '\t')) ++i;
  }

  static void put_utf8(std::string& out, uint32_t cp) {
    if (cp < 0x80) {
      out.push_back((char)cp);
    } else if (cp < 0x800) {
      out.push_back((char)(0xC0 | (cp >> 6)));
      out.push_back((char)(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
      out.push_back((char)(0xE0 | (cp >> 12)));
      out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      out.push_back((char)(0x80 | (cp & 0x3F)));
    } else {
      out.push_back((char)(0xF0 | (cp >> 18)));
      out.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
      out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      out.push_back((char)(0x80 | (cp & 0x3F)));
    }
  }

  static uint32_t hex4(const std::string& s, size_t i) {
    if (i + 4 > s.size()) throw std::runtime_error("json: bad \\u escape");
    uint32_t v = 0;
    for (size_t k = 0; k < 4; ++k) {
      char c = s[i + k];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else throw std::runtime_error("json: bad hex digit");
    }
    return v;
  }

  static std::string parse_string(const std::string& s, size_t& i) {
    if (s[i] != '"') throw std::runtime_error("json: expected string");
    ++i;
    std::string out;
    while (i < s.size()) {
      char c = s[i++];
      if (c == '"') return out;
      if (c != '\\') {
        out.push_back(c);
        continue;
      }
      if (i >= s.size()) break;
      char e = s[i++];
      switch (e) {
        case '"': out.push_back('"'); break;
        case '\\': out.push_back('\\'); break;
        case '/': out.push_back('/'); break;
        case 'b': out.push_back('\b'); break;
        case 'f': out.push_back('\f'); break;
        case 'n': out.push_back('\n'); break;
        case 'r': out.push_back('\r'); break;
        case 't': out.push_back('\t'); break;
        case 'u': {
          uint32_t cp = hex4(s, i);
          i += 4;
          if (cp >= 0xD800 && cp < 0xDC00 && i + 6 <= s.size() && s[i] == '\\' && s[i + 1] == 'u') {
            uint32_t lo = hex4(s, i + 2);
            if (lo >= 0xDC00 && lo < 0xE000) {
              cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
              i += 6;
            }
          }
          put_utf8(out, cp);
          break;
        }
        default: throw std::runtime_error("json: bad escape");
      }
    }
    throw std::runtime_error("json: unterminated string");
  }

  static Json parse_value(const std::string& s, size_t& i, int depth = 0) {
    if (depth > 256) throw std::runtime_error("json: nesting too deep");
    skip_ws(s, i);
    if (i >= s.size()) throw std::runtime_error("json: unexpected end");
    char c = s[i];
    if (c == '{') {
      ++i;
      Json j = object();
      skip_ws(s, i);
      if (i < s.size() && s[i] == '}') {
        ++i;
        return j;
      }
      while (true) {
        skip_ws(s, i);
        std::string k = parse_string(s, i);
        skip_ws(s, i);
        if (i >= s.size() || s[i] != ':') throw std::runtime_error("json: expected ':'");
        ++i;
        j.o_.emplace_back(std::move(k), parse_value(s, i, depth + 1));
        skip_ws(s, i);
        if (i < s.size() && s[i] == ',') {
          ++i;
          continue;
        }
        if (i < s.size() && s[i] == '}') {
          ++i;
          return j;
        }
        throw std::runtime_error("json: expected ',' or '}'");
      }
    }
    if (c == '[') {
      ++i;
      Json j = array();
      skip_ws(s, i);
      if (i < s.size() && s[i] == ']') {
        ++i;
        return j;
      }
      while (true) {
        j.a_.push_back(parse_value(s, i, depth + 1));
        skip_ws(s, i);
        if (i < s.size() && s[i] == ',') {
          ++i;
          continue;
        }
        if (i < s.size() && s[i] == ']') {
          ++i;
          return j;
        }
        throw std::runtime_error("json: expected ',' or ']'");
      }
    }
    if (c == '"') return Json(parse_string(s, i));
    if (s.compare(i, 4, "true") == 0) {
      i += 4;
      return Json(true);
    }
    if (s.compare(i, 5, "false") == 0) {
      i += 5;
      return Json(false);
    }
    if (s.compare(i, 4, "null") == 0) {
      i += 4;
      return Json();
    }
    // RFC 8259 number: -? (0 | [1-9][0-9]*) (. [0-9]+)? ([eE] [+-]? [0-9]+)?
    size_t st = i;
    bool is_float = false;
    auto digits = [&]() {
      size_t d0 = i;
      while (i < s.size() && s[i] >= '0' && s[i] <= '9') ++i;
      return i - d0;
    };
    if (i < s.size() && s[i] == '-') ++i;
    if (i >= s.size() || s[i] < '0' || s[i] > '9') throw std::runtime_error("json: unexpected character");
    if (s[i] == '0')
      ++i;
    else
      digits();
    if (i < s.size() && s[i] == '.') {
      ++i;
      is_float = true;
      if (digits() == 0) throw std::runtime_error("json: digits expected after '.'");
    }
    if (i < s.size() && (s[i] == 'e' || s[i] == 'E')) {
      ++i;
      is_float = true;
      if (i < s.size() && (s[i] == '+' || s[i] == '-')) ++i;
      if (digits() == 0) throw std::runtime_error("json: digits expected in the exponent");
    }
    std::string num = s.substr(st, i - st);
    if (!is_float) {
      try {
        return Json((long long)std::stoll(num));
      } catch (...) {
      }
    }
    return Json(std::stod(num));
  }
};

}  // namespace dsa
