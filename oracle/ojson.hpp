// Minimal JSON DOM for the CPU oracle (test infrastructure only).
// Objects keep insertion order (Go maps are unordered; lists such as taints are
// arrays, so order-sensitive data never depends on object order).
#pragma once
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace ojson {

struct Value {
  enum Kind { Null, Bool, Num, Str, Arr, Obj } kind = Null;
  bool b = false;
  double num = 0;
  std::string raw;  // number text (exact) or string contents
  std::vector<Value> arr;
  std::vector<std::pair<std::string, Value>> obj;

  const Value* get(const char* k) const {
    if (kind != Obj) return nullptr;
    for (auto& kv : obj)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
  bool is_null() const { return kind == Null; }
  std::string str(const std::string& dflt = "") const {
    if (kind == Str || kind == Num) return raw;
    return dflt;
  }
  long long i64(long long dflt = 0) const {
    if (kind == Num) return std::strtoll(raw.c_str(), nullptr, 10);
    if (kind == Str) return std::strtoll(raw.c_str(), nullptr, 10);
    return dflt;
  }
};

class Parser {
 public:
  Parser(const char* s, size_t n) : p_(s), e_(s + n) {}
  Value parse() {
    Value v = value();
    ws();
    if (p_ != e_) fail("trailing data");
    return v;
  }

 private:
  const char* p_;
  const char* e_;
  [[noreturn]] void fail(const char* m) { throw std::runtime_error(std::string("json: ") + m); }
  void ws() {
    while (p_ < e_ && (*p_ == ' ' || *p_ == '\n' || *p_ == '\t' || *p_ == '\r')) ++p_;
  }
  Value value() {
    ws();
    if (p_ >= e_) fail("eof");
    Value v;
    char c = *p_;
    if (c == '{') {
      v.kind = Value::Obj;
      ++p_;
      ws();
      if (p_ < e_ && *p_ == '}') { ++p_; return v; }
      for (;;) {
        ws();
        if (p_ >= e_ || *p_ != '"') fail("key");
        std::string k = string();
        ws();
        if (p_ >= e_ || *p_ != ':') fail(":");
        ++p_;
        v.obj.emplace_back(std::move(k), value());
        ws();
        if (p_ < e_ && *p_ == ',') { ++p_; continue; }
        if (p_ < e_ && *p_ == '}') { ++p_; break; }
        fail("object");
      }
    } else if (c == '[') {
      v.kind = Value::Arr;
      ++p_;
      ws();
      if (p_ < e_ && *p_ == ']') { ++p_; return v; }
      for (;;) {
        v.arr.push_back(value());
        ws();
        if (p_ < e_ && *p_ == ',') { ++p_; continue; }
        if (p_ < e_ && *p_ == ']') { ++p_; break; }
        fail("array");
      }
    } else if (c == '"') {
      v.kind = Value::Str;
      v.raw = string();
    } else if (c == 't' && e_ - p_ >= 4 && !std::strncmp(p_, "true", 4)) {
      v.kind = Value::Bool; v.b = true; p_ += 4;
    } else if (c == 'f' && e_ - p_ >= 5 && !std::strncmp(p_, "false", 5)) {
      v.kind = Value::Bool; v.b = false; p_ += 5;
    } else if (c == 'n' && e_ - p_ >= 4 && !std::strncmp(p_, "null", 4)) {
      p_ += 4;
    } else {
      const char* s = p_;
      while (p_ < e_ && (std::strchr("+-.eE", *p_) || (*p_ >= '0' && *p_ <= '9'))) ++p_;
      if (s == p_) fail("value");
      v.kind = Value::Num;
      v.raw.assign(s, p_);
      v.num = std::strtod(v.raw.c_str(), nullptr);
    }
    return v;
  }
  static void put_utf8(std::string& o, unsigned cp) {
    if (cp < 0x80) o += char(cp);
    else if (cp < 0x800) { o += char(0xC0 | (cp >> 6)); o += char(0x80 | (cp & 0x3F)); }
    else if (cp < 0x10000) { o += char(0xE0 | (cp >> 12)); o += char(0x80 | ((cp >> 6) & 0x3F)); o += char(0x80 | (cp & 0x3F)); }
    else { o += char(0xF0 | (cp >> 18)); o += char(0x80 | ((cp >> 12) & 0x3F)); o += char(0x80 | ((cp >> 6) & 0x3F)); o += char(0x80 | (cp & 0x3F)); }
  }
  unsigned hex4() {
    if (e_ - p_ < 4) fail("\\u");
    unsigned v = 0;
    for (int i = 0; i < 4; ++i) {
      char c = *p_++;
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else fail("hex");
    }
    return v;
  }
  std::string string() {
    ++p_;  // opening quote
    std::string o;
    while (p_ < e_ && *p_ != '"') {
      char c = *p_++;
      if (c != '\\') { o += c; continue; }
      if (p_ >= e_) fail("escape");
      char d = *p_++;
      switch (d) {
        case '"': o += '"'; break;
        case '\\': o += '\\'; break;
        case '/': o += '/'; break;
        case 'b': o += '\b'; break;
        case 'f': o += '\f'; break;
        case 'n': o += '\n'; break;
        case 'r': o += '\r'; break;
        case 't': o += '\t'; break;
        case 'u': {
          unsigned cp = hex4();
          if (cp >= 0xD800 && cp < 0xDC00 && e_ - p_ >= 6 && p_[0] == '\\' && p_[1] == 'u') {
            p_ += 2;
            unsigned lo = hex4();
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          put_utf8(o, cp);
          break;
        }
        default: fail("escape");
      }
    }
    if (p_ >= e_) fail("unterminated string");
    ++p_;
    return o;
  }
};

inline Value parse(const char* s, size_t n) { return Parser(s, n).parse(); }

}  // namespace ojson
