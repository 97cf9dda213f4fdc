// Small JSON reader for Kubernetes objects crossing the C ABI (product side).
#pragma once
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace ksg {
namespace json {

struct Node {
  enum T : uint8_t { NUL, BOOL, NUM, STR, ARR, OBJ };
  T t = NUL;
  bool b = false;
  std::string s;                 // string / number text
  std::vector<Node> items;       // ARR values, OBJ values
  std::vector<std::string> keys; // OBJ keys (parallel to items)

  const Node* operator[](const char* k) const {
    if (t != OBJ) return nullptr;
    for (size_t i = 0; i < keys.size(); ++i)
      if (keys[i] == k) return &items[i];
    return nullptr;
  }
  bool null() const { return t == NUL; }
  const std::string& text() const { return s; }
  long long num(long long d = 0) const { return (t == NUM || t == STR) && !s.empty() ? std::strtoll(s.c_str(), nullptr, 10) : d; }
  size_t size() const { return items.size(); }
};

class Reader {
 public:
  Reader(const char* b, size_t n) : c_(b), end_(b + n) {}
  Node read() {
    Node n;
    value(n);
    skip();
    if (c_ != end_) bad("trailing characters");
    return n;
  }

 private:
  const char* c_;
  const char* end_;
  [[noreturn]] void bad(const char* why) { throw std::runtime_error(std::string("invalid JSON: ") + why); }
  void skip() {
    while (c_ != end_ && (*c_ == ' ' || *c_ == '\t' || *c_ == '\n' || *c_ == '\r')) ++c_;
  }
  bool lit(const char* w) {
    size_t l = std::strlen(w);
    if ((size_t)(end_ - c_) >= l && std::memcmp(c_, w, l) == 0) { c_ += l; return true; }
    return false;
  }
  void value(Node& n) {
    skip();
    if (c_ == end_) bad("unexpected end");
    switch (*c_) {
      case '{': {
        ++c_;
        n.t = Node::OBJ;
        skip();
        if (c_ != end_ && *c_ == '}') { ++c_; return; }
        for (;;) {
          skip();
          if (c_ == end_ || *c_ != '"') bad("expected key");
          n.keys.emplace_back();
          str(n.keys.back());
          skip();
          if (c_ == end_ || *c_++ != ':') bad("expected ':'");
          n.items.emplace_back();
          value(n.items.back());
          skip();
          if (c_ != end_ && *c_ == ',') { ++c_; continue; }
          if (c_ != end_ && *c_ == '}') { ++c_; return; }
          bad("expected ',' or '}'");
        }
      }
      case '[': {
        ++c_;
        n.t = Node::ARR;
        skip();
        if (c_ != end_ && *c_ == ']') { ++c_; return; }
        for (;;) {
          n.items.emplace_back();
          value(n.items.back());
          skip();
          if (c_ != end_ && *c_ == ',') { ++c_; continue; }
          if (c_ != end_ && *c_ == ']') { ++c_; return; }
          bad("expected ',' or ']'");
        }
      }
      case '"':
        n.t = Node::STR;
        str(n.s);
        return;
      default:
        if (lit("true")) { n.t = Node::BOOL; n.b = true; return; }
        if (lit("false")) { n.t = Node::BOOL; return; }
        if (lit("null")) return;
        {
          const char* b = c_;
          while (c_ != end_ && (std::isdigit((unsigned char)*c_) || *c_ == '-' || *c_ == '+' || *c_ == '.' ||
                                *c_ == 'e' || *c_ == 'E'))
            ++c_;
          if (b == c_) bad("unexpected character");
          n.t = Node::NUM;
          n.s.assign(b, c_);
        }
    }
  }
  static void utf8(std::string& o, uint32_t cp) {
    if (cp < 0x80) { o.push_back((char)cp); return; }
    if (cp < 0x800) { o.push_back((char)(0xC0 | cp >> 6)); o.push_back((char)(0x80 | (cp & 63))); return; }
    if (cp < 0x10000) {
      o.push_back((char)(0xE0 | cp >> 12)); o.push_back((char)(0x80 | ((cp >> 6) & 63))); o.push_back((char)(0x80 | (cp & 63)));
      return;
    }
    o.push_back((char)(0xF0 | cp >> 18)); o.push_back((char)(0x80 | ((cp >> 12) & 63)));
    o.push_back((char)(0x80 | ((cp >> 6) & 63))); o.push_back((char)(0x80 | (cp & 63)));
  }
  uint32_t hex() {
    if (end_ - c_ < 4) bad("short \\u escape");
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) {
      char h = *c_++;
      v = v * 16 + (h >= '0' && h <= '9' ? h - '0' : h >= 'a' && h <= 'f' ? h - 'a' + 10 : h >= 'A' && h <= 'F' ? h - 'A' + 10 : (bad("bad hex"), 0));
    }
    return v;
  }
  void str(std::string& o) {
    ++c_;
    const char* run = c_;
    while (c_ != end_) {
      char ch = *c_;
      if (ch == '"') { o.append(run, c_); ++c_; return; }
      if (ch != '\\') { ++c_; continue; }
      o.append(run, c_);
      ++c_;
      if (c_ == end_) break;
      char e = *c_++;
      switch (e) {
        case 'n': o.push_back('\n'); break;
        case 't': o.push_back('\t'); break;
        case 'r': o.push_back('\r'); break;
        case 'b': o.push_back('\b'); break;
        case 'f': o.push_back('\f'); break;
        case 'u': {
          uint32_t cp = hex();
          if (cp >= 0xD800 && cp <= 0xDBFF && end_ - c_ >= 6 && c_[0] == '\\' && c_[1] == 'u') {
            c_ += 2;
            cp = 0x10000 + ((cp - 0xD800) << 10) + (hex() - 0xDC00);
          }
          utf8(o, cp);
          break;
        }
        default: o.push_back(e);
      }
      run = c_;
    }
    bad("unterminated string");
  }
};

inline Node parse(const char* b, size_t n) { return Reader(b, n).read(); }

}  // namespace json
}  // namespace ksg
