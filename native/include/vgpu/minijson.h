// Tiny JSON reader for test fixtures (objects, arrays, strings, numbers, bools,
// null).  Only used by the fake vendor libraries — never on a hot path.
#pragma once

#include <cctype>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace minijson {

struct Value {
  enum Kind { Null, Bool, Num, Str, Arr, Obj } kind = Null;
  bool b = false;
  double n = 0;
  std::string s;
  std::vector<Value> a;
  std::map<std::string, Value> o;

  const Value& operator[](const std::string& k) const {
    static Value null;
    auto it = o.find(k);
    return it == o.end() ? null : it->second;
  }
  const Value& operator[](size_t i) const {
    static Value null;
    return i < a.size() ? a[i] : null;
  }
  size_t size() const { return kind == Arr ? a.size() : o.size(); }
  double num(double d = 0) const { return kind == Num ? n : (kind == Bool ? (b ? 1 : 0) : d); }
  std::string str(const std::string& d = "") const { return kind == Str ? s : d; }
  bool truthy(bool d = false) const { return kind == Bool ? b : (kind == Num ? n != 0 : d); }
};

class Parser {
 public:
  explicit Parser(const std::string& t) : t_(t) {}
  bool parse(Value& v) {
    ws();
    if (!value(v)) return false;
    ws();
    return p_ == t_.size();
  }

 private:
  const std::string& t_;
  size_t p_ = 0;
  void ws() {
    while (p_ < t_.size() && isspace((unsigned char)t_[p_])) ++p_;
  }
  bool lit(const char* w) {
    size_t n = strlen(w);
    if (t_.compare(p_, n, w) != 0) return false;
    p_ += n;
    return true;
  }
  bool str(std::string& out) {
    if (t_[p_] != '"') return false;
    ++p_;
    while (p_ < t_.size() && t_[p_] != '"') {
      char c = t_[p_++];
      if (c == '\\' && p_ < t_.size()) {
        char e = t_[p_++];
        switch (e) {
          case 'n': out += '\n'; break;
          case 't': out += '\t'; break;
          case 'u': p_ += 4; out += '?'; break;
          default: out += e;
        }
      } else {
        out += c;
      }
    }
    if (p_ >= t_.size()) return false;
    ++p_;
    return true;
  }
  bool value(Value& v) {
    if (p_ >= t_.size()) return false;
    char c = t_[p_];
    if (c == '{') {
      v.kind = Value::Obj;
      ++p_;
      ws();
      if (t_[p_] == '}') { ++p_; return true; }
      for (;;) {
        ws();
        std::string k;
        if (!str(k)) return false;
        ws();
        if (t_[p_++] != ':') return false;
        ws();
        if (!value(v.o[k])) return false;
        ws();
        if (t_[p_] == ',') { ++p_; continue; }
        if (t_[p_] == '}') { ++p_; return true; }
        return false;
      }
    }
    if (c == '[') {
      v.kind = Value::Arr;
      ++p_;
      ws();
      if (t_[p_] == ']') { ++p_; return true; }
      for (;;) {
        ws();
        v.a.emplace_back();
        if (!value(v.a.back())) return false;
        ws();
        if (t_[p_] == ',') { ++p_; continue; }
        if (t_[p_] == ']') { ++p_; return true; }
        return false;
      }
    }
    if (c == '"') { v.kind = Value::Str; return str(v.s); }
    if (lit("true")) { v.kind = Value::Bool; v.b = true; return true; }
    if (lit("false")) { v.kind = Value::Bool; v.b = false; return true; }
    if (lit("null")) { v.kind = Value::Null; return true; }
    char* end = nullptr;
    v.n = strtod(t_.c_str() + p_, &end);
    if (end == t_.c_str() + p_) return false;
    v.kind = Value::Num;
    p_ = end - t_.c_str();
    return true;
  }
};

inline bool parse(const std::string& text, Value& out) { return Parser(text).parse(out); }

}  // namespace minijson
