// Minimal JSON value / parser / serializer for the node agent's
// line-delimited protocol (no external deps: the agent must build with just
// g++ on the MI355X host).
#pragma once
#include <cmath>
#include <cstdint>
#include <map>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

namespace pto {

struct Json {
  enum Type { Null, Bool, Num, Str, Arr, Obj } t = Null;
  bool b = false;
  double n = 0;
  std::string s;
  std::vector<Json> a;
  std::map<std::string, Json> o;

  Json() = default;
  Json(bool v) : t(Bool), b(v) {}
  Json(int v) : t(Num), n(v) {}
  Json(long v) : t(Num), n((double)v) {}
  Json(long long v) : t(Num), n((double)v) {}
  Json(unsigned long v) : t(Num), n((double)v) {}
  Json(double v) : t(Num), n(v) {}
  Json(const char* v) : t(Str), s(v) {}
  Json(const std::string& v) : t(Str), s(v) {}
  static Json array() { Json j; j.t = Arr; return j; }
  static Json object() { Json j; j.t = Obj; return j; }

  bool has(const std::string& k) const { return t == Obj && o.count(k); }
  const Json& operator[](const std::string& k) const {
    static const Json null;
    auto it = o.find(k);
    return it == o.end() ? null : it->second;
  }
  Json& operator[](const std::string& k) { t = Obj; return o[k]; }
  void push(const Json& v) { t = Arr; a.push_back(v); }
  std::string str(const std::string& def = "") const { return t == Str ? s : def; }
  double num(double def = 0) const { return t == Num ? n : (t == Bool ? (b ? 1 : 0) : def); }
  long long i64(long long def = 0) const { return t == Num ? (long long)n : def; }
  bool boolean(bool def = false) const { return t == Bool ? b : (t == Num ? n != 0 : def); }

  std::string dump() const {
    std::ostringstream os;
    write(os);
    return os.str();
  }
  void write(std::ostringstream& os) const {
    switch (t) {
      case Null: os << "null"; break;
      case Bool: os << (b ? "true" : "false"); break;
      case Num:
        if (std::isfinite(n) && n == (double)(long long)n && std::fabs(n) < 9e15) os << (long long)n;
        else if (std::isfinite(n)) { os.precision(17); os << n; }
        else os << "null";
        break;
      case Str: esc(os, s); break;
      case Arr: {
        os << '[';
        for (size_t i = 0; i < a.size(); ++i) { if (i) os << ','; a[i].write(os); }
        os << ']';
        break;
      }
      case Obj: {
        os << '{';
        bool first = true;
        for (auto& kv : o) {
          if (!first) os << ',';
          first = false;
          esc(os, kv.first);
          os << ':';
          kv.second.write(os);
        }
        os << '}';
        break;
      }
    }
  }
  static void esc(std::ostringstream& os, const std::string& v) {
    os << '"';
    for (unsigned char c : v) {
      switch (c) {
        case '"': os << "\\\""; break;
        case '\\': os << "\\\\"; break;
        case '\n': os << "\\n"; break;
        case '\r': os << "\\r"; break;
        case '\t': os << "\\t"; break;
        default:
          if (c < 0x20) { char buf[8]; snprintf(buf, sizeof buf, "\\u%04x", c); os << buf; }
          else os << c;
      }
    }
    os << '"';
  }

  // ---------------------------------------------------------------- parse
  static Json parse(const std::string& text) {
    size_t i = 0;
    Json v = parse_value(text, i);
    skip(text, i);
    if (i != text.size()) throw std::runtime_error("trailing characters in JSON");
    return v;
  }

 private:
  static void skip(const std::string& t, size_t& i) {
    while (i < t.size() && (t[i] == ' ' || t[i] == '\n' || t[i] == '\r' || t[i] == '\t')) ++i;
  }
  static Json parse_value(const std::string& t, size_t& i) {
    skip(t, i);
    if (i >= t.size()) throw std::runtime_error("unexpected end of JSON");
    char c = t[i];
    if (c == '{') {
      Json j = object();
      ++i;
      skip(t, i);
      if (i < t.size() && t[i] == '}') { ++i; return j; }
      while (true) {
        skip(t, i);
        Json k = parse_value(t, i);
        if (k.t != Str) throw std::runtime_error("object key must be a string");
        skip(t, i);
        if (i >= t.size() || t[i] != ':') throw std::runtime_error("expected ':'");
        ++i;
        j.o[k.s] = parse_value(t, i);
        skip(t, i);
        if (i < t.size() && t[i] == ',') { ++i; continue; }
        if (i < t.size() && t[i] == '}') { ++i; return j; }
        throw std::runtime_error("expected ',' or '}'");
      }
    }
    if (c == '[') {
      Json j = array();
      ++i;
      skip(t, i);
      if (i < t.size() && t[i] == ']') { ++i; return j; }
      while (true) {
        j.a.push_back(parse_value(t, i));
        skip(t, i);
        if (i < t.size() && t[i] == ',') { ++i; continue; }
        if (i < t.size() && t[i] == ']') { ++i; return j; }
        throw std::runtime_error("expected ',' or ']'");
      }
    }
    if (c == '"') {
      Json j;
      j.t = Str;
      ++i;
      while (i < t.size() && t[i] != '"') {
        if (t[i] == '\\' && i + 1 < t.size()) {
          char e = t[++i];
          switch (e) {
            case 'n': j.s += '\n'; break;
            case 't': j.s += '\t'; break;
            case 'r': j.s += '\r'; break;
            case 'b': j.s += '\b'; break;
            case 'f': j.s += '\f'; break;
            case 'u': {
              if (i + 4 >= t.size()) throw std::runtime_error("bad \\u escape");
              unsigned cp = std::stoul(t.substr(i + 1, 4), nullptr, 16);
              i += 4;
              if (cp < 0x80) j.s += (char)cp;
              else if (cp < 0x800) { j.s += (char)(0xC0 | (cp >> 6)); j.s += (char)(0x80 | (cp & 0x3F)); }
              else {
                j.s += (char)(0xE0 | (cp >> 12));
                j.s += (char)(0x80 | ((cp >> 6) & 0x3F));
                j.s += (char)(0x80 | (cp & 0x3F));
              }
              break;
            }
            default: j.s += e;
          }
          ++i;
        } else {
          j.s += t[i++];
        }
      }
      if (i >= t.size()) throw std::runtime_error("unterminated string");
      ++i;
      return j;
    }
    if (t.compare(i, 4, "true") == 0) { i += 4; return Json(true); }
    if (t.compare(i, 5, "false") == 0) { i += 5; return Json(false); }
    if (t.compare(i, 4, "null") == 0) { i += 4; return Json(); }
    size_t st = i;
    while (i < t.size() && (isdigit((unsigned char)t[i]) || t[i] == '-' || t[i] == '+' || t[i] == '.' ||
                            t[i] == 'e' || t[i] == 'E'))
      ++i;
    if (st == i) throw std::runtime_error("unexpected character in JSON");
    return Json(std::stod(t.substr(st, i - st)));
  }
};

}  // namespace pto
