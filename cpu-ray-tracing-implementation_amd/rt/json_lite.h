// json_lite.h -- a small JSON reader for the glTF loader (rt/gltf_loader.h).
//
// The reference parses .gltf files with a vendored JSON library (json.h); only the
// read side is needed here: null, booleans, numbers, strings (with \uXXXX escapes),
// arrays and objects, and the lookups the loader makes (`value(key, default)`,
// indexing, `size()`). Parse errors throw std::runtime_error with the byte offset.
#pragma once
#include <cstdint>
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace json_lite {

class value {
 public:
  enum kind_t { kNull, kBool, kNumber, kString, kArray, kObject };

  value() = default;
  kind_t kind() const { return kind_; }
  bool is_null() const { return kind_ == kNull; }
  bool is_number() const { return kind_ == kNumber; }
  bool is_string() const { return kind_ == kString; }
  bool is_array() const { return kind_ == kArray; }
  bool is_object() const { return kind_ == kObject; }

  // number of array elements or object members (0 for scalars and null, like the reference's json)
  size_t size() const {
    if (kind_ == kArray) return arr_.size();
    if (kind_ == kObject) return obj_.size();
    return 0;
  }
  bool contains(const std::string& k) const { return kind_ == kObject && obj_.count(k) != 0; }

  // missing keys / out-of-range indices read as null
  const value& operator[](const std::string& k) const {
    if (kind_ == kObject) {
      auto it = obj_.find(k);
      if (it != obj_.end()) return it->second;
    }
    return null_value();
  }
  const value& operator[](size_t i) const { return kind_ == kArray && i < arr_.size() ? arr_[i] : null_value(); }

  double as_number() const {
    if (kind_ != kNumber) throw std::runtime_error("json: not a number");
    return num_;
  }
  const std::string& as_string() const {
    if (kind_ != kString) throw std::runtime_error("json: not a string");
    return str_;
  }
  // obj.value(key, default): the member converted to the default's type, or the default
  int value_or(const std::string& k, int dflt) const {
    const value& v = (*this)[k];
    return v.is_number() ? (int)v.num_ : dflt;
  }
  std::string value_or(const std::string& k, const std::string& dflt) const {
    const value& v = (*this)[k];
    return v.is_string() ? v.str_ : dflt;
  }

  static value parse(const std::string& text) {
    size_t pos = 0;
    value v = parse_value(text, pos, 0);
    skip_ws(text, pos);
    if (pos != text.size()) fail("trailing characters", pos);
    return v;
  }

 private:
  kind_t kind_ = kNull;
  bool b_ = false;
  double num_ = 0;
  std::string str_;
  std::vector<value> arr_;
  std::map<std::string, value> obj_;

  static const value& null_value() {
    static const value n;
    return n;
  }
  [[noreturn]] static void fail(const char* what, size_t pos) {
    throw std::runtime_error(std::string("json: ") + what + " at byte " + std::to_string(pos));
  }
  static void skip_ws(const std::string& t, size_t& p) {
    while (p < t.size() && (t[p] == ' ' || t[p] == '\t' || t[p] == '\n' || t[p] == '\r')) p++;
  }
  static void expect(const std::string& t, size_t& p, const char* lit) {
    for (const char* c = lit; *c; c++, p++)
      if (p >= t.size() || t[p] != *c) fail("bad literal", p);
  }
  static void put_utf8(std::string& s, uint32_t cp) {
    if (cp < 0x80) {
      s += (char)cp;
    } else if (cp < 0x800) {
      s += (char)(0xC0 | (cp >> 6));
      s += (char)(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
      s += (char)(0xE0 | (cp >> 12));
      s += (char)(0x80 | ((cp >> 6) & 0x3F));
      s += (char)(0x80 | (cp & 0x3F));
    } else {
      s += (char)(0xF0 | (cp >> 18));
      s += (char)(0x80 | ((cp >> 12) & 0x3F));
      s += (char)(0x80 | ((cp >> 6) & 0x3F));
      s += (char)(0x80 | (cp & 0x3F));
    }
  }
  static uint32_t hex4(const std::string& t, size_t& p) {
    if (p + 4 > t.size()) fail("short \\u escape", p);
    uint32_t v = 0;
    for (int i = 0; i < 4; i++, p++) {
      char c = t[p];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= (uint32_t)(c - '0');
      else if (c >= 'a' && c <= 'f') v |= (uint32_t)(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') v |= (uint32_t)(c - 'A' + 10);
      else fail("bad \\u escape", p);
    }
    return v;
  }
  static std::string parse_string(const std::string& t, size_t& p) {
    if (t[p] != '"') fail("expected string", p);
    p++;
    std::string s;
    while (true) {
      if (p >= t.size()) fail("unterminated string", p);
      char c = t[p++];
      if (c == '"') break;
      if ((unsigned char)c < 0x20) fail("control character in string", p - 1);
      if (c != '\\') {
        s += c;
        continue;
      }
      if (p >= t.size()) fail("unterminated escape", p);
      char e = t[p++];
      switch (e) {
        case '"': s += '"'; break;
        case '\\': s += '\\'; break;
        case '/': s += '/'; break;
        case 'b': s += '\b'; break;
        case 'f': s += '\f'; break;
        case 'n': s += '\n'; break;
        case 'r': s += '\r'; break;
        case 't': s += '\t'; break;
        case 'u': {
          uint32_t cp = hex4(t, p);
          if (cp >= 0xD800 && cp < 0xDC00 && p + 1 < t.size() && t[p] == '\\' && t[p + 1] == 'u') {
            p += 2;
            uint32_t lo = hex4(t, p);
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          put_utf8(s, cp);
          break;
        }
        default: fail("bad escape", p - 1);
      }
    }
    return s;
  }
  static value parse_value(const std::string& t, size_t& p, int depth) {
    if (depth > 256) fail("nesting too deep", p);
    skip_ws(t, p);
    if (p >= t.size()) fail("unexpected end", p);
    value v;
    char c = t[p];
    if (c == '{') {
      v.kind_ = kObject;
      p++;
      skip_ws(t, p);
      if (p < t.size() && t[p] == '}') {
        p++;
        return v;
      }
      while (true) {
        skip_ws(t, p);
        std::string k = parse_string(t, p);
        skip_ws(t, p);
        if (p >= t.size() || t[p] != ':') fail("expected ':'", p);
        p++;
        v.obj_[k] = parse_value(t, p, depth + 1);
        skip_ws(t, p);
        if (p < t.size() && t[p] == ',') {
          p++;
          continue;
        }
        if (p < t.size() && t[p] == '}') {
          p++;
          return v;
        }
        fail("expected ',' or '}'", p);
      }
    }
    if (c == '[') {
      v.kind_ = kArray;
      p++;
      skip_ws(t, p);
      if (p < t.size() && t[p] == ']') {
        p++;
        return v;
      }
      while (true) {
        v.arr_.push_back(parse_value(t, p, depth + 1));
        skip_ws(t, p);
        if (p < t.size() && t[p] == ',') {
          p++;
          continue;
        }
        if (p < t.size() && t[p] == ']') {
          p++;
          return v;
        }
        fail("expected ',' or ']'", p);
      }
    }
    if (c == '"') {
      v.kind_ = kString;
      v.str_ = parse_string(t, p);
      return v;
    }
    if (c == 't') {
      expect(t, p, "true");
      v.kind_ = kBool;
      v.b_ = true;
      return v;
    }
    if (c == 'f') {
      expect(t, p, "false");
      v.kind_ = kBool;
      return v;
    }
    if (c == 'n') {
      expect(t, p, "null");
      return v;
    }
    // number: -?(0|[1-9][0-9]*)(\.[0-9]+)?([eE][+-]?[0-9]+)?
    size_t start = p;
    if (t[p] == '-') p++;
    if (p >= t.size() || !(t[p] >= '0' && t[p] <= '9')) fail("bad value", start);
    while (p < t.size() && ((t[p] >= '0' && t[p] <= '9') || t[p] == '.' || t[p] == 'e' || t[p] == 'E' ||
                            t[p] == '+' || t[p] == '-'))
      p++;
    std::string num = t.substr(start, p - start);
    char* end = nullptr;
    v.num_ = std::strtod(num.c_str(), &end);
    if (end != num.c_str() + num.size()) fail("bad number", start);
    v.kind_ = kNumber;
    return v;
  }
};

}  // namespace json_lite
