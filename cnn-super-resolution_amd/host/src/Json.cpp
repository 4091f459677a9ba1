#include "Json.hpp"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>

#include "Context.hpp"  // IOException

namespace srcnn {
namespace json {

const Value* Value::find(const std::string& key) const {
  for (auto& kv : object)
    if (kv.first == key) return &kv.second;
  return nullptr;
}

namespace {

struct Parser {
  const std::string& s;
  size_t i = 0;

  explicit Parser(const std::string& src) : s(src) {}

  [[noreturn]] void fail(const char* what) const {
    char buf[160];
    std::snprintf(buf, sizeof(buf), "Json parsing error: %s at offset %zu in: '%.20s'", what, i,
                  i < s.size() ? s.c_str() + i : "");
    throw IOException(buf);
  }

  void ws() {
    while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) ++i;
  }

  bool lit(const char* w) {
    size_t n = std::strlen(w);
    if (s.compare(i, n, w) == 0) {
      i += n;
      return true;
    }
    return false;
  }

  static void utf8(std::string& out, unsigned cp) {
    if (cp < 0x80) {
      out += char(cp);
    } else if (cp < 0x800) {
      out += char(0xC0 | (cp >> 6));
      out += char(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
      out += char(0xE0 | (cp >> 12));
      out += char(0x80 | ((cp >> 6) & 0x3F));
      out += char(0x80 | (cp & 0x3F));
    } else {
      out += char(0xF0 | (cp >> 18));
      out += char(0x80 | ((cp >> 12) & 0x3F));
      out += char(0x80 | ((cp >> 6) & 0x3F));
      out += char(0x80 | (cp & 0x3F));
    }
  }

  unsigned hex4() {
    if (i + 4 > s.size()) fail("bad \\u escape");
    unsigned v = 0;
    for (int k = 0; k < 4; ++k) {
      char c = s[i++];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= unsigned(c - '0');
      else if (c >= 'a' && c <= 'f') v |= unsigned(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') v |= unsigned(c - 'A' + 10);
      else fail("bad \\u escape");
    }
    return v;
  }

  std::string str() {
    if (s[i] != '"') fail("expected string");
    ++i;
    std::string out;
    while (true) {
      if (i >= s.size()) fail("unterminated string");
      char c = s[i++];
      if (c == '"') break;
      if (static_cast<unsigned char>(c) < 0x20) fail("control character in string");
      if (c != '\\') {
        out += c;
        continue;
      }
      if (i >= s.size()) fail("unterminated escape");
      char e = s[i++];
      switch (e) {
        case '"': out += '"'; break;
        case '\\': out += '\\'; break;
        case '/': out += '/'; break;
        case 'b': out += '\b'; break;
        case 'f': out += '\f'; break;
        case 'n': out += '\n'; break;
        case 'r': out += '\r'; break;
        case 't': out += '\t'; break;
        case 'u': {
          unsigned cp = hex4();
          if (cp >= 0xD800 && cp < 0xDC00 && lit("\\u")) {
            unsigned lo = hex4();
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          utf8(out, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
    return out;
  }

  double num() {
    size_t b = i;
    if (s[i] == '-') ++i;
    if (i >= s.size() || !(s[i] >= '0' && s[i] <= '9')) fail("expected number");
    while (i < s.size() && s[i] >= '0' && s[i] <= '9') ++i;
    if (i < s.size() && s[i] == '.') {
      ++i;
      if (i >= s.size() || !(s[i] >= '0' && s[i] <= '9')) fail("bad fraction");
      while (i < s.size() && s[i] >= '0' && s[i] <= '9') ++i;
    }
    if (i < s.size() && (s[i] == 'e' || s[i] == 'E')) {
      ++i;
      if (i < s.size() && (s[i] == '+' || s[i] == '-')) ++i;
      if (i >= s.size() || !(s[i] >= '0' && s[i] <= '9')) fail("bad exponent");
      while (i < s.size() && s[i] >= '0' && s[i] <= '9') ++i;
    }
    return std::strtod(s.substr(b, i - b).c_str(), nullptr);
  }

  Value value(int depth) {
    if (depth > 256) fail("nesting too deep");
    ws();
    if (i >= s.size()) fail("unexpected end of input");
    Value v;
    char c = s[i];
    if (c == '{') {
      v.tag = Tag::Object;
      ++i;
      ws();
      if (i < s.size() && s[i] == '}') {
        ++i;
        return v;
      }
      while (true) {
        ws();
        if (i >= s.size()) fail("unexpected end of input");
        std::string k = str();
        ws();
        if (i >= s.size() || s[i] != ':') fail("expected ':'");
        ++i;
        v.object.emplace_back(std::move(k), value(depth + 1));
        ws();
        if (i < s.size() && s[i] == ',') {
          ++i;
          continue;
        }
        if (i < s.size() && s[i] == '}') {
          ++i;
          break;
        }
        fail("expected ',' or '}'");
      }
    } else if (c == '[') {
      v.tag = Tag::Array;
      ++i;
      ws();
      if (i < s.size() && s[i] == ']') {
        ++i;
        return v;
      }
      while (true) {
        v.array.push_back(value(depth + 1));
        ws();
        if (i < s.size() && s[i] == ',') {
          ++i;
          continue;
        }
        if (i < s.size() && s[i] == ']') {
          ++i;
          break;
        }
        fail("expected ',' or ']'");
      }
    } else if (c == '"') {
      v.tag = Tag::String;
      v.string = str();
    } else if (c == '-' || (c >= '0' && c <= '9')) {
      v.tag = Tag::Number;
      v.number = num();
    } else if (lit("true")) {
      v.tag = Tag::True;
    } else if (lit("false")) {
      v.tag = Tag::False;
    } else if (lit("null")) {
      v.tag = Tag::Null;
    } else {
      fail("unexpected character");
    }
    return v;
  }
};

}  // namespace

Value parse(const std::string& text) {
  Parser p(text);
  Value v = p.value(0);
  p.ws();
  if (p.i != text.size()) p.fail("trailing characters");
  return v;
}

Value parse_file(const std::string& path, Tag root) {
  if (path.size() > 250) throw IOException("Filepath is too long");
  std::ifstream f(path, std::ios::binary);
  if (!f.is_open()) throw IOException("File not found: " + path);
  std::stringstream ss;
  ss << f.rdbuf();
  Value v = parse(ss.str());
  if (v.tag != root) throw std::runtime_error("Expected root of JSON file had invalid type");
  return v;
}

bool try_read_float(const std::string& key, const Value& v, float& lhs, const char* want) {
  if (key != want || v.tag != Tag::Number) return false;
  lhs = static_cast<float>(v.number);
  return true;
}

bool try_read_uint(const std::string& key, const Value& v, size_t& lhs, const char* want) {
  if (key != want || v.tag != Tag::Number) return false;
  lhs = static_cast<size_t>(static_cast<unsigned int>(v.number));
  return true;
}

bool try_read_string(const std::string& key, const Value& v, std::string& lhs, const char* want) {
  if (key != want || v.tag != Tag::String) return false;
  lhs = v.string;
  return true;
}

bool try_read_vector(const std::string& key, const Value& v, std::vector<float>& lhs,
                     const char* want) {
  if (key != want || v.tag != Tag::Array) return false;
  for (auto& e : v.array) lhs.push_back(static_cast<float>(e.number));
  return true;
}

std::string format_float(float x) {
  if (std::isnan(x)) return "NaN";
  if (std::isinf(x)) return x > 0 ? "Infinity" : "-Infinity";
  char buf[48];
  for (int prec = 6; prec <= 9; ++prec) {
    std::snprintf(buf, sizeof(buf), "%.*g", prec, static_cast<double>(x));
    if (std::strtof(buf, nullptr) == x) break;
  }
  return buf;
}

}  // namespace json
}  // namespace srcnn
