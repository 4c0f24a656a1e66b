#include "json.h"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <sstream>

namespace tfop {

namespace {

struct Parser {
  const std::string& s;
  size_t i = 0;
  explicit Parser(const std::string& t) : s(t) {}

  [[noreturn]] void fail(const char* msg) {
    throw JsonError(std::string("json parse error at offset ") + std::to_string(i) + ": " + msg);
  }
  void ws() {
    while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) ++i;
  }
  bool lit(const char* w) {
    size_t n = strlen(w);
    if (s.compare(i, n, w) == 0) {
      i += n;
      return true;
    }
    return false;
  }
  static void utf8(std::string& out, uint32_t cp) {
    if (cp < 0x80) {
      out += (char)cp;
    } else if (cp < 0x800) {
      out += (char)(0xC0 | (cp >> 6));
      out += (char)(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
      out += (char)(0xE0 | (cp >> 12));
      out += (char)(0x80 | ((cp >> 6) & 0x3F));
      out += (char)(0x80 | (cp & 0x3F));
    } else {
      out += (char)(0xF0 | (cp >> 18));
      out += (char)(0x80 | ((cp >> 12) & 0x3F));
      out += (char)(0x80 | ((cp >> 6) & 0x3F));
      out += (char)(0x80 | (cp & 0x3F));
    }
  }
  uint32_t hex4() {
    if (i + 4 > s.size()) fail("short \\u escape");
    uint32_t v = 0;
    for (int k = 0; k < 4; ++k) {
      char c = s[i++];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else fail("bad hex digit");
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
      if (c == '\\') {
        if (i >= s.size()) fail("bad escape");
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
            uint32_t cp = hex4();
            if (cp >= 0xD800 && cp < 0xDC00 && i + 6 <= s.size() && s[i] == '\\' && s[i + 1] == 'u') {
              i += 2;
              uint32_t lo = hex4();
              cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            }
            utf8(out, cp);
            break;
          }
          default: fail("bad escape");
        }
      } else {
        out += c;
      }
    }
    return out;
  }
  Json value() {
    ws();
    if (i >= s.size()) fail("unexpected end");
    char c = s[i];
    if (c == '{') {
      ++i;
      Json o = Json::object();
      ws();
      if (i < s.size() && s[i] == '}') {
        ++i;
        return o;
      }
      while (true) {
        ws();
        std::string k = str();
        ws();
        if (i >= s.size() || s[i] != ':') fail("expected ':'");
        ++i;
        o.as_object().emplace_back(std::move(k), value());
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
      return o;
    }
    if (c == '[') {
      ++i;
      Json a = Json::array();
      ws();
      if (i < s.size() && s[i] == ']') {
        ++i;
        return a;
      }
      while (true) {
        a.push_back(value());
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
      return a;
    }
    if (c == '"') return Json(str());
    if (lit("true")) return Json(true);
    if (lit("false")) return Json(false);
    if (lit("null")) return Json();
    size_t st = i;
    bool is_float = false;
    if (s[i] == '-') ++i;
    while (i < s.size() && (isdigit((unsigned char)s[i]) || s[i] == '.' || s[i] == 'e' || s[i] == 'E' ||
                            s[i] == '+' || s[i] == '-')) {
      if (s[i] == '.' || s[i] == 'e' || s[i] == 'E') is_float = true;
      ++i;
    }
    if (st == i) fail("unexpected character");
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

bool ieq(const std::string& a, const std::string& b) {
  if (a.size() != b.size()) return false;
  for (size_t k = 0; k < a.size(); ++k)
    if (tolower((unsigned char)a[k]) != tolower((unsigned char)b[k])) return false;
  return true;
}

}  // namespace

Json Json::parse(const std::string& text) {
  Parser p(text);
  Json v = p.value();
  p.ws();
  if (p.i != text.size()) p.fail("trailing characters");
  return v;
}

bool Json::as_bool() const {
  if (t_ != Bool) throw JsonError("not a bool");
  return b_;
}
int64_t Json::as_int() const {
  if (t_ == Int) return i_;
  if (t_ == Double) return (int64_t)d_;
  throw JsonError("not a number");
}
double Json::as_double() const {
  if (t_ == Double) return d_;
  if (t_ == Int) return (double)i_;
  throw JsonError("not a number");
}
const std::string& Json::as_string() const {
  if (t_ != String) throw JsonError("not a string");
  return s_;
}
const JsonArray& Json::as_array() const {
  if (t_ != Array) throw JsonError("not an array");
  return *a_;
}
JsonArray& Json::as_array() {
  if (t_ != Array) throw JsonError("not an array");
  return *a_;
}
const JsonObject& Json::as_object() const {
  if (t_ != Object) throw JsonError("not an object");
  return *o_;
}
JsonObject& Json::as_object() {
  if (t_ != Object) throw JsonError("not an object");
  return *o_;
}

const Json* Json::find(const std::string& k) const {
  if (t_ != Object) return nullptr;
  for (auto& kv : *o_)
    if (kv.first == k) return &kv.second;
  return nullptr;
}
Json* Json::find(const std::string& k) {
  if (t_ != Object) return nullptr;
  for (auto& kv : *o_)
    if (kv.first == k) return &kv.second;
  return nullptr;
}
const Json* Json::find_ci(const std::string& k) const {
  if (t_ != Object) return nullptr;
  if (const Json* v = find(k)) return v;
  for (auto& kv : *o_)
    if (ieq(kv.first, k)) return &kv.second;
  return nullptr;
}
Json& Json::operator[](const std::string& k) {
  if (t_ == Null) *this = object();
  if (Json* v = find(k)) return *v;
  o_->emplace_back(k, Json());
  return o_->back().second;
}
const Json& Json::at(const std::string& k) const {
  const Json* v = find(k);
  if (!v) throw JsonError("missing key " + k);
  return *v;
}
void Json::set(const std::string& k, Json v) { (*this)[k] = std::move(v); }
bool Json::erase(const std::string& k) {
  if (t_ != Object) return false;
  for (auto it = o_->begin(); it != o_->end(); ++it)
    if (it->first == k) {
      o_->erase(it);
      return true;
    }
  return false;
}
void Json::push_back(Json v) {
  if (t_ == Null) *this = array();
  as_array().push_back(std::move(v));
}
size_t Json::size() const {
  if (t_ == Array) return a_->size();
  if (t_ == Object) return o_->size();
  return 0;
}
Json& Json::operator[](size_t i) { return as_array().at(i); }
const Json& Json::operator[](size_t i) const { return as_array().at(i); }

std::string json_quote(const std::string& s) {
  std::string out = "\"";
  for (unsigned char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      // Go's encoding/json HTML-escapes these
      case '<': out += "\\u003c"; break;
      case '>': out += "\\u003e"; break;
      case '&': out += "\\u0026"; break;
      default:
        if (c < 0x20) {
          char buf[8];
          snprintf(buf, sizeof buf, "\\u%04x", c);
          out += buf;
        } else {
          out += (char)c;
        }
    }
  }
  out += '"';
  return out;
}

void Json::dump_to(std::string& out, int indent, int depth) const {
  auto nl = [&](int d) {
    if (indent > 0) {
      out += '\n';
      out.append((size_t)(indent * d), ' ');
    }
  };
  switch (t_) {
    case Null: out += "null"; break;
    case Bool: out += b_ ? "true" : "false"; break;
    case Int: out += std::to_string(i_); break;
    case Double: {
      if (std::isfinite(d_) && d_ == std::floor(d_) && std::fabs(d_) < 1e15) {
        out += std::to_string((long long)d_);
      } else {
        char buf[32];
        snprintf(buf, sizeof buf, "%.17g", d_);
        out += buf;
      }
      break;
    }
    case String: out += json_quote(s_); break;
    case Array: {
      if (a_->empty()) {
        out += "[]";
        break;
      }
      out += '[';
      for (size_t k = 0; k < a_->size(); ++k) {
        if (k) out += ',';
        nl(depth + 1);
        (*a_)[k].dump_to(out, indent, depth + 1);
      }
      nl(depth);
      out += ']';
      break;
    }
    case Object: {
      if (o_->empty()) {
        out += "{}";
        break;
      }
      out += '{';
      for (size_t k = 0; k < o_->size(); ++k) {
        if (k) out += ',';
        nl(depth + 1);
        out += json_quote((*o_)[k].first);
        out += indent > 0 ? ": " : ":";
        (*o_)[k].second.dump_to(out, indent, depth + 1);
      }
      nl(depth);
      out += '}';
      break;
    }
  }
}

std::string Json::dump() const {
  std::string out;
  dump_to(out, 0, 0);
  return out;
}
std::string Json::dump_pretty(int indent) const {
  std::string out;
  dump_to(out, indent, 0);
  return out;
}

Json Json::clone() const {
  switch (t_) {
    case Array: {
      JsonArray a;
      for (auto& v : *a_) a.push_back(v.clone());
      return Json(std::move(a));
    }
    case Object: {
      JsonObject o;
      for (auto& kv : *o_) o.emplace_back(kv.first, kv.second.clone());
      return Json(std::move(o));
    }
    default: return *this;
  }
}

bool Json::operator==(const Json& o) const {
  if (is_number() && o.is_number()) return as_double() == o.as_double();
  if (t_ != o.t_) return false;
  switch (t_) {
    case Null: return true;
    case Bool: return b_ == o.b_;
    case String: return s_ == o.s_;
    case Array: {
      if (a_->size() != o.a_->size()) return false;
      for (size_t k = 0; k < a_->size(); ++k)
        if ((*a_)[k] != (*o.a_)[k]) return false;
      return true;
    }
    case Object: {
      // order-insensitive object equality
      if (o_->size() != o.o_->size()) return false;
      for (auto& kv : *o_) {
        const Json* v = o.find(kv.first);
        if (!v || *v != kv.second) return false;
      }
      return true;
    }
    default: return false;
  }
}

}  // namespace tfop
