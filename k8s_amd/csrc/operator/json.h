// Minimal JSON value, parser and serializer for the TfJob control plane.
//
// Objects keep insertion order (the wire encoders below emit fields in the
// Go struct declaration order the reference uses, Appendix B of SURVEY.md),
// and lookups can be case-insensitive to mirror Go encoding/json decoding
// (`/root/reference/pkg/spec/tf_job.go` structs are decoded that way).
#pragma once

#include <cstdint>
#include <deque>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace tfop {

class Json;
using JsonArray = std::vector<Json>;
using JsonObject = std::deque<std::pair<std::string, Json>>;  // deque: references stay valid on insert

struct JsonError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

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
  Json(double v) : t_(Double), d_(v) {}
  Json(const char* s) : t_(String), s_(s) {}
  Json(std::string s) : t_(String), s_(std::move(s)) {}
  Json(JsonArray a) : t_(Array), a_(std::make_shared<JsonArray>(std::move(a))) {}
  Json(JsonObject o) : t_(Object), o_(std::make_shared<JsonObject>(std::move(o))) {}

  static Json array() { return Json(JsonArray{}); }
  static Json object() { return Json(JsonObject{}); }
  static Json parse(const std::string& text);

  Type type() const { return t_; }
  bool is_null() const { return t_ == Null; }
  bool is_bool() const { return t_ == Bool; }
  bool is_number() const { return t_ == Int || t_ == Double; }
  bool is_string() const { return t_ == String; }
  bool is_array() const { return t_ == Array; }
  bool is_object() const { return t_ == Object; }

  bool as_bool() const;
  int64_t as_int() const;
  double as_double() const;
  const std::string& as_string() const;
  const JsonArray& as_array() const;
  JsonArray& as_array();
  const JsonObject& as_object() const;
  JsonObject& as_object();

  // object access
  bool has(const std::string& k) const { return find(k) != nullptr; }
  const Json* find(const std::string& k) const;
  Json* find(const std::string& k);
  // Go-style case-insensitive field match (exact match preferred)
  const Json* find_ci(const std::string& k) const;
  Json& operator[](const std::string& k);  // inserts null if missing (object only; null becomes object)
  const Json& at(const std::string& k) const;
  void set(const std::string& k, Json v);
  bool erase(const std::string& k);

  // array access
  void push_back(Json v);
  size_t size() const;
  Json& operator[](size_t i);
  const Json& operator[](size_t i) const;

  std::string dump() const;            // compact
  std::string dump_pretty(int indent = 2) const;  // Go MarshalIndent style

  Json clone() const;  // deep copy (values share nested storage otherwise)
  bool operator==(const Json& o) const;
  bool operator!=(const Json& o) const { return !(*this == o); }

 private:
  void dump_to(std::string& out, int indent, int depth) const;
  Type t_;
  bool b_ = false;
  int64_t i_ = 0;
  double d_ = 0;
  std::string s_;
  std::shared_ptr<JsonArray> a_;
  std::shared_ptr<JsonObject> o_;
};

std::string json_quote(const std::string& s);

// helpers for optional fields
inline std::string get_str(const Json& o, const std::string& k, const std::string& def = "") {
  const Json* v = o.is_object() ? o.find_ci(k) : nullptr;
  return (v && v->is_string()) ? v->as_string() : def;
}

}  // namespace tfop
