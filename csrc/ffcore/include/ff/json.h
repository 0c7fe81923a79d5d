// Minimal JSON value type for the ffcore IR (graph file format, strategy
// files, rule corpora).  Value semantics, ordered object keys (std::map) so
// that serialisation is deterministic and usable as a hash/equality key.
//
// Parity: replaces the reference's nlohmann-json adapters used by every
// dtgen'd IR type (`lib/utils/include/utils/json/*`,
// `lib/pcg/include/pcg/file_format/v1/*`).
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <variant>
#include <vector>

namespace ff {

class Json {
 public:
  using Array = std::vector<Json>;
  using Object = std::map<std::string, Json>;
  enum class Kind { Null, Bool, Int, Double, String, Array, Object };

  Json() : v_(std::monostate{}) {}
  Json(std::nullptr_t) : v_(std::monostate{}) {}
  Json(bool b) : v_(b) {}
  Json(int i) : v_(static_cast<int64_t>(i)) {}
  Json(long i) : v_(static_cast<int64_t>(i)) {}
  Json(long long i) : v_(static_cast<int64_t>(i)) {}
  Json(unsigned i) : v_(static_cast<int64_t>(i)) {}
  Json(unsigned long i) : v_(static_cast<int64_t>(i)) {}
  Json(unsigned long long i) : v_(static_cast<int64_t>(i)) {}
  Json(double d) : v_(d) {}
  Json(float d) : v_(static_cast<double>(d)) {}
  Json(const char* s) : v_(std::string(s)) {}
  Json(std::string s) : v_(std::move(s)) {}
  Json(Array a) : v_(std::make_shared<Array>(std::move(a))) {}
  Json(Object o) : v_(std::make_shared<Object>(std::move(o))) {}
  template <typename T>
  Json(const std::vector<T>& xs) : v_(std::make_shared<Array>()) {
    auto& a = *std::get<std::shared_ptr<Array>>(v_);
    for (auto const& x : xs) a.push_back(Json(x));
  }

  static Json object() { return Json(Object{}); }
  static Json array() { return Json(Array{}); }

  Kind kind() const {
    switch (v_.index()) {
      case 0: return Kind::Null;
      case 1: return Kind::Bool;
      case 2: return Kind::Int;
      case 3: return Kind::Double;
      case 4: return Kind::String;
      case 5: return Kind::Array;
      default: return Kind::Object;
    }
  }
  bool is_null() const { return kind() == Kind::Null; }
  bool is_bool() const { return kind() == Kind::Bool; }
  bool is_int() const { return kind() == Kind::Int; }
  bool is_number() const { return kind() == Kind::Int || kind() == Kind::Double; }
  bool is_string() const { return kind() == Kind::String; }
  bool is_array() const { return kind() == Kind::Array; }
  bool is_object() const { return kind() == Kind::Object; }

  bool as_bool() const {
    if (is_bool()) return std::get<bool>(v_);
    if (is_int()) return std::get<int64_t>(v_) != 0;
    throw std::runtime_error("json: not a bool");
  }
  int64_t as_int() const {
    if (is_int()) return std::get<int64_t>(v_);
    if (kind() == Kind::Double) return static_cast<int64_t>(std::get<double>(v_));
    if (is_bool()) return std::get<bool>(v_) ? 1 : 0;
    throw std::runtime_error("json: not an int");
  }
  double as_double() const {
    if (kind() == Kind::Double) return std::get<double>(v_);
    if (is_int()) return static_cast<double>(std::get<int64_t>(v_));
    throw std::runtime_error("json: not a number");
  }
  const std::string& as_string() const {
    if (!is_string()) throw std::runtime_error("json: not a string");
    return std::get<std::string>(v_);
  }
  const Array& as_array() const {
    if (!is_array()) throw std::runtime_error("json: not an array");
    return *std::get<std::shared_ptr<Array>>(v_);
  }
  Array& as_array() {
    if (!is_array()) throw std::runtime_error("json: not an array");
    detach();
    return *std::get<std::shared_ptr<Array>>(v_);
  }
  const Object& as_object() const {
    if (!is_object()) throw std::runtime_error("json: not an object");
    return *std::get<std::shared_ptr<Object>>(v_);
  }
  Object& as_object() {
    if (!is_object()) throw std::runtime_error("json: not an object");
    detach();
    return *std::get<std::shared_ptr<Object>>(v_);
  }

  // object access
  Json& operator[](const std::string& k) {
    if (is_null()) *this = object();
    return as_object()[k];
  }
  const Json& at(const std::string& k) const {
    auto const& o = as_object();
    auto it = o.find(k);
    if (it == o.end()) throw std::runtime_error("json: missing key '" + k + "'");
    return it->second;
  }
  bool contains(const std::string& k) const {
    return is_object() && as_object().count(k) > 0;
  }
  const Json& at(size_t i) const { return as_array().at(i); }
  size_t size() const {
    if (is_array()) return as_array().size();
    if (is_object()) return as_object().size();
    return 0;
  }
  void push_back(Json j) {
    if (is_null()) *this = array();
    as_array().push_back(std::move(j));
  }

  std::vector<int64_t> as_int_vector() const {
    std::vector<int64_t> r;
    for (auto const& x : as_array()) r.push_back(x.as_int());
    return r;
  }

  std::string dump(int indent = -1) const;
  static Json parse(const std::string& s);

  bool operator==(const Json& o) const;
  bool operator!=(const Json& o) const { return !(*this == o); }
  bool operator<(const Json& o) const { return dump() < o.dump(); }

 private:
  void detach() {
    // copy-on-write so that Json has value semantics
    if (auto p = std::get_if<std::shared_ptr<Array>>(&v_)) {
      if (p->use_count() > 1) *p = std::make_shared<Array>(**p);
    } else if (auto q = std::get_if<std::shared_ptr<Object>>(&v_)) {
      if (q->use_count() > 1) *q = std::make_shared<Object>(**q);
    }
  }
  void dump_to(std::string& out, int indent, int depth) const;
  std::variant<std::monostate, bool, int64_t, double, std::string,
               std::shared_ptr<Array>, std::shared_ptr<Object>>
      v_;
};

}  // namespace ff
