#include "ff/json.h"

#include <cstdlib>

#include <cmath>
#include <cstdio>
#include <sstream>

namespace ff {

static void escape_into(std::string& out, const std::string& s) {
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
          std::snprintf(buf, sizeof buf, "\\u%04x", c);
          out += buf;
        } else {
          out.push_back(static_cast<char>(c));
        }
    }
  }
  out.push_back('"');
}

void Json::dump_to(std::string& out, int indent, int depth) const {
  auto nl = [&](int d) {
    if (indent >= 0) {
      out.push_back('\n');
      out.append(static_cast<size_t>(indent * d), ' ');
    }
  };
  switch (kind()) {
    case Kind::Null: out += "null"; break;
    case Kind::Bool: out += std::get<bool>(v_) ? "true" : "false"; break;
    case Kind::Int: out += std::to_string(std::get<int64_t>(v_)); break;
    case Kind::Double: {
      double d = std::get<double>(v_);
      if (!std::isfinite(d)) {
        out += (std::isnan(d) ? "NaN" : (d > 0 ? "Infinity" : "-Infinity"));
        break;
      }
      char buf[40];
      std::snprintf(buf, sizeof buf, "%.17g", d);
      std::string s(buf);
      if (s.find_first_of(".eE") == std::string::npos) s += ".0";
      out += s;
      break;
    }
    case Kind::String: escape_into(out, std::get<std::string>(v_)); break;
    case Kind::Array: {
      auto const& a = as_array();
      out.push_back('[');
      for (size_t i = 0; i < a.size(); ++i) {
        if (i) out.push_back(',');
        nl(depth + 1);
        a[i].dump_to(out, indent, depth + 1);
      }
      if (!a.empty()) nl(depth);
      out.push_back(']');
      break;
    }
    case Kind::Object: {
      auto const& o = as_object();
      out.push_back('{');
      bool first = true;
      for (auto const& kv : o) {
        if (!first) out.push_back(',');
        first = false;
        nl(depth + 1);
        escape_into(out, kv.first);
        out += indent >= 0 ? ": " : ":";
        kv.second.dump_to(out, indent, depth + 1);
      }
      if (!o.empty()) nl(depth);
      out.push_back('}');
      break;
    }
  }
}

std::string Json::dump(int indent) const {
  std::string out;
  dump_to(out, indent, 0);
  return out;
}

bool Json::operator==(const Json& o) const {
  if (kind() != o.kind()) {
    if (is_number() && o.is_number()) return as_double() == o.as_double();
    return false;
  }
  switch (kind()) {
    case Kind::Null: return true;
    case Kind::Bool: return std::get<bool>(v_) == std::get<bool>(o.v_);
    case Kind::Int: return std::get<int64_t>(v_) == std::get<int64_t>(o.v_);
    case Kind::Double: return std::get<double>(v_) == std::get<double>(o.v_);
    case Kind::String: return std::get<std::string>(v_) == std::get<std::string>(o.v_);
    case Kind::Array: return as_array() == o.as_array();
    case Kind::Object: return as_object() == o.as_object();
  }
  return false;
}

namespace {
struct Parser {
  const std::string& s;
  size_t i = 0;
  explicit Parser(const std::string& str) : s(str) {}

  [[noreturn]] void fail(const std::string& msg) {
    throw std::runtime_error("json parse error at " + std::to_string(i) + ": " + msg);
  }
  void ws() {
    while (i < s.size() && (s[i] == ' ' || s[i] == '\n' || s[i] == '\t' || s[i] == '\r')) ++i;
  }
  bool consume(const char* lit) {
    size_t n = std::char_traits<char>::length(lit);
    if (s.compare(i, n, lit) == 0) {
      i += n;
      return true;
    }
    return false;
  }
  static void put_utf8(std::string& out, uint32_t cp) {
    if (cp < 0x80) {
      out.push_back(static_cast<char>(cp));
    } else if (cp < 0x800) {
      out.push_back(static_cast<char>(0xC0 | (cp >> 6)));
      out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
      out.push_back(static_cast<char>(0xE0 | (cp >> 12)));
      out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
      out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    } else {
      out.push_back(static_cast<char>(0xF0 | (cp >> 18)));
      out.push_back(static_cast<char>(0x80 | ((cp >> 12) & 0x3F)));
      out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
      out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    }
  }
  std::string str() {
    if (s[i] != '"') fail("expected string");
    ++i;
    std::string out;
    while (i < s.size() && s[i] != '"') {
      char c = s[i++];
      if (c == '\\') {
        if (i >= s.size()) fail("bad escape");
        char e = s[i++];
        switch (e) {
          case 'n': out.push_back('\n'); break;
          case 't': out.push_back('\t'); break;
          case 'r': out.push_back('\r'); break;
          case 'b': out.push_back('\b'); break;
          case 'f': out.push_back('\f'); break;
          case 'u': {
            if (i + 4 > s.size()) fail("bad \\u");
            uint32_t cp = static_cast<uint32_t>(std::stoul(s.substr(i, 4), nullptr, 16));
            i += 4;
            if (cp >= 0xD800 && cp < 0xDC00 && i + 6 <= s.size() && s[i] == '\\' && s[i + 1] == 'u') {
              uint32_t lo = static_cast<uint32_t>(std::stoul(s.substr(i + 2, 4), nullptr, 16));
              i += 6;
              cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            }
            put_utf8(out, cp);
            break;
          }
          default: out.push_back(e);
        }
      } else {
        out.push_back(c);
      }
    }
    if (i >= s.size()) fail("unterminated string");
    ++i;
    return out;
  }
  Json value() {
    ws();
    if (i >= s.size()) fail("unexpected end");
    char c = s[i];
    if (c == '{') {
      ++i;
      Json::Object o;
      ws();
      if (s[i] == '}') {
        ++i;
        return Json(std::move(o));
      }
      while (true) {
        ws();
        std::string k = str();
        ws();
        if (s[i] != ':') fail("expected ':'");
        ++i;
        o[k] = value();
        ws();
        if (s[i] == ',') {
          ++i;
          continue;
        }
        if (s[i] == '}') {
          ++i;
          break;
        }
        fail("expected ',' or '}'");
      }
      return Json(std::move(o));
    }
    if (c == '[') {
      ++i;
      Json::Array a;
      ws();
      if (s[i] == ']') {
        ++i;
        return Json(std::move(a));
      }
      while (true) {
        a.push_back(value());
        ws();
        if (s[i] == ',') {
          ++i;
          continue;
        }
        if (s[i] == ']') {
          ++i;
          break;
        }
        fail("expected ',' or ']'");
      }
      return Json(std::move(a));
    }
    if (c == '"') return Json(str());
    if (consume("true")) return Json(true);
    if (consume("false")) return Json(false);
    if (consume("null")) return Json();
    if (consume("NaN")) return Json(std::nan(""));
    if (consume("Infinity")) return Json(HUGE_VAL);
    if (consume("-Infinity")) return Json(-HUGE_VAL);
    size_t start = i;
    bool is_float = false;
    if (s[i] == '-' || s[i] == '+') ++i;
    while (i < s.size()) {
      char d = s[i];
      if (d >= '0' && d <= '9') {
        ++i;
      } else if (d == '.' || d == 'e' || d == 'E' || d == '-' || d == '+') {
        is_float = true;
        ++i;
      } else {
        break;
      }
    }
    if (start == i) fail("unexpected character");
    std::string num = s.substr(start, i - start);
    // strtod, not std::stod: a subnormal (e.g. 4.9e-324, which to_json writes
    // for such doubles) sets ERANGE and std::stod throws; strtod returns it
    if (is_float) {
      char* end = nullptr;
      const double v = std::strtod(num.c_str(), &end);
      if (end == num.c_str()) fail("bad number");
      return Json(v);
    }
    return Json(static_cast<long long>(std::stoll(num)));
  }
};
}  // namespace

Json Json::parse(const std::string& s) {
  Parser p(s);
  Json v = p.value();
  p.ws();
  if (p.i != s.size()) p.fail("trailing characters");
  return v;
}

}  // namespace ff
