#include "common/strings.h"

#include <cctype>
#include <cerrno>
#include <cstdio>
#include <cstdlib>

namespace adp {

std::vector<std::string> Split(std::string_view s, char sep) {
  std::vector<std::string> out;
  size_t start = 0;
  for (size_t i = 0; i <= s.size(); ++i) {
    if (i == s.size() || s[i] == sep) {
      out.emplace_back(s.substr(start, i - start));
      start = i + 1;
    }
  }
  return out;
}

std::vector<std::string> SplitOn(std::string_view s, std::string_view sep) {
  std::vector<std::string> out;
  if (sep.empty()) {
    out.emplace_back(s);
    return out;
  }
  size_t start = 0;
  while (true) {
    size_t p = s.find(sep, start);
    if (p == std::string_view::npos) {
      out.emplace_back(s.substr(start));
      return out;
    }
    out.emplace_back(s.substr(start, p - start));
    start = p + sep.size();
  }
}

std::string Trim(std::string_view s) {
  size_t b = 0, e = s.size();
  while (b < e && std::isspace(static_cast<unsigned char>(s[b]))) ++b;
  while (e > b && std::isspace(static_cast<unsigned char>(s[e - 1]))) --e;
  return std::string(s.substr(b, e - b));
}

std::string Join(const std::vector<std::string>& parts, std::string_view sep) {
  std::string out;
  size_t n = 0;
  for (const auto& p : parts) n += p.size() + sep.size();
  out.reserve(n);
  for (size_t i = 0; i < parts.size(); ++i) {
    if (i) out.append(sep);
    out.append(parts[i]);
  }
  return out;
}

std::string ToLower(std::string_view s) {
  std::string out(s);
  for (auto& c : out) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  return out;
}

bool StartsWith(std::string_view s, std::string_view p) { return s.substr(0, p.size()) == p; }
bool EndsWith(std::string_view s, std::string_view p) {
  return s.size() >= p.size() && s.substr(s.size() - p.size()) == p;
}

std::optional<int64_t> ParseInt(std::string_view s) {
  if (s.empty()) return std::nullopt;
  std::string tmp(s);
  errno = 0;
  char* end = nullptr;
  long long v = std::strtoll(tmp.c_str(), &end, 10);
  if (errno != 0 || end != tmp.c_str() + tmp.size()) return std::nullopt;
  if (std::isspace(static_cast<unsigned char>(tmp[0]))) return std::nullopt;
  return static_cast<int64_t>(v);
}

std::optional<uint64_t> ParseUint(std::string_view s) {
  if (s.empty()) return std::nullopt;
  for (char c : s)
    if (c < '0' || c > '9') return std::nullopt;
  std::string tmp(s);
  errno = 0;
  char* end = nullptr;
  unsigned long long v = std::strtoull(tmp.c_str(), &end, 10);
  if (errno != 0 || end != tmp.c_str() + tmp.size()) return std::nullopt;
  return static_cast<uint64_t>(v);
}

std::optional<bool> ParseBool(std::string_view s) {
  std::string l = ToLower(Trim(s));
  if (l == "true" || l == "1" || l == "yes" || l == "on" || l == "t") return true;
  if (l == "false" || l == "0" || l == "no" || l == "off" || l == "f") return false;
  return std::nullopt;
}

std::string JsonEscape(std::string_view s) {
  std::string out;
  out.reserve(s.size() + 2);
  for (char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      default:
        if (static_cast<unsigned char>(c) < 0x20) {
          char buf[8];
          snprintf(buf, sizeof(buf), "\\u%04x", c);
          out += buf;
        } else {
          out += c;
        }
    }
  }
  return out;
}

std::string PathJoin(std::string_view a, std::string_view b) {
  std::string joined(a);
  if (!joined.empty() && !b.empty()) joined += '/';
  joined.append(b);
  std::string out;
  out.reserve(joined.size());
  for (char c : joined) {
    if (c == '/' && !out.empty() && out.back() == '/') continue;
    out += c;
  }
  if (out.size() > 1 && out.back() == '/') out.pop_back();
  return out;
}

std::string BaseName(std::string_view path) {
  while (path.size() > 1 && path.back() == '/') path.remove_suffix(1);
  size_t p = path.rfind('/');
  if (p == std::string_view::npos) return std::string(path);
  return std::string(path.substr(p + 1));
}

}  // namespace adp
