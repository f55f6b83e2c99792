#pragma once

#include <cstdint>
#include <optional>
#include <string>
#include <string_view>
#include <vector>

namespace adp {

std::vector<std::string> Split(std::string_view s, char sep);
std::vector<std::string> SplitOn(std::string_view s, std::string_view sep);
std::string Trim(std::string_view s);
std::string Join(const std::vector<std::string>& parts, std::string_view sep);
std::string ToLower(std::string_view s);
bool StartsWith(std::string_view s, std::string_view p);
bool EndsWith(std::string_view s, std::string_view p);
std::optional<int64_t> ParseInt(std::string_view s);     // base 10, whole string
std::optional<uint64_t> ParseUint(std::string_view s);   // base 10, whole string, no sign
std::optional<bool> ParseBool(std::string_view s);       // true/false/1/0/yes/no/on/off
std::string JsonEscape(std::string_view s);
// path.Join-like: joins and collapses duplicate '/' ("/" + "/dev/kfd" -> "/dev/kfd").
std::string PathJoin(std::string_view a, std::string_view b);
std::string BaseName(std::string_view path);

}  // namespace adp
