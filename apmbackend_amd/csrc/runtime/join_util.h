// String helpers reproducing the reference parser's JS one-liners, shared by the host join
// (join.cpp) and the device join's host pre-pass (devjoin.cpp).  ASCII / UTF-8 semantics as in
// jsutil.h; each cites the reference expression it reproduces.
#pragma once
#include <algorithm>
#include <cctype>
#include <string>
#include <string_view>
#include <vector>

#include "jsutil.h"

namespace apm {
namespace jstr {

inline constexpr std::string_view kUndef("undefined");

inline bool all_digits(std::string_view s) {
  if (s.empty()) return false;
  for (char c : s) if (c < '0' || c > '9') return false;
  return true;
}

inline bool icontains(std::string_view hay, std::string_view needle) {
  if (needle.size() > hay.size()) return false;
  for (size_t i = 0; i + needle.size() <= hay.size(); ++i) {
    size_t k = 0;
    for (; k < needle.size(); ++k)
      if (std::tolower((unsigned char)hay[i + k]) != std::tolower((unsigned char)needle[k])) break;
    if (k == needle.size()) return true;
  }
  return false;
}

// .replace(/[[\]]/g, '') -- returns a view when there is nothing to strip except the common
// "[x]" wrapper, else copies into `scratch`.
inline std::string_view strip_brackets(std::string_view s, std::string& scratch) {
  size_t a = 0, b = s.size();
  if (a < b && s[a] == '[') ++a;
  if (b > a && s[b - 1] == ']') --b;
  bool inner = false;
  for (size_t i = a; i < b; ++i) inner |= (s[i] == '[' || s[i] == ']');
  if (!inner) return s.substr(a, b - a);
  scratch.clear();
  for (char c : s) if (c != '[' && c != ']') scratch.push_back(c);
  return scratch;
}

// service.replace(/Provider\[/i, 'Provider:').replace(']', '')
inline std::string normalize_service(std::string_view raw) {
  std::string s(raw);
  for (size_t i = 0; i + 9 <= s.size(); ++i) {
    static const char pat[] = "provider[";
    size_t k = 0;
    for (; k < 9; ++k) if (std::tolower((unsigned char)s[i + k]) != pat[k]) break;
    if (k == 9) { s.replace(i, 9, "Provider:"); break; }
  }
  size_t b = s.find(']');
  if (b != std::string::npos) s.erase(b, 1);
  return s;
}

// line.replace(/<\/.*/,'').replace(/.*>/,'')
inline std::string xml_inner(std::string_view line) {
  std::string_view s = line;
  size_t p = s.find("</");
  if (p != std::string_view::npos) s = s.substr(0, p);
  size_t q = s.rfind('>');
  if (q != std::string_view::npos) s = s.substr(q + 1);
  return std::string(s);
}

// split(/<|>/)[2] of trim(line)
inline std::string_view angle_field2(std::string_view line) {
  std::string_view t = js::trim(line);
  int field = 0;
  size_t start = 0;
  for (size_t i = 0; i <= t.size(); ++i) {
    if (i == t.size() || t[i] == '<' || t[i] == '>') {
      if (field == 2) return t.substr(start, i - start);
      ++field;
      start = i + 1;
    }
  }
  return std::string_view();
}

inline std::vector<std::string_view> info_segment_tokens(std::string_view line) {
  // line.split(/INFO/)[1].trim().split(/[\s]+/)
  size_t p1 = line.find("INFO");
  if (p1 == std::string_view::npos) return {std::string_view()};
  size_t p2 = line.find("INFO", p1 + 4);
  std::string_view seg = line.substr(p1 + 4, p2 == std::string_view::npos ? std::string_view::npos : p2 - p1 - 4);
  return js::split_ws(js::trim(seg));
}

inline bool baf_match(std::string_view line) {  // /\[[^ ]+] +INFO /
  for (size_t i = 1; i < line.size(); ++i) {
    if (line[i] != ']') continue;
    size_t j = i + 1;
    if (j >= line.size() || line[j] != ' ') continue;
    while (j < line.size() && line[j] == ' ') ++j;
    if (line.compare(j, 5, "INFO ") != 0) continue;
    for (size_t k = i; k-- > 0;) {
      if (line[k] == ' ') break;
      if (line[k] == '[' && k + 1 < i) return true;
    }
  }
  return false;
}

}  // namespace jstr
}  // namespace apm
