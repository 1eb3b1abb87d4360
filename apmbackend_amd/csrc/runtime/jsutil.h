// Host-side JavaScript semantics used by the join workers and the record formatters:
// parseInt / Number / Date construction / whitespace splitting / toFixed / String(number).
// Each function documents the ECMAScript rule it reproduces; the Python twins live in
// apmbackend_amd/utils/{jsfmt,timeparse}.py and both are tested against node.
#pragma once
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <string_view>
#include <vector>

#include "../kernels/common.h"

namespace apm {
namespace js {

inline double nan() { return std::nan(""); }

// JS \s for ASCII plus the UTF-8 encodings of the Unicode space separators JS recognises.
// Returns the byte length of the whitespace code point at p (0 if none).
inline int ws_len(const uint8_t* p, const uint8_t* end) {
  const uint8_t c = *p;
  if (c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f') return 1;
  if (c < 0x80) return 0;
  const ptrdiff_t n = end - p;
  if (c == 0xC2 && n >= 2 && p[1] == 0xA0) return 2;                        // U+00A0
  if (c == 0xE1 && n >= 3 && p[1] == 0x9A && p[2] == 0x80) return 3;        // U+1680
  if (c == 0xE2 && n >= 3) {
    if (p[1] == 0x80 && ((p[2] >= 0x80 && p[2] <= 0x8A) || p[2] == 0xA8 || p[2] == 0xA9 || p[2] == 0xAF))
      return 3;                                                               // U+2000-200A, 2028, 2029, 202F
    if (p[1] == 0x81 && p[2] == 0x9F) return 3;                               // U+205F
  }
  if (c == 0xE3 && n >= 3 && p[1] == 0x80 && p[2] == 0x80) return 3;        // U+3000
  if (c == 0xEF && n >= 3 && p[1] == 0xBB && p[2] == 0xBF) return 3;        // U+FEFF
  return 0;
}

// str.split(/[\s]+/)
inline std::vector<std::string_view> split_ws(std::string_view s, size_t max_tokens = 64) {
  std::vector<std::string_view> out;
  const uint8_t* p = (const uint8_t*)s.data();
  const uint8_t* e = p + s.size();
  const uint8_t* tok = p;
  bool in_ws = false;
  while (p < e) {
    int w = ws_len(p, e);
    if (w) {
      if (!in_ws) { out.emplace_back((const char*)tok, p - tok); in_ws = true; if (out.size() >= max_tokens) return out; }
      p += w;
      tok = p;
    } else {
      in_ws = false;
      ++p;
    }
  }
  out.emplace_back((const char*)tok, e - tok);
  return out;
}

inline std::string_view trim(std::string_view s) {
  const uint8_t* p = (const uint8_t*)s.data();
  const uint8_t* e = p + s.size();
  while (p < e) { int w = ws_len(p, e); if (!w) break; p += w; }
  // right trim, ASCII fast path: drop ASCII whitespace from the end; the first non-whitespace
  // ASCII byte ends the string.  A non-ASCII byte at the end (possibly the tail of a multi-byte
  // whitespace such as U+00A0 / U+FEFF) falls back to the exact forward walk over [p, e).
  while (e > p && e[-1] < 0x80) {
    if (ws_len(e - 1, e) == 0) return std::string_view((const char*)p, e - p);
    --e;
  }
  const uint8_t* q = p;
  const uint8_t* last = p;
  while (q < e) { int w = ws_len(q, e); if (w) q += w; else { ++q; last = q; } }
  return std::string_view((const char*)p, last - p);
}

// parseInt(s) with radix undefined.
inline double parse_int(std::string_view s) {
  const uint8_t* p = (const uint8_t*)s.data();
  const uint8_t* e = p + s.size();
  while (p < e) { int w = ws_len(p, e); if (!w) break; p += w; }
  bool neg = false;
  if (p < e && (*p == '+' || *p == '-')) { neg = *p == '-'; ++p; }
  int radix = 10;
  if (e - p >= 2 && p[0] == '0' && (p[1] == 'x' || p[1] == 'X')) { radix = 16; p += 2; }
  const uint8_t* d0 = p;
  double v = 0;
  std::string digits;
  while (p < e) {
    int dv;
    if (*p >= '0' && *p <= '9') dv = *p - '0';
    else if (radix == 16 && *p >= 'a' && *p <= 'f') dv = *p - 'a' + 10;
    else if (radix == 16 && *p >= 'A' && *p <= 'F') dv = *p - 'A' + 10;
    else break;
    digits.push_back((char)*p);
    ++p;
    (void)dv;
  }
  if (p == d0) return nan();
  if (radix == 10) {
    // correctly rounded conversion of the decimal digit string (matches JS for long inputs)
    v = std::strtod(digits.c_str(), nullptr);
  } else {
    for (char c : digits) v = v * 16 + (c <= '9' ? c - '0' : (c | 32) - 'a' + 10);
  }
  return neg ? -v : v;
}

// Number(s) for the simple decimal strings that reach new Date(...).
inline double number(std::string_view s) {
  std::string_view t = trim(s);
  if (t.empty()) return 0.0;
  std::string tmp(t);
  const char* c = tmp.c_str();
  char* endp = nullptr;
  if (tmp.size() > 2 && c[0] == '0' && (c[1] == 'x' || c[1] == 'X')) {
    unsigned long long v = std::strtoull(c + 2, &endp, 16);
    return (*endp == 0) ? (double)v : nan();
  }
  if (tmp == "Infinity" || tmp == "+Infinity") return INFINITY;
  if (tmp == "-Infinity") return -INFINITY;
  for (char ch : tmp)
    if (!((ch >= '0' && ch <= '9') || ch == '.' || ch == 'e' || ch == 'E' || ch == '+' || ch == '-')) return nan();
  double v = std::strtod(c, &endp);
  return (*endp == 0) ? v : nan();
}

struct Tz {
  TzTable table;
};

inline double make_date(double y, double mon0, double d, double h, double mi, double s, double ms) {
  const double vals[7] = {y, mon0, d, h, mi, s, ms};
  for (double v : vals) if (!std::isfinite(v)) return nan();
  int64_t yi = (int64_t)std::trunc(y);
  if (yi >= 0 && yi <= 99) yi += 1900;
  return (double)make_date_ms(yi, (int64_t)std::trunc(mon0), (int64_t)std::trunc(d), (int64_t)std::trunc(h),
                              (int64_t)std::trunc(mi), (int64_t)std::trunc(s), (int64_t)std::trunc(ms));
}

// ISO form used by audit trails: YYYY-MM-DDTHH:MM[:SS[.fff]][Z|+HH:MM]
inline double parse_iso(std::string_view s, const TzTable& tz) {
  std::string_view t = trim(s);
  auto dig = [&](size_t i, size_t n, int64_t& out) {
    if (i + n > t.size()) return false;
    int64_t v = 0;
    for (size_t k = 0; k < n; ++k) { char c = t[i + k]; if (c < '0' || c > '9') return false; v = v * 10 + (c - '0'); }
    out = v; return true;
  };
  int64_t y, mo, d, h, mi, sec = 0, ms = 0;
  if (!dig(0, 4, y) || t.size() < 16 || t[4] != '-' || !dig(5, 2, mo) || t[7] != '-' || !dig(8, 2, d) ||
      t[10] != 'T' || !dig(11, 2, h) || t[13] != ':' || !dig(14, 2, mi))
    return nan();
  size_t i = 16;
  if (i < t.size() && t[i] == ':') {
    if (!dig(i + 1, 2, sec)) return nan();
    i += 3;
    if (i < t.size() && t[i] == '.') {
      ++i;
      size_t j = i;
      int64_t frac = 0; int nd = 0;
      while (j < t.size() && t[j] >= '0' && t[j] <= '9') { if (nd < 3) { frac = frac * 10 + (t[j] - '0'); ++nd; } ++j; }
      if (j == i) return nan();
      while (nd < 3) { frac *= 10; ++nd; }
      ms = frac; i = j;
    }
  }
  if (mo < 1 || mo > 12 || d < 1 || d > 31 || h > 24 || mi > 59 || sec > 59) return nan();
  const int64_t local = make_date_ms(y, mo - 1, d, h, mi, sec, ms);
  if (i == t.size()) return (double)local_to_utc(tz, local);
  if (t[i] == 'Z' && i + 1 == t.size()) return (double)local;
  if (t[i] == '+' || t[i] == '-') {
    int sg = t[i] == '-' ? -1 : 1;
    int64_t oh, om;
    if (!dig(i + 1, 2, oh)) return nan();
    size_t k = i + 3;
    if (k < t.size() && t[k] == ':') ++k;
    if (!dig(k, 2, om) || k + 2 != t.size()) return nan();
    return (double)(local - sg * (oh * 60 + om) * 60000);
  }
  return nan();
}

// convertStringDateToMs: returns false for the '' result (empty / falsy input).
inline bool convert_date(std::string_view s, const TzTable& tz, double& out) {
  if (s.empty()) return false;
  // /T.*-/
  size_t tpos = s.find('T');
  if (tpos != std::string_view::npos && s.find('-', tpos + 1) != std::string_view::npos) {
    out = parse_iso(s, tz);
    return true;
  }
  // trim().split(/-|[\s]+|:|,/)
  std::string_view t = trim(s);
  std::vector<std::string_view> parts;
  const uint8_t* p = (const uint8_t*)t.data();
  const uint8_t* e = p + t.size();
  const uint8_t* tok = p;
  while (p < e) {
    int w = ws_len(p, e);
    if (w) { parts.emplace_back((const char*)tok, p - tok); p += w; while (p < e && (w = ws_len(p, e))) p += w; tok = p; continue; }
    if (*p == '-' || *p == ':' || *p == ',') { parts.emplace_back((const char*)tok, p - tok); ++p; tok = p; continue; }
    ++p;
  }
  parts.emplace_back((const char*)tok, e - tok);
  double v[7];
  for (int i = 0; i < 7; ++i) v[i] = i < (int)parts.size() ? number(parts[i]) : nan();
  const double local = make_date(v[0], v[1] - 1, v[2], v[3], v[4], v[5], v[6]);
  out = std::isnan(local) ? nan() : (double)local_to_utc(tz, (int64_t)local);
  return true;
}

// ---------------------------------------------------------------- formatting
// String(x) for a JS number (shortest round-trip digits, ECMAScript exponent rules).
inline std::string num_str(double x) {
  if (std::isnan(x)) return "NaN";
  if (std::isinf(x)) return x > 0 ? "Infinity" : "-Infinity";
  if (x == 0) return "0";
  char buf[64];
  auto r = std::to_chars(buf, buf + sizeof(buf), std::fabs(x), std::chars_format::scientific);
  *r.ptr = 0;
  // buf = d.ddddde[+-]XX
  std::string m(buf);
  size_t epos = m.find('e');
  int exp = std::atoi(m.c_str() + epos + 1);
  std::string digits;
  for (size_t i = 0; i < epos; ++i) if (m[i] != '.') digits.push_back(m[i]);
  while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
  const int k = (int)digits.size();
  const int n = exp + 1;
  std::string out = x < 0 ? "-" : "";
  if (k <= n && n <= 21) { out += digits; out.append(n - k, '0'); }
  else if (0 < n && n <= 21) { out += digits.substr(0, n); out += '.'; out += digits.substr(n); }
  else if (-6 < n && n <= 0) { out += "0."; out.append(-n, '0'); out += digits; }
  else {
    const int e = n - 1;
    out += digits[0];
    if (k > 1) { out += '.'; out += digits.substr(1); }
    out += 'e'; out += e >= 0 ? '+' : '-'; out += std::to_string(e >= 0 ? e : -e);
  }
  return out;
}

// Number.prototype.toFixed(f) (exact decision on the binary value, ties to the larger n).
inline std::string to_fixed(double x, int f) {
  if (std::isnan(x)) return "NaN";
  if (std::fabs(x) >= 1e21) return num_str(x);
  const bool neg = x < 0;
  // x87 long double (64-bit mantissa) holds |x| * 10^f exactly for f <= 3 (53 + 10 bits), so
  // the ECMA-262 rule "n/10^f - x closest to 0, ties to the larger n" is decided exactly.
  long double scale = 1;
  for (int i = 0; i < f; ++i) scale *= 10;
  const long double p = (long double)std::fabs(x) * scale;  // fabs: (-0).toFixed() is "0.0"
  const long double q = floorl(p);
  const long double n = (p - q) >= 0.5L ? q + 1 : q;
  char buf[64];
  snprintf(buf, sizeof(buf), "%.0Lf", n);
  std::string digits(buf);
  if (f > 0) {
    if ((int)digits.size() <= f) digits.insert(0, f + 1 - digits.size(), '0');
    digits.insert(digits.size() - f, ".");
  }
  return (neg ? "-" : "") + digits;
}

// Write String(x) at p (at most 32 bytes: JS number strings are <= 25 chars); returns the end.
// Decimal digits of v written at p (two digits per step from a 200-byte table); returns the end.
inline char* put_u64(char* p, uint64_t v) {
  static const char kPairs[201] =
      "00010203040506070809101112131415161718192021222324252627282930313233343536373839"
      "40414243444546474849505152535455565758596061626364656667686970717273747576777879"
      "8081828384858687888990919293949596979899";
  char tmp[24];
  char* e = tmp + sizeof(tmp);
  char* q = e;
  while (v >= 100) {
    const unsigned r = (unsigned)(v % 100);
    v /= 100;
    q -= 2;
    std::memcpy(q, kPairs + 2 * r, 2);
  }
  if (v >= 10) {
    q -= 2;
    std::memcpy(q, kPairs + 2 * v, 2);
  } else {
    *--q = (char)('0' + v);
  }
  const size_t n = (size_t)(e - q);
  std::memcpy(p, q, n);
  return p + n;
}

inline char* put_num(char* p, double x) {
  if (x == x && x == std::trunc(x) && std::fabs(x) < 9007199254740992.0 && !(x == 0 && std::signbit(x))) {
    if (x < 0) *p++ = '-';
    return put_u64(p, (uint64_t)std::fabs(x));
  }
  const std::string s = num_str(x);  // NaN, fractions, huge: rare
  const size_t n = std::min<size_t>(s.size(), 32);
  std::memcpy(p, s.data(), n);
  return p + n;
}

// Append String(x): integral values below 2^53 take a digit loop, everything else num_str.
inline void append_num(std::string& out, double x) {
  if (x == x && x == std::trunc(x) && std::fabs(x) < 9007199254740992.0 && !(x == 0 && std::signbit(x))) {
    char buf[24];
    int n = 0;
    uint64_t v = (uint64_t)std::fabs(x);
    do { buf[n++] = (char)('0' + v % 10); v /= 10; } while (v);
    if (x < 0) out += '-';
    while (n) out += buf[--n];
    return;
  }
  out += num_str(x);
}

// entries.js nf(): undefined for NaN, else toFixed.
inline std::string nf(double x, int f = 1) { return std::isnan(x) ? "undefined" : to_fixed(x, f); }

}  // namespace js
}  // namespace apm
