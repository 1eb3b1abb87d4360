// Device helpers of the GPU join (devjoin.hip): JS number formatting for tx lines, BAF / SOAP
// account field extraction, and the open-addressing tables.  Host-callable twins of the
// formatting helpers are used by tests (bindings: gpu_num_str) to check them against
// js::num_str, which is itself checked against node.
#pragma once
#include "common.h"
#include "devjoin_types.h"

namespace apm {
namespace dj {

// join key of a logId on one JVM: skey = world-invariant key of the server (server_key_of)
__host__ __device__ inline uint64_t gkey_of(uint64_t lid_hash, uint64_t skey) {
  const uint64_t k = hash_mix(lid_hash ^ (skey * 0x9E3779B97F4A7C15ULL), 0xd6e8feb86659fd93ULL);
  return k ? k : 1;
}
// world-invariant keys of a server name / a log file path (the engine's ids are per rank)
__host__ __device__ inline uint64_t server_key_of(const char* name, size_t n) {
  return hash_bytes(name, n, 0x5e7e7e7e5e7e7e7eULL) | 1ULL;
}
__host__ __device__ inline uint64_t file_key_of(const char* path, size_t n) {
  return hash_bytes(path, n, 0xf11ef11ef11ef11eULL) | 1ULL;
}
__host__ __device__ inline uint64_t regkey_of(uint64_t svc, int32_t server) {
  const uint64_t k = hash_mix(svc ^ ((uint64_t)(uint32_t)(server + 7) * 0xC2B2AE3D27D4EB4FULL), 0x165667b19e3779f9ULL);
  return k ? k : 1;
}
// audit-trail map key: (file key, hash(auditTrailId)), never 0
__host__ __device__ inline uint64_t aud_key(uint64_t autr_hash, uint64_t fkey) {
  return hash_mix(autr_hash, 0x9e3779b97f4a7c15ULL + fkey) | 1ULL;
}
__host__ __device__ inline uint32_t home_of(uint64_t k, uint32_t mask) {
  return (uint32_t)((k * 0x9E3779B97F4A7C15ULL) >> 32) & mask;
}

// ------------------------------------------------------------------ JS String(number)
// String(x) for the values a tx line holds: parseInt / trunc results (integral), NaN, +-Inf.
// Integral |x| < 2^54: every integer there is representable with gaps <= 2, so the shortest
// round-trip digits are the integer's own digits.  Larger integral values (< 2^127): the
// ECMAScript rule (fewest digits n, then closest to x, then even) is decided exactly with
// 128-bit integers against the rounding interval of x.  Returns the length; `inexact` is set
// for values outside that domain (|x| >= 2^127 or fractional), printed with 17 digits.
__host__ __device__ inline int put_dec(char* p, unsigned __int128 v) {
  char t[48];
  int n = 0;
  do { t[n++] = (char)('0' + (int)(v % 10)); v /= 10; } while (v);
  for (int i = 0; i < n; ++i) p[i] = t[n - 1 - i];
  return n;
}

__host__ __device__ inline int u64_digits(uint64_t v) {
  int n = 1;
  uint64_t p = 10;
  while (n < 20 && v >= p) { ++n; p *= 10; }
  return n;
}

// n decimal digits of v at p (64-bit constant divisions: multiply-high, no 128-bit arithmetic)
__host__ __device__ inline void u64_write(char* p, uint64_t v, int n) {
  for (int i = n - 1; i >= 0; --i) { p[i] = (char)('0' + (int)(v % 10)); v /= 10; }
}

__host__ __device__ inline int js_num(char* p, double x, bool* inexact) {
  // p == nullptr: length only
  if (x != x) { if (p) { p[0] = 'N'; p[1] = 'a'; p[2] = 'N'; } return 3; }
  const bool neg = x < 0;
  const double ax = neg ? -x : x;
  if (ax < 18014398509481984.0 && ax == floor(ax)) {  // integral, < 2^54: the common case
    if (ax == 0) { if (p) p[0] = '0'; return 1; }    // -0 prints "0"
    const uint64_t v = (uint64_t)ax;
    const int nd = u64_digits(v);
    if (p) {
      if (neg) p[0] = '-';
      u64_write(p + (neg ? 1 : 0), v, nd);
    }
    return nd + (neg ? 1 : 0);
  }
  char buf[64];
  char* o = p ? p : buf;
  int n = 0;
  if (neg) { o[n++] = '-'; x = ax; }
  if (x == __builtin_inf()) {
    const char* s = "Infinity";
    for (int i = 0; i < 8; ++i) o[n + i] = s[i];
    return n + 8;
  }
  if (x < 1.7014118346046923e38 && x == floor(x)) {  // < 2^127
    int e2;
    const double fr = frexp(x, &e2);  // x = fr * 2^e2, fr in [0.5, 1)
    (void)fr;
    const unsigned __int128 M = (unsigned __int128)x;
    const int sh = e2 - 53;  // ulp = 2^sh (>= 2 here)
    const unsigned __int128 ulp = (unsigned __int128)1 << sh;
    const bool pow2 = (M & (M - 1)) == 0;
    const unsigned __int128 hi = ulp >> 1;
    const unsigned __int128 lo = pow2 ? (ulp >> 2) : (ulp >> 1);
    const bool even = ((M >> sh) & 1) == 0;  // significand parity: boundary values round to x
    auto inside = [&](unsigned __int128 c) {
      if (c >= M) { const unsigned __int128 d = c - M; return d < hi || (d == hi && even); }
      const unsigned __int128 d = M - c;
      return d < lo || (d == lo && even);
    };
    unsigned __int128 best = M, p10 = 1;
    for (int k = 1; k < 39; ++k) {
      const unsigned __int128 q = p10 * 10;
      if (q > M) break;
      const unsigned __int128 down = M - M % q, up = down + q;
      const bool di = inside(down), ui = inside(up);
      // any multiple of 10^k inside the (convex) interval makes the nearer of down / up fit, and
      // multiples of 10^(k+1) are multiples of 10^k: the first miss ends the search
      if (!di && !ui) break;
      unsigned __int128 c;
      if (di && ui) {
        const unsigned __int128 dd = M - down, du = up - M;
        c = dd < du ? down : (du < dd ? up : (((down / q) & 1) == 0 ? down : up));
      } else {
        c = di ? down : up;
      }
      best = c;
      p10 = q;
    }
    // digits of `best` with trailing zeros dropped; exponent form from 1e21 (ECMAScript)
    char d[48];
    int nd = put_dec(d, best);
    int tz = 0;
    while (nd - tz > 1 && d[nd - 1 - tz] == '0') ++tz;
    const int exp10 = nd - 1;  // x = d.ddd * 10^exp10
    if (exp10 < 21) {
      for (int i = 0; i < nd; ++i) o[n + i] = d[i];
      return n + nd;
    }
    const int k = nd - tz;
    o[n++] = d[0];
    if (k > 1) { o[n++] = '.'; for (int i = 1; i < k; ++i) o[n++] = d[i]; }
    o[n++] = 'e'; o[n++] = '+';
    n += put_dec(o + n, (unsigned __int128)exp10);
    return n;
  }
  // outside the tx-line domain: 17 significant digits (not guaranteed shortest)
  if (inexact) *inexact = true;
  int e10 = 0;
  double y = x;
  while (y >= 10.0) { y /= 10.0; ++e10; }
  while (y < 1.0) { y *= 10.0; --e10; }
  uint64_t m = (uint64_t)(y * 1e16 + 0.5);
  if (m >= 100000000000000000ULL) { m /= 10; ++e10; }
  char d[24];
  int nd = put_dec(d, m);
  while (nd > 1 && d[nd - 1] == '0') --nd;
  o[n++] = d[0];
  if (nd > 1) { o[n++] = '.'; for (int i = 1; i < nd; ++i) o[n++] = d[i]; }
  o[n++] = 'e';
  o[n++] = e10 >= 0 ? '+' : '-';
  n += put_dec(o + n, (unsigned __int128)(e10 >= 0 ? e10 : -e10));
  return n;
}

// ------------------------------------------------------------------ account strings
// parseInt(s) for a whitespace-free ASCII token.  Returns false when the host must decide
// (sign / hex prefix / more than 19 digits); else `out` = value (NaN when no digits).
__host__ __device__ inline bool simple_parse_int(const uint8_t* s, int n, double& out) {
  if (n > 0 && (s[0] == '+' || s[0] == '-')) return false;
  if (n >= 2 && s[0] == '0' && (s[1] == 'x' || s[1] == 'X')) return false;
  uint64_t v = 0;
  int nd = 0;
  while (nd < n && s[nd] >= '0' && s[nd] <= '9') {
    if (nd >= 19) return false;
    v = v * 10 + (uint64_t)(s[nd] - '0');
    ++nd;
  }
  out = nd == 0 ? __builtin_nan("") : (double)v;  // u64 -> double: correctly rounded
  return true;
}

__host__ __device__ inline bool all_digits(const uint8_t* s, int n) {
  if (n <= 0) return false;
  for (int i = 0; i < n; ++i)
    if (s[i] < '0' || s[i] > '9') return false;
  return true;
}

// attemptReadAccountNumberFromBAFInfo (:486-497) on token 3 [a, b): the token after the last
// "][", brackets removed, after the last ':'.  Writes the account bytes into `out` (cap 64);
// returns its length, or -1 if longer than the buffer (host decides).
__host__ __device__ inline int baf_account(const uint8_t* p, int a, int b, uint8_t* out) {
  int s = a;
  for (int i = a; i + 1 < b; ++i)
    if (p[i] == ']' && p[i + 1] == '[') s = i + 2;
  // after the last ':' of the bracket-free string == after the last ':' of [s, b)
  int c = s;
  for (int i = s; i < b; ++i)
    if (p[i] == ':') c = i + 1;
  int n = 0;
  for (int i = c; i < b; ++i) {
    if (p[i] == '[' || p[i] == ']') continue;
    if (n >= 64) return -1;
    out[n++] = p[i];
  }
  return n;
}

// split(/<|>/)[2] of the ASCII-trimmed line [0, len): field between the 2nd and 3rd delimiter.
__host__ __device__ inline void angle_field2(const uint8_t* p, int len, int& fs, int& fe) {
  int a = 0, b = len;
  while (a < b && (p[a] == ' ' || (p[a] >= 9 && p[a] <= 13))) ++a;
  while (b > a && (p[b - 1] == ' ' || (p[b - 1] >= 9 && p[b - 1] <= 13))) --b;
  int field = 0, start = a;
  fs = fe = -1;
  for (int i = a; i <= b; ++i) {
    if (i == b || p[i] == '<' || p[i] == '>') {
      if (field == 2) { fs = start; fe = i; return; }
      ++field;
      start = i + 1;
    }
  }
}

}  // namespace dj
}  // namespace apm
