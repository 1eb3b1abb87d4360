// Text line writer shared by the GPU encoders (format.hip K12 st/fs/COPY/fb rows, devjoin.hip
// tx lines).  Lines of neighbouring lanes are adjacent in the output, so a lane packs its bytes
// into a register and stores whole aligned dwords; only the first and last dword of a line, which
// it shares with the neighbouring lines, are written bytewise.
#pragma once

#include "devjoin_dev.h"

namespace apm {

// Rare paths of the writer, out of line: they fill a local buffer and return its length (bit 16:
// inexact).  They take no reference to the writer or the caller's flags -- a noinline member
// (or a bool& into one) puts the whole writer into scratch memory, which made every character of
// the hot path a scratch access (rocprofv3: 576-704 B of scratch per lane in k_write /
// k_format_write, profiles/r3_*).
__device__ __noinline__ static uint32_t text_js_num(char* buf, double x) {
  bool inexact = false;
  const int k = dj::js_num(buf, x, &inexact);
  return (uint32_t)k | (inexact ? 0x10000u : 0u);
}
__device__ __noinline__ static uint32_t text_u64(char* buf, uint64_t v) {
  char t[20];
  int k = 0;
  do { t[k++] = (char)('0' + v % 10); v /= 10; } while (v);
  for (int i = 0; i < k; ++i) buf[i] = t[k - 1 - i];
  return (uint32_t)k;
}
// |x| >= 2^53: x is an integer, so toFixed prints its digits and f zeros below 1e21 and
// String(x) (exponent form) from 1e21 (ECMA-262 Number.prototype.toFixed step 10); exact up to
// 2^127 (128-bit digits, shortest round-trip for String), bit 16 marks larger values.
__device__ __noinline__ static uint32_t text_big_fixed(char* buf, bool neg, double ax, int f) {
  if (ax >= 1e21) return text_js_num(buf, neg ? -ax : ax);
  int n = 0;
  if (neg) buf[n++] = '-';
  n += dj::put_dec(buf + n, (unsigned __int128)ax);
  buf[n++] = '.';
  for (int i = 0; i < f; ++i) buf[n++] = '0';
  return (uint32_t)n;
}

// W = false: the length pass (counts only).  W = true: bytes are packed into a
// 32-bit register and stored one aligned dword at a time; only the first and last dword of a
// line, which it shares with its neighbours' lines, are written bytewise.  (One ds_write_b8 per
// character from 64 lanes ~300 B apart was the write pass's cost: 8.65 LDS bank-conflict cycles
// per instruction, profiles/r2_pmc_kernels.md.)
template <bool W>
struct OutT {
  char* base;   // the line's first byte (W)
  uint32_t mis; // base's offset inside its dword
  uint32_t n = 0;
  uint32_t acc = 0;
  __device__ __forceinline__ explicit OutT(char* p) : base(p), mis(W ? (uint32_t)((uintptr_t)p & 3u) : 0u) {}
  __device__ __forceinline__ void store_dword() {
    // acc holds the dword ending at byte n - 1 (absolute alignment)
    if (n >= 4) {
      *reinterpret_cast<uint32_t*>(base + n - 4) = acc;
    } else {  // the line's first dword is shared with the previous line
      for (uint32_t b = 0; b < n; ++b) base[b] = (char)(acc >> (8u * ((mis + b) & 3u)));
    }
    acc = 0;
  }
  __device__ __forceinline__ void c(char ch) {
    if (W) {
      const uint32_t k = (mis + n) & 3u;
      acc |= (uint32_t)(uint8_t)ch << (8u * k);
      ++n;
      if (k == 3u) store_dword();
    } else {
      ++n;
    }
  }
  // the line's last (partial) dword, shared with the next line
  __device__ __forceinline__ void finish() {
    if (!W) return;
    const uint32_t k = (mis + n) & 3u;
    if (k == 0) return;
    const uint32_t b0 = n > k ? n - k : 0;
    for (uint32_t b = b0; b < n; ++b) base[b] = (char)(acc >> (8u * ((mis + b) & 3u)));
  }
  // Bytes from memory: one aligned 16-byte load per 16 bytes (the block around src), so a lane
  // waits on memory once per 16 characters instead of once per character.  The load may touch
  // up to 15 bytes before src / after src + len inside the same aligned 16-byte block (device
  // allocations are 256-byte aligned and padded, so that stays inside the allocation).
  __device__ __forceinline__ void s(const char* src, int len) {
    if (!W) { n += len; return; }
    const int lead = (int)((uintptr_t)src & 15u);
    const uint4* a = reinterpret_cast<const uint4*>(src - lead);
    for (int g = -lead; g < len; g += 16, ++a) {
      const uint4 v = *a;
      const uint32_t vw[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int i = g + k;
        if (i >= 0 && i < len) c((char)(vw[k >> 2] >> (8 * (k & 3))));
      }
    }
  }
  // bytes one at a time (kernel-argument strings: no over-read outside the argument block)
  __device__ __forceinline__ void sb(const char* src, int len) {
    if (!W) { n += len; return; }
    for (int i = 0; i < len; ++i) c(src[i]);
  }
  // a string literal: characters known at compile time
  template <int N>
  __device__ __forceinline__ void lit(const char (&str)[N]) {
    if (!W) { n += N - 1; return; }
#pragma unroll
    for (int i = 0; i < N - 1; ++i) c(str[i]);
  }
  __device__ __forceinline__ static int digits32(uint32_t v) {
    return v < 10u ? 1 : v < 100u ? 2 : v < 1000u ? 3 : v < 10000u ? 4 : v < 100000u ? 5
         : v < 1000000u ? 6 : v < 10000000u ? 7 : v < 100000000u ? 8 : v < 1000000000u ? 9 : 10;
  }
  // Unsigned decimal.  Nearly every value fits 32 bits, where division by 10 is a multiply-high
  // (64-bit division is a long emulated sequence on CDNA); the length pass only counts digits.
  __device__ __forceinline__ void u32(uint32_t v) {
    const int k = digits32(v);
    if (!W) { n += k; return; }
    // most significant digit first, each by constant divisors (multiply-high), no arrays
    constexpr uint32_t P10[10] = {1u, 10u, 100u, 1000u, 10000u, 100000u, 1000000u, 10000000u, 100000000u,
                                  1000000000u};
#pragma unroll
    for (int j = 9; j >= 0; --j)
      if (j < k) c((char)('0' + (v / P10[j]) % 10u));
  }
  // exactly 8 digits (leading zeros), 32-bit constant divisions
  __device__ __forceinline__ void u32_fixed8(uint32_t r) {
    if (!W) { n += 8; return; }
    constexpr uint32_t P10[8] = {1u, 10u, 100u, 1000u, 10000u, 100000u, 1000000u, 10000000u};
#pragma unroll
    for (int j = 7; j >= 0; --j) c((char)('0' + (r / P10[j]) % 10u));
  }
  // Above 2^32 -- the tx lines' epoch-ms timestamps and 16-digit account numbers, three per
  // line -- one 64-bit division by 10^8 splits v into two 32-bit halves formatted in registers
  // (the digit loop over 64-bit values into a local buffer lived in scratch memory).
  __device__ __forceinline__ void u(uint64_t v) {
    if (v <= 0xffffffffull) { u32((uint32_t)v); return; }
    if (v < 100000000ull * 0xffffffffull) {
      const uint64_t q = v / 100000000ull;
      const uint32_t r = (uint32_t)(v - q * 100000000ull);
      u32((uint32_t)q);
      u32_fixed8(r);
      return;
    }
    char buf[24];
    const uint32_t k = text_u64(buf, v);
    s(buf, (int)k);
  }
  __device__ __forceinline__ void i64(int64_t v) {
    if (v < 0) { c('-'); u((uint64_t)(-v)); } else u((uint64_t)v);
  }
  // String(x) of a JS Number, as dj::js_num prints it: integral |x| < 2^54 inline (-0 -> 0),
  // NaN, everything else through js_num into a local buffer (rare)
  __device__ __forceinline__ void jsnum(double x, bool& inexact) {
    if (x != x) { lit("NaN"); return; }
    const bool neg = x < 0;
    const double ax = neg ? -x : x;
    if (ax < 18014398509481984.0 && ax == floor(ax)) {
      if (ax == 0) { c('0'); return; }
      if (neg) c('-');
      u((uint64_t)ax);
      return;
    }
    char buf[64];
    const uint32_t r = text_js_num(buf, x);
    if (r >> 16) inexact = true;
    s(buf, (int)(r & 0xffffu));
  }
  // toFixed's integer n for |x| < 2^53: x * 10^f rounded, ties to the larger n (ECMA-262 21.1.3.3)
  __device__ __forceinline__ static uint64_t fixed_n(double ax, int f) {
    const double scale = f == 1 ? 10.0 : 100.0;
    const double pr = ax * scale;
    const double e = fma(ax, scale, -pr);  // exact: x * 10^f = pr + e
    uint64_t nn;
    if (pr >= 4503599627370496.0) {  // pr >= 2^52 is an integer: n = nearest integer to pr + e
      nn = (uint64_t)pr + (uint64_t)(int64_t)floor(e + 0.5);
    } else {
      const double q = floor(pr);
      const double d = (pr - q) - 0.5;
      nn = (uint64_t)q;
      if (d > 0 || (d == 0 && e >= 0)) ++nn;
    }
    return nn;
  }
  // nn = ip * 10^f + fr with constant divisors (32-bit when nn fits: nearly always)
  __device__ __forceinline__ static void split_fixed(uint64_t nn, int f, uint64_t& ip, uint32_t& fr) {
    if (nn <= 0xffffffffull) {
      const uint32_t v = (uint32_t)nn;
      if (f == 1) { ip = v / 10u; fr = v % 10u; } else { ip = v / 100u; fr = v % 100u; }
    } else if (f == 1) {
      ip = nn / 10u; fr = (uint32_t)(nn % 10u);
    } else {
      ip = nn / 100u; fr = (uint32_t)(nn % 100u);
    }
  }
  // nf(x, f): 'undefined' for NaN, else x.toFixed(f)
  __device__ __forceinline__ void fixed(double x, int f, bool& fallback) {
    if (x != x) { lit("undefined"); return; }
    const bool neg = x < 0;
    const double ax = neg ? -x : x;
    if (!(ax < 9007199254740992.0)) {  // >= 2^53: integral values (rare)
      char buf[64];
      const uint32_t r = text_big_fixed(buf, neg, ax, f);
      if (r >> 16) fallback = true;
      s(buf, (int)(r & 0xffffu));
      return;
    }
    const uint64_t nn = fixed_n(ax, f);
    if (neg) c('-');
    uint64_t ip;
    uint32_t fr;
    split_fixed(nn, f, ip, fr);
    u(ip);
    c('.');
    if (f == 2) { c((char)('0' + fr / 10u)); c((char)('0' + fr % 10u)); }
    else c((char)('0' + fr));
  }
  // String(parseFloat(x.toFixed(f))) -- a number as the DB row holds it (copyenc.cpp parses the
  // wire text back and prints it JS-style): NaN -> `nul` ('null' in JSON, '\N' as a COPY field).
  // Below 10^15 significant units the parsed value's shortest form is the toFixed text with
  // trailing fraction zeros dropped (a <= 15-digit decimal round-trips uniquely); -0 prints 0.
  __device__ __forceinline__ void js_fixed(double x, int f, bool json, bool& fallback) {
    if (x != x) { if (json) lit("null"); else lit("\\N"); return; }
    const bool neg = x < 0;
    const double ax = neg ? -x : x;
    if (!(ax < 9007199254740992.0)) {  // integral: toFixed -> parseFloat gives x back
      char buf[64];
      const uint32_t r = text_js_num(buf, x);
      if (r >> 16) fallback = true;
      s(buf, (int)(r & 0xffffu));
      return;
    }
    const uint64_t nn = fixed_n(ax, f);
    if (nn == 0) { c('0'); return; }
    if (nn >= 1000000000000000ULL) fallback = true;
    if (neg) c('-');
    uint64_t ip;
    uint32_t fr;
    split_fixed(nn, f, ip, fr);
    u(ip);
    if (fr == 0) return;
    c('.');
    if (f == 2) {
      c((char)('0' + fr / 10u));
      if (fr % 10u) c((char)('0' + fr % 10u));
    } else {
      c((char)('0' + fr));
    }
  }
  // a name as a COPY text field (device memory: 16-byte loads as in s())
  __device__ __forceinline__ void copy_char(char ch) {
    if (ch == '\\' || ch == '\t' || ch == '\n' || ch == '\r') {
      c('\\');
      c(ch == '\\' ? '\\' : (ch == '\t' ? 't' : (ch == '\n' ? 'n' : 'r')));
    } else {
      c(ch);
    }
  }
  __device__ __forceinline__ void copy_text(const char* src, int len) {
    if (!W) {
      for (int i = 0; i < len; ++i) {
        const char ch = src[i];
        n += (ch == '\\' || ch == '\t' || ch == '\n' || ch == '\r') ? 2 : 1;
      }
      return;
    }
    const int lead = (int)((uintptr_t)src & 15u);
    const uint4* a = reinterpret_cast<const uint4*>(src - lead);
    for (int g = -lead; g < len; g += 16, ++a) {
      const uint4 v = *a;
      const uint32_t vw[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int i = g + k;
        if (i >= 0 && i < len) copy_char((char)(vw[k >> 2] >> (8 * (k & 3))));
      }
    }
  }
};

}  // namespace apm
