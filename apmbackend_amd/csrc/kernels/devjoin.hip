// K4/K5/K6 on the GPU: the transaction join of stream_parse_transactions.js and the tx wire
// encoder (entries.js TxEntry.toCSVString), for every JVM of the rank at once.
//
// Reference: TTL caches recordCache / acctCache / needNumRecordCache (:211-239), saveAcctNum
// (:294-327), parseSoapLine (:352-376), EJB entry/exit (:378-446), CommonTiming entry/exit
// (:451-565), BAF salvage (:486-504), outputRecord (:264-290).  The host twin is
// runtime/join.cpp (kept as the `joinOnDevice: false` path and as the checkpoint format).
//
// Pipeline per batch (all on the join stream; see devjoin_types.h for the state layout):
//   k_build_ops    one lane per event -> JOp (field extraction, BAF account, SOAP effects)
//   k_soap_*       per-file SOAP request context: segmented scan of transition functions
//                  (summary -> per-file carry -> apply); account lines become JOP_ACCT
//   k_claim        key-table slot per op (find-or-insert, CAS), service registry claim
//   radix sort     ops by slot (stable: line order inside a key)
//   k_exp_*        needNumRecordCache expiry of the regions whose TTL passed (creation order)
//   k_group_walk   one lane per key: replays the key's ops in line order against its state
//   k_place        outputs to their single-stream position (expiries first, then line order)
// then, after the host named new services: k_resolve_len + scan (line lengths, stats index),
// k_write (tx text into the HBM ring, TxRec for K7/K9, rollover candidates).
#include "kernel_api.h"

#include <rocprim/rocprim.hpp>

#include <chrono>
#include <climits>
#include <cstdlib>
#include <cstddef>
#include <cstring>
#include <vector>

#include "devjoin_api.h"
#include "devjoin_dev.h"
#include "devscan.h"
#include "textout.h"

namespace apm {
using namespace dj;

namespace {

constexpr int TB = 256;

// Op grouping by sort (APM_OPSORT=sort, the A/B form of the slot lists, DJArgs::slot_head).  Keys
// are table slots [0, cap), cap (JOP_DIRECT) and cap + 1 (no op): table_bits + 1 bits; onesweep
// with 11-bit digits (two passes up to 22 bits), 8-bit digits above.  (rocprim's default runs a
// block sort + ~8 merge passes below 1M items: ~140 us per batch, profiles/r3_*.)
using OpSortCfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                             rocprim::default_config, 0>;
using OpSortCfg11 = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 8>, rocprim::kernel_config<1024, 8>, 11,
                                        rocprim::block_radix_rank_algorithm::match>,
    0>;
static int op_sort_bits(int table_bits) { return table_bits + 1; }
static bool opsort11(int table_bits) { return op_sort_bits(table_bits) <= 22; }

__device__ __forceinline__ uint32_t grid_n(uint32_t n) { return (n + TB - 1) / TB; }

// ------------------------------------------------------------------------ audit fields (K5)
// parseAppLine's string work (stream_parse_transactions.js:578-731) on one line, for ASCII lines
// with plain numbers and ISO dates that carry their offset; anything else -> the host (HOP_AUD).
constexpr uint32_t AUD_NIL = 0xffffffffu;

__device__ __forceinline__ bool ws_ascii(uint8_t c) { return c == ' ' || (c >= 9 && c <= 13); }

__device__ __forceinline__ void trim_ascii(const uint8_t* p, int& a, int& b) {
  while (a < b && ws_ascii(p[a])) ++a;
  while (b > a && ws_ascii(p[b - 1])) --b;
}

// parseInt of [a, b) with every '[' / ']' removed (whitespace-free); false: the host decides
// (sign / hex prefix / more than 19 digits) -- simple_parse_int() without the copy
__device__ bool parse_int_nobr(const uint8_t* p, int a, int b, double& out) {
  uint64_t x = 0;
  int nd = 0, k = 0;
  for (int i = a; i < b; ++i) {
    const uint8_t ch = p[i];
    if (ch == '[' || ch == ']') continue;
    if (k == 0 && (ch == '+' || ch == '-')) return false;
    if (k == 1 && nd == 1 && x == 0 && (ch == 'x' || ch == 'X')) return false;
    ++k;
    if (ch < '0' || ch > '9') break;
    if (nd >= 19) return false;
    x = x * 10 + (ch - '0');
    ++nd;
  }
  out = nd == 0 ? apm_nan() : (double)x;
  return true;
}

// convertStringDateToMs of [a, b): 1 = '' (empty input), 0 = `out` set (NaN if invalid),
// -1 = the host decides (non-ISO forms, ISO without an offset: local time needs the zone table)
__device__ int aud_date(const uint8_t* p, int a, int b, double& out) {
  if (a >= b) return 1;
  int tpos = -1;
  for (int i = a; i < b; ++i) if (p[i] == 'T') { tpos = i; break; }
  bool iso = false;
  if (tpos >= 0) for (int i = tpos + 1; i < b; ++i) if (p[i] == '-') { iso = true; break; }
  if (!iso) return -1;
  trim_ascii(p, a, b);
  const int n = b - a;
  const uint8_t* t = p + a;
  auto dig = [&](int i, int k, int64_t& v) {
    if (i + k > n) return false;
    v = 0;
    for (int j = 0; j < k; ++j) {
      const uint8_t c = t[i + j];
      if (c < '0' || c > '9') return false;
      v = v * 10 + (c - '0');
    }
    return true;
  };
  out = apm_nan();
  int64_t y, mo, d, h, mi, sec = 0, ms = 0;
  if (!dig(0, 4, y) || n < 16 || t[4] != '-' || !dig(5, 2, mo) || t[7] != '-' || !dig(8, 2, d) || t[10] != 'T' ||
      !dig(11, 2, h) || t[13] != ':' || !dig(14, 2, mi))
    return 0;
  int i = 16;
  if (i < n && t[i] == ':') {
    if (!dig(i + 1, 2, sec)) return 0;
    i += 3;
    if (i < n && t[i] == '.') {
      ++i;
      int j = i, nd = 0;
      int64_t frac = 0;
      while (j < n && t[j] >= '0' && t[j] <= '9') { if (nd < 3) { frac = frac * 10 + (t[j] - '0'); ++nd; } ++j; }
      if (j == i) return 0;
      while (nd < 3) { frac *= 10; ++nd; }
      ms = frac;
      i = j;
    }
  }
  if (mo < 1 || mo > 12 || d < 1 || d > 31 || h > 24 || mi > 59 || sec > 59) return 0;
  const int64_t local = make_date_ms(y, mo - 1, d, h, mi, sec, ms);
  if (i == n) return -1;
  if (t[i] == 'Z' && i + 1 == n) { out = (double)local; return 0; }
  if (t[i] == '+' || t[i] == '-') {
    const int sg = t[i] == '-' ? -1 : 1;
    int64_t oh, om;
    if (!dig(i + 1, 2, oh)) return 0;
    int k = i + 3;
    if (k < n && t[k] == ':') ++k;
    if (!dig(k, 2, om) || k + 2 != n) return 0;
    out = (double)(local - sg * (oh * 60 + om) * 60000);
  }
  return 0;
}

__device__ bool icontains_provider(const uint8_t* p, int a, int b) {
  const char* pat = "provider[";
  for (int i = a; i + 9 <= b; ++i) {
    int k = 0;
    for (; k < 9; ++k) {
      uint8_t c = p[i + k];
      if (c >= 'A' && c <= 'Z') c = (uint8_t)(c + 32);
      if (c != (uint8_t)pat[k]) break;
    }
    if (k == 9) return true;
  }
  return false;
}

// One pass over a line, 16 bytes per aligned load (the byte loops of the first version cost
// ~350 us per batch in dependent loads): non-ASCII, the first two ':' , split(/\s+/) tokens
// 0..5, the '=' of token 5, the first "</" and the last '>' before it.
struct LineScan {
  bool nonascii;
  int c1, c2;           // first ':' (-1), the next ':' after it (len)
  int t0s, t0e, t3s, t3e, t5s, t5e;  // tokens 0, 3, 5 of line.split(/[\s]+/) (start -1: none)
  int eq1, eq2;         // first '=' of token 5 (+1; -1 none), the next '=' (token end if none)
  int lt, gt;           // first "</" (len), last '>' before it (-1)
};

// (scalars only: an indexed token array would live in scratch memory)
__device__ void line_scan(const uint8_t* __restrict__ p, int len, LineScan& L) {
  bool na = false;
  int c1 = -1, c2 = len;
  int t0s = -1, t0e = -1, t3s = -1, t3e = -1, t5s = -1, t5e = -1;
  int eq1 = -1, eq2 = -1, lt = len, gt = -1;
  int tok = 0, tstart = 0;  // current token index / its start
  bool in_ws = false, lt_found = false;
  uint8_t prev = 0;
  const uintptr_t a0 = (uintptr_t)p & ~(uintptr_t)15;
  const int lead = (int)((uintptr_t)p - a0);
  for (int base = -lead; base < len; base += 16) {
    const uint4 v = *reinterpret_cast<const uint4*>(p + base);
    const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int i = base + j;
      if (i < 0 || i >= len) continue;
      const uint8_t c = (uint8_t)(w4[j >> 2] >> (8 * (j & 3)));
      na |= c >= 0x80;
      if (c == ':') {
        if (c1 < 0) c1 = i;
        else if (c2 == len) c2 = i;
      }
      if (!lt_found) {
        if (prev == '<' && c == '/') { lt = i - 1; lt_found = true; }
        else if (c == '>') gt = i;
      }
      if (ws_ascii(c)) {
        if (!in_ws) {
          if (tok == 0) { t0s = tstart; t0e = i; }
          else if (tok == 3) { t3s = tstart; t3e = i; }
          else if (tok == 5) { t5s = tstart; t5e = i; }
          ++tok;
          in_ws = true;
        }
        tstart = i + 1;
      } else {
        in_ws = false;
        if (tok == 5 && c == '=') {
          if (eq1 < 0) eq1 = i + 1;
          else if (eq2 < 0) eq2 = i;
        }
      }
      prev = c;
    }
  }
  if (tok == 0) { t0s = tstart; t0e = len; }
  else if (tok == 3) { t3s = tstart; t3e = len; }
  else if (tok == 5) { t5s = tstart; t5e = len; }
  if (eq1 >= 0 && eq2 < 0) eq2 = t5e;
  L.nonascii = na; L.c1 = c1; L.c2 = c2;
  L.t0s = t0s; L.t0e = t0e; L.t3s = t3s; L.t3e = t3e; L.t5s = t5s; L.t5e = t5e;
  L.eq1 = eq1; L.eq2 = eq2; L.lt = lt; L.gt = gt;
}

// attemptReadAccountNumberFromBAFInfo on token 3 [a, b) without a copy: the token after the last
// "][", brackets removed, after the last ':' (= baf_account()).  n = its length; digits = all
// digits; v = parseInt; false: the host decides (sign / hex prefix / more than 19 digits).
__device__ bool baf_account_scan(const uint8_t* p, int a, int b, int& n, bool& digits, double& v) {
  int st = a;
  for (int i = a; i + 1 < b; ++i) if (p[i] == ']' && p[i + 1] == '[') st = i + 2;
  int c = st;
  for (int i = st; i < b; ++i) if (p[i] == ':') c = i + 1;
  n = 0;
  digits = true;
  uint64_t x = 0;
  int nd = 0;
  bool in_digits = true;  // the parseInt prefix is still running
  for (int i = c; i < b; ++i) {
    const uint8_t ch = p[i];
    if (ch == '[' || ch == ']') continue;
    const bool d = ch >= '0' && ch <= '9';
    if (n == 0 && (ch == '+' || ch == '-')) return false;
    if (n == 1 && nd == 1 && x == 0 && (ch == 'x' || ch == 'X')) return false;
    digits &= d;
    if (in_digits) {
      if (d) {
        if (nd >= 19) return false;
        x = x * 10 + (ch - '0');
        ++nd;
      } else {
        in_digits = false;
      }
    }
    ++n;
  }
  v = nd == 0 ? apm_nan() : (double)x;
  if (n == 0) digits = false;
  return true;
}

// The AudF of an LK_APP event (batch-absolute refs); false when the host must derive it.
// p: the line's first byte (the batch, or k_host_flags' LDS stage at the same offset mod 16).
__device__ bool aud_fields(const Event& e, const uint8_t* __restrict__ p, uint64_t fkey, AudF& f) {
  const int len = (int)e.len;
  f.h_item = 0; f.el = apm_nan(); f.h_sw = 0; f.ts = apm_nan();
  f.ref = 0; f.len = 0; f.flags = 0; f.pad = 0; f.pad2[0] = f.pad2[1] = 0;
  LineScan L;
  line_scan(p, len, L);
  if (L.nonascii) return false;
  const uint32_t m = e.mask;
  if (m & PM_AUTR_MAP) {
    // logId = ws[0] without brackets; auditTrailId = ws[5].split('=')[1]; alt = the BAF account
    int s0 = L.t0s, e0 = L.t0e;
    if (s0 < 0) { s0 = e0 = 0; }
    if (s0 < e0 && p[s0] == '[') ++s0;
    if (e0 > s0 && p[e0 - 1] == ']') --e0;
    for (int i = s0; i < e0; ++i) if (p[i] == '[' || p[i] == ']') return false;  // inner brackets
    f.ref = e.off + (uint32_t)s0;
    f.len = (uint16_t)(e0 - s0);
    f.h_sw = hash_bytes(p + s0, (size_t)(e0 - s0));
    const uint64_t ah = L.eq1 < 0 ? hash_bytes("undefined", 9) : hash_bytes(p + L.eq1, (size_t)(L.eq2 - L.eq1));
    f.h_item = aud_key(ah, fkey);
    if ((m & PM_BAF) && L.t3s >= 0 && L.t3e > L.t3s) {
      int n;
      bool digits;
      double v;
      if (!baf_account_scan(p, L.t3s, L.t3e, n, digits, v)) return false;
      if (n > 0) {
        f.el = v;
        f.flags |= AF_ACCT;
        if (digits) f.flags |= AF_ACCT_VALID;
      }
    }
    return true;
  }
  if (m & PM_AUTR_HDR) {  // line.split(':')[1].trim()
    if (L.c1 < 0) return false;
    int a = L.c1 + 1, b = L.c2;
    trim_ascii(p, a, b);
    f.h_item = aud_key(hash_bytes(p + a, (size_t)(b - a)), fkey);
    return true;
  }
  // item role (a line inside the elapsed section): service = split(':')[0].trim(),
  // elapsed = split(':')[1].split(/\s+/)[0] without brackets
  {
    int a = 0, b = L.c1 >= 0 ? L.c1 : len;
    trim_ascii(p, a, b);
    f.h_item = hash_bytes(p + a, (size_t)(b - a));
    if (L.c1 >= 0) {
      int t = L.c1 + 1;
      while (t < L.c2 && !ws_ascii(p[t])) ++t;
      if (!parse_int_nobr(p, L.c1 + 1, t, f.el)) return false;
    }
  }
  if (m & (PM_SW_NAME | PM_SW_STARTTS | PM_SW_STOPTS)) {
    const int t = L.lt, s = L.gt >= 0 ? L.gt + 1 : 0;  // line.replace(/<\/.*/,'').replace(/.*>/,'')
    if (m & PM_SW_NAME) {
      f.ref = e.off + (uint32_t)s;
      f.len = (uint16_t)(t - s);
      f.h_sw = hash_bytes(p + s, (size_t)(t - s));
      if (!icontains_provider(p, s, t)) f.flags |= AF_TO_DB;
    } else {
      const int r = aud_date(p, s, t, f.ts);
      if (r < 0) return false;
      if (r == 1) f.flags |= AF_TS_EMPTY;
    }
  }
  return true;
}

// Non-audit events: the byte-level fields the join needs, derived once on the parse stream (next
// to needs_host, which scans the same bytes) and stored in the event's AudF slot, so k_build_ops
// -- on the join stream, the ingest thread's critical path -- only reads them:
//   CT exit with a BAF token: the account scan (el = value, PRE_BAF / PRE_BAF_VALID);
//   SOAP request start: hash of the logId field (h_item);  SOAP account / value: the parsed
//   number (el, PRE_SOAP_VALID).
// Returns -1: the host derives the event (needs_host), 0: nothing stored, 1: stored in f.
enum : uint8_t { PRE_BAF = 1, PRE_BAF_VALID = 2, PRE_SOAP_VALID = 4 };
// split(/<|>/)[2] of the ASCII-trimmed line [0, len) (dj::angle_field2), on the device: the
// delimiters of each dword found exactly by SWAR over aligned 16-byte loads -- one load per 16
// bytes instead of a dependent byte load per character (lane per SOAP line, ~100-200 bytes).
__device__ __forceinline__ uint32_t zero_bytes(uint32_t x) {  // 0x80 in every zero byte of x
  return ~((((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) | 0x7f7f7f7fu);
}
__device__ void angle_field2_dev(const uint8_t* __restrict__ p, int len, int& fs, int& fe) {
  auto ws = [](uint8_t c) { return c == ' ' || (c >= 9 && c <= 13); };
  int a = 0, b = len;
  while (a < b && ws(p[a])) ++a;
  while (b > a && ws(p[b - 1])) --b;
  fs = fe = -1;
  int seen = 0, start = -1;
  const int lead = (int)((uintptr_t)(p + a) & 15u);
  const uint4* q = reinterpret_cast<const uint4*>(p + a - lead);
  for (int g = a - lead; g < b; g += 16, ++q) {
    const uint4 v = *q;
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      uint32_t m = zero_bytes(w[k] ^ 0x3c3c3c3cu) | zero_bytes(w[k] ^ 0x3e3e3e3eu);  // '<' | '>'
      while (m) {
        const int i = g + 4 * k + (__builtin_ctz(m) >> 3);
        m &= m - 1;
        if (i < a || i >= b) continue;
        if (seen == 2) { fs = start; fe = i; return; }
        if (++seen == 2) start = i + 1;
      }
    }
  }
  if (seen == 2) { fs = start; fe = b; }
}

__device__ int pre_fields(const Event& e, const uint8_t* __restrict__ p, AudF& f, bool bytewise) {
  if (e.mask & PM_HOST) return -1;
  f.h_item = 0; f.el = apm_nan(); f.h_sw = 0; f.ts = apm_nan(); f.ref = 0; f.len = 0; f.flags = 0; f.pad = 0;
  if (e.kind >= LK_EJB_ENTRY && e.kind <= LK_CT_EXIT) {
    if (!(e.mask & PM_KEYS) || e.ntok < 3) return -1;
    if (e.kind == LK_CT_EXIT && (e.mask & PM_BAF)) {
      int n = 9;  // fewer than 4 tokens: the account string is "undefined" (NaN, not digits)
      bool digits = false;
      double v = apm_nan();
      if (e.ntok >= 4 && !baf_account_scan(p, e.t3s, e.t3e, n, digits, v)) return -1;
      f.el = v;
      f.flags = (uint8_t)((n > 0 ? PRE_BAF : 0) | (digits ? PRE_BAF_VALID : 0));
      return 1;
    }
    return 0;
  }
  if (e.kind == LK_SOAP) {
    const uint32_t m = e.mask;
    if (m & PM_SOAP_IN) {  // ws[1].split('=')[1]; no '=' -> has_log_id false -> "undefined"
      int s = -1, t = -1;
      if (e.ntok >= 2) {
        const int a0 = e.t1s, b0 = e.t1e;
        for (int k = a0; k < b0; ++k) if (p[k] == '=') { s = k + 1; break; }
        if (s >= 0) { t = b0; for (int k = s; k < b0; ++k) if (p[k] == '=') { t = k; break; } }
      }
      f.h_item = s >= 0 ? hash_bytes(p + s, (size_t)(t - s)) : hash_bytes("undefined", 9);
      return 1;
    }
    if (m & PM_SOAP_OUT) return 0;
    if (m & (PM_SOAP_ACCT | PM_SOAP_VALUE)) {
      if (!(m & PM_SOAP_ACCT) && (m & PM_SOAP_KEY)) return 0;  // KEY branch wins
      int fs, fe;
      if (bytewise) angle_field2(p, (int)e.len, fs, fe);  // (APM_PRE_BYTEWISE: A/B switch)
      else angle_field2_dev(p, (int)e.len, fs, fe);
      if (fs >= 0) {
        while (fs < fe && (p[fs] == ' ' || (p[fs] >= 9 && p[fs] <= 13))) ++fs;
        while (fe > fs && (p[fe - 1] == ' ' || (p[fe - 1] >= 9 && p[fe - 1] <= 13))) --fe;
        if (all_digits(p + fs, fe - fs)) {
          double v;
          if (!simple_parse_int(p + fs, fe - fs, v)) return -1;
          f.el = v;
          f.flags = PRE_SOAP_VALID;
        }
      }
      return 1;
    }
  }
  return 0;
}

enum : uint8_t { SEL_HOST = 1, SEL_MH = 2, SEL_WALK = 4 };

// Per-event selection counts packed into one u64 for the exclusive scan (a 16-byte struct scan
// took ~180 us per batch over 1M entries; u64 takes rocprim's atomic look-back path):
// host bits 0-21, mh bits 22-42, walk bits 43-63 (maxLinesPerBatch < 2^21, checked at init)
constexpr int SEL_MH_SHIFT = 22, SEL_WALK_SHIFT = 43;
__device__ __forceinline__ SelCount sel_unpack(uint64_t v) {
  return SelCount{(uint32_t)(v & ((1ull << SEL_MH_SHIFT) - 1)),
                  (uint32_t)((v >> SEL_MH_SHIFT) & ((1ull << (SEL_WALK_SHIFT - SEL_MH_SHIFT)) - 1)),
                  (uint32_t)(v >> SEL_WALK_SHIFT), 0u};
}

// Per event: host / audit-list flags and counts; the AudF of every audit line the GPU reads
// (computed once here, on the parse stream, and read by the join's k_build_ops).
//
// The byte work (the audit line scan, the SOAP logId / account fields, the BAF account token) is
// a lane walking its own line.  Reading the batch directly, every step of those walks waited on
// a dependent global load: 130 us a batch for ~45k events (profiles/r4_x, the largest kernel of
// the join side).  Now each lane first copies its line into an LDS slot with independent 16-byte
// loads (all in flight at once: one memory latency per line), at the same offset modulo 16 so
// the walks' aligned vector reads stay aligned, and walks it there.  Lines longer than a slot
// (rare) walk the batch as before.  APM_HF_STAGE=0 keeps the unstaged walk (A/B).
constexpr int HF_SLOT = 256;  // staged bytes per lane
// Slot pitch 272 B (68 dwords): with 256 B every lane's slot began on bank 0, so the 16 lanes of a
// ds_read_b128 group reading the same 16-byte block of their lines hit the same 4 banks -- 16.04
// conflict cycles per LDS instruction (profiles/r5_p); 68 dwords apart, 16 lanes cover all 64
// banks, and the b128 stores' 8-lane groups all 32.  68 KB per 256-lane block: still 2 per CU.
constexpr int HF_PITCH = HF_SLOT + 16;

__device__ __forceinline__ bool hf_needs_bytes(const Event& e) {
  if (e.kind == LK_APP) return !(e.mask & PM_HOST);
  if (e.mask & PM_HOST) return false;
  if (e.kind == LK_CT_EXIT) return (e.mask & PM_KEYS) && e.ntok >= 3 && (e.mask & PM_BAF);
  if (e.kind == LK_SOAP) return (e.mask & (PM_SOAP_IN | PM_SOAP_ACCT | PM_SOAP_VALUE)) != 0;
  return false;
}

__device__ __forceinline__ uint8_t hf_fields(const Event& e, const uint8_t* __restrict__ p, uint64_t fkey, AudF* aud,
                                             uint32_t i, int bytewise) {
  uint8_t fl = 0;
  if (e.kind == LK_APP) {
    bool host = (e.mask & PM_HOST) != 0;
    if (!host) {
      AudF f;
      host = !aud_fields(e, p, fkey, f);
      if (!host) aud[i] = f;
    }
    if (host) fl |= SEL_HOST;
  } else {
    AudF f;
    const int r = pre_fields(e, p, f, bytewise != 0);
    if (r < 0) fl |= SEL_HOST;
    else if (r > 0) aud[i] = f;  // read by k_build_ops
  }
  return fl;
}

// Wave-aggregated append of this lane's index when `want` (one atomic per wave); every lane of the
// wave calls it.  Returns the slot, ~0u when !want.
__device__ __forceinline__ uint32_t wave_append(bool want, uint32_t* counter) {
  const uint64_t m = __ballot(want);
  if (!m) return ~0u;
  const uint32_t lane = threadIdx.x & (APM_WAVE - 1);
  const uint32_t leader = (uint32_t)__ffsll((unsigned long long)m) - 1u;
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(counter, (uint32_t)__popcll(m));
  base = (uint32_t)__shfl((int)base, (int)leader, APM_WAVE);
  return want ? base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull)) : ~0u;
}

__device__ __forceinline__ uint64_t sel_pack(uint8_t fl) {
  return (uint64_t)(fl & SEL_HOST) | ((fl & SEL_MH) ? 1ull << SEL_MH_SHIFT : 0ull) |
         ((fl & SEL_WALK) ? 1ull << SEL_WALK_SHIFT : 0ull);
}

__device__ __forceinline__ uint8_t app_bits(const Event& e) {
  if (e.kind != LK_APP) return 0;
  return (e.mask & PM_AUTR_MAP) ? SEL_MH : (uint8_t)(SEL_WALK | ((e.mask & PM_AUTR_HDR) ? SEL_MH : 0));
}

// Byte work of one event: its line staged into this lane's LDS slot when it fits (independent
// 16-byte loads, one memory latency per line), then walked there.
__device__ __forceinline__ uint8_t hf_event(const Event& e, uint32_t i, const uint8_t* __restrict__ bytes,
                                            const uint32_t* __restrict__ chunk_file,
                                            const uint64_t* __restrict__ file_fkey, AudF* __restrict__ aud,
                                            uint8_t* stage, int bytewise, int staged) {
  const uint64_t fkey = e.kind == LK_APP ? file_fkey[chunk_file[e.chunk]] : 0;
  // (staging only decides where the walk reads: a staged line is a complete copy, so the field
  // functions -- which read bytes only in the cases hf_needs_bytes names -- are unchanged)
  const uint8_t* p = bytes + e.off;
  const uint32_t lead = e.off & 15u;
  const uint32_t nvec = (lead + e.len + 15u) >> 4;
  if (staged && hf_needs_bytes(e) && nvec * 16u <= (uint32_t)HF_SLOT) {
    // the line's aligned 16-byte blocks, four loads in flight before their LDS stores (sixteen
    // held at once put the array on scratch: 272 B of private memory per lane)
    const uint4* __restrict__ src = reinterpret_cast<const uint4*>(bytes + (e.off - lead));
    uint4* dst = reinterpret_cast<uint4*>(stage + threadIdx.x * HF_PITCH);
    for (uint32_t k = 0; k < nvec; k += 4) {
      const uint4 v0 = src[k];
      const uint4 v1 = k + 1 < nvec ? src[k + 1] : v0;
      const uint4 v2 = k + 2 < nvec ? src[k + 2] : v0;
      const uint4 v3 = k + 3 < nvec ? src[k + 3] : v0;
      dst[k] = v0;
      if (k + 1 < nvec) dst[k + 1] = v1;
      if (k + 2 < nvec) dst[k + 2] = v2;
      if (k + 3 < nvec) dst[k + 3] = v3;
    }
    p = stage + threadIdx.x * HF_PITCH + lead;
  }
  return (uint8_t)(hf_fields(e, p, fkey, aud, i, bytewise) | app_bits(e));
}

// Host / audit selection flags per event.  `split` (default): events whose flags need their line's
// bytes -- audit lines, SOAP request / account lines, CommonTiming exits with a BAF account, a
// minority of the batch -- are listed instead (audit lines from the front of `list`, the others
// from the back) and walked densely by k_host_flags_bytes; every other event is decided here
// from its Event alone.  One lane per event over the whole batch made every wave execute each of
// the walks its few byte events needed, the other lanes idle (the largest join-side kernel:
// 137 us a batch, profiles/r5_final2).  split == 0: the one-pass form (APM_HF_SPLIT=0, A/B).
template <bool SPLIT>
__global__ __launch_bounds__(TB) void k_host_flags(const Event* __restrict__ ev, const uint32_t* __restrict__ n_ev_dev,
                                                   const uint8_t* __restrict__ bytes, const uint32_t* __restrict__ chunk_file,
                                                   const uint64_t* __restrict__ file_fkey,
                                                   uint8_t* __restrict__ flag, uint64_t* __restrict__ val,
                                                   AudF* __restrict__ aud, SelCount* __restrict__ totals, uint32_t cap,
                                                   int bytewise, int staged, uint32_t* __restrict__ list,
                                                   uint32_t* __restrict__ list_n) {
  constexpr int split = SPLIT ? 1 : 0;
  // (the split form reads no bytes: no LDS stage, so the occupancy is register-bound)
  __shared__ __attribute__((aligned(16))) uint8_t stage[SPLIT ? 16 : TB * HF_PITCH];
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t n = min(*n_ev_dev, cap);
  if (blockIdx.x * blockDim.x >= n) return;  // (uniform per block: the grid is sized for the capacity)
  uint32_t ab = 0;
  Event e;
  bool defer = false, front = false;
  if (i < n) {
    e = ev[i];
    if (e.kind == LK_APP && (e.mask & (PM_AUTR_MAP | PM_SW_NAME))) ab = e.len;
    defer = split && hf_needs_bytes(e);
    front = defer && e.kind == LK_APP;
  }
  if (split) {  // (uniform: every lane takes part in both appends)
    const uint32_t f = wave_append(front, &list_n[0]);
    const uint32_t b = wave_append(defer && !front, &list_n[1]);
    if (front) list[f] = i;
    if (defer && !front) list[cap - 1 - b] = i;
  }
  if (i < n && !defer) {
    uint8_t fl;
    if constexpr (SPLIT) fl = (uint8_t)(hf_fields(e, bytes + e.off, 0, aud, i, bytewise) | app_bits(e));
    else fl = hf_event(e, i, bytes, chunk_file, file_fkey, aud, stage, bytewise, staged);
    flag[i] = fl;
    val[i] = sel_pack(fl);
  }
  // bytes of map / stopWatch-name lines: one atomic per wave (totals zeroed before the launch)
  for (int o = APM_WAVE / 2; o > 0; o >>= 1) ab += __shfl_xor(ab, o, APM_WAVE);
  if ((threadIdx.x & (APM_WAVE - 1)) == 0 && ab) atomicAdd(&totals->aud_bytes, ab);
}

// The listed events of k_host_flags: audit lines at [0, list_n[0]), the others at
// [cap - list_n[1], cap) -- each wave runs (nearly) one kind of walk with every lane busy.
__global__ __launch_bounds__(TB) void k_host_flags_bytes(const Event* __restrict__ ev, const uint8_t* __restrict__ bytes,
                                                         const uint32_t* __restrict__ chunk_file,
                                                         const uint64_t* __restrict__ file_fkey,
                                                         uint8_t* __restrict__ flag, uint64_t* __restrict__ val,
                                                         AudF* __restrict__ aud, uint32_t cap, int bytewise, int staged,
                                                         const uint32_t* __restrict__ list,
                                                         const uint32_t* __restrict__ list_n) {
  __shared__ __attribute__((aligned(16))) uint8_t stage[TB * HF_PITCH];
  const uint32_t nf = list_n[0], nb = list_n[1];
  const uint32_t b0 = blockIdx.x * blockDim.x, b1 = b0 + blockDim.x;
  if (b0 >= nf && b1 <= cap - nb) return;  // a block in the gap between the two lists (uniform)
  const uint32_t t = b0 + threadIdx.x;
  if (t >= cap || (t >= nf && t < cap - nb)) return;
  const uint32_t i = list[t];
  const Event e = ev[i];
  const uint8_t fl = hf_event(e, i, bytes, chunk_file, file_fkey, aud, stage, bytewise, staged);
  flag[i] = fl;
  val[i] = sel_pack(fl);
}

// host / map-header / walk lists, in event order (devscan.h over the batch's events only)
struct SelValF {
  const uint64_t* val;
  __device__ uint64_t operator()(uint32_t i) const { return val[i]; }
};
struct SelScatterG {
  const Event* ev;
  const uint8_t* flag;
  const uint64_t* total;
  Event* out;
  uint32_t *out_idx, *mh_idx, *walk_idx;
  SelCount* totals;
  __device__ void operator()(uint32_t i, uint64_t pos) const {
    if (i == 0) {
      const SelCount t = sel_unpack(*total);
      totals->host = t.host; totals->mh = t.mh; totals->walk = t.walk;
    }
    const uint8_t fl = flag[i];
    if (!fl) return;
    const SelCount p = sel_unpack(pos);
    if (fl & SEL_HOST) { out[p.host] = ev[i]; out_idx[p.host] = i; }
    if (fl & SEL_MH) mh_idx[p.mh] = i;
    if (fl & SEL_WALK) walk_idx[p.walk] = i;
  }
};

// ------------------------------------------------------------------------ op build
enum : uint8_t { SC_NONE = 0, SC_IN = 1, SC_OUT = 2, SC_ACCT = 3, SC_KEY = 4, SC_VALUE = 5 };

__device__ const HostOp* find_hop(const HostOp* __restrict__ h, uint32_t n, uint32_t ev) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (h[mid].ev < ev) lo = mid + 1; else hi = mid;
  }
  return (lo < n && h[lo].ev == ev) ? &h[lo] : nullptr;
}

__global__ __launch_bounds__(TB) void k_build_ops(DJArgs a) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n_ev) return;
  const Event e = a.ev[i];
  JOp op;
  op.gkey = 0; op.svc = 0; op.ts = apm_nan(); op.num = apm_nan(); op.aux = apm_nan(); op.aux2 = apm_nan();
  op.line = e.line; op.lid = 0; op.svc_ref = 0; op.lid_len = 0; op.svc_len = 0;
  op.flags = 0; op.op = JOP_NONE; op.pad = 0;
  const int32_t file = (int32_t)a.chunk_file[e.chunk];
  const int32_t server = a.file_server[file];
  const uint64_t skey = a.file_skey[file];
  op.server = server;
  uint8_t code = SC_NONE;
  double snum = apm_nan();
  uint64_t shash = 0;
  const uint8_t* p = a.bytes + e.off;
  if (e.kind == LK_APP) {  // K5 fields; a map line's BAF account is saved at once (saveAcctNum)
    AudF f;
    bool ok = false;
    if (a.host_flag[i] & SEL_HOST) {
      const HostOp* h = find_hop(a.hops, a.n_hops, i);
      if (h && h->kind == HOP_AUD) { f = *reinterpret_cast<const AudF*>(&h->op); ok = true; }
      if (!ok) {  // (no host op: the line is ignored, as the host pre-pass would)
        f.h_item = 0; f.el = apm_nan(); f.h_sw = 0; f.ts = apm_nan(); f.ref = 0; f.len = 0; f.flags = 0;
      }
      a.aud[i] = f;
    } else {
      f = a.aud[i];  // k_host_flags derived it
    }
    if ((e.mask & PM_AUTR_MAP) && (f.flags & AF_ACCT)) {
      if (!(f.flags & AF_ACCT_VALID)) {
        atomicAdd(&a.counts->invalid_acct, 1ULL);
      } else if (f.len > 0) {
        op.op = JOP_ACCT;
        op.gkey = gkey_of(f.h_sw, skey);
        op.num = f.el;
      }
    }
  } else if (a.host_flag[i] & SEL_HOST) {
    const HostOp* h = find_hop(a.hops, a.n_hops, i);
    if (h) {
      switch (h->kind) {
        case HOP_JOIN: op = h->op; break;
        case HOP_SOAP_IN: code = SC_IN; shash = h->lid_hash; break;
        case HOP_SOAP_OUT: code = SC_OUT; break;
        case HOP_SOAP_ACCT: if (h->op.flags & JF_BAF_VALID) { code = SC_ACCT; snum = h->op.num; } break;
        case HOP_SOAP_KEY: code = SC_KEY; break;
        case HOP_SOAP_VALUE: if (h->op.flags & JF_BAF_VALID) { code = SC_VALUE; snum = h->op.num; } break;
        default: break;
      }
    }
  } else if (e.kind >= LK_EJB_ENTRY && e.kind <= LK_CT_EXIT) {
    const bool ejb = e.kind <= LK_EJB_EXIT;
    const bool entry = e.kind == LK_EJB_ENTRY || e.kind == LK_CT_ENTRY;
    op.lid = e.off + e.t0s;
    op.lid_len = (uint16_t)(e.t0e - e.t0s);
    op.svc = e.svc;
    op.flags = JF_HAS_SVC | (ejb ? JF_EJB : 0);
    if (e.tAs == 0xffff) op.flags |= JF_SVC_UNDEF;
    else { op.svc_ref = e.off + e.tAs; op.svc_len = (uint16_t)(e.tAe - e.tAs); }
    op.ts = e.ts;
    const bool empty_lid = op.lid_len == 0;
    if (entry) {
      if (!empty_lid) { op.op = JOP_ENTRY; op.gkey = gkey_of(e.key, skey); }
      else op.flags = 0;  // parseEntry returns before naming the service
    } else {
      op.num = (e.kind == LK_EJB_EXIT || e.tBs != 0xffff) ? e.num : apm_nan();
      if (e.kind == LK_CT_EXIT && (e.mask & PM_BAF)) {  // account scanned by k_host_flags (pre_fields)
        const AudF& f = a.aud[i];
        if (f.flags & PRE_BAF) {
          op.flags |= JF_BAF;
          op.aux = f.el;
          if (f.flags & PRE_BAF_VALID) { op.flags |= JF_BAF_VALID; op.aux2 = f.el; }
        }
      }
      if (empty_lid) op.op = JOP_DIRECT;
      else { op.op = e.kind == LK_EJB_EXIT ? JOP_EJB_EXIT : JOP_CT_EXIT; op.gkey = gkey_of(e.key, skey); }
    }
  } else if (e.kind == LK_SOAP) {
    const uint32_t m = e.mask;
    // (the logId hash / the account number come from k_host_flags' pre_fields)
    if (m & PM_SOAP_IN) {
      code = SC_IN;
      shash = a.aud[i].h_item;
    } else if (m & PM_SOAP_OUT) {
      code = SC_OUT;
    } else if (m & (PM_SOAP_ACCT | PM_SOAP_KEY | PM_SOAP_VALUE)) {
      const bool acct = m & PM_SOAP_ACCT;
      if (!acct && (m & PM_SOAP_KEY)) {
        code = SC_KEY;
      } else {
        const AudF& f = a.aud[i];
        if (f.flags & PRE_SOAP_VALID) {
          snum = f.el;
          code = acct ? SC_ACCT : SC_VALUE;
        }
      }
    }
  }
  a.ops[i] = op;
  a.soap_code[i] = code;
  a.soap_num[i] = snum;
  a.soap_hash[i] = shash;
}

// ------------------------------------------------------------------------ SOAP context scan
// State: CONST form {tag 0 none / 1 ctx / 2 ctx + pull_next, L = IN event + 1 (0: carried)}.
// Functions: CONST (IN, OUT, valid account = saved and erased) or MAP (KEY, valid VALUE, others
// identity) acting on the tag only.  Composition is associative, so a wave scans 64 events with
// shuffles and chunks are split into segments whose summaries are chained per file.
constexpr uint32_t F_CONST = 1u << 31;
constexpr uint32_t F_ID = 1u | (2u << 2);
constexpr uint32_t F_KEY = 2u | (2u << 2);
constexpr uint32_t F_VALUE = 1u | (0u << 2);

__device__ __forceinline__ uint32_t map_tag(uint32_t g, uint32_t tag) {
  return tag == 0 ? 0u : (tag == 1 ? (g & 3u) : ((g >> 2) & 3u));
}
// g after f
__device__ __forceinline__ uint32_t fcompose(uint32_t g, uint32_t f) {
  if (g & F_CONST) return g;
  if (f & F_CONST) {
    const uint32_t t = map_tag(g, f & 3u);
    return t ? (F_CONST | t | (f & ~(F_CONST | 3u))) : F_CONST;
  }
  return map_tag(g, f & 3u) | (map_tag(g, (f >> 2) & 3u) << 2);
}
__device__ __forceinline__ uint32_t code_fn(uint8_t c, uint32_t ev) {
  switch (c) {
    case SC_IN: return F_CONST | 1u | ((ev + 1) << 2);
    case SC_OUT: case SC_ACCT: return F_CONST;
    case SC_KEY: return F_KEY;
    case SC_VALUE: return F_VALUE;
    default: return F_ID;
  }
}

__device__ __forceinline__ void soap_range(const uint32_t* lo_tab, uint32_t c, int g, uint32_t& lo, uint32_t& hi) {
  const uint32_t c0 = lo_tab[c], c1 = lo_tab[c + 1];
  const uint32_t n = c1 - c0;
  const uint32_t seg = ((n + SOAP_SEGS - 1) / SOAP_SEGS + APM_WAVE - 1) / APM_WAVE * APM_WAVE;
  lo = min(c1, c0 + (uint32_t)g * seg);
  hi = min(c1, lo + seg);
}

// inclusive wave scan of transition functions (lane order = event order)
__device__ __forceinline__ uint32_t wave_fscan(uint32_t f, int lane) {
#pragma unroll
  for (int d = 1; d < APM_WAVE; d <<= 1) {
    const uint32_t o = __shfl_up(f, d, APM_WAVE);
    if (lane >= d) f = fcompose(f, o);
  }
  return f;
}

// (also the folded fills of the join's counters and per-event output counts: the grid covers
// max(n_chunks, n_ev) + 1 lanes, and it runs before any kernel that touches them)
// (also the batch's zero fills of the join stream: the JoinCounts prefix, out_cnt, the audit
// carry of the next generation and the per-file first-chunk marks -- one launch, no memsets)
__global__ __launch_bounds__(TB) void k_chunk_events(const Event* __restrict__ ev, uint32_t n_ev, uint32_t n_chunks, uint32_t* __restrict__ lo,
                               uint32_t* __restrict__ zero_words, uint32_t n_zero_words, uint32_t* __restrict__ out_cnt,
                               uint32_t* __restrict__ carry_words, uint32_t n_carry_words,
                               uint32_t* __restrict__ first_chunk, uint32_t n_files) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < n_zero_words) zero_words[c] = 0;
  if (c <= n_ev) out_cnt[c] = 0;
  if (c < n_carry_words) carry_words[c] = 0;
  if (c < n_files) first_chunk[c] = 0xffffffffu;
  // lo[k] = first event of chunk k (events are in chunk order): lane i owns the chunk boundaries
  // between event i - 1 and event i -- two loads, no search (a binary search per chunk was ~16
  // dependent global loads deep, 27 us a batch for ~24 chunks)
  if (c > n_ev) return;
  const uint32_t prev = c == 0 ? 0u : ev[c - 1].chunk + 1u;  // chunks < prev start before event c
  const uint32_t cur = c == n_ev ? n_chunks + 1u : min(ev[c].chunk, n_chunks) + 1u;
  for (uint32_t k = prev; k < cur && k <= n_chunks; ++k) lo[k] = c;
}

__global__ __launch_bounds__(APM_WAVE) void k_soap_summary(DJArgs a) {
  const uint32_t c = blockIdx.x;
  const int g = blockIdx.y;
  if (c >= a.n_chunks || a.chunk_kind[c] != FILE_SOAP) return;
  const int lane = threadIdx.x;
  uint32_t lo, hi;
  soap_range(a.chunk_ev_lo, c, g, lo, hi);
  uint32_t acc = F_ID;
  for (uint32_t base = lo; base < hi; base += APM_WAVE) {
    const uint32_t i = base + lane;
    const uint32_t f = i < hi ? code_fn(a.soap_code[i], i) : F_ID;
    const uint32_t inc = wave_fscan(f, lane);
    acc = fcompose(__shfl(inc, APM_WAVE - 1, APM_WAVE), acc);
  }
  if (lane == 0) a.seg_f[(size_t)c * SOAP_SEGS + g] = acc;
}

__global__ __launch_bounds__(64) void k_soap_carry(DJArgs a) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= a.n_chunks || a.chunk_kind[c] != FILE_SOAP || !a.chunk_first[c]) return;
  const int32_t file = (int32_t)a.chunk_file[c];
  const SoapState s0 = a.soap_state[file];
  const uint64_t h0 = s0.lid_hash;
  uint32_t st = F_CONST | (uint32_t)s0.tag;  // L = 0: the carried context
  for (int32_t d = (int32_t)c; d >= 0; d = a.chunk_next[d]) {
    a.chain_hash[d] = h0;
    for (int g = 0; g < SOAP_SEGS; ++g) {
      a.seg_in[(size_t)d * SOAP_SEGS + g] = st;
      st = fcompose(a.seg_f[(size_t)d * SOAP_SEGS + g], st);
    }
  }
  SoapState s1;
  s1.tag = (int32_t)(st & 3u);
  s1.undef = 0;
  const uint32_t L = (st & ~F_CONST) >> 2;
  s1.lid_hash = s1.tag == 0 ? 0 : (L == 0 ? h0 : a.soap_hash[L - 1]);
  a.soap_state[file] = s1;
}

__global__ __launch_bounds__(APM_WAVE) void k_soap_apply(DJArgs a) {
  const uint32_t c = blockIdx.x;
  const int g = blockIdx.y;
  if (c >= a.n_chunks || a.chunk_kind[c] != FILE_SOAP) return;
  const int lane = threadIdx.x;
  uint32_t lo, hi;
  soap_range(a.chunk_ev_lo, c, g, lo, hi);
  if (lo >= hi) return;
  uint32_t st = a.seg_in[(size_t)c * SOAP_SEGS + g];
  const uint64_t h0 = a.chain_hash[c];
  const int32_t server = a.file_server[a.chunk_file[c]];
  const uint64_t skey = a.file_skey[a.chunk_file[c]];
  for (uint32_t base = lo; base < hi; base += APM_WAVE) {
    const uint32_t i = base + lane;
    const uint8_t code = i < hi ? a.soap_code[i] : SC_NONE;
    const uint32_t f = code_fn(code, i);
    const uint32_t inc = wave_fscan(f, lane);
    uint32_t exc = __shfl_up(inc, 1, APM_WAVE);
    if (lane == 0) exc = F_ID;
    const uint32_t before = fcompose(exc, st);
    const uint32_t tag = before & 3u;
    if ((code == SC_ACCT && tag != 0) || (code == SC_VALUE && tag == 2)) {
      const uint32_t L = (before & ~F_CONST) >> 2;
      const uint64_t h = L == 0 ? h0 : a.soap_hash[L - 1];
      JOp op = a.ops[i];
      op.op = JOP_ACCT;
      op.gkey = gkey_of(h, skey);
      op.num = a.soap_num[i];
      op.server = server;
      a.ops[i] = op;
    }
    st = fcompose(__shfl(inc, APM_WAVE - 1, APM_WAVE), st);
  }
}

// ------------------------------------------------------------------------ audit trail (K5)
// See devjoin_types.h "audit trail".  Kernels (join stream, after k_build_ops wrote a.aud):
//   k_aud_keys   sort input: carried map entries, then this batch's MAP / HDR events
//   radix sort   by (file, auditTrailId) key, stable
//   k_aud_autr   one lane per key: MAP sets the entry, HDR consumes it (AF_HDR_OK + its logId /
//                alt on the HDR's AudF); the entry still live at the end is carried
//   k_aud_chunks walk-list range of each chunk, first chunk of each file
//   k_aud_walk   one lane per block (HDR_OK) + one per file with a carried open block
__device__ __forceinline__ const uint8_t* aud_src(const DJArgs& a, uint8_t flags, uint32_t ref) {
  if (flags & AF_SRC_HOST) return a.hbuf + ref;
  if (flags & AF_SRC_AUD) return (const uint8_t*)a.gin.txt + ref;
  return a.bytes + ref;
}

// copy `len` bytes into the next generation's text; returns the offset (AUD_NIL: over capacity)
__device__ uint32_t aud_put_txt(const DJArgs& a, const uint8_t* src, uint32_t len) {
  if (!len) return 0;
  const uint32_t o = atomicAdd(&a.counts->aud_txt_n, len);
  if ((uint64_t)o + len > a.gout.cap_txt) { atomicAdd(&a.counts->aud_pad, 1u); return AUD_NIL; }
  for (uint32_t j = 0; j < len; ++j) a.gout.txt[o + j] = (char)src[j];
  return o;
}

__global__ __launch_bounds__(TB) void k_aud_keys(DJArgs a) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t nc = a.gin.n_autr;
  if (j >= nc + a.n_mh) return;
  a.aud_key[j] = j < nc ? a.gin.autr[j].key : a.aud[a.mh_idx[j - nc]].h_item;
  a.aud_ord[j] = j;
}

__global__ __launch_bounds__(TB) void k_aud_autr(DJArgs a) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t nc = a.gin.n_autr, N = nc + a.n_mh;
  if (j >= N) return;
  const uint64_t key = a.aud_key_sorted[j];
  if (j > 0 && a.aud_key_sorted[j - 1] == key) return;
  bool have = false;
  uint8_t src = 0;
  uint32_t ref = 0, len = 0;
  uint64_t lh = 0;
  double alt = apm_nan();
  for (uint32_t q = j; q < N && a.aud_key_sorted[q] == key; ++q) {
    const uint32_t o = a.aud_ord_sorted[q];
    if (o < nc) {  // carried entry (sorts first: stable, carried entries precede the batch's)
      const AutrEnt t = a.gin.autr[o];
      have = true; src = AF_SRC_AUD; ref = t.lid_off; len = t.lid_len; lh = t.lid_hash; alt = t.alt;
      continue;
    }
    const uint32_t ev = a.mh_idx[o - nc];
    AudF& f = a.aud[ev];
    if (a.ev[ev].mask & PM_AUTR_MAP) {  // auditTrailIdMap[autr] = {logId, alt}
      have = true; src = f.flags & AF_SRC_HOST; ref = f.ref; len = f.len; lh = f.h_sw; alt = f.el;
    } else if (have && len > 0) {  // header: the block starts; the entry is deleted
      f.flags = (uint8_t)((f.flags & ~(AF_SRC_HOST | AF_SRC_AUD)) | AF_HDR_OK | src);
      f.ref = ref; f.len = (uint16_t)len; f.h_sw = lh; f.el = alt;
      have = false;
    } else {  // no entry (or an empty logId): an audit error, nothing changes
      atomicAdd(&a.counts->audit_errors, 1ULL);
    }
  }
  if (!have) return;
  const uint32_t k = atomicAdd(&a.counts->aud_autr_n, 1u);
  if (k >= a.gout.cap_autr) { atomicAdd(&a.counts->aud_pad, 1u); return; }
  AutrEnt t;
  t.key = key; t.lid_hash = lh; t.alt = alt; t.lid_len = len;
  t.lid_off = aud_put_txt(a, aud_src(a, src, ref), len);
  a.gout.autr[k] = t;
}

__global__ __launch_bounds__(TB) void k_aud_chunks(DJArgs a) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < a.n_chunks && a.chunk_first[c]) a.file_first_chunk[a.chunk_file[c]] = (int32_t)c;
  // walk_lo[k] = first walk position of chunk k: lane q owns the boundaries between walk
  // positions q - 1 and q (walk events are in chunk order), as k_chunk_events does for events
  const uint32_t nw = a.n_walk;
  if (c > nw) return;
  const uint32_t prev = c == 0 ? 0u : a.ev[a.walk_idx[c - 1]].chunk + 1u;
  const uint32_t cur = c == nw ? a.n_chunks + 1u : min(a.ev[a.walk_idx[c]].chunk, a.n_chunks) + 1u;
  for (uint32_t k = prev; k < cur && k <= a.n_chunks; ++k) a.walk_lo[k] = c;
}

// first walk position at or after chunk c of a file (following its chunk chain)
__device__ __forceinline__ uint32_t walk_from_chunk(const DJArgs& a, int32_t c) {
  for (; c >= 0 && (uint32_t)c < a.n_chunks; c = a.chunk_next[c])
    if (a.walk_lo[c] < a.walk_lo[c + 1]) return a.walk_lo[c];
  return AUD_NIL;
}

__device__ __forceinline__ uint32_t walk_next(const DJArgs& a, uint32_t p, uint32_t chunk) {
  if (p + 1 < a.walk_lo[chunk + 1]) return p + 1;
  return walk_from_chunk(a, a.chunk_next[chunk]);
}

struct AudWalk {  // one open audit block (AuditCtx of the host state machine)
  bool elapsed, sw, has_svc, to_db;
  uint8_t lid_src, svc_src;
  uint64_t lid_hash, svc_hash;
  double alt;
  uint32_t lid_ref, lid_len, svc_ref, svc_len;
  uint32_t head, tail;  // queued elapsed entries (item slots), insertion order
};

__global__ __launch_bounds__(64) void k_aud_walk(DJArgs a) {
  const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t nw = a.n_walk;
  if (id >= nw + a.n_files) return;
  AudWalk w;
  uint32_t p, start;
  int32_t file;
  bool carried = id >= nw;
  if (carried) {
    file = (int32_t)(id - nw);
    const AudCarry c = a.gin.carry[file];
    if (!c.active) return;
    w.elapsed = c.elapsed; w.sw = c.sw; w.has_svc = c.has_svc; w.to_db = c.svc_to_db;
    w.lid_src = AF_SRC_AUD; w.svc_src = AF_SRC_AUD;
    w.lid_hash = c.lid_hash; w.svc_hash = c.svc_hash; w.alt = c.alt;
    w.lid_ref = c.lid_off; w.lid_len = c.lid_len; w.svc_ref = c.svc_off; w.svc_len = c.svc_len;
    w.head = w.tail = AUD_NIL;
    for (uint32_t j = 0; j < c.n_items; ++j) {  // carried queue -> slots nw + items_off + j
      const uint32_t s = nw + c.items_off + j;
      AudItem it = a.gin.items[c.items_off + j];
      it.next = AUD_NIL;
      a.aud_slots[s] = it;
      if (w.tail == AUD_NIL) w.head = s; else a.aud_slots[w.tail].next = s;
      w.tail = s;
    }
    start = AUD_NIL;
    p = walk_from_chunk(a, a.file_first_chunk[file]);
  } else {
    const uint32_t ev = a.walk_idx[id];
    if (!(a.aud[ev].flags & AF_HDR_OK)) return;
    file = (int32_t)a.chunk_file[a.ev[ev].chunk];
    start = p = id;
  }
  const int32_t server = a.file_server[file];
  const uint64_t skey = a.file_skey[file];
  while (p != AUD_NIL) {
    const uint32_t ev = a.walk_idx[p];
    const Event e = a.ev[ev];
    if (e.chunk >= a.n_chunks) break;  // (never: events are in chunk order)
    const uint32_t m = e.mask;
    const uint32_t np = walk_next(a, p, e.chunk);
    if (m & PM_AUTR_HDR) {
      const AudF f = a.aud[ev];
      if (f.flags & AF_HDR_OK) {
        if (p != start) return;  // the next block's lane takes over
        // serviceMap cleared, the block's logId / alt from the map entry
        w.elapsed = w.sw = w.has_svc = w.to_db = false;
        w.lid_src = f.flags & (AF_SRC_HOST | AF_SRC_AUD); w.lid_ref = f.ref; w.lid_len = f.len;
        w.lid_hash = f.h_sw; w.alt = f.el;
        w.svc_src = 0; w.svc_hash = 0; w.svc_ref = w.svc_len = 0;
        w.head = w.tail = AUD_NIL;
      }
      p = np;
      continue;
    }
    if (m & PM_EL_START) {
      w.elapsed = true;
    } else if (w.elapsed) {
      if (m & PM_EL_END) {
        w.elapsed = false;
      } else {  // serviceMap[service].push({elapsed})
        const AudF f = a.aud[ev];
        AudItem it;
        it.svc = f.h_item; it.el = f.el; it.start = apm_nan(); it.flags = 0; it.next = AUD_NIL;
        a.aud_slots[p] = it;
        if (w.tail == AUD_NIL) w.head = p; else a.aud_slots[w.tail].next = p;
        w.tail = p;
      }
    } else if (m & PM_SW_START) {
      w.sw = true;
    } else if (!w.sw) {
    } else if (m & PM_SW_END) {
      return;  // block closed: nothing open for this file after it
    } else if (m & PM_SW_NAME) {
      const AudF f = a.aud[ev];
      w.has_svc = true; w.svc_src = f.flags & AF_SRC_HOST; w.svc_ref = f.ref; w.svc_len = f.len;
      w.svc_hash = f.h_sw; w.to_db = (f.flags & AF_TO_DB) != 0;
    } else if (w.has_svc && w.svc_len > 0 && (m & (PM_SW_STARTTS | PM_SW_STOPTS))) {
      // the front of the active service's queue
      uint32_t prev = AUD_NIL, s = w.head;
      while (s != AUD_NIL && a.aud_slots[s].svc != w.svc_hash) { prev = s; s = a.aud_slots[s].next; }
      const AudF f = a.aud[ev];
      if (s == AUD_NIL) {
        atomicAdd(&a.counts->audit_errors, 1ULL);
      } else if (m & PM_SW_STARTTS) {
        AudItem& it = a.aud_slots[s];
        it.start = f.ts;
        it.flags = AI_START | ((f.flags & AF_TS_EMPTY) ? AI_START_EMPTY : 0u);
      } else {  // stopTime: the entry leaves the queue and becomes a transaction
        const AudItem it = a.aud_slots[s];
        if (prev == AUD_NIL) w.head = it.next; else a.aud_slots[prev].next = it.next;
        if (w.tail == s) w.tail = prev;
        JOp op;
        op.gkey = gkey_of(w.lid_hash, skey);
        op.svc = w.svc_hash;
        op.ts = f.ts;
        op.num = it.el;
        op.aux = it.start;
        op.aux2 = w.alt;
        op.line = e.line;
        op.server = server;
        op.lid = w.lid_ref; op.lid_len = (uint16_t)w.lid_len;
        op.svc_ref = w.svc_ref; op.svc_len = (uint16_t)w.svc_len;
        uint16_t fl = JF_HAS_SVC;
        if (f.flags & AF_TS_EMPTY) fl |= JF_TS_EMPTY;
        if (!(it.flags & AI_START) || (it.flags & AI_START_EMPTY)) fl |= JF_START_EMPTY;
        if (w.to_db) fl |= JF_TO_DB;
        if (w.lid_src & AF_SRC_HOST) fl |= JF_LID_HOST;
        if (w.lid_src & AF_SRC_AUD) fl |= JF_LID_AUD;
        if (w.svc_src & AF_SRC_HOST) fl |= JF_SVC_HOST;
        if (w.svc_src & AF_SRC_AUD) fl |= JF_SVC_AUD;
        op.flags = fl;
        op.op = JOP_AUDIT_TX;
        op.pad = 0; op.pad2[0] = op.pad2[1] = 0;
        a.ops[ev] = op;
      }
    }
    p = np;
  }
  // the batch ends inside this block: carry it (strings and queue into the next generation)
  AudCarry c;
  c.active = 1; c.elapsed = w.elapsed; c.sw = w.sw; c.has_svc = w.has_svc; c.svc_to_db = w.to_db;
  c.pad0[0] = c.pad0[1] = c.pad0[2] = 0;
  c.lid_hash = w.lid_hash; c.svc_hash = w.svc_hash; c.alt = w.alt;
  c.lid_len = w.lid_len; c.lid_off = aud_put_txt(a, aud_src(a, w.lid_src, w.lid_ref), w.lid_len);
  c.svc_len = w.svc_len; c.svc_off = aud_put_txt(a, aud_src(a, w.svc_src, w.svc_ref), w.svc_len);
  uint32_t n = 0;
  for (uint32_t s = w.head; s != AUD_NIL; s = a.aud_slots[s].next) ++n;
  const uint32_t o = n ? atomicAdd(&a.counts->aud_items_n, n) : 0;
  if ((uint64_t)o + n > a.gout.cap_items) {
    atomicAdd(&a.counts->aud_pad, 1u);
    n = 0;
  }
  uint32_t j = 0;
  for (uint32_t s = w.head; s != AUD_NIL && j < n; s = a.aud_slots[s].next, ++j) {
    AudItem it = a.aud_slots[s];
    it.next = 0;
    a.gout.items[o + j] = it;
  }
  c.items_off = o;
  c.n_items = n;
  a.gout.carry[file] = c;
}

// ------------------------------------------------------------------------ tables
// (`fresh`: set when this call created the key; the caller counts new keys once per wave -- a
// per-lane atomicAdd on the one n_keys_new word put ~every logId of the batch through a single
// L2 atomic unit)
// Probes the dense key array (DJArgs::keys); the claiming lane also writes the key into the slot's
// KeyState, which every later kernel reads.
__device__ uint32_t key_claim(KeyState* __restrict__ t, uint64_t* __restrict__ keys, uint32_t mask, uint64_t k,
                              int32_t server, JoinCounts* cnt, bool& fresh) {
  uint32_t h = home_of(k, mask);
  for (uint32_t probe = 0; probe <= mask; ++probe) {
    const uint32_t idx = (h + probe) & mask;
    const uint64_t cur = __hip_atomic_load(&keys[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == k) return idx;
    if (cur == 0) {
      const unsigned long long prev = atomicCAS((unsigned long long*)&keys[idx], 0ULL, (unsigned long long)k);
      if (prev == 0) {
        KeyState& s = t[idx];
        s.key = k;
        s.acct = apm_nan();
        s.acct_exp = -__builtin_inf();
        s.rec_exp = -__builtin_inf();
        s.need = -1;
        s.n_part = 0;
        s.pblk = 0;
        s.server = server;
        fresh = true;
        return idx;
      }
      if (prev == k) return idx;
    }
  }
  atomicAdd(&cnt->table_full, 1ULL);
  return 0xffffffffu;
}

__device__ int32_t reg_find(const RegSlot* __restrict__ t, uint32_t mask, uint64_t k) {
  uint32_t h = home_of(k, mask);
  for (uint32_t probe = 0; probe <= mask; ++probe) {
    const uint32_t idx = (h + probe) & mask;
    const uint64_t cur = t[idx].key;
    if (cur == k) return t[idx].raw;
    if (cur == 0) return RAW_EMPTY;
  }
  return RAW_EMPTY;
}

__global__ __launch_bounds__(TB) void k_claim(DJArgs a) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n_ev) return;
  const JOp& op = a.ops[i];
  const uint32_t cap = a.table_mask + 1;
  uint32_t key = cap + 1;  // no op
  bool fresh = false;
  if (op.op == JOP_DIRECT) key = cap;
  else if (op.op != JOP_NONE) {
    const uint32_t s = key_claim(a.table, a.keys, a.table_mask, op.gkey, op.server, a.counts, fresh);
    key = s == 0xffffffffu ? cap + 1 : s;
  }
  {  // new keys: one atomic per wave
    const uint64_t b = __ballot(fresh);
    const uint32_t lead = (uint32_t)__ffsll((unsigned long long)__ballot(1)) - 1u;
    if (b && (threadIdx.x & (APM_WAVE - 1)) == lead) atomicAdd(&a.counts->n_keys_new, (uint32_t)__popcll(b));
  }
  a.op_slot[i] = key;
  if (a.group_sort) {
    a.op_idx[i] = i;
  } else {  // push onto the key's list (the op that finds it empty leads the group)
    if (i == 0) { a.big[0] = 0; a.big[1] = 0; }
    a.op_idx[i] = key < cap ? atomicExch(&a.slot_head[key], i) : ~0u;
  }
  if (op.op != JOP_NONE && (op.flags & JF_HAS_SVC)) {
    const uint64_t k = regkey_of(op.svc, op.server);
    uint32_t h = home_of(k, a.reg_mask);
    for (uint32_t probe = 0; probe <= a.reg_mask; ++probe) {
      const uint32_t idx = (h + probe) & a.reg_mask;
      const uint64_t cur = __hip_atomic_load(&a.reg[idx].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (cur == k) break;
      if (cur == 0) {
        const unsigned long long prev = atomicCAS((unsigned long long*)&a.reg[idx].key, 0ULL, (unsigned long long)k);
        if (prev == 0) {
          a.reg[idx].raw = RAW_PENDING;
          const uint32_t m = atomicAdd(&a.counts->n_miss, 1u);
          if (m < a.miss_cap) {
            RegMiss r;
            r.svc = op.svc;
            r.server = op.server;
            r.name = op.svc_ref;
            r.name_len = op.svc_len;
            r.flags = op.flags & (JF_EJB | JF_SVC_UNDEF | JF_SVC_HOST | JF_SVC_AUD);
            r.slot = (int32_t)idx;
            a.miss[m] = r;
          }
          break;
        }
        if (prev == k) break;
      }
    }
  }
}

// ------------------------------------------------------------------------ chain-block pool
// Free block indices live in a ring: allocation takes positions [head, tail) (tail is fixed while
// the allocating kernel runs), frees append at ptail, and k_pool_fix publishes the freed ones
// (tail = ptail) once no allocating kernel is in flight.  So a block freed in a batch is never
// reused in that batch: k_write may still read a logId chain its expiry just released.  The host
// grows the pool before a batch until its free count covers the batch's worst case.
__device__ __forceinline__ uint8_t* blk_ptr(uint8_t* pool, int32_t b1) { return pool + (size_t)(b1 - 1) * CHAIN_BLK; }
__device__ __forceinline__ const uint8_t* blk_ptr(const uint8_t* pool, int32_t b1) {
  return pool + (size_t)(b1 - 1) * CHAIN_BLK;
}
__device__ __forceinline__ int32_t blk_next(const uint8_t* pool, int32_t b1) { return *(const int32_t*)blk_ptr(pool, b1); }

__device__ int32_t blk_alloc(const DJArgs& a) {
  const unsigned long long k = atomicAdd(&a.counts->pool_head, 1ULL);
  const unsigned long long tail = __hip_atomic_load(&a.counts->pool_tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (k >= tail) { atomicAdd(&a.counts->pool_fail, 1ULL); return 0; }
  const uint32_t b = a.pool_ring[k & a.pool_mask];
  *(int32_t*)(a.pool + (size_t)b * CHAIN_BLK) = 0;  // next
  return (int32_t)b + 1;
}

__device__ void chain_free(const uint8_t* pool, uint32_t* ring, uint32_t mask, JoinCounts* c, int32_t b1) {
  while (b1) {
    const int32_t nx = blk_next(pool, b1);
    const unsigned long long k = atomicAdd(&c->pool_ptail, 1ULL);
    ring[k & mask] = (uint32_t)(b1 - 1);
    b1 = nx;
  }
}

// block `bi` (0-based) of a chain
__device__ __forceinline__ int32_t chain_at(const uint8_t* pool, int32_t b1, int bi) {
  for (; bi > 0; --bi) b1 = blk_next(pool, b1);
  return b1;
}

// ---- open partials of a key (recordCache[logId] map): inline slots, then the PartBlk chain.
// A key's map holds one partial per service, so the order of the set is not observable (the
// reference only looks entries up by service and discards them on expiry).
__device__ int part_find(const DJArgs& a, const KeyState& ks, uint64_t svc) {
  int f = -1;
#pragma unroll
  for (int k = 0; k < KS_PARTS; ++k)
    if (k < ks.n_part && ks.part_svc[k] == svc) f = k;
  if (f >= 0 || ks.n_part <= KS_PARTS) return f;
  int j = KS_PARTS;
  for (int32_t b = ks.pblk; b && j < ks.n_part; b = blk_next(a.pool, b)) {
    const PartBlk* pb = (const PartBlk*)blk_ptr(a.pool, b);
    for (int k = 0; k < PBLK_N && j < ks.n_part; ++k, ++j)
      if (pb->svc[k] == svc) return j;
  }
  return -1;
}

__device__ __forceinline__ PartBlk* part_blk(const DJArgs& a, const KeyState& ks, int j) {
  return (PartBlk*)blk_ptr(a.pool, chain_at(a.pool, ks.pblk, (j - KS_PARTS) / PBLK_N));
}

__device__ double part_get_start(const DJArgs& a, const KeyState& ks, int f) {
  if (f >= KS_PARTS) return part_blk(a, ks, f)->start[(f - KS_PARTS) % PBLK_N];
  double v = 0;
#pragma unroll
  for (int k = 0; k < KS_PARTS; ++k)
    if (k == f) v = ks.part_start[k];
  return v;
}

__device__ void part_set(const DJArgs& a, KeyState& ks, int f, uint64_t svc, double start) {
  if (f >= KS_PARTS) {
    PartBlk* pb = part_blk(a, ks, f);
    pb->svc[(f - KS_PARTS) % PBLK_N] = svc;
    pb->start[(f - KS_PARTS) % PBLK_N] = start;
    return;
  }
#pragma unroll
  for (int k = 0; k < KS_PARTS; ++k)
    if (k == f) { ks.part_svc[k] = svc; ks.part_start[k] = start; }
}

__device__ bool part_append(const DJArgs& a, KeyState& ks, uint64_t svc, double start) {
  const int n = ks.n_part;
  if (n >= KS_PARTS && (n - KS_PARTS) % PBLK_N == 0) {  // the chain needs a new block
    const int32_t nb = blk_alloc(a);
    if (!nb) return false;
    atomicAdd(&a.counts->chain_parts, 1ULL);
    const int bi = (n - KS_PARTS) / PBLK_N;
    if (bi == 0) ks.pblk = nb;
    else *(int32_t*)blk_ptr(a.pool, chain_at(a.pool, ks.pblk, bi - 1)) = nb;
  }
  ks.n_part = n + 1;
  part_set(a, ks, n, svc, start);
  return true;
}

// map.delete(service): the last partial moves into the hole; an emptied tail block is freed
__device__ void part_remove(const DJArgs& a, KeyState& ks, int f) {
  const int last = ks.n_part - 1;
  if (f != last) {
    uint64_t sv = 0;
    double st = 0;
    if (last >= KS_PARTS) {
      const PartBlk* pb = part_blk(a, ks, last);
      sv = pb->svc[(last - KS_PARTS) % PBLK_N];
      st = pb->start[(last - KS_PARTS) % PBLK_N];
    } else {
#pragma unroll
      for (int k = 0; k < KS_PARTS; ++k)
        if (k == last) { sv = ks.part_svc[k]; st = ks.part_start[k]; }
    }
    part_set(a, ks, f, sv, st);
  }
  ks.n_part = last;
  if (last >= KS_PARTS && (last - KS_PARTS) % PBLK_N == 0) {
    const int bi = (last - KS_PARTS) / PBLK_N;
    if (bi == 0) {
      chain_free(a.pool, a.pool_ring, a.pool_mask, a.counts, ks.pblk);
      ks.pblk = 0;
    } else {
      int32_t* link = (int32_t*)blk_ptr(a.pool, chain_at(a.pool, ks.pblk, bi - 1));
      chain_free(a.pool, a.pool_ring, a.pool_mask, a.counts, *link);
      *link = 0;
    }
  }
}

__device__ void part_clear(const DJArgs& a, KeyState& ks) {
  if (ks.pblk) chain_free(a.pool, a.pool_ring, a.pool_mask, a.counts, ks.pblk);
  ks.pblk = 0;
  ks.n_part = 0;
}

// ------------------------------------------------------------------------ outputs
// outputRecord (:264-290): start falls back to end - elapsed; numbers pass through parseInt.
__device__ __forceinline__ TxDev make_tx(int32_t server, uint64_t svc, uint8_t src, uint32_t lid, uint32_t lid_len,
                                         double acct, double start_ms, bool start_empty, double end_ms, bool end_empty,
                                         double elapsed, bool to_db) {
  TxDev t;
  double s = start_empty ? apm_nan() : start_ms;
  const double e_for_sub = end_empty ? 0.0 : end_ms;  // JS: '' - n === -n
  if (!(s == s) || s == 0) s = e_for_sub - elapsed;
  t.start = isfinite(s) ? trunc(s) : apm_nan();
  t.end = end_empty ? apm_nan() : (isfinite(end_ms) ? trunc(end_ms) : apm_nan());
  t.acct = acct;
  t.elapsed = elapsed;
  t.svc = svc;
  t.server = server;
  t.lid = lid;
  t.lid_len = (uint16_t)lid_len;
  t.lid_src = lid_len ? src : LID_NONE;
  t.to_db = to_db ? 1 : 0;
  t.raw = -1;
  return t;
}

struct Emitter {
  TxDev* stage;
  DJOverflow* ovf;
  uint32_t* ovf_n;  // JoinCounts::pad[0]: overflow cursor
  uint32_t ev;
  uint32_t sub;
  __device__ void put(const TxDev& t) {
    if (sub < 2) {
      stage[(size_t)ev * 2 + sub] = t;
    } else {
      const uint32_t k = atomicAdd(ovf_n, 1u);
      if (k < DJ_OVF_CAP) {
        ovf[k].ev = ev;
        ovf[k].sub = sub;
        ovf[k].t = t;
      }
    }
    ++sub;
  }
};

__device__ __forceinline__ uint8_t lid_src_of(const JOp& op) {
  return (op.flags & JF_LID_HOST) ? LID_HOST : (op.flags & JF_LID_AUD) ? LID_AUD : LID_BATCH;
}

// needNumRecordCache entry of this batch's region (all share the batch's TTL clock)
__device__ int32_t need_alloc(DJArgs& a, const JOp& op, uint64_t gkey) {
  const uint32_t k = atomicAdd(&a.counts->n_need_new, 1u);
  if (k >= a.arena_limit) {
    atomicAdd(&a.counts->need_overflow, 1ULL);
    return -1;
  }
  const uint32_t idx = (uint32_t)((a.arena_base + k) & (uint64_t)(a.arena_cap - 1));
  NeedEnt& ne = a.arena[idx];
  ne.key = gkey;
  ne.exp = a.now + a.need_ttl;
  ne.created = (a.batch_no << 28) | (uint64_t)(op.line & 0xfffffffu);
  ne.server = op.server;
  ne.n = 0;
  ne.iblk = 0;
  ne.lblk = 0;
  ne.vidx = a.arena_base + k;
  uint32_t n = op.lid_len;
  const uint8_t* src = (op.flags & JF_LID_HOST) ? a.hbuf + op.lid
                      : (op.flags & JF_LID_AUD) ? (const uint8_t*)a.gin.txt + op.lid : a.bytes + op.lid;
  for (uint32_t j = 0; j < n && j < (uint32_t)NEED_LID; ++j) ne.lid[j] = (char)src[j];
  // a logId longer than the inline bytes continues in a LidBlk chain (the tx line prints it whole)
  int32_t prev = 0;
  for (uint32_t o = NEED_LID; o < n; o += LBLK_N) {
    const int32_t b = blk_alloc(a);
    if (!b) { atomicAdd(&a.counts->need_overflow, 1ULL); n = o; break; }
    atomicAdd(&a.counts->chain_lids, 1ULL);
    if (prev) *(int32_t*)blk_ptr(a.pool, prev) = b;
    else ne.lblk = b;
    LidBlk* lb = (LidBlk*)blk_ptr(a.pool, b);
    const uint32_t m = min((uint32_t)LBLK_N, n - o);
    for (uint32_t j = 0; j < m; ++j) lb->b[j] = (char)src[o + j];
    prev = b;
  }
  ne.lid_len = (int32_t)n;
  return (int32_t)idx;
}

// needMap.set(service, rec): a Map keeps the first insertion position of a service and replaces
// its value; new services append (inline items, then the NeedBlk chain)
__device__ void need_put(DJArgs& a, NeedEnt& ne, const NeedItem& it) {
  const int n = ne.n;
  for (int j = 0; j < n && j < NEED_ITEMS; ++j)
    if (ne.items[j].svc == it.svc) { ne.items[j] = it; return; }
  if (n > NEED_ITEMS) {
    int j = NEED_ITEMS;
    for (int32_t b = ne.iblk; b && j < n; b = blk_next(a.pool, b)) {
      NeedBlk* nb = (NeedBlk*)blk_ptr(a.pool, b);
      for (int k = 0; k < NBLK_N && j < n; ++k, ++j)
        if (nb->items[k].svc == it.svc) { nb->items[k] = it; return; }
    }
  }
  if (n < NEED_ITEMS) { ne.items[n] = it; ne.n = n + 1; return; }
  const int j = n - NEED_ITEMS;
  int32_t b;
  if (j % NBLK_N == 0) {
    b = blk_alloc(a);
    if (!b) { atomicAdd(&a.counts->need_overflow, 1ULL); return; }
    atomicAdd(&a.counts->chain_items, 1ULL);
    if (j == 0) ne.iblk = b;
    else *(int32_t*)blk_ptr(a.pool, chain_at(a.pool, ne.iblk, j / NBLK_N - 1)) = b;
  } else {
    b = chain_at(a.pool, ne.iblk, j / NBLK_N);
  }
  ((NeedBlk*)blk_ptr(a.pool, b))->items[j % NBLK_N] = it;
  ne.n = n + 1;
}

__device__ __forceinline__ const NeedItem& need_item(const uint8_t* pool, const NeedEnt& ne, int j, int32_t& b) {
  // j-th item; `b` = the block of item j - 1 (walks forward one block at a time)
  if (j < NEED_ITEMS) return ne.items[j];
  const int k = (j - NEED_ITEMS) % NBLK_N;
  if (k == 0) b = (j == NEED_ITEMS) ? ne.iblk : blk_next(pool, b);
  return ((const NeedBlk*)blk_ptr(pool, b))->items[k];
}

__device__ void need_drain(DJArgs& a, NeedEnt& ne, int32_t nidx, double acct, Emitter& em) {
  // saveAcctNum: every parked record of the logId is output with the new account (to_db false),
  // in insertion order (needMap.forEach)
  int32_t b = 0;
  for (int j = 0; j < ne.n; ++j) {
    const NeedItem& r = need_item(a.pool, ne, j, b);
    em.put(make_tx(ne.server, r.svc, LID_NEED, (uint32_t)nidx, (uint32_t)ne.lid_len, acct, r.start,
                   (r.flags & JF_START_EMPTY) != 0, r.end, (r.flags & JF_TS_EMPTY) != 0, r.elapsed, false));
  }
  if (ne.iblk) chain_free(a.pool, a.pool_ring, a.pool_mask, a.counts, ne.iblk);
  ne.iblk = 0;
  ne.n = 0;
}

__device__ __forceinline__ void walk_direct(const DJArgs& a, uint32_t ev) {  // JOP_DIRECT: empty logId, no cache state
  const JOp op = a.ops[ev];
  Emitter em{a.stage, a.ovf, &a.counts->pad[0], ev, 0};
  em.put(make_tx(op.server, op.svc, LID_NONE, 0, 0, (op.flags & JF_BAF) ? op.aux : apm_nan(), 0.0, true, op.ts,
                 (op.flags & JF_TS_EMPTY) != 0, op.num, false));
  a.out_cnt[ev] = em.sub;
}

template <class M>
__device__ void walk_group(DJArgs& a, uint32_t slot, const M& mem, uint32_t g);

// Slot lists (DJArgs::slot_head): the group's leader collects its members (pushed in any order)
// and walks them in line order.  Up to GW_SMALL members are kept sorted in registers -- every
// index is a compile-time one (insertion by min / max over the whole unrolled row, selection by
// a compare chain), so nothing goes to scratch memory; a larger group is queued for
// k_group_walk_big (its list is left in place).
constexpr uint32_t GW_SMALL = 16;
struct GwRow {
  uint32_t m[GW_SMALL];
  __device__ __forceinline__ void clear() {
#pragma unroll
    for (uint32_t k = 0; k < GW_SMALL; ++k) m[k] = ~0u;
  }
  // m ascending, +inf padded: m' = sorted(m + {j}) minus its largest (an +inf while not full)
  __device__ __forceinline__ void insert(uint32_t j) {
#pragma unroll
    for (uint32_t k = GW_SMALL - 1; k >= 1; --k) m[k] = min(m[k], max(m[k - 1], j));
    m[0] = min(m[0], j);
  }
  __device__ __forceinline__ uint32_t at(uint32_t q) const {
    uint32_t v = m[0];
#pragma unroll
    for (uint32_t k = 1; k < GW_SMALL; ++k) v = q == k ? m[k] : v;
    return v;
  }
};
__global__ __launch_bounds__(TB) void k_group_walk(DJArgs a) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n_ev) return;
  const uint32_t cap = a.table_mask + 1;
  if (a.group_sort) {
    const uint32_t slot = a.op_slot_sorted[i];
    if (slot > cap) return;  // no op
    if (slot == cap) { walk_direct(a, a.op_idx_sorted[i]); return; }
    if (i > 0 && a.op_slot_sorted[i - 1] == slot) return;  // not the first op of its key
    uint32_t g = 1;
    while (i + g < a.n_ev && a.op_slot_sorted[i + g] == slot) ++g;
    const uint32_t* m = a.op_idx_sorted + i;
    walk_group(a, slot, [m](uint32_t q) { return m[q]; }, g);
    return;
  }
  const uint32_t slot = a.op_slot[i];
  if (slot > cap) return;
  if (slot == cap) { walk_direct(a, i); return; }
  if (a.op_idx[i] != ~0u) return;  // not the group's leader (its list was not empty)
  GwRow m;
  m.clear();
  uint32_t g = 0;
  for (uint32_t j = a.slot_head[slot]; j != ~0u; j = a.op_idx[j]) {
    if (g == GW_SMALL) {
      a.op_slot_sorted[atomicAdd(&a.big[0], 1u)] = slot;
      return;
    }
    ++g;
    m.insert(j);
  }
  a.slot_head[slot] = ~0u;
  walk_group(a, slot, [&m](uint32_t q) { return m.at(q); }, g);
}

// Ascending sort of v[0, g) by one workgroup (LDS or global memory): a bitonic network whose merge
// steps start with the mirrored comparison, so every comparator puts the smaller value first and
// the virtual padding to a power of two (+inf past g) never moves.
__device__ void block_sort_asc(uint32_t* v, uint32_t g) {
  uint32_t np2 = 1;
  while (np2 < g) np2 <<= 1;
  for (uint32_t k = 2; k <= np2; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t t = threadIdx.x; t < np2 / 2; t += blockDim.x) {
        uint32_t lo, hi;
        if (j == (k >> 1)) {
          lo = (t / j) * k + t % j;
          hi = (t / j) * k + k - 1 - t % j;
        } else {
          lo = (t / j) * 2 * j + t % j;
          hi = lo + j;
        }
        if (hi < g) {
          const uint32_t x = v[lo], y = v[hi];
          if (x > y) { v[lo] = y; v[hi] = x; }
        }
      }
      __syncthreads();
    }
  }
}

// Groups of more than GW_SMALL ops (hot keys): one workgroup each -- thread 0 gathers the list,
// the workgroup sorts it (LDS up to GWB_LDS members), thread 0 walks it.
constexpr uint32_t GWB_LDS = 4096;
constexpr int GWB_THREADS = 256;
__global__ __launch_bounds__(GWB_THREADS) void k_group_walk_big(DJArgs a) {
  __shared__ uint32_t lds[GWB_LDS];
  __shared__ uint32_t s_g, s_off;
  const uint32_t nb = a.big[0];
  for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x) {
    const uint32_t slot = a.op_slot_sorted[b];
    if (threadIdx.x == 0) {
      uint32_t g = 0;
      for (uint32_t j = a.slot_head[slot]; j != ~0u; j = a.op_idx[j]) ++g;
      const uint32_t off = atomicAdd(&a.big[1], g);  // (members of all groups <= n_ev)
      uint32_t k = 0;
      for (uint32_t j = a.slot_head[slot]; j != ~0u; j = a.op_idx[j]) a.op_idx_sorted[off + k++] = j;
      a.slot_head[slot] = ~0u;
      s_g = g;
      s_off = off;
    }
    __syncthreads();
    const uint32_t g = s_g;
    uint32_t* v = a.op_idx_sorted + s_off;
    if (g <= GWB_LDS) {
      for (uint32_t t = threadIdx.x; t < g; t += blockDim.x) lds[t] = v[t];
      __syncthreads();
      v = lds;
    }
    block_sort_asc(v, g);
    if (threadIdx.x == 0) walk_group(a, slot, [v](uint32_t q) { return v[q]; }, g);
    __syncthreads();
  }
}

template <class M>
__device__ void walk_group(DJArgs& a, uint32_t slot, const M& mem, uint32_t g) {
  KeyState ks = a.table[slot];
  const double now = a.now;
  bool acct_live = ks.acct_exp >= now;
  if (!(ks.rec_exp >= now) && ks.n_part > 0) {  // expired recordCache entry: discarded (:220-224)
    atomicAdd(&a.counts->expired_partials, (unsigned long long)ks.n_part);
    part_clear(a, ks);
  }
  NeedEnt* ne = nullptr;
  int32_t nidx = -1;
  if (ks.need >= 0) {
    NeedEnt* c = &a.arena[ks.need];
    if (c->key == ks.key && c->exp >= now) { ne = c; nidx = ks.need; }
  }
  for (uint32_t q = 0; q < g; ++q) {
    const uint32_t ev = mem(q);
    const JOp op = a.ops[ev];
    Emitter em{a.stage, a.ovf, &a.counts->pad[0], ev, 0};
    const bool ts_empty = (op.flags & JF_TS_EMPTY) != 0;
    switch (op.op) {
      case JOP_ENTRY: {
        if (!(ks.rec_exp >= now)) { ks.rec_exp = now + a.rec_ttl; part_clear(a, ks); }
        const int f = part_find(a, ks, op.svc);
        if (f >= 0) part_set(a, ks, f, op.svc, op.ts);
        else if (!part_append(a, ks, op.svc, op.ts)) atomicAdd(&a.counts->partial_overflow, 1ULL);
        break;
      }
      case JOP_EJB_EXIT:
      case JOP_CT_EXIT: {
        const bool ct = op.op == JOP_CT_EXIT;
        const int f = (ks.rec_exp >= now) ? part_find(a, ks, op.svc) : -1;
        if (f < 0) {
          if (!ct) { atomicAdd(&a.counts->ejb_unmatched, 1ULL); break; }
          // salvageRecordAndOutput (:500-504): BAF account saved under this logId, then the
          // record is output without a logId
          if ((op.flags & JF_BAF) && (op.flags & JF_BAF_VALID)) {
            ks.acct = op.aux2; ks.acct_exp = now + a.acct_ttl; acct_live = true;
            if (ne && ne->n) need_drain(a, *ne, nidx, op.aux2, em);
          } else if (op.flags & JF_BAF) {
            atomicAdd(&a.counts->invalid_acct, 1ULL);
          }
          em.put(make_tx(op.server, op.svc, LID_NONE, 0, 0, (op.flags & JF_BAF) ? op.aux : apm_nan(), 0.0, true,
                         op.ts, ts_empty, op.num, false));
          break;
        }
        const double pstart = part_get_start(a, ks, f);
        auto remove_part = [&]() { part_remove(a, ks, f); };
        if (acct_live) {
          remove_part();
          em.put(make_tx(op.server, op.svc, lid_src_of(op), op.lid, op.lid_len, ks.acct, pstart, false, op.ts,
                         ts_empty, op.num, false));
          break;
        }
        if (!ne) { nidx = need_alloc(a, op, ks.key); ne = nidx >= 0 ? &a.arena[nidx] : nullptr; ks.need = nidx; }
        double alt = apm_nan();
        if (ct && (op.flags & JF_BAF)) {
          alt = op.aux;
          if (op.flags & JF_BAF_VALID) {  // may drain the records parked before this one
            ks.acct = op.aux2; ks.acct_exp = now + a.acct_ttl; acct_live = true;
            if (ne && ne->n) need_drain(a, *ne, nidx, op.aux2, em);
          } else {
            atomicAdd(&a.counts->invalid_acct, 1ULL);
          }
        }
        if (ne) {
          NeedItem it;
          it.svc = op.svc; it.start = pstart; it.end = op.ts; it.elapsed = op.num; it.alt = alt;
          it.flags = ts_empty ? JF_TS_EMPTY : 0; it.pad = 0;
          need_put(a, *ne, it);
        }
        remove_part();
        break;
      }
      case JOP_ACCT: {
        ks.acct = op.num; ks.acct_exp = now + a.acct_ttl; acct_live = true;
        if (ne && ne->n) need_drain(a, *ne, nidx, op.num, em);
        break;
      }
      case JOP_AUDIT_TX: {
        const bool to_db = (op.flags & JF_TO_DB) != 0;
        if (acct_live) {
          em.put(make_tx(op.server, op.svc, lid_src_of(op), op.lid, op.lid_len, ks.acct, op.aux,
                         (op.flags & JF_START_EMPTY) != 0, op.ts, ts_empty, op.num, to_db));
          break;
        }
        if (!ne) { nidx = need_alloc(a, op, ks.key); ne = nidx >= 0 ? &a.arena[nidx] : nullptr; ks.need = nidx; }
        if (ne) {
          NeedItem it;
          it.svc = op.svc; it.start = op.aux; it.end = op.ts; it.elapsed = op.num; it.alt = op.aux2;
          it.flags = (ts_empty ? JF_TS_EMPTY : 0) | ((op.flags & JF_START_EMPTY) ? JF_START_EMPTY : 0) | (to_db ? JF_TO_DB : 0);
          it.pad = 0;
          need_put(a, *ne, it);
        }
        break;
      }
      default: break;
    }
    a.out_cnt[ev] = em.sub;
  }
  a.table[slot] = ks;
}

// ---- expiry of needNumRecordCache regions (NodeCache 'expired' -> outputRecord, :226-239)
__global__ __launch_bounds__(TB) void k_exp_keys(DJArgs a) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= a.n_exp_entries) return;
  uint64_t rem = e, v = 0;
  for (uint32_t r = 0; r < a.n_exp_regions; ++r) {
    const uint64_t n = a.exp_hi[r] - a.exp_lo[r];
    if (rem < n) { v = a.exp_lo[r] + rem; break; }
    rem -= n;
  }
  const uint32_t idx = (uint32_t)(v & (uint64_t)(a.arena_cap - 1));
  const NeedEnt& ne = a.arena[idx];
  a.exp_key[e] = ne.n > 0 ? ne.created : ~0ULL;
  a.exp_idx[e] = idx;
  if (ne.n == 0) {  // drained entry: gone (k_exp_emit clears the others)
    a.arena[idx].key = 0;
    if (ne.lblk) chain_free(a.pool, a.pool_ring, a.pool_mask, a.counts, ne.lblk);
  }
}

__global__ __launch_bounds__(TB) void k_exp_count(DJArgs a) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e > a.n_exp_entries) return;
  if (e == a.n_exp_entries) { a.exp_cnt[e] = 0; return; }
  a.exp_cnt[e] = a.exp_key_sorted[e] == ~0ULL ? 0u : (uint32_t)a.arena[a.exp_idx_sorted[e]].n;
}

__global__ void k_exp_emit(DJArgs a) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e == 0) {
    a.counts->n_exp_out = a.n_exp_entries ? a.exp_pos[a.n_exp_entries] : 0;
    atomicAdd(&a.counts->need_expired, (unsigned long long)a.counts->n_exp_out);
  }
  if (e >= a.n_exp_entries) return;
  const uint32_t n = a.exp_cnt[e];
  if (!n) return;
  const uint32_t idx = a.exp_idx_sorted[e];
  NeedEnt& ne = a.arena[idx];
  const uint32_t base = a.exp_pos[e];
  int32_t b = 0;
  for (uint32_t k = 0; k < n && base + k < a.out_cap; ++k) {
    const NeedItem& r = need_item(a.pool, ne, (int)k, b);
    a.out[base + k] = make_tx(ne.server, r.svc, LID_NEED, idx, (uint32_t)ne.lid_len, r.alt, r.start,
                              (r.flags & JF_START_EMPTY) != 0, r.end, (r.flags & JF_TS_EMPTY) != 0, r.elapsed,
                              (r.flags & JF_TO_DB) != 0);
  }
  // chains go back to the pool; their bytes stay readable until the next batch (k_write still
  // prints this entry's logId: `lblk` is left in place)
  if (ne.iblk) chain_free(a.pool, a.pool_ring, a.pool_mask, a.counts, ne.iblk);
  if (ne.lblk) chain_free(a.pool, a.pool_ring, a.pool_mask, a.counts, ne.lblk);
  ne.iblk = 0;
  ne.n = 0;
  ne.key = 0;  // the entry is gone (an expired region is reused by later batches)
}

__global__ __launch_bounds__(TB) void k_place(DJArgs a) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t base = a.counts->n_exp_out;
  if (i == 0) a.counts->n_out = base + a.out_pos[a.n_ev];
  if (i >= a.n_ev * 2) return;
  const uint32_t ev = i >> 1, sub = i & 1;
  if (sub >= a.out_cnt[ev]) return;
  const uint32_t p = base + a.out_pos[ev] + sub;
  if (p < a.out_cap) a.out[p] = a.stage[(size_t)ev * 2 + sub];
}

__global__ __launch_bounds__(TB) void k_place_ovf(DJArgs a) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t n = min(a.counts->pad[0], DJ_OVF_CAP);
  if (k >= n) return;
  const DJOverflow& o = a.ovf[k];
  const uint32_t p = a.counts->n_exp_out + a.out_pos[o.ev] + o.sub;
  if (p < a.out_cap) a.out[p] = o.t;
}

// ------------------------------------------------------------------------ format (K6)
struct U4 {
  uint32_t x, y, z, w;
};
struct U4Plus {
  __device__ __host__ U4 operator()(const U4& a, const U4& b) const { return U4{a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; }
};

__device__ __forceinline__ const char* lid_ptr(const DJFormatArgs& f, const TxDev& t) {
  switch (t.lid_src) {
    case LID_BATCH: return (const char*)f.bytes + t.lid;
    case LID_HOST: return (const char*)f.hbuf + t.lid;
    case LID_NEED: return f.arena[t.lid & (f.arena_cap - 1)].lid;
    case LID_AUD: return f.aud_txt + t.lid;
    default: return "";
  }
}

__device__ __forceinline__ bool stat_usable(const TxDev& t) { return !t.to_db && t.end == t.end && t.end >= 10000.0; }

__device__ uint32_t line_len(const DJFormatArgs& f, const TxDev& t) {
  if (t.raw < 0) return 0;
  const RawSvc rs = f.raw[t.raw];
  uint32_t n = 3 + rs.srv_len + 1 + rs.norm_len + 1 + t.lid_len + 1;
  n += js_num(nullptr, t.acct, nullptr) + 1 + js_num(nullptr, t.start, nullptr) + 1 + js_num(nullptr, t.end, nullptr) +
       1 + js_num(nullptr, t.elapsed, nullptr) + 1 + 1;
  return n + 1;  // '\n'
}

__global__ __launch_bounds__(TB) void k_resolve_len(DJFormatArgs f) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t n = f.n_out;
  U4* lens = reinterpret_cast<U4*>(f.lens);
  if (i == n) { lens[n] = U4{0, 0, 0, 0}; return; }
  if (i > n) return;
  TxDev t = f.out[i];
  const int32_t raw = reg_find(f.reg, f.reg_mask, regkey_of(t.svc, t.server));
  t.raw = raw >= 0 ? raw : -1;
  f.out[i].raw = t.raw;
  const uint32_t len = line_len(f, t);
  const bool st = stat_usable(t);
  lens[i] = U4{len, st ? 1u : 0u, t.to_db ? 0u : len, t.to_db ? len : 0u};
  if (t.to_db) atomicAdd(&f.counts->n_db, 1u);
  else if (!st) atomicAdd(&f.counts->n_dropped, 1u);
}

// Totals, the batch's ring region and the write verdict (DeviceJoin::ring_reserve's rules, from
// the head / low the host passed: the low only grows, so a stale one is the stricter bound).
__global__ void k_plan_totals(DJFormatArgs f) {
  const U4 o = reinterpret_cast<const U4*>(f.offs)[f.n_out];
  f.counts->text_bytes = o.x;
  f.counts->n_stats = o.y;
  f.counts->tx_text_bytes = o.z;
  f.counts->db_text_bytes = o.w;
  const uint64_t base = ring_place(f.ring_head, o.x, f.ring_cap);
  uint32_t v = DJ_WRITE_OK;
  if ((uint64_t)o.x > f.ring_cap / 4) v = DJ_WRITE_TOO_BIG;
  else if (base + o.x > f.ring_low + f.ring_cap) v = DJ_WRITE_RING_FULL;
  else if ((f.want_tx && o.z > f.txt_cap) || (f.want_db && o.w > f.txt_cap)) v = DJ_WRITE_TXT;
  *f.ring_pos = base;
  f.counts->pad[1] = v;
}

// One tx wire line (TransactionEntry.toCSVString) through a line writer: the head (names and
// logId: copies) and the tail (numbers: formatting) -- k_write gives them to different waves.
__device__ __forceinline__ uint32_t tx_head_len(const TxDev& t, const RawSvc& rs) {
  return 3u + rs.srv_len + 1u + rs.norm_len + 1u + t.lid_len + 1u;
}
template <class O>
__device__ __forceinline__ void tx_line_head(const DJFormatArgs& f, const TxDev& t, const RawSvc& rs, O& o);
template <class O>
__device__ __forceinline__ void tx_line_tail(const TxDev& t, const RawSvc& rs, O& o, bool& inexact) {
  o.jsnum(t.acct, inexact); o.c('|');
  o.jsnum(t.start, inexact); o.c('|');
  o.jsnum(t.end, inexact); o.c('|');
  o.jsnum(t.elapsed, inexact); o.c('|');
  o.c(rs.toplevel ? 'Y' : 'N');
  o.c('\n');
}
template <class O>
__device__ __forceinline__ void tx_line(const DJFormatArgs& f, const TxDev& t, const RawSvc& rs, O& o, bool& inexact) {
  tx_line_head(f, t, rs, o);
  tx_line_tail(t, rs, o, inexact);
}
template <class O>
__device__ __forceinline__ void tx_line_head(const DJFormatArgs& f, const TxDev& t, const RawSvc& rs, O& o) {
  o.lit("tx|");
  o.s(f.names + rs.srv_off, rs.srv_len);
  o.c('|');
  o.s(f.names + rs.norm_off, rs.norm_len);
  o.c('|');
  if (t.lid_src != LID_NEED || t.lid_len <= NEED_LID) {
    o.s(lid_ptr(f, t), t.lid_len);
  } else {
    const NeedEnt& ne = f.arena[t.lid & (f.arena_cap - 1)];
    o.s((const char*)ne.lid, NEED_LID);
    int rem = (int)t.lid_len - NEED_LID;
    for (int32_t b = ne.lblk; b && rem > 0; b = blk_next(f.pool, b)) {
      const LidBlk* lb = (const LidBlk*)blk_ptr(f.pool, b);
      const int m = rem < LBLK_N ? rem : LBLK_N;
      o.s((const char*)lb->b, m);
      rem -= m;
    }
  }
  o.c('|');
}

// The lines of consecutive tx are adjacent in the ring (and in the tx / db text).  One 64-lane
// block per 64 consecutive tx: each lane formats its ring line into an LDS stage at the line's
// offset modulo 4 (dword stores, textout.h), then the wave copies the block's byte range out one
// dword per lane per store -- 256 contiguous bytes per store instruction instead of 64 lanes
// storing into 64 lines ~95 B apart.  A block whose lines do not fit the stage (logIds of kB)
// writes its lines to the ring directly.  (The batch's ring region never wraps: ring_reserve.)
constexpr int TXW_LINES = 64;
constexpr int TXW_THREADS = 2 * TXW_LINES;  // wave 0: the lines' heads, wave 1: their tails
constexpr uint32_t TXW_LDS = 8192;
__device__ __forceinline__ void write_one(const DJFormatArgs& f, const TxDev& t, uint32_t i, uint64_t ring_base,
                                          char* staged_line);
__device__ __forceinline__ void write_tail(const DJFormatArgs& f, const TxDev& t, uint32_t i, uint64_t ring_base,
                                           char* staged_line);

__device__ __forceinline__ void txw_copy_out(const char* __restrict__ lds, char* __restrict__ out, uint32_t g0,
                                             uint32_t g1) {
  const uint32_t a0 = g0 & ~3u;
  const uint32_t nd = (g1 - a0 + 3) / 4;
  for (uint32_t d = threadIdx.x; d < nd; d += blockDim.x) {
    const uint32_t ga = a0 + 4 * d;
    if (ga >= g0 && ga + 4 <= g1) {
      *reinterpret_cast<uint32_t*>(out + ga) = *reinterpret_cast<const uint32_t*>(lds + 4 * d);
    } else {  // the block's first / last dword is shared with a neighbouring block: byte stores
      for (uint32_t b = 0; b < 4; ++b)
        if (ga + b >= g0 && ga + b < g1) out[ga + b] = lds[4 * d + b];
    }
  }
}

__global__ __launch_bounds__(TXW_THREADS) void k_write(DJFormatArgs f) {
  __shared__ __align__(16) char stage[TXW_LDS];
  if (f.counts->pad[1] != DJ_WRITE_OK) return;  // (uniform: the plan's verdict)
  const uint64_t ring_base = *f.ring_pos;
  const uint32_t j0 = blockIdx.x * TXW_LINES;
  const uint32_t j1 = min(f.n_out, j0 + TXW_LINES);
  const bool tail = threadIdx.x >= (unsigned)TXW_LINES;  // uniform per wave
  const uint32_t i = j0 + (threadIdx.x & (TXW_LINES - 1));
  const U4* offs = reinterpret_cast<const U4*>(f.offs);
  // physical ring offsets of the block's byte range (contiguous: the region does not wrap)
  const uint64_t rb = ring_base & (f.ring_cap - 1);
  const uint32_t p0 = (uint32_t)(rb + offs[j0].x), p1 = (uint32_t)(rb + offs[j1].x);
  const bool staged = p1 - (p0 & ~3u) <= TXW_LDS;  // uniform across the block
  if (i < j1) {
    const TxDev t = f.out[i];
    char* const sl = staged ? stage + ((uint32_t)(rb + offs[i].x) - (p0 & ~3u)) : nullptr;
    if (t.raw >= 0) {
      if (tail) write_tail(f, t, i, ring_base, sl);
      else write_one(f, t, i, ring_base, sl);
    }
  }
  if (staged) {
    __syncthreads();
    txw_copy_out(stage, f.ring, p0, p1);
  }
}

// the numbers of the ring line, after its head (the other wave of the block writes the head)
__device__ __forceinline__ void write_tail(const DJFormatArgs& f, const TxDev& t, uint32_t i, uint64_t ring_base,
                                           char* staged_line) {
  const U4 o = reinterpret_cast<const U4*>(f.offs)[i];
  const uint64_t vpos = ring_base + o.x;
  char* p0 = staged_line ? staged_line : f.ring + (vpos & (f.ring_cap - 1));
  const RawSvc rs = f.raw[t.raw];
  bool inexact = false;
  OutT<true> w(p0 + tx_head_len(t, rs));
  tx_line_tail(t, rs, w, inexact);
  w.finish();
}

// the head of the ring line, the tx / db stream copies of the whole line, the stats record
__device__ __forceinline__ void write_one(const DJFormatArgs& f, const TxDev& t, uint32_t i, uint64_t ring_base,
                                          char* staged_line) {
  const U4 o = reinterpret_cast<const U4*>(f.offs)[i];
  const U4 l = reinterpret_cast<const U4*>(f.lens)[i];
  const uint64_t vpos = ring_base + o.x;
  char* p0 = staged_line ? staged_line : f.ring + (vpos & (f.ring_cap - 1));
  const RawSvc rs = f.raw[t.raw];
  bool inexact = false;
  {
    OutT<true> w(p0);
    tx_line_head(f, t, rs, w);
    w.finish();
  }
  const uint32_t len = l.x;
  if (f.want_tx && !t.to_db) {
    OutT<true> w(f.txt_tx + o.z);
    tx_line(f, t, rs, w, inexact);
    w.finish();
  }
  if (f.want_db && t.to_db) {
    OutT<true> w(f.txt_db + o.w);
    tx_line(f, t, rs, w, inexact);
    w.finish();
  }
  if (l.y) {
    const uint32_t j = o.y;
    TxRec r;
    r.end_ms = (int64_t)t.end;
    const int32_t s = f.raw_series[t.raw];
    r.series = s;
    const double e = t.elapsed;
    r.elapsed = (e == e && e >= -2147483647.0 && e <= 2147483647.0) ? (int32_t)e : ELAPSED_NAN;
    f.tx[j] = r;
    f.tx_raw[j] = t.raw;
    f.tx_gid[j] = (int64_t)((vpos << 20) | (uint64_t)(len - 1));
    f.tx_bucket[j] = r.end_ms / 10000;
    if (s < 0) atomicMin(&f.raw_first[t.raw], (int32_t)j);
  }
}

__global__ __launch_bounds__(TB) void k_cands(DJFormatArgs f) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (f.counts->pad[1] != DJ_WRITE_OK || j >= f.counts->n_stats) return;
  if (j == 0 || f.tx_bmax[j] > f.tx_bmax[j - 1]) {
    const uint32_t k = atomicAdd(&f.counts->n_cand, 1u);
    f.cand[k] = j;
    f.cand_bucket[k] = f.tx_bucket[j];
  }
  const int32_t r = f.tx_raw[j];
  // raw_first[r] == j: k_write stored series -1 for tx j (the first such of raw r).  Not
  // `raw_series[r] < 0` re-read here: the stats stream's scatter of a newly resolved raw may land
  // between k_write and this kernel, and the tx would then keep series -1 unreported (a lost
  // sample, seen as a flaky st difference between two identical engines).
  if (f.raw_first[r] == (int32_t)j) {
    const uint32_t k = atomicAdd(&f.counts->n_unresolved, 1u);
    f.unresolved[2 * k] = j;
    f.unresolved[2 * k + 1] = (uint32_t)r;
  }
}

__global__ void k_reset_first(DJFormatArgs f) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (f.counts->pad[1] != DJ_WRITE_OK || j >= f.counts->n_stats) return;
  const int32_t r = f.tx_raw[j];
  if (f.raw_first[r] != INT_MAX) f.raw_first[r] = INT_MAX;
}

// ------------------------------------------------------------------------ rebuild / ring
__global__ void k_rebuild(const KeyState* __restrict__ old, uint32_t old_cap, KeyState* __restrict__ fresh,
                          uint32_t mask, const NeedEnt* __restrict__ arena, uint32_t arena_cap, double now,
                          JoinCounts* cnt, unsigned long long* live, const uint8_t* pool, uint32_t* pool_ring,
                          uint32_t pool_mask) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= old_cap) return;
  KeyState s = old[i];
  if (!s.key) return;
  const bool rec = s.rec_exp >= now && s.n_part > 0;
  const bool acct = s.acct_exp >= now;
  bool need = false;
  if (s.need >= 0) {
    const NeedEnt& ne = arena[(uint32_t)s.need & (arena_cap - 1)];
    need = ne.key == s.key && ne.exp >= now;
  }
  if (!rec && s.n_part > 0 && !(s.rec_exp >= now)) atomicAdd(&cnt->expired_partials, (unsigned long long)s.n_part);
  if (!rec && s.pblk) {  // the partials are dropped with the key (or with their expired map)
    chain_free(pool, pool_ring, pool_mask, cnt, s.pblk);
    s.pblk = 0;
  }
  if (!rec && !acct && !need) return;
  if (!(s.rec_exp >= now)) s.n_part = 0;
  uint32_t h = home_of(s.key, mask);
  for (uint32_t probe = 0; probe <= mask; ++probe) {
    const uint32_t idx = (h + probe) & mask;
    if (atomicCAS((unsigned long long*)&fresh[idx].key, 0ULL, (unsigned long long)s.key) == 0ULL) {
      fresh[idx] = s;
      atomicAdd(live, 1ULL);
      return;
    }
  }
}

// Same-size rebuild in place.  A linear-probing table is a set of clusters (maximal runs of
// occupied slots); every key's home lies in its own cluster, so dropping the dead keys of a cluster
// and re-inserting the live ones in slot order into the emptied cluster keeps every key
// reachable from its home -- cluster by cluster, with no other cluster touched.  One
// thread owns the clusters that start in its RB_SEG-slot segment (walking past the segment's end
// when a cluster does); the vacated tail slots get key 0.  No second table, no memset of one, no
// atomics on the table: k_rebuild (the growth path) reinserted every live key by CAS into a zeroed
// copy -- ~0.42 ms a rebuild at the headline's 2M slots, the periodic p99 step.
constexpr uint32_t RB_SEG = 8;

// The first cluster start of each segment, found before any slot moves (the owner of the
// previous segment's last cluster may vacate slot lo-1 while this segment is compacted).
__global__ void k_rebuild_starts(const KeyState* __restrict__ t, uint32_t cap, uint32_t* __restrict__ starts) {
  const uint32_t seg = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t n_seg = cap / RB_SEG;
  if (seg >= n_seg) return;
  const uint32_t mask = cap - 1, lo = seg * RB_SEG, hi = lo + RB_SEG;
  uint32_t p = lo;
  if (t[(lo + mask) & mask].key != 0)  // slot lo-1 occupied: the cluster through lo is not ours
    while (p < hi && t[p].key != 0) ++p;
  starts[seg] = p;
}

__device__ __forceinline__ bool rb_live(KeyState& s, const NeedEnt* __restrict__ arena, uint32_t arena_cap, double now,
                                        JoinCounts* cnt, const uint8_t* pool, uint32_t* pool_ring, uint32_t pool_mask,
                                        bool& changed) {
  // (the liveness rules of k_rebuild)
  const bool rec = s.rec_exp >= now && s.n_part > 0;
  const bool acct = s.acct_exp >= now;
  bool need = false;
  if (s.need >= 0) {
    const NeedEnt& ne = arena[(uint32_t)s.need & (arena_cap - 1)];
    need = ne.key == s.key && ne.exp >= now;
  }
  if (!rec && s.n_part > 0 && !(s.rec_exp >= now)) atomicAdd(&cnt->expired_partials, (unsigned long long)s.n_part);
  if (!rec && s.pblk) {
    chain_free(pool, pool_ring, pool_mask, cnt, s.pblk);
    s.pblk = 0;
    changed = true;
  }
  if (!rec && !acct && !need) return false;
  if (!(s.rec_exp >= now) && s.n_part != 0) { s.n_part = 0; changed = true; }
  return true;
}

constexpr int RB_TB = 128;      // threads per block of k_rebuild_inplace
constexpr int RB_BITS = 1024;   // longest cluster compacted (longer ones are left as they are)
__global__ __launch_bounds__(RB_TB) void k_rebuild_inplace(KeyState* __restrict__ t, uint32_t cap,
                                                           const uint32_t* __restrict__ starts,
                                                           const NeedEnt* __restrict__ arena, uint32_t arena_cap,
                                                           double now, JoinCounts* cnt, unsigned long long* live,
                                                           const uint8_t* pool, uint32_t* pool_ring, uint32_t pool_mask) {
  // per thread: which slots of its current cluster hold a placed key (LDS, 128 B a thread)
  __shared__ uint32_t occ_s[RB_TB][RB_BITS / 32];
  uint32_t* occ = occ_s[threadIdx.x];
  const uint32_t seg = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t n_seg = cap / RB_SEG;
  uint32_t n_live = 0;
  if (seg < n_seg) {
    const uint32_t mask = cap - 1, hi = seg * RB_SEG + RB_SEG;
    uint64_t p = starts[seg];  // (unwrapped positions: a cluster may run past the table's end)
    while (p < hi) {
      if (t[p & mask].key == 0) { ++p; continue; }
      uint64_t q = p;
      while (t[q & mask].key != 0 && q < p + cap) ++q;  // the cluster is [p, q) (bounded: a full table)
      const uint32_t L = (uint32_t)(q - p);
      if (L > RB_BITS) {  // (not at <= 5/8 load in practice) left as it is: its keys count as live
        n_live += L;
        p = q + 1;
        continue;
      }
      for (uint32_t i = 0; i < (L + 31) / 32; ++i) occ[i] = 0;
      // The live keys re-inserted in slot order into the emptied cluster: each at the first free
      // slot at or after its home.  A key never lands past its old slot (the keys placed before
      // it came from slots before it, each no later than it was), so the walk reads every slot
      // before anything is written there.
      for (uint64_t r = p; r < q; ++r) {
        KeyState s = t[r & mask];
        bool changed = false;
        if (!rb_live(s, arena, arena_cap, now, cnt, pool, pool_ring, pool_mask, changed)) continue;
        uint32_t i = (uint32_t)(r - (((uint32_t)r - home_of(s.key, mask)) & mask) - p);  // home, from p
        while (i < L && (occ[i >> 5] & (1u << (i & 31)))) ++i;  // (<= r - p, see above)
        if (i >= L) i = (uint32_t)(r - p);  // (unreachable; keeps the LDS index in range)
        occ[i >> 5] |= 1u << (i & 31);
        if (p + i != r || changed) t[(p + i) & mask] = s;
        ++n_live;
      }
      for (uint32_t i = 0; i < L; ++i)  // every slot no key was placed in is empty now
        if (!(occ[i >> 5] & (1u << (i & 31)))) t[(p + i) & mask].key = 0;
      p = q + 1;
    }
  }
  for (int o = APM_WAVE / 2; o > 0; o >>= 1) n_live += __shfl_xor(n_live, o, APM_WAVE);
  if ((threadIdx.x & (APM_WAVE - 1)) == 0 && n_live) atomicAdd(live, (unsigned long long)n_live);
}

__global__ __launch_bounds__(TB) void k_rebase_gids(const int64_t* __restrict__ gid, int64_t n,
                                                    const uint32_t* __restrict__ offs, uint64_t base,
                                                    int64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (int64_t)(((base + offs[i]) << 20) | ((uint64_t)gid[i] & 0xfffffu));
}

__global__ void k_gather_len(const int64_t* __restrict__ gid, int64_t n_upper, const int64_t* __restrict__ d_n,
                             uint32_t* __restrict__ lens) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > n_upper) return;
  const int64_t n = d_n ? *d_n : n_upper;
  lens[i] = i >= n ? 0u : (uint32_t)((uint64_t)gid[i] & 0xfffffu) + 1u;
}

// Released lines out of the text ring into one contiguous blob, line-block-centric.  A block
// owns GL_LINES consecutive output lines: their offsets and ring positions are staged in LDS by
// one coalesced load, then the block's lanes copy the block's byte range in 16-byte output
// chunks -- the chunk's line by a binary search over the LDS offsets, the bytes by aligned
// 16-byte ring loads and a byte funnel shift (v_alignbyte), two lines merged by a byte mask,
// one 16-byte store.  (The previous output-centric kernel searched the line offsets in HBM: a
// chain of ~20 dependent global loads per block before any byte moved -- 22-26 GB/s.)
constexpr int GL_LINES = 128;
constexpr int GL_TB = 256;

// 16 bytes at byte offset o (0..16) of the 32-byte window w[0..7]
__device__ __forceinline__ uint4 window16(const uint32_t (&w)[8], uint32_t o) {
  const uint32_t q = o >> 2, rb = o & 3u;
  uint32_t d[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const uint32_t a0 = w[k < 8 ? k : 7], a1 = w[k + 1 < 8 ? k + 1 : 7], a2 = w[k + 2 < 8 ? k + 2 : 7],
                   a3 = w[k + 3 < 8 ? k + 3 : 7], a4 = w[k + 4 < 8 ? k + 4 : 7];
    d[k] = q == 0 ? a0 : q == 1 ? a1 : q == 2 ? a2 : q == 3 ? a3 : a4;
  }
  uint4 r;
  r.x = __builtin_amdgcn_alignbyte(d[1], d[0], rb);
  r.y = __builtin_amdgcn_alignbyte(d[2], d[1], rb);
  r.z = __builtin_amdgcn_alignbyte(d[3], d[2], rb);
  r.w = __builtin_amdgcn_alignbyte(d[4], d[3], rb);
  return r;
}

// 16 bytes starting at p, of which only the first `avail` (>= 1) are known to be inside the
// line (the ring allocation): the second aligned block is loaded only when those bytes reach it.
__device__ __forceinline__ uint4 load_line16(const char* p, uint32_t avail) {
  const uint32_t sh = (uint32_t)((uintptr_t)p & 15u);
  const uint4* pa = reinterpret_cast<const uint4*>(p - sh);
  const uint4 v0 = pa[0];
  const uint4 v1 = sh + avail > 16u ? pa[1] : v0;
  const uint32_t w[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
  return window16(w, sh);
}

// bytes [0, k) from a, [k, 16) from b
__device__ __forceinline__ uint4 merge16(uint4 a, uint4 b, uint32_t k) {
  auto m = [k](uint32_t x, uint32_t y, uint32_t i) -> uint32_t {
    const uint32_t lo = 4u * i;
    if (k >= lo + 4u) return x;
    if (k <= lo) return y;
    const uint32_t mask = (1u << (8u * (k - lo))) - 1u;
    return (x & mask) | (y & ~mask);
  };
  return make_uint4(m(a.x, b.x, 0), m(a.y, b.y, 1), m(a.z, b.z, 2), m(a.w, b.w, 3));
}

__global__ __launch_bounds__(GL_TB) void k_gather_lines(const int64_t* __restrict__ gid, int64_t n,
                                                        const char* __restrict__ ring, uint64_t ring_cap,
                                                        const uint32_t* __restrict__ offs, char* __restrict__ out) {
  __shared__ uint32_t s_off[GL_LINES + 1];
  __shared__ uint64_t s_src[GL_LINES];
  const int64_t l0 = (int64_t)blockIdx.x * GL_LINES;
  const int cnt = (int)min<int64_t>(GL_LINES, n - l0);
  for (int i = threadIdx.x; i <= cnt; i += GL_TB) s_off[i] = offs[l0 + i];
  for (int i = threadIdx.x; i < cnt; i += GL_TB) s_src[i] = ((uint64_t)gid[l0 + i] >> 20) & (ring_cap - 1);
  __syncthreads();
  const uint32_t O0 = s_off[0], O1 = s_off[cnt];
  const uint32_t c0 = O0 >> 4, c1 = (O1 + 15u) >> 4;
  int lo_hint = 0;
  for (uint32_t c = c0 + threadIdx.x; c < c1; c += GL_TB) {
    const uint32_t p = c << 4;
    // last line l with s_off[l] <= max(p, O0) (chunks advance, so the search starts at the hint)
    const uint32_t q = p < O0 ? O0 : p;
    int lo = lo_hint, hi = cnt;
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (s_off[mid] <= q) lo = mid; else hi = mid;
    }
    lo_hint = lo;
    if (p >= O0 && p + 16u <= O1) {
      const uint32_t eA = s_off[lo + 1];
      const char* a = ring + s_src[lo] + (p - s_off[lo]);
      if (p + 16u <= eA) {  // one line
        *reinterpret_cast<uint4*>(out + p) = load_line16(a, 16u);
        continue;
      }
      if (lo + 2 <= cnt && p + 16u <= s_off[lo + 2]) {  // two lines: A's tail, then B's head
        const uint32_t dA = eA - p;  // 1..15
        const uint4 va = load_line16(a, dA);
        const uint4 vb = load_line16(ring + s_src[lo + 1], 16u - dA);
        const uint32_t w[8] = {0u, 0u, 0u, 0u, vb.x, vb.y, vb.z, vb.w};
        *reinterpret_cast<uint4*>(out + p) = merge16(va, window16(w, 16u - dA), dA);
        continue;
      }
    }
    // block edges (bytes of a neighbouring block are not ours) and chunks over 3+ lines: bytes
    int l = lo;
    for (uint32_t k = 0; k < 16u; ++k) {
      const uint32_t pos = p + k;
      if (pos < O0) continue;
      if (pos >= O1) break;
      while (pos >= s_off[l + 1]) ++l;
      out[pos] = ring[s_src[l] + (pos - s_off[l])];
    }
  }
}

// Join-cache occupancy at clock `now` (the reference's CACHE_STATS, stream_parse_transactions.js:
// 329-335): [0] occupied table slots, [1] acctCache entries live, [2] recordCache entries live,
// [3] open partials in them, [4] needNumRecordCache entries (parked logIds).  Grid-stride, wave
// reduction, one atomic per wave per counter.
__global__ __launch_bounds__(256) void k_cache_stats(const KeyState* __restrict__ t, uint32_t cap, double now,
                                                     unsigned long long* __restrict__ out) {
  unsigned long long c[5] = {0, 0, 0, 0, 0};
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += gridDim.x * blockDim.x) {
    const KeyState& k = t[i];
    if (!k.key) continue;
    c[0] += 1;
    c[1] += k.acct_exp >= now;
    const bool rec = k.rec_exp >= now && k.n_part > 0;
    c[2] += rec;
    c[3] += rec ? (unsigned long long)k.n_part : 0ull;
    c[4] += k.need >= 0;
  }
  for (int j = 0; j < 5; ++j) {
    unsigned long long v = c[j];
    for (int o = APM_WAVE / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, APM_WAVE);
    if ((threadIdx.x & (APM_WAVE - 1)) == 0 && v) atomicAdd(out + j, v);
  }
}

__global__ __launch_bounds__(1024) void k_min_pos(const int64_t* __restrict__ gid, int64_t n, unsigned long long* out) {
  // grid-stride per lane, wave shuffle, one LDS pass per block, one atomic per block (a single
  // atomicMin per wave on one address serialised ~6k waves in the L2 atomic unit: 81 us)
  __shared__ unsigned long long red[1024 / APM_WAVE];
  // four independent loads in flight per lane per step: one load per step left every lane
  // waiting a full HBM latency per element
  unsigned long long v = ~0ULL;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    const uint64_t g0 = (uint64_t)gid[i], g1 = (uint64_t)gid[i + stride];
    const uint64_t g2 = (uint64_t)gid[i + 2 * stride], g3 = (uint64_t)gid[i + 3 * stride];
    const unsigned long long a = (g0 >> 20) < (g1 >> 20) ? (g0 >> 20) : (g1 >> 20);
    const unsigned long long b = (g2 >> 20) < (g3 >> 20) ? (g2 >> 20) : (g3 >> 20);
    const unsigned long long m = a < b ? a : b;
    v = m < v ? m : v;
  }
  for (; i < n; i += stride) {
    const unsigned long long p = (unsigned long long)((uint64_t)gid[i] >> 20);
    v = p < v ? p : v;
  }
  for (int o = APM_WAVE / 2; o > 0; o >>= 1) {
    const unsigned long long x = __shfl_xor(v, o, APM_WAVE);
    v = x < v ? x : v;
  }
  if ((threadIdx.x & (APM_WAVE - 1)) == 0) red[threadIdx.x / APM_WAVE] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)(blockDim.x / APM_WAVE); ++w) v = red[w] < v ? red[w] : v;
    if (v != ~0ULL) atomicMin(out, v);
  }
}

__global__ void k_relocate(int64_t* __restrict__ gid, int64_t n, char* __restrict__ ring, uint64_t ring_cap,
                           uint64_t below, uint64_t dst_base, unsigned long long* cursor) {
  const int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / APM_WAVE;
  const int lane = threadIdx.x & (APM_WAVE - 1);
  if (w >= n) return;
  const uint64_t g = (uint64_t)gid[w];
  const uint64_t pos = g >> 20;
  if (pos >= below) return;
  const uint32_t len = (uint32_t)(g & 0xfffffu) + 1u;
  unsigned long long at = 0;
  if (lane == 0) at = atomicAdd(cursor, (unsigned long long)len);
  at = __shfl(at, 0, APM_WAVE);
  const uint64_t np = dst_base + at;
  const char* src = ring + (pos & (ring_cap - 1));
  char* dst = ring + (np & (ring_cap - 1));
  for (uint32_t k = lane; k < len; k += APM_WAVE) dst[k] = src[k];
  if (lane == 0) gid[w] = (int64_t)((np << 20) | (g & 0xfffffu));
}

// ------------------------------------------------------------------------ pool / arena upkeep
__global__ void k_pool_fix(JoinCounts* c) {
  const unsigned long long h = c->pool_head, t = c->pool_tail;
  c->pool_head = h < t ? h : t;  // failed allocations overshoot head
  c->pool_tail = c->pool_ptail;
}

__global__ void k_pool_init(uint32_t* ring, uint32_t n, JoinCounts* c) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) ring[i] = i;
  if (i == 0) { c->pool_head = 0; c->pool_tail = n; c->pool_ptail = n; }
}

__global__ void k_pool_grow(const uint32_t* __restrict__ old_ring, uint32_t old_mask, uint32_t* __restrict__ fresh,
                            uint32_t old_n, uint32_t new_n, const JoinCounts* c) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned long long head = c->pool_head;
  const uint32_t avail = (uint32_t)(c->pool_tail - head);
  if (i < avail) fresh[i] = old_ring[(head + i) & old_mask];
  else if (i < avail + (new_n - old_n)) fresh[i] = old_n + (i - avail);
}

__global__ void k_pool_grow_set(JoinCounts* c, uint32_t old_n, uint32_t new_n) {
  const unsigned long long avail = c->pool_tail - c->pool_head;
  c->pool_head = 0;
  c->pool_tail = c->pool_ptail = avail + (new_n - old_n);
}

__global__ void k_arena_move(const NeedEnt* __restrict__ old, uint32_t old_cap, NeedEnt* __restrict__ fresh,
                             uint32_t fresh_cap, uint64_t lo, uint64_t n) {
  constexpr int Q = sizeof(NeedEnt) / 16;
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t e = t / Q;
  if (e >= n) return;
  const uint64_t v = lo + e;
  const uint4* s = reinterpret_cast<const uint4*>(old + (v & (old_cap - 1)));
  uint4* d = reinterpret_cast<uint4*>(fresh + (v & (fresh_cap - 1)));
  d[t % Q] = s[t % Q];
}

__global__ void k_arena_remap(KeyState* __restrict__ table, uint32_t cap, const NeedEnt* __restrict__ old,
                              uint32_t old_cap, uint32_t fresh_cap, uint64_t lo, uint64_t hi) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cap) return;
  KeyState& s = table[i];
  if (!s.key || s.need < 0) return;
  const NeedEnt& ne = old[(uint32_t)s.need & (old_cap - 1)];
  s.need = (ne.key == s.key && ne.vidx >= lo && ne.vidx < hi) ? (int32_t)(ne.vidx & (fresh_cap - 1)) : -1;
}

// ------------------------------------------------------------------------ checkpoint helpers
// chain blocks idx[0..n) (1-based) -> out[0..n), 16 bytes per lane
__global__ void k_gather_blocks(const uint8_t* __restrict__ pool, const int32_t* __restrict__ idx, uint32_t n,
                                uint8_t* __restrict__ out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  constexpr uint32_t Q = CHAIN_BLK / 16;
  if (t >= n * Q) return;
  const uint32_t b = t / Q, q = t % Q;
  reinterpret_cast<uint4*>(out)[(size_t)b * Q + q] =
      reinterpret_cast<const uint4*>(pool + (size_t)(idx[b] - 1) * CHAIN_BLK)[q];
}

// ------------------------------------------------------------------------ small helpers
__global__ void k_reg_fill(RegSlot* __restrict__ reg, const int32_t* __restrict__ pairs, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) reg[pairs[2 * i]].raw = pairs[2 * i + 1];
}

__global__ void k_scatter_i32(int32_t* __restrict__ dst, const int32_t* __restrict__ pairs, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[pairs[2 * i]] = pairs[2 * i + 1];
}

__global__ void k_fill_series(TxRec* __restrict__ tx, const int32_t* __restrict__ raw, uint32_t n,
                              const int32_t* __restrict__ raw_series, unsigned long long* __restrict__ unmapped) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (tx[i].series >= 0) return;
  const int32_t s = raw_series[raw[i]];
  tx[i].series = s;
  if (s < 0 && unmapped) atomicAdd(unmapped, 1ULL);  // series table full: counted, not silent
}

__global__ void k_gather_u8(const uint8_t* __restrict__ src, const int32_t* __restrict__ idx, uint32_t n,
                            uint8_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = src[idx[i]];
}

// number of sorted endTs <= edge (upper bound)
__global__ void k_count_le(const int64_t* __restrict__ end, int64_t n, int64_t edge, int64_t* __restrict__ out) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (end[mid] <= edge) lo = mid + 1; else hi = mid;
  }
  *out = lo;
}

__global__ void k_keys_sync(const KeyState* __restrict__ t, uint32_t cap, uint64_t* __restrict__ keys) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < cap) keys[i] = t[i].key;
}

}  // namespace
}  // namespace apm

extern "C" {
using namespace apm;

// APM_DJ_DEBUG=1: synchronize after every launch of the join and name the first that fails
// APM_DJ_MARKS=1: the host clock after each launch of the join chain (apm_dj_marks; the engine
// turns them into trace spans): where the ingest thread's launch time goes.  Diagnostics for
// one engine per process (the marks are process-wide).
static bool dj_marks_on() {
  static const bool v = [] { const char* e = std::getenv("APM_DJ_MARKS"); return e && e[0] == '1'; }();
  return v;
}
constexpr int DJ_MARKS = 64;
static double g_mark_t[DJ_MARKS];
static const char* g_mark_n[DJ_MARKS];
static int g_mark_k = 0;

static void dj_check(hipStream_t s, const char* what) {
  if (dj_marks_on() && g_mark_k < DJ_MARKS) {
    g_mark_t[g_mark_k] =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
    g_mark_n[g_mark_k++] = what;
  }
  static const bool dbg = std::getenv("APM_DJ_DEBUG") != nullptr;
  if (!dbg) return;
  const hipError_t e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    fprintf(stderr, "[devjoin debug] %s: %s\n", what, hipGetErrorString(e));
    fflush(stderr);
    abort();
  }
}

// one 4-byte field (at byte `off`) of each of n records of `stride` bytes -> out[n] (8-byte: two
// consecutive words, out[2i], out[2i+1])
__global__ void k_gather_field(const uint8_t* __restrict__ base, size_t stride, uint32_t n, int words,
                               uint32_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t* p = reinterpret_cast<const uint32_t*>(base + (size_t)i * stride);
  for (int k = 0; k < words; ++k) out[(size_t)i * words + k] = p[k];
}

void apm_dj_gather_field(const void* base, size_t stride, uint32_t n, int words, uint32_t* out, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_gather_field, dim3((n + TB - 1) / TB), dim3(TB), 0, s, (const uint8_t*)base, stride, n, words, out);
}

int apm_dj_take_marks(double* t, const char** names, int cap) {
  const int k = std::min(g_mark_k, cap);
  for (int i = 0; i < k; ++i) { t[i] = g_mark_t[i]; names[i] = g_mark_n[i]; }
  g_mark_k = 0;
  return k;
}

size_t apm_dj_tmp_bytes(uint32_t max_ev, uint32_t max_out, int table_bits) {
  size_t a = 0, b = 0, c = 0, d = 0, e = 0;
  const size_t n = std::max<size_t>(max_ev, 1) + 1;
  HIP_OK(rocprim::exclusive_scan(nullptr, a, (uint8_t*)nullptr, (uint32_t*)nullptr, 0u, n, rocprim::plus<uint32_t>(),
                                 (hipStream_t)0));
  HIP_OK(rocprim::radix_sort_pairs<OpSortCfg>(nullptr, b, (uint32_t*)nullptr, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                   (uint32_t*)nullptr, n, 0, op_sort_bits(table_bits), (hipStream_t)0));
  {
    size_t b11 = 0;
    HIP_OK(rocprim::radix_sort_pairs<OpSortCfg11>(nullptr, b11, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                                  (uint32_t*)nullptr, (uint32_t*)nullptr, n, 0, op_sort_bits(table_bits),
                                                  (hipStream_t)0));
    b = std::max(b, b11);
  }
  HIP_OK(rocprim::radix_sort_pairs(nullptr, c, (uint64_t*)nullptr, (uint64_t*)nullptr, (uint32_t*)nullptr,
                                   (uint32_t*)nullptr, n, 0, 64, (hipStream_t)0));
  HIP_OK(rocprim::exclusive_scan(nullptr, d, (U4*)nullptr, (U4*)nullptr, U4{0, 0, 0, 0}, (size_t)max_out + 1, U4Plus(),
                                 (hipStream_t)0));
  HIP_OK(rocprim::inclusive_scan(nullptr, e, (int64_t*)nullptr, (int64_t*)nullptr, (size_t)max_out + 1,
                                 rocprim::maximum<int64_t>(), (hipStream_t)0));
  size_t f = 0;
  HIP_OK(rocprim::exclusive_scan(nullptr, f, (uint64_t*)nullptr, (uint64_t*)nullptr, (uint64_t)0, n,
                                 rocprim::plus<uint64_t>(), (hipStream_t)0));
  return std::max(std::max(std::max(a, b), std::max(c, d)), std::max(e, f)) + 4096;
}

static int pre_bytewise() {
  static const int v = [] { const char* e = std::getenv("APM_PRE_BYTEWISE"); return e && e[0] == '1' ? 1 : 0; }();
  return v;
}
static int hf_split() {
  static const int v = [] { const char* e = std::getenv("APM_HF_SPLIT"); return e && e[0] == '0' ? 0 : 1; }();
  return v;
}
static int hf_staged() {
  static const int v = [] { const char* e = std::getenv("APM_HF_STAGE"); return e && e[0] == '0' ? 0 : 1; }();
  return v;
}
int apm_dj_select_host(DJArgs* a, const uint32_t* d_n_ev, uint32_t max_ev, hipStream_t s) {
  HIP_OK(hipMemsetAsync(a->n_host, 0, sizeof(SelCount), s));
  if (max_ev == 0) return 0;
  // the listed byte events: scratch in sel_pos (written by the selection scan only afterwards;
  // max_ev + 64 u64 words hold the max_ev u32 list entries and the two counts)
  const int split = hf_split();
  uint32_t* list = reinterpret_cast<uint32_t*>(a->sel_pos);
  uint32_t* list_n = list + max_ev;
  if (split) HIP_OK(hipMemsetAsync(list_n, 0, 8, s));
  const dim3 grid((max_ev + TB - 1) / TB);
  if (split)
    hipLaunchKernelGGL(k_host_flags<true>, grid, dim3(TB), 0, s, a->ev, d_n_ev, a->bytes, a->chunk_file, a->file_fkey,
                       a->host_flag, a->sel_val, a->aud, a->n_host, max_ev, pre_bytewise(), hf_staged(), list, list_n);
  else
    hipLaunchKernelGGL(k_host_flags<false>, grid, dim3(TB), 0, s, a->ev, d_n_ev, a->bytes, a->chunk_file, a->file_fkey,
                       a->host_flag, a->sel_val, a->aud, a->n_host, max_ev, pre_bytewise(), hf_staged(), list, list_n);
  dj_check(s, "k_host_flags");
  if (split) {
    hipLaunchKernelGGL(k_host_flags_bytes, grid, dim3(TB), 0, s, a->ev, a->bytes, a->chunk_file, a->file_fkey,
                       a->host_flag, a->sel_val, a->aud, max_ev, pre_bytewise(), hf_staged(), list, list_n);
    dj_check(s, "k_host_flags_bytes");
  }
  // sel_pos: the tile sums, then the packed total (sel_pos has max_ev + 64 entries)
  uint64_t* total = a->sel_pos + (max_ev + DS_TILE - 1) / DS_TILE + 1;
  if (ds_scan_apply<uint64_t>(SelValF{a->sel_val},
                              SelScatterG{a->ev, a->host_flag, total, a->host_ev, a->host_ev_idx, a->mh_idx,
                                          a->walk_idx, a->n_host},
                              d_n_ev, max_ev, a->sel_pos, total, s) != 0)
    return -1;
  dj_check(s, "k_ds_scan (host selection)");
  return 0;
}

// K5: map / header matching, then the block walks (their stopTime ops land in a->ops)
static int apm_dj_audit(DJArgs* a, bool filled, hipStream_t s) {
  // (filled: k_chunk_events already zeroed the carry and the first-chunk marks)
  if (a->n_files && !filled) HIP_OK(hipMemsetAsync(a->gout.carry, 0, (size_t)a->n_files * sizeof(AudCarry), s));
  const uint32_t N = a->gin.n_autr + a->n_mh;
  if (N) {
    hipLaunchKernelGGL(k_aud_keys, dim3((N + TB - 1) / TB), dim3(TB), 0, s, *a);
    dj_check(s, "k_aud_keys");
    size_t need = 0;
    HIP_OK(rocprim::radix_sort_pairs(nullptr, need, a->aud_key, a->aud_key_sorted, a->aud_ord, a->aud_ord_sorted,
                                     (size_t)N, 0, 64, s));
    if (need > a->tmp_bytes) return -1;
    HIP_OK(rocprim::radix_sort_pairs(a->tmp, need, a->aud_key, a->aud_key_sorted, a->aud_ord, a->aud_ord_sorted,
                                     (size_t)N, 0, 64, s));
    dj_check(s, "rocprim_radix_sort_pairs");
    hipLaunchKernelGGL(k_aud_autr, dim3((N + TB - 1) / TB), dim3(TB), 0, s, *a);
    dj_check(s, "k_aud_autr");
  }
  // an open block always carries its (non-empty) logId: no carry text, no carried block
  if (a->n_walk || a->gin.n_txt) {
    if (a->n_files && !filled) HIP_OK(hipMemsetAsync(a->file_first_chunk, 0xff, (size_t)a->n_files * 4, s));
    const uint32_t lanes = std::max(a->n_chunks + 1, a->n_walk + 1);
    hipLaunchKernelGGL(k_aud_chunks, dim3((lanes + TB - 1) / TB), dim3(TB), 0, s, *a);
    dj_check(s, "k_aud_chunks");
    const uint32_t L = a->n_walk + a->n_files;
    hipLaunchKernelGGL(k_aud_walk, dim3((L + 63) / 64), dim3(64), 0, s, *a);
    dj_check(s, "k_aud_walk");
  }
  return 0;
}

int apm_dj_join(DJArgs* a, hipStream_t s) {
  const uint32_t n = a->n_ev;
  const uint32_t cap = a->table_mask + 1;
  static_assert(offsetof(JoinCounts, ejb_unmatched) % 4 == 0, "JoinCounts zero range");
  const uint32_t zw = (uint32_t)(offsetof(JoinCounts, ejb_unmatched) / 4);
  if (n) {
    static_assert(sizeof(AudCarry) % 4 == 0, "carry words");
    const uint32_t cw = a->n_files * (uint32_t)(sizeof(AudCarry) / 4);
    const uint32_t lanes = std::max(std::max(std::max(a->n_chunks + 1, n + 1), zw), cw);
    hipLaunchKernelGGL(k_chunk_events, dim3((lanes + TB - 1) / TB), dim3(TB), 0, s, a->ev, n, a->n_chunks,
                       a->chunk_ev_lo, (uint32_t*)a->counts, zw, a->out_cnt, (uint32_t*)a->gout.carry, cw,
                       (uint32_t*)a->file_first_chunk, a->n_files);
    dj_check(s, "k_chunk_events");
    hipLaunchKernelGGL(k_build_ops, dim3((n + TB - 1) / TB), dim3(TB), 0, s, *a);
    dj_check(s, "k_build_ops");
  } else {
    HIP_OK(hipMemsetAsync(a->counts, 0, offsetof(JoinCounts, ejb_unmatched), s));
  }
  // (also for a batch without events: the carry moves to the next generation)
  if (apm_dj_audit(a, n != 0, s) != 0) return -1;
  if (n) {
    hipLaunchKernelGGL(k_soap_summary, dim3(a->n_chunks, SOAP_SEGS), dim3(APM_WAVE), 0, s, *a);
    dj_check(s, "k_soap_summary");
    hipLaunchKernelGGL(k_soap_carry, dim3((a->n_chunks + 63) / 64), dim3(64), 0, s, *a);
    dj_check(s, "k_soap_carry");
    hipLaunchKernelGGL(k_soap_apply, dim3(a->n_chunks, SOAP_SEGS), dim3(APM_WAVE), 0, s, *a);
    dj_check(s, "k_soap_apply");
    hipLaunchKernelGGL(k_claim, dim3((n + TB - 1) / TB), dim3(TB), 0, s, *a);
    dj_check(s, "k_claim");
    size_t need = 0;
    if (!a->group_sort) {
      // (slot lists: no sort)
    } else if (opsort11(a->table_bits)) {
      HIP_OK(rocprim::radix_sort_pairs<OpSortCfg11>(nullptr, need, a->op_slot, a->op_slot_sorted, a->op_idx,
                                                    a->op_idx_sorted, (size_t)n, 0, op_sort_bits(a->table_bits), s));
      if (need > a->tmp_bytes) return -1;
      HIP_OK(rocprim::radix_sort_pairs<OpSortCfg11>(a->tmp, need, a->op_slot, a->op_slot_sorted, a->op_idx,
                                                    a->op_idx_sorted, (size_t)n, 0, op_sort_bits(a->table_bits), s));
    } else {
      HIP_OK(rocprim::radix_sort_pairs<OpSortCfg>(nullptr, need, a->op_slot, a->op_slot_sorted, a->op_idx,
                                                  a->op_idx_sorted, (size_t)n, 0, op_sort_bits(a->table_bits), s));
      if (need > a->tmp_bytes) return -1;
      HIP_OK(rocprim::radix_sort_pairs<OpSortCfg>(a->tmp, need, a->op_slot, a->op_slot_sorted, a->op_idx,
                                                  a->op_idx_sorted, (size_t)n, 0, op_sort_bits(a->table_bits), s));
    }
  }
  (void)cap;
  // expiry first: its outputs precede every line emission, and it must read the expiring entries
  // before this batch's region allocations (disjoint by construction) and drains
  const uint32_t E = a->n_exp_entries;
  if (E) {
    hipLaunchKernelGGL(k_exp_keys, dim3((E + TB - 1) / TB), dim3(TB), 0, s, *a);
    dj_check(s, "k_exp_keys");
    size_t need = 0;
    HIP_OK(rocprim::radix_sort_pairs(nullptr, need, a->exp_key, a->exp_key_sorted, a->exp_idx, a->exp_idx_sorted,
                                     (size_t)E, 0, 64, s));
    if (need > a->tmp_bytes) return -1;
    HIP_OK(rocprim::radix_sort_pairs(a->tmp, need, a->exp_key, a->exp_key_sorted, a->exp_idx, a->exp_idx_sorted,
                                     (size_t)E, 0, 64, s));
    dj_check(s, "rocprim_radix_sort_pairs");
    hipLaunchKernelGGL(k_exp_count, dim3((E + 1 + TB - 1) / TB), dim3(TB), 0, s, *a);
    dj_check(s, "k_exp_count");
    need = 0;
    HIP_OK(rocprim::exclusive_scan(nullptr, need, a->exp_cnt, a->exp_pos, 0u, (size_t)E + 1,
                                   rocprim::plus<uint32_t>(), s));
    if (need > a->tmp_bytes) return -1;
    HIP_OK(rocprim::exclusive_scan(a->tmp, need, a->exp_cnt, a->exp_pos, 0u, (size_t)E + 1,
                                   rocprim::plus<uint32_t>(), s));
    dj_check(s, "rocprim_exclusive_scan");
  }
  hipLaunchKernelGGL(k_exp_emit, dim3((std::max<uint32_t>(E, 1) + TB - 1) / TB), dim3(TB), 0, s, *a);
  dj_check(s, "k_exp_emit");
  if (n) {
    hipLaunchKernelGGL(k_group_walk, dim3((n + TB - 1) / TB), dim3(TB), 0, s, *a);
    dj_check(s, "k_group_walk");
    if (!a->group_sort) {  // (a few idle workgroups when no group is big)
      hipLaunchKernelGGL(k_group_walk_big, dim3(32), dim3(GWB_THREADS), 0, s, *a);
      dj_check(s, "k_group_walk_big");
    }
    size_t need = 0;
    HIP_OK(rocprim::exclusive_scan(nullptr, need, a->out_cnt, a->out_pos, 0u, (size_t)n + 1,
                                   rocprim::plus<uint32_t>(), s));
    if (need > a->tmp_bytes) return -1;
    HIP_OK(rocprim::exclusive_scan(a->tmp, need, a->out_cnt, a->out_pos, 0u, (size_t)n + 1,
                                   rocprim::plus<uint32_t>(), s));
    dj_check(s, "rocprim_exclusive_scan");
    hipLaunchKernelGGL(k_place, dim3((2 * n + TB - 1) / TB), dim3(TB), 0, s, *a);
    dj_check(s, "k_place");
    hipLaunchKernelGGL(k_place_ovf, dim3(DJ_OVF_CAP / TB), dim3(TB), 0, s, *a);
    dj_check(s, "k_place_ovf");
  } else {
    HIP_OK(hipMemsetAsync(a->out_pos, 0, 4, s));
    hipLaunchKernelGGL(k_place, dim3(1), dim3(TB), 0, s, *a);
    dj_check(s, "k_place");
  }
  hipLaunchKernelGGL(k_pool_fix, dim3(1), dim3(1), 0, s, a->counts);
  dj_check(s, "k_pool_fix");
  return 0;
}

int apm_dj_plan(DJFormatArgs* f, hipStream_t s) {
  const uint32_t n = f->n_out;
  hipLaunchKernelGGL(k_resolve_len, dim3((n + 1 + TB - 1) / TB), dim3(TB), 0, s, *f);
  dj_check(s, "k_resolve_len");
  size_t need = 0;
  U4* lens = reinterpret_cast<U4*>(f->lens);
  U4* offs = reinterpret_cast<U4*>(f->offs);
  HIP_OK(rocprim::exclusive_scan(nullptr, need, lens, offs, U4{0, 0, 0, 0}, (size_t)n + 1, U4Plus(), s));
  if (need > f->tmp_bytes) return -1;
  HIP_OK(rocprim::exclusive_scan(f->tmp, need, lens, offs, U4{0, 0, 0, 0}, (size_t)n + 1, U4Plus(), s));
  dj_check(s, "rocprim_exclusive_scan (plan)");
  hipLaunchKernelGGL(k_plan_totals, dim3(1), dim3(1), 0, s, *f);
  dj_check(s, "k_plan_totals");
  return 0;
}

// Sized by n_out (host-known after sync A): the stats count n_stats <= n_out is on the device
// only.  The max scan runs over n_out entries -- the ones past n_stats are stale and affect no
// prefix below it.
int apm_dj_write(DJFormatArgs* f, hipStream_t s) {
  const uint32_t n = f->n_out;
  if (!n) return 0;
  hipLaunchKernelGGL(k_write, dim3((n + TXW_LINES - 1) / TXW_LINES), dim3(TXW_THREADS), 0, s, *f);
  dj_check(s, "k_write");
  size_t need = 0;
  HIP_OK(rocprim::inclusive_scan(nullptr, need, f->tx_bucket, f->tx_bmax, (size_t)n, rocprim::maximum<int64_t>(), s));
  if (need > f->tmp_bytes) return -1;
  HIP_OK(rocprim::inclusive_scan(f->tmp, need, f->tx_bucket, f->tx_bmax, (size_t)n, rocprim::maximum<int64_t>(), s));
  dj_check(s, "rocprim_inclusive_scan (bucket max)");
  hipLaunchKernelGGL(k_cands, dim3((n + TB - 1) / TB), dim3(TB), 0, s, *f);
  hipLaunchKernelGGL(k_reset_first, dim3((n + TB - 1) / TB), dim3(TB), 0, s, *f);
  dj_check(s, "k_cands+k_reset_first");
  return 0;
}

namespace {
struct KeyLive {
  __device__ bool operator()(const KeyState& k) const { return k.key != 0; }
};
}  // namespace

size_t apm_dj_live_tmp_bytes(uint32_t cap) {
  size_t b = 0;
  HIP_OK(rocprim::select(nullptr, b, (const KeyState*)nullptr, (KeyState*)nullptr, (uint32_t*)nullptr, cap, KeyLive(),
                         (hipStream_t)0));
  return b;
}

void apm_dj_live_compact(const KeyState* table, uint32_t cap, KeyState* out, uint32_t* d_n, void* tmp,
                         size_t tmp_bytes, hipStream_t s) {
  HIP_OK(rocprim::select(tmp, tmp_bytes, table, out, d_n, cap, KeyLive(), s));
}

size_t apm_dj_rebuild_scratch_bytes(uint32_t cap) { return ((size_t)cap / RB_SEG + 1) * 4; }

void apm_dj_rebuild_inplace(KeyState* table, uint32_t cap, uint32_t* scratch, const NeedEnt* arena, uint32_t arena_cap,
                            double now, JoinCounts* counts, unsigned long long* live, uint8_t* pool,
                            uint32_t* pool_ring, uint32_t pool_mask, hipStream_t s) {
  if (cap < RB_SEG || (cap & (cap - 1))) throw std::runtime_error("in-place rebuild: table size not a power of two >= 8");
  const uint32_t n_seg = cap / RB_SEG;
  hipLaunchKernelGGL(k_rebuild_starts, dim3((n_seg + TB - 1) / TB), dim3(TB), 0, s, table, cap, scratch);
  dj_check(s, "k_rebuild_starts");
  hipLaunchKernelGGL(k_rebuild_inplace, dim3((n_seg + RB_TB - 1) / RB_TB), dim3(RB_TB), 0, s, table, cap, scratch, arena,
                     arena_cap, now, counts, live, pool, pool_ring, pool_mask);
  dj_check(s, "k_rebuild_inplace");
  hipLaunchKernelGGL(k_pool_fix, dim3(1), dim3(1), 0, s, counts);
}

// Test entry (bindings: dj_rebuild_selftest): a table of `cap` slots filled to `load` by linear
// probing with random keys, a `dead` fraction of them expired (no account / record / need), the
// in-place (or, copy=true, the reinsert) rebuild run on it, and the result checked on the host.
// out: {live counted on the device, live expected, survivors reachable from their home with the
// payload they had, dead keys left, slots occupied after, probe length sum before, after, rebuild us}
std::vector<double> apm_dj_rebuild_selftest(uint32_t cap, double load, double dead, uint64_t seed, bool copy) {
  std::vector<KeyState> h(cap);
  std::memset(h.data(), 0, (size_t)cap * sizeof(KeyState));
  const uint32_t mask = cap - 1;
  uint64_t x = seed * 0x9E3779B97F4A7C15ull + 1;
  auto rnd = [&]() { x ^= x >> 12; x ^= x << 25; x ^= x >> 27; return x * 0x2545F4914F6CDD1Dull; };
  const double now = 1000.0;
  const uint32_t n = (uint32_t)(load * cap);
  uint64_t want_live = 0, probes_before = 0;
  for (uint32_t i = 0; i < n; ++i) {
    uint64_t k = rnd() | 1;
    uint32_t idx = home_of(k, mask);
    uint32_t d = 0;
    while (h[idx].key && h[idx].key != k) { idx = (idx + 1) & mask; ++d; }
    if (h[idx].key == k) continue;
    KeyState& e = h[idx];
    e.key = k;
    const bool is_dead = (double)(rnd() >> 11) * (1.0 / 9007199254740992.0) < dead;
    e.acct = (double)(k % 1000003);  // payload
    e.acct_exp = is_dead ? now - 1 : now + 10;
    e.rec_exp = -__builtin_inf();
    e.need = -1;
    e.n_part = 0;
    e.pblk = 0;
    want_live += !is_dead;
    probes_before += d;
  }
  KeyState* d_t = nullptr;
  KeyState* d_f = nullptr;
  uint32_t* d_scr = nullptr;
  NeedEnt* d_arena = nullptr;
  JoinCounts* d_c = nullptr;
  unsigned long long* d_live = nullptr;
  HIP_OK(hipMalloc((void**)&d_t, (size_t)cap * sizeof(KeyState)));
  HIP_OK(hipMalloc((void**)&d_f, (size_t)cap * sizeof(KeyState)));
  HIP_OK(hipMalloc((void**)&d_scr, apm_dj_rebuild_scratch_bytes(cap)));
  HIP_OK(hipMalloc((void**)&d_arena, sizeof(NeedEnt)));
  HIP_OK(hipMalloc((void**)&d_c, sizeof(JoinCounts)));
  HIP_OK(hipMalloc((void**)&d_live, 8));
  HIP_OK(hipMemset(d_arena, 0, sizeof(NeedEnt)));
  HIP_OK(hipMemset(d_c, 0, sizeof(JoinCounts)));
  HIP_OK(hipMemset(d_live, 0, 8));
  HIP_OK(hipMemset(d_f, 0, (size_t)cap * sizeof(KeyState)));
  HIP_OK(hipMemcpy(d_t, h.data(), (size_t)cap * sizeof(KeyState), hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  HIP_OK(hipEventCreate(&e0));
  HIP_OK(hipEventCreate(&e1));
  HIP_OK(hipEventRecord(e0, 0));
  if (copy)
    apm_dj_rebuild(d_t, cap, d_f, mask, d_arena, 1, now, d_c, d_live, nullptr, nullptr, 0, 0);
  else
    apm_dj_rebuild_inplace(d_t, cap, d_scr, d_arena, 1, now, d_c, d_live, nullptr, nullptr, 0, 0);
  HIP_OK(hipEventRecord(e1, 0));
  HIP_OK(hipEventSynchronize(e1));
  float ms = 0;
  HIP_OK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long live = 0;
  HIP_OK(hipMemcpy(&live, d_live, 8, hipMemcpyDeviceToHost));
  std::vector<KeyState> r(cap);
  HIP_OK(hipMemcpy(r.data(), copy ? d_f : d_t, (size_t)cap * sizeof(KeyState), hipMemcpyDeviceToHost));
  for (void* p : {(void*)d_t, (void*)d_f, (void*)d_scr, (void*)d_arena, (void*)d_c, (void*)d_live}) HIP_OK(hipFree(p));
  HIP_OK(hipEventDestroy(e0));
  HIP_OK(hipEventDestroy(e1));
  uint64_t found = 0, dead_left = 0, occupied = 0, probes_after = 0;
  for (uint32_t i = 0; i < cap; ++i) {
    const KeyState& e = h[i];
    if (!e.key) continue;
    uint32_t idx = home_of(e.key, mask), d = 0;
    while (r[idx].key && r[idx].key != e.key && d <= mask) { idx = (idx + 1) & mask; ++d; }
    const bool there = r[idx].key == e.key;
    if (e.acct_exp >= now) {
      found += there && r[idx].acct == e.acct && r[idx].acct_exp == e.acct_exp && r[idx].need == -1;
      probes_after += d;
    } else {
      dead_left += there;
    }
  }
  for (uint32_t i = 0; i < cap; ++i) occupied += r[i].key != 0;
  return {(double)live, (double)want_live, (double)found, (double)dead_left, (double)occupied, (double)probes_before,
          (double)probes_after, 1000.0 * ms};
}
void apm_dj_rebuild(const KeyState* old, uint32_t old_cap, KeyState* fresh, uint32_t fresh_mask, const NeedEnt* arena,
                    uint32_t arena_cap, double now, JoinCounts* counts, unsigned long long* live, uint8_t* pool,
                    uint32_t* pool_ring, uint32_t pool_mask, hipStream_t s) {
  if (old_cap)
    hipLaunchKernelGGL(k_rebuild, dim3((old_cap + TB - 1) / TB), dim3(TB), 0, s, old, old_cap, fresh, fresh_mask, arena,
                       arena_cap, now, counts, live, pool, pool_ring, pool_mask);
  hipLaunchKernelGGL(k_pool_fix, dim3(1), dim3(1), 0, s, counts);
}

void apm_dj_gather_blocks(const uint8_t* pool, const int32_t* idx, uint32_t n, uint8_t* out, hipStream_t s) {
  if (!n) return;
  const uint32_t t = n * (CHAIN_BLK / 16);
  hipLaunchKernelGGL(k_gather_blocks, dim3((t + TB - 1) / TB), dim3(TB), 0, s, pool, idx, n, out);
}

void apm_dj_pool_init(uint32_t* ring, uint32_t n, JoinCounts* counts, hipStream_t s) {
  hipLaunchKernelGGL(k_pool_init, dim3((n + TB - 1) / TB), dim3(TB), 0, s, ring, n, counts);
}

void apm_dj_pool_grow(const uint32_t* old_ring, uint32_t old_mask, uint32_t* fresh_ring, uint32_t old_n, uint32_t new_n,
                      JoinCounts* counts, hipStream_t s) {
  hipLaunchKernelGGL(k_pool_grow, dim3((new_n + TB - 1) / TB), dim3(TB), 0, s, old_ring, old_mask, fresh_ring, old_n,
                     new_n, counts);
  hipLaunchKernelGGL(k_pool_grow_set, dim3(1), dim3(1), 0, s, counts, old_n, new_n);
}

void apm_dj_arena_grow(const NeedEnt* old, uint32_t old_cap, NeedEnt* fresh, uint32_t fresh_cap, uint64_t lo,
                       uint64_t hi, KeyState* table, uint32_t table_cap, hipStream_t s) {
  const uint64_t n = hi - lo;
  const uint64_t threads = n * (sizeof(NeedEnt) / 16);
  if (n) hipLaunchKernelGGL(k_arena_move, dim3((unsigned)((threads + TB - 1) / TB)), dim3(TB), 0, s, old, old_cap, fresh,
                            fresh_cap, lo, n);
  hipLaunchKernelGGL(k_arena_remap, dim3((table_cap + TB - 1) / TB), dim3(TB), 0, s, table, table_cap, old, old_cap,
                     fresh_cap, lo, hi);
}

int apm_dj_gather_plan(const int64_t* gid, int64_t n_upper, const int64_t* d_n, uint32_t* lens, uint32_t* offs,
                       void* tmp, size_t tmp_bytes, hipStream_t s) {
  hipLaunchKernelGGL(k_gather_len, dim3((unsigned)((n_upper + 1 + TB - 1) / TB)), dim3(TB), 0, s, gid, n_upper, d_n, lens);
  size_t need = 0;
  HIP_OK(rocprim::exclusive_scan(nullptr, need, lens, offs, 0u, (size_t)n_upper + 1, rocprim::plus<uint32_t>(), s));
  if (need > tmp_bytes) return -1;
  HIP_OK(rocprim::exclusive_scan(tmp, need, lens, offs, 0u, (size_t)n_upper + 1, rocprim::plus<uint32_t>(), s));
  return 0;
}

void apm_dj_gather_copy(const int64_t* gid, int64_t n, const char* ring, uint64_t ring_cap, const uint32_t* offs,
                        char* out, uint64_t total_bytes, hipStream_t s) {
  if (n <= 0 || total_bytes == 0) return;
  (void)total_bytes;  // (the blocks derive their byte ranges from offs)
  hipLaunchKernelGGL(k_gather_lines, dim3((unsigned)((n + GL_LINES - 1) / GL_LINES)), dim3(GL_TB), 0, s, gid, n, ring,
                     ring_cap, offs, out);
}

void apm_dj_rebase_gids(const int64_t* gid, int64_t n, const uint32_t* offs, uint64_t base, int64_t* out,
                        hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_rebase_gids, dim3((unsigned)((n + TB - 1) / TB)), dim3(TB), 0, s, gid, n, offs, base, out);
}

void apm_dj_min_pos(const int64_t* gid, int64_t n, unsigned long long* out, hipStream_t s) {
  if (n <= 0) return;
  // >= 2 blocks per CU once the pool is large (512 atomics at most on the one result word)
  const unsigned blocks = (unsigned)std::min<int64_t>(512, (n + 1023) / 1024);
  hipLaunchKernelGGL(k_min_pos, dim3(blocks), dim3(1024), 0, s, gid, n, out);
}

void apm_dj_relocate(int64_t* gid, int64_t n, char* ring, uint64_t ring_cap, uint64_t below, uint64_t dst_base,
                     unsigned long long* cursor, hipStream_t s) {
  if (n <= 0) return;
  const int64_t threads = n * APM_WAVE;
  hipLaunchKernelGGL(k_relocate, dim3((unsigned)((threads + TB - 1) / TB)), dim3(TB), 0, s, gid, n, ring, ring_cap,
                     below, dst_base, cursor);
}

void apm_dj_reg_fill(RegSlot* reg, const int32_t* pairs, uint32_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_reg_fill, dim3((n + TB - 1) / TB), dim3(TB), 0, s, reg, pairs, n);
}
void apm_dj_scatter_i32(int32_t* dst, const int32_t* pairs, uint32_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_scatter_i32, dim3((n + TB - 1) / TB), dim3(TB), 0, s, dst, pairs, n);
}
void apm_dj_fill_series(TxRec* tx, const int32_t* raw, uint32_t n, const int32_t* raw_series,
                        unsigned long long* unmapped, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_fill_series, dim3((n + TB - 1) / TB), dim3(TB), 0, s, tx, raw, n, raw_series, unmapped);
}
void apm_dj_gather_u8(const uint8_t* src, const int32_t* idx, uint32_t n, uint8_t* out, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_gather_u8, dim3((n + TB - 1) / TB), dim3(TB), 0, s, src, idx, n, out);
}
void apm_dj_keys_sync(const apm::KeyState* table, uint32_t cap, uint64_t* keys, hipStream_t s) {
  hipLaunchKernelGGL(k_keys_sync, dim3((cap + 255) / 256), dim3(256), 0, s, table, cap, keys);
  dj_check(s, "k_keys_sync");
}

void apm_dj_cache_stats(const apm::KeyState* table, uint32_t cap, double now, unsigned long long* out, hipStream_t s) {
  HIP_OK(hipMemsetAsync(out, 0, 5 * sizeof(unsigned long long), s));
  const unsigned blocks = std::max(1u, std::min<unsigned>(1024, (cap + TB - 1) / TB));
  hipLaunchKernelGGL(k_cache_stats, dim3(blocks), dim3(TB), 0, s, table, cap, now, out);
}

void apm_dj_count_le(const int64_t* end, int64_t n, int64_t edge, int64_t* out, hipStream_t s) {
  hipLaunchKernelGGL(k_count_le, dim3(1), dim3(1), 0, s, end, n, edge, out);
}

}  // extern "C"
