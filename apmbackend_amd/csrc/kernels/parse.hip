// K1-K3: line indexing, classification and field location for raw WildFly log bytes.
//
// Reference behaviour: stream_parse_transactions.js readLine (:741-791) and the regexes at
// :346-350, :449, :567-575, :734-739; tokenisation `line.split(/[\s]+/)` and
// `line.split(/INFO/)[1].trim().split(/[\s]+/)`; timestamps via convertStringDateToMs
// (:242-256).
//
// Design (MI355X): the batch is one contiguous byte buffer holding whole-line chunks, one chunk
// per log file.  K1 finds newlines with 16-byte vector loads and a block scan; K2 gives every
// line one lane, stages the block's byte range in LDS (64 KiB) and classifies the line with a
// single pass that tests all pattern families at each byte; relevant lines become fixed-layout
// Event records written in line order by an ordered stream compaction (flag scan).  Noise lines
// (the vast majority) never leave the GPU.  The stateful join (K4-K6) runs downstream on the
// GPU too (devjoin.hip), reading the same device bytes; only the rare lines it cannot read alone
// (non-ASCII, exotic number / date forms) are re-derived by the host pre-pass from the pinned
// host copy (runtime/devjoin.cpp).
#include "kernel_api.h"

#include <rocprim/rocprim.hpp>

#include "devscan.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace apm {

constexpr int NL_BLOCK = 256;
constexpr int NL_TILE = NL_BLOCK * 16;     // bytes per block in the newline pass
constexpr int PARSE_BLOCK = 256;           // lines per block in the parse pass
constexpr int PARSE_LDS = 32 * 1024;       // staged bytes per block (+ 8 KB token table: 4 blocks / CU)

// --------------------------------------------------------------------------------- K1
// Each block covers NL_PER consecutive 4 KB tiles (one 16-byte vector per lane per tile, all of
// them loaded before the first is used: four loads in flight per lane instead of one, a quarter of
// the blocks) and still reports one newline count per 4 KB tile -- the granularity tile_off[]
// has for k_parse_tiles.  (One tile a block: 38 + 47 us a batch for 28 MB, profiles/r6_g.)
constexpr int NL_PER = 4;

__device__ __forceinline__ uint32_t nl_count16(const uint4 v) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t c = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    // count bytes equal to '\n' (0x0a) in a 32-bit word: exact per-byte SWAR (no borrow between
    // bytes -- the (x - 0x01..) & ~x form also flags a 0x0b right after a '\n', and k_nl_write,
    // which counts exactly, would then leave holes in line_end)
    const uint32_t x = w[k] ^ 0x0a0a0a0aU;
    const uint32_t t = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
    c += __popc(t);
  }
  return c;
}

__global__ __launch_bounds__(NL_BLOCK) void k_nl_count(const uint8_t* __restrict__ bytes, uint64_t n,
                                                      uint32_t* __restrict__ tile_counts, uint8_t* __restrict__ pad,
                                                      uint32_t tiles) {
  // (folded fills) the 64 zero bytes after the batch that K2's 16-byte loads may touch, and the
  // scan's extra tile entry -- no block reads either of them
  if (blockIdx.x == 0 && threadIdx.x < 64) pad[threadIdx.x] = 0;
  if (blockIdx.x == 0 && threadIdx.x == 64) tile_counts[tiles] = 0;
  uint4 v[NL_PER];
  uint64_t base[NL_PER];
#pragma unroll
  for (int k = 0; k < NL_PER; ++k) {
    base[k] = ((uint64_t)blockIdx.x * NL_PER + k) * NL_TILE + threadIdx.x * 16;
    if (base[k] + 16 <= n) v[k] = *reinterpret_cast<const uint4*>(bytes + base[k]);
  }
  // per tile counts packed two to a word (a tile has at most 4096 newlines: 16 bits each)
  uint32_t pk[NL_PER / 2] = {0, 0};
#pragma unroll
  for (int k = 0; k < NL_PER; ++k) {
    uint32_t c = 0;
    if (base[k] + 16 <= n) {
      c = nl_count16(v[k]);
    } else {
      for (uint64_t i = base[k]; i < n && i < base[k] + 16; ++i) c += bytes[i] == '\n';
    }
    pk[k >> 1] += c << (16 * (k & 1));
  }
  __shared__ uint32_t red[NL_PER / 2][NL_BLOCK / APM_WAVE];
#pragma unroll
  for (int h = 0; h < NL_PER / 2; ++h) {
    uint32_t c = pk[h];
    for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o, APM_WAVE);
    if ((threadIdx.x & 63) == 0) red[h][threadIdx.x >> 6] = c;
  }
  __syncthreads();
  if (threadIdx.x < NL_PER) {
    const int k = threadIdx.x;
    uint32_t sum = 0;
    for (int i = 0; i < NL_BLOCK / APM_WAVE; ++i) sum += red[k >> 1][i];
    const uint32_t tile = blockIdx.x * NL_PER + k;
    if (tile < tiles) tile_counts[tile] = (sum >> (16 * (k & 1))) & 0xFFFFu;
  }
}

// Writes the byte position of every '\n' (= line end) in order; tile_off = exclusive scan of the
// per-tile counts.
__global__ __launch_bounds__(NL_BLOCK) void k_nl_write(const uint8_t* __restrict__ bytes, uint64_t n,
                                                      const uint32_t* __restrict__ tile_off,
                                                      uint32_t* __restrict__ line_end, uint32_t* __restrict__ n_lines,
                                                      uint32_t tiles) {
  if (blockIdx.x == 0 && threadIdx.x == 0) *n_lines = tile_off[tiles];  // (folded D2D copy)
  uint4 v[NL_PER];
#pragma unroll
  for (int k = 0; k < NL_PER; ++k) {
    const uint64_t base = ((uint64_t)blockIdx.x * NL_PER + k) * NL_TILE + threadIdx.x * 16;
    v[k] = base + 16 <= n ? *reinterpret_cast<const uint4*>(bytes + base) : make_uint4(0, 0, 0, 0);
  }
  typedef rocprim::block_scan<int, NL_BLOCK> Scan;
  __shared__ typename Scan::storage_type st;
#pragma unroll
  for (int k = 0; k < NL_PER; ++k) {
    const uint32_t tile = blockIdx.x * NL_PER + k;
    if (tile >= tiles) break;  // (uniform per block)
    const uint64_t base = (uint64_t)tile * NL_TILE + threadIdx.x * 16;
    uint8_t b[16];
    if (base + 16 <= n) {
      const uint32_t w[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int j = 0; j < 4; ++j) b[q * 4 + j] = (uint8_t)(w[q] >> (8 * j));
      }
    } else {
      for (int i = 0; i < 16; ++i) b[i] = (base + i < n) ? bytes[base + i] : 0;
    }
    int c = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) c += b[i] == '\n';
    int excl;
    Scan().exclusive_scan(c, excl, 0, st);
    uint32_t pos = tile_off[tile] + excl;
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (b[i] == '\n') line_end[pos++] = (uint32_t)(base + i);
    __syncthreads();  // (the scan storage is reused by the next tile)
  }
}

// --------------------------------------------------------------------------------- K2 helpers
__device__ __forceinline__ bool is_ws(uint8_t c) {
  // ' ' and \t \n \v \f \r (9..13) as one shift-and-mask
  return c <= 32 && ((0x100003E00ULL >> c) & 1ULL);
}
__device__ __forceinline__ bool is_digit(uint8_t c) { return c >= '0' && c <= '9'; }
__device__ __forceinline__ uint8_t lower(uint8_t c) { return (c >= 'A' && c <= 'Z') ? c + 32 : c; }

template <int N>
__device__ __forceinline__ bool match_at(const uint8_t* p, int i, int len, const char (&lit)[N]) {
  if (i + N - 1 > len) return false;
#pragma unroll
  for (int k = 0; k < N - 1; ++k)
    if (p[i + k] != (uint8_t)lit[k]) return false;
  return true;
}

// token indices the classifier reads -> register slot (tokens 0-3 for the Event, 1/2 for the
// timestamp, 9/11/13 for the EJB service / elapsed fields)
constexpr int NTOKSLOT = 7;
__device__ __forceinline__ constexpr int tok_slot(int k) {
  return k <= 3 ? k : (k == 9 ? 4 : (k == 11 ? 5 : (k == 13 ? 6 : 0)));
}
__device__ __forceinline__ void tok_put(uint16_t (&arr)[NTOKSLOT], int k, uint16_t v) {
  constexpr int idx[NTOKSLOT] = {0, 1, 2, 3, 9, 11, 13};
#pragma unroll
  for (int j = 0; j < NTOKSLOT; ++j) arr[j] = k == idx[j] ? v : arr[j];
}
__device__ __forceinline__ void tok_put_if(uint16_t (&arr)[NTOKSLOT], bool on, int k, uint16_t v) {
  tok_put(arr, on ? k : -1, v);
}
// token index -> slot (0xF: a token the classifier never reads), one nibble per index 0..15
constexpr uint64_t kTokSlotTab = 0xFF6F5F4FFFFF3210ULL;
__device__ __forceinline__ int tok_slot_of(int k) { return k < 16 ? (int)((kTokSlotTab >> (4 * k)) & 0xFu) : 15; }

// four characters packed little-endian, as they sit in a byte window p[i-3..i]
template <int N>
__device__ __forceinline__ constexpr uint32_t pk4(const char (&lit)[N]) {
  static_assert(N == 5, "pk4 takes exactly four characters");
  return (uint32_t)(uint8_t)lit[0] | ((uint32_t)(uint8_t)lit[1] << 8) | ((uint32_t)(uint8_t)lit[2] << 16) |
         ((uint32_t)(uint8_t)lit[3] << 24);
}

// SWAR byte classes over one dword (four bytes): 0x80 in every byte position that qualifies.
// Exact per byte (no borrow across bytes), so the markers compress to bit masks.
__device__ __forceinline__ uint32_t swar_eq(uint32_t d, uint32_t k4) {
  const uint32_t x = d ^ k4;
  return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
}
// JS \s over ASCII: ' ' or 9..13 (\t \n \v \f \r); bytes >= 0x80 never qualify
__device__ __forceinline__ uint32_t swar_ws(uint32_t d) {
  const uint32_t y = d & 0x7F7F7F7Fu;
  const uint32_t rng = (y + 0x77777777u) & ~(y + 0x72727272u) & ~d & 0x80808080u;  // 9 <= b < 14
  return rng | swar_eq(d, 0x20202020u);
}
// 0x80 byte markers -> 4 bits (byte k -> bit k)
__device__ __forceinline__ uint32_t swar_bits(uint32_t t) { return (((t >> 7) * 0x00204081u) >> 21) & 0xFu; }

// Byte-class masks of 16 bytes d[0..3] (byte j -> bit j), d[4] = the next four bytes: whitespace,
// non-ASCII, and pattern triggers (a window p[j..j+3] that is "INFO", ": Re", or starts with '<')
struct Masks16 {
  uint32_t ws, na, trig;
};
__device__ __forceinline__ Masks16 masks16(const uint32_t (&d)[5]) {
  Masks16 r{0u, 0u, 0u};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    r.ws |= swar_bits(swar_ws(d[q])) << (4 * q);
    r.na |= swar_bits(d[q] & 0x80808080u) << (4 * q);
    r.trig |= swar_bits(swar_eq(d[q], 0x3C3C3C3Cu)) << (4 * q);  // '<'
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t w = k == 0 ? d[q] : __builtin_amdgcn_alignbyte(d[q + 1], d[q], k);
      r.trig |= ((w == pk4("INFO")) | (w == pk4(": Re"))) ? (1u << (4 * q + k)) : 0u;
    }
  }
  return r;
}

template <int N>
__device__ __forceinline__ bool match_at_ci(const uint8_t* p, int i, int len, const char (&lit)[N]) {
  if (i + N - 1 > len) return false;
#pragma unroll
  for (int k = 0; k < N - 1; ++k)
    if (lower(p[i + k]) != (uint8_t)lit[k]) return false;
  return true;
}

// JS parseInt on an ASCII token without leading whitespace. Returns false if the host must
// decide (hex prefix, > 15 digits).
__device__ inline bool parse_int_tok(const uint8_t* p, int s, int e, double& out) {
  int i = s;
  bool neg = false;
  if (i < e && (p[i] == '+' || p[i] == '-')) { neg = p[i] == '-'; ++i; }
  if (i + 1 < e && p[i] == '0' && (p[i + 1] == 'x' || p[i + 1] == 'X')) return false;
  int64_t v = 0;
  int nd = 0;
  while (i < e && is_digit(p[i])) {
    v = v * 10 + (p[i] - '0');
    ++i;
    if (++nd > 15) return false;
  }
  out = nd == 0 ? apm_nan() : (neg ? -(double)v : (double)v);
  return true;
}

// Parse "t1 t2" as convertStringDateToMs does for the plain log form. Fast path only for
// pieces that are pure digit strings; anything else is deferred to the host (returns false).
__device__ inline bool parse_log_ts(const uint8_t* p, int s1, int e1, int s2, int e2,
                                    const TzTable& tz, double& out, bool& strict) {
  // pieces split on '-', ':', ','  (whitespace only separates t1 and t2)
  int64_t v[8];
  int np = 0;
  int nd[8];
  strict = false;
  for (int pass = 0; pass < 2; ++pass) {
    const int s = pass ? s2 : s1, e = pass ? e2 : e1;
    int64_t cur = 0;
    int cnt = 0;
    for (int i = s; i <= e; ++i) {
      const bool end = i == e;
      const uint8_t c = end ? '-' : p[i];
      if (c == '-' || c == ':' || c == ',') {
        if (np >= 8) return false;
        v[np] = cur; nd[np] = cnt; ++np;
        cur = 0; cnt = 0;
        if (end) break;
      } else if (is_digit(c)) {
        cur = cur * 10 + (c - '0');
        if (++cnt > 12) return false;
      } else {
        return false;  // 'T', signs, letters, exponent forms ... host decides
      }
    }
  }
  if (np < 7) {
    out = apm_nan();  // fewer than 7 fields -> new Date(..., undefined) -> NaN
    return np >= 2;   // np<2 cannot happen for two tokens; keep host path for safety
  }
  // Number("") === 0 for empty pieces: cnt==0 -> value 0 (already)
  const int64_t yr = (v[0] >= 0 && v[0] <= 99) ? v[0] + 1900 : v[0];  // Date(y,...) two-digit rule
  const int64_t local = make_date_ms(yr, v[1] - 1, v[2], v[3], v[4], v[5], v[6]);
  out = (double)local_to_utc(tz, local);
  strict = np == 7 && nd[0] == 4 && nd[1] == 2 && nd[2] == 2 && nd[3] == 2 && nd[4] == 2 &&
           nd[5] == 2 && nd[6] >= 1 && nd[6] <= 3;
  return true;
}

// The log form every WildFly line carries, "YYYY-MM-DD HH:MM:SS,mmm", without the piece loop:
// 22 independent byte reads, fixed separator / digit checks, then the same date arithmetic as
// parse_log_ts (whose result it reproduces exactly, strict form).  false: not this exact shape.
__device__ __forceinline__ bool parse_log_ts_fixed(const uint8_t* p, int s1, int e1, int s2, int e2,
                                                   const TzTable& tz, double& out) {
  if (e1 - s1 != 10 || e2 - s2 != 12) return false;
  uint32_t a[10], b[12];
#pragma unroll
  for (int k = 0; k < 10; ++k) a[k] = (uint32_t)p[s1 + k] - '0';
#pragma unroll
  for (int k = 0; k < 12; ++k) b[k] = (uint32_t)p[s2 + k] - '0';
  // separators ('-' - '0', ':' - '0', ',' - '0' wrap around as unsigned)
  bool ok = a[4] == (uint32_t)('-' - '0') && a[7] == (uint32_t)('-' - '0') && b[2] == (uint32_t)(':' - '0') &&
            b[5] == (uint32_t)(':' - '0') && b[8] == (uint32_t)(',' - '0');
  constexpr int da[8] = {0, 1, 2, 3, 5, 6, 8, 9};
  constexpr int db[9] = {0, 1, 3, 4, 6, 7, 9, 10, 11};
#pragma unroll
  for (int k = 0; k < 8; ++k) ok &= a[da[k]] <= 9u;
#pragma unroll
  for (int k = 0; k < 9; ++k) ok &= b[db[k]] <= 9u;
  if (!ok) return false;
  const int64_t y = a[0] * 1000 + a[1] * 100 + a[2] * 10 + a[3];
  const int64_t mo = a[5] * 10 + a[6], d = a[8] * 10 + a[9];
  const int64_t h = b[0] * 10 + b[1], mi = b[3] * 10 + b[4], sec = b[6] * 10 + b[7];
  const int64_t ms = b[9] * 100 + b[10] * 10 + b[11];
  const int64_t yr = y <= 99 ? y + 1900 : y;  // Date(y, ...) two-digit rule, as parse_log_ts
  out = (double)local_to_utc(tz, make_date_ms(yr, mo - 1, d, h, mi, sec, ms));
  return true;
}

struct ParseArgs {
  const uint8_t* bytes;
  const uint32_t* line_end;     // position of '\n' for each line
  const uint32_t* chunk_begin;  // n_chunks + 1 byte offsets
  const uint8_t* chunk_kind;    // FileKind per chunk
  const uint32_t* n_lines_dev;  // produced by k_nl_write's scan
  uint32_t cap_lines;           // grid coverage; keep[] is zeroed in [n_lines, cap_lines)
  uint32_t n_chunks;
  Event* ev_tmp;                // per-line event slot
  uint32_t* line_mask;          // per-line pattern mask (for the section scan)
  uint8_t* keep;                // per-line compaction flag
  unsigned long long* watermark;  // max leading timestamp (ms, biased by 2^62)
  unsigned long long* prof;       // APM_PARSE_PROF: per-phase shader cycles (nullptr: off)
  TzTable tz;
};

// APM_PARSE_PROF phase counters: wave-time (lane 0's clock) per phase, summed over waves
enum : int { PP_STAGE = 0, PP_SCAN, PP_HITS, PP_LINES, PP_WAVES, PP_COOP, PP_SERIAL, PP_HEAD, PP_TAIL, PP_N = 10 };
__device__ __forceinline__ void pprof(const ParseArgs& a, int k, long long& t) {
  if (a.prof) {
    const long long now = clock64();
    if ((threadIdx.x & (APM_WAVE - 1)) == 0) atomicAdd(&a.prof[k], (unsigned long long)(now - t));
    t = now;
  }
}

// the chunk holding byte `pos`, searched in chunks [lo, hi] (a block narrows the range once from
// its first and last byte, so a line's search is usually empty)
__device__ __forceinline__ uint32_t find_chunk_in(const uint32_t* cb, uint32_t lo, uint32_t hi, uint32_t pos) {
  while (lo < hi) {
    uint32_t mid = (lo + hi + 1) >> 1;
    if (cb[mid] <= pos) lo = mid; else hi = mid - 1;
  }
  return lo;
}

__device__ __forceinline__ uint32_t find_chunk(const uint32_t* cb, uint32_t n_chunks, uint32_t pos) {
  uint32_t lo = 0, hi = n_chunks - 1;
  while (lo < hi) {
    uint32_t mid = (lo + hi + 1) >> 1;
    if (cb[mid] <= pos) lo = mid; else hi = mid - 1;
  }
  return lo;
}

template <int STRIDE = PARSE_BLOCK>
__device__ __forceinline__ unsigned long long parse_line(const ParseArgs& a, const uint8_t* __restrict__ base,
                                                         uint32_t o, uint32_t li, uint32_t ls, uint32_t le,
                                                         uint32_t c_lo, uint32_t c_hi, uint16_t* tp);

// per-line pattern flags beyond the PM_* mask
enum : uint32_t { XF_EJB_ENTRY = 1, XF_EJB_EXIT = 2, XF_CT_START = 4, XF_CT_STOP = 8, XF_BAF = 16, XF_NONASCII = 32 };

// A pattern trigger whose four bytes p[s..s+3] start an "INFO", ": Re" or a '<' tag: the full
// matches (readLine's regexes, stream_parse_transactions.js:346-350, :449, :567-575, :734-739).
// INFO occurrences (info1 / info2) are tracked by the caller.
template <class P>
__device__ __forceinline__ void probe_flags(P p, int len, int s, uint32_t& m, uint32_t& xf) {
  const uint32_t w4 = (uint32_t)p[s] | ((uint32_t)p[s + 1] << 8) | ((uint32_t)p[s + 2] << 16) |
                      ((uint32_t)p[s + 3] << 24);
  if (w4 == pk4("INFO")) {
    int j = s + 4;
    while (j < len && p[j] == ' ') ++j;
    if (match_at(p, j, len, "[CommonTiming] The EJB")) xf |= XF_EJB_ENTRY;
    if (match_at(p, j, len, "[CommonTiming] Total time")) xf |= XF_EJB_EXIT;
    if (match_at(p, j, len, "CommonTiming::Start")) xf |= XF_CT_START;
    if (match_at(p, j, len, "CommonTiming::Stop")) xf |= XF_CT_STOP;
    if (match_at(p, s, len, "INFO  auditTrailId=")) m |= PM_AUTR_MAP;
    // BAF  \[[^ ]+] +INFO  : the ']' is the last non-space before the spaces preceding an
    // "INFO ", with a '[' at least two columns before it and no space in between
    if (!(xf & XF_BAF) && s + 4 < len && p[s + 4] == ' ' && s >= 1 && p[s - 1] == ' ') {
      int kk0 = s - 1;
      while (kk0 >= 0 && p[kk0] == ' ') --kk0;
      if (kk0 >= 0 && p[kk0] == ']')
        for (int kk = kk0 - 2; kk >= 0 && p[kk] != ' '; --kk)
          if (p[kk] == '[') { xf |= XF_BAF; break; }
    }
    return;
  }
  if (w4 == pk4(": Re")) {
    if (match_at(p, s, len, ": RequestTrace [stopWatchList=")) m |= PM_EL_START;
    return;
  }
  if ((w4 & 0xffu) != '<') return;
  const uint32_t w4l = (uint32_t)lower(p[s]) | ((uint32_t)lower(p[s + 1]) << 8) |
                       ((uint32_t)lower(p[s + 2]) << 16) | ((uint32_t)lower(p[s + 3]) << 24);
  if (w4 == pk4("<sto")) {
    if (match_at(p, s, len, "<stopWatchList>")) m |= PM_SW_START;
    if (match_at(p, s, len, "<stopTime>")) m |= PM_SW_STOPTS;
  } else if (w4 == pk4("</st")) {
    if (match_at(p, s, len, "</stopWatchList>")) m |= PM_SW_END;
  } else if (w4 == pk4("<nam")) {
    if (match_at(p, s, len, "<name>")) m |= PM_SW_NAME;
  } else if (w4 == pk4("<sta")) {
    if (match_at(p, s, len, "<startTime>")) m |= PM_SW_STARTTS;
  } else if (w4 == pk4("<val")) {
    if (match_at(p, s, len, "<value>")) m |= PM_SOAP_VALUE;
  }
  if (w4l == pk4("<acc")) {
    if (match_at_ci(p, s, len, "<accountnumber>")) m |= PM_SOAP_ACCT;
  } else if (w4l == pk4("<key")) {
    if (match_at_ci(p, s, len, "<key>accountnumber</key>")) m |= PM_SOAP_KEY;
  }
}

template <int STRIDE>
__device__ __forceinline__ unsigned long long line_tail(const ParseArgs& a, const uint8_t* __restrict__ p, int len,
                                                        uint32_t li, Event& ev, uint8_t fk, int ntok, uint32_t m,
                                                        uint32_t xf, int info1, int info2, const uint16_t* tp,
                                                        int bias);
// Event fields every line gets; false for a line that ends here (empty, or > 65000 bytes: the
// host takes it verbatim)
__device__ __forceinline__ bool line_head(const ParseArgs& a, const uint8_t* __restrict__ p, uint32_t li,
                                          uint32_t ls, uint32_t le, uint32_t c_lo, uint32_t c_hi, Event& ev,
                                          uint8_t& fk, int& len);

// --------------------------------------------------------------------------------- K2
__global__ __launch_bounds__(PARSE_BLOCK) void k_parse_lines(ParseArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[PARSE_LDS];
  // token start/end positions of the tokens the classifier reads, slot-major (lane-adjacent
  // entries): one LDS store per token boundary instead of a 7-way register select per byte
  __shared__ uint16_t tok_lds[2 * NTOKSLOT][PARSE_BLOCK];
  long long pt = a.prof ? clock64() : 0;
  const uint32_t n_lines = *a.n_lines_dev;
  const uint32_t first = blockIdx.x * PARSE_BLOCK;
  if (first >= n_lines) {
    const uint32_t li = first + threadIdx.x;
    if (li < a.cap_lines) a.keep[li] = 0;
    return;
  }
  const uint32_t last = min(first + PARSE_BLOCK, n_lines);  // exclusive
  const uint32_t r0 = first == 0 ? 0 : a.line_end[first - 1] + 1;
  const uint32_t r1 = a.line_end[last - 1] + 1;
  // Stage the block's bytes [r0, r1) in LDS with 16-byte loads when they fit.
  const uint32_t a0 = r0 & ~15u;
  const uint32_t span = r1 - a0;
  const bool staged = span <= PARSE_LDS;
  if (staged) {
    // four 16-byte loads per lane in flight before the LDS stores, so the stage costs one memory
    // latency per 16 KB instead of one per 4 KB (the buffer is padded by >= 16 bytes on the
    // host, so a full vector load is in bounds)
    const uint32_t nvec = (span + 15) >> 4;
    const uint4* __restrict__ src = reinterpret_cast<const uint4*>(a.bytes + a0);
    uint4* dst = reinterpret_cast<uint4*>(lds);
    const uint32_t t = threadIdx.x;
    for (uint32_t i = t; i < nvec; i += 4 * PARSE_BLOCK) {
      const bool b1 = i + PARSE_BLOCK < nvec, b2 = i + 2 * PARSE_BLOCK < nvec, b3 = i + 3 * PARSE_BLOCK < nvec;
      const uint4 v0 = src[i];
      const uint4 v1 = b1 ? src[i + PARSE_BLOCK] : v0;
      const uint4 v2 = b2 ? src[i + 2 * PARSE_BLOCK] : v0;
      const uint4 v3 = b3 ? src[i + 3 * PARSE_BLOCK] : v0;
      dst[i] = v0;
      if (b1) dst[i + PARSE_BLOCK] = v1;
      if (b2) dst[i + 2 * PARSE_BLOCK] = v2;
      if (b3) dst[i + 3 * PARSE_BLOCK] = v3;
    }
  }
  __syncthreads();
  pprof(a, PP_STAGE, pt);
  const uint32_t li = first + threadIdx.x;
  unsigned long long wm = 0;
  if (li >= last) {
    if (li < a.cap_lines) a.keep[li] = 0;
  } else {
    const uint32_t ls = li == 0 ? 0 : a.line_end[li - 1] + 1;
    const uint32_t le = a.line_end[li];
    // Two inlined copies of the line parser, one per address space.  A single copy behind
    // `staged ? lds : global` sees a generic pointer and issues a flat load for every byte
    // (rocprofv3 before the split: 9M VMEM reads per run, ~150 LDS conflict cycles per LDS op).
    const uint32_t c_lo = find_chunk(a.chunk_begin, a.n_chunks, r0), c_hi = find_chunk(a.chunk_begin, a.n_chunks, r1 - 1);
    wm = staged ? parse_line<PARSE_BLOCK>(a, lds, ls - a0, li, ls, le, c_lo, c_hi, &tok_lds[0][threadIdx.x])
                : parse_line<PARSE_BLOCK>(a, a.bytes, ls, li, ls, le, c_lo, c_hi, &tok_lds[0][threadIdx.x]);
  }
  if (a.prof) {
    pprof(a, PP_LINES, pt);
    if ((threadIdx.x & (APM_WAVE - 1)) == 0) atomicAdd(&a.prof[PP_WAVES], 1ull);
  }
  // Watermark: one atomic per wave.  A per-lane atomicMax on the single watermark word put 64
  // same-address atomics per wave through one L2 atomic unit, serialising the whole grid.
  for (int off = APM_WAVE / 2; off > 0; off >>= 1) {
    const unsigned long long o2 = __shfl_xor(wm, off, APM_WAVE);
    wm = o2 > wm ? o2 : wm;
  }
  if ((threadIdx.x & (APM_WAVE - 1)) == 0 && wm) atomicMax(a.watermark, wm);
}

__device__ __forceinline__ bool line_head(const ParseArgs& a, const uint8_t* __restrict__ p, uint32_t li,
                                          uint32_t ls, uint32_t le, uint32_t c_lo, uint32_t c_hi, Event& ev,
                                          uint8_t& fk, int& len) {
  len = (int)(le - ls);
  if (len > 0 && p[len - 1] == '\r') --len;

  ev.line = li;
  ev.chunk = find_chunk_in(a.chunk_begin, c_lo, c_hi, ls);
  ev.off = ls;
  ev.len = (uint32_t)len;
  ev.mask = 0;
  ev.kind = LK_NONE;
  ev.ntok = 0;
  ev.pad0 = 0;
  ev.t0s = ev.t0e = ev.t1s = ev.t1e = ev.t2s = ev.t2e = ev.t3s = ev.t3e = 0xffff;
  ev.tAs = ev.tAe = ev.tBs = ev.tBe = 0xffff;
  ev.ts = apm_nan();
  ev.num = apm_nan();
  ev.key = 0;
  ev.svc = 0;
  fk = a.chunk_kind[ev.chunk];
  if (len <= 0 || len > 65000) {
    // empty lines are skipped by readLine; absurdly long lines go to the host verbatim
    a.keep[li] = (len > 65000) ? 1 : 0;
    if (len > 65000) { ev.kind = fk == FILE_SOAP ? LK_SOAP : LK_APP; ev.mask = PM_HOST; }
    a.line_mask[li] = ev.mask;
    a.ev_tmp[li] = ev;
    return false;
  }
  return true;
}

// --------------------------------------------------------------------------------- K2, by tile
// One wave per 4 KB tile of the batch: the lines that START in the tile.  The wave stages the
// tile (plus up to 1 KB of the last lines' tails) in LDS, then scans it cooperatively, 16 bytes
// per lane per step (1 KB per wave step, conflict-free ds_read_b128): SWAR byte classes,
// token starts / ends / line starts as bit masks, and one wave-wide segmented scan per step of
// (line starts, token starts since the last line start, pattern triggers) that gives every
// boundary its line and token rank.  Pattern triggers are matched afterwards one lane per
// trigger, and the per-line tail (timestamp, classification, join keys) runs one lane per line.
// No lane walks a line byte by byte, so long and short lines cost the same per byte, and no
// lane waits on another's line.  Lines the cooperative pass cannot hold (more than TMAXL lines in
// a tile, more than THITS triggers, a tail beyond the stage) take parse_line.
constexpr int TILE = NL_TILE;             // 4096: tile_off[] of the newline pass indexes tiles
constexpr int TSTAGE = TILE + 1024;       // staged bytes per tile
constexpr int TMAXL = 128;                // lines per tile in the cooperative pass
constexpr int THITS = 256;                // pattern triggers per tile

// packed scan element: line starts (bits 0-12), "has a line start" (bit 13), token starts since
// the last line start, saturated at 31 (bits 14-18), pattern triggers (bits 19-31)
__device__ __forceinline__ uint32_t tscan_op(uint32_t x, uint32_t y) {  // x before y
  const uint32_t ls = (x & 0x1FFFu) + (y & 0x1FFFu);
  const uint32_t hits = (x >> 19) + (y >> 19);
  uint32_t seg, has;
  if (y & 0x2000u) {
    seg = (y >> 14) & 31u;
    has = 1u;
  } else {
    seg = min(((x >> 14) & 31u) + ((y >> 14) & 31u), 31u);
    has = (x >> 13) & 1u;
  }
  return ls | (has << 13) | (seg << 14) | (hits << 19);
}

__global__ __launch_bounds__(APM_WAVE) void k_parse_tiles(ParseArgs a, uint64_t n, const uint32_t* __restrict__ tile_off) {
  __shared__ __attribute__((aligned(16))) uint8_t st[TSTAGE + 32];
  __shared__ uint16_t tok[2 * NTOKSLOT][TMAXL];
  __shared__ uint16_t c_ls[TMAXL], c_le[TMAXL];
  __shared__ uint8_t c_nt[TMAXL];
  __shared__ uint32_t c_m[TMAXL], c_xf[TMAXL], c_i1[TMAXL], c_i2[TMAXL];
  __shared__ uint32_t hit[THITS];
  const int lane = threadIdx.x;
  long long pt = a.prof ? clock64() : 0;
  const uint32_t n_lines = *a.n_lines_dev;
  // lines past the batch: clear their compaction flags (grid-stride)
  for (uint32_t li = n_lines + blockIdx.x * APM_WAVE + lane; li < a.cap_lines; li += gridDim.x * APM_WAVE)
    a.keep[li] = 0;
  const uint64_t T0 = (uint64_t)blockIdx.x * TILE;
  if (T0 >= n) return;
  const uint64_t T1 = min(T0 + TILE, n);
  // lines starting in [T0, T1): global indices [first_li, end_li)
  const bool own0 = T0 == 0 || a.bytes[T0 - 1] == '\n';
  const bool own1 = a.bytes[T1 - 1] == '\n';
  const uint32_t first_li = tile_off[blockIdx.x] + (own0 ? 0u : 1u);
  const uint32_t end_li = min(min(tile_off[blockIdx.x + 1] + (own1 ? 0u : 1u), n_lines), a.cap_lines);
  if (first_li >= end_li) return;
  const uint32_t n_own = end_li - first_li;
  const uint32_t s0 = (first_li == 0 ? 0u : a.line_end[first_li - 1] + 1u) - (uint32_t)T0;  // stage offsets
  const uint32_t e_last = a.line_end[end_li - 1] - (uint32_t)T0;
  const uint32_t staged = (uint32_t)min<uint64_t>(TSTAGE, n - T0);
  const uint32_t vend = min(e_last, staged - 1u);  // last byte the scan attributes
  // ---- stage: five 16-byte loads per lane in flight (the batch is padded by >= 256 bytes)
  {
    static_assert(TSTAGE == 5 * 1024, "five 1 KB wave loads");
    const uint4* __restrict__ src = reinterpret_cast<const uint4*>(a.bytes + T0) + lane;
    uint4* dst = reinterpret_cast<uint4*>(st) + lane;
    const uint32_t o = 16u * lane;
    const uint4 z = make_uint4(0u, 0u, 0u, 0u);
    const uint4 v0 = o <= vend ? src[0] : z;
    const uint4 v1 = o + 1024u <= vend ? src[64] : z;
    const uint4 v2 = o + 2048u <= vend ? src[128] : z;
    const uint4 v3 = o + 3072u <= vend ? src[192] : z;
    const uint4 v4 = o + 4096u <= vend ? src[256] : z;
    dst[0] = v0;
    dst[64] = v1;
    dst[128] = v2;
    dst[192] = v3;
    dst[256] = v4;
    if (lane < 8) reinterpret_cast<uint32_t*>(st + TSTAGE)[lane] = 0u;
    for (int l = lane; l < TMAXL; l += APM_WAVE) {
      c_le[l] = 0xFFFFu;
      c_m[l] = 0u;
      c_xf[l] = 0u;
      c_i1[l] = 0xFFFFFFFFu;
      c_i2[l] = 0xFFFFFFFFu;
    }
  }
  __syncthreads();
  pprof(a, PP_STAGE, pt);
  // ---- cooperative scan
  uint32_t carry = 0u;                 // scan state before this step
  uint32_t prev_last = '\n';           // byte before this step's first byte (s0 is a line start)
  for (uint32_t k0 = s0 & ~15u; k0 <= vend; k0 += 1024) {
    const uint32_t off = k0 + 16u * lane;  // this lane's 16 bytes
    uint32_t d[5] = {0u, 0u, 0u, 0u, 0u};
    if (off <= vend) {
      const uint4 v = *reinterpret_cast<const uint4*>(st + off);
      d[0] = v.x, d[1] = v.y, d[2] = v.z, d[3] = v.w;
      d[4] = *reinterpret_cast<const uint32_t*>(st + off + 16);
    }
    const Masks16 mk = masks16(d);
    uint32_t nl = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) nl |= swar_bits(swar_eq(d[q], 0x0A0A0A0Au)) << (4 * q);
    // attributed bytes: s0 <= off + j <= vend
    uint32_t valid = 0xFFFFu;
    if (off < s0) valid = s0 - off >= 16 ? 0u : (0xFFFFu << (s0 - off)) & 0xFFFFu;
    if (off + 15 > vend) valid &= off > vend ? 0u : (0xFFFFu >> (15u - (vend - off)));
    // previous byte's class: from the lane below, lane 0 from the last step
    const uint32_t up = __shfl_up(d[3] >> 24, 1, APM_WAVE);
    const uint32_t pb = lane == 0 ? prev_last : up;
    const uint32_t pb_ws = (pb <= 32u && ((0x100003E00ULL >> pb) & 1ULL)) ? 1u : 0u;
    const uint32_t pb_nl = pb == '\n' ? 1u : 0u;
    prev_last = __shfl(d[3] >> 24, APM_WAVE - 1, APM_WAVE);
    const uint32_t ws = mk.ws;
    const uint32_t prev_ws = ((ws << 1) | pb_ws) & 0xFFFFu;
    const uint32_t lsm = ((nl << 1) | pb_nl) & valid;                     // line starts
    const uint32_t tsm = ((~ws & prev_ws) | (lsm & ws & ~nl)) & valid;    // token starts (+ leading '')
    const uint32_t tem = ws & ~prev_ws & valid;                           // ends of non-empty tokens
    const uint32_t nlm = nl & valid;                                      // line ends
    const uint32_t him = mk.trig & valid & ~nl;                           // pattern triggers
    // scan element of this lane
    uint32_t e = (uint32_t)__popc(lsm) | ((uint32_t)__popc(him) << 19);
    if (lsm) {
      const int hb = 31 - __clz(lsm);
      e |= 0x2000u | ((uint32_t)__popc(tsm >> hb) << 14);
    } else {
      e |= (uint32_t)__popc(tsm) << 14;
    }
    uint32_t inc = e;
#pragma unroll
    for (int o = 1; o < APM_WAVE; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o, APM_WAVE);
      if (lane >= o) inc = tscan_op(y, inc);
    }
    const uint32_t exc_w = __shfl_up(inc, 1, APM_WAVE);
    const uint32_t exc = lane == 0 ? carry : tscan_op(carry, exc_w);
    carry = tscan_op(carry, __shfl(inc, APM_WAVE - 1, APM_WAVE));
    // walk this lane's boundaries in byte order
    int L = (int)(exc & 0x1FFFu) - 1;      // line of the bytes before the first line start
    uint32_t rank = (exc >> 14) & 31u;     // token starts seen in that line
    uint32_t bnd = lsm | tsm | tem | nlm;
    while (bnd) {
      const int j = __builtin_ctz(bnd);
      bnd &= bnd - 1;
      const uint32_t bit = 1u << j;
      const uint16_t pos = (uint16_t)(off + j);
      if (lsm & bit) {
        ++L;
        rank = 0;
        if (L < TMAXL) c_ls[L] = pos;
      }
      if (L >= TMAXL) continue;
      if ((tem & bit) && rank > 0) {
        const int sl = tok_slot_of((int)rank - 1);
        if (sl != 15) tok[NTOKSLOT + sl][L] = pos;
      }
      if (tsm & bit) {
        const int sl = tok_slot_of((int)rank);
        if (sl != 15) {
          tok[sl][L] = pos;
          if (ws & bit) tok[NTOKSLOT + sl][L] = pos;  // the leading ''
        }
        rank = min(rank + 1u, 31u);
      }
      if (nlm & bit) {
        c_le[L] = pos;
        c_nt[L] = (uint8_t)rank;
      }
    }
    // non-ASCII bytes (rare): flag their lines
    uint32_t na = mk.na & valid;
    while (na) {
      const int j = __builtin_ctz(na);
      na &= na - 1;
      const int l2 = (int)(exc & 0x1FFFu) - 1 + __popc(lsm & ((2u << j) - 1u));
      if (l2 < TMAXL) atomicOr(&c_xf[l2], (uint32_t)XF_NONASCII);
    }
    // pattern triggers -> the tile's hit list
    uint32_t hm = him;
    uint32_t hidx = exc >> 19;
    while (hm) {
      const int j = __builtin_ctz(hm);
      hm &= hm - 1;
      const int l2 = (int)(exc & 0x1FFFu) - 1 + __popc(lsm & ((2u << j) - 1u));
      if (hidx < THITS && l2 < TMAXL) hit[hidx] = ((uint32_t)l2 << 16) | (off + j);
      ++hidx;
    }
  }
  const uint32_t n_hits = carry >> 19;
  const bool coop_ok = n_hits <= THITS;
  __syncthreads();
  pprof(a, PP_SCAN, pt);
  // ---- pattern triggers: full matches, one lane per trigger
  if (coop_ok) {
    for (uint32_t h = lane; h < n_hits; h += APM_WAVE) {
      const uint32_t L = hit[h] >> 16, pos = hit[h] & 0xFFFFu;
      if (L >= TMAXL || c_le[L] == 0xFFFFu) continue;
      const uint8_t* p = st + c_ls[L];
      int len = (int)c_le[L] - (int)c_ls[L];
      if (len > 0 && p[len - 1] == '\r') --len;
      const int s = (int)pos - (int)c_ls[L];
      if (s + 3 >= len) continue;  // the window must lie inside the line
      if (p[s] == 'I' && p[s + 1] == 'N' && p[s + 2] == 'F' && p[s + 3] == 'O') atomicMin(&c_i1[L], (uint32_t)s);
      uint32_t m = 0, xf = 0;
      probe_flags(p, len, s, m, xf);
      if (m) atomicOr(&c_m[L], m);
      if (xf) atomicOr(&c_xf[L], xf);
    }
    __syncthreads();
    // second INFO of each line (INFO occurrences cannot overlap)
    for (uint32_t h = lane; h < n_hits; h += APM_WAVE) {
      const uint32_t L = hit[h] >> 16, pos = hit[h] & 0xFFFFu;
      if (L >= TMAXL || c_le[L] == 0xFFFFu) continue;
      const uint8_t* p = st + pos;
      const uint32_t s = pos - c_ls[L];
      if (p[0] == 'I' && p[1] == 'N' && p[2] == 'F' && p[3] == 'O' && s > c_i1[L]) atomicMin(&c_i2[L], s);
    }
    __syncthreads();
  }
  pprof(a, PP_HITS, pt);
  // ---- per line: the tail (or the whole line on the lane, for lines the pass did not hold)
  unsigned long long wm = 0;
  unsigned long long n_coop = 0, n_ser = 0;
  const uint32_t c_lo = find_chunk(a.chunk_begin, a.n_chunks, (uint32_t)T0 + s0);
  const uint32_t c_hi = find_chunk(a.chunk_begin, a.n_chunks, a.line_end[end_li - 1]);
  for (uint32_t L = lane; L < n_own; L += APM_WAVE) {
    const uint32_t li = first_li + L;
    const uint32_t ls = li == 0 ? 0u : a.line_end[li - 1] + 1u, le = a.line_end[li];
    uint16_t* tp = &tok[0][L % TMAXL];
    unsigned long long w;
    if (coop_ok && L < TMAXL && c_le[L] != 0xFFFFu) {
      const uint32_t o = ls - (uint32_t)T0;
      const uint8_t* __restrict__ p = st + o;
      Event ev;
      uint8_t fk;
      int len;
      const long long th0 = a.prof ? clock64() : 0;
      if (!line_head(a, p, li, ls, le, c_lo, c_hi, ev, fk, len)) continue;
      const long long th1 = a.prof ? clock64() : 0;
      int ntok = c_nt[L];
      if (ntok < 16 && is_ws(p[len - 1])) {  // trailing ''
        const int sl = tok_slot_of(ntok);
        if (sl != 15) tp[sl * TMAXL] = tp[(NTOKSLOT + sl) * TMAXL] = (uint16_t)(o + len);
        ++ntok;
      }
      const int i1 = c_i1[L] == 0xFFFFFFFFu ? -1 : (int)c_i1[L];
      const int i2 = c_i2[L] == 0xFFFFFFFFu ? -1 : (int)c_i2[L];
      w = line_tail<TMAXL>(a, p, len, li, ev, fk, ntok, c_m[L], c_xf[L], i1, i2, tp, (int)o);
      ++n_coop;
      if (a.prof) {  // lane-summed
        atomicAdd(&a.prof[PP_HEAD], (unsigned long long)(th1 - th0));
        atomicAdd(&a.prof[PP_TAIL], (unsigned long long)(clock64() - th1));
      }
    } else if (le - (uint32_t)T0 < staged) {
      w = parse_line<TMAXL>(a, st, ls - (uint32_t)T0, li, ls, le, c_lo, c_hi, tp);
      ++n_ser;
    } else {
      w = parse_line<TMAXL>(a, a.bytes, ls, li, ls, le, c_lo, c_hi, tp);
      ++n_ser;
    }
    wm = w > wm ? w : wm;
  }
  if (a.prof) {
    pprof(a, PP_LINES, pt);
    if (lane == 0) atomicAdd(&a.prof[PP_WAVES], 1ull);
    if (n_coop) atomicAdd(&a.prof[PP_COOP], n_coop);
    if (n_ser) atomicAdd(&a.prof[PP_SERIAL], n_ser);
  }
  for (int o = APM_WAVE / 2; o > 0; o >>= 1) {
    const unsigned long long o2 = __shfl_xor(wm, o, APM_WAVE);
    wm = o2 > wm ? o2 : wm;
  }
  if (lane == 0 && wm) atomicMax(a.watermark, wm);
}

// One line, one lane: `base + o` is its first byte; `base` is 16-byte aligned (LDS stage or the
// batch).  tp: this lane's column of a token table (entry k at tp[k * STRIDE]; starts in rows
// 0..6, ends in rows 7..13)
template <int STRIDE>
__device__ __forceinline__ unsigned long long parse_line(const ParseArgs& a, const uint8_t* __restrict__ base,
                                                         uint32_t o, uint32_t li, uint32_t ls, uint32_t le,
                                                         uint32_t c_lo, uint32_t c_hi, uint16_t* tp) {
  const uint8_t* __restrict__ p = base + o;
  Event ev;
  uint8_t fk;
  int len;
  if (!line_head(a, p, li, ls, le, c_lo, c_hi, ev, fk, len)) return 0;

  // ---- single pass: whitespace tokens 0..13, pattern tests, INFO occurrences.  Boundaries of
  // the tokens the classifier reads (0-3, 9, 11, 13) go to the LDS table (one store each).
  auto TS = [&](int sl) -> uint16_t& { return tp[sl * STRIDE]; };
  auto TE = [&](int sl) -> uint16_t& { return tp[(NTOKSLOT + sl) * STRIDE]; };
  int ntok = 0;
  bool in_tok = false;
  if (len > 0 && is_ws(p[0])) { TS(0) = 0; TE(0) = 0; ntok = 1; }  // split gives '' first
  int info1 = -1, info2 = -1;
  bool nonascii = false;
  uint32_t m = 0, xf = 0;
  // 16 bytes per step (one aligned 16-byte read, ds_read_b128 from the stage, plus the next
  // dword for pattern windows that straddle it): byte classes as SWAR bit masks, token starts
  // and ends as mask arithmetic on them, and only the boundaries (about one per 6 bytes) and
  // the pattern triggers walked one by one.  The byte-serial first version spent ~30 VALU
  // instructions per byte on token bookkeeping.
  const uint8_t* __restrict__ al = base + (o & ~15u);
  const int lead = (int)(o & 15u);
  for (int g = -lead; g < len; g += 16, al += 16) {
    const uint4 v = *reinterpret_cast<const uint4*>(al);
    const uint32_t d[5] = {v.x, v.y, v.z, v.w, *reinterpret_cast<const uint32_t*>(al + 16)};
    const Masks16 mk = masks16(d);
    // active bytes: 0 <= g + j < len
    const uint32_t lo = g < 0 ? (0xFFFFu << (-g)) & 0xFFFFu : 0xFFFFu;
    const uint32_t act = len - g >= 16 ? lo : lo & ((1u << (len - g)) - 1u);
    const uint32_t ws = mk.ws & act, tk = ~mk.ws & act;
    const uint32_t prev_tk = ((tk << 1) | (in_tok ? 1u : 0u)) & act;
    uint32_t ev = (tk & ~prev_tk) | (ws & prev_tk);  // token starts | token ends, in byte order
    in_tok = (tk >> (31 - __clz(act))) & 1u;  // at the last active byte (act != 0 here)
    nonascii |= (mk.na & act) != 0u;
    if (ntok >= 16) {
      ntok += __popc(ws & prev_tk);
    } else {
      while (ev) {
        const int j = __builtin_ctz(ev);
        ev &= ev - 1;
        const bool start = (tk >> j) & 1u;
        const int sl = tok_slot_of(ntok);
        if (sl != 15) {
          if (start) TS(sl) = (uint16_t)(g + j);
          else TE(sl) = (uint16_t)(g + j);
        }
        ntok += start ? 0 : 1;
      }
    }
    // windows p[s..s+3] wholly inside the line: s = g + j >= 0 and s + 3 < len
    const int wmax = len - 4 - g;  // largest j allowed
    uint32_t hits = wmax < 0 ? 0u : mk.trig & lo & (wmax >= 15 ? 0xFFFFu : ((2u << wmax) - 1u));
    while (hits) {
      const int k = __builtin_ctz(hits);
      hits &= hits - 1;
      const int s = g + k;
      if (p[s] == 'I' && p[s + 1] == 'N' && p[s + 2] == 'F' && p[s + 3] == 'O') {
        if (info1 < 0) info1 = s;
        else if (info2 < 0 && s >= info1 + 4) info2 = s;
      }
      probe_flags(p, len, s, m, xf);
    }
  }
  if (in_tok) {
    const int sl = tok_slot_of(ntok);
    if (sl != 15) TE(sl) = (uint16_t)len;
    ++ntok;
  } else if (is_ws(p[len - 1]) && ntok < 16) {  // trailing ''
    const int sl = tok_slot_of(ntok);
    if (sl != 15) { TS(sl) = (uint16_t)len; TE(sl) = (uint16_t)len; }
    ++ntok;
  }
  if (nonascii) xf |= XF_NONASCII;
  return line_tail<STRIDE>(a, p, len, li, ev, fk, ntok, m, xf, info1, info2, tp, 0);
}

// The per-line tail shared by the serial and the cooperative scans: line-anchored patterns,
// tokens 0-3, the leading timestamp, classification (reference dispatch order), join keys.
// tp: the line's token-table column (stride STRIDE); entries are positions minus `bias`.
template <int STRIDE>
__device__ __forceinline__ unsigned long long line_tail(const ParseArgs& a, const uint8_t* __restrict__ p, int len,
                                                        uint32_t li, Event& ev, uint8_t fk, int ntok, uint32_t m,
                                                        uint32_t xf, int info1, int info2, const uint16_t* tp,
                                                        int bias) {
  auto TS = [&](int sl) -> int { return (int)tp[sl * STRIDE] - bias; };
  auto TE = [&](int sl) -> int { return (int)tp[(NTOKSLOT + sl) * STRIDE] - bias; };
  // line-anchored patterns
  if (p[0] == ']') m |= PM_EL_END;
  if (match_at(p, 0, len, "Audit Trail id")) {
    int j = 14;
    while (j < len && p[j] == ' ') ++j;
    if (j < len && p[j] == ':') m |= PM_AUTR_HDR;
  }
  if (match_at(p, 0, len, "=== jbossId")) {
    for (int i = 11; i + 4 <= len; ++i) {
      if (p[i] == 'I' && p[i + 1] == 'O' && p[i + 2] == '=') {
        if (p[i + 3] == 'I') m |= PM_SOAP_IN;
        if (p[i + 3] == 'O') m |= PM_SOAP_OUT;
      }
    }
  }
  if (xf & XF_BAF) m |= PM_BAF;
  if (xf & XF_NONASCII) m |= PM_HOST;
  const bool ejb_entry = xf & XF_EJB_ENTRY, ejb_exit = xf & XF_EJB_EXIT;
  const bool ct_start = xf & XF_CT_START, ct_stop = xf & XF_CT_STOP;

  ev.ntok = (uint8_t)min(ntok, 15);
  auto tok = [&](int k, uint16_t& s, uint16_t& e) {
    if (k < ntok && k < 16) { s = (uint16_t)TS(tok_slot(k)); e = (uint16_t)TE(tok_slot(k)); }
  };
  tok(0, ev.t0s, ev.t0e);
  tok(1, ev.t1s, ev.t1e);
  tok(2, ev.t2s, ev.t2e);
  tok(3, ev.t3s, ev.t3e);

  // ---- leading-timestamp watermark + ts field
  bool ts_host = false;  // only matters for the timestamped CommonTiming kinds
  unsigned long long wm = 0;  // leading-timestamp watermark candidate (biased), 0 = none
  if (ntok >= 3) {
    double t;
    bool strict;
    const int s1 = TS(tok_slot(1)), e1 = TE(tok_slot(1)), s2 = TS(tok_slot(2)), e2 = TE(tok_slot(2));
    strict = true;
    if (parse_log_ts_fixed(p, s1, e1, s2, e2, a.tz, t) || parse_log_ts(p, s1, e1, s2, e2, a.tz, t, strict)) {
      ev.ts = t;
      if (strict && t == t) {
        wm = (unsigned long long)((long long)t + (1LL << 62));
      }
    } else {
      ts_host = true;
    }
  }

  // ---- classification by file kind (reference dispatch order)
  uint8_t kind = LK_NONE;
  if (fk == FILE_SOAP) {
    // parseSoapLine: IN, OUT, then (with context) ACCT, KEY, VALUE
    if (m & (PM_SOAP_IN | PM_SOAP_OUT | PM_SOAP_ACCT | PM_SOAP_KEY | PM_SOAP_VALUE)) kind = LK_SOAP;
    m &= (PM_SOAP_IN | PM_SOAP_OUT | PM_SOAP_ACCT | PM_SOAP_KEY | PM_SOAP_VALUE | PM_HOST);
  } else {
    if (fk == FILE_SERVER && ejb_entry) kind = LK_EJB_ENTRY;
    else if (fk == FILE_SERVER && ejb_exit) kind = LK_EJB_EXIT;
    else if (ct_start) kind = LK_CT_ENTRY;
    else if (ct_stop) kind = LK_CT_EXIT;
    else if (fk == FILE_APP) {
      m &= ~(PM_SOAP_IN | PM_SOAP_OUT | PM_SOAP_ACCT | PM_SOAP_KEY | PM_SOAP_VALUE);
      if (m & (PM_AUTR_MAP | PM_AUTR_HDR | PM_EL_START | PM_EL_END | PM_SW_START | PM_SW_END |
               PM_SW_NAME | PM_SW_STARTTS | PM_SW_STOPTS))
        kind = LK_APP;
    }
    if (kind == LK_EJB_ENTRY) {
      tok(13, ev.tAs, ev.tAe);
    } else if (kind == LK_EJB_EXIT) {
      tok(9, ev.tAs, ev.tAe);
      tok(11, ev.tBs, ev.tBe);
      if (11 < ntok && !parse_int_tok(p, TS(tok_slot(11)), TE(tok_slot(11)), ev.num)) m |= PM_HOST;
    } else if (kind == LK_CT_ENTRY || kind == LK_CT_EXIT) {
      // line.split(/INFO/)[1].trim().split(/[\s]+/)
      const int s0 = info1 + 4;
      const int e0 = info2 >= 0 ? info2 : len;
      if (info2 >= 0) m |= PM_HAS_INFO2;
      int k = 0;
      bool it = false;
      int cs = 0;
      for (int i = s0; i <= e0; ++i) {
        const bool w = (i == e0) || is_ws(p[i]);
        if (!w && !it) { it = true; cs = i; }
        if (w && it) {
          it = false;
          if (k == 1) { ev.tAs = (uint16_t)cs; ev.tAe = (uint16_t)i; }
          if (k == 5) { ev.tBs = (uint16_t)cs; ev.tBe = (uint16_t)i; }
          ++k;
          if (k > 5) break;
        }
      }
      if (kind == LK_CT_EXIT && ev.tBs != 0xffff &&
          !parse_int_tok(p, ev.tBs, ev.tBe, ev.num)) m |= PM_HOST;
    }
  }
  if (ts_host && kind >= LK_EJB_ENTRY && kind <= LK_CT_EXIT) m |= PM_HOST;
  // join keys: logId = token 0 without its [..] wrapper (.replace(/[[\]]/g,'')); lines with
  // brackets inside the logId keep the raw token and are keyed on the host
  if (kind >= LK_EJB_ENTRY && kind <= LK_CT_EXIT && !(m & PM_HOST) && ntok >= 1) {
    int a0 = ev.t0s, b0 = ev.t0e;
    if (a0 < b0 && p[a0] == '[') ++a0;
    if (b0 > a0 && p[b0 - 1] == ']') --b0;
    bool inner = false;
    for (int i = a0; i < b0; ++i) inner |= (p[i] == '[' || p[i] == ']');
    if (!inner) {
      ev.t0s = (uint16_t)a0;
      ev.t0e = (uint16_t)b0;
      ev.key = hash_bytes(p + a0, (size_t)(b0 - a0));
      const uint64_t seed = kind <= LK_EJB_EXIT ? kHashSeedEjb : kHashSeed;
      ev.svc = ev.tAs != 0xffff ? hash_bytes(p + ev.tAs, (size_t)(ev.tAe - ev.tAs), seed)
                                : hash_bytes("undefined", 9, seed);
      m |= PM_KEYS;
    }
  }
  ev.kind = kind;
  ev.mask = m;
  a.line_mask[li] = m;
  a.keep[li] = kind != LK_NONE;
  a.ev_tmp[li] = ev;
  return wm;
}

// Elapsed-section marking for app files: a line is "in section" when the last of
// {EL_START (open), EL_END (close)} before it in its file is an open; the state carries across
// batches per file.  Two passes over SEC_SEGS segments per chunk (one wave each) instead of one
// wave walking a whole chunk 64 lines at a time (~120 us of dependent loads per batch):
//   k_section_summary: the last open/close event of each segment (0 none, 1 open, 2 close);
//   k_section_apply:   incoming state = the nearest earlier segment with an event (else the
//                      file's carried state), then the 64-lane ballot walk of its own segment.
constexpr int SEC_SEGS = 32;

__device__ __forceinline__ void section_events(uint32_t m, bool valid, bool& is_open, bool& is_close) {
  is_open = valid && (m & PM_EL_START);
  // Only `^]` can end a section (a header with an unknown autrId does not reset the flag, and
  // a line that is also an auditTrailId map line never reaches the elapsed branch).  Treating
  // fewer lines as closers can only over-approximate the section, which the host tolerates.
  is_close = valid && (m & PM_EL_END) && !(m & PM_AUTR_MAP) && !is_open;
}

__device__ __forceinline__ void section_range(const uint32_t* chunk_line_lo, uint32_t c, int g, uint32_t& lo,
                                              uint32_t& hi) {
  const uint32_t c0 = chunk_line_lo[c], c1 = chunk_line_lo[c + 1];
  const uint32_t n = c1 - c0;
  const uint32_t seg = ((n + SEC_SEGS - 1) / SEC_SEGS + APM_WAVE - 1) / APM_WAVE * APM_WAVE;
  lo = min(c1, c0 + (uint32_t)g * seg);
  hi = min(c1, lo + seg);
}

__global__ __launch_bounds__(APM_WAVE) void k_section_summary(const uint32_t* __restrict__ chunk_line_lo,
                                                              const uint8_t* __restrict__ chunk_kind,
                                                              const uint32_t* __restrict__ chunk_file, uint32_t n_chunks,
                                                              const uint32_t* __restrict__ line_mask,
                                                              const uint8_t* __restrict__ file_open,
                                                              uint8_t* __restrict__ seg_state,
                                                              uint8_t* __restrict__ chunk_init) {
  const uint32_t c = blockIdx.x;
  const int g = blockIdx.y;
  if (c >= n_chunks || chunk_kind[c] != FILE_APP) return;
  const int lane = threadIdx.x;
  if (g == 0 && lane == 0) chunk_init[c] = file_open[chunk_file[c]];  // read before the apply pass writes it
  uint32_t lo, hi;
  section_range(chunk_line_lo, c, g, lo, hi);
  uint8_t st = 0;
  for (uint32_t base = lo; base < hi; base += APM_WAVE) {
    const uint32_t li = base + lane;
    const bool valid = li < hi;
    bool is_open, is_close;
    section_events(valid ? line_mask[li] : 0, valid, is_open, is_close);
    const unsigned long long om = __ballot(is_open), cm = __ballot(is_close);
    if (om | cm) st = ((om >> (63 - __clzll(om | cm))) & 1ULL) ? 1 : 2;
  }
  if (lane == 0) seg_state[(size_t)c * SEC_SEGS + g] = st;
}

__global__ __launch_bounds__(APM_WAVE) void k_section_apply(const uint32_t* __restrict__ chunk_line_lo,
                                                            const uint8_t* __restrict__ chunk_kind,
                                                            const uint32_t* __restrict__ chunk_file, uint32_t n_chunks,
                                                            uint32_t* __restrict__ line_mask,
                                                            uint8_t* __restrict__ keep, Event* __restrict__ ev_tmp,
                                                            uint8_t* __restrict__ file_open,
                                                            const uint8_t* __restrict__ seg_state,
                                                            const uint8_t* __restrict__ chunk_init) {
  const uint32_t c = blockIdx.x;
  const int g = blockIdx.y;
  if (c >= n_chunks || chunk_kind[c] != FILE_APP) return;
  const int lane = threadIdx.x;
  bool open = chunk_init[c] != 0;
  for (int h = g - 1; h >= 0; --h) {
    const uint8_t st = seg_state[(size_t)c * SEC_SEGS + h];
    if (st) { open = st == 1; break; }
  }
  uint32_t lo, hi;
  section_range(chunk_line_lo, c, g, lo, hi);
  for (uint32_t base = lo; base < hi; base += APM_WAVE) {
    const uint32_t li = base + lane;
    const bool valid = li < hi;
    const uint32_t m = valid ? line_mask[li] : 0;
    bool is_open, is_close;
    section_events(m, valid, is_open, is_close);
    const unsigned long long om = __ballot(is_open);
    const unsigned long long cm = __ballot(is_close);
    const unsigned long long below = lane ? ((1ULL << lane) - 1ULL) : 0ULL;
    const unsigned long long ob = om & below, cb = cm & below;
    bool in;
    if (!ob && !cb) in = open;
    else {
      const int lo_ = ob ? 63 - __clzll(ob) : -1;
      const int lc_ = cb ? 63 - __clzll(cb) : -1;
      in = lo_ > lc_;
    }
    if (valid && in && !is_open) {
      line_mask[li] = m | PM_IN_SECTION;
      if (!keep[li]) {
        keep[li] = 1;
        ev_tmp[li].kind = LK_APP;
      }
      ev_tmp[li].mask |= PM_IN_SECTION;
    }
    // carry: state after lane 63
    const unsigned long long all = om | cm;
    if (all) {
      const int l = 63 - __clzll(all);
      open = (om >> l) & 1ULL;
    }
  }
  if (g == SEC_SEGS - 1 && lane == 0) {  // the chunk's final state, carried to the next batch
    bool fin = chunk_init[c] != 0;
    for (int h = SEC_SEGS - 1; h >= 0; --h) {
      const uint8_t st = seg_state[(size_t)c * SEC_SEGS + h];
      if (st) { fin = st == 1; break; }
    }
    file_open[chunk_file[c]] = fin ? 1 : 0;
  }
}

// First line of every chunk: the newline pass's per-tile line counts bound the search to the lines
// ending in the chunk start's 4 KB tile (~7 dependent loads, not ~20 over the whole batch: this
// one-lane-per-chunk kernel was pure load latency, 38 us a batch, profiles/r6_g).
__global__ void k_chunk_lines(const uint32_t* __restrict__ chunk_begin, uint32_t n_chunks,
                              const uint32_t* __restrict__ line_end, const uint32_t* __restrict__ n_lines_dev,
                              uint32_t* __restrict__ chunk_line_lo, const uint32_t* __restrict__ tile_off,
                              uint32_t tiles) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c > n_chunks) return;
  const uint32_t n_lines = *n_lines_dev;
  // first line whose end >= chunk_begin[c]: lines ending before tile t number tile_off[t], and
  // the line through tile t's end is at most tile_off[t + 1]
  const uint32_t pos = chunk_begin[c];
  const uint32_t t = pos / (uint32_t)NL_TILE;
  uint32_t lo = t < tiles ? tile_off[t] : n_lines, hi = t < tiles ? tile_off[t + 1] : n_lines;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if (line_end[mid] < pos) lo = mid + 1; else hi = mid;
  }
  chunk_line_lo[c] = lo;
}

struct KeepF {
  const uint8_t* keep;
  __device__ uint32_t operator()(uint32_t i) const { return keep[i]; }
};
struct CompactG {  // keep[i]: event i lands at its rank among the kept lines (line order)
  const uint8_t* keep;
  const Event* ev_tmp;
  Event* out;
  __device__ void operator()(uint32_t i, uint32_t p) const {
    if (keep[i]) out[p] = ev_tmp[i];
  }
};

}  // namespace apm

extern "C" {

constexpr size_t APM_SCAN_TMP = 32u << 20;

size_t apm_parse_workspace_bytes(uint64_t max_bytes, uint32_t max_lines, uint32_t max_chunks) {
  using namespace apm;
  const uint64_t tiles = (max_bytes + NL_TILE - 1) / NL_TILE + 2;
  size_t b = 0;
  b += tiles * 8 + 64;
  b += (size_t)max_lines * (4 + 4 + 4 + 1) + 64;
  b += (size_t)max_lines * sizeof(Event) + 64;
  b += (size_t)(max_chunks + 2) * 4 + 256;
  b += (size_t)(max_chunks + 2) * (SEC_SEGS + 1) + 256;  // section summaries + carried states
  b += APM_SCAN_TMP;
  return b;
}

// K1+K2 (+ section scan + ordered compaction) for one batch already resident on the device.
// Results stay on the device: events[0..*d_n_events), *d_n_lines, the watermark max.
int apm_parse_batch(const uint8_t* d_bytes, uint64_t n_bytes, const uint32_t* d_chunk_begin,
                    const uint8_t* d_chunk_kind, const uint32_t* d_chunk_file, uint32_t n_chunks,
                    void* d_ws, uint32_t max_lines, apm::Event* d_events, uint32_t* d_n_events,
                    uint32_t* d_n_lines, unsigned long long* d_watermark, uint8_t* d_file_open,
                    const apm::TzTable* tz, hipStream_t stream) {
  using namespace apm;
  const uint32_t tiles = (uint32_t)((n_bytes + NL_TILE - 1) / NL_TILE);
  if (tiles == 0 || n_chunks == 0) {
    HIP_OK(hipMemsetAsync(d_n_events, 0, 4, stream));
    HIP_OK(hipMemsetAsync(d_n_lines, 0, 4, stream));
    HIP_OK(hipMemsetAsync(const_cast<uint8_t*>(d_bytes) + n_bytes, 0, 64, stream));
    return 0;
  }
  const uint32_t cap = (uint32_t)std::min<uint64_t>(max_lines, n_bytes);
  uint8_t* w = (uint8_t*)d_ws;
  auto carve = [&](size_t bytes) { uint8_t* r = (uint8_t*)(((uintptr_t)w + 63) & ~(uintptr_t)63); w = r + bytes; return r; };
  uint32_t* tile_counts = (uint32_t*)carve((size_t)(tiles + 1) * 4);
  uint32_t* tile_off = (uint32_t*)carve((size_t)(tiles + 1) * 4);
  uint32_t* line_end = (uint32_t*)carve((size_t)max_lines * 4);
  Event* ev_tmp = (Event*)carve((size_t)max_lines * sizeof(Event));
  uint32_t* line_mask = (uint32_t*)carve((size_t)max_lines * 4);
  uint32_t* pos = (uint32_t*)carve((size_t)max_lines * 4);
  uint8_t* keep = carve((size_t)max_lines);
  uint32_t* chunk_line_lo = (uint32_t*)carve((size_t)(n_chunks + 2) * 4);
  uint8_t* seg_state = carve((size_t)(n_chunks + 2) * SEC_SEGS);
  uint8_t* chunk_init = carve((size_t)(n_chunks + 2));
  void* scan_tmp = carve(APM_SCAN_TMP);

  const uint32_t nl_blocks = (tiles + NL_PER - 1) / NL_PER;
  hipLaunchKernelGGL(k_nl_count, dim3(nl_blocks), dim3(NL_BLOCK), 0, stream, d_bytes, n_bytes, tile_counts,
                     const_cast<uint8_t*>(d_bytes) + n_bytes, tiles);
  size_t tmp_bytes = 0;
  HIP_OK(rocprim::exclusive_scan(nullptr, tmp_bytes, tile_counts, tile_off, 0u, tiles + 1,
                                 rocprim::plus<uint32_t>(), stream));
  if (tmp_bytes > APM_SCAN_TMP) return -1;
  HIP_OK(rocprim::exclusive_scan(scan_tmp, tmp_bytes, tile_counts, tile_off, 0u, tiles + 1,
                                 rocprim::plus<uint32_t>(), stream));
  hipLaunchKernelGGL(k_nl_write, dim3(nl_blocks), dim3(NL_BLOCK), 0, stream, d_bytes, n_bytes, tile_off, line_end,
                     d_n_lines, tiles);

  ParseArgs pa;
  pa.bytes = d_bytes;
  pa.line_end = line_end;
  pa.chunk_begin = d_chunk_begin;
  pa.chunk_kind = d_chunk_kind;
  pa.n_lines_dev = d_n_lines;
  pa.cap_lines = cap;
  pa.n_chunks = n_chunks;
  pa.ev_tmp = ev_tmp;
  pa.line_mask = line_mask;
  pa.keep = keep;
  pa.watermark = d_watermark;
  pa.tz = *tz;
  // APM_PARSE_PROF=1: per-phase cycle counters, printed to stderr every 50 batches
  static unsigned long long* d_prof = nullptr;
  static int prof_batches = 0;
  static const bool prof_on = getenv("APM_PARSE_PROF") != nullptr;
  if (prof_on && !d_prof) {
    HIP_OK(hipMalloc((void**)&d_prof, PP_N * 8));
    HIP_OK(hipMemsetAsync(d_prof, 0, PP_N * 8, stream));
  }
  pa.prof = prof_on ? d_prof : nullptr;
  // K2 kernel: the lane-per-line kernel (one block per 256 lines) by default; APM_PARSE=tile
  // selects the cooperative wave-per-tile kernel (experimental: on the edge-case corpus it still
  // emits events for lines the model drops, tests/test_engine_gpu.py _edge_corpus)
  const char* mode_env = getenv("APM_PARSE");  // read per batch: tests switch it in-process
  const bool by_line = !(mode_env && strcmp(mode_env, "tile") == 0);
  if (by_line)
    hipLaunchKernelGGL(k_parse_lines, dim3((cap + PARSE_BLOCK - 1) / PARSE_BLOCK), dim3(PARSE_BLOCK), 0,
                       stream, pa);
  else
    hipLaunchKernelGGL(k_parse_tiles, dim3(tiles), dim3(APM_WAVE), 0, stream, pa, n_bytes, (const uint32_t*)tile_off);
  if (prof_on && ++prof_batches % 50 == 0) {
    unsigned long long h[PP_N];
    HIP_OK(hipMemcpyAsync(h, d_prof, sizeof h, hipMemcpyDeviceToHost, stream));
    HIP_OK(hipStreamSynchronize(stream));
    const double w = h[PP_WAVES] ? (double)h[PP_WAVES] : 1.0;
    fprintf(stderr, "[parse prof %s] %d batches, %.0f waves/batch; cycles per wave: stage %.0f scan %.0f hits %.0f "
            "lines %.0f; lines coop %llu serial %llu; per coop line: head %.0f tail %.0f\n", by_line ? "line" : "tile",
            prof_batches, w / prof_batches, h[PP_STAGE] / w, h[PP_SCAN] / w, h[PP_HITS] / w, h[PP_LINES] / w,
            (unsigned long long)h[PP_COOP], (unsigned long long)h[PP_SERIAL],
            h[PP_COOP] ? (double)h[PP_HEAD] / h[PP_COOP] : 0.0, h[PP_COOP] ? (double)h[PP_TAIL] / h[PP_COOP] : 0.0);
  }
  hipLaunchKernelGGL(k_chunk_lines, dim3((n_chunks + 1 + 255) / 256), dim3(256), 0, stream, d_chunk_begin,
                     n_chunks, line_end, d_n_lines, chunk_line_lo, tile_off, tiles);
  hipLaunchKernelGGL(k_section_summary, dim3(n_chunks, SEC_SEGS), dim3(APM_WAVE), 0, stream, chunk_line_lo,
                     d_chunk_kind, d_chunk_file, n_chunks, line_mask, d_file_open, seg_state, chunk_init);
  hipLaunchKernelGGL(k_section_apply, dim3(n_chunks, SEC_SEGS), dim3(APM_WAVE), 0, stream, chunk_line_lo,
                     d_chunk_kind, d_chunk_file, n_chunks, line_mask, keep, ev_tmp, d_file_open, seg_state,
                     chunk_init);
  // ordered compaction of the kept events over the batch's lines only (devscan.h: the count is
  // read on the device; `pos` holds the tile sums), the event count -> *d_n_events
  if (ds_scan_apply<uint32_t>(KeepF{keep}, CompactG{keep, ev_tmp, d_events}, d_n_lines, cap, pos, d_n_events,
                              stream) != 0)
    return -1;
  return 0;
}

}  // extern "C"
