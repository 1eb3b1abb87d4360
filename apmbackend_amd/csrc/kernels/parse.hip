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
// (the vast majority) never leave the GPU.  Stateful joins run downstream on the host join
// workers, which read strings from the pinned host copy of the same bytes.
#include "kernel_api.h"

#include <rocprim/rocprim.hpp>

#include <algorithm>

namespace apm {

constexpr int NL_BLOCK = 256;
constexpr int NL_TILE = NL_BLOCK * 16;     // bytes per block in the newline pass
constexpr int PARSE_BLOCK = 256;           // lines per block in the parse pass
constexpr int PARSE_LDS = 32 * 1024;       // staged bytes per block (+ 8 KB token table: 4 blocks / CU)

// --------------------------------------------------------------------------------- K1
__global__ __launch_bounds__(NL_BLOCK) void k_nl_count(const uint8_t* __restrict__ bytes, uint64_t n,
                                                      uint32_t* __restrict__ tile_counts) {
  const uint64_t base = (uint64_t)blockIdx.x * NL_TILE + threadIdx.x * 16;
  int c = 0;
  if (base + 16 <= n) {
    const uint4 v = *reinterpret_cast<const uint4*>(bytes + base);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      // count bytes equal to '\n' (0x0a) in a 32-bit word (SWAR)
      uint32_t x = w[k] ^ 0x0a0a0a0aU;
      uint32_t t = (x - 0x01010101U) & ~x & 0x80808080U;
      c += __popc(t);
    }
  } else {
    for (uint64_t i = base; i < n && i < base + 16; ++i) c += bytes[i] == '\n';
  }
  // block reduction
  __shared__ int red[NL_BLOCK / APM_WAVE];
  for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o, APM_WAVE);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int s = 0;
    for (int i = 0; i < NL_BLOCK / APM_WAVE; ++i) s += red[i];
    tile_counts[blockIdx.x] = s;
  }
}

// Writes the byte position of every '\n' (= line end) in order; tile_off = exclusive scan.
__global__ __launch_bounds__(NL_BLOCK) void k_nl_write(const uint8_t* __restrict__ bytes, uint64_t n,
                                                      const uint32_t* __restrict__ tile_off,
                                                      uint32_t* __restrict__ line_end) {
  const uint64_t base = (uint64_t)blockIdx.x * NL_TILE + threadIdx.x * 16;
  uint8_t b[16];
  int c = 0;
  if (base + 16 <= n) {
    const uint4 v = *reinterpret_cast<const uint4*>(bytes + base);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
      for (int j = 0; j < 4; ++j) b[k * 4 + j] = (uint8_t)(w[k] >> (8 * j));
    }
  } else {
    for (int i = 0; i < 16; ++i) b[i] = (base + i < n) ? bytes[base + i] : 0;
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) c += b[i] == '\n';
  // block exclusive scan of c
  typedef rocprim::block_scan<int, NL_BLOCK> Scan;
  __shared__ typename Scan::storage_type st;
  int excl;
  Scan().exclusive_scan(c, excl, 0, st);
  uint32_t pos = tile_off[blockIdx.x] + excl;
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (b[i] == '\n') line_end[pos++] = (uint32_t)(base + i);
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
  TzTable tz;
};

__device__ __forceinline__ uint32_t find_chunk(const uint32_t* cb, uint32_t n_chunks, uint32_t pos) {
  uint32_t lo = 0, hi = n_chunks - 1;
  while (lo < hi) {
    uint32_t mid = (lo + hi + 1) >> 1;
    if (cb[mid] <= pos) lo = mid; else hi = mid - 1;
  }
  return lo;
}

__device__ __forceinline__ unsigned long long parse_line(const ParseArgs& a, const uint8_t* __restrict__ base,
                                                         uint32_t o, uint32_t li, uint32_t ls, uint32_t le,
                                                         uint16_t* tp);

// --------------------------------------------------------------------------------- K2
__global__ __launch_bounds__(PARSE_BLOCK) void k_parse_lines(ParseArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[PARSE_LDS];
  // token start/end positions of the tokens the classifier reads, slot-major (lane-adjacent
  // entries): one LDS store per token boundary instead of a 7-way register select per byte
  __shared__ uint16_t tok_lds[2 * NTOKSLOT][PARSE_BLOCK];
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
    const uint32_t nvec = (span + 15) >> 4;
    for (uint32_t i = threadIdx.x; i < nvec; i += PARSE_BLOCK) {
      const uint64_t g = (uint64_t)a0 + ((uint64_t)i << 4);
      uint4 v;
      // the buffer is padded by >= 16 bytes on the host, so a full vector load is in bounds
      v = *reinterpret_cast<const uint4*>(a.bytes + g);
      *reinterpret_cast<uint4*>(lds + (i << 4)) = v;
    }
  }
  __syncthreads();
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
    wm = staged ? parse_line(a, lds, ls - a0, li, ls, le, &tok_lds[0][threadIdx.x])
                : parse_line(a, a.bytes, ls, li, ls, le, &tok_lds[0][threadIdx.x]);
  }
  // Watermark: one atomic per wave.  A per-lane atomicMax on the single watermark word put 64
  // same-address atomics per wave through one L2 atomic unit, serialising the whole grid.
  for (int off = APM_WAVE / 2; off > 0; off >>= 1) {
    const unsigned long long o2 = __shfl_xor(wm, off, APM_WAVE);
    wm = o2 > wm ? o2 : wm;
  }
  if ((threadIdx.x & (APM_WAVE - 1)) == 0 && wm) atomicMax(a.watermark, wm);
}

// One line: `base + o` is its first byte; `base` is 16-byte aligned (LDS stage or the batch).
// tp: this lane's column of the block's token table (entry k at tp[k * PARSE_BLOCK]; starts in
// rows 0..6, ends in rows 7..13)
__device__ __forceinline__ unsigned long long parse_line(const ParseArgs& a, const uint8_t* __restrict__ base,
                                                         uint32_t o, uint32_t li, uint32_t ls, uint32_t le,
                                                         uint16_t* tp) {
  const uint8_t* __restrict__ p = base + o;
  int len = (int)(le - ls);
  if (len > 0 && p[len - 1] == '\r') --len;

  Event ev;
  ev.line = li;
  ev.chunk = find_chunk(a.chunk_begin, a.n_chunks, ls);
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
  const uint8_t fk = a.chunk_kind[ev.chunk];
  if (len <= 0 || len > 65000) {
    // empty lines are skipped by readLine; absurdly long lines go to the host verbatim
    a.keep[li] = (len > 65000) ? 1 : 0;
    if (len > 65000) { ev.kind = fk == FILE_SOAP ? LK_SOAP : LK_APP; ev.mask = PM_HOST; }
    a.line_mask[li] = ev.mask;
    a.ev_tmp[li] = ev;
    return 0;
  }

  // ---- single pass: whitespace tokens 0..13, pattern tests, INFO occurrences
  // Start/end of the tokens the classifier reads (0-3, 9, 11, 13), kept in registers: an array
  // indexed by the lane-varying token count forced a per-write waterfall / scratch access
  auto TS = [&](int sl) -> uint16_t& { return tp[sl * PARSE_BLOCK]; };
  auto TE = [&](int sl) -> uint16_t& { return tp[(NTOKSLOT + sl) * PARSE_BLOCK]; };
  int ntok = 0;
  bool in_tok = false;
  if (len > 0 && is_ws(p[0])) { TS(0) = 0; TE(0) = 0; ntok = 1; }  // split gives '' first
  int info1 = -1, info2 = -1;
  bool ejb_entry = false, ejb_exit = false, ct_start = false, ct_stop = false;
  bool baf = false, nonascii = false;
  uint32_t m = 0;
  // The per-byte path is branch-free (rocprofv3: the branchy first version issued ~2 SALU
  // exec-mask instructions per VALU one): token bounds by select, and pattern triggers tested on
  // a 4-byte register window p[i-3..i].  Bytes arrive 16 at a time (one aligned 16-byte load:
  // ds_read_b128 from the stage), so a lane waits on memory once per 16 bytes instead of once
  // per byte; positions where some pattern's first four bytes end are collected in a bit mask
  // and matched after the 16 bytes, in order (the rare path re-reads the line).
  uint32_t win = 0;
  const uint8_t* __restrict__ al = base + (o & ~15u);
  const int lead = (int)(o & 15u);
  for (int g = -lead; g < len; g += 16, al += 16) {
    const uint4 v = *reinterpret_cast<const uint4*>(al);
    const uint32_t vw[4] = {v.x, v.y, v.z, v.w};
    uint32_t hits = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int i = g + k;
      const bool act = i >= 0 && i < len;
      const uint8_t c = (uint8_t)(vw[k >> 2] >> (8 * (k & 3)));
      nonascii |= act && c >= 0x80;
      const bool w = is_ws(c);
      const bool tstart = act && !w && !in_tok;
      const bool tend = act && w && in_tok;
      if (tstart | tend) {
        const int sl = tok_slot_of(ntok);
        if (sl != 15) {
          if (tstart) TS(sl) = (uint16_t)i;
          else TE(sl) = (uint16_t)i;
        }
      }
      ntok += tend ? 1 : 0;
      in_tok = act ? !w : in_tok;
      const uint32_t nwin = (win >> 8) | ((uint32_t)c << 24);
      win = act ? nwin : win;
      // ('<' also covers the case-insensitive "<acc" / "<key" triggers)
      const bool probe = (win == pk4("INFO")) | (win == pk4(": Re")) | ((win & 0xffu) == '<');
      hits |= (act && i >= 3 && probe) ? (1u << k) : 0u;
    }
    while (hits) {
      const int k = __builtin_ctz(hits);
      hits &= hits - 1;
      const int s = g + k - 3;
      const uint32_t w4 = (uint32_t)p[s] | ((uint32_t)p[s + 1] << 8) | ((uint32_t)p[s + 2] << 16) |
                          ((uint32_t)p[s + 3] << 24);
      const uint32_t w4l = (uint32_t)lower(p[s]) | ((uint32_t)lower(p[s + 1]) << 8) |
                           ((uint32_t)lower(p[s + 2]) << 16) | ((uint32_t)lower(p[s + 3]) << 24);
      if (w4 == pk4("INFO")) {
        if (info1 < 0) info1 = s;
        else if (info2 < 0 && s >= info1 + 4) info2 = s;
        int j = s + 4;
        while (j < len && p[j] == ' ') ++j;
        if (match_at(p, j, len, "[CommonTiming] The EJB")) ejb_entry = true;
        if (match_at(p, j, len, "[CommonTiming] Total time")) ejb_exit = true;
        if (match_at(p, j, len, "CommonTiming::Start")) ct_start = true;
        if (match_at(p, j, len, "CommonTiming::Stop")) ct_stop = true;
        if (match_at(p, s, len, "INFO  auditTrailId=")) m |= PM_AUTR_MAP;
        // BAF  \[[^ ]+] +INFO  : the ']' is the last non-space before the spaces preceding an
        // "INFO ", with a '[' at least two columns before it and no space in between
        if (!baf && s + 4 < len && p[s + 4] == ' ' && s >= 1 && p[s - 1] == ' ') {
          int kk0 = s - 1;
          while (kk0 >= 0 && p[kk0] == ' ') --kk0;
          if (kk0 >= 0 && p[kk0] == ']')
            for (int kk = kk0 - 2; kk >= 0 && p[kk] != ' '; --kk)
              if (p[kk] == '[') { baf = true; break; }
        }
      } else if (w4 == pk4(": Re")) {
        if (match_at(p, s, len, ": RequestTrace [stopWatchList=")) m |= PM_EL_START;
      } else if ((w4 & 0xffu) == '<') {
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
  if (baf) m |= PM_BAF;
  if (nonascii) m |= PM_HOST;

  ev.ntok = (uint8_t)min(ntok, 15);
  auto tok = [&](int k, uint16_t& s, uint16_t& e) {
    if (k < ntok && k < 16) { s = TS(tok_slot(k)); e = TE(tok_slot(k)); }
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
    if (parse_log_ts(p, TS(tok_slot(1)), TE(tok_slot(1)), TS(tok_slot(2)), TE(tok_slot(2)), a.tz, t, strict)) {
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

__global__ void k_chunk_lines(const uint32_t* __restrict__ chunk_begin, uint32_t n_chunks,
                              const uint32_t* __restrict__ line_end, const uint32_t* __restrict__ n_lines_dev,
                              uint32_t* __restrict__ chunk_line_lo) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c > n_chunks) return;
  const uint32_t n_lines = *n_lines_dev;
  // first line whose end >= chunk_begin[c]
  const uint32_t pos = chunk_begin[c];
  uint32_t lo = 0, hi = n_lines;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if (line_end[mid] < pos) lo = mid + 1; else hi = mid;
  }
  chunk_line_lo[c] = lo;
}

__global__ void k_compact(const Event* __restrict__ ev_tmp, const uint8_t* __restrict__ keep,
                          const uint32_t* __restrict__ pos, uint32_t n, Event* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && keep[i]) out[pos[i]] = ev_tmp[i];
}

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

  hipLaunchKernelGGL(k_nl_count, dim3(tiles), dim3(NL_BLOCK), 0, stream, d_bytes, n_bytes, tile_counts);
  HIP_OK(hipMemsetAsync(tile_counts + tiles, 0, 4, stream));
  size_t tmp_bytes = 0;
  HIP_OK(rocprim::exclusive_scan(nullptr, tmp_bytes, tile_counts, tile_off, 0u, tiles + 1,
                                 rocprim::plus<uint32_t>(), stream));
  if (tmp_bytes > APM_SCAN_TMP) return -1;
  HIP_OK(rocprim::exclusive_scan(scan_tmp, tmp_bytes, tile_counts, tile_off, 0u, tiles + 1,
                                 rocprim::plus<uint32_t>(), stream));
  hipLaunchKernelGGL(k_nl_write, dim3(tiles), dim3(NL_BLOCK), 0, stream, d_bytes, n_bytes, tile_off, line_end);
  HIP_OK(hipMemcpyAsync(d_n_lines, tile_off + tiles, 4, hipMemcpyDeviceToDevice, stream));

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
  hipLaunchKernelGGL(k_parse_lines, dim3((cap + PARSE_BLOCK - 1) / PARSE_BLOCK), dim3(PARSE_BLOCK), 0,
                     stream, pa);
  hipLaunchKernelGGL(k_chunk_lines, dim3((n_chunks + 1 + 255) / 256), dim3(256), 0, stream, d_chunk_begin,
                     n_chunks, line_end, d_n_lines, chunk_line_lo);
  hipLaunchKernelGGL(k_section_summary, dim3(n_chunks, SEC_SEGS), dim3(APM_WAVE), 0, stream, chunk_line_lo,
                     d_chunk_kind, d_chunk_file, n_chunks, line_mask, d_file_open, seg_state, chunk_init);
  hipLaunchKernelGGL(k_section_apply, dim3(n_chunks, SEC_SEGS), dim3(APM_WAVE), 0, stream, chunk_line_lo,
                     d_chunk_kind, d_chunk_file, n_chunks, line_mask, keep, ev_tmp, d_file_open, seg_state,
                     chunk_init);
  tmp_bytes = 0;
  HIP_OK(rocprim::exclusive_scan(nullptr, tmp_bytes, keep, pos, 0u, cap, rocprim::plus<uint32_t>(), stream));
  if (tmp_bytes > APM_SCAN_TMP) return -1;
  HIP_OK(rocprim::exclusive_scan(scan_tmp, tmp_bytes, keep, pos, 0u, cap, rocprim::plus<uint32_t>(), stream));
  hipLaunchKernelGGL(k_compact, dim3((cap + 255) / 256), dim3(256), 0, stream, ev_tmp, keep, pos, cap, d_events);
  tmp_bytes = 0;
  HIP_OK(rocprim::reduce(nullptr, tmp_bytes, keep, d_n_events, 0u, cap, rocprim::plus<uint32_t>(), stream));
  if (tmp_bytes > APM_SCAN_TMP) return -1;
  HIP_OK(rocprim::reduce(scan_tmp, tmp_bytes, keep, d_n_events, 0u, cap, rocprim::plus<uint32_t>(), stream));
  return 0;
}

}  // extern "C"
