// K13 for the released `db` rows, on the GPU: wire tx lines in the text ring -> COPY rows of the
// transactions table, byte for byte what the host encoder produces (copyenc.cpp encode_line,
// "tx" branch; the reference's TransactionEntry.toPostgresObject, entries.js:23-42, inserted by
// stream_insert_db.js:277-353).  The wire text is parsed as the host does -- split on '|', JS
// parseInt of the numeric fields -- not rebuilt from the join's values, so a '|' inside a name
// shifts the fields exactly as it does there.
//
// Row: ts(end) \t ts(start) \t server \t service \t logId \t int(acct) \t int(elapsed) \t top \n
//   ts(x)   parseInt -> 'YYYY-MM-DD HH:MM:SS.mmm+00' (UTC); NaN -> \N
//   int(x)  String(parseInt(x)); NaN -> \N
//   strings COPY-escaped (\\ \t \n \r); a missing field -> \N
//
// Outside the domain handled here the line is flagged (`fb` counter) and the engine encodes
// the whole release on the host instead: a first field other than "tx", a numeric field with
// leading whitespace or control bytes, a hex prefix, or more than 19 significant digits.
#include "kernel_api.h"

#include <algorithm>
#include <random>
#include <string>
#include <vector>

#include <rocprim/rocprim.hpp>

#include "devjoin_api.h"
#include "devjoin_dev.h"
#include "textout.h"

namespace apm {
namespace {

constexpr int TC_TB = 256;
constexpr int TC_SEP = 9;  // separators recorded: fields 0..8 (tx|srv|norm|lid|acct|start|end|elapsed|top)

struct TxFields {
  const char* p;
  uint32_t len;
  uint32_t nsep;          // '|' seen (capped at TC_SEP)
  uint32_t sep[TC_SEP];   // position of the k-th '|' (len when absent)
  __device__ __forceinline__ bool has(int k) const { return (uint32_t)k <= nsep; }
  __device__ __forceinline__ uint32_t st(int k) const { return k == 0 ? 0u : sep[k - 1] + 1u; }
  __device__ __forceinline__ uint32_t en(int k) const { return sep[k]; }
};

// one pass over the line: 16-byte loads, the '|' bytes of each dword found exactly by SWAR
__device__ __forceinline__ void split_fields(const char* p, uint32_t len, TxFields& f) {
  f.p = p;
  f.len = len;
  f.nsep = 0;
#pragma unroll
  for (int k = 0; k < TC_SEP; ++k) f.sep[k] = len;
  const int lead = (int)((uintptr_t)p & 15u);
  const uint4* a = reinterpret_cast<const uint4*>(p - lead);
  for (int g = -lead; g < (int)len && f.nsep < (uint32_t)TC_SEP; g += 16, ++a) {
    const uint4 v = *a;
    const uint32_t vw[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const uint32_t x = vw[w] ^ 0x7c7c7c7cu;  // '|' bytes -> 0
      uint32_t m = ~((((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) | 0x7f7f7f7fu);  // 0x80 per zero byte
      while (m) {
        const int b = __builtin_ctz(m) >> 3;
        m &= m - 1;
        const int i = g + 4 * w + b;
        if (i < 0 || i >= (int)len) continue;
#pragma unroll
        for (int k = 0; k < TC_SEP; ++k)
          if ((uint32_t)k == f.nsep) f.sep[k] = (uint32_t)i;
        if (f.nsep < (uint32_t)TC_SEP) ++f.nsep;
      }
    }
  }
}

// JS parseInt (radix 10) of field bytes [s, e): false = NaN.  fb: outside the handled domain.
__device__ __forceinline__ bool parse_int_field(const char* p, uint32_t s, uint32_t e, bool& neg, uint64_t& v,
                                                bool& fb) {
  neg = false;
  v = 0;
  uint32_t i = s;
  if (i < e) {
    const uint8_t c0 = (uint8_t)p[i];
    if (c0 <= 0x20 || c0 >= 0x80) { fb = true; return false; }  // (JS whitespace would be skipped)
    if (c0 == '+' || c0 == '-') { neg = c0 == '-'; ++i; }
  }
  if (i + 1 < e && p[i] == '0' && (p[i + 1] | 32) == 'x') { fb = true; return false; }
  bool any = false;
  int sig = 0;
  for (; i < e; ++i) {
    const uint32_t d = (uint32_t)(uint8_t)p[i] - '0';
    if (d > 9) break;
    any = true;
    if (sig || d) {
      if (++sig > 19) { fb = true; return false; }  // (19 digits always fit 64 bits)
      v = v * 10 + d;
    }
  }
  return any;
}

template <bool W>
__device__ __forceinline__ void put_ts(OutT<W>& o, const TxFields& f, int k, bool& fb) {
  bool neg;
  uint64_t v;
  // (ts_text's range: |ms| <= 8.64e15, exact in a double)
  if (!f.has(k) || !parse_int_field(f.p, f.st(k), f.en(k), neg, v, fb) || v > 8640000000000000ull) {
    o.lit("\\N");
    return;
  }
  const int64_t t = neg ? -(int64_t)v : (int64_t)v;
  int64_t days = t / 86400000, rem = t % 86400000;
  if (rem < 0) { rem += 86400000; --days; }
  int y;
  unsigned mo, d;
  {
    int64_t z = days + 719468;
    const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
    const unsigned doe = (unsigned)(z - era * 146097);
    const unsigned yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
    const unsigned doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
    const unsigned mp = (5 * doy + 2) / 153;
    d = doy - (153 * mp + 2) / 5 + 1;
    mo = mp < 10 ? mp + 3 : mp - 9;
    y = (int)(yoe + era * 400) + (mo <= 2);
  }
  // "%04d": the sign counts toward the width
  if (y < 0) {
    o.c('-');
    const uint32_t ay = (uint32_t)(-y);
    if (ay < 100) o.c('0');
    if (ay < 10) o.c('0');
    o.u32(ay);
  } else {
    const uint32_t uy = (uint32_t)y;
    if (uy < 1000) o.c('0');
    if (uy < 100) o.c('0');
    if (uy < 10) o.c('0');
    o.u32(uy);
  }
  const uint32_t r = (uint32_t)rem;
  const uint32_t hh = r / 3600000u, mi = r / 60000u % 60u, ss = r / 1000u % 60u, ms = r % 1000u;
  o.c('-');
  o.c((char)('0' + mo / 10)); o.c((char)('0' + mo % 10));
  o.c('-');
  o.c((char)('0' + d / 10)); o.c((char)('0' + d % 10));
  o.c(' ');
  o.c((char)('0' + hh / 10)); o.c((char)('0' + hh % 10));
  o.c(':');
  o.c((char)('0' + mi / 10)); o.c((char)('0' + mi % 10));
  o.c(':');
  o.c((char)('0' + ss / 10)); o.c((char)('0' + ss % 10));
  o.c('.');
  o.c((char)('0' + ms / 100)); o.c((char)('0' + ms / 10 % 10)); o.c((char)('0' + ms % 10));
  o.lit("+00");
}

template <bool W>
__device__ __forceinline__ void put_int(OutT<W>& o, const TxFields& f, int k, bool& fb) {
  bool neg;
  uint64_t v;
  if (!f.has(k) || !parse_int_field(f.p, f.st(k), f.en(k), neg, v, fb)) { o.lit("\\N"); return; }
  // String(parseInt(x)): the digits are an exact integer v; the parsed Number is v rounded to a
  // double (nearest-even, as the host's strtod), printed JS-style (exact below 2^53; -0 -> 0)
  bool inexact = false;
  const double x = (double)v;
  o.jsnum(neg ? -x : x, inexact);
}

template <bool W>
__device__ __forceinline__ void put_str(OutT<W>& o, const TxFields& f, int k) {
  if (!f.has(k)) { o.lit("\\N"); return; }
  o.copy_text(f.p + f.st(k), (int)(f.en(k) - f.st(k)));
}

template <bool W>
__device__ __forceinline__ void tx_copy_row(const TxFields& f, OutT<W>& o, bool& fb) {
  if (!(f.en(0) == 2 && f.p[0] == 't' && f.p[1] == 'x')) fb = true;  // (the host drops such lines)
  put_ts(o, f, 6, fb); o.c('\t');
  put_ts(o, f, 5, fb); o.c('\t');
  put_str(o, f, 1); o.c('\t');
  put_str(o, f, 2); o.c('\t');
  put_str(o, f, 3); o.c('\t');
  put_int(o, f, 4, fb); o.c('\t');
  put_int(o, f, 7, fb); o.c('\t');
  put_str(o, f, 8);
  o.c('\n');
}

// released line i: ring position << 20 | (length without '\n')
__device__ __forceinline__ const char* tc_line(const int64_t* gid, int64_t i, const char* ring, uint64_t ring_cap,
                                               uint32_t& len) {
  const uint64_t g = (uint64_t)gid[i];
  len = (uint32_t)(g & 0xfffffu);
  return ring + ((g >> 20) & (ring_cap - 1));
}

__global__ __launch_bounds__(TC_TB) void k_txcopy_len(const int64_t* __restrict__ gid, int64_t n_upper,
                                                      const int64_t* __restrict__ d_n, const char* __restrict__ ring,
                                                      uint64_t ring_cap, uint32_t* __restrict__ lens,
                                                      uint32_t* __restrict__ fb_count) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > n_upper) return;
  const int64_t n = d_n ? *d_n : n_upper;
  if (i >= n) { lens[i] = 0; return; }
  uint32_t len;
  const char* p = tc_line(gid, i, ring, ring_cap, len);
  TxFields f;
  split_fields(p, len, f);
  OutT<false> o(nullptr);
  bool fb = false;
  tx_copy_row(f, o, fb);
  lens[i] = o.n;
  if (fb) atomicAdd(fb_count, 1u);
}

__global__ __launch_bounds__(TC_TB) void k_txcopy_write(const int64_t* __restrict__ gid, int64_t n,
                                                        const char* __restrict__ ring, uint64_t ring_cap,
                                                        const uint32_t* __restrict__ offs, char* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t len;
  const char* p = tc_line(gid, i, ring, ring_cap, len);
  TxFields f;
  split_fields(p, len, f);
  OutT<true> o(out + offs[i]);
  bool fb = false;
  tx_copy_row(f, o, fb);
  o.finish();
}

}  // namespace
}  // namespace apm

using namespace apm;

int apm_dj_txcopy_plan(const int64_t* gid, int64_t n_upper, const int64_t* d_n, const char* ring, uint64_t ring_cap,
                       uint32_t* lens, uint32_t* offs, uint32_t* fb_count, void* tmp, size_t tmp_bytes, hipStream_t s) {
  hipLaunchKernelGGL(k_txcopy_len, dim3((unsigned)((n_upper + 1 + TC_TB - 1) / TC_TB)), dim3(TC_TB), 0, s, gid, n_upper,
                     d_n, ring, ring_cap, lens, fb_count);
  size_t need = 0;
  HIP_OK(rocprim::exclusive_scan(nullptr, need, lens, offs, 0u, (size_t)n_upper + 1, rocprim::plus<uint32_t>(), s));
  if (need > tmp_bytes) return -1;
  HIP_OK(rocprim::exclusive_scan(tmp, need, lens, offs, 0u, (size_t)n_upper + 1, rocprim::plus<uint32_t>(), s));
  return 0;
}

void apm_dj_txcopy_write(const int64_t* gid, int64_t n, const char* ring, uint64_t ring_cap, const uint32_t* offs,
                         char* out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_txcopy_write, dim3((unsigned)((n + TC_TB - 1) / TC_TB)), dim3(TC_TB), 0, s, gid, n, ring,
                     ring_cap, offs, out);
}

namespace apm {

// Test entry: COPY rows of wire lines in a device buffer (line i = [line_off[i], line_off[i + 1])
// without its '\n'), through the same kernels; returns the fallback count.
int apm_txcopy_lines(const char* d_text, const uint64_t* h_line_off, int64_t n, std::string& out_rows) {
  std::vector<int64_t> h_gid((size_t)n);
  uint64_t cap = 1;
  while (cap < h_line_off[n] + 64) cap <<= 1;
  for (int64_t i = 0; i < n; ++i) {
    const uint64_t len = h_line_off[i + 1] - h_line_off[i] - 1;
    h_gid[(size_t)i] = (int64_t)((h_line_off[i] << 20) | len);
  }
  int64_t* d_gid = nullptr;
  uint32_t *d_lens = nullptr, *d_offs = nullptr, *d_fb = nullptr;
  HIP_OK(hipMalloc(&d_gid, (size_t)n * 8 + 8));
  HIP_OK(hipMalloc(&d_lens, ((size_t)n + 1) * 4));
  HIP_OK(hipMalloc(&d_offs, ((size_t)n + 1) * 4));
  HIP_OK(hipMalloc(&d_fb, 4));
  HIP_OK(hipMemset(d_fb, 0, 4));
  HIP_OK(hipMemcpy(d_gid, h_gid.data(), (size_t)n * 8, hipMemcpyHostToDevice));
  size_t need = 0;
  HIP_OK(rocprim::exclusive_scan(nullptr, need, d_lens, d_offs, 0u, (size_t)n + 1, rocprim::plus<uint32_t>(), 0));
  void* tmp = nullptr;
  HIP_OK(hipMalloc(&tmp, need + 256));
  if (apm_dj_txcopy_plan(d_gid, n, nullptr, d_text, cap, d_lens, d_offs, d_fb, tmp, need + 256, 0) != 0)
    throw std::runtime_error("txcopy scan scratch");
  uint32_t total = 0, fb = 0;
  HIP_OK(hipMemcpy(&total, d_offs + n, 4, hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(&fb, d_fb, 4, hipMemcpyDeviceToHost));
  char* d_out = nullptr;
  HIP_OK(hipMalloc(&d_out, (size_t)total + 64));
  apm_dj_txcopy_write(d_gid, n, d_text, cap, d_offs, d_out, 0);
  out_rows.resize(total);
  HIP_OK(hipMemcpy(out_rows.data(), d_out, total, hipMemcpyDeviceToHost));
  HIP_OK(hipFree(d_out));
  HIP_OK(hipFree(tmp));
  HIP_OK(hipFree(d_gid));
  HIP_OK(hipFree(d_lens));
  HIP_OK(hipFree(d_offs));
  HIP_OK(hipFree(d_fb));
  return (int)fb;
}


// Isolated timing of the release kernels (tools/release_bench.py): n synthetic wire tx lines
// (16-digit accounts, 13-digit timestamps, ~100 B) laid out contiguously in a ring, released in
// a shuffled order (released lines hop between the batch regions of the ring), gathered `iters`
// times by k_gather_lines and encoded as COPY rows by the txcopy kernels, each alone on one
// stream.  Returns {lines, wire_bytes, copy_bytes, gather_us, txcopy_us (plan + write),
// txcopy_write_us, fallbacks}.
std::vector<double> apm_release_bench(int64_t n, int iters, uint64_t seed) {
  std::mt19937_64 rng(seed);
  std::string text;
  std::vector<int64_t> gid((size_t)n);
  char buf[256];
  for (int64_t i = 0; i < n; ++i) {
    const int jvm = (int)(rng() % 8), svc = (int)(rng() % 10000);
    const unsigned long long acct = 1000000000000000ull + rng() % 9000000000000000ull;
    const long long start = 1578391200000ll + (long long)(rng() % 600000), el = (long long)(rng() % 2000);
    const int k = std::snprintf(buf, sizeof buf, "tx|jvm%02d|S:getSvc%04d|JVM%02d-%08lld|%llu|%lld|%lld|%lld|%c", jvm,
                                svc, jvm, (long long)i, acct, start, start + el, el, (rng() & 1) ? 'Y' : 'N');
    gid[(size_t)i] = (int64_t)(((uint64_t)text.size() << 20) | (uint64_t)k);
    text.append(buf, (size_t)k);
    text += '\n';
  }
  std::shuffle(gid.begin(), gid.end(), rng);
  uint64_t cap = 1;
  while (cap < text.size() + 64) cap <<= 1;
  char *d_ring = nullptr, *d_out = nullptr;
  int64_t* d_gid = nullptr;
  uint32_t *d_lens = nullptr, *d_offs = nullptr, *d_fb = nullptr;
  HIP_OK(hipMalloc(&d_ring, cap));
  HIP_OK(hipMemset(d_ring, 0, cap));
  HIP_OK(hipMemcpy(d_ring, text.data(), text.size(), hipMemcpyHostToDevice));
  HIP_OK(hipMalloc(&d_gid, (size_t)n * 8 + 8));
  HIP_OK(hipMemcpy(d_gid, gid.data(), (size_t)n * 8, hipMemcpyHostToDevice));
  HIP_OK(hipMalloc(&d_lens, ((size_t)n + 1) * 4));
  HIP_OK(hipMalloc(&d_offs, ((size_t)n + 1) * 4));
  HIP_OK(hipMalloc(&d_fb, 4));
  HIP_OK(hipMemset(d_fb, 0, 4));
  HIP_OK(hipMalloc(&d_out, text.size() * 3 + 64));
  size_t need = 0;
  HIP_OK(rocprim::exclusive_scan(nullptr, need, d_lens, d_offs, 0u, (size_t)n + 1, rocprim::plus<uint32_t>(), 0));
  void* tmp = nullptr;
  HIP_OK(hipMalloc(&tmp, need + 256));
  hipStream_t st;
  HIP_OK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  HIP_OK(hipEventCreate(&e0));
  HIP_OK(hipEventCreate(&e1));
  auto elapsed_us = [&]() {
    float ms = 0;
    HIP_OK(hipEventSynchronize(e1));
    HIP_OK(hipEventElapsedTime(&ms, e0, e1));
    return 1000.0 * ms / iters;
  };
  // wire gather
  if (apm_dj_gather_plan(d_gid, n, nullptr, d_lens, d_offs, tmp, need + 256, st) != 0) throw std::runtime_error("bench scan");
  apm_dj_gather_copy(d_gid, n, d_ring, cap, d_offs, d_out, text.size(), st);  // warm
  HIP_OK(hipEventRecord(e0, st));
  for (int i = 0; i < iters; ++i) apm_dj_gather_copy(d_gid, n, d_ring, cap, d_offs, d_out, text.size(), st);
  HIP_OK(hipEventRecord(e1, st));
  const double gather_us = elapsed_us();
  // COPY rows: plan + write, then write alone
  if (apm_dj_txcopy_plan(d_gid, n, nullptr, d_ring, cap, d_lens, d_offs, d_fb, tmp, need + 256, st) != 0)
    throw std::runtime_error("bench scan");
  HIP_OK(hipEventRecord(e0, st));
  for (int i = 0; i < iters; ++i) {
    if (apm_dj_txcopy_plan(d_gid, n, nullptr, d_ring, cap, d_lens, d_offs, d_fb, tmp, need + 256, st) != 0)
      throw std::runtime_error("bench scan");
    apm_dj_txcopy_write(d_gid, n, d_ring, cap, d_offs, d_out, st);
  }
  HIP_OK(hipEventRecord(e1, st));
  const double txcopy_us = elapsed_us();
  HIP_OK(hipEventRecord(e0, st));
  for (int i = 0; i < iters; ++i) apm_dj_txcopy_write(d_gid, n, d_ring, cap, d_offs, d_out, st);
  HIP_OK(hipEventRecord(e1, st));
  const double write_us = elapsed_us();
  uint32_t copy_bytes = 0, fb = 0;
  HIP_OK(hipMemcpy(&copy_bytes, d_offs + n, 4, hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(&fb, d_fb, 4, hipMemcpyDeviceToHost));
  HIP_OK(hipEventDestroy(e0));
  HIP_OK(hipEventDestroy(e1));
  HIP_OK(hipStreamDestroy(st));
  for (void* p : {(void*)d_ring, (void*)d_out, (void*)d_gid, (void*)d_lens, (void*)d_offs, (void*)d_fb, tmp})
    HIP_OK(hipFree(p));
  return {(double)n, (double)text.size(), (double)copy_bytes, gather_us, txcopy_us, write_us, (double)fb};
}

}  // namespace apm
