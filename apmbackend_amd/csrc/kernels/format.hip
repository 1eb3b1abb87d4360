// K12: st / fs record encoding on the GPU (entries.js StatEntry.toCSVString :71-73,
// FullStatEntry.toCSVString :116-118, nf() :116).
//
// Every rollover emits one `st` line per live series and one `fs` line per (series, LAG) -- for
// 80k series and two LAGs that is ~25 MB of text per 10 s interval, far too much to format on
// the host thread that owns the pipeline.  The classic two-pass scheme:
//   pass 1  one lane per series in emission order: line lengths (st, sum over LAGs of fs)
//   scan    exclusive prefix sums (rocprim) -> byte offsets
//   pass 2  same lane re-formats straight into the output at its offset
// Number printing reproduces Number.prototype.toFixed exactly: the rounding decision uses the
// error-free product x*10^f = p + e (fma), ties to the larger n (ECMA-262 21.1.3.3), then the
// integer n is printed with the decimal point inserted f digits from the right.  From 2^52 the
// scaled product is an integer and the error term alone decides; from 2^53 the value itself is
// an integer; from 1e21 JS prints String(x).  Only |x| >= 2^127 is not exact (flagged, counted).
#include "kernel_api.h"  // (common.h pulls <cstring> in before rocprim)
#include "devjoin_dev.h"
#include "textout.h"

#include <rocprim/rocprim.hpp>

#include <cstdlib>

namespace apm {

namespace {

template <bool W>
__device__ __forceinline__ void head(OutT<W>& o, bool st, const FormatArgs& a, int32_t s) {
  if (st) o.lit("st|"); else o.lit("fs|");
  o.sb(a.ts_wire, a.ts_wire_len);
  const int4 nm = a.series_names[s];
  o.s(a.names + nm.x, nm.y);
  o.c('|');
  o.s(a.names + nm.z, nm.w);
  o.c('|');
}

// st line of emission position i (empty for a series without a tx yet)
template <bool W>
__device__ __forceinline__ void st_line(const FormatArgs& a, int32_t i, OutT<W>& st, bool& fb) {
  const int32_t s = a.perm[i];
  const WinStat w = a.win[s];
  if (!w.active) return;
  head(st, true, a, s);
  st.fixed(w.tpm, 2, fb); st.c('|');
  st.fixed(w.avg, 1, fb); st.c('|');
  st.fixed(w.p75, 1, fb); st.c('|');
  st.fixed(w.p95, 1, fb); st.c('\n');
}

// fs line j = (emission position i, LAG rank li): lines of one series are consecutive, LAGs
// ascending (FullStatEntry per LAG, stream_calc_z_score.js:282-306)
template <bool W>
__device__ __forceinline__ void fs_line(const FormatArgs& a, int32_t j, OutT<W>& fs, bool& fb) {
  const int32_t i = j / a.n_lags, li = j - i * a.n_lags;
  const int32_t s = a.perm[i];
  const WinStat w = a.win[s];
  if (!w.active) return;
  const int l = a.lag_order[li];
  const ZOut z = a.z[l][s];
  const double x[NSTAT] = {w.avg, w.p75, w.p95};
  if (a.fs_copy) {
    // FullStatEntry.toPostgresObject (entries.js:120-151) as COPY text, field for field what
    // copyenc.cpp makes of the wire line
    const int4 nm = a.series_names[s];
    fs.sb(a.ts_copy, a.ts_copy_len);
    fs.c('\t');
    fs.copy_text(a.names + nm.x, nm.y);
    fs.c('\t');
    fs.copy_text(a.names + nm.z, nm.w);
    fs.c('\t');
    fs.js_fixed(w.tpm, 2, false, fb);
    fs.c('\t');
    fs.u((uint64_t)a.lag_value[l]);
    fs.lit("\t{\"average\":");
#pragma unroll
    for (int k = 0; k < NSTAT; ++k) {
      if (k == 1) fs.lit(",\"per75\":");
      if (k == 2) fs.lit(",\"per95\":");
      const char* nmk = k == 0 ? "average" : (k == 1 ? "per75" : "per95");
      const int nl = k == 0 ? 7 : 5;
      fs.js_fixed(x[k], 1, true, fb);
      fs.lit(",\""); fs.sb(nmk, nl); fs.lit("avg\":");
      fs.js_fixed(z.mean[k], 1, true, fb);
      fs.lit(",\""); fs.sb(nmk, nl); fs.lit("lb\":");
      fs.js_fixed(z.lb[k], 1, true, fb);
      fs.lit(",\""); fs.sb(nmk, nl); fs.lit("ub\":");
      fs.js_fixed(z.ub[k], 1, true, fb);
      fs.lit(",\""); fs.sb(nmk, nl); fs.lit("signal\":");
      fs.i64(z.sig[k]);
    }
    fs.c('}');
    fs.c('\n');
  } else {
    head(fs, false, a, s);
    fs.u((uint64_t)a.lag_value[l]);
    fs.c('|');
    fs.fixed(w.tpm, 2, fb);
#pragma unroll
    for (int k = 0; k < NSTAT; ++k) {
      fs.c('|');
      fs.fixed(x[k], 1, fb); fs.c(':');
      fs.fixed(z.mean[k], 1, fb); fs.c(':');
      fs.fixed(z.lb[k], 1, fb); fs.c(':');
      fs.fixed(z.ub[k], 1, fb); fs.c(':');
      // averageSignal is printed raw, the percentile signals through nf (entries.js:117)
      if (k == 0) fs.i64(z.sig[k]);
      else fs.fixed((double)z.sig[k], 1, fb);
    }
    fs.c('\n');
  }
}

// Length pass: one lane per LINE (st: n, fs: n * n_lags), not per series -- ~3x the waves of
// a series per lane, which the formatting's long dependent VALU chains need for latency hiding
// (80k series were ~1.2 waves per SIMD).
__global__ __launch_bounds__(256) void k_format_len(FormatArgs a) {
  const int32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  const int32_t nfs = a.n * a.n_lags;
  bool fb = false;
  if (j < a.n) {
    OutT<false> o(nullptr);
    if (a.want_st) st_line(a, j, o, fb);
    a.st_len[j] = o.n;
  } else if (j == a.n) {
    a.st_len[a.n] = 0;  // scan sentinel (-> total)
  }
  if (j < nfs) {
    OutT<false> o(nullptr);
    if (a.want_fs) fs_line(a, j, o, fb);
    a.fs_len[j] = o.n;
  } else if (j == nfs) {
    a.fs_len[nfs] = 0;
  }
  if (fb) atomicAdd(a.fallback, 1);
}

// Write pass, one wave per 64 consecutive lines of one stream, so the wave's output is one
// contiguous byte range.  Each lane formats its line into an LDS stage at the same offset modulo
// 4 as in the output (dword stores, see OutT), then the wave copies the range out one dword per
// lane per store (256 B per store instruction).  A block whose range does not fit the stage
// (very long names) writes its lines to HBM directly.
constexpr int FMT_WAVE_LINES = 64;
// Stage size: 8 / 12 / 16 / 24 KB by the bytes of an average 64-line block of the previous
// batch's longer stream (FormatArgs::stage_hint); a block a little over the stage writes to HBM
// directly -- the next size up costs occupancy on every block (this latency-bound writer runs
// LDS-limited).  A fixed 8 KB stage held only st blocks: 64 fs wire lines (~150 B) are ~9.6 KB,
// so nearly every fs block wrote to HBM directly (46 of 7233 LDS instructions per dispatch,
// profiles/r5_n); 12 KB: the write pass 75 -> 47 us per batch, 16 KB 77 us (profiles/r5_o).
// Stage layouts that avoid the stores' bank conflicts (odd-pitch per-line slots, rows rotated by
// index: 0.6-0.7 conflict cycles per LDS instruction against 5.1-6.6 here) measured slower: more
// LDS per block, or computed store addresses (no immediate offsets) that took the writer from 105
// to 162 VGPRs (profiles/r5_q .. r5_u).  APM_FMT_STAGE=0 / 8 / 12 / 16 / 24 forces one.
constexpr uint32_t FMT_LDS = 8192;

__device__ __forceinline__ void wave_copy_out(const char* __restrict__ lds, char* __restrict__ out, uint32_t g0,
                                              uint32_t g1) {
  const uint32_t a0 = g0 & ~3u;
  const uint32_t nd = (g1 - a0 + 3) / 4;
  for (uint32_t d = threadIdx.x; d < nd; d += FMT_WAVE_LINES) {
    const uint32_t ga = a0 + 4 * d;
    if (ga >= g0 && ga + 4 <= g1) {
      *reinterpret_cast<uint32_t*>(out + ga) = *reinterpret_cast<const uint32_t*>(lds + 4 * d);
    } else {  // the block's first / last dword is shared with a neighbour: byte stores
      for (uint32_t b = 0; b < 4; ++b)
        if (ga + b >= g0 && ga + b < g1) out[ga + b] = lds[4 * d + b];
    }
  }
}

template <uint32_t LDS>
__global__ __launch_bounds__(FMT_WAVE_LINES) void k_format_write(FormatArgs a, int32_t st_blocks) {
  __shared__ __align__(16) char stage[LDS ? LDS : 16];
  const bool is_st = (int32_t)blockIdx.x < st_blocks;
  const int32_t nl = is_st ? a.n : a.n * a.n_lags;
  const int32_t j0 = (is_st ? (int32_t)blockIdx.x : (int32_t)blockIdx.x - st_blocks) * FMT_WAVE_LINES;
  const int32_t j1 = min(nl, j0 + FMT_WAVE_LINES);
  const int32_t j = j0 + (int32_t)threadIdx.x;
  const uint32_t* off = is_st ? a.st_off : a.fs_off;
  char* out = is_st ? a.st_out : a.fs_out;
  const uint32_t g0 = off[j0], g1 = off[j1];
  const bool lds = LDS != 0 && (g1 - (g0 & ~3u)) <= LDS;  // uniform across the block
  if (j < j1) {
    bool fb = false;
    OutT<true> o(lds ? stage + (off[j] - (g0 & ~3u)) : out + off[j]);
    if (is_st) st_line(a, j, o, fb);
    else fs_line(a, j, o, fb);
    o.finish();
  }
  __syncthreads();
  if (lds) wave_copy_out(stage, out, g0, g1);
}

// ---- fb: fleet baseline rows ------------------------------------------------------------
// wire: fb|<edge_ts>|<service>|<lag>|<n>|<avg mean>:<avg std>|<p75 mean>:<p75 std>|<p95 mean>:<p95 std>
// COPY: <ts>\t<service>\t<lag>\t<n>\t{"averagemean":..,"averagestd":..,"per75mean":..,...}
// mean / std: of the series' z-score baseline means across the fleet (population std).
template <bool WRITE>
__device__ __forceinline__ uint32_t fleet_row(const FleetFormatArgs& a, int32_t i, char* dst, bool& fb) {
  const int32_t slot = a.slot_lo + i / a.n_lags, li = i % a.n_lags;
  const int l = a.lag_order[li];
  const double* m = a.moments + ((size_t)slot * a.n_lags + l) * NSTAT * 3;
  OutT<WRITE> o(WRITE ? dst : nullptr);
  const double n0 = m[0];
  if (n0 > 0) {
    const int2 nm = a.names[slot];
    double mean[NSTAT], sd[NSTAT];
    for (int k = 0; k < NSTAT; ++k) {
      const double n = m[k * 3 + 0];
      if (n > 0) {
        mean[k] = m[k * 3 + 1] / n;
        sd[k] = sqrt(fmax(m[k * 3 + 2] / n - mean[k] * mean[k], 0.0));
      } else {
        mean[k] = sd[k] = apm_nan();
      }
    }
    if (a.copy) {
      o.sb(a.ts, a.ts_len); o.c('\t');
      o.copy_text(a.chars + nm.x, nm.y); o.c('\t');
      o.u((uint64_t)a.lag_value[l]); o.c('\t');
      o.u((uint64_t)n0); o.c('\t');
      const char* key[NSTAT] = {"average", "per75", "per95"};
      const int kl[NSTAT] = {7, 5, 5};
      o.c('{');
      for (int k = 0; k < NSTAT; ++k) {
        if (k) o.c(',');
        o.c('"'); o.sb(key[k], kl[k]); o.lit("mean\":"); o.js_fixed(mean[k], 1, true, fb);
        o.lit(",\""); o.sb(key[k], kl[k]); o.lit("std\":"); o.js_fixed(sd[k], 1, true, fb);
      }
      o.c('}');
    } else {
      o.lit("fb|"); o.i64(a.edge_ts); o.c('|');
      o.s(a.chars + nm.x, nm.y); o.c('|');
      o.u((uint64_t)a.lag_value[l]); o.c('|');
      o.u((uint64_t)n0);
      for (int k = 0; k < NSTAT; ++k) {
        o.c('|'); o.fixed(mean[k], 1, fb); o.c(':'); o.fixed(sd[k], 1, fb);
      }
    }
    o.c('\n');
  }
  o.finish();
  return o.n;
}

// Two passes, no scan launch and no look-back: k_fleet_len stores each 64-row wave's byte total;
// k_fleet_rows has every wave add up the totals before it (<= a few hundred words, 64 lanes at a
// time), scan its own rows across lanes, format them into an LDS stage laid out like the output
// and copy the stage out with dword stores.  (Round 4's one-pass decoupled look-back made each wave
// wait for its predecessor's inclusive prefix: on the lowest-priority stream, behind other
// streams' waves, a serial chain of 313 waves -- 100-240 us for ~1.3 MB, ~13 GB/s,
// profiles/r5_n / r5_o timeline.)
constexpr uint32_t FLEET_LDS = 16384;
// Rows per wave (the other lanes carry none): a row's formatting is a long dependent chain per
// lane, and 64 rows a wave left ~313 waves for the headline's 20k rows -- a third of the chip's
// 1024 SIMDs with one latency-bound wave each (101 us isolated, profiles/r5_v).  16 rows a wave
// put four times the waves in flight.  APM_FB_RPW (16 / 32 / 64) for A/B.
int fleet_rows_per_wave() {
  static const int v = [] {
    const char* e = std::getenv("APM_FB_RPW");
    const int r = e ? std::atoi(e) : 16;
    return (r == 8 || r == 16 || r == 32 || r == 64) ? r : 16;
  }();
  return v;
}

__global__ __launch_bounds__(FMT_WAVE_LINES) void k_fleet_len(FleetFormatArgs a, int rpw) {
  const int32_t n = a.n_slots * a.n_lags;
  const int32_t i = (int)threadIdx.x < rpw ? (int32_t)blockIdx.x * rpw + (int32_t)threadIdx.x : n;
  bool fb = false;
  uint32_t len = i < n ? fleet_row<false>(a, i, nullptr, fb) : 0u;
  if (fb) atomicAdd(a.fallback, 1);  // (counted here only)
#pragma unroll
  for (int d = FMT_WAVE_LINES / 2; d > 0; d >>= 1) len += __shfl_xor(len, d, FMT_WAVE_LINES);
  if (threadIdx.x == 0) a.status[blockIdx.x] = len;
}

__global__ __launch_bounds__(FMT_WAVE_LINES) void k_fleet_rows(FleetFormatArgs a, int rpw) {
  __shared__ __align__(16) char stage[FLEET_LDS];
  const int32_t n = a.n_slots * a.n_lags;
  const int32_t i = (int)threadIdx.x < rpw ? (int32_t)blockIdx.x * rpw + (int32_t)threadIdx.x : n;
  const int lane = (int)threadIdx.x;
  bool fb = false;
  const uint32_t len = i < n ? fleet_row<false>(a, i, nullptr, fb) : 0u;
  // wave scan of the row lengths
  uint32_t inc = len;
#pragma unroll
  for (int d = 1; d < FMT_WAVE_LINES; d <<= 1) {
    const uint32_t y = __shfl_up(inc, d, FMT_WAVE_LINES);
    if (lane >= d) inc += y;
  }
  const uint32_t total = __shfl(inc, FMT_WAVE_LINES - 1, FMT_WAVE_LINES);
  // the waves before this one
  uint32_t prefix = 0;
  for (uint32_t k = (uint32_t)lane; k < blockIdx.x; k += FMT_WAVE_LINES) prefix += (uint32_t)a.status[k];
#pragma unroll
  for (int d = FMT_WAVE_LINES / 2; d > 0; d >>= 1) prefix += __shfl_xor(prefix, d, FMT_WAVE_LINES);
  if (blockIdx.x == gridDim.x - 1 && lane == 0) *a.total = prefix + total;
  const uint32_t g0 = prefix, g1 = prefix + total;
  const uint32_t off = prefix + inc - len;
  const bool lds = (g1 - (g0 & ~3u)) <= FLEET_LDS;  // uniform across the wave
  bool fb2 = false;
  if (i < n && len) fleet_row<true>(a, i, lds ? stage + (off - (g0 & ~3u)) : a.out + off, fb2);
  __syncthreads();
  if (lds) wave_copy_out(stage, a.out, g0, g1);
}

__global__ void k_fixed_batch(const double* x, int n, int f, char* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  bool fb = false;
  OutT<true> o(out + (size_t)i * 32);
  o.fixed(x[i], f, fb);
  o.c('\0');
  o.finish();
  if (fb) {
    OutT<true> q(out + (size_t)i * 32);
    q.lit("<fallback>");
    q.c('\0');
    q.finish();
  }
}

}  // namespace

}  // namespace apm

extern "C" {
using namespace apm;

size_t apm_format_tmp_bytes(int32_t n_max) {
  size_t b = 0;
  rocprim::exclusive_scan(nullptr, b, (uint32_t*)nullptr, (uint32_t*)nullptr, 0u, (size_t)n_max + 1,
                          rocprim::plus<uint32_t>(), (hipStream_t)0);
  return b;
}

// Lengths + scan: afterwards st_off/fs_off[0..n] hold exclusive offsets, [n] = total bytes.
// The *_len / *_off arrays hold n + 1 entries.
int apm_format_plan(FormatArgs* a, void* tmp, size_t tmp_bytes, hipStream_t stream) {
  if (a->n <= 0) return 0;
  // a->fallback accumulates (values beyond 2^127, printed inexactly) and is never reset here
  const int32_t lanes = a->n * a->n_lags + 1;  // >= n + 1 (n_lags >= 1)
  hipLaunchKernelGGL(k_format_len, dim3((lanes + 255) / 256), dim3(256), 0, stream, *a);
  size_t need = tmp_bytes;
  if (rocprim::exclusive_scan(tmp, need, a->st_len, a->st_off, 0u, (size_t)a->n + 1, rocprim::plus<uint32_t>(),
                              stream) != hipSuccess)
    return -1;
  need = tmp_bytes;
  if (rocprim::exclusive_scan(tmp, need, a->fs_len, a->fs_off, 0u, (size_t)a->n * a->n_lags + 1,
                              rocprim::plus<uint32_t>(), stream) != hipSuccess)
    return -1;
  return 0;
}

// Test hook: nf(x[i], f) into 32-byte NUL-terminated slots.
void apm_format_fixed_batch(const double* d_x, int n, int f, char* d_out, hipStream_t stream) {
  if (n > 0) hipLaunchKernelGGL(k_fixed_batch, dim3((n + 255) / 256), dim3(256), 0, stream, d_x, n, f, d_out);
}

uint32_t apm_fleet_format_blocks(int32_t n_rows) {
  const int32_t rpw = fleet_rows_per_wave();
  return (uint32_t)((std::max<int32_t>(n_rows, 1) + rpw - 1) / rpw);
}

// two launches; afterwards *a->total holds the bytes written (device)
void apm_fleet_format(FleetFormatArgs* a, hipStream_t stream) {
  const int32_t n = a->n_slots * a->n_lags;
  if (n <= 0) {
    HIP_OK(hipMemsetAsync(a->total, 0, 4, stream));
    return;
  }
  const dim3 grid(apm_fleet_format_blocks(n));
  const int rpw = fleet_rows_per_wave();
  hipLaunchKernelGGL(k_fleet_len, grid, dim3(FMT_WAVE_LINES), 0, stream, *a, rpw);
  hipLaunchKernelGGL(k_fleet_rows, grid, dim3(FMT_WAVE_LINES), 0, stream, *a, rpw);
}

void apm_format_write(FormatArgs* a, hipStream_t stream) {
  if (a->n <= 0) return;
  const int32_t st_blocks = a->want_st ? (a->n + FMT_WAVE_LINES - 1) / FMT_WAVE_LINES : 0;
  const int32_t fs_blocks = a->want_fs ? (a->n * a->n_lags + FMT_WAVE_LINES - 1) / FMT_WAVE_LINES : 0;
  const dim3 grid(st_blocks + fs_blocks);
  if (grid.x == 0) return;
  static const int forced = [] {
    const char* e = std::getenv("APM_FMT_STAGE");  // diagnostic: stage KB (0 = no LDS stage)
    return e ? std::atoi(e) : -1;
  }();
  const uint32_t want = forced >= 0 ? (uint32_t)forced * 1024u : (a->stage_hint ? a->stage_hint : 12288u);
  if (forced == 0)
    hipLaunchKernelGGL(k_format_write<0>, grid, dim3(FMT_WAVE_LINES), 0, stream, *a, st_blocks);
  else if (want <= 7168)
    hipLaunchKernelGGL(k_format_write<FMT_LDS>, grid, dim3(FMT_WAVE_LINES), 0, stream, *a, st_blocks);
  else if (want <= 12800)
    hipLaunchKernelGGL(k_format_write<12288>, grid, dim3(FMT_WAVE_LINES), 0, stream, *a, st_blocks);
  else if (want <= 16896)
    hipLaunchKernelGGL(k_format_write<16384>, grid, dim3(FMT_WAVE_LINES), 0, stream, *a, st_blocks);
  else
    hipLaunchKernelGGL(k_format_write<24576>, grid, dim3(FMT_WAVE_LINES), 0, stream, *a, st_blocks);
}

}  // extern "C"
