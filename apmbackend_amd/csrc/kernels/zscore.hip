// K10 smoothed z-score update and K11 alert decision.
//
// Reference behaviour: stream_calc_z_score.js processZScoreStats (:66-104) / processData
// (:195-311) with util_methods.js average / standardDeviation (:10-50, quirk Q1: sigma is
// sqrt(mean)); stream_process_alerts.js processFSEntry (:348-471) (hard max, signal gates,
// alertOnBothOnly, leaky counter Q6).
//
// Layout (MI355X): the history list of every (series, lag, stat) is a ring in HBM laid out
// ring[lag][stat][pos][series]: every active series pushes exactly one value per rollover, so
// all series of a lag share the write position (head = rollover index mod LAG) and a warp of
// consecutive series reads/writes one contiguous row -> fully coalesced.  The mean is kept as a
// compensated (Neumaier) fp64 running sum + valid count, updated O(1) per rollover.  Drift is
// bounded by a staggered resync: every rollover one contiguous range of R = ceil(S/K) series
// gets its window re-summed from the ring by k_zscore_resync (a [64 series x P partitions] tile
// grid: a wave covers 64 consecutive series of one ring row -> coalesced 512 B reads, and the
// partitions spread the L-long walk over P waves), and k_zscore folds the P partials in a fixed
// order.  In "exact" mode each thread re-sums its window sequentially (the JS summation order),
// which is bit-identical to the reference.
//
// Ring dtype: fp64 (parity), fp32, or bf16 (capacity mode, BASELINE config 2): values are
// rounded on store and every moment is taken over the value *as stored*.
#include "kernel_api.h"

namespace apm {


template <typename T> __device__ __forceinline__ double ld(const T* p) { return (double)*p; }
template <typename T> __device__ __forceinline__ void st(T* p, double v) { *p = (T)v; }
// bf16 ring: raw uint16 storage, round-to-nearest-even from fp32, NaN preserved
template <> __device__ __forceinline__ double ld<uint16_t>(const uint16_t* p) {
  return (double)__uint_as_float((uint32_t)*p << 16);
}
template <> __device__ __forceinline__ void st<uint16_t>(uint16_t* p, double v) {
  const float f = (float)v;
  uint32_t u = __float_as_uint(f);
  if (f != f) { *p = 0x7FC0; return; }
  u += 0x7FFFu + ((u >> 16) & 1u);
  *p = (uint16_t)(u >> 16);
}

__device__ __forceinline__ void neumaier(double& s, double& c, double x) {
  const double t = s + x;
  if (fabs(s) >= fabs(x)) c += (s - t) + x; else c += (x - t) + s;
  s = t;
}

__device__ __forceinline__ bool valid(double v) { return v == v; }

// Partial window sums for the resync range [rs_lo, rs_lo + rs_n): block = 64 series x 4
// partitions, grid = (ceil(rs_n/64), P/4, NSTAT).
template <typename T>
__global__ __launch_bounds__(256) void k_zscore_resync(ZArgs a) {
  const int j = blockIdx.x * 64 + threadIdx.x;
  const int p = blockIdx.y * 4 + threadIdx.y;
  const int k = blockIdx.z;
  if (j >= a.rs_n || p >= a.rs_parts) return;
  const int s = a.rs_lo + j;
  const int L = a.lag, S = a.S;
  double sum = 0, comp = 0, sq = 0, sqc = 0;
  int c = 0;
  if (s < a.n_series) {
    const int n = a.len[s];
    const int per = (L + a.rs_parts - 1) / a.rs_parts;
    const int i0 = p * per, i1 = min(n, i0 + per);
    const int oldest = (a.head - n + L) % L;
    const T* col = reinterpret_cast<const T*>(a.ring) + (size_t)k * L * S + s;
    int pos = oldest + i0;
    if (pos >= L) pos -= L;
    int i = i0;
    // RS_BATCH ring rows loaded before the first is summed: that many 512 B row loads in flight
    // per wave instead of one behind each compensated add (same order, same result)
    constexpr int RS_BATCH = 8;
    for (; i + RS_BATCH <= i1; i += RS_BATCH) {
      double v[RS_BATCH];
#pragma unroll
      for (int u = 0; u < RS_BATCH; ++u) {
        v[u] = ld(col + (size_t)pos * S);
        if (++pos == L) pos = 0;
      }
#pragma unroll
      for (int u = 0; u < RS_BATCH; ++u)
        if (valid(v[u])) { neumaier(sum, comp, v[u]); neumaier(sq, sqc, v[u] * v[u]); ++c; }
    }
    for (; i < i1; ++i) {
      const double v = ld(col + (size_t)pos * S);
      if (valid(v)) { neumaier(sum, comp, v); neumaier(sq, sqc, v * v); ++c; }
      if (++pos == L) pos = 0;
    }
  }
  const size_t o = ((size_t)k * a.rs_parts + p) * a.rs_n + j;
  a.rs_part[o * 4 + 0] = sum; a.rs_part[o * 4 + 1] = comp;
  a.rs_part[o * 4 + 2] = sq; a.rs_part[o * 4 + 3] = sqc;
  a.rs_cnt[o] = c;
}

// The same partial sums on the matrix cores.  A wave owns 16 consecutive series x one partition
// and walks the partition's window positions two at a time; each step is one
// v_mfma_f64_16x16x4f64 with
//   A[i][k] (16 series x 4):  k=0: v(i, pos), k=1: v(i, pos+1), k=2: v(i, pos)^2, k=3: v(i, pos+1)^2
//   B[k][j] (4 x 16, const):  column 0 = (1,1,0,0), column 1 = (0,0,1,1), other columns 0
// so C[i][0] accumulates the window sum and C[i][1] the sum of squares of series i: a masked
// ones-matrix tile reduction over the [LAG x series] ring slab (values outside a series' window
// and NaN entries enter as 0 and are not counted).  The accumulation is plain fp64 in the matrix
// core (no Neumaier term: partial comp = 0), which is what rolling mode's periodic resync needs.
// Grid: (ceil(rs_n / 16), ceil(P / 4), NSTAT), 4 waves per block (one partition each).
typedef double apm_f64x4z __attribute__((ext_vector_type(4)));

template <typename T>
__global__ __launch_bounds__(256) void k_zscore_resync_mfma(ZArgs a) {
  __shared__ double g[4][16][3];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int i16 = lane & 15, kk = lane >> 4;       // A operand: series i16, column kk
  const int j = blockIdx.x * 16 + i16;
  const int p = blockIdx.y * 4 + wave;
  const int k = blockIdx.z;
  const int L = a.lag, S = a.S;
  const bool part_ok = p < a.rs_parts;             // uniform per wave
  const int s = a.rs_lo + j;
  const bool ser_ok = j < a.rs_n && s < a.n_series;
  const int n = ser_ok ? a.len[s] : 0;
  const int per = (L + a.rs_parts - 1) / a.rs_parts;
  const int i0 = p * per;
  const int oldest = (a.head - n + L) % L;
  const T* col = reinterpret_cast<const T*>(a.ring) + (size_t)k * L * S + (ser_ok ? s : 0);
  const int which = kk & 1;                         // pos or pos + 1
  const bool square = kk >= 2;
  const double bval = (i16 == 0 && kk < 2) || (i16 == 1 && kk >= 2) ? 1.0 : 0.0;  // B[kk][i16]
  apm_f64x4z acc = {0.0, 0.0, 0.0, 0.0};
  int cnt = 0;
  if (part_ok) {
    for (int i = i0; i < i0 + per && i < L; i += 2) {  // uniform bounds across the wave
      const int wi = i + which;
      double v = 0.0;
      if (ser_ok && wi < i0 + per && wi < n) {
        int pos = oldest + wi;
        if (pos >= L) pos -= L;
        const double x = ld(col + (size_t)pos * S);
        if (valid(x)) {
          v = square ? x * x : x;
          if (!square) ++cnt;
        }
      }
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(v, bval, acc, 0, 0, 0);
    }
  }
  // counts: lanes kk = 0, 1 of series i16 (lanes i16 and i16 + 16)
  cnt += __shfl_down(cnt, 16, 64);
  // D[row][col]: lane l, accumulator r holds row 4 r + l / 16, column l % 16
  if (i16 < 2)
#pragma unroll
    for (int r = 0; r < 4; ++r) g[wave][4 * r + kk][i16] = acc[r];
  if (kk == 0) g[wave][i16][2] = (double)cnt;
  __syncthreads();
  if (part_ok && kk == 0 && j < a.rs_n) {
    const size_t o = ((size_t)k * a.rs_parts + p) * a.rs_n + j;
    a.rs_part[o * 4 + 0] = g[wave][i16][0];
    a.rs_part[o * 4 + 1] = 0.0;
    a.rs_part[o * 4 + 2] = g[wave][i16][1];
    a.rs_part[o * 4 + 3] = 0.0;
    a.rs_cnt[o] = (int)g[wave][i16][2];
  }
}

// One thread per (series, stat): grid (ceil(n/256), NSTAT).  The three stats of a series are
// independent recurrences, and a thread per series left ~1.2 waves per SIMD at 80k series --
// too few to hide the HBM latency of its five moment loads + ring row per stat (73 us per LAG
// at 80k series before the split).  k_zscore_commit then publishes `valid` and bumps the list
// length (every stat thread must read the old length first).
template <typename T>
__global__ __launch_bounds__(256) void k_zscore(ZArgs a) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  const int k = blockIdx.y;
  if (s >= a.n_series) return;
  const WinStat w = a.win[s];
  if (!w.active) return;
  ZOut* const op = a.out + s;
  const int L = a.lag;
  const int S = a.S;
  const int n = a.len[s];
  const double T_ = a.thr[s];
  const double I_ = a.infl[s];
  T* ring = reinterpret_cast<T*>(a.ring);
  const int head = a.head;
  const int last_pos = head == 0 ? L - 1 : head - 1;
  const int oldest = (head - n + L) % L;
  const bool exact = a.exact != 0;
  const bool resync = !exact && s >= a.rs_lo && s < a.rs_lo + a.rs_n;
  {
    T* col = ring + (size_t)k * L * S + s;  // element pos at col[pos * S]
    double sum = a.sum[k * S + s], comp = a.comp[k * S + s];
    int c = a.cnt[k * S + s];
    double sq = a.sumsq[k * S + s], sqc = a.sqcomp[k * S + s];
    if (resync) {
      sum = 0; comp = 0; sq = 0; sqc = 0; c = 0;
      const int j = s - a.rs_lo;
      for (int p = 0; p < a.rs_parts; ++p) {  // fixed order -> deterministic
        const size_t o = ((size_t)k * a.rs_parts + p) * a.rs_n + j;
        neumaier(sum, comp, a.rs_part[o * 4 + 0]); comp += a.rs_part[o * 4 + 1];
        neumaier(sq, sqc, a.rs_part[o * 4 + 2]); sqc += a.rs_part[o * 4 + 3];
        c += a.rs_cnt[o];
      }
    }
    if (exact && n > 0) {
      // sequential left-to-right sum from 0, as Array.prototype.average does
      double es = 0.0, eq = 0.0;
      int ec = 0;
      for (int i = 0; i < n; ++i) {
        int pos = oldest + i;
        if (pos >= L) pos -= L;
        const double v = ld(col + (size_t)pos * S);
        if (valid(v)) { es = es + v; eq += v * v; ++ec; }
      }
      sum = es; comp = 0.0; c = ec; sq = eq; sqc = 0.0;
    }
    const double x = k == 0 ? w.avg : (k == 1 ? w.p75 : w.p95);
    double stored = x;
    double mean = apm_nan(), lb = apm_nan(), ub = apm_nan();
    int sig = 0;
    if (n >= L) {
      bool mean_ok = c > 0;
      if (mean_ok) mean = exact ? sum / (double)c : (sum + comp) / (double)c;
      double sd = apm_nan();
      bool sd_ok = false;
      if (mean_ok) {
        if (!a.sigma_stddev) {
          if (mean > 0) { sd = sqrt(mean); sd_ok = true; }           // mean==0 -> undefined
        } else {
          const double m2 = (sq + sqc) / (double)c - mean * mean;
          if (m2 > 0) { sd = sqrt(m2); sd_ok = true; }
        }
      }
      if (mean_ok && sd_ok) {
        lb = mean - T_ * sd;
        ub = mean + T_ * sd;
        if (valid(x) && fabs(x - mean) > T_ * sd) {
          sig = x > mean ? 1 : -1;
          const double last = ld(col + (size_t)last_pos * S);
          if (valid(last)) stored = I_ * x + (1.0 - I_) * last;
        }
      }
    }
    // evict the oldest value (it occupies the head slot once the list is full), then push
    T* slot = col + (size_t)head * S;
    if (n >= L) {
      const double old = ld(slot);
      if (valid(old)) { neumaier(sum, comp, -old); neumaier(sq, sqc, -old * old); --c; }
    }
    st(slot, stored);
    const double sv = ld(slot);  // value as stored (ring dtype may round)
    if (valid(sv)) { neumaier(sum, comp, sv); neumaier(sq, sqc, sv * sv); ++c; }
    a.sum[k * S + s] = sum; a.comp[k * S + s] = comp; a.cnt[k * S + s] = c;
    a.sumsq[k * S + s] = sq; a.sqcomp[k * S + s] = sqc;
    op->mean[k] = mean; op->lb[k] = lb; op->ub[k] = ub; op->sig[k] = (int8_t)sig;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void k_zscore_commit(ZArgs a) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= a.n_series) return;
  const bool act = a.win[s].active != 0;
  a.out[s].valid = act ? 1 : 0;
  if (act) {
    const int n = a.len[s];
    a.len[s] = n < a.lag ? n + 1 : a.lag;
  }
}

// Warm start: fill a lag's ring with a synthetic pre-history (per-series baseline * jitter)
// so that a benchmark exercises fully populated 1 h / 1 day windows from the first interval.
template <typename T>
__global__ void k_zscore_warm(ZArgs a, int fill, uint64_t seed, const WinStat* base) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= a.n_series) return;
  const int L = a.lag, S = a.S;
  T* ring = reinterpret_cast<T*>(a.ring);
  const int n = min(fill, L);
  const int oldest = (a.head - n + L) % L;
  for (int k = 0; k < NSTAT; ++k) {
    const double b = k == 0 ? base[s].avg : (k == 1 ? base[s].p75 : base[s].p95);
    double es = 0.0, eq = 0.0;
    int ec = 0;
    uint64_t x = seed ^ (0x9E3779B97F4A7C15ULL * (uint64_t)(s * 3 + k + 1));
    for (int i = 0; i < n; ++i) {
      x ^= x << 13; x ^= x >> 7; x ^= x << 17;
      const double j = 0.9 + 0.2 * (double)(x >> 11) * (1.0 / 9007199254740992.0);
      double v = b == b ? js_round_fixed(b * j, 1) : apm_nan();
      int pos = oldest + i;
      if (pos >= L) pos -= L;
      T* p = ring + (size_t)k * L * S + (size_t)pos * S + s;
      st(p, v);
      v = ld(p);
      if (valid(v)) { es = es + v; eq += v * v; ++ec; }
    }
    a.sum[k * S + s] = es; a.comp[k * S + s] = 0; a.cnt[k * S + s] = ec;
    a.sumsq[k * S + s] = eq; a.sqcomp[k * S + s] = 0;
  }
  a.len[s] = n;
}

// --------------------------------------------------------------------------------- K11

__global__ __launch_bounds__(256) void k_alert_eval(AlertArgs a) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= a.n_series) return;
  const WinStat w = a.win[s];
  if (!w.active) return;
  const ZOut z = a.z[s];
  int cnt = a.counter[s];
  bool inc = false, trigger = false;
  uint32_t causes = 0;
  const bool windowed = a.window > 1 && a.threshold > 1;
  auto fire = [&](int cause) {
    if (!inc) { if (cnt <= a.window) ++cnt; inc = true; }
    if (windowed) {
      if (cnt >= a.threshold) { trigger = true; causes |= 1u << cause; }
    } else {
      trigger = true; causes |= 1u << cause;
    }
  };
  if (!a.lag_suppressed && !a.suppressed[s]) {
    const double hm = a.hard_max[s];
    if (w.avg == w.avg && w.avg > hm) fire(0);
    if (w.p75 == w.p75 && w.p75 > hm) fire(1);
    int both = 0;
    const bool tpm_ok = w.tpm == w.tpm && w.tpm > a.hard_min_tpm;
    if (z.sig[0] > 0 && w.avg == w.avg && w.avg > a.hard_min_ms && tpm_ok) {
      if (!a.both_only) fire(2); else ++both;
    }
    if (z.sig[1] > 0 && w.p75 == w.p75 && w.p75 > a.hard_min_ms && tpm_ok) {
      if (!a.both_only) fire(3); else ++both;
    }
    if (a.both_only && both >= 2) fire(4);
  }
  if (!inc && cnt > 0) --cnt;
  if (cnt < 0) cnt = 0;
  a.counter[s] = cnt;
  if (trigger && a.cool_t) {
    const double ct = a.cool_t[s];
    if (ct == ct && !((a.now - ct) / 1000.0 > a.cool_s)) trigger = false;  // in cooldown (host rule)
  }
  if (trigger) {
    const int j = atomicAdd(a.n_out, 1);
    if (j < a.max_out) {
      AlertRec r;
      r.series = s;
      r.lag_idx = a.lag_idx;
      r.causes = causes;
      r.pad = 0;
      r.order = a.emit_key[s] * (uint64_t)a.n_lags + (uint64_t)a.lag_idx;
      a.out[j] = r;
    }
  }
}

__global__ void k_scatter_f64(double* __restrict__ dst, const int32_t* __restrict__ idx,
                              const double* __restrict__ val, int32_t n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[idx[i]] = val[i];
}

}  // namespace apm

namespace apm {
template <typename T>
void launch_zscore(ZArgs* a, hipStream_t stream) {
  if (!a->exact && a->rs_n > 0) {
    if (a->rs_mfma) {
      const dim3 g((a->rs_n + 15) / 16, (a->rs_parts + 3) / 4, NSTAT);
      hipLaunchKernelGGL(k_zscore_resync_mfma<T>, g, dim3(256), 0, stream, *a);
    } else {
      const dim3 g((a->rs_n + 63) / 64, (a->rs_parts + 3) / 4, NSTAT), b(64, 4);
      hipLaunchKernelGGL(k_zscore_resync<T>, g, b, 0, stream, *a);
    }
  }
  hipLaunchKernelGGL(k_zscore<T>, dim3((a->n_series + 255) / 256, NSTAT), dim3(256), 0, stream, *a);
  hipLaunchKernelGGL(k_zscore_commit<T>, dim3((a->n_series + 255) / 256), dim3(256), 0, stream, *a);
}

}  // namespace apm

extern "C" {
using namespace apm;

void apm_scatter_f64(double* dst, const int32_t* idx, const double* val, int32_t n, hipStream_t stream) {
  if (n > 0) hipLaunchKernelGGL(k_scatter_f64, dim3((n + 255) / 256), dim3(256), 0, stream, dst, idx, val, n);
}

void apm_zscore(ZArgs* a, int dtype_bytes, hipStream_t stream) {
  if (a->n_series <= 0) return;
  if (dtype_bytes == 8) launch_zscore<double>(a, stream);
  else if (dtype_bytes == 4) launch_zscore<float>(a, stream);
  else launch_zscore<uint16_t>(a, stream);
}

void apm_zscore_warm(ZArgs* a, int dtype_bytes, int fill, uint64_t seed, const WinStat* base, hipStream_t stream) {
  if (a->n_series <= 0) return;
  const dim3 g((a->n_series + 255) / 256), b(256);
  if (dtype_bytes == 8) hipLaunchKernelGGL(k_zscore_warm<double>, g, b, 0, stream, *a, fill, seed, base);
  else if (dtype_bytes == 4) hipLaunchKernelGGL(k_zscore_warm<float>, g, b, 0, stream, *a, fill, seed, base);
  else hipLaunchKernelGGL(k_zscore_warm<uint16_t>, g, b, 0, stream, *a, fill, seed, base);
}

struct AlertGather {
  const AlertRec* alerts;
  const int32_t* n_dev;  // the K11 candidate count (device)
  const WinStat* win;
  const ZOut* z[MAX_LAGS];
  AlertRec* alerts_out;  // host-mapped pinned buffers: the records land in host memory directly
  WinStat* win_out;
  ZOut* z_out;
  int32_t* n_out;
  int32_t max_n;
  int32_t rows;
};

// One pass after K11: the candidate count, the candidates and (for al rows) their window stats and
// z-score rows are written straight into pinned host memory, so the stats thread learns the
// count, and reads the rows, by waiting on one event instead of a stream drain + three D2H copies.
__global__ void k_alert_gather(AlertGather a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int raw = *a.n_dev;
  const int n = min(raw, a.max_n);
  if (i == 0) { a.n_out[0] = n; a.n_out[1] = raw; }  // (raw > n: candidates dropped, counted)
  if (i >= n) return;
  const AlertRec r = a.alerts[i];
  a.alerts_out[i] = r;
  if (!a.rows) return;
  a.win_out[i] = a.win[r.series];
  a.z_out[i] = a.z[r.lag_idx][r.series];
}

void apm_alert_gather(const AlertRec* alerts, const int32_t* n_dev, int32_t max_n, const WinStat* win,
                      const ZOut* const* z_by_lag, int32_t n_lags, int32_t rows, AlertRec* alerts_out, WinStat* win_out,
                      ZOut* z_out, int32_t* n_out, hipStream_t stream) {
  if (max_n <= 0) return;
  AlertGather a{};
  a.alerts = alerts; a.n_dev = n_dev; a.win = win; a.alerts_out = alerts_out; a.win_out = win_out; a.z_out = z_out;
  a.n_out = n_out; a.max_n = max_n; a.rows = rows;
  for (int l = 0; l < n_lags && l < MAX_LAGS; ++l) a.z[l] = z_by_lag[l];
  hipLaunchKernelGGL(k_alert_gather, dim3((max_n + 255) / 256), dim3(256), 0, stream, a);
}

void apm_alert_eval(AlertArgs* a, hipStream_t stream) {
  if (a->n_series <= 0) return;
  hipLaunchKernelGGL(k_alert_eval, dim3((a->n_series + 255) / 256), dim3(256), 0, stream, *a);
}

}  // extern "C"
