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
// compensated (Neumaier) fp64 running sum + valid count, updated O(1) per rollover; a staggered
// exact sequential recompute (the JS summation order) resynchronises every K rollovers.  In
// "exact" mode the sequential sum is recomputed every time, which is bit-identical to JS.
#include "kernel_api.h"

namespace apm {


template <typename T> __device__ __forceinline__ double ld(const T* p) { return (double)*p; }
template <typename T> __device__ __forceinline__ void st(T* p, double v) { *p = (T)v; }

__device__ __forceinline__ void neumaier(double& s, double& c, double x) {
  const double t = s + x;
  if (fabs(s) >= fabs(x)) c += (s - t) + x; else c += (x - t) + s;
  s = t;
}

__device__ __forceinline__ bool valid(double v) { return v == v; }

template <typename T>
__global__ __launch_bounds__(256) void k_zscore(ZArgs a) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= a.n_series) return;
  const WinStat w = a.win[s];
  ZOut o;
  o.valid = 0;
  if (!w.active) { a.out[s] = o; return; }
  o.valid = 1;
  const int L = a.lag;
  const int S = a.S;
  const int n = a.len[s];
  const double T_ = a.thr[s];
  const double I_ = a.infl[s];
  T* ring = reinterpret_cast<T*>(a.ring);
  const int head = a.head;
  const int last_pos = head == 0 ? L - 1 : head - 1;
  const int oldest = (head - n + L) % L;
  const bool resync = a.exact || (a.resync_k > 0 && ((a.rollover_idx + s) % a.resync_k) == 0);
  const double xs[NSTAT] = {w.avg, w.p75, w.p95};
#pragma unroll
  for (int k = 0; k < NSTAT; ++k) {
    T* col = ring + (size_t)k * L * S + s;  // element pos at col[pos * S]
    double sum = a.sum[k * S + s], comp = a.comp[k * S + s];
    int c = a.cnt[k * S + s];
    double sq = a.sumsq[k * S + s], sqc = a.sqcomp[k * S + s];
    if (resync && n > 0) {
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
    const double x = xs[k];
    double stored = x;
    double mean = apm_nan(), lb = apm_nan(), ub = apm_nan();
    int sig = 0;
    if (n >= L) {
      bool mean_ok = c > 0;
      if (mean_ok) mean = resync ? sum / (double)c : (sum + comp) / (double)c;
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
    o.mean[k] = mean; o.lb[k] = lb; o.ub[k] = ub; o.sig[k] = (int8_t)sig;
  }
  a.len[s] = n < L ? n + 1 : L;
  a.out[s] = o;
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

}  // namespace apm

extern "C" {
using namespace apm;

void apm_zscore(ZArgs* a, int dtype_bytes, hipStream_t stream) {
  if (a->n_series <= 0) return;
  const dim3 g((a->n_series + 255) / 256), b(256);
  if (dtype_bytes == 8) hipLaunchKernelGGL(k_zscore<double>, g, b, 0, stream, *a);
  else hipLaunchKernelGGL(k_zscore<float>, g, b, 0, stream, *a);
}

void apm_zscore_warm(ZArgs* a, int dtype_bytes, int fill, uint64_t seed, const WinStat* base, hipStream_t stream) {
  if (a->n_series <= 0) return;
  const dim3 g((a->n_series + 255) / 256), b(256);
  if (dtype_bytes == 8) hipLaunchKernelGGL(k_zscore_warm<double>, g, b, 0, stream, *a, fill, seed, base);
  else hipLaunchKernelGGL(k_zscore_warm<float>, g, b, 0, stream, *a, fill, seed, base);
}

void apm_alert_eval(AlertArgs* a, hipStream_t stream) {
  if (a->n_series <= 0) return;
  hipLaunchKernelGGL(k_alert_eval, dim3((a->n_series + 255) / 256), dim3(256), 0, stream, *a);
}

}  // extern "C"
