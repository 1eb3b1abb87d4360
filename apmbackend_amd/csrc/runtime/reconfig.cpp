// Live reconfiguration of a running engine (config hot reload).
//
// Reference behaviour, per stage, on every config file change (util_methods.js:297-348 watcher):
//   * z-score: `updateAllServiceSettings` re-applies the defaults + per-service overrides to every
//     series, creating the entry of a new LAG (its history starts empty), and
//     `removeStaleLagData` deletes the lists of LAGs no longer configured
//     (stream_calc_z_score.js:152-193, 362-382);
//   * alerts: every gate is read from the config for each fs entry -- window, threshold, hard
//     min ms / tpm, hard max (and its per-service override), alertOnBothOnly, suppressed LAGs and
//     services, the cooldown (stream_process_alerts.js:335-471).  The leaky counters are keyed by
//     LAG value and survive a LAG's removal;
//   * stats: consumeQueue toggles consumption (the service pauses ingest for it).
//
// MI355X engine: a reload is *staged* on the ingest thread and applied by the stats thread at the
// start of the batch it is tagged with, so it never drains the pipeline.  With lock-step ranks the
// tag is agreed node-wide: every rank reports the newest generation it has staged in the
// per-batch clock all-reduce (as -gen under MAX, i.e. the minimum), and a generation every rank
// holds is tagged with the same batch on every rank -- all ranks switch at one batch boundary, so
// the node-wide alert decisions and the fleet exchange (whose message size depends on the LAG
// count) stay identical across ranks.
#include <algorithm>
#include <chrono>
#include <cstring>
#include <stdexcept>

#include "engine.h"

namespace apm {

namespace {
double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

void check_window(int window, int buffer, int interval_len) {
  // (the ring holds any window the HBM does: window + buffer + 1 slots of maxSeries cells each)
  if (window < 1 || buffer < 0 || interval_len < 1 || (int64_t)window + buffer > (1 << 20))
    throw std::runtime_error("stats window: windowSizeInIntervals >= 1, bufferSizeInIntervals >= 0, "
                             "intervalLengthInSeconds >= 1 (got " + std::to_string(window) + " / " +
                             std::to_string(buffer) + " / " + std::to_string(interval_len) + ")");
}

void Engine::stage_reconfig(const ReconfigSpec& spec) {
  if (spec.n_lags < 1 || spec.n_lags > MAX_LAGS)
    throw std::runtime_error("reconfigure: 1.." + std::to_string(MAX_LAGS) + " LAG settings");
  check_window(spec.window, spec.buffer, spec.interval_len);
  for (int l = 0; l < spec.n_lags; ++l)
    if (spec.lags[l] < 1) throw std::runtime_error("reconfigure: LAG must be >= 1");
  std::lock_guard<std::mutex> g(rc_mu_);
  if (lockstep_) {
    rc_staged_.push_back(spec);  // tagged once every rank has it (lockstep_sync)
  } else {
    rc_tagged_.push_back({batch_no_, spec});
  }
}

uint64_t Engine::reconfig_staged_gen() {
  std::lock_guard<std::mutex> g(rc_mu_);
  uint64_t gmax = 0;
  for (const auto& s : rc_staged_) gmax = std::max(gmax, s.gen);
  return gmax;
}

// Ingest thread, inside the clock exchange of batch `batch_no_`: `node_min` is the smallest
// newest-staged generation over the ranks.
void Engine::reconfig_agree(uint64_t node_min) {
  std::lock_guard<std::mutex> g(rc_mu_);
  while (!rc_staged_.empty() && rc_staged_.front().gen <= node_min) {
    node_cool_ms_ = rc_staged_.front().cooldown_ms;  // the node-wide decisions switch here too
    rc_tagged_.push_back({batch_no_, rc_staged_.front()});
    rc_staged_.pop_front();
  }
}

// Stats thread (or flush with the stats thread idle): apply every reload tagged <= `upto`.
void Engine::apply_reconfig_pending(uint64_t upto) {
  std::vector<ReconfigSpec> due;
  {
    std::lock_guard<std::mutex> g(rc_mu_);
    while (!rc_tagged_.empty() && rc_tagged_.front().first <= upto) {
      due.push_back(std::move(rc_tagged_.front().second));
      rc_tagged_.pop_front();
    }
  }
  for (const ReconfigSpec& r : due) apply_reconfig(r);
}

void Engine::apply_reconfig(const ReconfigSpec& r) {
  const double t0 = now_ms();
  // the rollover lane decides alerts with these settings and reads the lag table: let it finish
  finish_rollover();
  bool lag_change = r.n_lags != cfg_.n_lags;
  for (int l = 0; l < r.n_lags && !lag_change; ++l) lag_change = r.lags[l] != cfg_.lags[l];
  if (lag_change) {
    checkpoint_wait();  // a streamed snapshot's writer may still read the rings about to be freed
    // kernels of the previous rollover (formatting on the output stream, K10/K11 and the fleet
    // pack on the stats stream) still read the old per-LAG arrays.  Only those two streams: a
    // device-wide sync would also wait for the collective stream, whose lock-step all-reduce may
    // be waiting for a peer -- tying this thread to peer progress (fleet_pack_locked avoids it)
    HIP_OK(hipStreamSynchronize(stream_));
    HIP_OK(hipStreamSynchronize(out_stream_));
    const int32_t S = cfg_.max_series;
    LagState nl[MAX_LAGS] = {};
    bool kept[MAX_LAGS] = {};
    for (int i = 0; i < r.n_lags; ++i) {
      int j = -1;
      for (int o = 0; o < cfg_.n_lags; ++o)
        if (!kept[o] && cfg_.lags[o] == r.lags[i]) { j = o; break; }
      if (j >= 0) {  // a kept LAG keeps its history, moments and counters
        nl[i] = lag_[j];
        kept[j] = true;
        continue;
      }
      // a new LAG: empty history (len 0; the ring head is the shared rollover index mod LAG)
      LagState& L = nl[i];
      L.ring = dmalloc((size_t)NSTAT * r.lags[i] * S * cfg_.ring_bytes);
      L.len = (int32_t*)dmalloc((size_t)S * 4);
      L.sum = (double*)dmalloc((size_t)NSTAT * S * 8);
      L.comp = (double*)dmalloc((size_t)NSTAT * S * 8);
      L.sumsq = (double*)dmalloc((size_t)NSTAT * S * 8);
      L.sqcomp = (double*)dmalloc((size_t)NSTAT * S * 8);
      L.cnt = (int32_t*)dmalloc((size_t)NSTAT * S * 4);
      L.thr = (double*)dmalloc((size_t)S * 8);
      L.infl = (double*)dmalloc((size_t)S * 8);
      L.out = (ZOut*)dmalloc((size_t)S * sizeof(ZOut));
      // the alerts stage's leaky counters are keyed by LAG value and never deleted: a LAG that
      // comes back resumes the counters it had when it was removed
      auto st = counter_stash_.find(r.lags[i]);
      if (st != counter_stash_.end()) {
        L.counter = st->second;
        counter_stash_.erase(st);
      } else {
        L.counter = (int32_t*)dmalloc((size_t)S * 4);
      }
    }
    for (int o = 0; o < cfg_.n_lags; ++o) {
      if (kept[o]) continue;
      LagState& L = lag_[o];
      for (void* p : {L.ring, (void*)L.len, (void*)L.sum, (void*)L.comp, (void*)L.sumsq, (void*)L.sqcomp,
                      (void*)L.cnt, (void*)L.thr, (void*)L.infl, (void*)L.out})
        dfree(p);
      if (counter_stash_.count(cfg_.lags[o])) dfree(counter_stash_[cfg_.lags[o]]);
      counter_stash_[cfg_.lags[o]] = L.counter;
    }
    for (int l = 0; l < MAX_LAGS; ++l) lag_[l] = l < r.n_lags ? nl[l] : LagState{};
    cfg_.n_lags = r.n_lags;
    for (int l = 0; l < MAX_LAGS; ++l) cfg_.lags[l] = l < r.n_lags ? r.lags[l] : 0;
    const double* sp[MAX_LAGS] = {};
    const double* cp[MAX_LAGS] = {};
    const int32_t* np[MAX_LAGS] = {};
    for (int l = 0; l < cfg_.n_lags; ++l) { sp[l] = lag_[l].sum; cp[l] = lag_[l].comp; np[l] = lag_[l].cnt; }
    HIP_OK(hipMemcpy(d_lag_sum_ptrs_, sp, sizeof(sp), hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_lag_comp_ptrs_, cp, sizeof(cp), hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_lag_cnt_ptrs_, np, sizeof(np), hipMemcpyHostToDevice));
    ck_all_dirty_ = true;  // an incremental chain cannot span two LAG sets: the next one is a base
    ++lag_set_changes_;
  }
  for (int l = 0; l < MAX_LAGS; ++l) {
    cfg_.thr[l] = l < r.n_lags ? r.thr[l] : 0.0;
    cfg_.infl[l] = l < r.n_lags ? r.infl[l] : 0.0;
    cfg_.lag_suppressed[l] = l < r.n_lags ? r.lag_suppressed[l] : 0;
  }
  // stats (stream_calc_stats.js:228-261 re-reads them on every change; used from the next
  // rollover on).  removeOldBuckets keeps NUM_KEEP_INTERVALS = window + buffer buckets: a larger
  // window fills in as new buckets arrive (older ones were deleted at the last rollover, here as
  // there); a NaN-poisoned series stays poisoned until its bucket leaves the new keep range.
  if (r.window != cfg_.window || r.buffer != cfg_.buffer) {
    const int32_t dk = (r.window + r.buffer) - (cfg_.window + cfg_.buffer);
    if (dk != 0 && n_series_ > 0) {
      HIP_OK(hipStreamSynchronize(stream_));
      std::vector<int32_t> nu((size_t)n_series_);
      HIP_OK(hipMemcpy(nu.data(), d_nan_until_, nu.size() * 4, hipMemcpyDeviceToHost));
      for (auto& v : nu) v += dk;  // (never poisoned: 0x80808080, far below any bucket either way)
      HIP_OK(hipMemcpy(d_nan_until_, nu.data(), nu.size() * 4, hipMemcpyHostToDevice));
    }
    // a longer window than the ring holds: grow it first (live buckets keep their samples)
    grow_ring(ring_slots_for(r.window, r.buffer));
    cfg_.window = r.window;
    cfg_.buffer = r.buffer;
    ++window_changes_;
  }
  cfg_.interval_len = r.interval_len;
  cfg_.alert_window = r.alert_window;
  cfg_.alert_threshold = r.alert_threshold;
  cfg_.hard_min_ms = r.hard_min_ms;
  cfg_.hard_min_tpm = r.hard_min_tpm;
  cfg_.hard_max_ms = r.hard_max_ms;
  cfg_.both_only = r.both_only;
  cfg_.cooldown_ms = r.cooldown_ms;
  overrides_ = r.overrides;
  // updateAllServiceSettings: defaults (Q4 aliasing restarts from the new defaults) + overrides
  // for every series the z-score stage has seen, in its emission order
  for (int l = 0; l < MAX_LAGS; ++l) { alias_thr_[l] = cfg_.thr[l]; alias_infl_[l] = cfg_.infl[l]; }
  {
    std::lock_guard<std::mutex> sg(series_mu_);
    std::vector<int32_t> order(n_series_);
    for (int32_t i = 0; i < n_series_; ++i) order[i] = i;
    std::sort(order.begin(), order.end(),
              [&](int32_t a, int32_t b) { return series_[a].emit_key < series_[b].emit_key; });
    for (int32_t s : order) if (zscore_seen_[s]) apply_series_settings(s);
  }
  upload_series_tables(0);  // stream-ordered before the next rollover's kernels
  // (K11's cooldown pre-filter keeps its per-series alert times: only the window length changed)
  rc_applied_gen_.store(r.gen);
  ++reconfigs_applied_;
  trace_event("reconfigure", t0, now_ms(), 1);
}

}  // namespace apm
