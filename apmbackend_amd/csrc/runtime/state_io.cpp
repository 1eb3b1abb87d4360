// Structured state access for the reference resume-file importer/exporter
// (runtime/resume_compat.py).  The reference persists its stages as JSON:
//   calc_stats  servers -> services -> buckets {label: [elapsed...]}, latestBucket, minHeap
//   z-score     servers -> services -> lags {LAG: {THRESHOLD, INFLUENCE, avgList, per75List,
//               per95List}}
//   alerts      alerts {service: last AlertEntry} (+ recentAlertCounts, reset on load)
// These entry points read / write exactly that information from / into the device-resident
// engine state: series table, live bucket cells, z-score rings (chronological lists), pending
// release pool (tx lines), alert cooldowns and leaky counters.  Imports target a fresh engine
// (no batches processed yet), mirroring a reference stage starting from its resume file.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>

#include "engine.h"

namespace apm {

namespace {

void neumaier(double& s, double& c, double x) {
  const double t = s + x;
  if (std::fabs(s) >= std::fabs(x)) c += (s - t) + x; else c += (x - t) + s;
  s = t;
}

double ring_load(const void* p, int rb) {
  if (rb == 8) return *(const double*)p;
  if (rb == 4) return (double)*(const float*)p;
  uint32_t u = (uint32_t)(*(const uint16_t*)p) << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return (double)f;
}

void ring_store(void* p, int rb, double v) {
  if (rb == 8) { *(double*)p = v; return; }
  if (rb == 4) { *(float*)p = (float)v; return; }
  const float f = (float)v;
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if (f != f) { *(uint16_t*)p = 0x7FC0; return; }
  u += 0x7FFFu + ((u >> 16) & 1u);
  *(uint16_t*)p = (uint16_t)(u >> 16);
}

}  // namespace

void Engine::require_fresh(const char* what) {
  if (batch_no_ != 0 || rollover_idx_ != 0)
    throw std::runtime_error(std::string(what) + " needs an engine that has not processed any batch");
}

std::vector<std::pair<std::string, std::string>> Engine::export_series() {
  flush();
  std::vector<std::pair<std::string, std::string>> r;
  r.reserve(series_.size());
  for (auto& si : series_) r.emplace_back(servers_[si.server], dict_.service_name(si.service));
  return r;
}

int32_t Engine::import_series(const std::string& server, const std::string& service) {
  flush();
  const int32_t sv = add_server(server);
  const int32_t id = dict_.service_id(service);
  const int32_t s = series_for(sv, id);
  if (s < 0) throw std::runtime_error("import_series: maxSeries exhausted");
  return s;
}

// ---------------------------------------------------------------- buckets

BucketDump Engine::export_buckets() {
  flush();
  HIP_OK(hipStreamSynchronize(stream_));
  BucketDump d;
  d.latest = latest_;
  const int32_t S = cfg_.max_series, n = n_series_, cap = cfg_.cell_cap;
  std::vector<int32_t> spill_n(nslot_), counts(n), cells((size_t)n * cap);
  HIP_OK(hipMemcpy(spill_n.data(), d_spill_n_, (size_t)nslot_ * 4, hipMemcpyDeviceToHost));
  std::vector<int64_t> slots;
  for (int slot = 0; slot < nslot_; ++slot)
    if (slot_bucket_[slot] != NO_BUCKET) slots.push_back(slot);
  std::sort(slots.begin(), slots.end(), [&](int a, int b) { return slot_bucket_[a] < slot_bucket_[b]; });
  for (int64_t slot : slots) {
    const int64_t b = slot_bucket_[slot];
    HIP_OK(hipMemcpy(counts.data(), d_counts_cells_ + (size_t)slot * S, (size_t)n * 4, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(cells.data(), d_cells_ + (size_t)slot * S * cap, (size_t)n * cap * 4, hipMemcpyDeviceToHost));
    const int32_t ns = std::min(spill_n[slot], cfg_.spill_cap);
    std::vector<int32_t> sp_s(ns), sp_v(ns);
    if (ns) {
      HIP_OK(hipMemcpy(sp_s.data(), d_spill_series_ + (size_t)slot * cfg_.spill_cap, (size_t)ns * 4, hipMemcpyDeviceToHost));
      HIP_OK(hipMemcpy(sp_v.data(), d_spill_val_ + (size_t)slot * cfg_.spill_cap, (size_t)ns * 4, hipMemcpyDeviceToHost));
    }
    std::vector<std::vector<int32_t>> extra;
    if (ns) extra.resize(n);
    for (int32_t k = 0; k < ns; ++k)
      if (sp_s[k] >= 0 && sp_s[k] < n) extra[sp_s[k]].push_back(sp_v[k]);
    for (int32_t s = 0; s < n; ++s) {
      if (counts[s] <= 0) continue;
      d.series.push_back(s);
      d.bucket.push_back(b);
      const int32_t k0 = std::min(counts[s], cap);
      int32_t c = 0;
      for (int32_t k = 0; k < k0; ++k, ++c) d.values.push_back(cells[(size_t)s * cap + k]);
      if (ns)
        for (int32_t v : extra[s]) { d.values.push_back(v); ++c; }
      d.count.push_back(c);
    }
  }
  return d;
}

void Engine::import_buckets(int64_t latest, const std::vector<int32_t>& series, const std::vector<int64_t>& bucket,
                            const std::vector<int32_t>& count, const std::vector<int32_t>& values) {
  flush();
  require_fresh("import_buckets");
  const int32_t S = cfg_.max_series, n = n_series_, cap = cfg_.cell_cap;
  if (series.size() != bucket.size() || series.size() != count.size())
    throw std::runtime_error("import_buckets: array sizes differ");
  latest_ = latest;
  const int64_t keep = cfg_.window + cfg_.buffer;
  std::map<int64_t, std::vector<size_t>> by_bucket;
  std::vector<size_t> off(series.size() + 1, 0);
  for (size_t i = 0; i < series.size(); ++i) off[i + 1] = off[i] + (size_t)count[i];
  if (off.back() != values.size()) throw std::runtime_error("import_buckets: values size mismatch");
  for (size_t i = 0; i < series.size(); ++i)
    if (bucket[i] >= latest - keep && bucket[i] <= latest) by_bucket[bucket[i]].push_back(i);
  for (auto& kv : by_bucket) {
    const int64_t b = kv.first;
    const int slot = (int)(((b % nslot_) + nslot_) % nslot_);
    if (slot_bucket_[slot] != NO_BUCKET && slot_bucket_[slot] != b) throw std::runtime_error("import_buckets: slot clash");
    slot_bucket_[slot] = b;
    std::vector<int32_t> counts(n, 0), cells((size_t)n * cap, 0), sp_s, sp_v;
    for (size_t i : kv.second) {
      const int32_t s = series[i];
      if (s < 0 || s >= n) throw std::runtime_error("import_buckets: bad series id");
      for (size_t j = off[i]; j < off[i + 1]; ++j) {
        const int32_t k = counts[s]++;
        if (k < cap) cells[(size_t)s * cap + k] = values[j];
        else { sp_s.push_back(s); sp_v.push_back(values[j]); }
      }
      h_active_[s] = 1;
    }
    if ((int64_t)sp_s.size() > cfg_.spill_cap) throw std::runtime_error("import_buckets: spill capacity exceeded");
    const int32_t sn = (int32_t)sp_s.size();
    HIP_OK(hipMemcpy(d_counts_cells_ + (size_t)slot * S, counts.data(), (size_t)n * 4, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_cells_ + (size_t)slot * S * cap, cells.data(), (size_t)n * cap * 4, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_spill_n_ + slot, &sn, 4, hipMemcpyHostToDevice));
    if (sn) {
      HIP_OK(hipMemcpy(d_spill_series_ + (size_t)slot * cfg_.spill_cap, sp_s.data(), (size_t)sn * 4, hipMemcpyHostToDevice));
      HIP_OK(hipMemcpy(d_spill_val_ + (size_t)slot * cfg_.spill_cap, sp_v.data(), (size_t)sn * 4, hipMemcpyHostToDevice));
    }
  }
  // every imported series existed in the reference's servers map: it gets stats rows
  std::vector<uint8_t> act(n, 0);
  for (int32_t s = 0; s < n; ++s) act[s] = h_active_[s];
  for (int32_t s : series) act[s] = 1, h_active_[s] = 1;
  HIP_OK(hipMemcpy(d_active_, act.data(), (size_t)n, hipMemcpyHostToDevice));
}

// ---------------------------------------------------------------- z-score history

void Engine::export_history(int lag_idx, int32_t lo, int32_t hi, std::vector<int32_t>& len, std::vector<double>& vals) {
  flush();
  if (lag_idx < 0 || lag_idx >= cfg_.n_lags) throw std::runtime_error("bad lag index");
  HIP_OK(hipStreamSynchronize(stream_));
  lo = std::max(0, lo);
  hi = std::min(hi, n_series_);
  const int32_t m = std::max(0, hi - lo), S = cfg_.max_series, L = cfg_.lags[lag_idx], rb = cfg_.ring_bytes;
  LagState& LS = lag_[lag_idx];
  len.assign(m, 0);
  if (m) HIP_OK(hipMemcpy(len.data(), LS.len + lo, (size_t)m * 4, hipMemcpyDeviceToHost));
  vals.assign((size_t)m * NSTAT * L, std::nan(""));
  const int head = (int)(rollover_idx_ % L);
  std::vector<uint8_t> row((size_t)m * rb);
  for (int k = 0; k < NSTAT; ++k)
    for (int pos = 0; pos < L; ++pos) {
      if (!m) break;
      HIP_OK(hipMemcpy(row.data(), (const char*)LS.ring + ((size_t)k * L + pos) * S * rb + (size_t)lo * rb, (size_t)m * rb,
                       hipMemcpyDeviceToHost));
      for (int32_t j = 0; j < m; ++j) {
        const int n = len[j];
        const int oldest = (head - n + L) % L;
        const int i = (pos - oldest + L) % L;  // chronological index of this slot
        if (i < n) vals[((size_t)j * NSTAT + k) * L + i] = ring_load(&row[(size_t)j * rb], rb);
      }
    }
}

void Engine::import_history(int lag_idx, const std::vector<int32_t>& series, const std::vector<int32_t>& len,
                            const std::vector<double>& vals) {
  flush();
  require_fresh("import_history");
  if (lag_idx < 0 || lag_idx >= cfg_.n_lags) throw std::runtime_error("bad lag index");
  const int32_t S = cfg_.max_series, L = cfg_.lags[lag_idx], rb = cfg_.ring_bytes, n = n_series_;
  if (series.size() != len.size() || vals.size() != series.size() * NSTAT * (size_t)L)
    throw std::runtime_error("import_history: array sizes differ");
  LagState& LS = lag_[lag_idx];
  std::vector<int32_t> h_len(n);
  HIP_OK(hipMemcpy(h_len.data(), LS.len, (size_t)n * 4, hipMemcpyDeviceToHost));
  std::vector<double> sum((size_t)NSTAT * n), comp((size_t)NSTAT * n), sq((size_t)NSTAT * n), sqc((size_t)NSTAT * n);
  std::vector<int32_t> cnt((size_t)NSTAT * n);
  for (int k = 0; k < NSTAT; ++k) {
    HIP_OK(hipMemcpy(sum.data() + (size_t)k * n, LS.sum + (size_t)k * S, (size_t)n * 8, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(comp.data() + (size_t)k * n, LS.comp + (size_t)k * S, (size_t)n * 8, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(sq.data() + (size_t)k * n, LS.sumsq + (size_t)k * S, (size_t)n * 8, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(sqc.data() + (size_t)k * n, LS.sqcomp + (size_t)k * S, (size_t)n * 8, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(cnt.data() + (size_t)k * n, LS.cnt + (size_t)k * S, (size_t)n * 4, hipMemcpyDeviceToHost));
  }
  const int head = (int)(rollover_idx_ % L);
  // ring rows [k][pos][0..n): read-modify-write row by row
  std::vector<uint8_t> row((size_t)n * rb);
  for (int k = 0; k < NSTAT; ++k)
    for (int pos = 0; pos < L; ++pos) {
      char* dev = (char*)LS.ring + ((size_t)k * L + pos) * S * rb;
      HIP_OK(hipMemcpy(row.data(), dev, (size_t)n * rb, hipMemcpyDeviceToHost));
      bool dirty = false;
      for (size_t j = 0; j < series.size(); ++j) {
        const int32_t s = series[j];
        const int m = std::min(len[j], L);
        const int oldest = (head - m + L) % L;
        const int i = (pos - oldest + L) % L;
        if (i < m) {
          ring_store(&row[(size_t)s * rb], rb, vals[((size_t)j * NSTAT + k) * L + i]);
          dirty = true;
        }
      }
      if (dirty) HIP_OK(hipMemcpy(dev, row.data(), (size_t)n * rb, hipMemcpyHostToDevice));
    }
  for (size_t j = 0; j < series.size(); ++j) {
    const int32_t s = series[j];
    if (s < 0 || s >= n) throw std::runtime_error("import_history: bad series id");
    const int m = std::min(len[j], L);
    h_len[s] = m;
    for (int k = 0; k < NSTAT; ++k) {
      double a = 0, c = 0, q = 0, qc = 0;
      int ct = 0;
      for (int i = 0; i < m; ++i) {
        double v = vals[((size_t)j * NSTAT + k) * L + i];
        // the value as the ring stores it
        uint8_t tmp[8];
        ring_store(tmp, rb, v);
        v = ring_load(tmp, rb);
        if (v == v) { neumaier(a, c, v); neumaier(q, qc, v * v); ++ct; }
      }
      sum[(size_t)k * n + s] = a; comp[(size_t)k * n + s] = c; sq[(size_t)k * n + s] = q;
      sqc[(size_t)k * n + s] = qc; cnt[(size_t)k * n + s] = ct;
    }
    if (!zscore_seen_[s]) {
      zscore_seen_[s] = 1;
      unseen_.erase(std::remove(unseen_.begin(), unseen_.end(), s), unseen_.end());
      apply_series_settings(s);  // the reference re-reads THRESHOLD/INFLUENCE from config on load
    }
  }
  HIP_OK(hipMemcpy(LS.len, h_len.data(), (size_t)n * 4, hipMemcpyHostToDevice));
  for (int k = 0; k < NSTAT; ++k) {
    HIP_OK(hipMemcpy(LS.sum + (size_t)k * S, sum.data() + (size_t)k * n, (size_t)n * 8, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(LS.comp + (size_t)k * S, comp.data() + (size_t)k * n, (size_t)n * 8, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(LS.sumsq + (size_t)k * S, sq.data() + (size_t)k * n, (size_t)n * 8, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(LS.sqcomp + (size_t)k * S, sqc.data() + (size_t)k * n, (size_t)n * 8, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(LS.cnt + (size_t)k * S, cnt.data() + (size_t)k * n, (size_t)n * 4, hipMemcpyHostToDevice));
  }
  upload_series_tables(0);
}

std::vector<double> Engine::export_lag_settings(int lag_idx) {
  flush();
  std::vector<double> r;
  for (int32_t s = 0; s < n_series_; ++s) {
    r.push_back(h_thr_[(size_t)s * MAX_LAGS + lag_idx]);
    r.push_back(h_infl_[(size_t)s * MAX_LAGS + lag_idx]);
  }
  return r;
}

// ---------------------------------------------------------------- release pool

std::vector<std::pair<int64_t, std::string>> Engine::export_pending() {
  flush();
  HIP_OK(hipStreamSynchronize(stream_));
  std::vector<int64_t> ends((size_t)pool_n_ + tail_n_), gids((size_t)pool_n_ + tail_n_);
  if (pool_n_) {
    HIP_OK(hipMemcpy(ends.data(), d_pool_end_[pool_cur_] + pool_off_, (size_t)pool_n_ * 8, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(gids.data(), d_pool_gid_[pool_cur_] + pool_off_, (size_t)pool_n_ * 8, hipMemcpyDeviceToHost));
  }
  if (tail_n_) {
    HIP_OK(hipMemcpy(ends.data() + pool_n_, d_tail_end_, (size_t)tail_n_ * 8, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(gids.data() + pool_n_, d_tail_gid_, (size_t)tail_n_ * 8, hipMemcpyDeviceToHost));
  }
  std::vector<std::pair<int64_t, std::string>> r;
  if (dev()) {  // lines in the HBM text ring (gather order = pool, then tail)
    const std::string text = ring_text(d_pool_gid_[pool_cur_] + pool_off_, pool_n_) + ring_text(d_tail_gid_, tail_n_);
    size_t p = 0;
    for (size_t i = 0; i < ends.size(); ++i) {
      const size_t len = (size_t)((uint64_t)gids[i] & 0xfffffu);
      r.emplace_back(ends[i], text.substr(p, len));
      p += len + 1;
    }
    std::stable_sort(r.begin(), r.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    return r;
  }
  for (size_t i = 0; i < ends.size(); ++i) {
    const uint64_t g = (uint64_t)gids[i];
    auto it = line_blocks_.find((uint32_t)(g >> 44));
    std::string line;
    if (it != line_blocks_.end()) {
      const size_t off = (size_t)((g >> 12) & 0xffffffffu);
      size_t len = (size_t)(g & 0xfff);
      if (len == 4095) len = it->second.data.find('\n', off) - off;
      line = it->second.data.substr(off, len);
    }
    r.emplace_back(ends[i], std::move(line));
  }
  std::stable_sort(r.begin(), r.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  return r;
}

void Engine::import_pending(const std::vector<int64_t>& ends, const std::vector<std::string>& lines) {
  flush();
  require_fresh("import_pending");
  if (ends.size() != lines.size()) throw std::runtime_error("import_pending: sizes differ");
  if (ends.empty()) return;
  if (pool_n_ + tail_n_ + (int64_t)ends.size() > cfg_.pool_cap) throw std::runtime_error("import_pending: pool full");
  if (dev()) {  // into the HBM text ring
    std::string text;
    std::vector<int64_t> gid(ends.size());
    for (size_t i = 0; i < ends.size(); ++i) {
      gid[i] = (int64_t)(((uint64_t)text.size() << 20) | (uint64_t)std::min<size_t>(lines[i].size(), 0xfffff));
      text += lines[i];
      text += '\n';
    }
    const uint64_t base = dj_->ring_reserve(text.size());
    for (auto& g : gid) g = (int64_t)(((((uint64_t)g >> 20) + base) << 20) | ((uint64_t)g & 0xfffffu));
    HIP_OK(hipMemcpy(dj_->ring() + (base & (dj_->ring_cap() - 1)), text.data(), text.size(), hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_tail_end_ + tail_n_, ends.data(), ends.size() * 8, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_tail_gid_ + tail_n_, gid.data(), ends.size() * 8, hipMemcpyHostToDevice));
    tail_n_ += (int64_t)ends.size();
    return;
  }
  const uint32_t id = (line_block_seq_++) & 0xFFFFFu;
  LineBlock& blk = line_blocks_[id];
  std::vector<int64_t> gid(ends.size());
  for (size_t i = 0; i < ends.size(); ++i) {
    const uint64_t off = blk.data.size();
    blk.data += lines[i];
    blk.data += '\n';
    gid[i] = (int64_t)(((uint64_t)id << 44) | (off << 12) | (uint64_t)std::min<size_t>(lines[i].size(), 4095));
    const int64_t b = ends[i] / 10000;
    pool_bucket_count_[b] += 1;
    if (ends[i] == b * 10000) pool_exact_edge_[b] += 1;
  }
  blk.live = (int64_t)ends.size();
  HIP_OK(hipMemcpy(d_tail_end_ + tail_n_, ends.data(), ends.size() * 8, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(d_tail_gid_ + tail_n_, gid.data(), ends.size() * 8, hipMemcpyHostToDevice));
  tail_n_ += (int64_t)ends.size();
}

// ---------------------------------------------------------------- alerts

std::vector<std::pair<std::string, double>> Engine::export_cooldowns() {
  flush();
  return cooldown_entries();
}

void Engine::import_cooldowns(const std::vector<std::pair<std::string, double>>& c) {
  flush();
  for (auto& kv : c) put_cooldown(kv.first, kv.second);
  rebuild_cool();
}

std::vector<int32_t> Engine::export_alert_counters(int lag_idx) {
  flush();
  std::vector<int32_t> r(n_series_);
  if (n_series_) HIP_OK(hipMemcpy(r.data(), lag_[lag_idx].counter, (size_t)n_series_ * 4, hipMemcpyDeviceToHost));
  return r;
}

void Engine::import_alert_counters(int lag_idx, const std::vector<int32_t>& series, const std::vector<int32_t>& counts) {
  flush();
  std::vector<int32_t> r = export_alert_counters(lag_idx);
  for (size_t i = 0; i < series.size(); ++i)
    if (series[i] >= 0 && series[i] < n_series_) r[series[i]] = counts[i];
  if (n_series_) HIP_OK(hipMemcpy(lag_[lag_idx].counter, r.data(), (size_t)n_series_ * 4, hipMemcpyHostToDevice));
}

}  // namespace apm
