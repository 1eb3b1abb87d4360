// Versioned binary checkpoint of one engine (one GPU / rank): everything needed to resume the
// pipeline mid-stream with identical output.
//
// The reference persists each stage separately as JSON every 60 s and on SIGTERM
// (stream_calc_stats.js:54-87 buckets + minHeap, stream_calc_z_score.js:37-64 per-lag history
// lists, stream_process_alerts.js:111-142, stream_insert_db.js:166-180) and loses the parser's
// join caches and tail positions on every restart.  Here one file holds:
//   topology (servers, files, service dictionary), series table + settings, log-time clock,
//   join caches of every shard (acct/record/need TTL caches, SOAP + audit contexts), the GPU
//   parse carry (open elapsed sections), live bucket cells, the z-score rings + rolling moments
//   + leaky counters of every LAG, the release pool + pending tx lines, alert cooldowns, and
//   undelivered output.
// Only the live part of device arrays is written: n_series columns of each ring row (2-D D2H
// copies through a pinned bounce buffer), compacted bucket cells.  Tail offsets live with the
// tailer (Python service writes them next to this file).
#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <thread>
#include <cstring>
#include <memory>

#include "../kernels/devjoin_api.h"
#include "binio.h"
#include "d2h.h"
#include "engine.h"

namespace apm {

namespace {

struct SeriesRec { int32_t server, service; uint64_t emit_key; };
struct I64Pair { int64_t a, b; };

// 2-D device <-> file copies of `rows` rows of `width` bytes taken from a pitched device array.
constexpr size_t kBounce = 64u << 20;

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void d2h_rows(BinWriter& w, const void* dev, size_t pitch, size_t width, size_t rows, void* bounce,
              hipStream_t st) {
  if (!width || !rows) return;
  if (CkDefer* d = ck_defer())
    if (d->take(w, dev, pitch, width, rows, st)) return;
  const size_t per = std::max<size_t>(1, kBounce / width);
  for (size_t r = 0; r < rows; r += per) {
    const size_t nr = std::min(per, rows - r);
    HIP_OK(hipMemcpy2DAsync(bounce, width, (const char*)dev + r * pitch, pitch, width, nr, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    w.raw(bounce, width * nr);
  }
}

void h2d_rows(BinReader& rd, void* dev, size_t pitch, size_t width, size_t rows, void* bounce, hipStream_t st) {
  if (!width || !rows) return;
  const size_t per = std::max<size_t>(1, kBounce / width);
  for (size_t r = 0; r < rows; r += per) {
    const size_t nr = std::min(per, rows - r);
    rd.raw(bounce, width * nr);
    HIP_OK(hipMemcpy2DAsync((char*)dev + r * pitch, pitch, bounce, width, width, nr, hipMemcpyHostToDevice, st));
    HIP_OK(hipStreamSynchronize(st));
  }
}

// A device array as BinWriter::vec writes it.  With a pinned bounce buffer the D2H runs at
// full link speed (a pageable destination is staged by the runtime in small pieces).
template <class T>
void d2h_vec(BinWriter& w, const T* dev, size_t n, hipStream_t st, void* bounce = nullptr) {
  if (bounce) {
    w.pod<uint64_t>(n);
    write_dev(w, dev, n * sizeof(T), st, (char*)bounce, kBounce);  // (deferred while a snapshot is taken)
    return;
  }
  std::vector<T> h(n);
  if (n) {
    HIP_OK(hipMemcpyAsync(h.data(), dev, n * sizeof(T), hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
  }
  w.vec(h);
}

template <class T>
size_t h2d_vec(BinReader& rd, T* dev, size_t cap, hipStream_t st) {
  std::vector<T> h = rd.vec<T>();
  if (h.size() > cap) throw std::runtime_error("checkpoint: array larger than this engine's capacity");
  if (!h.empty()) {
    HIP_OK(hipMemcpyAsync(dev, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice, st));
    HIP_OK(hipStreamSynchronize(st));
  }
  return h.size();
}

}  // namespace

// ------------------------------------------------------------------------------ JoinShard

void JoinShard::save(BinWriter& w) {
  w.pod(now_);
  w.pod(batch_no_);
  w.pod(counters);
  // raw service interning (order defines the ids)
  w.pod<uint64_t>(raw_svc_.size());
  for (auto& r : raw_svc_) { w.str(r.raw); w.str(r.norm); w.pod(r.norm_id); w.pod(r.toplevel); w.pod(r.hash); }
  // TTL caches
  w.pod<uint64_t>(acct_.size());
  acct_.for_each([&](uint64_t k, AcctEntry& e) { w.pod(k); w.pod(e); });
  w.pod<uint64_t>(record_.size());
  record_.for_each([&](uint64_t k, RecordEntry& e) {
    w.pod(k);
    w.pod(e.exp);
    w.pod<uint64_t>(e.items.size());
    for (auto& p : e.items) w.pod(p);
  });
  w.pod<uint64_t>(need_.size());
  need_.for_each([&](uint64_t k, NeedEntry& e) {
    w.pod(k);
    w.pod(e.exp);
    w.pod(e.created);
    w.str(e.log_id);
    w.vec(e.items);
  });
  for (auto* q : {&acct_fifo_, &record_fifo_, &need_fifo_}) {
    w.pod<uint64_t>(q->size());
    for (auto& x : *q) { w.pod(x.first); w.pod(x.second); }
  }
  // per-file contexts
  w.pod<uint64_t>(soap_.size());
  for (size_t f = 0; f < soap_.v.size(); ++f) {
    if (!soap_.present[f]) continue;
    const SoapCtx& c = soap_.v[f];
    w.pod((int32_t)f); w.str(c.log_id); w.pod(c.has_log_id); w.pod(c.pull_next);
  }
  w.pod<uint64_t>(audit_.size());
  for (auto& kv : audit_) {
    const AuditCtx& c = kv.second;
    w.pod(kv.first);
    w.pod<uint64_t>(c.autr_map.size());
    for (auto& a : c.autr_map) { w.str(a.first); w.str(a.second.first); w.str(a.second.second); }
    w.pod(c.active); w.str(c.active_log_id); w.str(c.active_alt); w.str(c.active_service);
    w.pod(c.has_active_service); w.pod(c.elapsed_flag); w.pod(c.sw_flag);
    w.pod<uint64_t>(c.service_map.size());
    for (auto& sm : c.service_map) {
      w.str(sm.first);
      w.pod<uint64_t>(sm.second.size());
      for (auto& it : sm.second) { w.str(it.elapsed); w.pod(it.has_start); w.str(it.start_ts); }
    }
  }
}

void JoinShard::load(BinReader& rd) {
  rd.pod(now_);
  rd.pod(batch_no_);
  rd.pod(counters);
  raw_svc_.clear();
  raw_svc_map_.clear();
  svc_info_.clear();
  svc_text_.clear();
  const uint64_t nr = rd.pod<uint64_t>();
  for (uint64_t i = 0; i < nr; ++i) {
    RawService r;
    r.raw = rd.str();
    r.norm = rd.str();
    rd.pod(r.norm_id);
    rd.pod(r.toplevel);
    rd.pod(r.hash);
    if (!raw_svc_map_.find(r.hash)) raw_svc_map_[r.hash] = (int32_t)i + 1;  // first occurrence wins, as when built
    svc_info_.push_back(SvcInfo{(uint32_t)svc_text_.size(), (uint32_t)r.norm.size(), r.norm_id, (uint32_t)r.raw.size(),
                                r.toplevel});
    svc_text_ += r.norm;
    raw_svc_.push_back(std::move(r));
  }
  acct_.clear();
  for (uint64_t n = rd.pod<uint64_t>(); n; --n) {
    const uint64_t k = rd.pod<uint64_t>();
    acct_[k] = rd.pod<AcctEntry>();
  }
  record_.clear();
  for (uint64_t n = rd.pod<uint64_t>(); n; --n) {
    const uint64_t k = rd.pod<uint64_t>();
    RecordEntry& e = record_[k];
    rd.pod(e.exp);
    for (uint64_t m = rd.pod<uint64_t>(); m; --m) e.items.push_back(rd.pod<Partial>());
  }
  need_.clear();
  for (uint64_t n = rd.pod<uint64_t>(); n; --n) {
    const uint64_t k = rd.pod<uint64_t>();
    NeedEntry& e = need_[k];
    rd.pod(e.exp);
    rd.pod(e.created);
    e.log_id = rd.str();
    e.items = rd.vec<Need>();
  }
  for (auto* q : {&acct_fifo_, &record_fifo_, &need_fifo_}) {
    q->clear();
    for (uint64_t n = rd.pod<uint64_t>(); n; --n) {
      const uint64_t k = rd.pod<uint64_t>();
      q->push_back({k, rd.pod<double>()});
    }
  }
  soap_.clear();
  for (uint64_t n = rd.pod<uint64_t>(); n; --n) {
    const int32_t f = rd.pod<int32_t>();
    SoapCtx c;
    c.log_id = rd.str();
    rd.pod(c.has_log_id);
    rd.pod(c.pull_next);
    soap_.put(f) = std::move(c);
  }
  audit_.clear();
  for (uint64_t n = rd.pod<uint64_t>(); n; --n) {
    const int32_t f = rd.pod<int32_t>();
    AuditCtx& c = audit_[f];
    for (uint64_t m = rd.pod<uint64_t>(); m; --m) {
      std::string a = rd.str(), b = rd.str(), d = rd.str();
      c.autr_map.push_back({a, {b, d}});
    }
    rd.pod(c.active); c.active_log_id = rd.str(); c.active_alt = rd.str(); c.active_service = rd.str();
    rd.pod(c.has_active_service); rd.pod(c.elapsed_flag); rd.pod(c.sw_flag);
    for (uint64_t m = rd.pod<uint64_t>(); m; --m) {
      std::string name = rd.str();
      std::deque<AuditItem> items;
      for (uint64_t j = rd.pod<uint64_t>(); j; --j) {
        AuditItem it;
        it.elapsed = rd.str();
        rd.pod(it.has_start);
        it.start_ts = rd.str();
        items.push_back(std::move(it));
      }
      c.service_map.push_back({name, std::move(items)});
    }
  }
}

// ------------------------------------------------------------------------------ Engine

void Engine::checkpoint_quiesce(const char* what) {
  flush();
  if (prefetched_) throw std::runtime_error(std::string(what) + ": a prefetched batch is pending (process it first)");
  HIP_OK(hipStreamSynchronize(parse_stream_));
  HIP_OK(hipStreamSynchronize(stream_));
}

uint64_t Engine::dump_state(const std::string& path, const std::string& reason) {
  std::string j = "{";
  auto num = [&](const char* k, double v) {
    char b[64];
    std::snprintf(b, sizeof b, "%.17g", v);
    if (j.size() > 1) j += ",";
    j += "\"" + std::string(k) + "\":" + (v == v && v - v == 0 ? std::string(b) : std::string("null"));
  };
  auto arr = [&](const char* k, const std::vector<double>& v) {
    if (j.size() > 1) j += ",";
    j += "\"" + std::string(k) + "\":[";
    for (size_t i = 0; i < v.size(); ++i) {
      char b[64];
      std::snprintf(b, sizeof b, "%.17g", v[i]);
      j += (i ? "," : "") + (v[i] == v[i] && v[i] - v[i] == 0 ? std::string(b) : std::string("null"));
    }
    j += "]";
  };
  const EngineMetrics& m = metrics_;
  num("batch_no", (double)batch_no_);
  num("watermark_ms", watermark_);
  num("latest_bucket", (double)latest_);
  num("rollover_idx", (double)rollover_idx_);
  num("n_series", (double)n_series_);
  num("max_series", (double)cfg_.max_series);
  num("device_bytes", (double)device_bytes_);
  num("batches", (double)m.batches); num("lines", (double)m.lines); num("bytes", (double)m.bytes);
  num("events", (double)m.events); num("tx", (double)m.tx); num("tx_dropped", (double)m.tx_dropped);
  num("rollovers", (double)m.rollovers); num("alerts", (double)m.alerts); num("released", (double)m.released);
  num("series_overflow_tx", (double)m.series_overflow_tx); num("spill_dropped", (double)m.spill_dropped);
  num("spill_capacity", (double)cfg_.spill_cap); num("spill_grows", (double)m.spill_grows);
  num("pending_tx", (double)(pool_n_ + tail_n_)); num("pending_tx_capacity", (double)cfg_.pool_cap);
  {
    std::vector<double> sb(nslot_), sn(nslot_);
    for (int s = 0; s < nslot_; ++s) {
      sb[s] = slot_bucket_[s] == NO_BUCKET ? -1.0 : (double)slot_bucket_[s];
      sn[s] = h_spill_snap_ ? (double)h_spill_snap_[s] : -1.0;
    }
    arr("slot_bucket", sb);
    arr("spill_fill_last_snapshot", sn);
  }
  if (dj_) {
    const JoinCounters c = dj_->counters();
    num("join_tx", (double)c.tx); num("join_partial_overflow", (double)c.partial_overflow);
    num("join_need_overflow", (double)c.need_overflow); num("join_table_full", (double)c.table_full);
    num("join_pool_exhausted", (double)c.pool_exhausted); num("join_table_slots", (double)c.table_slots);
    num("join_keys_live", (double)dj_->keys_live()); num("join_need_live", (double)dj_->need_live());
    num("join_need_arena", (double)c.need_arena_entries); num("join_chain_pool_blocks", (double)c.chain_pool_blocks);
    num("join_raw_services", (double)dj_->n_raw());
    num("tx_ring_head", (double)dj_->ring_head()); num("tx_ring_low", (double)dj_->ring_low());
    num("tx_ring_capacity", (double)dj_->ring_cap());
  }
  if (coll_) {
    num("coll_nranks", coll_->nranks());
    num("coll_rank", coll_->rank());
    num("coll_aborted", coll_->aborted() ? 1 : 0);
    num("fleet_rounds", (double)fleet_rounds_);
  }
  j += "}";
  BinWriter w(path);
  w.begin(SEC_DUMP);
  w.str(reason);
  w.str(j);
  w.end();
  write_series_dump(w);
  w.commit();
  return w.bytes();
}

// Per-series device state of the fatal dump (SEC_DUMP_SERIES): the window statistics of the last
// rollover, and per LAG the history length, leaky alert counter, z-score bounds / signals and
// rolling moments -- the ring-buffer metadata and per-series state SURVEY 2.2 maps heapdump to.
// Best effort: a faulted device context cannot be read; the section then says so (and why).
void Engine::write_series_dump(BinWriter& w) {
  const int32_t n = n_series_, S = cfg_.max_series;
  std::string err;
  auto rd = [&](void* dst, const void* src, size_t bytes) {
    if (!err.empty() || !bytes) return;
    const hipError_t e = hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost);
    if (e != hipSuccess) err = hipGetErrorString(e);
  };
  std::vector<WinStat> win((size_t)n);
  rd(win.data(), d_win_, (size_t)n * sizeof(WinStat));
  struct PerLag { std::vector<int32_t> len, counter, cnt; std::vector<ZOut> z; std::vector<double> sum; };
  std::vector<PerLag> pl((size_t)cfg_.n_lags);
  for (int l = 0; l < cfg_.n_lags; ++l) {
    PerLag& p = pl[(size_t)l];
    p.len.resize((size_t)n); p.counter.resize((size_t)n); p.z.resize((size_t)n);
    p.sum.resize((size_t)n * NSTAT); p.cnt.resize((size_t)n * NSTAT);
    rd(p.len.data(), lag_[l].len, (size_t)n * 4);
    rd(p.counter.data(), lag_[l].counter, (size_t)n * 4);
    rd(p.z.data(), lag_[l].out, (size_t)n * sizeof(ZOut));
    for (int k = 0; k < NSTAT; ++k) {
      rd(p.sum.data() + (size_t)k * n, lag_[l].sum + (size_t)k * S, (size_t)n * 8);
      rd(p.cnt.data() + (size_t)k * n, lag_[l].cnt + (size_t)k * S, (size_t)n * 4);
    }
  }
  if (!err.empty()) (void)hipGetLastError();
  std::string h = "{\"n\":" + std::to_string(err.empty() ? n : 0) + ",\"lags\":[";
  for (int l = 0; l < cfg_.n_lags; ++l) h += (l ? "," : "") + std::to_string(cfg_.lags[l]);
  h += "],\"device_readable\":" + std::string(err.empty() ? "true" : "false") + ",\"error\":\"";
  for (char c : err) h += (c == '"' || c == '\\') ? ' ' : c;
  h += "\"}";
  w.begin(SEC_DUMP_SERIES);
  w.str(h);
  const int32_t m = err.empty() ? n : 0;
  std::vector<std::string> srv((size_t)m), svc((size_t)m);
  {
    std::lock_guard<std::mutex> g(series_mu_);
    for (int32_t s = 0; s < m; ++s) {
      srv[(size_t)s] = servers_[series_[s].server];
      svc[(size_t)s] = dict_.service_name(series_[s].service);
    }
  }
  w.strs(srv);
  w.strs(svc);
  std::vector<double> wv((size_t)m * 6);
  for (int32_t s = 0; s < m; ++s) {
    const WinStat& x = win[(size_t)s];
    double* o = wv.data() + (size_t)s * 6;
    o[0] = x.tpm; o[1] = x.avg; o[2] = x.p75; o[3] = x.p95; o[4] = x.n; o[5] = x.active;
  }
  w.vec(wv);
  for (int l = 0; l < cfg_.n_lags; ++l) {
    PerLag& p = pl[(size_t)l];
    if (!m) { p.len.clear(); p.counter.clear(); p.sum.clear(); p.cnt.clear(); }
    std::vector<double> zv((size_t)m * 4 * NSTAT);
    for (int32_t s = 0; s < m; ++s) {
      const ZOut& z = p.z[(size_t)s];
      double* o = zv.data() + (size_t)s * 4 * NSTAT;
      for (int k = 0; k < NSTAT; ++k) {
        o[k] = z.mean[k]; o[NSTAT + k] = z.lb[k]; o[2 * NSTAT + k] = z.ub[k]; o[3 * NSTAT + k] = z.sig[k];
      }
    }
    w.vec(p.len);
    w.vec(p.counter);
    w.vec(zv);
    w.vec(p.sum);
    w.vec(p.cnt);
  }
  w.end();
}

uint64_t Engine::save_state(const std::string& path, const std::string& extra) {
  checkpoint_wait();  // an asynchronous checkpoint in flight finishes first
  checkpoint_quiesce("save_state");
  void* bounce = nullptr;
  HIP_OK(hipHostMalloc(&bounce, kBounce, hipHostMallocDefault));
  struct Guard { void* p; ~Guard() { hipHostFree(p); } } guard{bounce};
  BinWriter w(path);
  write_small_sections(w);
  // rings: every row of every LAG, synchronously through the bounce buffer
  w.begin(SEC_RING);
  const int32_t S = cfg_.max_series, n = n_series_;
  const size_t rb = (size_t)cfg_.ring_bytes;
  for (int l = 0; l < cfg_.n_lags; ++l) {
    std::vector<int32_t> heads(cfg_.lags[l]);
    for (int32_t h = 0; h < cfg_.lags[l]; ++h) heads[h] = h;
    w.pod<int32_t>(n);
    w.vec(heads);
    d2h_rows(w, lag_[l].ring, (size_t)S * rb, (size_t)n * rb, (size_t)NSTAT * cfg_.lags[l], bounce, stream_);
  }
  w.end();
  w.begin(SEC_EXTRA);
  w.str(extra);
  w.end();
  w.commit();
  ck_all_dirty_ = true;  // a standalone file does not extend an incremental chain
  return w.bytes();
}

// Every section but the rings.  Device arrays are read synchronously (the engine is quiescent).
void Engine::write_small_sections(BinWriter& w) {
  const int32_t S = cfg_.max_series, n = n_series_;
  if (!h_ck_bounce_) HIP_OK(hipHostMalloc(&h_ck_bounce_, kBounce, hipHostMallocDefault));
  void* bounce = h_ck_bounce_;

  w.begin(SEC_CONFIG);
  w.pod(cfg_.max_series); w.pod(cfg_.n_lags); w.raw(cfg_.lags, sizeof(cfg_.lags)); w.pod(cfg_.ring_bytes);
  w.pod(cfg_.cell_cap); w.pod(cfg_.spill_cap); w.pod(cfg_.pool_cap); w.pod(cfg_.window); w.pod(cfg_.buffer);
  w.end();

  w.begin(SEC_TOPOLOGY);
  w.strs(servers_);
  w.pod<uint64_t>(files_.size());
  for (auto& f : files_) { w.str(f.path); w.pod(f.server); w.pod(f.kind); }
  w.strs(dict_.services_snapshot());
  w.end();

  w.begin(SEC_SERIES);
  {
    std::vector<SeriesRec> sr(series_.size());
    for (size_t i = 0; i < series_.size(); ++i) sr[i] = {series_[i].server, series_[i].service, series_[i].emit_key};
    w.vec(sr);
  }
  w.vec(server_rank_); w.vec(server_next_service_); w.pod(next_server_rank_);
  w.vec(server_gidx_); w.vec(server_first_batch_);
  w.vec(h_thr_); w.vec(h_infl_); w.vec(h_hard_max_); w.vec(h_suppressed_); w.vec(h_emit_key_);
  w.vec(zscore_seen_); w.vec(h_active_); w.vec(unseen_);
  w.raw(alias_thr_, sizeof(alias_thr_)); w.raw(alias_infl_, sizeof(alias_infl_));
  w.end();

  w.begin(SEC_CLOCK);
  w.pod(watermark_); w.pod(batch_no_); w.pod(latest_); w.pod(rollover_idx_);
  w.vec(slot_bucket_);  // (its size is the ring's slot count)
  w.pod(next_gid_); w.pod(line_block_seq_);
  w.end();

  double tt = now_ms();
  auto mark = [&](const char* name) {  // per-section spans of the ingest stall (trace)
    const double t = now_ms();
    trace_event(name, tt, t, 0);
    tt = t;
  };
  mark("ck.host");
  w.begin(SEC_JOIN);
  w.pod<uint8_t>(dev() ? 1 : 0);
  if (dev()) {
    dj_->save(w);
    for (const auto& sp : dj_->save_spans) trace_event(sp.first, sp.second.first, sp.second.second, 0);
    w.vec(h_raw_series_);
  } else {
    w.pod<uint64_t>(shards_.size());
    for (auto& sh : shards_) sh->save(w);
  }
  w.end();

  mark("ck.join");
  w.begin(SEC_PARSE);
  d2h_vec(w, d_file_open_, 1 << 16, stream_, bounce);
  w.end();

  w.begin(SEC_BUCKETS);
  d2h_vec(w, d_active_, (size_t)n, stream_, bounce);
  {
    std::vector<int32_t> spill_n(nslot_);
    HIP_OK(hipMemcpy(spill_n.data(), d_spill_n_, (size_t)nslot_ * 4, hipMemcpyDeviceToHost));
    // the occupied cells of every live slot, packed on the device in one pass (scan + gather),
    // then written per slot straight from the pinned bounce
    std::vector<int32_t> slots;
    for (int slot = 0; slot < nslot_; ++slot)
      if (slot_bucket_[slot] != NO_BUCKET) slots.push_back(slot);
    const int k = (int)slots.size();
    const int32_t cap = cfg_.cell_cap;
    const uint64_t N = (uint64_t)k * (uint64_t)n;
    std::vector<uint32_t> bnd((size_t)k + 1, 0);
    // the packing scratch is about one more copy of the window cells: when HBM cannot hold it the
    // cells are packed on the host instead (slower, same bytes) -- a checkpoint never fails on it
    bool dev_pack = false;
    if (N) {
      if (N + 1 > ck_pack_n_) {
        auto drop = [this]() {
          for (void** q : {(void**)&d_ck_lens_, (void**)&d_ck_offs_, (void**)&d_ck_packed_, &d_ck_ptmp_}) {
            dfree(*q);
            *q = nullptr;
          }
          ck_pack_n_ = 0;
          ck_ptmp_bytes_ = 0;
        };
        drop();
        const uint64_t want = (N + 1) * 5 / 4;
        const size_t tb = apm_ck_pack_tmp_bytes(want);
        d_ck_lens_ = (uint32_t*)dmalloc_try(want * 4);
        d_ck_offs_ = (uint32_t*)dmalloc_try(want * 4);
        d_ck_packed_ = (int32_t*)dmalloc_try(want * (size_t)cap * 4);
        d_ck_ptmp_ = dmalloc_try(tb);
        if (d_ck_lens_ && d_ck_offs_ && d_ck_packed_ && d_ck_ptmp_) {
          ck_pack_n_ = want;
          ck_ptmp_bytes_ = tb;
        } else {
          drop();
        }
      }
      if (!d_ck_slots_) d_ck_slots_ = (int32_t*)dmalloc_try((size_t)nslot_ * 4);
      dev_pack = ck_pack_n_ >= N + 1 && d_ck_slots_;
    }
    if (dev_pack) {
      HIP_OK(hipMemcpyAsync(d_ck_slots_, slots.data(), (size_t)k * 4, hipMemcpyHostToDevice, stream_));
      if (apm_ck_pack_cells(d_counts_cells_, d_cells_, d_ck_slots_, k, n, S, cap, d_ck_lens_, d_ck_offs_, d_ck_ptmp_,
                            ck_ptmp_bytes_, d_ck_packed_, stream_) != 0)
        throw std::runtime_error("checkpoint: cell packing scratch too small");
      for (int i = 0; i <= k; ++i)
        HIP_OK(hipMemcpyAsync(&bnd[(size_t)i], d_ck_offs_ + (size_t)i * n, 4, hipMemcpyDeviceToHost, stream_));
      HIP_OK(hipStreamSynchronize(stream_));
    }
    for (int i = 0; i < k; ++i) {
      const int slot = slots[(size_t)i];
      w.pod<int32_t>(slot);
      w.pod<uint64_t>((uint64_t)n);  // counts (vec layout)
      write_dev(w, d_counts_cells_ + (size_t)slot * S, (size_t)n * 4, stream_, (char*)bounce, kBounce);
      if (dev_pack) {
        const uint64_t tot = bnd[(size_t)i + 1] - bnd[(size_t)i];
        w.pod<uint64_t>(tot);  // packed cells (vec layout)
        write_dev(w, d_ck_packed_ + bnd[(size_t)i], (size_t)tot * 4, stream_, (char*)bounce, kBounce);
      } else {  // host packing (no HBM for the scratch)
        std::vector<int32_t> cnt((size_t)n), cells((size_t)n * cap), packed;
        d2h_bounced(cnt.data(), d_counts_cells_ + (size_t)slot * S, (size_t)n * 4, stream_, (char*)bounce, kBounce);
        d2h_bounced(cells.data(), d_cells_ + (size_t)slot * S * cap, (size_t)n * cap * 4, stream_, (char*)bounce, kBounce);
        for (int32_t j = 0; j < n; ++j) {
          const int32_t c = std::max(0, std::min(cnt[(size_t)j], cap));
          packed.insert(packed.end(), cells.begin() + (ptrdiff_t)j * cap, cells.begin() + (ptrdiff_t)j * cap + c);
        }
        w.vec(packed);
      }
      const int32_t ns = std::min(spill_n[slot], cfg_.spill_cap);
      w.pod(spill_n[slot]);
      d2h_vec(w, d_spill_series_ + (size_t)slot * cfg_.spill_cap, (size_t)ns, stream_, bounce);
      d2h_vec(w, d_spill_val_ + (size_t)slot * cfg_.spill_cap, (size_t)ns, stream_, bounce);
    }
    w.pod<int32_t>(-1);
  }
  d2h_vec(w, d_nan_until_, (size_t)n, stream_, bounce);
  w.end();

  mark("ck.buckets");
  w.begin(SEC_ZSCORE);
  for (int l = 0; l < cfg_.n_lags; ++l) {
    LagState& L = lag_[l];
    d2h_vec(w, L.len, (size_t)n, stream_, bounce);
    d2h_vec(w, L.counter, (size_t)n, stream_, bounce);
    for (double* a : {L.sum, L.comp, L.sumsq, L.sqcomp}) d2h_rows(w, a, (size_t)S * 8, (size_t)n * 8, NSTAT, bounce, stream_);
    d2h_rows(w, L.cnt, (size_t)S * 4, (size_t)n * 4, NSTAT, bounce, stream_);
  }
  w.end();

  mark("ck.zscore");
  w.begin(SEC_POOL);
  w.pod(pool_off_); w.pod(pool_n_); w.pod(tail_n_);
  {
    std::vector<I64Pair> bc, ee;
    for (auto& kv : pool_bucket_count_) bc.push_back({kv.first, kv.second});
    for (auto& kv : pool_exact_edge_) ee.push_back({kv.first, kv.second});
    w.vec(bc);
    w.vec(ee);
  }
  d2h_vec(w, d_pool_end_[pool_cur_] + pool_off_, (size_t)pool_n_, stream_, bounce);
  d2h_vec(w, d_pool_gid_[pool_cur_] + pool_off_, (size_t)pool_n_, stream_, bounce);
  d2h_vec(w, d_tail_end_, (size_t)tail_n_, stream_, bounce);
  if (dev()) {
    // pending lines live in the HBM text ring: saved as one blob (pool lines, then tail lines)
    // with each gid rebased to its offset in the blob -- rebased on the device from the text
    // gather's own offsets and read with the other deferred sections (was: a synchronous D2H of
    // every gid and a host pass over them inside the checkpoint's ingest stall)
    const int64_t* srcs[2] = {d_pool_gid_[pool_cur_] + pool_off_, d_tail_gid_};
    const int64_t cnt[2] = {pool_n_, tail_n_};
    const size_t n_g = (size_t)(pool_n_ + tail_n_);
    if (n_g > ck_gids_cap_) {
      dfree(d_ck_gids_);
      ck_gids_cap_ = n_g + n_g / 4 + 1024;
      d_ck_gids_ = (int64_t*)dmalloc_try(ck_gids_cap_ * 8);
      if (!d_ck_gids_) ck_gids_cap_ = 0;
    }
    std::vector<int64_t> gids;
    if (!d_ck_gids_) {  // no HBM for it: the host pass
      gids.resize(n_g);
      d2h_bounced(gids.data(), srcs[0], (size_t)pool_n_ * 8, stream_, (char*)bounce, kBounce);
      d2h_bounced(gids.data() + pool_n_, srcs[1], (size_t)tail_n_ * 8, stream_, (char*)bounce, kBounce);
      uint64_t off = 0;
      for (auto& g : gids) {
        const uint64_t len = (uint64_t)g & 0xfffffu;
        g = (int64_t)((off << 20) | len);
        off += len + 1;
      }
    }
    // the text (pool lines, then tail lines): gathered on the device, written straight from the
    // pinned bounce into the snapshot (was: a hipMalloc + pageable copy + two string copies)
    uint32_t tot[2] = {0, 0};
    for (int k = 0; k < 2; ++k) {
      if (cnt[k] <= 0) continue;
      if (apm_dj_gather_plan(srcs[k], cnt[k], nullptr, d_rel_lens_, d_rel_offs_, d_release_tmp_, release_tmp_bytes_, stream_) != 0)
        throw std::runtime_error("checkpoint: ring text scratch too small");
      if (d_ck_gids_)
        apm_dj_rebase_gids(srcs[k], cnt[k], d_rel_offs_, k ? (uint64_t)tot[0] : 0, d_ck_gids_ + (k ? pool_n_ : 0),
                           stream_);
      HIP_OK(hipMemcpyAsync(&tot[k], d_rel_offs_ + cnt[k], 4, hipMemcpyDeviceToHost, stream_));
      HIP_OK(hipStreamSynchronize(stream_));
      if (!tot[k]) continue;
      const size_t need = ((size_t)tot[k] + 15) & ~(size_t)15;
      if (need > ck_text_cap_[k]) {
        dfree(d_ck_text_[k]);
        ck_text_cap_[k] = need + need / 4;
        d_ck_text_[k] = (char*)dmalloc_try(ck_text_cap_[k]);
        if (!d_ck_text_[k]) ck_text_cap_[k] = 0;
      }
      if (d_ck_text_[k])
        apm_dj_gather_copy(srcs[k], cnt[k], dj_->ring(), dj_->ring_cap(), d_rel_offs_, d_ck_text_[k], tot[k], stream_);
    }
    if (d_ck_gids_) d2h_vec(w, d_ck_gids_, n_g, stream_, bounce);  // (deferred while a snapshot is taken)
    else w.vec(gids);
    w.pod<uint64_t>((uint64_t)tot[0] + tot[1]);
    for (int k = 0; k < 2; ++k) {
      if (!tot[k]) continue;
      if (d_ck_text_[k] && ck_text_cap_[k] >= tot[k]) {
        write_dev(w, d_ck_text_[k], tot[k], stream_, (char*)bounce, kBounce);
      } else {  // no HBM for the gather target: line by line out of the ring on the host
        const std::string t = ring_text(srcs[k], cnt[k]);
        if (t.size() != tot[k]) throw std::runtime_error("checkpoint: pending-line text size changed");
        w.raw(t.data(), t.size());
      }
    }
  } else {
    d2h_vec(w, d_tail_gid_, (size_t)tail_n_, stream_);
    w.pod<uint64_t>(line_blocks_.size());
    for (auto& kv : line_blocks_) { w.pod(kv.first); w.pod(kv.second.live); w.str(kv.second.data); }
  }
  w.end();

  mark("ck.pool");
  w.begin(SEC_ALERTS);
  {
    const auto cool = cooldown_entries();
    w.pod<uint64_t>(cool.size());
    for (auto& kv : cool) { w.str(kv.first); w.pod(kv.second); }
  }
  w.end();

  w.begin(SEC_OUTPUTS);
  for (int k = 0; k < N_OUT; ++k) w.str(blob_[k]);
  w.end();

  w.begin(SEC_METRICS);
  {
    EngineMetrics m = metrics_;
    const uint64_t sc[] = {m.batches, m.bytes, m.lines, m.events, m.tx, m.tx_db, m.tx_dropped, m.rollovers,
                           m.alerts, m.alert_candidates, m.released};
    for (uint64_t v : sc) w.pod(v);
  }
  w.end();
}

namespace {
bool is_chain_manifest(const std::string& path) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) throw std::runtime_error("checkpoint: cannot open " + path);
  char m[8] = {0};
  const size_t got = std::fread(m, 1, 8, f);
  std::fclose(f);
  return got == 8 && std::memcmp(m, "APMCHAIN", 8) == 0;
}

std::string dir_of(const std::string& path) {
  const size_t slash = path.rfind('/');
  return slash == std::string::npos ? "." : (slash == 0 ? "/" : path.substr(0, slash));
}

// manifest: "APMCHAIN 1\n" then one file name (relative to the manifest's directory) per line,
// base first, increments in order
std::vector<std::string> read_chain(const std::string& path) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) throw std::runtime_error("checkpoint: cannot open " + path);
  std::vector<std::string> out;
  char line[4096];
  bool first = true;
  while (std::fgets(line, sizeof line, f)) {
    std::string l(line);
    while (!l.empty() && (l.back() == '\n' || l.back() == '\r')) l.pop_back();
    if (first) { first = false; continue; }
    if (!l.empty()) out.push_back(dir_of(path) + "/" + l);
  }
  std::fclose(f);
  if (out.empty()) throw std::runtime_error("checkpoint: empty chain manifest " + path);
  return out;
}

void fsync_dir(const std::string& path) {
  const int dfd = ::open(dir_of(path).c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
  if (dfd >= 0) { ::fsync(dfd); ::close(dfd); }
}

void write_text_atomic(const std::string& path, const std::string& body) {
  const std::string tmp = path + ".tmp";
  FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) throw std::runtime_error("checkpoint: cannot open " + tmp);
  if (std::fwrite(body.data(), 1, body.size(), f) != body.size()) { std::fclose(f); throw std::runtime_error("checkpoint: write failed"); }
  std::fflush(f);
  ::fsync(::fileno(f));
  std::fclose(f);
  if (std::rename(tmp.c_str(), path.c_str()) != 0) throw std::runtime_error("checkpoint: rename failed");
  fsync_dir(path);
}
}  // namespace

std::string Engine::load_state(const std::string& path) {
  if (is_chain_manifest(path)) {
    // incremental chain: the newest file holds the current small state; rings are the base's rows
    // overwritten by each increment's dirty rows, in order
    const std::vector<std::string> chain = read_chain(path);
    std::string extra = load_small_state(chain.back());
    for (const auto& f : chain) apply_ring_file(f);
    ck_all_dirty_ = true;
    return extra;
  }
  std::string extra = load_small_state(path);
  apply_ring_file(path);
  ck_all_dirty_ = true;
  return extra;
}

void Engine::apply_ring_file(const std::string& path) {
  void* bounce = nullptr;
  HIP_OK(hipHostMalloc(&bounce, kBounce, hipHostMallocDefault));
  struct Guard { void* p; ~Guard() { hipHostFree(p); } } guard{bounce};
  BinReader rd(path);
  rd.skip_to(SEC_RING);
  const int32_t S = cfg_.max_series;
  const size_t rb = (size_t)cfg_.ring_bytes;
  for (int l = 0; l < cfg_.n_lags; ++l) {
    int32_t nc = rd.pod<int32_t>();
    const bool row_major = nc < 0;  // a streamed snapshot: [row][stat][series] (write_streamed_ring)
    if (row_major) nc = -nc - 1;
    const std::vector<int32_t> heads = rd.vec<int32_t>();
    if (nc > n_series_) throw std::runtime_error("checkpoint: ring section wider than the series table");
    for (int32_t h : heads)
      if (h < 0 || h >= cfg_.lags[l]) throw std::runtime_error("checkpoint: bad ring row");
    if (row_major) {
      for (int32_t h : heads) {
        char* dst = (char*)lag_[l].ring + (size_t)h * S * rb;
        h2d_rows(rd, dst, (size_t)cfg_.lags[l] * S * rb, (size_t)nc * rb, NSTAT, bounce, stream_);
      }
      continue;
    }
    for (int k = 0; k < NSTAT; ++k)
      for (size_t i = 0; i < heads.size();) {  // runs of consecutive rows are contiguous in the file
        size_t j = i + 1;
        while (j < heads.size() && heads[j] == heads[j - 1] + 1) ++j;
        char* dst = (char*)lag_[l].ring + ((size_t)k * cfg_.lags[l] + (size_t)heads[i]) * S * rb;
        h2d_rows(rd, dst, (size_t)S * rb, (size_t)nc * rb, j - i, bounce, stream_);
        i = j;
      }
  }
  HIP_OK(hipStreamSynchronize(stream_));
}

std::string Engine::load_small_state(const std::string& path) {
  checkpoint_wait();
  flush();
  if (batch_no_ != 0 || n_series_ != 0 || !files_.empty())
    throw std::runtime_error("load_state needs a freshly constructed engine (no files, no batches)");
  const int32_t S = cfg_.max_series;
  void* bounce = nullptr;
  HIP_OK(hipHostMalloc(&bounce, kBounce, hipHostMallocDefault));
  struct Guard { void* p; ~Guard() { hipHostFree(p); } } guard{bounce};
  BinReader rd(path);

  rd.begin(SEC_CONFIG);
  {
    int32_t ms, cc, sc, win, buf;
    int nl, rb;
    int64_t pc;
    int32_t lags[MAX_LAGS];
    rd.pod(ms); rd.pod(nl); rd.raw(lags, sizeof(lags)); rd.pod(rb); rd.pod(cc); rd.pod(sc); rd.pod(pc);
    rd.pod(win); rd.pod(buf);
    if (nl != cfg_.n_lags || std::memcmp(lags, cfg_.lags, sizeof(lags)) != 0)
      throw std::runtime_error("checkpoint: LAG set differs from this engine's configuration");
    if (rb != cfg_.ring_bytes) throw std::runtime_error("checkpoint: ring dtype differs");
    if (cc != cfg_.cell_cap) throw std::runtime_error("checkpoint: bucket cell layout differs");
    if (sc > cfg_.spill_cap) grow_spill(sc);  // the saving engine had grown its spill lists
    if (win != cfg_.window || buf != cfg_.buffer) throw std::runtime_error("checkpoint: stats window differs");
    (void)ms; (void)pc;  // capacities may grow; checked per array below
  }

  rd.begin(SEC_TOPOLOGY);
  {
    auto servers = rd.strs();
    for (auto& s : servers) add_server(s);
    const uint64_t nf = rd.pod<uint64_t>();
    for (uint64_t i = 0; i < nf; ++i) {
      std::string p = rd.str();
      const int32_t srv = rd.pod<int32_t>();
      const uint8_t kind = rd.pod<uint8_t>();
      add_file(p, kind, servers.at(srv));
    }
    auto services = rd.strs();
    for (size_t i = 0; i < services.size(); ++i)
      if (dict_.service_id(services[i]) != (int32_t)i) throw std::runtime_error("checkpoint: dictionary mismatch");
  }

  rd.begin(SEC_SERIES);
  {
    auto sr = rd.vec<SeriesRec>();
    if ((int64_t)sr.size() > S) throw std::runtime_error("checkpoint: more series than maxSeries");
    server_rank_ = rd.vec<int32_t>();
    server_next_service_ = rd.vec<int32_t>();
    rd.pod(next_server_rank_);
    server_gidx_ = rd.vec<int32_t>();
    server_first_batch_ = rd.vec<int64_t>();
    h_thr_ = rd.vec<double>(); h_infl_ = rd.vec<double>(); h_hard_max_ = rd.vec<double>();
    h_suppressed_ = rd.vec<uint8_t>(); h_emit_key_ = rd.vec<uint64_t>();
    zscore_seen_ = rd.vec<int32_t>(); h_active_ = rd.vec<uint8_t>(); unseen_ = rd.vec<int32_t>();
    rd.raw(alias_thr_, sizeof(alias_thr_)); rd.raw(alias_infl_, sizeof(alias_infl_));
    series_.clear();
    series_map_.clear();
    ser_tab_.clear();
    ser_raw_.clear();
    for (size_t i = 0; i < sr.size(); ++i) {
      series_.push_back(SeriesInfo{sr[i].server, sr[i].service, sr[i].emit_key});
      series_map_[((uint64_t)(uint32_t)(sr[i].server + 1) << 32) | (uint32_t)sr[i].service] = (int32_t)i + 1;
      // K12 name tables, rebuilt in creation order exactly as series_for builds them
      const int32_t server = sr[i].server, service = sr[i].service;
      if ((int32_t)server_name_off_.size() <= server) server_name_off_.resize(server + 1, -1);
      if ((int32_t)service_name_off_.size() <= service) service_name_off_.resize(service + 1, -1);
      if (server_name_off_[server] < 0) server_name_off_[server] = intern_name(servers_[server]);
      if (service_name_off_[service] < 0) service_name_off_[service] = intern_name(dict_.service_name(service));
      h_ser_names_.push_back(server_name_off_[server]);
      h_ser_names_.push_back((int32_t)servers_[server].size());
      h_ser_names_.push_back(service_name_off_[service]);
      h_ser_names_.push_back((int32_t)dict_.service_name(service).size());
      max_name_len_ = std::max(max_name_len_, servers_[server].size() + dict_.service_name(service).size());
    }
    n_series_ = (int32_t)sr.size();
    perm_dirty_ = true;
    h_perm_.clear();
    h_perm_key_.clear();
    perm_uploaded_ = 0;
    series_service_uploaded_ = 0;
    svc_csr_n_ = -1;
  }
  const int32_t n = n_series_;

  rd.begin(SEC_CLOCK);
  rd.pod(watermark_); rd.pod(batch_no_); rd.pod(latest_); rd.pod(rollover_idx_);
  // the saver's ring may have another slot count (gpu.bucketRingSlots, a reload that grew it):
  // its buckets are placed at b % nslot_ of this ring, grown first if they do not fit
  const std::vector<int64_t> file_bucket = rd.vec<int64_t>();
  {
    int32_t live = 0;
    int64_t lo = INT64_MAX, hi = INT64_MIN;
    for (int64_t b : file_bucket)
      if (b != NO_BUCKET) { ++live; lo = std::min(lo, b); hi = std::max(hi, b); }
    if (live && hi - lo + 1 > nslot_) grow_ring((int32_t)(hi - lo + 1));
    std::fill(slot_bucket_.begin(), slot_bucket_.end(), NO_BUCKET);
    for (int64_t b : file_bucket)
      if (b != NO_BUCKET) slot_bucket_[(size_t)(((b % nslot_) + nslot_) % nslot_)] = b;
  }
  auto ring_slot_of = [&](int32_t fslot) -> int32_t {
    if (fslot < 0 || (size_t)fslot >= file_bucket.size() || file_bucket[(size_t)fslot] == NO_BUCKET)
      throw std::runtime_error("checkpoint: bad slot");
    const int64_t b = file_bucket[(size_t)fslot];
    return (int32_t)(((b % nslot_) + nslot_) % nslot_);
  };
  rd.pod(next_gid_); rd.pod(line_block_seq_);

  rd.begin(SEC_JOIN);
  {
    const uint8_t mode = rd.pod<uint8_t>();
    if (mode != (dev() ? 1 : 0))
      throw std::runtime_error("checkpoint: written with a different gpu.joinOnDevice setting");
    if (dev()) {
      dj_->load(rd);
      h_raw_series_ = rd.vec<int32_t>();
      std::vector<int32_t> pairs;
      for (size_t i = 0; i < h_raw_series_.size(); ++i)
        if (h_raw_series_[i] >= 0) { pairs.push_back((int32_t)i); pairs.push_back(h_raw_series_[i]); }
      if (!pairs.empty()) {
        int32_t* d = nullptr;
        HIP_OK(hipMalloc((void**)&d, pairs.size() * 4));
        HIP_OK(hipMemcpy(d, pairs.data(), pairs.size() * 4, hipMemcpyHostToDevice));
        apm_dj_scatter_i32(dj_->d_raw_series(), d, (uint32_t)(pairs.size() / 2), stream_);
        HIP_OK(hipStreamSynchronize(stream_));
        HIP_OK(hipFree(d));
      }
    } else {
      const uint64_t ns = rd.pod<uint64_t>();
      if (ns != shards_.size()) throw std::runtime_error("checkpoint: shard count mismatch");
      for (auto& sh : shards_) sh->load(rd);
    }
  }

  rd.begin(SEC_PARSE);
  h2d_vec(rd, d_file_open_, 1 << 16, stream_);

  rd.begin(SEC_BUCKETS);
  h2d_vec(rd, d_active_, (size_t)S, stream_);
  {
    std::vector<int32_t> cells((size_t)n * cfg_.cell_cap);
    for (;;) {
      const int32_t fslot = rd.pod<int32_t>();
      if (fslot < 0) break;
      const int32_t slot = ring_slot_of(fslot);
      auto counts = rd.vec<int32_t>();
      auto packed = rd.vec<int32_t>();
      if ((int32_t)counts.size() != n) throw std::runtime_error("checkpoint: bucket counts size");
      size_t p = 0;
      for (int32_t s = 0; s < n; ++s)
        for (int32_t k = 0; k < std::min(counts[s], cfg_.cell_cap); ++k) cells[(size_t)s * cfg_.cell_cap + k] = packed.at(p++);
      HIP_OK(hipMemcpy(d_counts_cells_ + (size_t)slot * S, counts.data(), (size_t)n * 4, hipMemcpyHostToDevice));
      HIP_OK(hipMemcpy(d_cells_ + (size_t)slot * S * cfg_.cell_cap, cells.data(), (size_t)n * cfg_.cell_cap * 4,
                       hipMemcpyHostToDevice));
      const int32_t sn = rd.pod<int32_t>();
      HIP_OK(hipMemcpy(d_spill_n_ + slot, &sn, 4, hipMemcpyHostToDevice));
      h2d_vec(rd, d_spill_series_ + (size_t)slot * cfg_.spill_cap, (size_t)cfg_.spill_cap, stream_);
      h2d_vec(rd, d_spill_val_ + (size_t)slot * cfg_.spill_cap, (size_t)cfg_.spill_cap, stream_);
    }
  }
  h2d_vec(rd, d_nan_until_, (size_t)S, stream_);
  spill_resync();  // the restored fill levels bound the next appends

  rd.begin(SEC_ZSCORE);
  for (int l = 0; l < cfg_.n_lags; ++l) {
    LagState& L = lag_[l];
    h2d_vec(rd, L.len, (size_t)S, stream_);
    h2d_vec(rd, L.counter, (size_t)S, stream_);
    for (double* a : {L.sum, L.comp, L.sumsq, L.sqcomp}) h2d_rows(rd, a, (size_t)S * 8, (size_t)n * 8, NSTAT, bounce, stream_);
    h2d_rows(rd, L.cnt, (size_t)S * 4, (size_t)n * 4, NSTAT, bounce, stream_);
  }

  rd.begin(SEC_POOL);
  {
    int64_t off, pn, tn;
    rd.pod(off); rd.pod(pn); rd.pod(tn);
    auto bc = rd.vec<I64Pair>();
    auto ee = rd.vec<I64Pair>();
    pool_bucket_count_.clear();
    pool_exact_edge_.clear();
    for (auto& x : bc) pool_bucket_count_[x.a] = x.b;
    for (auto& x : ee) pool_exact_edge_[x.a] = x.b;
    pool_cur_ = 0;
    pool_off_ = 0;
    pool_n_ = (int64_t)h2d_vec(rd, d_pool_end_[0], (size_t)cfg_.pool_cap, stream_);
    h2d_vec(rd, d_pool_gid_[0], (size_t)cfg_.pool_cap, stream_);
    tail_n_ = (int64_t)h2d_vec(rd, d_tail_end_, (size_t)cfg_.pool_cap, stream_);
    if (dev()) {
      auto gids = rd.vec<int64_t>();
      const std::string text = rd.str();
      if ((int64_t)gids.size() != pool_n_ + tail_n_) throw std::runtime_error("checkpoint: pool size mismatch");
      // the blob goes to the start of the (fresh) ring: blob offsets are ring positions
      if (text.size() > dj_->ring_cap() / 2) throw std::runtime_error("checkpoint: pending tx text exceeds the ring");
      if (!text.empty()) HIP_OK(hipMemcpy(dj_->ring(), text.data(), text.size(), hipMemcpyHostToDevice));
      dj_->reset_ring(text.size());
      if (pool_n_) HIP_OK(hipMemcpy(d_pool_gid_[0], gids.data(), (size_t)pool_n_ * 8, hipMemcpyHostToDevice));
      if (tail_n_) HIP_OK(hipMemcpy(d_tail_gid_, gids.data() + pool_n_, (size_t)tail_n_ * 8, hipMemcpyHostToDevice));
      *h_ring_min_ = ~0ULL;
      ring_low_pending_ = UINT64_MAX;
    } else {
      h2d_vec(rd, d_tail_gid_, (size_t)cfg_.pool_cap, stream_);
      if (pool_n_ != pn || tail_n_ != tn) throw std::runtime_error("checkpoint: pool size mismatch");
      line_blocks_.clear();
      for (uint64_t k = rd.pod<uint64_t>(); k; --k) {
        const uint32_t id = rd.pod<uint32_t>();
        LineBlock& b = line_blocks_[id];
        rd.pod(b.live);
        b.data = rd.str();
      }
    }
    (void)off;
  }

  rd.begin(SEC_ALERTS);
  last_alert_.clear();
  node_cool_.clear();
  for (uint64_t k = rd.pod<uint64_t>(); k; --k) {
    std::string key = rd.str();
    put_cooldown(key, rd.pod<double>());
  }
  rebuild_cool();

  rd.begin(SEC_OUTPUTS);
  for (int k = 0; k < N_OUT; ++k) blob_[k] = rd.str();

  rd.begin(SEC_METRICS);
  {
    uint64_t* sc[] = {&metrics_.batches, &metrics_.bytes, &metrics_.lines, &metrics_.events, &metrics_.tx,
                      &metrics_.tx_db, &metrics_.tx_dropped, &metrics_.rollovers, &metrics_.alerts,
                      &metrics_.alert_candidates, &metrics_.released};
    for (uint64_t* v : sc) rd.pod(*v);
  }
  rd.skip_to(SEC_EXTRA);
  std::string extra = rd.str();
  rd.finish();
  upload_series_tables(0);
  HIP_OK(hipStreamSynchronize(stream_));
  return extra;
}

// ------------------------------------------------------------------------------ async checkpoint
//
// The ingest thread pays only for a consistent snapshot: the small sections are serialised to
// memory (their device arrays are small), and the ring rows written since the previous
// checkpoint (one row per rollover per LAG; all rows for a new base) are copied D2D into an HBM
// staging area on the engine stream -- ~5 TB/s, so even a full 17 GB ring costs a few ms.  A
// writer thread then drains the staging area D2H on its own stream through a pinned bounce
// buffer, writes + fsyncs the file, and appends it to the chain manifest (atomic rename).  A new
// base starts a fresh chain (and retires the old files) after kMaxChain increments.
int64_t Engine::checkpoint_async(const std::string& prefix, const std::string& extra, bool force_base,
                                 std::function<void()> pre_commit) {
  {
    std::lock_guard<std::mutex> lk(ck_mu_);
    if (ck_busy_) { ++ck_skipped_; return -1; }
  }
  const double t0 = now_ms();
  checkpoint_quiesce("checkpoint_async");
  trace_event("ck.quiesce", t0, now_ms(), 0);
  auto job = std::make_shared<CkJob>();
  const bool base = force_base || ck_all_dirty_ || ck_chain_.empty() || ck_prefix_ != prefix ||
                    (int)ck_chain_.size() > kMaxChain;
  job->base = base;
  job->prefix = prefix;
  job->seq = ++ck_seq_;
  job->name = prefix.substr(prefix.rfind('/') + 1) + (base ? ".b" : ".i") + std::to_string(job->seq) + ".ckpt";
  job->path = dir_of(prefix) + "/" + job->name;
  job->extra = extra;
  job->pre_commit = std::move(pre_commit);
  {
    // the small sections' device reads become D2D copies into HBM staging (1.5x the previous
    // snapshot's want, at least 1 GiB -- the process's first snapshot has no previous want and
    // read everything synchronously: 34-36 ms stalls, profiles/r5_final2; a read that does not
    // fit is still done synchronously)
    CkDefer def;
    constexpr size_t kMinStage = (size_t)1 << 30;
    if (ck_defer_want_ > ck_defer_cap_ || !d_ck_defer_) {
      if (d_ck_defer_) {
        HIP_OK(hipFree(d_ck_defer_));
        std::lock_guard<std::mutex> g(alloc_mu_);
        device_bytes_ -= ck_defer_cap_;
      }
      const size_t cap = std::max(ck_defer_want_ + ck_defer_want_ / 2, kMinStage);
      if (hipMalloc((void**)&d_ck_defer_, cap) != hipSuccess) {
        (void)hipGetLastError();
        d_ck_defer_ = nullptr;
        ck_defer_cap_ = 0;
      } else {
        ck_defer_cap_ = cap;
        std::lock_guard<std::mutex> g(alloc_mu_);
        device_bytes_ += cap;
      }
    }
    def.stage = d_ck_defer_;
    def.cap = ck_defer_cap_;
    MemBlob spare;
    {
      std::lock_guard<std::mutex> lk(ck_mu_);
      spare = std::move(ck_blob_spare_);
    }
    BinWriter mw{BinWriter::Memory{}, std::move(spare), ck_blob_hint_};
    ck_defer() = &def;
    const double ts0 = now_ms();
    try {
      write_small_sections(mw);
    } catch (...) {
      ck_defer() = nullptr;
      throw;
    }
    ck_defer() = nullptr;
    ck_defer_want_ = def.want;
    ck_deferred_bytes_ = def.used;
    // the D2D copies complete before the engine resumes (~TB/s: under a millisecond for the
    // snapshot's ~100 MB): a source array another stream writes next (the parse carry on the parse
    // stream, the z-score state on the rollover lane's) cannot change under a queued copy
    const double ts1 = now_ms();
    for (hipStream_t ds : def.streams) HIP_OK(hipStreamSynchronize(ds));
    trace_event("ck.small_sections", ts0, ts1, 0);
    trace_event("ck.defer_sync", ts1, now_ms(), 0);
    for (const auto& h : def.holes) job->holes.push_back({h.blob_off, h.stage_off, h.len});
    job->patches = std::move(def.patches);
    job->blob = mw.take_memory();
    ck_blob_hint_ = job->blob.size() + job->blob.size() / 8 + (1u << 20);
  }
  // dirty ring rows -> HBM staging (D2D, stream-ordered after the quiesce point)
  const double tring = now_ms();
  const int32_t S = cfg_.max_series, n = n_series_;
  const size_t rb = (size_t)cfg_.ring_bytes;
  const int64_t r1 = rollover_idx_;
  size_t need = 0;
  for (int l = 0; l < cfg_.n_lags; ++l) {
    const int32_t L = cfg_.lags[l];
    CkJob::Lag lg;
    lg.n_cols = n;
    const int64_t dirty = base ? L : std::min<int64_t>(L, r1 - ck_ridx_);
    const int32_t h0 = base || dirty == L ? 0 : (int32_t)(ck_ridx_ % L);
    for (int64_t i = 0; i < dirty; ++i) lg.heads.push_back((int32_t)((h0 + i) % L));
    lg.off = need;
    need += (size_t)NSTAT * lg.heads.size() * n * rb;
    job->lags.push_back(std::move(lg));
  }
  const size_t cap = cfg_.ck_stage_bytes > 0 ? (size_t)cfg_.ck_stage_bytes : SIZE_MAX;
  const size_t row_bytes = (size_t)NSTAT * n * rb;  // one ring position of one LAG, every stat
  if (need > cap && n > 0) {
    // Streamed snapshot: the ring rows do not fit the staging cap (rings sized toward HBM).  Stage
    // the rows the next rollovers overwrite first -- position (r1 + i) % L of every LAG, i = 0, 1,
    // ... -- in 80 % of the cap; the writer reads the others from the live ring in overwrite order,
    // and ck_guard_rollover copies a row aside (the other 20 %) if a rollover reaches it first.
    job->streamed = true;
    const size_t main_cap = cap / 5 * 4, side_cap = cap - main_cap;
    if (!ck_side_ev_) HIP_OK(hipEventCreateWithFlags(&ck_side_ev_, hipEventDisableTiming));
    std::lock_guard<std::mutex> g(cks_mu_);
    cks_ = CkStream{};
    cks_.on = true;
    cks_.n_cols = n;
    cks_.state.resize(cfg_.n_lags);
    cks_.off.resize(cfg_.n_lags);
    std::vector<std::vector<int32_t>> order(cfg_.n_lags);
    for (int l = 0; l < cfg_.n_lags; ++l) {
      const int32_t L = cfg_.lags[l];
      cks_.state[l].assign((size_t)L, CKR_NONE);
      cks_.off[l].assign((size_t)L, 0);
      std::vector<int32_t> hs = job->lags[l].heads;  // this snapshot's rows, by next overwrite
      std::sort(hs.begin(), hs.end(), [&](int32_t a, int32_t b) {
        return ((a - r1 % L) % L + L) % L < ((b - r1 % L) % L + L) % L;
      });
      order[l] = std::move(hs);
      for (int32_t h : order[l]) cks_.state[l][(size_t)h] = CKR_LIVE;
    }
    // round-robin over the LAGs by overwrite rank: row i of every LAG before row i + 1 of any
    size_t staged = 0;
    std::vector<std::vector<int32_t>> stg(cfg_.n_lags);
    for (size_t i = 0;; ++i) {
      bool any = false, full = false;
      for (int l = 0; l < cfg_.n_lags && !full; ++l) {
        if (i >= order[l].size()) continue;
        any = true;
        if (staged + row_bytes > main_cap) { full = true; break; }
        stg[l].push_back(order[l][i]);
        cks_.state[l][(size_t)order[l][i]] = CKR_STAGED;
        staged += row_bytes;
      }
      if (!any || full) break;
    }
    // staging layout: each LAG's staged rows together in overwrite order (consecutive ring
    // positions, so a run of them is one strided copy per stat below, not one copy per row)
    size_t at = 0;
    for (int l = 0; l < cfg_.n_lags; ++l)
      for (int32_t h : stg[l]) { cks_.off[l][(size_t)h] = at; at += row_bytes; }
    // file order per LAG: the live rows in overwrite order (the writer races the rollovers), then
    // the staged ones
    for (int l = 0; l < cfg_.n_lags; ++l) {
      std::vector<int32_t> fo;
      for (int32_t h : order[l])
        if (cks_.state[l][(size_t)h] == CKR_LIVE) fo.push_back(h);
      for (int32_t h : stg[l]) fo.push_back(h);
      job->lags[l].heads = std::move(fo);
    }
    need = staged + side_cap;
    cks_.side_cap = side_cap;
  }
  ck_last_need_ = need;
  if (need > ck_stage_bytes_) {
    free_ck_stage();
    // Sized once for the rings at maxSeries (capped): a service's first checkpoint comes while few
    // series exist, and growing the staging at a later base put a 2 GiB hipFree + hipMalloc into
    // that base's ingest stall (2.1 ms of 11-15 ms, profiles/r6_l servicetrace ck.ring_stage).
    size_t full = 0;
    for (int l = 0; l < cfg_.n_lags; ++l) full += (size_t)NSTAT * cfg_.lags[l] * (size_t)S * rb;
    const size_t want = job->streamed ? need : std::min(cap, std::max(need + need / 8, full));  // (room for the series table)
    if (hipMalloc(&d_ck_stage_, want) != hipSuccess) {
      (void)hipGetLastError();
      d_ck_stage_ = nullptr;
      {
        std::lock_guard<std::mutex> g(cks_mu_);
        cks_.on = false;
      }
      // not enough HBM for a snapshot: fall back to the synchronous writer
      ck_all_dirty_ = true;
      if (job->pre_commit) job->pre_commit();  // (first: see checkpoint_writer)
      const uint64_t bytes = save_state(job->path, extra);
      job->base = true;
      finish_chain(job, bytes);
      ck_last_stall_ms_ = now_ms() - t0;
      ++ck_sync_fallbacks_;
      ck_ridx_ = r1;
      ck_all_dirty_ = false;
      return job->seq;
    }
    ck_stage_bytes_ = want;
    std::lock_guard<std::mutex> g(alloc_mu_);
    device_bytes_ += want;
  }
  if (job->streamed) {
    // staged rows: all NSTAT planes of a position together (the row-major file layout)
    std::lock_guard<std::mutex> g(cks_mu_);
    d_ck_side_ = (char*)d_ck_stage_ + (need - cks_.side_cap);
    // a run of staged rows at consecutive positions h0 .. h0 + m - 1 (ascending offsets): per stat
    // one 2D copy, source pitch = a ring position, destination pitch = a staged row (the
    // per-row form was ~900 copies and ~6 ms of ingest stall per base at the headline)
    for (int l = 0; l < cfg_.n_lags; ++l) {
      const int32_t L = cfg_.lags[l];
      for (int32_t h = 0; h < L;) {
        if (cks_.state[l][(size_t)h] != CKR_STAGED) { ++h; continue; }
        int32_t m = 1;
        while (h + m < L && cks_.state[l][(size_t)(h + m)] == CKR_STAGED &&
               cks_.off[l][(size_t)(h + m)] == cks_.off[l][(size_t)h] + (size_t)m * row_bytes)
          ++m;
        for (int k = 0; k < NSTAT; ++k) {
          char* dst = (char*)d_ck_stage_ + cks_.off[l][(size_t)h] + (size_t)k * n * rb;
          const char* src = (const char*)lag_[l].ring + ((size_t)k * L + (size_t)h) * S * rb;
          HIP_OK(hipMemcpy2DAsync(dst, row_bytes, src, (size_t)S * rb, (size_t)n * rb, (size_t)m,
                                  hipMemcpyDeviceToDevice, stream_));
        }
        h += m;
      }
    }
    ++ck_streamed_;
  } else {
    for (int l = 0; l < cfg_.n_lags; ++l) {
      const CkJob::Lag& lg = job->lags[l];
      const int32_t L = cfg_.lags[l];
      char* dst = (char*)d_ck_stage_ + lg.off;
      for (int k = 0; k < NSTAT; ++k)
        for (size_t i = 0; i < lg.heads.size();) {
          size_t j = i + 1;
          while (j < lg.heads.size() && lg.heads[j] == lg.heads[j - 1] + 1) ++j;
          const char* src = (const char*)lag_[l].ring + ((size_t)k * L + (size_t)lg.heads[i]) * S * rb;
          if (n > 0)
            HIP_OK(hipMemcpy2DAsync(dst, (size_t)n * rb, src, (size_t)S * rb, (size_t)n * rb, j - i,
                                    hipMemcpyDeviceToDevice, stream_));
          dst += (j - i) * (size_t)n * rb;
          i = j;
        }
    }
  }
  if (!ck_ev_) HIP_OK(hipEventCreateWithFlags(&ck_ev_, hipEventDisableTiming));
  HIP_OK(hipEventRecord(ck_ev_, stream_));
  trace_event("ck.ring_stage", tring, now_ms(), 0);
  ck_ridx_ = r1;
  ck_all_dirty_ = false;
  ck_prefix_ = prefix;
  ck_last_stall_ms_ = now_ms() - t0;
  ck_last_mode_ = base ? 1 : 0;
  ck_last_ring_rows_ = 0;
  for (const auto& lg : job->lags) ck_last_ring_rows_ += (int64_t)lg.heads.size();
  {
    std::lock_guard<std::mutex> lk(ck_mu_);
    ck_busy_ = true;
    ck_job_ = job;
  }
  if (!ck_thread_.joinable()) ck_thread_ = std::thread([this] { checkpoint_writer(); });
  ck_cv_.notify_all();
  return job->seq;
}

// Writer thread: the ring section of a streamed snapshot, row-major -- the NSTAT planes of a
// position together; n_cols is stored as -(n_cols + 1), which tells apply_ring_file / merge the
// layout.  Each row comes from the staging, the side copy a rollover made, or the live ring (read
// under the CKR_READING mark, which a rollover about to overwrite that row waits out).
void Engine::write_streamed_ring(const std::shared_ptr<CkJob>& job, BinWriter& w, char* bounce) {
  const int32_t S = cfg_.max_series;
  const size_t rb = (size_t)cfg_.ring_bytes;
  // test hook: a slow checkpoint disk (per-row delay), so rollovers overtake the writer
  static const int delay_us = [] { const char* e = std::getenv("APM_CK_ROW_DELAY_US"); return e ? std::atoi(e) : 0; }();
  for (size_t l = 0; l < job->lags.size(); ++l) {
    const CkJob::Lag& lg = job->lags[l];
    const int32_t L = cfg_.lags[l];
    const size_t width = (size_t)lg.n_cols * rb;
    w.pod<int32_t>(-lg.n_cols - 1);
    w.vec(lg.heads);
    for (int32_t h : lg.heads) {
      uint8_t st;
      size_t off;
      bool sync = false;
      {
        std::lock_guard<std::mutex> lk(cks_mu_);
        st = cks_.state[l][(size_t)h];
        off = cks_.off[l][(size_t)h];
        if (st == CKR_LIVE) cks_.state[l][(size_t)h] = CKR_READING;
        if (st == CKR_SIDE && cks_.side_sync) { sync = true; cks_.side_sync = false; }
      }
      if (sync) HIP_OK(hipEventSynchronize(ck_side_ev_));  // every side copy queued so far has run
      const char* src;
      size_t pitch;
      if (st == CKR_LIVE) {
        src = (const char*)lag_[l].ring + (size_t)h * S * rb;
        pitch = (size_t)L * S * rb;
      } else if (st == CKR_STAGED || st == CKR_SIDE) {
        src = (st == CKR_STAGED ? (const char*)d_ck_stage_ : (const char*)d_ck_side_) + off;
        pitch = width;
      } else {
        throw std::runtime_error("checkpoint: streamed ring row in state " + std::to_string(st));
      }
      d2h_rows(w, src, pitch, width, NSTAT, bounce, ck_stream_);
      if (delay_us > 0) std::this_thread::sleep_for(std::chrono::microseconds(delay_us));
      {
        std::lock_guard<std::mutex> lk(cks_mu_);
        cks_.state[l][(size_t)h] = CKR_DONE;
        if (st == CKR_LIVE) ++cks_.live_rows;
      }
      cks_cv_.notify_all();
    }
  }
}

// Stats thread, before rollover r's K10 writes ring position r % L of every LAG: a streamed
// snapshot's row the writer has not read yet is copied aside first (D2D on this stream, ordered
// before the overwrite); while the writer is reading it -- or the side staging is full -- the
// rollover waits for the writer (counted: guard_stalls).
void Engine::ck_guard_rollover(int64_t r) {
  std::unique_lock<std::mutex> lk(cks_mu_);
  if (!cks_.on) return;
  const int32_t S = cfg_.max_series;
  const size_t rb = (size_t)cfg_.ring_bytes;
  const size_t width = (size_t)cks_.n_cols * rb, row_bytes = (size_t)NSTAT * width;
  bool copied = false;
  for (int l = 0; l < cfg_.n_lags && l < (int)cks_.state.size(); ++l) {
    const int32_t L = cfg_.lags[l];
    if ((int32_t)cks_.state[l].size() != L) continue;
    const int32_t h = (int32_t)(r % L);
    for (;;) {
      if (!cks_.on) return;
      uint8_t& st = cks_.state[l][(size_t)h];
      if (st == CKR_LIVE && cks_.side_used + row_bytes <= cks_.side_cap) {
        HIP_OK(hipMemcpy2DAsync(d_ck_side_ + cks_.side_used, width, (const char*)lag_[l].ring + (size_t)h * S * rb,
                                (size_t)L * S * rb, width, NSTAT, hipMemcpyDeviceToDevice, stream_));
        cks_.off[l][(size_t)h] = cks_.side_used;
        cks_.side_used += row_bytes;
        st = CKR_SIDE;
        ++cks_.side_rows;
        copied = true;
        break;
      }
      if (st != CKR_LIVE && st != CKR_READING) break;
      ++cks_.stalls;
      cks_cv_.wait(lk);
    }
  }
  if (copied) {
    HIP_OK(hipEventRecord(ck_side_ev_, stream_));
    cks_.side_sync = true;
  }
}

void Engine::free_ck_stage() {
  if (!d_ck_stage_) return;
  HIP_OK(hipFree(d_ck_stage_));
  d_ck_stage_ = nullptr;
  std::lock_guard<std::mutex> g(alloc_mu_);
  device_bytes_ -= ck_stage_bytes_;
  ck_stage_bytes_ = 0;
}

void Engine::checkpoint_writer() {
  if (!ck_stream_) HIP_OK(hipStreamCreateWithFlags(&ck_stream_, hipStreamNonBlocking));
  void* bounce = nullptr;
  HIP_OK(hipHostMalloc(&bounce, kBounce, hipHostMallocDefault));
  for (;;) {
    std::shared_ptr<CkJob> job;
    {
      std::unique_lock<std::mutex> lk(ck_mu_);
      ck_cv_.wait(lk, [&] { return ck_stop_ || ck_job_ != nullptr; });
      if (ck_stop_ && !ck_job_) break;
      job = ck_job_;
    }
    const double t0 = now_ms();
    uint64_t bytes = 0;
    std::string err;
    try {
      // The sink snapshot first: its flushes' buffers (zero-copy engine text held by the writer
      // lanes) are released once its bytes are written, not after the engine's state file and its
      // fsync -- the engine's double-buffered output text never waits for a checkpoint write.
      // (It only has to be in place before the manifest names this checkpoint: finish_chain.)
      if (job->pre_commit) job->pre_commit();
      HIP_OK(hipEventSynchronize(ck_ev_));
      for (const auto& h : job->holes)  // the deferred small-section reads, into their blob holes
        d2h_bounced(job->blob.p + h[0], d_ck_defer_ + h[1], h[2], ck_stream_, (char*)bounce, kBounce);
      for (const auto& pt : job->patches) std::memcpy(job->blob.p + pt.first, &pt.second, 4);
      BinWriter w(job->path);
      w.raw(job->blob.data(), job->blob.size());
      w.begin(SEC_RING);
      const size_t rb = (size_t)cfg_.ring_bytes;
      if (job->streamed) write_streamed_ring(job, w, (char*)bounce);
      for (const auto& lg : job->lags) {
        if (job->streamed) break;
        w.pod<int32_t>(lg.n_cols);
        w.vec(lg.heads);
        size_t left = (size_t)NSTAT * lg.heads.size() * (size_t)lg.n_cols * rb;
        const char* src = (const char*)d_ck_stage_ + lg.off;
        while (left) {
          const size_t c = std::min(left, kBounce);
          HIP_OK(hipMemcpyAsync(bounce, src, c, hipMemcpyDeviceToHost, ck_stream_));
          HIP_OK(hipStreamSynchronize(ck_stream_));
          w.raw(bounce, c);
          src += c;
          left -= c;
        }
      }
      w.end();
      w.begin(SEC_EXTRA);
      w.str(job->extra);
      w.end();
      w.commit();
      fsync_dir(job->path);
      bytes = w.bytes();
      finish_chain(job, bytes);
    } catch (const std::exception& e) {
      err = e.what();
    }
    if (job->streamed) {  // (also on a failure: rollovers must not wait for a writer that gave up)
      {
        std::lock_guard<std::mutex> lk(cks_mu_);
        cks_.on = false;
        ck_streamed_live_ += cks_.live_rows;
        ck_side_rows_ += cks_.side_rows;
        ck_guard_stalls_ += cks_.stalls;
      }
      cks_cv_.notify_all();
    }
    {
      std::lock_guard<std::mutex> lk(ck_mu_);
      ck_last_write_ms_ = now_ms() - t0;
      if (!err.empty()) {
        ck_error_ = err;
        ck_all_dirty_ = true;  // the chain did not get this increment: restart with a base
      } else {
        ck_last_bytes_ = bytes;
        ++ck_done_;
      }
      ck_blob_spare_ = std::move(job->blob);  // the next snapshot serialises into it
      ck_job_.reset();
      ck_busy_ = false;
    }
    ck_cv_.notify_all();
  }
  hipHostFree(bounce);
}

// Appends a written file to the chain manifest (or starts a new chain with a base) and removes
// the files the new manifest no longer names.
void Engine::finish_chain(const std::shared_ptr<CkJob>& job, uint64_t bytes) {
  (void)bytes;
  const std::string dir = dir_of(job->prefix);
  auto names = [&](const std::string& manifest) {  // file names of a manifest on disk ({} if none)
    std::vector<std::string> v;
    try {
      if (!is_chain_manifest(manifest)) return v;
      for (const auto& p : read_chain(manifest)) v.push_back(p.substr(p.rfind('/') + 1));
    } catch (const std::exception&) {
    }
    return v;
  };
  std::vector<std::string> drop;
  if (job->base) {
    if (!ck_disk_chains_read_) {  // a restarted process: the chains its predecessor left
      ck_disk_chains_read_ = true;
      if (ck_chain_.empty()) ck_chain_ = names(job->prefix + ".ckpt");
      if (ck_prev_chain_.empty()) ck_prev_chain_ = names(job->prefix + ".prev.ckpt");
    }
    // the replaced chain becomes the previous one; the one before it goes
    drop = ck_prev_chain_;
    ck_prev_chain_ = ck_chain_;
    ck_chain_.assign(1, job->name);
    if (!ck_prev_chain_.empty()) {
      std::string prev = "APMCHAIN 1\n";
      for (const auto& f : ck_prev_chain_) prev += f + "\n";
      write_text_atomic(job->prefix + ".prev.ckpt", prev);
    }
  } else {
    ck_chain_.push_back(job->name);
  }
  std::string body = "APMCHAIN 1\n";
  for (const auto& f : ck_chain_) body += f + "\n";
  write_text_atomic(job->prefix + ".ckpt", body);
  for (const auto& f : drop) {
    if (std::find(ck_chain_.begin(), ck_chain_.end(), f) != ck_chain_.end()) continue;
    if (std::find(ck_prev_chain_.begin(), ck_prev_chain_.end(), f) != ck_prev_chain_.end()) continue;
    std::remove((dir + "/" + f).c_str());
  }
}

uint64_t Engine::checkpoint_wait() {
  std::unique_lock<std::mutex> lk(ck_mu_);
  ck_cv_.wait(lk, [&] { return !ck_busy_; });
  if (!ck_error_.empty()) {
    std::string e = ck_error_;
    ck_error_.clear();
    throw std::runtime_error("checkpoint writer: " + e);
  }
  return ck_last_bytes_;
}

void Engine::checkpoint_shutdown() {
  {
    std::lock_guard<std::mutex> lk(ck_mu_);
    ck_stop_ = true;
  }
  ck_cv_.notify_all();
  if (ck_thread_.joinable()) ck_thread_.join();
  if (d_ck_stage_) { hipFree(d_ck_stage_); d_ck_stage_ = nullptr; ck_stage_bytes_ = 0; }
  if (d_ck_defer_) { hipFree(d_ck_defer_); d_ck_defer_ = nullptr; ck_defer_cap_ = 0; }
  if (h_ck_bounce_) { hipHostFree(h_ck_bounce_); h_ck_bounce_ = nullptr; }
  if (ck_ev_) { hipEventDestroy(ck_ev_); ck_ev_ = nullptr; }
  if (ck_side_ev_) { hipEventDestroy(ck_side_ev_); ck_side_ev_ = nullptr; }
  if (ck_stream_) { hipStreamDestroy(ck_stream_); ck_stream_ = nullptr; }
}

CheckpointInfo Engine::checkpoint_info() {
  std::lock_guard<std::mutex> lk(ck_mu_);
  CheckpointInfo c;
  c.busy = ck_busy_;
  c.done = ck_done_;
  c.skipped = ck_skipped_;
  c.sync_fallbacks = ck_sync_fallbacks_;
  c.chain_len = (int)ck_chain_.size();
  c.last_base = ck_last_mode_ == 1;
  c.last_stall_ms = ck_last_stall_ms_;
  c.last_write_ms = ck_last_write_ms_;
  c.last_bytes = ck_last_bytes_;
  c.stage_bytes = ck_stage_bytes_;
  c.last_ring_rows = ck_last_ring_rows_;
  c.last_deferred_bytes = ck_deferred_bytes_;
  c.streamed = ck_streamed_;
  c.streamed_live_rows = ck_streamed_live_;
  c.side_rows = ck_side_rows_;
  c.guard_stalls = ck_guard_stalls_;
  c.stage_cap = cfg_.ck_stage_bytes > 0 ? (uint64_t)cfg_.ck_stage_bytes : 0;
  return c;
}

// Text of `n` pending lines (gids into the HBM ring) in gid order, each with its '\n'.
std::string Engine::ring_text(const int64_t* d_gid, int64_t n) {
  if (n <= 0) return std::string();
  if (apm_dj_gather_plan(d_gid, n, nullptr, d_rel_lens_, d_rel_offs_, d_release_tmp_, release_tmp_bytes_, stream_) != 0)
    throw std::runtime_error("ring_text: scratch too small");
  uint32_t total = 0;
  HIP_OK(hipMemcpyAsync(&total, d_rel_offs_ + n, 4, hipMemcpyDeviceToHost, stream_));
  HIP_OK(hipStreamSynchronize(stream_));
  std::string out(total, '\0');
  if (total) {
    char* d = nullptr;
    HIP_OK(hipMalloc((void**)&d, ((size_t)total + 15) & ~(size_t)15));
    apm_dj_gather_copy(d_gid, n, dj_->ring(), dj_->ring_cap(), d_rel_offs_, d, total, stream_);
    HIP_OK(hipMemcpyAsync(&out[0], d, total, hipMemcpyDeviceToHost, stream_));
    HIP_OK(hipStreamSynchronize(stream_));
    HIP_OK(hipFree(d));
  }
  return out;
}

}  // namespace apm
