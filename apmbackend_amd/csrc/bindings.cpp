// Python bindings for the native runtime (pybind11, no torch headers).
//
//   _apm_native.Engine        -- the GPU pipeline (engine.h)
//   _apm_native.JoinHarness   -- the host join workers alone, fed with Python-built events
//                                (CPU-testable; used by tests/test_join_native.py)
//   _apm_native.js_*          -- JS-exact number formatting helpers (parity tests)
//   _apm_native.Tailer / proc_* / synth_* are registered from their own translation units.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>
#include <memory>

#include "kernels/kernel_api.h"
#include "runtime/engine.h"
#include "runtime/format.h"
#include "runtime/jsutil.h"
#include "runtime/merge.h"

namespace apm {
namespace copyenc {
void encode_blob(std::string_view blob, std::string* out, int64_t* counts);
}
int apm_txcopy_lines(const char* d_text, const uint64_t* h_line_off, int64_t n, std::string& out_rows);  // txcopy.hip
std::vector<double> apm_release_bench(int64_t n, int iters, uint64_t seed);                               // txcopy.hip
}  // namespace apm

namespace py = pybind11;
using namespace apm;

void register_tailer(py::module_& m);
void register_synth(py::module_& m);
void register_procstat(py::module_& m);
void register_dbsink(py::module_& m);

namespace {

template <class T>
T get(const py::dict& d, const char* k, T dflt) {
  if (d.contains(k)) return d[k].cast<T>();
  return dflt;
}

TzTable tz_from(const py::dict& d) {
  TzTable tz{};
  tz.n = 1;
  tz.local_start[0] = INT64_MIN / 2;
  tz.offset_ms[0] = 0;
  if (d.contains("tz_table")) {
    auto rows = d["tz_table"].cast<std::vector<std::pair<int64_t, int64_t>>>();
    tz.n = (int)std::min<size_t>(rows.size(), 64);
    for (int i = 0; i < tz.n; ++i) { tz.local_start[i] = rows[i].first; tz.offset_ms[i] = rows[i].second; }
    if (tz.n == 0) { tz.n = 1; tz.local_start[0] = INT64_MIN / 2; tz.offset_ms[0] = 0; }
  }
  return tz;
}

EngineConfig config_from(const py::dict& d) {
  EngineConfig c;
  c.device = get<int>(d, "device", 0);
  c.max_series = get<int32_t>(d, "max_series", c.max_series);
  c.cell_cap = get<int32_t>(d, "cell_cap", c.cell_cap);
  c.spill_cap = get<int32_t>(d, "spill_cap", c.spill_cap);
  c.max_batch_bytes = get<uint64_t>(d, "max_batch_bytes", c.max_batch_bytes);
  c.max_lines = get<uint32_t>(d, "max_lines", c.max_lines);
  c.max_chunks = get<uint32_t>(d, "max_chunks", c.max_chunks);
  c.pool_cap = get<int64_t>(d, "pool_cap", c.pool_cap);
  c.max_tx_per_batch = get<int32_t>(d, "max_tx_per_batch", c.max_tx_per_batch);
  c.max_alerts = get<int32_t>(d, "max_alerts", c.max_alerts);
  c.ring_bytes = get<int>(d, "ring_bytes", c.ring_bytes);
  c.exact_mean = get<int>(d, "exact_mean", c.exact_mean);
  c.sigma_stddev = get<int>(d, "sigma_stddev", c.sigma_stddev);
  c.resync_k = get<int>(d, "resync_k", c.resync_k);
  c.resync_mfma = get<bool>(d, "resync_mfma", c.resync_mfma);
  c.emulate_aliasing = get<int>(d, "emulate_aliasing", c.emulate_aliasing);
  if (d.contains("lags")) {
    auto lags = d["lags"].cast<std::vector<std::tuple<int, double, double>>>();
    c.n_lags = (int)std::min<size_t>(lags.size(), MAX_LAGS);
    for (int i = 0; i < c.n_lags; ++i) {
      c.lags[i] = std::get<0>(lags[i]);
      c.thr[i] = std::get<1>(lags[i]);
      c.infl[i] = std::get<2>(lags[i]);
    }
  }
  if (d.contains("lag_suppressed")) {
    auto v = d["lag_suppressed"].cast<std::vector<int>>();
    for (size_t i = 0; i < v.size() && i < MAX_LAGS; ++i) c.lag_suppressed[i] = v[i];
  }
  c.alert_window = get<int>(d, "alert_window", c.alert_window);
  c.alert_threshold = get<int>(d, "alert_threshold", c.alert_threshold);
  c.hard_min_ms = get<double>(d, "hard_min_ms", c.hard_min_ms);
  c.hard_min_tpm = get<double>(d, "hard_min_tpm", c.hard_min_tpm);
  c.hard_max_ms = get<double>(d, "hard_max_ms", c.hard_max_ms);
  c.both_only = get<int>(d, "both_only", c.both_only);
  c.cooldown_ms = get<double>(d, "cooldown_ms", c.cooldown_ms);
  c.cooldown_by_service = get<int>(d, "cooldown_by_service", c.cooldown_by_service);
  c.alert_clock_entry = get<int>(d, "alert_clock_entry", c.alert_clock_entry);
  c.interval_len = get<int>(d, "interval_len", c.interval_len);
  c.window = get<int>(d, "window", c.window);
  c.buffer = get<int>(d, "buffer", c.buffer);
  c.nslot = get<int>(d, "nslot", c.nslot);
  c.ck_stage_bytes = get<int64_t>(d, "ck_stage_bytes", c.ck_stage_bytes);
  c.record_ttl_ms = get<double>(d, "record_ttl_ms", c.record_ttl_ms);
  c.acct_ttl_ms = get<double>(d, "acct_ttl_ms", c.acct_ttl_ms);
  c.need_ttl_ms = get<double>(d, "need_ttl_ms", c.need_ttl_ms);
  c.tz = tz_from(d);
  c.join_threads = get<int>(d, "join_threads", c.join_threads);
  c.pin_threads = get<bool>(d, "pin_threads", c.pin_threads);
  c.coll_timeout_ms = get<double>(d, "coll_timeout_ms", c.coll_timeout_ms);
  c.coll_init_timeout_ms = get<double>(d, "coll_init_timeout_ms", c.coll_init_timeout_ms);
  c.node_cooldown = get<int>(d, "node_cooldown", c.node_cooldown);
  c.outputs = get<uint32_t>(d, "outputs", c.outputs);
  c.async_stats = get<int>(d, "async_stats", c.async_stats);
  c.device_join = get<int>(d, "device_join", c.device_join);
  c.join_table_bits = get<int>(d, "join_table_bits", c.join_table_bits);
  c.need_arena = get<uint32_t>(d, "need_arena", c.need_arena);
  c.join_chain_blocks = get<uint32_t>(d, "join_chain_blocks", c.join_chain_blocks);
  c.tx_ring_bytes = get<uint64_t>(d, "tx_ring_bytes", c.tx_ring_bytes);
  c.max_raw_services = get<uint32_t>(d, "max_raw_services", c.max_raw_services);
  return c;
}

ServiceOverride override_from(const py::dict& d) {
  ServiceOverride o;
  if (d.contains("thr")) {
    auto v = d["thr"].cast<std::vector<py::object>>();
    for (size_t i = 0; i < v.size() && i < MAX_LAGS; ++i)
      if (!v[i].is_none()) { o.has_thr[i] = true; o.thr[i] = v[i].cast<double>(); }
  }
  if (d.contains("infl")) {
    auto v = d["infl"].cast<std::vector<py::object>>();
    for (size_t i = 0; i < v.size() && i < MAX_LAGS; ++i)
      if (!v[i].is_none()) { o.has_infl[i] = true; o.infl[i] = v[i].cast<double>(); }
  }
  o.hard_max = get<double>(d, "hard_max", 0.0);
  o.suppressed = get<bool>(d, "suppressed", false);
  return o;
}

std::vector<Chunk> chunks_from(const std::vector<std::tuple<int32_t, uint64_t, uint64_t>>& v) {
  std::vector<Chunk> out;
  out.reserve(v.size());
  for (auto& t : v) out.push_back(Chunk{std::get<0>(t), std::get<1>(t), std::get<2>(t)});
  return out;
}

py::dict metrics_dict(const EngineMetrics& m) {
  py::dict d;
  d["batches"] = m.batches; d["bytes"] = m.bytes; d["lines"] = m.lines; d["events"] = m.events;
  d["tx"] = m.tx; d["tx_db"] = m.tx_db; d["tx_dropped"] = m.tx_dropped; d["rollovers"] = m.rollovers;
  d["alerts"] = m.alerts; d["alert_candidates"] = m.alert_candidates;
  d["alert_candidates_dropped"] = m.alert_candidates_dropped; d["released"] = m.released;
  d["staged_batches"] = m.staged_batches;
  d["t_join_shards_ms"] = m.t_join_shards_ms; d["t_merge_ms"] = m.t_merge_ms;
  d["t_shard_busy_ms"] = m.t_shard_busy_ms; d["t_shard_max_ms"] = m.t_shard_max_ms;
  d["t_out_ms"] = m.t_out_ms;
  d["t_lockstep_ms"] = m.t_lockstep_ms; d["t_lockstep_max_ms"] = m.t_lockstep_max_ms;
  d["t_lockstep_stats_ms"] = m.t_lockstep_stats_ms;
  d["db_copy_rows"] = m.db_copy_rows; d["db_copy_fallbacks"] = m.db_copy_fallbacks;
  d["t_stats_tx_ms"] = m.t_stats_tx_ms; d["t_rollover_ms"] = m.t_rollover_ms;
  d["t_format_ms"] = m.t_format_ms; d["t_release_ms"] = m.t_release_ms;
  d["formatted_bytes"] = m.formatted_bytes; d["lockstep_rollovers"] = m.lockstep_rollovers; d["format_fallbacks"] = m.format_fallbacks;
  d["t_parse_ms"] = m.t_parse_ms; d["t_join_ms"] = m.t_join_ms; d["t_stats_ms"] = m.t_stats_ms;
  d["t_total_ms"] = m.t_total_ms;
  d["series_overflow_tx"] = m.series_overflow_tx;
  d["spill_dropped"] = m.spill_dropped;
  d["nan_windows_clipped"] = m.nan_windows_clipped;
  d["tx_capacity_grows"] = m.tx_capacity_grows;
  d["spill_grows"] = m.spill_grows;
  d["spill_capacity"] = m.spill_capacity;
  d["rollover_latency_ms"] = m.rollover_latency_ms;
  return d;
}

py::dict counters_dict(const JoinCounters& c) {
  py::dict d;
  d["events"] = c.events; d["tx"] = c.tx; d["tx_db"] = c.tx_db; d["expired_partials"] = c.expired_partials;
  d["need_expired"] = c.need_expired; d["ejb_exit_unmatched"] = c.ejb_exit_unmatched;
  d["invalid_acct"] = c.invalid_acct; d["audit_errors"] = c.audit_errors; d["host_fallback"] = c.host_fallback;
  d["partial_overflow"] = c.partial_overflow; d["need_overflow"] = c.need_overflow; d["table_full"] = c.table_full;
  d["pool_exhausted"] = c.pool_exhausted; d["chain_partial_blocks"] = c.chain_partial_blocks;
  d["chain_need_blocks"] = c.chain_need_blocks; d["chain_logid_blocks"] = c.chain_logid_blocks;
  d["table_slots"] = c.table_slots; d["table_grows"] = c.table_grows; d["table_rebuilds"] = c.table_rebuilds; d["trims"] = c.trims;
  d["need_arena_entries"] = c.need_arena_entries; d["arena_grows"] = c.arena_grows;
  d["chain_pool_blocks"] = c.chain_pool_blocks; d["pool_grows"] = c.pool_grows;
  d["host_events"] = c.host_events;
  return d;
}

// Host join alone (CPU): events built by Python (apmbackend_amd.ops.parse_ref) are fed to the
// shards exactly as Engine::process_batch does after the GPU parse.
class JoinHarness {
 public:
  explicit JoinHarness(const py::dict& d) {
    cfg_.record_ttl_ms = get<double>(d, "record_ttl_ms", 120000);
    cfg_.acct_ttl_ms = get<double>(d, "acct_ttl_ms", 120000);
    cfg_.need_ttl_ms = get<double>(d, "need_ttl_ms", 30000);
    cfg_.tz = tz_from(d);
  }
  int32_t add_file(const std::string& path, int kind, const std::string& server) {
    int32_t sid;
    auto it = server_ids_.find(server);
    if (it == server_ids_.end()) {
      sid = (int32_t)servers_.size();
      servers_.push_back(server);
      server_ids_[server] = sid;
      shards_.emplace_back(new JoinShard(cfg_, &dict_, &files_, &servers_));
    } else {
      sid = it->second;
    }
    files_.push_back(FileInfo{path, sid, (uint8_t)kind});
    return (int32_t)files_.size() - 1;
  }
  // events: bytes of packed apm::Event; batch: the batch bytes; chunk_file: chunk -> file id
  std::vector<std::pair<std::string, std::string>> process(py::bytes events, py::bytes batch,
                                                           std::vector<int32_t> chunk_file, double now) {
    std::string ev = events;
    std::string by = batch;
    const Event* e = reinterpret_cast<const Event*>(ev.data());
    const size_t n = ev.size() / sizeof(Event);
    std::vector<std::pair<uint32_t, uint32_t>> range(shards_.size(), {0, 0});
    uint32_t i = 0;
    while (i < n) {
      const int32_t srv = files_[chunk_file[e[i].chunk]].server;
      uint32_t j = i;
      while (j < n && files_[chunk_file[e[j].chunk]].server == srv) ++j;
      range[srv] = {i, j};
      i = j;
    }
    std::vector<std::pair<std::string, std::string>> out;
    std::vector<TxOut> all;
    for (size_t s = 0; s < shards_.size(); ++s) {
      shards_[s]->out().clear();
      shards_[s]->begin_batch(now, batch_no_);
      if (range[s].second > range[s].first)
        shards_[s]->process(e + range[s].first, range[s].second - range[s].first, (const uint8_t*)by.data(),
                            chunk_file);
      for (auto& t : shards_[s]->out()) all.push_back(t);
    }
    std::stable_sort(all.begin(), all.end(), [](const TxOut& a, const TxOut& b) { return a.seq < b.seq; });
    for (auto& t : all)
      out.push_back({t.to_db ? "db_insert" : "transactions", shards_[t.server]->text().substr(t.line_off, t.line_len)});
    ++batch_no_;
    return out;
  }
  py::dict counters() {
    JoinCounters t;
    for (auto& s : shards_) {
      t.events += s->counters.events; t.tx += s->counters.tx; t.need_expired += s->counters.need_expired;
      t.expired_partials += s->counters.expired_partials; t.ejb_exit_unmatched += s->counters.ejb_exit_unmatched;
      t.invalid_acct += s->counters.invalid_acct; t.audit_errors += s->counters.audit_errors;
      t.host_fallback += s->counters.host_fallback; t.tx_db += s->counters.tx_db;
    }
    return counters_dict(t);
  }

 private:
  JoinConfig cfg_;
  Dictionary dict_;
  std::vector<FileInfo> files_;
  std::vector<std::string> servers_;
  std::unordered_map<std::string, int32_t> server_ids_;
  std::vector<std::unique_ptr<JoinShard>> shards_;
  uint64_t batch_no_ = 0;
};

}  // namespace

extern "C" const char* apm_csrc_hash();  // build/native/provenance.cpp (generated at build time)

PYBIND11_MODULE(_apm_native, m) {
  m.doc() = "apm-mi355x native runtime (HIP kernels for gfx950 + host runtime)";
  m.def("csrc_hash", []() { return std::string(apm_csrc_hash()); });
  m.attr("EVENT_SIZE") = (int)sizeof(Event);
  m.def("hash_bytes", [](py::bytes b, uint64_t seed) {
    const std::string s = b;
    return hash_bytes(s.data(), s.size(), seed);
  }, py::arg("data"), py::arg("seed") = kHashSeed);
  m.attr("NSLOT_MIN") = NSLOT_MIN;
  m.attr("MAX_LAGS") = MAX_LAGS;

  // TCP host transport on host buffers (CPU tests of the multi-process collective path)
  py::class_<Collective>(m, "HostCollective")
      .def(py::init([](const std::string& addr, int port, int n, int rank, double timeout_ms) {
             py::gil_scoped_release rel;
             return make_host_collective(addr, port, n, rank, timeout_ms).release();
           }),
           py::arg("addr"), py::arg("port"), py::arg("nranks"), py::arg("rank"), py::arg("timeout_ms") = 30000.0)
      .def("all_reduce", [](Collective& c, std::vector<double> v, bool max) {
        py::gil_scoped_release rel;
        return c.all_reduce_host(v, max);
      }, py::arg("values"), py::arg("max") = false)
      .def("all_gather", [](Collective& c, py::bytes b) {
        std::string s = b;
        std::vector<uint8_t> v(s.begin(), s.end()), out;
        { py::gil_scoped_release rel; out = c.all_gather_host(v); }
        return py::bytes((const char*)out.data(), out.size());
      })
      .def("abort", &Collective::abort)
      .def("aborted", &Collective::aborted)
      .def_property_readonly("rank", &Collective::rank)
      .def_property_readonly("nranks", &Collective::nranks);
  py::class_<LocalGroup, std::shared_ptr<LocalGroup>>(m, "LocalCollGroup")
      .def(py::init([](int n, double timeout_ms) { return make_local_group(n, timeout_ms); }), py::arg("n"),
           py::arg("timeout_ms") = 120000.0);

  py::class_<Engine>(m, "Engine")
      .def(py::init([](const py::dict& d) { return new Engine(config_from(d)); }))
      .def("add_file", &Engine::add_file)
      .def("add_server", &Engine::add_server)
      .def("set_override", [](Engine& e, const std::string& svc, const py::dict& d) { e.set_override(svc, override_from(d)); })
      .def("clear_overrides", &Engine::clear_overrides)
      .def("refresh_series_settings", &Engine::refresh_series_settings)
      .def("stage_reconfig", [](Engine& e, const py::dict& ecfg, const py::dict& overrides, uint64_t gen) {
        const EngineConfig c = config_from(ecfg);
        ReconfigSpec r;
        r.gen = gen;
        r.n_lags = c.n_lags;
        for (int l = 0; l < MAX_LAGS; ++l) {
          r.lags[l] = c.lags[l]; r.thr[l] = c.thr[l]; r.infl[l] = c.infl[l]; r.lag_suppressed[l] = c.lag_suppressed[l];
        }
        r.alert_window = c.alert_window; r.alert_threshold = c.alert_threshold; r.both_only = c.both_only;
        r.hard_min_ms = c.hard_min_ms; r.hard_min_tpm = c.hard_min_tpm; r.hard_max_ms = c.hard_max_ms;
        r.cooldown_ms = c.cooldown_ms;
        r.interval_len = c.interval_len; r.window = c.window; r.buffer = c.buffer;
        for (auto kv : overrides) r.overrides[kv.first.cast<std::string>()] = override_from(kv.second.cast<py::dict>());
        e.stage_reconfig(r);
      }, py::arg("ecfg"), py::arg("overrides"), py::arg("gen"))
      .def("reconfig_info", [](Engine& e) {
        py::dict d;
        d["applied_gen"] = e.reconfig_applied_gen(); d["applied"] = e.reconfigs_applied();
        d["lag_set_changes"] = e.lag_set_changes();
        d["window_changes"] = e.window_changes();
        d["ring_slots"] = e.ring_slots();
        d["ring_grows"] = e.ring_grows();
        return d;
      })
      .def("lag_values", &Engine::lag_values)
      .def("cache_stats", [](Engine& e, bool drain) {
        std::vector<uint64_t> v;
        { py::gil_scoped_release rel; v = e.cache_stats(drain); }
        py::dict d;
        if (v.size() == 6) {
          d["slots"] = v[0]; d["occupied"] = v[1]; d["acct"] = v[2]; d["record"] = v[3]; d["partials"] = v[4];
          d["need"] = v[5];
        }
        return d;
      }, py::arg("drain") = true)
      .def("process_batch",
           [](Engine& e, py::buffer buf, const std::vector<std::tuple<int32_t, uint64_t, uint64_t>>& chunks,
              double now) {
             py::buffer_info bi = buf.request();
             const uint8_t* p = (const uint8_t*)bi.ptr;
             const uint64_t n = (uint64_t)(bi.size * bi.itemsize);
             auto ch = chunks_from(chunks);
             py::gil_scoped_release rel;
             e.process_batch(p, n, ch, now);
           },
           py::arg("buf"), py::arg("chunks"), py::arg("now") = -1.0)
      .def("process_batch_ptr",
           [](Engine& e, uintptr_t ptr, uint64_t n, const std::vector<std::tuple<int32_t, uint64_t, uint64_t>>& chunks,
              double now, uintptr_t next_ptr, uint64_t next_n,
              const std::vector<std::tuple<int32_t, uint64_t, uint64_t>>& next_chunks) {
             auto ch = chunks_from(chunks);
             auto nch = chunks_from(next_chunks);
             py::gil_scoped_release rel;
             e.process_batch((const uint8_t*)ptr, n, ch, now, next_ptr ? (const uint8_t*)next_ptr : nullptr, next_n,
                             next_ptr ? &nch : nullptr);
           },
           py::arg("ptr"), py::arg("n"), py::arg("chunks"), py::arg("now") = -1.0, py::arg("next_ptr") = 0,
           py::arg("next_n") = 0,
           py::arg("next_chunks") = std::vector<std::tuple<int32_t, uint64_t, uint64_t>>())
      .def("stage_batch_ptr",
           [](Engine& e, uintptr_t ptr, uint64_t n) {
             py::gil_scoped_release rel;
             e.stage_batch((const uint8_t*)ptr, n);
           },
           py::arg("ptr"), py::arg("n"))
      .def("process_tx_lines", [](Engine& e, py::bytes b, double now) {
             std::string v = b;
             py::gil_scoped_release rel;
             e.process_tx_lines(v, now);
           }, py::arg("blob"), py::arg("now") = -1.0)
      .def("take", &Engine::take, py::call_guard<py::gil_scoped_release>())
      .def("flush", &Engine::flush, py::call_guard<py::gil_scoped_release>())
      .def("dump_state", [](Engine& e, const std::string& path, const std::string& reason) {
        py::gil_scoped_release rel;
        return e.dump_state(path, reason);
      })
      .def("save_state", [](Engine& e, const std::string& path, py::bytes extra) {
             std::string x = extra;
             py::gil_scoped_release rel;
             return e.save_state(path, x);
           }, py::arg("path"), py::arg("extra") = py::bytes(""))
      .def("checkpoint_async", [](Engine& e, const std::string& prefix, py::bytes extra, bool force_base) {
             std::string x = extra;
             py::gil_scoped_release rel;
             return e.checkpoint_async(prefix, x, force_base);
           }, py::arg("prefix"), py::arg("extra") = py::bytes(""), py::arg("force_base") = false)
      .def("checkpoint_wait", &Engine::checkpoint_wait, py::call_guard<py::gil_scoped_release>())
      .def("checkpoint_info", [](Engine& e) {
        const CheckpointInfo c = e.checkpoint_info();
        py::dict d;
        d["busy"] = c.busy; d["done"] = c.done; d["skipped"] = c.skipped; d["sync_fallbacks"] = c.sync_fallbacks;
        d["chain_len"] = c.chain_len; d["last_base"] = c.last_base; d["last_stall_ms"] = c.last_stall_ms;
        d["last_write_ms"] = c.last_write_ms; d["last_bytes"] = c.last_bytes; d["stage_bytes"] = c.stage_bytes;
        d["last_deferred_bytes"] = c.last_deferred_bytes;
        d["streamed"] = c.streamed; d["streamed_live_rows"] = c.streamed_live_rows;
        d["side_rows"] = c.side_rows; d["guard_stalls"] = c.guard_stalls; d["stage_cap"] = c.stage_cap;
        d["last_ring_rows"] = c.last_ring_rows;
        return d;
      })
      .def("export_series", &Engine::export_series, py::call_guard<py::gil_scoped_release>())
      .def("import_series", &Engine::import_series, py::call_guard<py::gil_scoped_release>())
      .def("export_buckets", [](Engine& e) {
        BucketDump d;
        { py::gil_scoped_release rel; d = e.export_buckets(); }
        return py::make_tuple(d.latest, d.series, d.bucket, d.count, d.values);
      })
      .def("import_buckets", &Engine::import_buckets, py::call_guard<py::gil_scoped_release>())
      .def("export_history", [](Engine& e, int lag_idx, int32_t lo, int32_t hi) {
        std::vector<int32_t> len;
        std::vector<double> vals;
        { py::gil_scoped_release rel; e.export_history(lag_idx, lo, hi, len, vals); }
        return py::make_tuple(len, py::bytes((const char*)vals.data(), vals.size() * 8));
      })
      .def("import_history", [](Engine& e, int lag_idx, const std::vector<int32_t>& series,
                                const std::vector<int32_t>& len, py::bytes vals) {
        std::string b = vals;
        std::vector<double> v(b.size() / 8);
        std::memcpy(v.data(), b.data(), v.size() * 8);
        py::gil_scoped_release rel;
        e.import_history(lag_idx, series, len, v);
      })
      .def("export_lag_settings", &Engine::export_lag_settings)
      .def("export_pending", &Engine::export_pending, py::call_guard<py::gil_scoped_release>())
      .def("import_pending", &Engine::import_pending, py::call_guard<py::gil_scoped_release>())
      .def("export_cooldowns", &Engine::export_cooldowns)
      .def("import_cooldowns", &Engine::import_cooldowns)
      .def("export_alert_counters", &Engine::export_alert_counters)
      .def("import_alert_counters", &Engine::import_alert_counters)
      .def("cooldown_by_service", &Engine::cooldown_by_service)
      .def("set_trace", &Engine::set_trace)
      .def("take_trace", [](Engine& e) {
        std::vector<TraceEvent> t;
        { py::gil_scoped_release rel; t = e.take_trace(); }
        py::list out;
        for (auto& x : t) out.append(py::make_tuple(std::string(x.name), x.t0_ms, x.t1_ms, x.tid, x.batch));
        return out;
      })
      .def("set_server_context", &Engine::set_server_context, py::arg("server"), py::arg("ts_ms"),
           py::arg("gauges"), py::arg("host_load") = 0.0)
      .def("load_state", [](Engine& e, const std::string& path) {
             std::string x;
             { py::gil_scoped_release rel; x = e.load_state(path); }
             return py::bytes(x);
           })
      .def("take_bytes", [](Engine& e, const std::string& k) {
        std::string b;
        { py::gil_scoped_release rel; b = e.take_bytes(k); }
        return py::bytes(b);
      })
      .def("set_sink_fd", &Engine::set_sink_fd, py::call_guard<py::gil_scoped_release>())
      .def("set_fs_copy", &Engine::set_fs_copy, py::call_guard<py::gil_scoped_release>())
      .def("set_db_copy", &Engine::set_db_copy, py::call_guard<py::gil_scoped_release>())
      .def("sink_bytes", &Engine::sink_bytes)
      .def("lane_cpus", &Engine::lane_cpus)
      .def("last_events", [](Engine& e) { return py::bytes(e.last_events()); })
      .def("warm_history", &Engine::warm_history)
      .def("metrics", [](Engine& e, bool drain) {
        // drain=False: the counters as they stand (a batch or two behind), without draining the
        // pipeline -- the periodic stat lines must not stall ingest
        EngineMetrics m;
        { py::gil_scoped_release rel; m = drain ? e.metrics() : e.metrics_nowait(); }
        return metrics_dict(m);
      }, py::arg("drain") = true)
      .def("join_counters", [](Engine& e) { return counters_dict(e.join_counters()); })
      .def("n_series", &Engine::n_series)
      .def("n_services", &Engine::n_services)
      .def("services", &Engine::services)
      .def("files", [](Engine& e) {
        std::vector<std::tuple<std::string, int, std::string>> r;
        for (auto& f : e.files()) r.emplace_back(f.path, (int)f.kind, e.servers()[f.server]);
        return r;
      })
      .def("servers", &Engine::servers)
      .def("watermark", &Engine::watermark)
      .def("batch_no", &Engine::batch_no)
      .def("device_bytes", &Engine::device_bytes)
      .def("trim_device_memory", &Engine::trim_device_memory, py::call_guard<py::gil_scoped_release>())
      .def("stream_handle", [](Engine& e) { return (uintptr_t)e.stream(); })
      .def("comm_stream_handle", [](Engine& e) { return (uintptr_t)e.comm_stream(); })
      .def_static("fleet_unique_id", []() {
        auto v = Engine::fleet_unique_id();
        return py::bytes((const char*)v.data(), v.size());
      })
      .def("fleet_init", [](Engine& e, py::bytes uid, int nranks, int rank, int32_t cap, py::bytes clock_uid) {
        std::string s = uid, c = clock_uid;
        std::vector<uint8_t> v(s.begin(), s.end()), cv(c.begin(), c.end());
        py::gil_scoped_release rel;
        e.fleet_init(v, cv, nranks, rank, cap);
      }, py::arg("uid"), py::arg("nranks"), py::arg("rank"), py::arg("cap"), py::arg("clock_uid") = py::bytes(""))
      .def("fleet_merged", [](Engine& e) {
        std::vector<double> v;
        { py::gil_scoped_release rel; v = e.fleet_merged(); }
        return py::bytes((const char*)v.data(), v.size() * 8);
      })
      .def("fleet_rounds", &Engine::fleet_rounds)
      .def("gram_tail_series", [](Engine& e) { return e.last_gram_tail_; })
      .def("node_metrics", &Engine::node_metrics)
      .def("fleet_slot_names", [](Engine& e) { return e.fleet_slot_names(); })
      .def("fleet_info", [](Engine& e) {
        py::dict d;
        const auto i = e.fleet_info();
        d["slots"] = i[0]; d["registry_rounds"] = i[1]; d["registry_overflow"] = i[2]; d["fb_rows"] = i[3]; d["nranks"] = i[4];
        return d;
      })
      .def("fleet_init_local", [](Engine& e, std::shared_ptr<LocalGroup> g, int rank, int32_t cap, bool lockstep) {
        py::gil_scoped_release rel;
        e.fleet_init_local(std::move(g), rank, cap, lockstep);
      }, py::arg("group"), py::arg("rank"), py::arg("cap"), py::arg("lockstep") = true)
      .def("fleet_init_host", [](Engine& e, const std::string& addr, int port, int nranks, int rank, int32_t cap,
                                 bool lockstep) {
        py::gil_scoped_release rel;
        e.fleet_init_host(addr, port, nranks, rank, cap, lockstep);
      }, py::arg("addr"), py::arg("port"), py::arg("nranks"), py::arg("rank"), py::arg("cap"), py::arg("lockstep") = true)
      .def("set_server_index", &Engine::set_server_index)
      .def("node_drain", [](Engine& e) { py::gil_scoped_release rel; e.node_drain(); })
      .def("pack_service_moments", [](Engine& e, uintptr_t dst, int32_t cap, bool atomic_path) {
        e.pack_service_moments((double*)dst, cap, e.comm_stream(), atomic_path);
      }, py::arg("dst"), py::arg("cap"), py::arg("atomic_path") = false)
      .def("winstats", [](Engine& e) {
        std::vector<WinStat> w;
        e.download_winstats(w);
        std::vector<std::tuple<int, int, double, double, double, double>> out;
        for (int i = 0; i < e.n_series(); ++i) out.emplace_back(w[i].active, w[i].n, w[i].tpm, w[i].avg, w[i].p75, w[i].p95);
        return out;
      });

  py::class_<JoinHarness>(m, "JoinHarness")
      .def(py::init<const py::dict&>())
      .def("add_file", &JoinHarness::add_file)
      .def("process", &JoinHarness::process)
      .def("counters", &JoinHarness::counters);

  m.def("alloc_pinned", &Engine::alloc_pinned);
  // re-shard merge of old ranks' checkpoints (runtime/merge.h), host only
  m.def("checkpoint_batches", &checkpoint_batches, py::arg("path"));
  m.def("merge_checkpoints", [](const std::vector<std::string>& inputs, const std::vector<std::string>& servers,
                                const std::string& out, const py::bytes& extra, uint64_t batch_no) {
    MergeResult r;
    const std::string ex = extra;
    {
      py::gil_scoped_release rel;
      r = merge_checkpoints(inputs, servers, out, ex, batch_no);
    }
    py::dict d;
    d["batch_no"] = r.batch_no; d["series"] = r.series; d["keys"] = r.keys; d["need"] = r.need;
    d["pending"] = r.pending; d["raw"] = r.raw; d["files"] = r.files; d["servers"] = r.servers;
    d["used"] = r.used;
    py::list ex_l;
    for (const auto& e : r.extras) ex_l.append(py::bytes(e));
    d["extras"] = ex_l;
    return d;
  }, py::arg("inputs"), py::arg("servers"), py::arg("out"), py::arg("extra") = py::bytes(""), py::arg("batch_no") = 0);
  m.def("free_pinned", &Engine::free_pinned);
  m.def("memcpy_to", [](uintptr_t dst, py::bytes b, uint64_t off) {
    std::string_view v = b;
    std::memcpy((char*)dst + off, v.data(), v.size());
  });
  m.def("copy_encode", [](py::bytes blob) {
    // wire lines -> Postgres COPY text per table type (runtime/sinks.py is the Python twin)
    std::string b = blob;
    std::string out[5];
    int64_t counts[5] = {0, 0, 0, 0, 0};
    {
      py::gil_scoped_release rel;
      copyenc::encode_blob(b, out, counts);
    }
    py::dict d;
    const char* names[5] = {"tx", "fs", "al", "jx", "fb"};
    for (int k = 0; k < 5; ++k) d[names[k]] = py::make_tuple(py::bytes(out[k]), counts[k]);
    return d;
  });
  m.def("set_blocking_sync", [](int device) {
    // before anything else creates the device's runtime state (bench.py, ranks sharing a GPU):
    // stream / event waits block instead of spinning
    HIP_OK(hipSetDevice(device));
    return hipSetDeviceFlags(hipDeviceScheduleBlockingSync) == hipSuccess;
  });
  m.def("release_bench", [](int64_t n, int iters, uint64_t seed) {
    std::vector<double> r;
    {
      py::gil_scoped_release rel;
      r = apm_release_bench(n, iters, seed);
    }
    py::dict d;
    const char* k[7] = {"lines", "wire_bytes", "copy_bytes", "gather_us", "txcopy_us", "txcopy_write_us", "fallbacks"};
    for (int i = 0; i < 7; ++i) d[k[i]] = r[(size_t)i];
    return d;
  }, py::arg("n") = 60000, py::arg("iters") = 20, py::arg("seed") = 1);
  m.def("dj_rebuild_selftest", [](uint32_t cap, double load, double dead, uint64_t seed, bool copy) {
    std::vector<double> r;
    {
      py::gil_scoped_release rel;
      r = apm_dj_rebuild_selftest(cap, load, dead, seed, copy);
    }
    py::dict d;
    const char* k[8] = {"live", "want_live", "found", "dead_left", "occupied", "probes_before", "probes_after", "us"};
    for (int i = 0; i < 8; ++i) d[k[i]] = r[(size_t)i];
    return d;
  }, py::arg("cap"), py::arg("load") = 0.55, py::arg("dead") = 0.3, py::arg("seed") = 1, py::arg("copy") = false);
  m.def("txcopy_lines", [](py::bytes blob) {
    // newline-terminated wire tx lines -> (COPY rows from the GPU encoder, fallback count)
    std::string b = blob;
    std::vector<uint64_t> off{0};
    for (size_t i = 0; i < b.size(); ++i)
      if (b[i] == '\n') off.push_back(i + 1);
    if (off.back() != b.size()) throw std::invalid_argument("txcopy_lines: the last line needs its newline");
    const int64_t n = (int64_t)off.size() - 1;
    std::string rows;
    int fb = 0;
    {
      py::gil_scoped_release rel;
      uint64_t cap = 1;
      while (cap < b.size() + 64) cap <<= 1;
      char* d = nullptr;
      HIP_OK(hipMalloc(&d, cap));
      HIP_OK(hipMemset(d, 0, cap));
      HIP_OK(hipMemcpy(d, b.data(), b.size(), hipMemcpyHostToDevice));
      fb = n ? apm_txcopy_lines(d, off.data(), n, rows) : 0;
      HIP_OK(hipFree(d));
    }
    return py::make_tuple(py::bytes(rows), fb);
  });
  m.def("flatmap_selftest", [](int n_ops, uint64_t seed, int key_space) {
    // randomized FlatMap / SmallVec vs std containers (CPU test of the join's data structures)
    FlatMap<int64_t> fm(16);
    std::unordered_map<uint64_t, int64_t> ref;
    uint64_t x = seed | 1;
    auto rnd = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; };
    for (int i = 0; i < n_ops; ++i) {
      const uint64_t k = 1 + rnd() % (uint64_t)key_space;
      const int op = (int)(rnd() % 3);
      if (op == 0) { fm[k] = (int64_t)i; ref[k] = i; }
      else if (op == 1) { if (fm.erase(k) != (ref.erase(k) == 1)) return false; }
      else {
        int64_t* v = fm.find(k);
        auto it = ref.find(k);
        if ((v != nullptr) != (it != ref.end())) return false;
        if (v && *v != it->second) return false;
      }
      if (fm.size() != ref.size()) return false;
    }
    SmallVec<int, 2> sv;
    std::vector<int> rv;
    for (int i = 0; i < 2000; ++i) {
      if (rnd() % 3 || rv.empty()) { sv.push_back(i); rv.push_back(i); }
      else {
        const size_t j = rnd() % rv.size();
        sv.erase(sv.begin() + j);
        rv.erase(rv.begin() + j);
      }
      if (sv.size() != rv.size() || !std::equal(rv.begin(), rv.end(), sv.begin())) return false;
    }
    return true;
  });
  m.def("gpu_to_fixed", [](const std::vector<double>& xs, int f) {
    // K12 number printer on the device (test hook): nf(x, f) per value
    const int n = (int)xs.size();
    double* dx = nullptr;
    char* dout = nullptr;
    std::vector<char> h((size_t)n * 32);
    HIP_OK(hipMalloc(&dx, std::max(1, n) * 8));
    HIP_OK(hipMalloc(&dout, std::max<size_t>(32, h.size())));
    HIP_OK(hipMemcpy(dx, xs.data(), (size_t)n * 8, hipMemcpyHostToDevice));
    apm_format_fixed_batch(dx, n, f, dout, 0);
    HIP_OK(hipMemcpy(h.data(), dout, h.size(), hipMemcpyDeviceToHost));
    HIP_OK(hipFree(dx));
    HIP_OK(hipFree(dout));
    std::vector<std::string> r;
    for (int i = 0; i < n; ++i) r.emplace_back(h.data() + (size_t)i * 32);
    return r;
  });
  m.def("js_to_fixed", [](double x, int f) { return js::to_fixed(x, f); });
  m.def("js_num_str", [](double x) { return js::num_str(x); });
  m.def("js_parse_int", [](const std::string& s) { return js::parse_int(s); });
  m.def("js_convert_date", [](const std::string& s, const py::dict& tz) {
    double v;
    TzTable t = tz_from(tz);
    if (!js::convert_date(s, t, v)) return py::object(py::none());
    return py::object(py::float_(v));
  });
  m.def("js_round_fixed", [](double x, int f) { return js_round_fixed(x, f); });

  register_tailer(m);
  register_synth(m);
  register_procstat(m);
  register_dbsink(m);
}
