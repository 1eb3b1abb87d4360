// apm::Engine -- one MI355X-resident APM pipeline (one process per GPU).
//
//   host batch (pinned) --H2D--> K1/K2 parse (GPU) --D2H events--> join workers (host, per JVM)
//   --tx--> K7 bucket append / rollover: K8 window stats -> K10 z-score (per LAG) -> K11 alert
//   eval (GPU) --D2H alert candidates--> cooldown + sinks (host).  K9 keeps the released-tx pool
//   sorted by endTs on the GPU.
//
// The engine is the fused equivalent of the reference's five stage processes
// (stream_parse_transactions -> stream_calc_stats -> stream_calc_z_score ->
// stream_process_alerts -> stream_insert_db) with the RabbitMQ hops replaced by device buffers.
#pragma once
#include <hip/hip_runtime.h>

#include "binio.h"

#include <array>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../apm_types.h"
#include "../kernels/kernel_api.h"
#include "collective.h"
#include "devjoin.h"
#include "join.h"

namespace apm {

constexpr int64_t NO_BUCKET = INT64_MIN;  // empty bucket slot

struct ServiceOverride {
  bool has_thr[MAX_LAGS] = {false, false, false, false};
  bool has_infl[MAX_LAGS] = {false, false, false, false};
  double thr[MAX_LAGS] = {0, 0, 0, 0};
  double infl[MAX_LAGS] = {0, 0, 0, 0};
  double hard_max = 0;  // 0 = use default (the reference ignores falsy overrides)
  bool suppressed = false;
};

// A config reload as the engine applies it (reconfig.cpp): the new LAG set with its default
// THRESHOLD / INFLUENCE / suppression, the alert gates, and the per-service override table (LAG
// positions in the new order).  `gen` orders reloads (the config file's mtime in ms).
struct ReconfigSpec {
  uint64_t gen = 0;
  int n_lags = 0;
  int32_t lags[MAX_LAGS] = {0, 0, 0, 0};
  double thr[MAX_LAGS] = {0, 0, 0, 0};
  double infl[MAX_LAGS] = {0, 0, 0, 0};
  int lag_suppressed[MAX_LAGS] = {0, 0, 0, 0};
  int alert_window = 60, alert_threshold = 45, both_only = 1;
  double hard_min_ms = 200, hard_min_tpm = 1.0, hard_max_ms = 10000, cooldown_ms = 15 * 60000.0;
  int interval_len = 10, window = 30, buffer = 6;  // streamCalcStats (live: the next rollover on)
  std::map<std::string, ServiceOverride> overrides;
};

// Bounds of a stats window: window >= 1, buffer >= 0, interval >= 1 (the reference's are the
// same); removeOldBuckets keeps window + buffer buckets, so the bucket ring needs window + buffer
// + 1 slots -- it is sized for the configured window and grows on a reload to a longer one.
void check_window(int window, int buffer, int interval_len);
int32_t ring_slots_for(int window, int buffer);  // max(NSLOT_MIN, window + buffer + 1)

struct EngineConfig {
  int device = 0;
  int32_t max_series = 1 << 17;
  int32_t cell_cap = 16;
  int32_t spill_cap = 1 << 20;
  uint64_t max_batch_bytes = 64ull << 20;
  uint32_t max_lines = 1u << 21;
  uint32_t max_chunks = 4096;
  int64_t pool_cap = 1 << 23;
  int32_t max_tx_per_batch = 1 << 21;
  int32_t max_alerts = 1 << 16;
  int ring_bytes = 8;            // 8 = float64, 4 = float32, 2 = bfloat16
  int exact_mean = 0;
  int sigma_stddev = 0;
  int resync_k = 360;
  bool resync_mfma = false;  // rolling-mode window re-sum on the matrix cores (gpu.resyncOnMatrixCores; the VALU form is faster: profiles/r6_l)
  int n_lags = 2;
  int32_t lags[MAX_LAGS] = {360, 8640, 0, 0};
  double thr[MAX_LAGS] = {20.0, 15.0, 0, 0};
  double infl[MAX_LAGS] = {0.1, 0.0, 0, 0};
  int emulate_aliasing = 0;
  // alerts (streamProcessAlerts)
  int alert_window = 60;
  int alert_threshold = 45;
  double hard_min_ms = 200;
  double hard_min_tpm = 1.0;
  double hard_max_ms = 10000;
  int both_only = 1;
  int lag_suppressed[MAX_LAGS] = {0, 0, 0, 0};
  double cooldown_ms = 15 * 60000.0;
  int cooldown_by_service = 1;
  int alert_clock_entry = 1;
  // stats (streamCalcStats)
  int interval_len = 10;
  int window = 30;
  int buffer = 6;
  int nslot = 0;  // bucket ring slots (gpu.bucketRingSlots; 0 = ring_slots_for(window, buffer))
  int64_t ck_stage_bytes = (int64_t)2048 << 20;  // HBM staging of a snapshot's ring rows (gpu.checkpointStageMB; 0 = unbounded)
  // parse
  double record_ttl_ms = 120000, acct_ttl_ms = 120000, need_ttl_ms = 30000;
  TzTable tz{};
  int join_threads = 0;
  bool pin_threads = false;  // pin host lanes to GPU-local physical cores (APM_PIN_THREADS overrides)
  // outputs: bit k of `outputs` materialises stream k (OutKind) in the reference wire format
  uint32_t outputs = 0;
  int async_stats = 1;      // overlap batch i's stats with batch i+1's parse + join
  // RCCL watchdog: a collective not complete after this long (a dead or wedged peer) aborts the
  // communicator and throws, so the supervisor restarts the rank group from its checkpoint
  double coll_timeout_ms = 300000;
  double coll_init_timeout_ms = 120000;  // RCCL communicator init deadline (fail fast, no silent hang)
  // lock-step ranks resolve the per-service alert cooldown node-wide: alert candidates are
  // all-gathered and decided in the global emission order (engine.cpp, "node-wide cooldown")
  int node_cooldown = 1;
  // K4/K6 on the GPU (devjoin.hip); 0 = host join workers (join.cpp)
  int device_join = 1;
  int join_table_bits = 21;          // key-table slots (128 B each)
  uint32_t need_arena = 1u << 18;    // needNumRecordCache entries (512 B each)
  uint32_t join_chain_blocks = 0;    // initial chain-block pool of the GPU join (256 B each; 0 = auto)
  uint64_t tx_ring_bytes = 4ull << 30;  // HBM text ring of pending (unreleased) tx lines
  uint32_t max_raw_services = 1u << 20;
};

// Output streams (queue names of the reference, config/apm_config.json:12,87,99-100,113-114,178):
//   TRANSACTIONS  parse -> stats  tx lines   (only for the AMQP bridge; fused internally)
//   AUDIT_DB      parse -> db     tx lines of audit non-Provider records (Q18)
//   DB            stats -> db     released tx lines in endTs order (K9)
//   ST            stats -> z      st lines  (fused internally; bridge only)
//   FS            z -> alerts/db  fs lines (one per series per LAG)
//   AL            alerts -> db    al lines
//   SX            new: per-JVM rollup fused with JMX / VM gauges (K14), one line per server
enum OutKind { OUT_TRANSACTIONS = 0, OUT_AUDIT_DB, OUT_DB, OUT_ST, OUT_FS, OUT_AL, OUT_SX, OUT_FB, N_OUT };
// streams written by the engine's output lane (released tx, st, fs); the stats thread owns the rest
constexpr uint32_t kLaneKinds = (1u << OUT_DB) | (1u << OUT_ST) | (1u << OUT_FS);
const char* out_kind_name(int k);
int out_kind_of(const std::string& name);

// Live bucket contents for the reference resume exporter: (series, bucket, count) rows and
// the concatenated elapsed values.
struct BucketDump {
  int64_t latest = 0;
  std::vector<int32_t> series;
  std::vector<int64_t> bucket;
  std::vector<int32_t> count;
  std::vector<int32_t> values;
};

// One stage interval of the pipeline (Chrome-trace "X" event); tid 0 = ingest, 1 = stats.
struct TraceEvent {
  const char* name;
  double t0_ms, t1_ms;
  int tid;
  uint64_t batch;
};

struct Chunk {
  int32_t file;
  uint64_t begin, end;  // byte range in the batch (must end with '\n')
};

// In-process consumer of an output stream (runtime/dbsink.cpp DbSink).
struct ByteSink {
  virtual ~ByteSink() = default;
  virtual void write_bytes(int kind, const char* p, size_t n) = 0;
  // [p, p + n) stays valid and unchanged until `hold` is released: a sink may keep references
  // instead of copying (default: copy)
  virtual void write_bytes_held(int kind, const char* p, size_t n, std::shared_ptr<const void> hold) {
    (void)hold;
    write_bytes(kind, p, n);
  }
  // Same, with the row boundaries known: row r is [row_off[r], row_off[r + 1]) (nrows + 1
  // entries, row_off[nrows] == n; empty rows allowed).  row_off is only read during the call.
  virtual void write_rows_held(int kind, const char* p, size_t n, const uint32_t* row_off, size_t nrows,
                               std::shared_ptr<const void> hold) {
    (void)row_off;
    (void)nrows;
    write_bytes_held(kind, p, n, std::move(hold));
  }
};

struct CheckpointInfo {
  bool busy = false;
  uint64_t done = 0, skipped = 0, sync_fallbacks = 0;
  int chain_len = 0;
  bool last_base = false;
  double last_stall_ms = 0, last_write_ms = 0;
  uint64_t last_bytes = 0, stage_bytes = 0;
  int64_t last_ring_rows = 0;  // ring rows (over all LAGs) the last checkpoint carried
  uint64_t last_deferred_bytes = 0;  // small-section bytes the last snapshot read D2D (not on the ingest thread)
  // streamed bases (ring larger than gpu.checkpointStageMB): rows read from the live ring by the
  // writer, rows a rollover copied aside first, rollovers that waited for the writer
  uint64_t streamed = 0, streamed_live_rows = 0, side_rows = 0, guard_stalls = 0;
  uint64_t stage_cap = 0;
};

struct EngineMetrics {
  uint64_t batches = 0, bytes = 0, lines = 0, events = 0, tx = 0, tx_db = 0, tx_dropped = 0;
  uint64_t rollovers = 0, alerts = 0, alert_candidates = 0, series = 0, released = 0;
  uint64_t staged_batches = 0;      // parses whose input was already on the device (stage_batch)
  uint64_t alert_candidates_dropped = 0;  // beyond maxAlertCandidates in one rollover (reported)
  uint64_t formatted_bytes = 0, format_fallbacks = 0, lockstep_rollovers = 0;
  uint64_t series_overflow_tx = 0;  // tx whose series could not be created (gpu.maxSeries full)
  uint64_t spill_dropped = 0;       // samples lost to a full bucket spill list (gpu.bucketOverflowCapacity)
  uint64_t nan_windows_clipped = 0; // NaN windows larger than the JS-emulation scratch (percentiles clipped)
  uint64_t tx_capacity_grows = 0;   // per-batch tx staging doubled (instead of failing the batch)
  uint64_t spill_grows = 0;         // bucket spill lists grown (instead of dropping window samples)
  int64_t spill_capacity = 0;       // spill entries per bucket slot (current)
  double t_parse_ms = 0, t_join_ms = 0, t_stats_ms = 0, t_total_ms = 0;
  double t_join_shards_ms = 0, t_merge_ms = 0;                 // split of t_join_ms
  double t_shard_busy_ms = 0, t_shard_max_ms = 0;              // per batch: mean / max of one shard's join
  double t_stats_tx_ms = 0, t_rollover_ms = 0, t_format_ms = 0, t_release_ms = 0;  // inside t_stats_ms
  double t_out_ms = 0;                        // output lane: released-line gather + st/fs emission
  uint64_t db_copy_rows = 0, db_copy_fallbacks = 0;  // released db rows encoded on the GPU / releases encoded on the host
  double t_lockstep_ms = 0, t_lockstep_max_ms = 0;  // ingest thread in the per-batch lock-step rounds (sum / worst)
  double t_lockstep_stats_ms = 0;  // stats thread waiting for the newest-bucket round
  std::vector<double> rollover_latency_ms;   // batch arrival -> alert decision per rollover
};

void pin_current_thread(int cpu);
std::vector<int> local_core_slice(int device);  // this GPU's share of its NUMA node's physical cores

class ThreadPool {
 public:
  explicit ThreadPool(int n, const std::vector<int>& cpus = {});
  ~ThreadPool();
  // `meanwhile` (optional) runs on the calling thread while the workers execute the tasks; an
  // exception it throws is rethrown after every task has finished.
  void run(int n_tasks, const std::function<void(int)>& fn, const std::function<void()>* meanwhile = nullptr);
  int size() const { return (int)workers_.size(); }

 private:
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)>* fn_ = nullptr;
  int n_tasks_ = 0, done_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

// One background thread running posted tasks in order; wait(id) returns once task `id` is done
// and rethrows the first exception a task threw.
class TaskLane {
 public:
  TaskLane();
  ~TaskLane();
  uint64_t post(std::function<void()> fn);
  void wait(uint64_t id);
  void wait_all();

 private:
  std::thread th_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
  uint64_t posted_ = 0, done_ = 0;
  std::string err_;
  bool stop_ = false;
};

class Engine {
 public:
  explicit Engine(const EngineConfig& cfg);
  ~Engine();

  int32_t add_server(const std::string& name);
  int32_t add_file(const std::string& path, int kind, const std::string& server);
  void set_override(const std::string& service, const ServiceOverride& o);
  void clear_overrides();
  void refresh_series_settings();
  // Config hot reload without a pipeline drain (reconfig.cpp): staged now, applied by the stats
  // thread at a batch boundary (with lock-step ranks: the same boundary on every rank).
  void stage_reconfig(const ReconfigSpec& spec);
  uint64_t reconfig_applied_gen() const { return rc_applied_gen_.load(); }
  uint64_t reconfigs_applied() const { return reconfigs_applied_.load(); }
  uint64_t lag_set_changes() const { return lag_set_changes_.load(); }
  uint64_t window_changes() const { return window_changes_.load(); }
  int32_t ring_slots() const { return nslot_; }
  uint64_t ring_grows() const { return ring_grows_; }
  std::vector<int32_t> lag_values() { flush(); return std::vector<int32_t>(cfg_.lags, cfg_.lags + cfg_.n_lags); }

  // Process one batch. `now_override` < 0 uses the engine watermark clock.  If the caller
  // already has the next batch, passing it launches its H2D + parse kernels before this batch's
  // host join (double-buffered parse slots); the next call must then pass that same batch (its
  // bytes must stay valid until that call returns).
  void process_batch(const uint8_t* host_bytes, uint64_t n_bytes, const std::vector<Chunk>& chunks,
                     double now_override = -1.0, const uint8_t* next_bytes = nullptr, uint64_t next_n = 0,
                     const std::vector<Chunk>* next_chunks = nullptr);
  bool prefetch_pending() const { return prefetched_; }
  // Two-ahead input copy (device join only): starts the H2D of the batch after the next one into a
  // third device buffer on its own stream, so that batch's parse kernels -- launched by the next
  // process_batch -- find their input on the device instead of behind a 28 MB host-link copy.
  // The bytes must be passed unchanged (same pointer and size, canonical chunks) to that later
  // launch and stay valid until it; anything else just ignores the staged copy.
  void stage_batch(const uint8_t* host_bytes, uint64_t n_bytes);
  // tx CSV lines (a reference parser stage's `transactions` queue) straight into the stats stage
  void process_tx_lines(const std::string& blob, double now = -1.0);

  // Text outputs accumulated since the last take: "transactions", "audit_db", "db", "st", "fs",
  // "al" (enabled by EngineConfig::outputs).  take() splits into lines; take_bytes() hands out
  // the newline-terminated blob.
  std::vector<std::string> take(const std::string& kind);
  std::string take_bytes(const std::string& kind);
  // Route a stream to a file descriptor: the stats thread write()s each batch's blob to it (a
  // COPY/queue spool file, a pipe to the DB loader, /dev/null).  fd < 0 detaches.
  void set_sink_fd(const std::string& kind, int fd);
  // Route a stream to an in-process consumer (the native DB sink): the output lane hands it each
  // batch's bytes directly -- no Python, no extra copy.  nullptr detaches.
  void set_byte_sink(const std::string& kind, std::shared_ptr<ByteSink> sink);
  // fs stream as Postgres COPY rows (K12 formats the DB row directly; the DB sink skips encoding)
  void set_fs_copy(bool on);
  // released db rows as COPY rows of the transactions table, encoded on the GPU (device join
  // only; returns whether it is on)
  bool set_db_copy(bool on);
  bool db_copy() const { return db_copy_; }
  bool fs_copy() const { return fs_copy_; }
  static int pg_timestamp(int64_t ms, char* out);
  uint64_t sink_bytes(const std::string& kind) { flush(); return sink_bytes_[out_kind_of(kind)]; }

  // Exogenous per-JVM gauges (JMX jx record fields in JmxEntry order + VM load) fused into the
  // per-interval server rollup (K14, "sx" stream).  Returns false for a server this engine
  // does not own.
  bool set_server_context(const std::string& server, double ts_ms, const std::vector<double>& gauges,
                          double host_load);

  // Stage tracing (also emitted as roctx ranges for rocprofv3 --marker-trace).
  void set_trace(bool on) { trace_on_ = on; }
  std::vector<TraceEvent> take_trace();

  // Binary checkpoint of the whole pipeline state (checkpoint.cpp).  load_state needs a freshly
  // constructed engine with the same LAG set / ring dtype / bucket layout.  Returns bytes written.
  // `extra` is an opaque blob stored with the state (the service keeps its tail offsets there, so
  // one fsync + rename covers both); load_state returns it.  load_state also accepts a chain
  // manifest written by checkpoint_async (base + increments).
  uint64_t save_state(const std::string& path, const std::string& extra = std::string());
  // Fatal-path state dump (the analogue of the reference's heapdump / node-oom-heapdump,
  // apm_manager.js:12-18): host-side state only -- a faulted GPU context cannot be read -- as one
  // section of the checkpoint file format: reason, clocks, batch ids, counters, capacities and
  // fill levels (JSON text).  Returns the bytes written.
  uint64_t dump_state(const std::string& path, const std::string& reason);
  std::string load_state(const std::string& path);
  // Asynchronous incremental checkpoint into `<prefix>.ckpt` (chain manifest) + `<prefix>.{b,i}N.ckpt`:
  // the calling thread pays for a consistent snapshot (small sections + dirty ring rows copied
  // D2D into HBM staging); a writer thread does the D2H, file write and fsync.  Returns the
  // checkpoint sequence number, or -1 when the previous one is still being written (skipped).
  int64_t checkpoint_async(const std::string& prefix, const std::string& extra, bool force_base = false,
                           std::function<void()> pre_commit = {});
  uint64_t checkpoint_wait();  // waits for the writer; rethrows its error
  CheckpointInfo checkpoint_info();

  // Structured state access for the reference resume importer/exporter (state_io.cpp).
  std::vector<std::pair<std::string, std::string>> export_series();
  int32_t import_series(const std::string& server, const std::string& service);
  BucketDump export_buckets();
  void import_buckets(int64_t latest, const std::vector<int32_t>& series, const std::vector<int64_t>& bucket,
                      const std::vector<int32_t>& count, const std::vector<int32_t>& values);
  // history of series [lo, hi) for one LAG: len[j], vals[j][stat][LAG] chronological (NaN pad)
  void export_history(int lag_idx, int32_t lo, int32_t hi, std::vector<int32_t>& len, std::vector<double>& vals);
  void import_history(int lag_idx, const std::vector<int32_t>& series, const std::vector<int32_t>& len,
                      const std::vector<double>& vals);
  std::vector<double> export_lag_settings(int lag_idx);  // [series][thr, infl]
  std::vector<std::pair<int64_t, std::string>> export_pending();
  void import_pending(const std::vector<int64_t>& ends, const std::vector<std::string>& lines);
  std::vector<std::pair<std::string, double>> export_cooldowns();
  void import_cooldowns(const std::vector<std::pair<std::string, double>>& c);
  std::vector<int32_t> export_alert_counters(int lag_idx);
  void import_alert_counters(int lag_idx, const std::vector<int32_t>& series, const std::vector<int32_t>& counts);
  bool cooldown_by_service() const { return cfg_.cooldown_by_service != 0; }

  // Warm the z-score rings with a synthetic pre-history (benchmarks).
  void warm_history(uint64_t seed);

  // Fleet baseline exchange: per-service moments packed into `dst` (device pointer, doubles,
  // layout [n_services][n_lags][NSTAT][3] = count, sum, sumsq of the current ring means).
  int32_t n_services() const { return dict_.n_services(); }
  // atomic_path: the per-series fp64 atomic scatter instead of the MFMA Gram kernel (tests)
  void pack_service_moments(double* d_dst, int32_t n_services_cap, hipStream_t stream, bool atomic_path = false);
  // Native RCCL fleet exchange (see engine.cpp): rank 0 creates the id, every rank inits.
  static std::vector<uint8_t> fleet_unique_id();
  // clock_uid non-empty: lock-step clocks (node-wide watermark + rollover bucket) so N ranks
  // reproduce the single-stream reference per series.  (Only its presence matters: every
  // collective of a rank runs on ONE communicator, see engine.cpp.)
  void fleet_init(const std::vector<uint8_t>& uid, const std::vector<uint8_t>& clock_uid, int nranks, int rank,
                  int32_t n_services_cap);
  // Collective: call on every rank at the same point of the batch sequence.  Exchanges the
  // batches not yet exchanged and returns [cap][n_lags][NSTAT][3] of the newest.
  std::vector<double> fleet_merged();
  // node-wide slot -> service name (rows of fleet_merged), and {slots, registry rounds, slots
  // refused (maxServices full), fb rows emitted}
  std::vector<std::string> fleet_slot_names() { flush(); return reg_names_; }
  std::vector<uint64_t> fleet_info() {
    flush();  // (waits for both emission lanes)
    return {(uint64_t)reg_names_.size(), reg_rounds_, reg_overflow_, fb_rows_, (uint64_t)fleet_nranks_};
  }
  uint64_t fleet_rounds() const { return fleet_rounds_; }
  // node-wide sums of {ranks, batches, lines, events, bytes, tx, tx_db, released, rollovers,
  // alert candidates, alerts, series} as of the last interval edge's exchange (empty: none yet)
  std::vector<double> node_metrics();
  // Same exchange over an in-process group (tests: N engines of one process share one GPU).
  void fleet_init_local(std::shared_ptr<LocalGroup> group, int rank, int32_t n_services_cap, bool lockstep);
  // one process per rank over the TCP host transport (collective.h: HostCollective)
  void fleet_init_host(const std::string& addr, int port, int nranks, int rank, int32_t n_services_cap, bool lockstep);
  // Position of `server` in the node-wide server list (ranks own disjoint slices of it).  The
  // node-wide alert order ranks servers by (first batch with a series, this index); default =
  // local registration order, which is the global order on a single rank.
  void set_server_index(const std::string& server, int32_t global_index);
  // Collective: resolve every queued node-wide alert candidate (end of stream / before reading
  // the al stream).  Extra exchange rounds run until every rank's queue is empty.
  void node_drain();

  // Wait for the in-flight stats stage (process_batch returns while it still runs).
  void flush();
  EngineMetrics metrics() { flush(); return metrics_; }
  EngineMetrics metrics_nowait() {
    std::lock_guard<std::mutex> g(out_mu_);
    EngineMetrics m = metrics_;
    m.t_out_ms += t_out_ms_;
    return m;
  }
  // (cache_stats(false): the join table as the join stream leaves it, without draining)
  std::vector<uint64_t> cache_stats(bool drain);
  const std::vector<std::string>& servers() const { return servers_; }
  const std::vector<FileInfo>& files() const { return files_; }
  const std::vector<int>& lane_cpus() const { return lane_cpus_; }
  std::vector<std::string> services() const { return dict_.services_snapshot(); }
  int32_t n_series() const { return n_series_; }
  double watermark() const { return watermark_; }
  uint64_t batch_no() const { return batch_no_; }  // batches processed (node-wide equal in lock-step)
  hipStream_t stream() const { return stream_; }
  hipStream_t comm_stream() const { return stream_; }  // (the stats stream: callers flush() first)
  // HBM held: the engine's own buffers plus the device join's (which grow and shrink)
  size_t device_bytes() const { return device_bytes_ + (dj_ ? dj_->device_bytes() : 0); }
  // requestGC (util_methods.js:398-417 runGC, sent by apm_manager.js:475-512 on a memory
  // threshold): between batches, hand grow-only device memory back -- the join's key table and
  // need arena shrink to their live entries (>= their configured size), spill lists above 2x
  // their fill, checkpoint packing scratch and staging (re-made on demand).  Returns
  // {bytes before, bytes after}.
  std::pair<size_t, size_t> trim_device_memory();
  JoinCounters join_counters() const;
  // join-cache occupancy (device join: a reduction over the key table at the watermark clock;
  // host join: the shards' map sizes): {slots, occupied, acct, record, partials, need}
  std::vector<uint64_t> cache_stats() { return cache_stats(true); }

  // events of the last batch (host copy) for kernel verification
  std::string last_events() const;
  // pinned host memory for zero-copy ingest (bench corpus, tailer)
  static uintptr_t alloc_pinned(size_t n);
  static void free_pinned(uintptr_t p);

  // Device views for tests / exchange
  void download_winstats(std::vector<WinStat>& out);
  void download_zout(int lag_idx, std::vector<ZOut>& out);

 private:
  struct SeriesInfo { int32_t server, service; uint64_t emit_key; };
  int32_t series_for(int32_t server, int32_t service);
  void apply_series_settings(int32_t s);
  // live reconfiguration (reconfig.cpp)
  std::mutex rc_mu_;
  std::deque<ReconfigSpec> rc_staged_;                           // lock-step: awaiting the node
  std::deque<std::pair<uint64_t, ReconfigSpec>> rc_tagged_;      // (batch, spec), batches ascend
  std::atomic<uint64_t> rc_applied_gen_{0}, reconfigs_applied_{0}, lag_set_changes_{0}, window_changes_{0};
  std::map<int32_t, int32_t*> counter_stash_;                    // removed LAG -> its alert counters
  uint64_t reconfig_staged_gen();
  void reconfig_agree(uint64_t node_min);
  void apply_reconfig_pending(uint64_t upto);
  void apply_reconfig(const ReconfigSpec& r);
  // LAG set of each fleet slot's pack (the exchange and the fb rows run on the ingest thread)
  int pack_nlags_[2] = {0, 0};
  int32_t pack_lags_[2][MAX_LAGS] = {};
  void compute_series_settings(int32_t s, double* thr, double* infl, double& hard_max, uint8_t& suppressed);
  void stats_for_batch(std::vector<TxOut>& txs, double batch_t0);
  void stats_for_batch_dev(DevJoinBatch& b, double batch_t0);
  void post_stats_dev(DevJoinBatch&& b, double t0, int sync_slot);
  void release_device(int64_t edge_ts);   // K9 with the device join: count + gather on the GPU
  void release_device_finish();
  void refresh_unseen_active();
  std::string ring_text(const int64_t* d_gid, int64_t n);  // pending lines out of the HBM ring
  void ensure_bucket_slot(int64_t b);
  void do_rollover(int64_t L, double batch_t0);
  void flush_alerts(int64_t edge_ts);
  void finish_rollover();
  bool roll_pending_ = false;  // do_rollover queued; its decision is made by finish_rollover
  int64_t roll_edge_ts_ = 0;
  double roll_batch_t0_ = 0;
  uint64_t roll_round_ = 0;        // exchange round of the pending rollover's batch
  uint64_t roll_ring_base_ = 0;    // text-ring base of the batch being processed at the rollover
  // Rollover lane: the second half of a rollover (wait for the candidates and the released count,
  // queue the released lines' gather, decide the alerts) runs here, so the stats thread goes on
  // with the next batch instead of waiting for its GPU chain.  The next rollover (or flush) waits
  // for it first; series_mu_ guards series_ growth against the lane's reads.
  std::unique_ptr<TaskLane> roll_lane_;
  bool roll_lane_mode_ = false;  // fixed at construction (APM_ROLL_LANE, outputs): same on every rank
  uint64_t roll_task_ = 0;
  bool roll_posted_ = false;
  std::mutex series_mu_;
  std::mutex alloc_mu_;            // allocations_ / device_bytes_
  std::mutex roll_mu_;
  std::condition_variable roll_cv_;
  int64_t roll_done_round_ = -1;   // newest round whose alert candidates are queued (node mode)
  void finish_rollover_body();
  void wait_roll_round(uint64_t round);
  void format_rollover_text(int64_t edge_ts);       // K12 on the GPU
  void format_rollover_text_host(int64_t edge_ts);  // fallback (|value| >= 1e13)
  void sync_format_tables();
  int32_t intern_name(const std::string& name);
  void* regrow(void* old, size_t& cap, size_t need);
  void dfree(void* p);
  void emit_bytes(int kind, const char* p, size_t n);
  // staging buffer k (st/fs 0, 1; fb 2, 3) is referenced by the sink until its holds are released
  void emit_bytes_held(int kind, const char* p, size_t n, int k, const uint32_t* row_off = nullptr,
                       size_t nrows = 0);
  void wait_fmt_holds(int k);
  static constexpr int FMT_RING = 4, REL_RING = 4;
  struct FmtHolds {  // shared with the holds: a release after the engine is gone stays safe
    std::mutex mu;
    std::condition_variable cv;
    // st/fs device-written staging 0, 1 (APM_FMT_HOST); fb staging 2, 3; released db text 4, 5;
    // st/fs host ring 6 .. 6 + FMT_RING; released db text ring after it
    int n[6 + FMT_RING + REL_RING] = {};
  };
  std::shared_ptr<FmtHolds> fmt_holds_ = std::make_shared<FmtHolds>();
  void upload_series_tables(int32_t lo);
  void pack_moments_locked(double* d_dst, int32_t cap, hipStream_t stream, bool atomic_path = false);
  void fleet_pack_locked();
  void fleet_exchange_upto(uint64_t rounds);
  void fleet_setup(int32_t cap, bool lockstep);
  // node-wide cooldown (ingest thread): one all-gather round per exchanged batch
  void node_round(uint64_t round, bool wait, bool all = false);
  void node_resolve();
  void node_take_text();
  void coll_wait(hipStream_t s, hipEvent_t ev, const char* what);
  void lockstep_issue(double watermark_through_batch);
  int lockstep_collect(int64_t batch_max_bucket);
  int64_t lockstep_latest(int slot);
  void apply_latest_locked(int64_t g, double batch_t0);
  void stats_worker();
  void post_stats(std::vector<std::vector<TxOut>>&& outs, bool multi, double t0, int sync_slot = -1);
  void drain_sinks(uint32_t kinds = ~0u);
  void drain_kind(int k);
  // output lane (see engine.cpp): waits for the D2H of released-tx ids / formatted text and
  // writes those streams, off the stats thread's critical path
  void out_worker();
  uint64_t post_out(std::function<void()> fn);
  void out_wait(uint64_t task);
  void out_wait_idle();
  void release_gather(int k, int64_t released);
  bool want(int k) const { return (cfg_.outputs >> k) & 1u; }
  void* dmalloc(size_t bytes);
  void* dmalloc_try(size_t bytes);
  void require_fresh(const char* what);
  void trace_event(const char* name, double t0, double t1, int tid);
  bool trace_on_ = false;
  std::mutex trace_mu_;
  std::vector<TraceEvent> trace_;

  EngineConfig cfg_;
  hipStream_t stream_ = nullptr, parse_stream_ = nullptr;
  // fleet exchange + lock-step clocks: ONE communicator, driven only by the ingest thread on
  // coll_stream_, so every rank issues the same collectives in the same order (engine.cpp)
  std::unique_ptr<Collective> coll_;
  hipStream_t coll_stream_ = nullptr;
  bool lockstep_ = false;
  // lock-step exchanges (engine.cpp lockstep_issue / lockstep_collect): d_sync_ [0,4) clocks,
  // [4,8) newest bucket; h_sync_ (pinned) [4,8) clock result, [8 + 4 s, 12 + 4 s) bucket result of
  // ring slot s (batch & 3), read by the stats thread
  double* d_sync_ = nullptr;
  double* h_sync_ = nullptr;
  hipEvent_t clock_ev_ = nullptr;
  hipEvent_t bucket_ev_[4] = {nullptr, nullptr, nullptr, nullptr};
  bool clock_pending_ = false;
  int32_t fleet_cap_ = 0;
  size_t fleet_elems_ = 0;
  double* fleet_buf_[2] = {nullptr, nullptr};
  hipEvent_t fleet_ev_[2] = {nullptr, nullptr};    // all-reduce of the slot done (coll stream)
  hipEvent_t pack_ev_[2] = {nullptr, nullptr};     // pack of the slot done (comm stream)
  int fleet_nranks_ = 0;
  bool fleet_skip_solo_ = false;
  std::vector<int64_t> shard_maxb_;  // per-shard newest bucket (one cache line each), lock-step clock
  uint64_t fleet_rounds_ = 0;  // exchanges issued (ingest thread)
  uint64_t fleet_posted_ = 0;  // batches posted since fleet_init (ingest thread)
  // device-join batches defer their fleet exchange (rounds < fleet_due_) into the next batch's
  // join-kernel window; every later caller exchanges up to fleet_posted_ anyway
  uint64_t fleet_due_ = 0;
  uint64_t fleet_packed_ = 0;  // batches packed (stats thread)
  // ---- node-wide alert cooldown.  The stats thread queues this rank's candidates (with their
  // al-row payload, formatted while the rollover's stats are current); the ingest thread
  // all-gathers them once per exchanged batch and, when every rank has sent everything up to
  // that batch, decides all pooled candidates in the global order -- identically on every rank.
  struct NodeCand {  // wire record (64 B), same on every rank
    int64_t edge_ts;
    int64_t first_batch;  // batch in which the server got its first series
    int32_t gidx;         // node-wide server index
    uint32_t seq;         // service first-appearance order within the server
    int32_t lag_idx;
    uint32_t causes;
    uint64_t key;         // cooldown key hash (service, or server + service)
    double now;           // alert timestamp
    int32_t rank;
    uint32_t local_id;    // index into the owner's payload list
    uint64_t pad;
  };
  struct NodeHdr { int32_t count, all_sent, pad[14]; };  // 64 B
  // a candidate's fs text is formatted only if it wins the node-wide cooldown (node_resolve)
  // (no strings: an alert storm queues thousands of candidates per rollover; names are looked up
  // for the winners only)
  struct NodePayload { uint64_t seq_batch; NodeCand c; int32_t series; int32_t lag; WinStat w; ZOut z; };
  bool node_mode_ = false;
  double node_cool_ms_ = 0;  // ingest thread's cooldown (a reload switches it at the agreed batch)
  // candidates per rank per round: an alert storm (thousands of new keys per interval) must not
  // outgrow the exchange, or the unsent backlog and the decision lag grow without bound
  int32_t node_cap_ = 4096;
  std::mutex node_mu_;                     // node_q_ / node_text_
  std::deque<NodePayload> node_q_;         // stats thread -> ingest thread (unsent)
  std::deque<NodePayload> node_sent_;      // sent, awaiting a decision (ingest); local ids are
  uint32_t node_sent_base_ = 0;            // consecutive: payload of id i = node_sent_[i - base]
  // node-wide cooldowns by key hash (checkpointed inside last_alert_ as "\x02" + 16 hex digits)
  std::unordered_map<uint64_t, double> node_cool_;
  uint32_t node_next_id_ = 0;
  std::vector<NodeCand> node_pool_;        // gathered, undecided (ingest thread)
  std::string node_text_;                  // decided al rows of this rank -> blob_[OUT_AL]
  uint64_t node_alerts_ = 0;
  bool node_round_pending_ = false;        // a gather is in flight (coll stream)
  // ---- node-wide service registry (fleet.cpp).  Each rank interns services in its own order,
  // so the moments matrix is indexed by a node-wide *slot*: new services travel (hash + name) in
  // an all-gather of the lock-step round, and every rank assigns slots to unseen hashes in rank
  // order -- identical tables everywhere, no coordinator.
  // one round carries a whole shard's worth of new services (10k names ~ 400 KB), so the
  // registry settles within the first batches instead of trickling through the timed region
  static constexpr size_t kRegBlock = 1 << 20;
  static constexpr int kRegMaxEntries = 32768;
  struct RegPending { int32_t id; uint64_t hash; std::string name; uint64_t tag; };  // tag: batch queued in
  std::mutex reg_mu_;
  std::deque<RegPending> reg_pending_;                     // stats thread -> ingest thread
  struct RegAssigned { int32_t id, slot; uint64_t tag; };  // adopted by the pack of batch >= tag
  std::vector<RegAssigned> reg_assigned_;                  // ingest -> stats thread
  std::vector<uint8_t> reg_queued_;                        // stats thread: dict id queued
  int32_t reg_scan_series_ = 0;                            // stats thread: series scanned
  std::vector<int32_t> fleet_slot_;                        // stats thread: dict id -> slot (-1)
  std::unordered_map<uint64_t, int32_t> reg_slot_;         // ingest thread: hash -> slot
  std::vector<std::string> reg_names_;                     // ingest thread: slot -> name
  uint64_t reg_overflow_ = 0, reg_rounds_ = 0;
  uint8_t *d_reg_send_ = nullptr, *d_reg_recv_ = nullptr, *h_reg_send_ = nullptr, *h_reg_recv_ = nullptr;
  int32_t reg_sent_ = 0;
  void reg_collect_locked();                 // stats thread: queue services of new series
  void reg_apply_locked();                   // stats thread: adopt assigned slots
  int32_t reg_pending_count();
  void reg_round();                          // ingest thread: all-gather + slot assignment
  int32_t svc_key(int32_t s) const;          // moments row of series s (slot, or dict id alone)
  // ---- fb stream: fleet-merged per-service baselines (rank 0, after a rollover's exchange)
  int64_t pack_edge_[2] = {0, 0};            // stats thread: newest rollover edge of the packed batch
  int64_t last_edge_ts_ = 0;                 // stats thread: newest rollover edge so far
  uint64_t last_edge_seen_ = 0;
  std::string h_fb_chars_;                   // slot names (ingest thread)
  std::vector<int32_t> h_fb_names_;          // {off, len} per slot
  char* d_fb_chars_ = nullptr;
  size_t fb_chars_cap_ = 0, fb_chars_up_ = 0;
  int32_t* d_fb_names_ = nullptr;
  size_t fb_names_cap_ = 0;
  int32_t fb_slots_up_ = 0;
  unsigned long long* d_fb_status_ = nullptr;  // per-wave byte totals of k_fleet_len (+ 2 totals)
  uint32_t fb_status_n_ = 0;
  hipStream_t fb_stream_ = nullptr;          // fb formatting (low priority; never the collective stream)
  hipEvent_t fb_src_ev_[2] = {nullptr, nullptr};   // moments slot all-reduced (coll stream)
  char* d_fb_out_[2] = {nullptr, nullptr};
  size_t fb_out_cap_[2] = {0, 0};
  char* h_fb_out_[2] = {nullptr, nullptr};
  size_t h_fb_cap_[2] = {0, 0};
  uint32_t* h_fb_total_ = nullptr;
  hipEvent_t fb_ev_[2] = {nullptr, nullptr};
  uint64_t fb_task_[2] = {0, 0};
  int fb_k_ = 0;
  uint64_t fb_rows_ = 0;
  bool fleet_emit_fb(int slot);              // ingest thread, after the slot's all-reduce
  bool node_all_sent_ = true;              // every rank's last round sent everything
  uint8_t* d_node_send_ = nullptr;
  uint8_t* d_node_recv_ = nullptr;
  uint8_t* h_node_send_ = nullptr;         // pinned
  uint8_t* h_node_recv_ = nullptr;         // pinned
  hipEvent_t node_ev_ = nullptr;
  uint64_t stats_seq_ = 0;                 // stats thread: batch index of the job being processed
  uint64_t stats_round_ = 0;               // stats thread: its exchange round
  std::vector<int32_t> server_gidx_;
  std::vector<int64_t> server_first_batch_;
  // stats thread
  struct StatsJob {
    std::vector<std::vector<TxOut>> outs;  // per shard, merged by the stats thread into txs
    bool multi = false;
    std::vector<TxOut> txs; std::vector<std::string> text; double t0 = 0;
    int sync_slot = -1;  // lock-step: ring slot of this batch's node-wide newest-bucket exchange
    bool dev = false;                 // device join: `dj` instead of outs / txs
    uint64_t seq = 0;                 // batch index (the ingest thread's batch_no_)
    uint64_t round = 0;               // exchange round (posts since fleet_init)
    DevJoinBatch dj;
  };
  std::vector<std::string>* cur_text_ = nullptr;  // text arenas of the job being processed
  std::thread stats_thread_;
  std::mutex st_mu_;
  std::condition_variable st_cv_;
  StatsJob st_job_;
  std::vector<std::vector<TxOut>> out_pool_;  // emptied shard output vectors (capacity kept)
  std::mutex out_pool_mu_;
  bool st_has_job_ = false, st_busy_ = false, st_stop_ = false;
  std::string st_error_;
  // output lane: FIFO of emit tasks; it owns the db / st / fs streams (kLaneKinds)
  std::thread out_thread_;
  std::mutex out_mu_;
  std::condition_variable out_cv_;
  std::deque<std::function<void()>> out_q_;
  uint64_t out_posted_ = 0, out_done_ = 0;
  bool out_stop_ = false;
  std::string out_error_;
  double t_out_ms_ = 0;  // lane busy time (folded into metrics_ by flush)
  uint64_t formatted_bytes_lane_ = 0;  // st/fs bytes emitted by the lane (folded by flush)
  size_t device_bytes_ = 0;
  std::vector<void*> allocations_;
  std::unordered_map<void*, size_t> alloc_bytes_;

  // files / servers / dictionaries
  std::vector<std::string> servers_;
  std::unordered_map<std::string, int32_t> server_ids_;
  std::vector<FileInfo> files_;
  Dictionary dict_;
  std::vector<std::unique_ptr<JoinShard>> shards_;  // one per server
  std::unique_ptr<ThreadPool> pool_;
  // device join: the next batch's parse finish + host pre-pass, overlapping this batch's join
  std::unique_ptr<TaskLane> ahead_lane_;
  std::unique_ptr<TaskLane> fb_lane_;  // rank 0's fb rows: D2H + emission beside the output lane
  // node-wide counters: all-reduce(SUM) of this rank's counters at every interval edge, async on
  // the collective stream (SURVEY 2.4 "ncclAllReduce of counters/metrics")
  static constexpr int kNodeMetrics = 12;
  double* d_nm_ = nullptr;
  double* h_nm_send_ = nullptr;
  double* h_nm_recv_ = nullptr;
  hipEvent_t nm_ev_ = nullptr;
  bool nm_pending_ = false;
  std::mutex nm_mu_;
  std::vector<double> node_metrics_;  // last completed reduction
  void node_metrics_round();
  uint64_t ahead_task_ = 0;
  std::vector<int> lane_cpus_;  // pinned placement (empty: unpinned)
  std::vector<double> shard_ms_;  // per-shard join time of the current batch (stride 16)

  // series
  FlatMap<int32_t> series_map_{1 << 16};  // ((server + 1) << 32 | service) -> series + 1
  std::vector<std::vector<int32_t>> ser_tab_;  // cache of series_map_: [server][service] -> series / -1
  // [server][shard-local raw service id] -> series / -1: the tx loop's lookup.  Rows are as long
  // as the shard's own service list (a few thousand), where ser_tab_ rows span the global
  // service dictionary (100k ids x 32 servers = 12.8 MB for the firehose shard: a miss per tx).
  std::vector<std::vector<int32_t>> ser_raw_;
  void ser_tab_put(int32_t server, int32_t service, int32_t s) {
    if (server < 0 || service < 0 || service >= (1 << 20)) return;
    if ((size_t)server >= ser_tab_.size()) ser_tab_.resize((size_t)server + 1);
    auto& row = ser_tab_[server];
    if ((size_t)service >= row.size()) row.resize(std::max<size_t>((size_t)service + 1, row.size() * 2), -1);
    row[service] = s;
  }
  std::vector<SeriesInfo> series_;
  int32_t n_series_ = 0;
  std::vector<int32_t> server_rank_;            // first-appearance rank per server in the stats stream
  std::vector<int32_t> server_next_service_;
  int32_t next_server_rank_ = 0;
  std::map<std::string, ServiceOverride> overrides_;
  double alias_thr_[MAX_LAGS], alias_infl_[MAX_LAGS];  // defaults as mutated by Q4 emulation
  std::vector<double> h_thr_, h_infl_, h_hard_max_;
  std::vector<uint8_t> h_suppressed_;
  std::vector<uint64_t> h_emit_key_;
  std::vector<int32_t> zscore_seen_;            // series already initialised in the z-score stage
  std::vector<uint8_t> h_active_;               // host mirror of the stats `active` flag
  std::vector<int32_t> unseen_;                 // series not yet initialised in the z-score stage

  // device join (cfg_.device_join): tables, ring, per-slot batch buffers
  std::unique_ptr<DeviceJoin> dj_;
  const DevJoinBatch* cur_dj_ = nullptr;       // stats thread: batch being processed
  uint64_t ring_low_pending_ = UINT64_MAX;     // ring base of the batch at the last min_pos launch
  unsigned long long* d_ring_min_ = nullptr;
  unsigned long long* h_ring_min_ = nullptr;
  unsigned long long* hd_ring_min_ = nullptr;  // device view (apm_export)
  int64_t* d_rel_n_ = nullptr;
  int64_t* h_rel_n_ = nullptr;
  int64_t* hd_rel_n_ = nullptr;
  uint32_t* d_rel_lens_ = nullptr;
  uint32_t* d_rel_offs_ = nullptr;
  uint32_t* d_rel_fb_ = nullptr;  // released lines outside the GPU COPY encoder's domain (txcopy.hip)
  uint32_t* h_rel_total_ = nullptr;            // [2]
  uint32_t* hd_rel_total_ = nullptr;
  char* d_rel_text_[2] = {nullptr, nullptr};
  size_t rel_text_cap_[2] = {0, 0};
  // pinned released-line text, a ring (the sink's spool writers hold a slot until written; with
  // two the release lane waited 1.7 ms per batch for them, profiles/r5_s)
  char* h_rel_text_[REL_RING] = {};
  size_t h_rel_text_cap_[REL_RING] = {};
  int rel_ring_k_ = 0;  // stats thread
  uint32_t* h_rel_offs_[2] = {nullptr, nullptr};  // pinned: the released rows' offsets (sink flush cuts)
  size_t h_rel_offs_cap_[2] = {0, 0};
  hipStream_t out_stream_ = nullptr;
  std::vector<int32_t> h_raw_series_;          // stats thread mirror of the raw -> series table
  // pinned staging of the stats thread's H2D uploads: kStage buffers used in rotation, each
  // reused only after its previous copy completed (an event), so no upload waits for the stream
  static constexpr int kStage = 32;  // > the uploads of a few batches (a batch with new series makes ~10)
  char* h_stage_[kStage] = {};
  size_t h_stage_cap_[kStage] = {};
  size_t stage_max_ = 0;
  hipEvent_t stage_ev_[kStage] = {};
  int stage_k_ = 0;
  void h2d(void* d, const void* h_pinned, size_t n, hipStream_t s);  // kernel copies (never block)
  void d2h(void* h_pinned, const void* d, size_t n, hipStream_t s);
  char* stage(size_t bytes);
  void stage_done();
  int32_t* d_pairs_ = nullptr;
  size_t pairs_bytes_ = 0;
  int32_t* pinned_pairs(size_t n_ints);
  void pinned_pairs_done() { stage_done(); }
  size_t max_name_len_ = 0;  // longest server + service name of any series (K12 output bound)
  int32_t* d_unseen_idx_ = nullptr;
  uint8_t* d_unseen_flag_ = nullptr;
  uint8_t* h_unseen_flag_ = nullptr;
  unsigned long long* d_unmapped_ = nullptr;
  bool dev() const { return dj_ != nullptr; }

  // parse buffers
  uint8_t* d_bytes_ = nullptr;
  // double-buffered parse slots (host side): staging bytes, chunk tables, events, counters
  struct ParseSlot {
    uint8_t* h_bytes = nullptr;                 // pinned staging (non-canonical batches)
    uint32_t* h_chunk_begin = nullptr;
    uint8_t* h_chunk_kind = nullptr;
    uint32_t* h_chunk_file = nullptr;
    Event* h_events = nullptr;
    Event* d_events_host = nullptr;             // device alias of h_events (zero-copy compaction)
    uint32_t* h_counts = nullptr;               // [0]=n_events [1]=n_lines
    unsigned long long* h_watermark = nullptr;
    const uint8_t* hb = nullptr;                // bytes the join reads (caller's or staging)
    const uint8_t* src = nullptr;               // caller's pointer (prefetch identity check)
    uint64_t src_n = 0, n_bytes = 0;
    std::vector<int32_t> chunk_file;
    uint32_t n_events = 0, n_lines = 0;
    uint32_t spec_copied = 0;                   // events already D2H'd behind the parse kernels
    bool pending = false;
  } pslot_[2];
  uint32_t spec_events_ = 0;                    // speculative D2H size for the next prefetched parse
  int cur_slot_ = 0, last_slot_ = 0;
  bool prefetched_ = false;
  // stage_batch: the batch whose H2D is queued on in_stage_stream_ (identity check at its launch)
  const uint8_t* in_stage_src_ = nullptr;
  uint64_t in_stage_n_ = 0;
  hipStream_t in_stage_stream_ = nullptr;
  hipEvent_t in_stage_ev_ = nullptr;
  void launch_parse(ParseSlot& ps, const uint8_t* host_bytes, uint64_t n_bytes, const std::vector<Chunk>& chunks,
                    bool speculative = false);
  void process_batch_dev_tail(ParseSlot& ps, double t0, double now_override, const uint8_t* next_bytes,
                              uint64_t next_n, const std::vector<Chunk>* next_chunks);
  void finish_parse(ParseSlot& ps);
  double batch_watermark(const ParseSlot& ps) const;  // watermark_ advanced by the slot's parse
  uint32_t* d_chunk_begin_[2] = {nullptr, nullptr};  // per parse slot (the device join reads them)
  uint8_t* d_chunk_kind_[2] = {nullptr, nullptr};
  uint32_t* d_chunk_file_[2] = {nullptr, nullptr};
  void* d_parse_ws_ = nullptr;
  Event* d_events_ = nullptr;
  uint32_t* d_counts_ = nullptr;                // [0]=n_events [1]=n_lines
  unsigned long long* d_watermark_ = nullptr;
  uint8_t* d_file_open_ = nullptr;
  TzTable* d_tz_unused_ = nullptr;

  // stats state
  int32_t* d_counts_cells_ = nullptr;
  int32_t* d_cells_ = nullptr;
  int32_t* d_spill_n_ = nullptr;
  int32_t* d_spill_series_ = nullptr;
  int32_t* d_spill_val_ = nullptr;
  int32_t* d_spill_series_alt_ = nullptr;  // sort target before K8 (swapped with the live lists)
  int32_t* d_spill_val_alt_ = nullptr;
  void* d_spill_tmp_ = nullptr;
  size_t spill_tmp_bytes_ = 0;
  int32_t* h_spill_snap_ = nullptr;   // pinned [nslot_], written by K7 after every append
  int32_t* hd_spill_snap_ = nullptr;  // its device alias
  // Spill sizing (no sample is ever dropped): spill_n[slot] <= spill_bound(slot) = the exact fill
  // of the newest completed append snapshot + every sample appended after it (any may spill), or
  // every sample appended since the slot was cleared.  spill_reserve() grows the lists before an
  // append whose worst case exceeds them.
  uint64_t spill_added_ = 0;
  std::vector<uint64_t> spill_clear_at_;  // [nslot_]
  struct SpillMark { hipEvent_t ev = nullptr; uint64_t added = 0; bool live = false; };
  static constexpr int kSpillMarks = 4;
  SpillMark spill_mark_[kSpillMarks];
  int spill_mark_k_ = 0;
  void spill_reserve(uint32_t n);
  void spill_marked();
  void spill_resync();
  void grow_spill(int32_t cap);
  void spill_sort();
  unsigned long long* d_spill_drop_ = nullptr;  // K7 samples lost to a full spill list
  uint8_t* d_active_ = nullptr;
  // bucket ring: bucket b lives in slot b % nslot_ (slot_bucket_[slot], NO_BUCKET = free)
  int32_t nslot_ = NSLOT_MIN;
  std::vector<int64_t> slot_bucket_;
  uint64_t ring_grows_ = 0;
  int32_t* d_win_slots_ = nullptr;  // K8's window slots when the window is longer than K8_INLINE_SLOTS
  void alloc_ring(int32_t nslot);   // the ring's device / pinned arrays at nslot slots (fresh engine)
  void grow_ring(int32_t nslot);    // the same with every live bucket moved to its new slot
  int64_t latest_ = 0;
  int64_t rollover_idx_ = 0;
  WinStat* d_win_ = nullptr;
  int32_t* d_big_list_ = nullptr;
  int32_t* d_big_n_ = nullptr;
  int32_t* d_nan_until_ = nullptr;   // [S] NaN-live horizon per series (ordered K7 append)
  int32_t* d_ord_list_ = nullptr;
  int32_t* d_ord_n_ = nullptr;
  int32_t* d_nan_list_ = nullptr;    // K8 series whose window holds a NaN sample
  int32_t* d_nan_n_ = nullptr;
  int32_t* d_js_scratch_ = nullptr;  // [JS_BLOCKS][kJsCap]
  static constexpr int32_t kJsCap = 1 << 18;
  StatsState stats_state() const;
  void grow_tx_capacity(uint32_t need, uint32_t keep);
  int64_t ord_cap_ = 0;

  // checkpoint (checkpoint.cpp)
  struct CkJob {
    struct Lag { int32_t n_cols = 0; std::vector<int32_t> heads; size_t off = 0; };
    bool streamed = false;  // ring section row-major, rows staged / read live / copied aside (CkStream)
    bool base = false;
    int64_t seq = 0;
    std::string prefix, name, path, extra;
    MemBlob blob;                 // the small sections, serialised at the snapshot
    std::vector<Lag> lags;
    // run by the writer thread before it writes the engine's file (the DB sink's pending-flush
    // snapshot, whose held buffers it releases once written); the manifest names the checkpoint
    // only after both: a throw fails this checkpoint
    std::function<void()> pre_commit;
    // deferred device reads of the small sections (d2h.h CkDefer): blob holes the writer fills
    // from the staging (the D2D copies into it completed within the snapshot)
    std::vector<std::array<size_t, 3>> holes;  // {blob offset, staging offset, bytes}
    std::vector<std::pair<size_t, int32_t>> patches;  // stored after the holes are filled
  };
  static constexpr int kMaxChain = 16;
  // Streamed base snapshot: the z-score rings can fill most of HBM, so a base whose rows exceed
  // the staging cap stages only the rows the next rollovers overwrite first; the writer reads the
  // others from the live ring, and a rollover about to overwrite a row not yet read copies it
  // aside first (copy-before-overwrite, ck_guard_rollover).  Per (lag, position) row state:
  enum : uint8_t { CKR_NONE = 0, CKR_LIVE, CKR_READING, CKR_STAGED, CKR_SIDE, CKR_DONE };
  struct CkStream {
    bool on = false;
    std::vector<std::vector<uint8_t>> state;  // [lag][ring position]
    std::vector<std::vector<size_t>> off;     // staging (CKR_STAGED) or side (CKR_SIDE) offset
    size_t side_used = 0, side_cap = 0;
    bool side_sync = false;                   // side copies queued on stream_ since the writer's last sync
    int32_t n_cols = 0;                       // series in the snapshot's rows
    uint64_t live_rows = 0, side_rows = 0, stalls = 0;
  } cks_;
  std::mutex cks_mu_;
  std::condition_variable cks_cv_;
  char* d_ck_side_ = nullptr;
  uint64_t ck_streamed_ = 0, ck_streamed_live_ = 0, ck_side_rows_ = 0, ck_guard_stalls_ = 0;
  hipEvent_t ck_side_ev_ = nullptr;   // after the newest side copy (stream_)
  void ck_guard_rollover(int64_t r);  // stats thread, before K10 of rollover r writes ring rows
  void write_streamed_ring(const std::shared_ptr<CkJob>& job, class BinWriter& w, char* bounce);
  // staging of the deferred small-section reads (one checkpoint in flight at a time)
  char* d_ck_defer_ = nullptr;
  size_t ck_defer_cap_ = 0, ck_defer_want_ = 0;
  uint64_t ck_deferred_bytes_ = 0;  // of the last snapshot (checkpoint_info)
  void checkpoint_quiesce(const char* what);
  void write_small_sections(class BinWriter& w);
  void write_series_dump(class BinWriter& w);
  std::string load_small_state(const std::string& path);
  void apply_ring_file(const std::string& path);
  void checkpoint_writer();
  void free_ck_stage();
  void resize_spill(int32_t cap);  // grow_spill / the trim (cap >= every slot's fill)
  int32_t init_spill_cap_ = 0;
  void finish_chain(const std::shared_ptr<CkJob>& job, uint64_t bytes);
  void checkpoint_shutdown();
  std::mutex ck_mu_;
  std::condition_variable ck_cv_;
  std::thread ck_thread_;
  std::shared_ptr<CkJob> ck_job_;
  bool ck_busy_ = false, ck_stop_ = false, ck_all_dirty_ = true;
  std::string ck_error_, ck_prefix_;
  std::vector<std::string> ck_chain_;
  // the chain a base replaced, kept on disk as <prefix>.prev.ckpt until the next base: every rank
  // of a lock-step node then still holds a batch common to all ranks when one of them dies while
  // the others write an aligned base (finish_chain)
  std::vector<std::string> ck_prev_chain_;
  bool ck_disk_chains_read_ = false;
  int64_t ck_seq_ = 0, ck_ridx_ = 0;
  int ck_last_mode_ = 0;
  uint64_t ck_done_ = 0, ck_skipped_ = 0, ck_sync_fallbacks_ = 0, ck_last_bytes_ = 0;
  int64_t ck_last_ring_rows_ = 0;
  double ck_last_stall_ms_ = 0, ck_last_write_ms_ = 0;
  void* d_ck_stage_ = nullptr;
  size_t ck_stage_bytes_ = 0;
  size_t ck_last_need_ = 0;  // ring staging the last snapshot needed (trim keeps up to 2x)
  void* h_ck_bounce_ = nullptr;
  size_t ck_blob_hint_ = 0;         // size of the last small-section blob (reserve)
  MemBlob ck_blob_spare_;           // the last written snapshot's blob buffer, reused (ck_mu_)
  char* d_ck_text_[2] = {nullptr, nullptr};  // pending-line text gathered for a checkpoint
  int64_t* d_ck_gids_ = nullptr;             // the pending lines' gids rebased to that text
  size_t ck_gids_cap_ = 0;
  size_t ck_text_cap_[2] = {0, 0};
  // checkpoint cell packing (device scan + gather of the occupied bucket cells)
  int32_t* d_ck_slots_ = nullptr;
  uint32_t *d_ck_lens_ = nullptr, *d_ck_offs_ = nullptr;
  int32_t* d_ck_packed_ = nullptr;
  void* d_ck_ptmp_ = nullptr;
  uint64_t ck_pack_n_ = 0;
  size_t ck_ptmp_bytes_ = 0;
  hipEvent_t ck_ev_ = nullptr;
  hipStream_t ck_stream_ = nullptr;

  // z-score state per lag
  struct LagState {
    void* ring = nullptr;
    int32_t* len = nullptr;
    double *sum = nullptr, *comp = nullptr, *sumsq = nullptr, *sqcomp = nullptr;
    int32_t* cnt = nullptr;
    double *thr = nullptr, *infl = nullptr;
    ZOut* out = nullptr;
    int32_t* counter = nullptr;
  } lag_[MAX_LAGS];
  static constexpr int RS_PARTS = 64;
  int32_t rs_range_ = 0;
  double* rs_part_ = nullptr;
  int32_t* rs_cnt_ = nullptr;
  double* d_hard_max_ = nullptr;
  void* d_lag_sum_ptrs_ = nullptr;
  void* d_lag_comp_ptrs_ = nullptr;
  void* d_lag_cnt_ptrs_ = nullptr;
  int32_t* d_series_service_ = nullptr;
  int32_t series_service_uploaded_ = 0;
  // series grouped by service (CSR) for the MFMA Gram pack; rebuilt when series are added
  std::vector<int32_t> h_svc_off_, h_svc_ids_;
  int32_t* d_svc_off_ = nullptr;
  int32_t* d_svc_ids_ = nullptr;
  size_t svc_off_cap_ = 0, svc_ids_cap_ = 0;
  int32_t svc_csr_n_ = -1, svc_csr_cap_ = -1;
  int32_t* h_tail_csr_[2] = {nullptr, nullptr};  // per-batch CSR of the series added since the snapshot (pinned, alternating)
  size_t tail_csr_cap_[2] = {0, 0};
  hipEvent_t tail_csr_ev_[2] = {nullptr, nullptr};
  int tail_k_ = 0;
  int32_t* d_tail_csr_ = nullptr;
  size_t d_tail_csr_cap_ = 0;
  std::pair<int32_t, int32_t> tail_csr_for_{-1, -1};  // (CSR snapshot size, n_series) of the uploaded tail
  int32_t tail_csr_m_ = 0;
  std::map<int32_t, std::vector<int32_t>> tail_by_svc_;  // the tail's series per row, in series order
  int32_t tail_upto_ = -1;                               // series [svc_csr_n_, tail_upto_) are in it
 public:
  int64_t last_gram_tail_ = 0;  // series the last Gram pack took from the tail CSR (tests)
 private:
  int32_t* h_series_service_ = nullptr;  // pinned mirror of d_series_service_ (append-only uploads)
  uint8_t* d_suppressed_ = nullptr;
  uint64_t* d_emit_key_ = nullptr;

  // alerts
  AlertRec* d_alerts_ = nullptr;
  int32_t* d_n_alerts_ = nullptr;
  AlertRec* h_alerts_ = nullptr;
  WinStat* h_alert_win_ = nullptr;  // pinned; candidate rows written by apm_alert_gather
  ZOut* h_alert_z_ = nullptr;       // pinned
  int32_t* h_n_alerts_ = nullptr;
  AlertRec* hd_alerts_ = nullptr;  // device views of the four pinned buffers above
  WinStat* hd_alert_win_ = nullptr;
  ZOut* hd_alert_z_ = nullptr;
  int32_t* hd_n_alerts_ = nullptr;
  hipEvent_t ev_alerts_ = nullptr;  // the rollover's candidates are in host memory
  hipEvent_t ev_release_ = nullptr; // the rollover's device release (K9 part 1) exported its counts
  std::unordered_map<std::string, double> last_alert_;  // cooldown key -> alertTimestamp
  // K11 cooldown pre-filter (AlertArgs::cool_t): per series, the time of its cooldown key's latest
  // alert; cool_series_ maps a key (hash as in NodeCand::key) to this rank's series (series_mu_)
  double* d_cool_t_ = nullptr;
  std::unordered_map<uint64_t, std::vector<int32_t>> cool_series_;
  double roll_now_ = 0;                    // `now` of the rollover in flight (K11 and the decision)
  int32_t* h_cool_idx_ = nullptr;          // pinned staging of cooldown updates
  double* h_cool_val_ = nullptr;
  size_t cool_cap_ = 0;
  hipEvent_t cool_ev_ = nullptr;
  uint64_t cool_key_of(int32_t s) const;   // (series_mu_ held, or the series_ owner)
  void cool_mark(const std::vector<std::pair<uint64_t, double>>& wins, hipStream_t st);
  void rebuild_cool();
  static std::string node_cool_key(uint64_t k) {
    std::string s(17, '\x02');
    for (int i = 0; i < 16; ++i) s[1 + i] = "0123456789abcdef"[(k >> (60 - 4 * i)) & 15];
    return s;
  }
  static bool parse_node_cool_key(const std::string& s, uint64_t& k) {
    if (s.size() != 17 || s[0] != '\x02') return false;
    k = 0;
    for (int i = 1; i < 17; ++i) {
      const char c = s[i];
      const int v = c >= '0' && c <= '9' ? c - '0' : (c >= 'a' && c <= 'f' ? c - 'a' + 10 : -1);
      if (v < 0) return false;
      k = (k << 4) | (uint64_t)v;
    }
    return true;
  }
  // every cooldown entry, node-wide ones in their string form (checkpoint / export)
  std::vector<std::pair<std::string, double>> cooldown_entries() const {
    std::vector<std::pair<std::string, double>> v(last_alert_.begin(), last_alert_.end());
    for (auto& kv : node_cool_) v.emplace_back(node_cool_key(kv.first), kv.second);
    return v;
  }
  void put_cooldown(const std::string& key, double t) {
    uint64_t k;
    if (parse_node_cool_key(key, k)) node_cool_[k] = t;
    else last_alert_[key] = t;
  }

  // tx upload + release pool
  TxRec* d_tx_ = nullptr;
  TxRec* h_tx_ = nullptr;
  int64_t* d_gid_ = nullptr;
  int64_t* h_gid_ = nullptr;
  int64_t *d_tail_end_ = nullptr, *d_tail_gid_ = nullptr, *d_sort_end_ = nullptr, *d_sort_gid_ = nullptr;
  int64_t *d_pool_end_[2] = {nullptr, nullptr}, *d_pool_gid_[2] = {nullptr, nullptr};
  int pool_cur_ = 0;
  int64_t pool_off_ = 0, pool_n_ = 0, tail_n_ = 0;
  void* d_release_tmp_ = nullptr;
  size_t release_tmp_bytes_ = 0;
  std::map<int64_t, int64_t> pool_bucket_count_;   // endTs bucket -> pending count (host mirror)
  std::map<int64_t, int64_t> pool_exact_edge_;     // endTs == bucket start count
  int64_t* h_release_gid_[2] = {nullptr, nullptr};  // ping-pong D2H targets of released ids
  hipEvent_t ev_rel_[2] = {nullptr, nullptr};
  uint64_t rel_task_[2] = {0, 0};                    // output-lane task that reads each buffer
  // Released db lines get a lane (thread) and a stream of their own (APM_REL_LANE=0: the st / fs
  // output lane, as before): their D2H + emission overlap the st / fs D2H instead of queueing
  // behind it in one FIFO -- the production path is output-lane bound (profiles/r5_e).
  std::unique_ptr<TaskLane> rel_lane_;
  hipStream_t rel_stream_ = nullptr;
  bool rel_lane_on_ = true;
  uint64_t post_rel(std::function<void()> fn);
  void rel_wait(uint64_t task);
  int rel_k_ = 0;
  int64_t next_gid_ = 0;
  // Released-tx line store: each stats batch appends its pending tx lines to one block; the
  // pool payload (gid) is (block << 32 | offset).  A block is freed when its last line is
  // released (lines leave in endTs order, so blocks drain roughly in age order).
  struct LineBlock { std::string data; int64_t live = 0; };
  std::unordered_map<uint32_t, LineBlock> line_blocks_;  // guarded by blocks_mu_ while the lanes run
  std::mutex blocks_mu_;
  std::mutex arena_mu_;
  std::vector<std::string> arena_pool_;          // drained release blocks, reused as shard arenas
  void recycle_arena(std::string&& a);
  uint32_t line_block_seq_ = 0;

  uint32_t last_n_events_ = 0;

  // watermark clock
  double watermark_ = 0;
  uint64_t batch_no_ = 0;

  // K12 formatter tables: names (server + service strings), per-series name refs, emission order
  std::string h_names_;
  std::unordered_map<std::string, int32_t> name_off_;
  std::vector<int32_t> server_name_off_, service_name_off_;
  std::vector<int32_t> h_ser_names_;            // 4 per series
  std::vector<int32_t> h_perm_;
  std::vector<uint64_t> h_perm_key_;  // emit keys of h_perm_, same order
  int64_t perm_uploaded_ = 0;          // d_perm_ holds h_perm_[0, perm_uploaded_)
  bool perm_dirty_ = true;
  size_t names_uploaded_ = 0, names_cap_ = 0;
  int32_t ser_names_uploaded_ = 0;
  char* d_names_ = nullptr;
  int32_t* d_ser_names_ = nullptr;
  int32_t* d_perm_ = nullptr;
  uint32_t *d_fmt_len_ = nullptr, *d_fmt_off_ = nullptr;  // st [S + 1] then fs [S * MAX_LAGS + 1] (len, off)
  int32_t* d_fmt_fallback_ = nullptr;
  void* d_fmt_tmp_ = nullptr;
  size_t fmt_tmp_bytes_ = 0;
  char* d_fmt_out_[2] = {nullptr, nullptr};
  size_t fmt_out_cap_[2] = {0, 0};
  char* h_fmt_out_[2] = {nullptr, nullptr};      // pinned ping-pong staging for the D2H of formatted text
  size_t h_fmt_cap_[2] = {0, 0};
  // APM_FMT_HOST=1: K12 writes the st/fs text straight into h_fmt_out_ (device alias hd_fmt_out_)
  // over the host link -- no HBM round trip, no D2H copy on the output lane
  bool fmt_host_ = false;
  char* hd_fmt_out_[2] = {nullptr, nullptr};
  hipEvent_t ev_fmt_[2] = {nullptr, nullptr};
  uint64_t fmt_task_[2] = {0, 0};
  // Pinned st/fs staging the output lane copies into, a ring deeper than the device double
  // buffer: the sink's spool writers hold a slot until written (zero-copy COPY rows), and with
  // the two device slots the lane waited for the writes of the batch before last (0.42 ms per
  // batch, profiles/r5_q/service_trace_summary.txt).
  char* h_fmt_ring_[FMT_RING] = {};
  size_t h_fmt_ring_cap_[FMT_RING] = {};
  int fmt_ring_k_ = 0;  // stats thread
  // K12's LDS stage: bytes of an average 64-line block of the longer stream in the last batch
  std::atomic<uint32_t> fmt_block_bytes_{0};
  void note_fmt_block(size_t st_bytes, size_t st_lines, size_t fs_bytes, size_t fs_lines) {
    const size_t a = std::max(st_lines ? st_bytes / st_lines : 0, fs_lines ? fs_bytes / fs_lines : 0);
    if (a) fmt_block_bytes_.store((uint32_t)std::min<size_t>(a * 64, 1u << 20), std::memory_order_relaxed);
  }
  int fmt_k_ = 0;
  uint32_t* h_fmt_meta_ = nullptr;               // pinned: per slot k, [4k] st total, [4k+1] fs total
  // pinned: per slot k, the fs row offsets of the last format (K12's scan), so a COPY sink cuts
  // its flushes without scanning the text
  uint32_t* h_fs_off_[2] = {nullptr, nullptr};
  size_t h_fs_off_cap_[2] = {0, 0};
  size_t fs_rows_[2] = {0, 0};
  uint32_t* hd_fmt_meta_ = nullptr;

  // text outputs
  std::string blob_[N_OUT];
  int sink_fd_[N_OUT] = {-1, -1, -1, -1, -1, -1, -1, -1};
  std::shared_ptr<ByteSink> byte_sink_[N_OUT];
  bool fs_copy_ = false;
  bool db_copy_ = false;
  bool rel_copy_ = false;         // the pending release was planned as COPY rows
  bool txcopy_force_fb_ = false;
  // APM_D2H_KERNEL=1: the output lane's D2H of st / fs / db text by the engine's copy kernel
  // (16-byte lanes, at most APM_D2H_BLOCKS workgroups -- default 32 -- into the mapped pinned
  // buffer) instead of hipMemcpyAsync (ROCclr's blit: one 512-lane workgroup on every CU)
  bool d2h_kernel_ = false;
  uint32_t d2h_blocks_ = 32;
  // APM_D2H_SDMA=1: the same copies as hipMemcpyDeviceToDeviceNoCU into the pinned buffer (a DMA
  // engine, no compute units)
  bool d2h_sdma_ = false;
  // APM_D2H_SPLIT=N: lane copies of >= 4 MB in N pieces alternating over out_stream_ and a second
  // output stream (two copies in flight on the host link)
  int d2h_split_ = 1;
  hipStream_t out_stream2_ = nullptr;
  void lane_sync();  // both output streams
  int cu_reserved_ = 0;  // CUs kept out of the parse / stats / output streams (APM_CU_RESERVE)
  void lane_d2h(void* h, const void* d, size_t n, hipStream_t s = nullptr);  // (null: the output stream)  // APM_TXCOPY_FORCE_FALLBACK=1: every release takes the host path (tests)
  uint64_t sink_bytes_[N_OUT] = {0, 0, 0, 0, 0, 0, 0, 0};
  // K14 server rollup + exogenous context
  std::vector<double> h_ctx_;                    // [servers][CTX_FIELDS] (stats thread)
  bool ctx_dirty_ = false;
  // set_server_context -> stats thread: rows tagged with the batch they precede, applied when
  // the stats thread starts that batch (no pipeline drain per JMX sample)
  struct CtxUpdate { uint64_t batch; int32_t server; double row[CTX_FIELDS]; };
  std::mutex ctx_mu_;
  std::vector<CtxUpdate> ctx_pending_;
  void apply_ctx_pending(uint64_t upto);
  size_t roll_cap_ = 0;                          // servers the device buffers hold
  double* d_ctx_ = nullptr;
  unsigned long long* d_roll_acc_ = nullptr;
  double* d_roll_out_ = nullptr;
  double* h_roll_out_ = nullptr;
  int32_t* d_series_server_ = nullptr;
  int32_t series_server_uploaded_ = 0;
  void server_rollup(int64_t edge_ts);
  void format_server_rollup(int64_t edge_ts);
  EngineMetrics metrics_;
  hipEvent_t ev_a_, ev_b_;
};

}  // namespace apm
