// Host driver of the GPU join (kernels/devjoin.hip): one per engine.
//
// Per batch (ingest thread):
//   1. the parse stream selects the events the GPU does not resolve alone (apm_dj_select_host)
//      and copies them to pinned memory with the parse counts;
//   2. host pre-pass (this file): the field re-derivation of PM_HOST lines (and of audit lines
//      the GPU cannot read alone) becomes HostOps (sorted by event);
//   3. join kernels (ops, audit trail K5, SOAP scan, grouping, expiry, group walk, placement)
//                                                                                   -> sync A;
//   4. new (server, raw service) names are interned on the host and the registry updated;
//   5. resolve + line lengths + scans, the batch's ring region and write verdict (placed on the
//      device: no host sync here);
//   6. tx text into the HBM ring, stats hand-off arrays, rollover candidates       -> sync C.
// The stats thread then consumes the slot's device arrays (TxRec / raw id / ring gid), exactly
// where the host join handed it TxOut vectors before.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../apm_types.h"
#include "../kernels/devjoin_api.h"
#include "join.h"

namespace apm {

struct DevJoinConfig {
  uint32_t max_events = 1u << 20;   // events (relevant lines) per batch (< 2^21: packed selection scan)
  uint64_t max_batch_bytes = 64ull << 20;
  uint32_t max_chunks = 4096;
  int table_bits = 21;              // key-table slots (KeyState, 128 B)
  int reg_bits = 20;                // service registry slots
  uint32_t max_raw = 1u << 20;      // distinct (server, raw service)
  uint32_t arena_cap = 1u << 20;    // NeedEnt entries (512 B), power of two (grows)
  uint32_t pool_blocks = 0;         // initial chain-block pool (256 B blocks; 0 = auto, grows)
  uint64_t ring_bytes = 4ull << 30; // tx text ring (power of two)
  double record_ttl_ms = 120000, acct_ttl_ms = 120000, need_ttl_ms = 30000;
  TzTable tz{};
  int device = 0;
};

// Result of one batch for the stats thread (device arrays live in the slot until released).
struct DevJoinBatch {
  int slot = 0;
  uint32_t n_out = 0, n_stats = 0, n_db = 0, n_dropped = 0;
  std::vector<std::pair<uint32_t, int64_t>> cands;      // (stats position, bucket), ascending
  std::vector<std::pair<uint32_t, int32_t>> unresolved; // (stats position, raw id), ascending
  std::string text_tx, text_db;                         // "transactions" / "audit_db" streams
  uint64_t ring_base = 0;
  int64_t max_bucket = INT64_MIN;
  TxRec* d_tx = nullptr;
  int32_t* d_raw = nullptr;
  int64_t* d_gid = nullptr;
};

class DeviceJoin {
 public:
  DeviceJoin(const DevJoinConfig& cfg, Dictionary* dict, const std::vector<FileInfo>* files,
             const std::vector<std::string>* servers);
  ~DeviceJoin();

  // device buffers the parse kernels of slot k write into
  uint8_t* d_bytes(int k) { return sl_[k].d_bytes; }
  // A third batch buffer for the two-ahead H2D (Engine::stage_batch), allocated on first use;
  // swap_stage(k) hands it to slot k (whose previous buffer becomes the staging buffer).
  uint8_t* d_stage() {
    if (!d_stage_bytes_) {
      d_stage_bytes_ = (uint8_t*)dmalloc(cfg_.max_batch_bytes + 256);
      // dmalloc's zero fill is queued on the join stream: the staged copy (another stream) must
      // not land before it (seen: a staged batch parsed as zeros, test_two_ahead_input_staging_*)
      HIP_OK(hipStreamSynchronize(stream_));
    }
    return d_stage_bytes_;
  }
  void swap_stage(int k) { std::swap(sl_[k].d_bytes, d_stage_bytes_); }
  Event* d_events(int k) { return sl_[k].d_events; }
  // after the parse kernels (parse stream): select host events, queue their D2H (speculative)
  void select_host(int k, const uint32_t* d_n_ev, uint32_t max_ev, hipStream_t ps);
  // chunk tables of slot k for the SOAP chain (host computes next / first per file)
  void set_chunks(int k, const std::vector<int32_t>& chunk_file, const uint32_t* d_chunk_file,
                  const uint8_t* d_chunk_kind, hipStream_t ps);
  // after the parse stream synced: finish the host-event copy (n_ev known)
  void finish_select(int k, hipStream_t ps);
  // the batch join; host_bytes = the host copy of the batch (same layout as d_bytes(k))
  // `parallel(n, fn)` runs fn(0..n-1) on the engine's worker pool (host pre-pass per file)
  using ParallelFor = std::function<void(int, const std::function<void(int)>&)>;
  // `meanwhile` runs on this thread after the join kernels are queued, before the first wait
  void run(int k, const uint8_t* host_bytes, uint32_t n_ev, uint64_t n_bytes, double now, uint64_t batch_no, bool want_tx,
           bool want_db, DevJoinBatch& out, const ParallelFor& parallel = nullptr,
           const std::function<void()>* meanwhile = nullptr);
  // the host pre-pass of the NEXT batch (slot k, its parse finished), run on another thread while
  // this batch's join completes; run(k) then uploads its ops instead of doing the pre-pass
  // itself.  The pre-pass is stateless (field derivation only), so the result is the same.
  // The caller orders it: run(k) starts only after prepass_ahead(k) returned.
  void prepass_ahead(int k, const uint8_t* host_bytes, const ParallelFor& parallel);
  // the stats thread finished with slot k's arrays (event recorded on its stream)
  void release_slot(int k, hipStream_t stats_stream);

  // raw service table for the stats thread (append-only, never reallocated)
  int32_t raw_server(int32_t raw) const { return raw_info_[raw].server; }
  int32_t raw_service(int32_t raw) const { return raw_info_[raw].norm_id; }
  int32_t n_raw() const { return n_raw_.load(std::memory_order_acquire); }
  int32_t* d_raw_series() { return d_raw_series_; }

  // text ring (virtual positions; physical = pos & (cap - 1))
  char* ring() { return d_ring_; }
  uint64_t ring_cap() const { return cfg_.ring_bytes; }
  // stats thread: lowest position still referenced (pool / tail / unprocessed batches)
  void set_ring_low(uint64_t low);
  uint64_t ring_head() const { return ring_head_.load(std::memory_order_acquire); }
  uint64_t ring_low() const { return ring_low_.load(std::memory_order_acquire); }
  uint64_t keys_live() const { return keys_live_ + keys_since_rebuild_; }
  uint64_t need_live() const { return arena_head_ - (regions_.empty() ? arena_head_ : regions_.front().lo); }
  // reserve `bytes` at the ring head (thread-safe; relocation by the stats thread also uses it)
  uint64_t ring_reserve(uint64_t bytes);
  void reset_ring(uint64_t head);  // checkpoint load: pending lines were placed at [0, head)

  JoinCounters counters() const;
  // occupancy of the join caches at clock `now` (join stream idle): table slots, occupied, acct
  // live, record live, open partials, need live -- the reference's CACHE_STATS
  // (sync = false: the counts of the previous call, the new count queued -- stat lines)
  std::vector<uint64_t> cache_stats(double now, bool sync = true);

  // checkpoint of the GPU join state (checkpoint.cpp): key table (live entries), need arena
  // (live regions), SOAP contexts, service registry, audit-trail carry, counters
  void save(class BinWriter& w);
  void load(class BinReader& r);
  // phase boundaries of the last run() (steady-clock ms): prepass, join launched, sync A,
  // registered, plan queued, sync C, end -- for the engine's stage trace
  static constexpr int kPhases = 8;
  double phase_t[kPhases + 1] = {0};
  std::vector<std::pair<const char*, std::pair<double, double>>> spans;  // finer trace spans of run()
  std::vector<std::pair<const char*, std::pair<double, double>>> save_spans;  // spans of the last save()
  const JoinCounts& last_counts() const { return *h_counts_; }
  size_t device_bytes() const { return device_bytes_; }
  // requestGC (join stream idle, between batches): the grow-only key table and need arena go
  // back to the smallest power of two (not below their configured size) that keeps their live
  // entries at <= 1/4 load, the spare table and text staging are released.  Returns bytes freed.
  size_t trim(double now);

 private:
  struct Slot {
    uint8_t* d_bytes = nullptr;
    Event* d_events = nullptr;
    uint8_t* host_flag = nullptr;
    Event* d_host_ev = nullptr;
    uint32_t* d_host_idx = nullptr;
    uint32_t* d_mh_idx = nullptr;      // audit map / header events
    uint32_t* d_walk_idx = nullptr;    // audit block-walk events
    AudF* d_aud = nullptr;             // audit fields per event (parse-side selection writes them)
    SelCount* d_n_host = nullptr;
    Event* h_host_ev = nullptr;        // pinned
    uint32_t* h_host_idx = nullptr;    // pinned
    SelCount* h_n_host = nullptr;      // pinned
    uint32_t spec = 0;                 // host events already copied speculatively
    int32_t* d_chunk_next = nullptr;
    uint8_t* d_chunk_first = nullptr;
    int32_t* h_chunk_next = nullptr;   // pinned
    uint8_t* h_chunk_first = nullptr;  // pinned
    const uint32_t* d_chunk_file = nullptr;
    const uint8_t* d_chunk_kind = nullptr;
    uint32_t n_chunks = 0;
    std::vector<int32_t> chunk_file;
    // stats hand-off arrays
    TxRec* d_tx = nullptr;
    int32_t* d_tx_raw = nullptr;
    int64_t* d_tx_gid = nullptr;
    hipEvent_t free_ev = nullptr;      // recorded by the stats thread after its last use
    bool used = false;
  } sl_[2];

  struct RawInfo { int32_t server; int32_t norm_id; uint64_t svc; };

  void* dmalloc(size_t bytes);
  // One file's share of the host pre-pass (field re-derivation of the lines of one file)
  struct PrepassTask {
    int32_t file = -1;
    std::vector<uint32_t> idx;   // host-event indices (ascending)
    std::vector<HostOp> hops;
    std::string hbuf;
    uint64_t audit_errors = 0, invalid_acct = 0, pm_host = 0;
    uint32_t put(std::string_view s) { const uint32_t o = (uint32_t)hbuf.size(); hbuf.append(s.data(), s.size()); return o; }
  };
  void host_prepass(int k, const uint8_t* host_bytes, uint32_t n_host, const ParallelFor& parallel,
                    std::vector<HostOp>& hops, std::string& hbuf);
  void host_event(PrepassTask& t, const Event& e, uint32_t ev, const uint8_t* host_bytes);
  void on_app(PrepassTask& t, const Event& e, uint32_t ev, std::string_view line);
  void save_tables(class BinWriter& w);  // checkpoint: key table, need arena, chain blocks (memory writer)
  // K5 carry: generation g of the audit state (devjoin_api.h AudGen); capacity for the next batch
  void aud_reserve(AudGen& g, uint32_t autr, uint32_t items, uint64_t txt);
  int32_t intern_name(const std::string& s);
  void register_misses(const uint8_t* host_bytes, uint32_t n_miss, hipStream_t s);
  // Capacity before a batch of n_ev events (`bytes` of lines + host-op bytes): the key table keeps
  // every key of the batch under half load (rebuilt, then doubled), the need arena can open one
  // entry per event, the chain pool covers one block per event plus every logId byte.  All grow;
  // none drops state.  Expiring need regions are still live here (they are emitted this batch).
  void ensure_capacity(uint32_t n_ev, uint64_t bytes, double now);
  void rebuild_table(double now, uint32_t new_cap);
  void rebuild_table_async(double now);
  // a rebuild queued without waiting for its live count is safe only if the worst case -- every
  // key since the last count still live, plus n_ev new keys -- stays within 5/8 of the table
  bool async_rebuild_fits(uint64_t n_ev) const {
    return (keys_live_ + keys_since_rebuild_ + n_ev) * 8 <= (uint64_t)table_cap_ * 5;
  }
  void ensure_rest(uint32_t n_ev, uint64_t bytes);  // ensure_capacity after the key table
  void rebuild_inplace(double now);                  // same-size rebuild, queued (count -> d_live_)
  static bool rebuild_copy();                        // APM_REBUILD_COPY=1: reinsert into the spare (A/B)
  void idle_upkeep(double now, uint32_t n_next);    // end of a batch: table upkeep while the host works
  void grow_arena(uint32_t new_cap, uint64_t lo);
  void grow_pool(uint64_t need_free);
  uint64_t pool_avail(bool exact);
  void ensure_tmp();
  void dfree(void* p, size_t bytes);

  DevJoinConfig cfg_;
  uint32_t init_table_cap_ = 0, init_arena_cap_ = 0;  // configured sizes: trim never goes below
  Dictionary* dict_;
  const std::vector<FileInfo>* files_;
  const std::vector<std::string>* servers_;
  hipStream_t stream_ = nullptr;  // join stream
  // flags of the host-op staging (read by a kernel over the host link): APM_HOPS_NC=1 allocates it
  // non-coherent (the GPU may then fetch whole cache lines)
  static unsigned host_flags_() {
    static const unsigned f = [] {
      const char* e = std::getenv("APM_HOPS_NC");
      return (e && e[0] == '1') ? (unsigned)hipHostMallocNonCoherent : (unsigned)hipHostMallocDefault;
    }();
    return f;
  }
  size_t device_bytes_ = 0;
  uint8_t* d_stage_bytes_ = nullptr;  // two-ahead H2D target (d_stage / swap_stage)
  std::vector<void*> allocs_;

  // host pre-pass output of the current batch
  std::vector<HostOp> hops_;
  std::string hbuf_;
  std::vector<HostOp> hops_ahead_;  // prepass_ahead's result for slot ahead_k_
  std::string hbuf_ahead_;
  int ahead_k_ = -1;
  HostOp* h_hops_ = nullptr;     // pinned
  uint8_t* h_hbuf_ = nullptr;    // pinned
  const void* hd_hops_ = nullptr;  // device views (apm_copy reads them over the host link)
  const void* hd_hbuf_ = nullptr;
  const void* hd_exp_ = nullptr;
  size_t h_hops_cap_ = 0, h_hbuf_cap_ = 0;
  HostOp* d_hops_ = nullptr;
  uint8_t* d_hbuf_ = nullptr;
  size_t d_hops_cap_ = 0, d_hbuf_cap_ = 0;
  std::vector<PrepassTask> tasks_;
  uint32_t last_host_ = 0;
  void* d_sel_tmp_ = nullptr;  // rocprim scratch of the host-event selection (parse stream)
  size_t sel_tmp_bytes_ = 0;
  uint64_t audit_errors_ = 0, host_pm_ = 0, host_invalid_acct_ = 0, host_events_ = 0, events_ = 0, tx_ = 0, tx_db_ = 0;

  // device state
  DJArgs a_{};
  DJFormatArgs f_{};
  KeyState* d_table_ = nullptr;
  // dense key array probed by k_claim (DJArgs::keys), re-derived from the table after every
  // rewrite other than k_claim's (rebuilds, restore): sync_keys()
  uint64_t* d_keys_ = nullptr;
  uint32_t keys_cap_ = 0;
  bool keys_stale_ = true;
  void sync_keys();
  unsigned long long* d_cstats_ = nullptr;  // cache_stats result (5 counters)
  unsigned long long* h_cstats_ = nullptr;  // (pinned)
  unsigned long long cstats_last_[5] = {0, 0, 0, 0, 0};
  uint32_t cstats_cap_ = 0, cstats_last_cap_ = 0;
  hipEvent_t cstats_ev_ = nullptr;
  bool cstats_pending_ = false, cstats_have_ = false;
  KeyState* d_table_spare_ = nullptr;  // same-size rebuild target (no allocation per rebuild)
  uint32_t table_cap_ = 0;
  int table_bits_ = 0;
  uint64_t keys_since_rebuild_ = 0, keys_live_ = 0;
  bool live_pending_ = false;  // an in-order rebuild's live count is on its way to h_live_
  hipEvent_t live_ev_ = nullptr;  // recorded after that count's D2H
  bool spare_clean_ = false;   // d_table_spare_ is zeroed (the next rebuild skips its memset)
  uint32_t* d_rb_scratch_ = nullptr;  // per-segment cluster starts of the in-place rebuild
  size_t rb_scratch_bytes_ = 0;
  uint8_t* d_pool_ = nullptr;          // chain blocks
  uint32_t* d_pool_ring_ = nullptr;    // free-index ring
  uint32_t pool_n_ = 0;                // blocks (power of two)
  unsigned long long* h_live_ = nullptr;  // pinned
  // growth events (reported in counters())
  uint64_t table_grows_ = 0, arena_grows_ = 0, pool_grows_ = 0, table_rebuilds_ = 0, trims_ = 0;
  RegSlot* d_reg_ = nullptr;
  RegMiss* d_miss_ = nullptr;
  RegMiss* h_miss_ = nullptr;
  uint32_t miss_cap_ = 0;
  NeedEnt* d_arena_ = nullptr;
  uint64_t arena_head_ = 0;      // virtual
  struct Region { uint64_t lo, hi; double exp; };
  std::deque<Region> regions_;   // live need regions, creation order
  uint64_t* d_exp_lo_ = nullptr;
  uint64_t* d_exp_hi_ = nullptr;
  uint64_t* h_exp_ = nullptr;    // pinned [2][64]
  SoapState* d_soap_ = nullptr;
  // audit trail (K5): carry generations (batch k reads aud_gen_[aud_cur_], writes the other),
  // per-event fields, key sort, walk tables
  AudGen aud_gen_[2]{};
  int aud_cur_ = 0;
  uint64_t* d_sel_val_ = nullptr;  // selection scan (parse stream, one batch at a time)
  uint64_t* d_sel_pos_ = nullptr;
  uint64_t *d_aud_key_ = nullptr, *d_aud_key_sorted_ = nullptr;
  uint32_t *d_aud_ord_ = nullptr, *d_aud_ord_sorted_ = nullptr;
  uint32_t aud_key_cap_ = 0;
  uint32_t* d_walk_lo_ = nullptr;
  int32_t* d_file_first_ = nullptr;
  AudItem* d_aud_slots_ = nullptr;
  uint32_t aud_slots_cap_ = 0;
  // checkpoint: pinned bounce for the large D2H reads of save()
  static constexpr size_t kCkBounce = 32u << 20;
  char* h_ck_bounce_ = nullptr;
  uint32_t soap_cap_ = 0;
  int32_t* d_file_server_ = nullptr;
  uint64_t* d_file_skey_ = nullptr;      // per file: world-invariant key of its server (gkey_of)
  uint64_t* d_file_fkey_ = nullptr;      // per file: world-invariant key of the file (aud_key)
  std::vector<uint64_t> h_file_skey_, h_file_fkey_;
  void sync_file_keys();
  size_t files_uploaded_ = 0;
  RawSvc* d_rawtab_ = nullptr;
  int32_t* d_raw_series_ = nullptr;
  int32_t* d_raw_first_ = nullptr;
  std::vector<RawInfo> raw_info_;          // reserved to max_raw: stable for the stats thread
  std::atomic<int32_t> n_raw_{0};
  std::string names_;
  std::unordered_map<std::string, int32_t> name_off_;
  char* d_names_ = nullptr;
  size_t names_uploaded_ = 0, names_cap_ = 0;
  int32_t* d_reg_fill_ = nullptr;          // (slot, raw) pairs
  int32_t* h_reg_fill_ = nullptr;
  RawSvc* h_rawtab_ = nullptr;
  // outputs
  TxDev* d_out_ = nullptr;
  uint32_t out_cap_ = 0;
  uint32_t* d_lens_ = nullptr;
  uint32_t* d_offs_ = nullptr;
  int64_t* d_bucket_ = nullptr;
  int64_t* d_bmax_ = nullptr;
  uint32_t* d_cand_ = nullptr;
  int64_t* d_cand_bucket_ = nullptr;
  uint32_t* d_unres_ = nullptr;
  uint32_t* h_cand_ = nullptr;
  int64_t* h_cand_bucket_ = nullptr;
  uint32_t* h_unres_ = nullptr;
  char* d_txt_tx_ = nullptr;
  char* d_txt_db_ = nullptr;
  size_t txt_cap_ = 0;
  char* h_txt_ = nullptr;
  size_t h_txt_cap_ = 0;
  // copied back before their sizes are known (no sync between the plan and the write): the
  // previous batch's sizes x 2; a larger batch copies the rest after sync C
  uint32_t last_tx_bytes_ = 0, last_db_bytes_ = 0, last_cands_ = 0;
  uint64_t* d_ring_pos_ = nullptr;  // this batch's ring base (k_plan_totals)
  // op grouping by slot lists (DJArgs::slot_head): one head per table slot, all empty between
  // batches (so a same-size rebuild keeps them valid); re-made when the table size changes
  uint32_t* d_slot_head_ = nullptr;
  uint32_t heads_cap_ = 0;
  uint32_t* d_big_ = nullptr;
  bool group_sort_ = false;  // APM_OPSORT=sort
  uint64_t write_regrows_ = 0;      // write passes redone after the text staging grew
  void ensure_txt(size_t bytes);
  void* d_tmp_ = nullptr;
  size_t tmp_bytes_ = 0;
  JoinCounts* d_counts_ = nullptr;
  JoinCounts* h_counts_ = nullptr;
  unsigned long long* d_live_ = nullptr;
  // scratch of the join kernels (sized by max_events)
  JOp* d_ops_ = nullptr;
  uint8_t* d_soap_code_ = nullptr;
  double* d_soap_num_ = nullptr;
  uint64_t* d_soap_hash_ = nullptr;
  uint32_t* d_chunk_ev_lo_ = nullptr;
  uint32_t* d_seg_f_ = nullptr;
  uint32_t* d_seg_in_ = nullptr;
  uint64_t* d_chain_hash_ = nullptr;
  uint32_t *d_op_slot_ = nullptr, *d_op_slot_sorted_ = nullptr, *d_op_idx_ = nullptr, *d_op_idx_sorted_ = nullptr;
  uint64_t *d_exp_key_ = nullptr, *d_exp_key_sorted_ = nullptr;
  uint32_t *d_exp_idx_ = nullptr, *d_exp_idx_sorted_ = nullptr, *d_exp_cnt_ = nullptr, *d_exp_pos_ = nullptr;
  uint32_t exp_cap_ = 0;
  uint32_t* d_out_cnt_ = nullptr;
  uint32_t* d_out_pos_ = nullptr;
  TxDev* d_stage_ = nullptr;
  DJOverflow* d_ovf_ = nullptr;
  // ring
  char* d_ring_ = nullptr;
  std::mutex ring_mu_;
  std::atomic<uint64_t> ring_head_{0};
  std::atomic<uint64_t> ring_low_{0};
};

}  // namespace apm
