// Host join workers: the stateful half of the transaction parser.
//
// The GPU (csrc/kernels/parse.hip) reduces raw log bytes to ordered Event records for the
// relevant lines only.  A JoinShard consumes the events of the files it owns (one shard per
// JVM host) and reproduces the reference's sequential state machines exactly
// (stream_parse_transactions.js:210-731):
//   * SOAP request context -> account capture (:352-376, saveAcctNum :294-327),
//   * EJB and standard CommonTiming entry/exit joins through recordCache (:378-565),
//   * BAF account salvage (:486-504),
//   * the audit-trail state machine (:578-731),
//   * the three NodeCache TTL caches, modelled with the engine's log-time clock: the clock is
//     constant inside a batch and every cache is swept at the batch boundary, so lazy expiry on
//     get/has can never fire mid-batch; need-cache expiry emits records (:226-239).
// Output: completed transactions in line order, tagged for the stats stage or db_insert.
//
// Data layout: keys are 64-bit hashes of the logId bytes (flatmap.h::hash_bytes; no allocation
// on lookup; a 64-bit collision between two live logIds of one JVM is treated as impossible),
// services are interned per shard (hash of the raw name -> compact SvcInfo with the normalized
// global id and the normalized text in one arena, one dictionary lock per new name; the same
// collision stance, backed by a length check), and every TTL cache keeps a FIFO of
// (key, expiry) so a sweep costs O(expired), not O(size).
//
// Memory-level parallelism: the maps are far larger than a core's caches (tens of thousands of
// live logIds per JVM), so process() runs a lookahead over the batch's events and prefetches
// the map slots an event will touch several events before it is handled.  Map values are kept
// to one cache line (Partial 16 B, RecordEntry 56 B).
#pragma once
#include <cstdint>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "../apm_types.h"
#include "flatmap.h"
#include "jsutil.h"

namespace apm {

class BinWriter;
class BinReader;

struct TxOut {
  uint64_t seq;          // merge key: line emissions (1<<63)|(line<<12)|sub; expiries creation<<12|sub
  int32_t server;        // server id (== shard index: the line lives in that shard's text arena)
  int32_t service;       // normalized service id
  int32_t raw_svc;       // the shard's interned raw service id (dense per shard: series lookup key)
  double end_ms;         // endTs (NaN when '')
  double elapsed;        // parseInt(elapsed)
  uint32_t line_off;     // wire-format tx line (entries.js:16-21, no newline) in the shard arena
  uint32_t line_len;
  bool to_db;            // insertToDb (audit non-Provider records)
  bool toplevel;         // service matches /^S:/
};

// Global dictionary of normalized service names shared by all shards.
class Dictionary {
 public:
  int32_t service_id(std::string_view normalized);
  const std::string& service_name(int32_t id) const {
    std::lock_guard<std::mutex> g(mu_);
    return services_[id];
  }
  int32_t n_services() const {
    std::lock_guard<std::mutex> g(mu_);
    return (int32_t)services_.size();
  }
  std::vector<std::string> services_snapshot() const {
    std::lock_guard<std::mutex> g(mu_);
    return std::vector<std::string>(services_.begin(), services_.end());
  }

 private:
  mutable std::mutex mu_;
  std::unordered_map<std::string, int32_t> svc_map_;
  std::deque<std::string> services_;  // stable references
};

struct FileInfo {
  std::string path;
  int32_t server;
  uint8_t kind;  // FileKind
};

struct JoinConfig {
  double record_ttl_ms = 120000;
  double acct_ttl_ms = 120000;
  double need_ttl_ms = 30000;
  TzTable tz;
};

struct JoinCounters {
  uint64_t events = 0, tx = 0, tx_db = 0, expired_partials = 0, need_expired = 0;
  uint64_t ejb_exit_unmatched = 0, invalid_acct = 0, audit_errors = 0, host_fallback = 0;
  // device join capacity: losses (must stay 0: every structure grows) and growth / chain use
  uint64_t partial_overflow = 0, need_overflow = 0, table_full = 0, pool_exhausted = 0;
  uint64_t chain_partial_blocks = 0, chain_need_blocks = 0, chain_logid_blocks = 0;
  uint64_t table_slots = 0, table_grows = 0, table_rebuilds = 0, need_arena_entries = 0, arena_grows = 0, trims = 0;
  uint64_t chain_pool_blocks = 0, pool_grows = 0;
  uint64_t host_events = 0;  // events resolved by the host pre-pass (audit blocks, PM_HOST lines)
};

// Cache-line aligned: the shards of a process are joined concurrently, one worker each, and
// every event writes the shard's counters / cursor / output vector.  Unaligned, neighbouring
// shards shared boundary lines (one's write cursor next to the other's config), and the
// resulting false sharing made the parallel join ~3x slower than the same join run alone.
class alignas(128) JoinShard {
 public:
  JoinShard(const JoinConfig& cfg, Dictionary* dict, const std::vector<FileInfo>* files,
            const std::vector<std::string>* servers)
      : cfg_(cfg), dict_(dict), files_(files), servers_(servers), acct_(1 << 16), record_(1 << 16), need_(1 << 12),
        raw_svc_map_(1 << 12) {}

  void begin_batch(double now_ms, uint64_t batch_no);
  // Process the events of one batch that belong to this shard. `bytes` is the host copy of the
  // batch, `chunk_file` maps chunk index -> file id.
  void process(const Event* ev, size_t n, const uint8_t* bytes, const std::vector<int32_t>& chunk_file);

  std::vector<TxOut>& out() { return out_; }
  // Formatted tx lines of this batch (TxOut::line_off/len index into it); cleared by begin_batch.
  std::string& text() { return text_; }
  JoinCounters counters;

  // checkpoint (checkpoint.cpp)
  void save(BinWriter& w);
  void load(BinReader& r);

  size_t n_partial_logids() const { return record_.size(); }
  size_t n_need_logids() const { return need_.size(); }
  size_t n_acct() const { return acct_.size(); }

 private:
  // start '' (unparseable timestamp) is start_ms = NaN: outputRecord treats both the same way
  struct Partial { int32_t svc; int32_t server; double start_ms; };
  struct Need {
    int32_t svc;          // shard-local raw service id
    int32_t server;
    double start_ms; bool start_empty;
    double end_ms; bool end_empty;
    double elapsed;
    double alt_acct;      // parseInt(altAcctNum || '')
    bool insert_to_db;
  };
  struct AcctEntry { double acct = 0; double exp = 0; };
  struct RecordEntry { double exp = 0; SmallVec<Partial, 2> items; };
  struct NeedEntry { double exp = 0; uint64_t created = 0; std::string log_id; std::vector<Need> items; };
  struct SoapCtx { std::string log_id; bool has_log_id = false; bool pull_next = false; };
  struct AuditItem { std::string elapsed; bool has_start = false; std::string start_ts; };
  struct AuditCtx {
    std::vector<std::pair<std::string, std::pair<std::string, std::string>>> autr_map;  // autrId -> (logId, alt)
    bool active = false;
    std::string active_log_id, active_alt, active_service;
    bool has_active_service = false;
    bool elapsed_flag = false, sw_flag = false;
    std::vector<std::pair<std::string, std::deque<AuditItem>>> service_map;
  };
  struct RawService { std::string raw; std::string norm; int32_t norm_id; bool toplevel; uint64_t hash; };
  struct SvcInfo { uint32_t norm_off, norm_len; int32_t norm_id; uint32_t raw_len; bool toplevel; };
  // per-file SOAP request context, indexed by file id (erase keeps the string's storage, so a
  // view of the last logId stays valid until the file's next request line)
  struct SoapTable {
    std::vector<SoapCtx> v;
    std::vector<uint8_t> present;
    SoapCtx* find(int32_t f) { return (f >= 0 && (size_t)f < v.size() && present[f]) ? &v[f] : nullptr; }
    SoapCtx& put(int32_t f) {
      if ((size_t)f >= v.size()) { v.resize((size_t)f + 1); present.resize((size_t)f + 1, 0); }
      present[f] = 1;
      return v[f];
    }
    void erase(int32_t f) { if (f >= 0 && (size_t)f < present.size()) present[f] = 0; }
    size_t size() const { size_t n = 0; for (uint8_t p : present) n += p; return n; }
    void clear() { v.clear(); present.clear(); }
  };

  static uint64_t key_of(std::string_view s) { return hash_bytes(s.data(), s.size()); }
  static uint64_t svc_hash(bool ejb, std::string_view name) {
    return hash_bytes(name.data(), name.size(), ejb ? kHashSeedEjb : kHashSeed);
  }
  int32_t raw_service(std::string_view raw) { return raw_service(false, raw); }
  int32_t raw_service(bool ejb, std::string_view name) { return raw_service(svc_hash(ejb, name), ejb, name); }
  // interned ("S:" if ejb) + name with its hash precomputed (PM_KEYS events: by the parse kernel)
  int32_t raw_service(uint64_t h, bool ejb, std::string_view name);
  int32_t intern_service(std::string raw, uint64_t h);
  void prefetch_event(const Event& e, const uint8_t* bytes);
  void sweep();
  void expire_need(NeedEntry& nm);
  NeedEntry& need_map(uint64_t key, std::string_view log_id);
  RecordEntry& record_map(uint64_t key);
  void save_acct(std::string_view acct, int32_t file, int source, std::string_view alt_log_id, uint64_t seq);
  void output(int32_t server, int32_t svc, std::string_view log_id, double acct, double start_ms, bool start_empty,
              double end_ms, bool end_empty, double elapsed, bool to_db, uint64_t seq);
  std::string_view baf_acct(const Event& e, std::string_view line, std::string_view tok3, int32_t file, std::string_view log_id,
                            uint64_t seq, std::string& scratch);

  void on_soap(const Event& e, std::string_view line, int32_t file, uint64_t seq);
  void on_ejb(const Event& e, std::string_view line, int32_t file, bool entry, uint64_t seq);
  void on_ct(const Event& e, std::string_view line, int32_t file, bool entry, uint64_t seq);
  void on_app(const Event& e, std::string_view line, int32_t file, uint64_t seq);

  JoinConfig cfg_;
  Dictionary* dict_;
  const std::vector<FileInfo>* files_;
  const std::vector<std::string>* servers_;
  std::string text_;
  double now_ = 0;
  uint64_t batch_no_ = 0;
  uint64_t cur_line_ = 0;
  FlatMap<AcctEntry> acct_;
  FlatMap<RecordEntry> record_;
  FlatMap<NeedEntry> need_;
  std::deque<std::pair<uint64_t, double>> acct_fifo_, record_fifo_, need_fifo_;
  SoapTable soap_;
  std::unordered_map<int32_t, AuditCtx> audit_;
  FlatMap<int32_t> raw_svc_map_;  // svc_hash(raw name) -> id + 1
  std::vector<RawService> raw_svc_;  // cold: checkpoint / collision path
  std::vector<SvcInfo> svc_info_;    // hot: indexed by raw id
  std::string svc_text_;             // normalized names, SvcInfo::norm_off/len
  std::vector<TxOut> out_;
  uint32_t sub_ = 0;
};

}  // namespace apm
