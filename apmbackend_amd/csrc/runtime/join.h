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
//   * the three NodeCache TTL caches, modelled with the engine's log-time clock: lazy expiry on
//     get/has plus a sweep at every batch boundary, need-cache expiry emitting records (:226-239).
// Output: completed transactions in line order, tagged for the stats stage or db_insert.
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
#include "jsutil.h"

namespace apm {

struct TxOut {
  uint64_t seq;          // merge key: line emissions (1<<63)|(line<<12)|sub; expiries creation<<12|sub
  int32_t server;        // server id
  int32_t service;       // normalized service id
  std::string log_id;
  double acct;           // parseInt(acctNum)      (NaN prints "NaN")
  double start_ms;       // startTs as TxEntry holds it (parseInt of startMs)
  double end_ms;         // endTs (NaN when '')
  double elapsed;        // parseInt(elapsed)
  bool to_db;            // insertToDb (audit non-Provider records)
  bool toplevel;         // service matches /^S:/
};

// Global dictionaries shared by all shards (mutex-protected inserts, lock-free reads of
// per-shard caches).
class Dictionary {
 public:
  int32_t service_id(std::string_view normalized);
  const std::string& service_name(int32_t id) const { return services_[id]; }
  int32_t n_services() const { return (int32_t)services_.size(); }
  std::vector<std::string> services_snapshot() const {
    std::lock_guard<std::mutex> g(mu_);
    return services_;
  }

 private:
  mutable std::mutex mu_;
  std::unordered_map<std::string, int32_t> svc_map_;
  std::vector<std::string> services_;
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
};

class JoinShard {
 public:
  JoinShard(const JoinConfig& cfg, Dictionary* dict, const std::vector<FileInfo>* files)
      : cfg_(cfg), dict_(dict), files_(files) {}

  void begin_batch(double now_ms, uint64_t batch_no);
  // Process the events of one batch that belong to this shard. `bytes` is the host copy of the
  // batch, `chunk_file` maps chunk index -> file id.
  void process(const Event* ev, size_t n, const uint8_t* bytes, const std::vector<int32_t>& chunk_file);

  std::vector<TxOut>& out() { return out_; }
  JoinCounters counters;

  // checkpoint support (text form, see engine checkpoint)
  size_t n_partial_logids() const { return record_.size(); }
  size_t n_need_logids() const { return need_.size(); }
  size_t n_acct() const { return acct_.size(); }

 private:
  struct Partial { std::string service_raw; int32_t server; double start_ms; bool start_empty; };
  struct Need {
    std::string service_raw;
    int32_t server;
    double start_ms; bool start_empty;
    double end_ms; bool end_empty;
    double elapsed;
    std::string alt_acct;  // altAcctNum ('' if none)
    bool insert_to_db;
  };
  template <class V> struct TtlEntry { V v; double exp; };
  struct RecordMap { std::vector<Partial> items; };
  struct NeedMap { std::vector<Need> items; uint64_t created = 0; };
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

  // NodeCache-like helpers (insertion-ordered where order is observable)
  template <class M> bool alive(M& m, const std::string& k, bool is_need);
  void sweep();
  void expire_need(const std::string& log_id, NeedMap& nm);
  void save_acct(std::string_view acct, int32_t file, int source, std::string_view alt_log_id, uint64_t seq);
  NeedMap& need_map(const std::string& log_id);
  void output(int32_t server, std::string_view service_raw, std::string_view log_id, double acct,
              double start_ms, bool start_empty, double end_ms, bool end_empty, double elapsed, bool to_db,
              uint64_t seq);
  std::string baf_acct(std::string_view line, const std::vector<std::string_view>& toks, int32_t file,
                       std::string_view log_id, uint64_t seq);

  void on_soap(const Event& e, std::string_view line, int32_t file, uint64_t seq);
  void on_ejb(const Event& e, std::string_view line, int32_t file, bool entry, uint64_t seq);
  void on_ct(const Event& e, std::string_view line, int32_t file, bool entry, uint64_t seq);
  void on_app(const Event& e, std::string_view line, int32_t file, uint64_t seq);

  JoinConfig cfg_;
  Dictionary* dict_;
  const std::vector<FileInfo>* files_;
  double now_ = 0;
  uint64_t batch_no_ = 0;
  uint64_t cur_line_ = 0;
  // caches: key -> entry; insertion order tracked in parallel deques for sweeps
  std::unordered_map<std::string, TtlEntry<std::string>> acct_;
  std::unordered_map<std::string, TtlEntry<RecordMap>> record_;
  std::unordered_map<std::string, TtlEntry<NeedMap>> need_;
  std::deque<std::pair<std::string, double>> need_order_;  // (logId, exp) FIFO for expiry emission
  std::unordered_map<int32_t, SoapCtx> soap_;
  std::unordered_map<int32_t, AuditCtx> audit_;
  std::vector<TxOut> out_;
  uint32_t sub_ = 0;
};

}  // namespace apm
