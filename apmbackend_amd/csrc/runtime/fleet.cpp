// Node-wide service registry and the fb (fleet baseline) stream.
//
// The fleet all-reduce (engine.cpp fleet_exchange_upto) sums a [slot][lag][stat][3] moments
// matrix over the ranks.  Each rank interns services in its own first-appearance order, so the
// matrix row of a service must be a node-wide *slot*, agreed without a coordinator:
//   * the stats thread queues every service of a newly created series (hash + name, tagged with
//     the batch it was packed in);
//   * the ingest thread's lock-step all-reduce carries "entries pending" (MAX over ranks); when
//     any rank has some, every rank enters one all-gather of fixed-size blocks
//     {count, (hash, name)...} and assigns slots to unseen hashes in rank order -- the same
//     table on every rank;
//   * the stats thread adopts the (service, slot) pairs at the pack of the batch they were
//     assigned in (a batch tag), so every rank starts counting a service in the same exchange.
// Only entries queued two or more batches back are sent: post_stats(k - 1) returning guarantees
// the stats thread finished batch k - 2 on every rank, so block contents do not depend on thread
// timing and the slot numbering is deterministic.
//
// fb rows (every rank, its slice of the slots): after the all-reduce of a batch whose stats
// performed a rollover, K12's fleet formatter (format.hip) turns the merged moments into one row
// per (service, LAG) -- the fleet
// mean and spread of the per-JVM z-score baselines ("is getFoo slow on one JVM or everywhere?",
// SURVEY §2.4) -- either as `fb|...` wire lines or as COPY rows for the DB sink
// (apm_fleet_stats), D2H'd and emitted by the output lane.
#include <hip/hip_runtime.h>

#include <cstring>

#include <algorithm>

#include "engine.h"

namespace apm {

namespace {
uint64_t fnv1a(const std::string& s) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : s) { h ^= c; h *= 1099511628211ull; }
  return h ? h : 1;
}
struct RegHdr { int32_t count, bytes; };
struct RegEntry { uint64_t hash; uint32_t off, len; };
}  // namespace

int32_t Engine::svc_key(int32_t s) const {
  const int32_t v = series_[s].service;
  if (!coll_ || !lockstep_) return v;  // one rank without lock-step: the dictionary id is node-wide
  return (size_t)v < fleet_slot_.size() ? fleet_slot_[v] : -1;
}

void Engine::reg_collect_locked() {
  if (!lockstep_) return;
  std::lock_guard<std::mutex> g(reg_mu_);
  for (; reg_scan_series_ < n_series_; ++reg_scan_series_) {
    const int32_t v = series_[reg_scan_series_].service;
    if ((size_t)v >= reg_queued_.size()) reg_queued_.resize((size_t)v + 1, 0);
    if (reg_queued_[v]) continue;
    reg_queued_[v] = 1;
    const std::string name = dict_.service_name(v);
    reg_pending_.push_back(RegPending{v, fnv1a(name), name, fleet_packed_});
  }
}

void Engine::reg_apply_locked() {
  std::lock_guard<std::mutex> g(reg_mu_);
  bool any = false;
  size_t keep = 0;
  for (size_t i = 0; i < reg_assigned_.size(); ++i) {
    const RegAssigned& a = reg_assigned_[i];
    if (a.tag > fleet_packed_) { reg_assigned_[keep++] = a; continue; }
    if ((size_t)a.id >= fleet_slot_.size()) fleet_slot_.resize((size_t)a.id + 1, -1);
    fleet_slot_[a.id] = a.slot;
    any = true;
  }
  reg_assigned_.resize(keep);
  if (any) {  // some series change rows: rewrite the series -> row table and the Gram CSR
    series_service_uploaded_ = 0;
    svc_csr_n_ = -1;
  }
}

int32_t Engine::reg_pending_count() {
  std::lock_guard<std::mutex> g(reg_mu_);
  int32_t n = 0;
  for (const auto& p : reg_pending_) {
    if (p.tag + 2 > fleet_posted_) break;  // queued in a batch the stats thread may still be on
    ++n;
  }
  return n;
}

void Engine::reg_round() {
  const int nr = fleet_nranks_;
  RegHdr* hdr = (RegHdr*)h_reg_send_;
  RegEntry* ent = (RegEntry*)(h_reg_send_ + sizeof(RegHdr));
  char* chars = (char*)(ent + kRegMaxEntries);
  const size_t char_cap = kRegBlock - sizeof(RegHdr) - sizeof(RegEntry) * kRegMaxEntries;
  int32_t n = 0;
  uint32_t used = 0;
  {
    std::lock_guard<std::mutex> g(reg_mu_);
    for (const auto& p : reg_pending_) {
      if (p.tag + 2 > fleet_posted_ || n >= kRegMaxEntries) break;
      const uint32_t len = (uint32_t)std::min<size_t>(p.name.size(), 4096);
      if (used + len > char_cap) break;
      ent[n] = RegEntry{p.hash, used, len};
      std::memcpy(chars + used, p.name.data(), len);
      used += len;
      ++n;
    }
  }
  hdr->count = n;
  hdr->bytes = (int32_t)used;
  HIP_OK(hipMemcpyAsync(d_reg_send_, h_reg_send_, kRegBlock, hipMemcpyHostToDevice, coll_stream_));
  coll_->all_gather(d_reg_send_, d_reg_recv_, kRegBlock, coll_stream_);
  HIP_OK(hipMemcpyAsync(h_reg_recv_, d_reg_recv_, kRegBlock * (size_t)nr, hipMemcpyDeviceToHost, coll_stream_));
  coll_wait(coll_stream_, nullptr, "service registry");
  ++reg_rounds_;
  // every rank walks the same blocks in the same order: identical slot tables
  const int32_t cap = fleet_cap_;
  for (int r = 0; r < nr; ++r) {
    const uint8_t* blk = h_reg_recv_ + kRegBlock * (size_t)r;
    const RegHdr* h = (const RegHdr*)blk;
    const RegEntry* e = (const RegEntry*)(blk + sizeof(RegHdr));
    const char* c = (const char*)(e + kRegMaxEntries);
    for (int32_t i = 0; i < h->count; ++i) {
      if (reg_slot_.count(e[i].hash)) continue;
      if ((int32_t)reg_names_.size() >= cap) { reg_slot_[e[i].hash] = -1; ++reg_overflow_; continue; }
      const int32_t slot = (int32_t)reg_names_.size();
      reg_slot_[e[i].hash] = slot;
      reg_names_.emplace_back(c + e[i].off, e[i].len);
      h_fb_names_.push_back((int32_t)h_fb_chars_.size());
      h_fb_names_.push_back((int32_t)e[i].len);
      h_fb_chars_.append(c + e[i].off, e[i].len);
    }
  }
  // this rank's sent entries now have slots: hand them to the stats thread (adopted at the pack
  // of the batch this round belongs to, on every rank)
  std::lock_guard<std::mutex> g(reg_mu_);
  for (int32_t i = 0; i < n; ++i) {
    const RegPending& p = reg_pending_.front();
    reg_assigned_.push_back(RegAssigned{p.id, reg_slot_[p.hash], fleet_posted_});
    reg_pending_.pop_front();
  }
}

// fb rows of the exchange in moments slot `slot`, formatted on fb_stream_ (low priority) after
// the all-reduce (fb_src_ev_) -- never on the collective stream, where the next batch's 16-byte
// clock all-reduce, which every rank's ingest thread waits for, would queue behind them.  Each
// rank formats and emits its own slice of the service slots (all ranks hold the merged moments),
// so the formatting cost is split N ways instead of falling on rank 0 inside every rank's step.
// Returns true when the rows were queued (fb_stream_ then waits for fb_src_ev_[slot]).
bool Engine::fleet_emit_fb(int slot) {
  const int32_t n_all = (int32_t)reg_names_.size();
  if (n_all == 0) return false;
  const int nr = std::max(1, fleet_nranks_), me = coll_->rank();
  const int32_t lo = (int32_t)((int64_t)n_all * me / nr), hi = (int32_t)((int64_t)n_all * (me + 1) / nr);
  const int k = fb_k_;
  fb_k_ ^= 1;
  if (!fb_lane_) fb_lane_.reset(new TaskLane());  // fb rows get their own emission lane
  fb_lane_->wait(fb_task_[k]);  // slot k's previous D2H + emission is done
  // slot names -> device, on the fb stream BEFORE it waits for this exchange's all-reduce: the
  // host waits for the upload (pageable source) and only the fb stream's earlier work, which
  // waited for an exchange that completed long ago -- never for a peer rank
  bool uploaded = false;
  if (fb_chars_up_ < h_fb_chars_.size()) {
    if (h_fb_chars_.size() > fb_chars_cap_) {
      HIP_OK(hipStreamSynchronize(fb_stream_));  // (regrow frees the buffer the stream may read)
      d_fb_chars_ = (char*)regrow(d_fb_chars_, fb_chars_cap_, h_fb_chars_.size() * 2 + 4096);
      fb_chars_up_ = 0;
    }
    HIP_OK(hipMemcpyAsync(d_fb_chars_ + fb_chars_up_, h_fb_chars_.data() + fb_chars_up_,
                          h_fb_chars_.size() - fb_chars_up_, hipMemcpyHostToDevice, fb_stream_));
    fb_chars_up_ = h_fb_chars_.size();
    uploaded = true;
  }
  if (fb_slots_up_ < n_all) {
    if ((size_t)n_all * 8 > fb_names_cap_) {
      HIP_OK(hipStreamSynchronize(fb_stream_));
      d_fb_names_ = (int32_t*)regrow(d_fb_names_, fb_names_cap_, (size_t)n_all * 16 + 4096);
      fb_slots_up_ = 0;
    }
    HIP_OK(hipMemcpyAsync(d_fb_names_ + 2 * fb_slots_up_, h_fb_names_.data() + 2 * fb_slots_up_,
                          (size_t)(n_all - fb_slots_up_) * 8, hipMemcpyHostToDevice, fb_stream_));
    fb_slots_up_ = n_all;
    uploaded = true;
  }
  if (uploaded) HIP_OK(hipStreamSynchronize(fb_stream_));  // pageable sources: keep them alive until copied
  const int n_lags = pack_nlags_[slot];  // the LAG set of this slot's pack (a reload may have changed cfg_)
  const int32_t* lags = pack_lags_[slot];
  const int32_t rows = (hi - lo) * n_lags;
  const uint32_t blocks = apm_fleet_format_blocks(rows);
  if (blocks > fb_status_n_) {
    HIP_OK(hipStreamSynchronize(fb_stream_));
    if (d_fb_status_) dfree(d_fb_status_);
    fb_status_n_ = std::max<uint32_t>(blocks * 2, apm_fleet_format_blocks(2 * fleet_cap_ * MAX_LAGS));
    d_fb_status_ = (unsigned long long*)dmalloc((size_t)fb_status_n_ * 8 + 64);
  }
  size_t longest = 0;
  for (size_t i = 1; i < h_fb_names_.size(); i += 2) longest = std::max<size_t>(longest, (size_t)h_fb_names_[i]);
  const size_t cap_bytes = (size_t)rows * (260 + 2 * longest) + 64;
  if (cap_bytes > fb_out_cap_[k]) d_fb_out_[k] = (char*)regrow(d_fb_out_[k], fb_out_cap_[k], cap_bytes);
  // the exchange's all-reduce (coll stream) before the rows read the merged moments
  HIP_OK(hipStreamWaitEvent(fb_stream_, fb_src_ev_[slot], 0));
  FleetFormatArgs fa{};
  fa.moments = fleet_buf_[slot];
  fa.names = reinterpret_cast<const int2*>(d_fb_names_);
  fa.chars = d_fb_chars_;
  fa.slot_lo = lo;
  fa.n_slots = hi - lo;
  fa.n_lags = n_lags;
  std::vector<int> order(n_lags);
  for (int l = 0; l < n_lags; ++l) order[l] = l;
  std::sort(order.begin(), order.end(), [&](int a, int b) { return lags[a] < lags[b]; });
  for (int l = 0; l < n_lags; ++l) { fa.lag_order[l] = order[l]; fa.lag_value[l] = lags[l]; }
  fa.edge_ts = pack_edge_[slot];
  fa.copy = fs_copy_ ? 1 : 0;
  fa.ts_len = pg_timestamp(fa.edge_ts, fa.ts);
  fa.status = d_fb_status_;
  fa.total = reinterpret_cast<uint32_t*>(d_fb_status_ + fb_status_n_) + k;
  fa.out = d_fb_out_[k];
  fa.fallback = d_fmt_fallback_;
  apm_fleet_format(&fa, fb_stream_);
  HIP_OK(hipMemcpyAsync(h_fb_total_ + k, fa.total, 4, hipMemcpyDeviceToHost, fb_stream_));
  HIP_OK(hipEventRecord(fb_ev_[k], fb_stream_));
  char* dst = d_fb_out_[k];
  fb_task_[k] = fb_lane_->post([this, k, dst]() {
    HIP_OK(hipEventSynchronize(fb_ev_[k]));
    const size_t total = h_fb_total_[k];
    wait_fmt_holds(2 + k);  // the sink still writes from this buffer (zero-copy COPY rows)
    if (total > h_fb_cap_[k]) {
      if (h_fb_out_[k]) HIP_OK(hipHostFree(h_fb_out_[k]));
      h_fb_cap_[k] = total * 3 / 2 + (1 << 16);
      HIP_OK(hipHostMalloc((void**)&h_fb_out_[k], h_fb_cap_[k], hipHostMallocDefault));
    }
    if (total) {
      HIP_OK(hipMemcpy(h_fb_out_[k], dst, total, hipMemcpyDeviceToHost));
      uint64_t rows = 0;  // (memchr: vectorised; a byte loop over 18 MB cost ~3 ms of this lane)
      for (const char* p = h_fb_out_[k]; (p = (const char*)std::memchr(p, '\n', h_fb_out_[k] + total - p)); ++p) ++rows;
      fb_rows_ += rows;
      emit_bytes_held(OUT_FB, h_fb_out_[k], total, 2 + k);
    }
  });
  return true;
}

}  // namespace apm
