// Host driver of the GPU join -- see devjoin.h.  The PM_HOST field re-derivation mirrors
// runtime/join.cpp (JoinShard::on_app / on_ejb / on_ct / on_soap), which stays the reference
// implementation of the cache semantics (`gpu.joinOnDevice: false`).
#include "devjoin.h"

#include <algorithm>
#include <chrono>
#include <climits>
#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

#include "../kernels/common.h"
#include "binio.h"
#include "d2h.h"
#include "../kernels/devjoin_dev.h"
#include "../kernels/kernel_api.h"
#include "join_util.h"
#include "jsutil.h"

namespace apm {

using namespace jstr;

namespace {
double clock_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

JOp blank_op(const Event& e, int32_t server) {
  JOp op;
  std::memset(&op, 0, sizeof(op));
  op.ts = op.num = op.aux = op.aux2 = js::nan();
  op.line = e.line;
  op.server = server;
  op.op = JOP_NONE;
  return op;
}

uint64_t pow2_at_least(uint64_t v) {
  uint64_t p = 1;
  while (p < v) p <<= 1;
  return p;
}
}  // namespace

void* DeviceJoin::dmalloc(size_t bytes) {
  void* p = nullptr;
  bytes = (bytes + 255) & ~(size_t)255;
  HIP_OK(hipMalloc(&p, bytes));
  HIP_OK(hipMemsetAsync(p, 0, bytes, stream_));
  allocs_.push_back(p);
  device_bytes_ += bytes;
  return p;
}

// the join stream must be idle (callers synchronize first)
void DeviceJoin::dfree(void* p, size_t bytes) {
  if (!p) return;
  auto it = std::find(allocs_.begin(), allocs_.end(), p);
  if (it != allocs_.end()) allocs_.erase(it);
  HIP_OK(hipFree(p));
  device_bytes_ -= (bytes + 255) & ~(size_t)255;
}

DeviceJoin::DeviceJoin(const DevJoinConfig& cfg, Dictionary* dict, const std::vector<FileInfo>* files,
                       const std::vector<std::string>* servers)
    : cfg_(cfg), dict_(dict), files_(files), servers_(servers) {
  cfg_.ring_bytes = pow2_at_least(std::max<uint64_t>(cfg_.ring_bytes, 1ull << 24));
  cfg_.arena_cap = (uint32_t)pow2_at_least(std::max<uint32_t>(cfg_.arena_cap, 1024));
  HIP_OK(hipSetDevice(cfg_.device));
  // The join is the ingest thread's critical path (it waits for it twice per batch); the stats,
  // output and next-batch parse streams carry bulk work that is pipelined behind it.  A
  // high-priority stream gets a hardware queue of its own instead of sharing one (round robin
  // over GPU_MAX_HW_QUEUES = 4) with a 20 MB st/fs D2H blit.  APM_JOIN_PRIO=0: default priority.
  {
    int lo = 0, hi = 0;
    HIP_OK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    const char* pe = std::getenv("APM_JOIN_PRIO");
    HIP_OK(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, pe && pe[0] == '0' ? lo : hi));
  }
  const uint32_t E = std::max<uint32_t>(cfg_.max_events, 1024);
  out_cap_ = 2 * E + (1u << 16);
  for (int k = 0; k < 2; ++k) {
    Slot& s = sl_[k];
    s.d_bytes = (uint8_t*)dmalloc(cfg_.max_batch_bytes + 256);
    s.d_events = (Event*)dmalloc((size_t)E * sizeof(Event));
    s.host_flag = (uint8_t*)dmalloc(E + 64);
    s.d_host_ev = (Event*)dmalloc((size_t)E * sizeof(Event));
    s.d_host_idx = (uint32_t*)dmalloc((size_t)E * 4);
    s.d_mh_idx = (uint32_t*)dmalloc((size_t)E * 4);
    s.d_walk_idx = (uint32_t*)dmalloc((size_t)E * 4);
    s.d_aud = (AudF*)dmalloc((size_t)E * sizeof(AudF));
    s.d_n_host = (SelCount*)dmalloc(64);
    HIP_OK(hipHostMalloc((void**)&s.h_host_ev, (size_t)E * sizeof(Event), hipHostMallocDefault));
    HIP_OK(hipHostMalloc((void**)&s.h_host_idx, (size_t)E * 4, hipHostMallocDefault));
    HIP_OK(hipHostMalloc((void**)&s.h_n_host, 64, hipHostMallocDefault));
    std::memset(s.h_n_host, 0, 64);
    s.d_chunk_next = (int32_t*)dmalloc(((size_t)cfg_.max_chunks + 2) * 4);
    s.d_chunk_first = (uint8_t*)dmalloc((size_t)cfg_.max_chunks + 2);
    HIP_OK(hipHostMalloc((void**)&s.h_chunk_next, ((size_t)cfg_.max_chunks + 2) * 4, hipHostMallocDefault));
    HIP_OK(hipHostMalloc((void**)&s.h_chunk_first, (size_t)cfg_.max_chunks + 2, hipHostMallocDefault));
    s.d_tx = (TxRec*)dmalloc((size_t)out_cap_ * sizeof(TxRec));
    s.d_tx_raw = (int32_t*)dmalloc((size_t)out_cap_ * 4);
    s.d_tx_gid = (int64_t*)dmalloc((size_t)out_cap_ * 8);
    HIP_OK(hipEventCreateWithFlags(&s.free_ev, hipEventDisableTiming));
  }
  table_bits_ = cfg_.table_bits;
  table_cap_ = 1u << table_bits_;
  init_table_cap_ = table_cap_;
  init_arena_cap_ = cfg_.arena_cap;
  d_table_ = (KeyState*)dmalloc((size_t)table_cap_ * sizeof(KeyState));
  d_reg_ = (RegSlot*)dmalloc(((size_t)1 << cfg_.reg_bits) * sizeof(RegSlot));
  miss_cap_ = E;
  d_miss_ = (RegMiss*)dmalloc((size_t)miss_cap_ * sizeof(RegMiss));
  HIP_OK(hipHostMalloc((void**)&h_miss_, (size_t)miss_cap_ * sizeof(RegMiss), hipHostMallocDefault));
  d_arena_ = (NeedEnt*)dmalloc((size_t)cfg_.arena_cap * sizeof(NeedEnt));
  d_exp_lo_ = (uint64_t*)dmalloc(8 * 4096);
  d_exp_hi_ = (uint64_t*)dmalloc(8 * 4096);
  HIP_OK(hipHostMalloc((void**)&h_exp_, 2 * 8 * 4096, hipHostMallocDefault));
  HIP_OK(hipHostGetDevicePointer((void**)&hd_exp_, h_exp_, 0));
  soap_cap_ = 1u << 16;
  d_soap_ = (SoapState*)dmalloc((size_t)soap_cap_ * sizeof(SoapState));
  if (E >= (1u << 21)) throw std::runtime_error("device join: gpu.maxLinesPerBatch must be below 2^21");
  d_sel_val_ = (uint64_t*)dmalloc(((size_t)E + 64) * 8);
  d_sel_pos_ = (uint64_t*)dmalloc(((size_t)E + 64) * 8);
  d_walk_lo_ = (uint32_t*)dmalloc(((size_t)cfg_.max_chunks + 2) * 4);
  d_file_first_ = (int32_t*)dmalloc((size_t)soap_cap_ * 4);
  for (AudGen& g : aud_gen_) {
    g.carry = (AudCarry*)dmalloc((size_t)soap_cap_ * sizeof(AudCarry));
    aud_reserve(g, 4096, 16384, 1u << 20);
  }
  d_file_server_ = (int32_t*)dmalloc((size_t)soap_cap_ * 4);
  d_file_skey_ = (uint64_t*)dmalloc((size_t)soap_cap_ * 8);
  d_file_fkey_ = (uint64_t*)dmalloc((size_t)soap_cap_ * 8);
  h_file_skey_.reserve(soap_cap_);  // (the pre-pass lane reads them while files are added)
  h_file_fkey_.reserve(soap_cap_);
  d_rawtab_ = (RawSvc*)dmalloc((size_t)cfg_.max_raw * sizeof(RawSvc));
  d_raw_series_ = (int32_t*)dmalloc((size_t)cfg_.max_raw * 4);
  d_raw_first_ = (int32_t*)dmalloc((size_t)cfg_.max_raw * 4);
  HIP_OK(hipMemsetAsync(d_raw_series_, 0xff, (size_t)cfg_.max_raw * 4, stream_));
  HIP_OK(hipMemsetAsync(d_raw_first_, 0x7f, (size_t)cfg_.max_raw * 4, stream_));
  raw_info_.reserve(cfg_.max_raw);
  HIP_OK(hipHostMalloc((void**)&h_rawtab_, (size_t)cfg_.max_raw * sizeof(RawSvc), hipHostMallocDefault));
  d_reg_fill_ = (int32_t*)dmalloc((size_t)E * 8);
  HIP_OK(hipHostMalloc((void**)&h_reg_fill_, (size_t)E * 8, hipHostMallocDefault));
  d_out_ = (TxDev*)dmalloc((size_t)out_cap_ * sizeof(TxDev));
  d_lens_ = (uint32_t*)dmalloc(((size_t)out_cap_ + 1) * 16);
  d_offs_ = (uint32_t*)dmalloc(((size_t)out_cap_ + 1) * 16);
  d_bucket_ = (int64_t*)dmalloc((size_t)out_cap_ * 8);
  d_bmax_ = (int64_t*)dmalloc((size_t)out_cap_ * 8);
  d_cand_ = (uint32_t*)dmalloc((size_t)out_cap_ * 4);
  d_cand_bucket_ = (int64_t*)dmalloc((size_t)out_cap_ * 8);
  d_unres_ = (uint32_t*)dmalloc((size_t)out_cap_ * 8);
  HIP_OK(hipHostMalloc((void**)&h_cand_, (size_t)out_cap_ * 4, hipHostMallocDefault));
  HIP_OK(hipHostMalloc((void**)&h_cand_bucket_, (size_t)out_cap_ * 8, hipHostMallocDefault));
  HIP_OK(hipHostMalloc((void**)&h_unres_, (size_t)out_cap_ * 8, hipHostMallocDefault));
  ensure_tmp();
  sel_tmp_bytes_ = apm_dj_tmp_bytes(E, 1024, 8);
  d_sel_tmp_ = dmalloc(sel_tmp_bytes_);
  d_counts_ = (JoinCounts*)dmalloc(sizeof(JoinCounts));
  HIP_OK(hipHostMalloc((void**)&h_counts_, sizeof(JoinCounts), hipHostMallocDefault));
  std::memset(h_counts_, 0, sizeof(JoinCounts));
  d_live_ = (unsigned long long*)dmalloc(64);
  HIP_OK(hipHostMalloc((void**)&h_live_, 64, hipHostMallocDefault));
  // chain-block pool (overflow of the per-key partial / parked-record / logId storage); grows
  // before any batch whose worst case exceeds its free blocks
  pool_n_ = (uint32_t)pow2_at_least(cfg_.pool_blocks ? std::max<uint32_t>(cfg_.pool_blocks, 1024)
                                                   : std::max<uint32_t>(E / 2, 1u << 16));
  d_pool_ = (uint8_t*)dmalloc((size_t)pool_n_ * CHAIN_BLK);
  d_pool_ring_ = (uint32_t*)dmalloc((size_t)pool_n_ * 4);
  apm_dj_pool_init(d_pool_ring_, pool_n_, d_counts_, stream_);
  h_counts_->pool_tail = h_counts_->pool_ptail = pool_n_;
  d_ops_ = (JOp*)dmalloc((size_t)E * sizeof(JOp));
  d_soap_code_ = (uint8_t*)dmalloc(E);
  d_soap_num_ = (double*)dmalloc((size_t)E * 8);
  d_soap_hash_ = (uint64_t*)dmalloc((size_t)E * 8);
  d_chunk_ev_lo_ = (uint32_t*)dmalloc(((size_t)cfg_.max_chunks + 2) * 4);
  d_seg_f_ = (uint32_t*)dmalloc(((size_t)cfg_.max_chunks + 2) * SOAP_SEGS * 4);
  d_seg_in_ = (uint32_t*)dmalloc(((size_t)cfg_.max_chunks + 2) * SOAP_SEGS * 4);
  d_chain_hash_ = (uint64_t*)dmalloc(((size_t)cfg_.max_chunks + 2) * 8);
  d_op_slot_ = (uint32_t*)dmalloc(((size_t)E + 1) * 4);
  d_op_slot_sorted_ = (uint32_t*)dmalloc(((size_t)E + 1) * 4);
  d_op_idx_ = (uint32_t*)dmalloc(((size_t)E + 1) * 4);
  d_op_idx_sorted_ = (uint32_t*)dmalloc(((size_t)E + 1) * 4);
  exp_cap_ = cfg_.arena_cap;
  d_exp_key_ = (uint64_t*)dmalloc(((size_t)exp_cap_ + 1) * 8);
  d_exp_key_sorted_ = (uint64_t*)dmalloc(((size_t)exp_cap_ + 1) * 8);
  d_exp_idx_ = (uint32_t*)dmalloc(((size_t)exp_cap_ + 1) * 4);
  d_exp_idx_sorted_ = (uint32_t*)dmalloc(((size_t)exp_cap_ + 1) * 4);
  d_exp_cnt_ = (uint32_t*)dmalloc(((size_t)exp_cap_ + 1) * 4);
  d_exp_pos_ = (uint32_t*)dmalloc(((size_t)exp_cap_ + 1) * 4);
  d_out_cnt_ = (uint32_t*)dmalloc(((size_t)E + 1) * 4);
  d_out_pos_ = (uint32_t*)dmalloc(((size_t)E + 1) * 4);
  d_stage_ = (TxDev*)dmalloc((size_t)E * 2 * sizeof(TxDev));
  d_ovf_ = (DJOverflow*)dmalloc((size_t)DJ_OVF_CAP * sizeof(DJOverflow));
  d_ring_ = (char*)dmalloc(cfg_.ring_bytes);
  d_ring_pos_ = (uint64_t*)dmalloc(8);
  d_big_ = (uint32_t*)dmalloc(8);
  {
    const char* e = std::getenv("APM_OPSORT");
    group_sort_ = e && std::strcmp(e, "sort") == 0;
  }
  HIP_OK(hipStreamSynchronize(stream_));
}

// the tx / audit_db text staging of the write pass: >= `bytes` each (the join stream is idle or
// about to use it after this call; hipFree orders against the device)
void DeviceJoin::ensure_txt(size_t bytes) {
  if (bytes <= txt_cap_ && d_txt_tx_) return;
  const size_t cap = std::max(bytes, txt_cap_);
  char* p = nullptr;
  HIP_OK(hipMalloc((void**)&p, cap * 2));
  if (d_txt_tx_) { HIP_OK(hipFree(d_txt_tx_)); device_bytes_ -= txt_cap_ * 2; }
  d_txt_tx_ = p;
  d_txt_db_ = p + cap;
  txt_cap_ = cap;
  device_bytes_ += cap * 2;
}

DeviceJoin::~DeviceJoin() {
  hipStreamSynchronize(stream_);
  if (live_ev_) hipEventDestroy(live_ev_);
  for (auto& s : sl_) {
    hipHostFree(s.h_host_ev); hipHostFree(s.h_host_idx); hipHostFree(s.h_n_host);
    hipHostFree(s.h_chunk_next); hipHostFree(s.h_chunk_first);
    hipEventDestroy(s.free_ev);
  }
  hipHostFree(h_miss_); hipHostFree(h_exp_); hipHostFree(h_rawtab_); hipHostFree(h_reg_fill_);
  hipHostFree(h_cand_); hipHostFree(h_cand_bucket_); hipHostFree(h_unres_); hipHostFree(h_counts_); hipHostFree(h_live_);
  if (h_cstats_) hipHostFree(h_cstats_);
  if (cstats_ev_) hipEventDestroy(cstats_ev_);
  if (h_hops_) hipHostFree(h_hops_);
  if (h_hbuf_) hipHostFree(h_hbuf_);
  if (h_txt_) hipHostFree(h_txt_);
  if (h_ck_bounce_) hipHostFree(h_ck_bounce_);
  if (d_txt_tx_) hipFree(d_txt_tx_);
  for (void* p : allocs_) hipFree(p);
  hipStreamDestroy(stream_);
}

// ---------------------------------------------------------------------------- parse-side hooks
// World-invariant keys of the files registered since the last call (their server's and their
// own), host copies (read by the pre-pass lane: reserved, never reallocated) and device tables
// (blocking copy: ordered before any kernel launched after it, on any stream).
void DeviceJoin::sync_file_keys() {
  const size_t n = files_->size();
  if (n <= h_file_fkey_.size()) return;
  if (n > soap_cap_) throw std::runtime_error("device join: too many files");
  const size_t lo = h_file_fkey_.size();
  if (lo == 0) HIP_OK(hipStreamSynchronize(stream_));  // (dmalloc zeroed the tables on the join stream)
  for (size_t i = lo; i < n; ++i) {
    const FileInfo& f = (*files_)[i];
    const std::string& srv = (*servers_)[f.server];
    h_file_skey_.push_back(dj::server_key_of(srv.data(), srv.size()));
    h_file_fkey_.push_back(dj::file_key_of(f.path.data(), f.path.size()));
  }
  HIP_OK(hipMemcpy(d_file_skey_ + lo, h_file_skey_.data() + lo, (n - lo) * 8, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(d_file_fkey_ + lo, h_file_fkey_.data() + lo, (n - lo) * 8, hipMemcpyHostToDevice));
}

void DeviceJoin::select_host(int k, const uint32_t* d_n_ev, uint32_t max_ev, hipStream_t ps) {
  Slot& s = sl_[k];
  sync_file_keys();
  DJArgs a{};
  a.ev = s.d_events;
  a.bytes = s.d_bytes;
  a.host_flag = s.host_flag;
  a.chunk_file = s.d_chunk_file;  // (set_chunks ran first)
  a.file_fkey = d_file_fkey_;
  a.aud = s.d_aud;
  a.sel_val = d_sel_val_;
  a.sel_pos = d_sel_pos_;
  a.host_ev = s.d_host_ev;
  a.host_ev_idx = s.d_host_idx;
  a.mh_idx = s.d_mh_idx;
  a.walk_idx = s.d_walk_idx;
  a.n_host = s.d_n_host;
  a.tmp = d_sel_tmp_;  // own scratch: the join of the previous batch runs concurrently
  a.tmp_bytes = sel_tmp_bytes_;
  if (apm_dj_select_host(&a, d_n_ev, std::min<uint32_t>(max_ev, cfg_.max_events), ps) != 0)
    throw std::runtime_error("device join: scan scratch too small");
  HIP_OK(hipMemcpyAsync(s.h_n_host, s.d_n_host, sizeof(SelCount), hipMemcpyDeviceToHost, ps));
  // speculative copy of the host events (last count + 25 %): usually all of them
  s.spec = std::min<uint32_t>(cfg_.max_events, last_host_ + last_host_ / 4 + 256);
  HIP_OK(hipMemcpyAsync(s.h_host_ev, s.d_host_ev, (size_t)s.spec * sizeof(Event), hipMemcpyDeviceToHost, ps));
  HIP_OK(hipMemcpyAsync(s.h_host_idx, s.d_host_idx, (size_t)s.spec * 4, hipMemcpyDeviceToHost, ps));
}

void DeviceJoin::set_chunks(int k, const std::vector<int32_t>& chunk_file, const uint32_t* d_chunk_file,
                            const uint8_t* d_chunk_kind, hipStream_t ps) {
  Slot& s = sl_[k];
  const uint32_t n = (uint32_t)chunk_file.size();
  std::unordered_map<int32_t, int32_t> last;
  for (uint32_t c = 0; c < n; ++c) {
    s.h_chunk_next[c] = -1;
    auto it = last.find(chunk_file[c]);
    if (it == last.end()) {
      s.h_chunk_first[c] = 1;
    } else {
      s.h_chunk_first[c] = 0;
      s.h_chunk_next[it->second] = (int32_t)c;
    }
    last[chunk_file[c]] = (int32_t)c;
  }
  if (n) {
    HIP_OK(hipMemcpyAsync(s.d_chunk_next, s.h_chunk_next, (size_t)n * 4, hipMemcpyHostToDevice, ps));
    HIP_OK(hipMemcpyAsync(s.d_chunk_first, s.h_chunk_first, n, hipMemcpyHostToDevice, ps));
  }
  s.d_chunk_file = d_chunk_file;
  s.d_chunk_kind = d_chunk_kind;
  s.n_chunks = n;
  s.chunk_file = chunk_file;
}

void DeviceJoin::finish_select(int k, hipStream_t ps) {
  Slot& s = sl_[k];
  const uint32_t n = s.h_n_host->host;
  if (n > s.spec) {
    HIP_OK(hipMemcpyAsync(s.h_host_ev + s.spec, s.d_host_ev + s.spec, (size_t)(n - s.spec) * sizeof(Event),
                          hipMemcpyDeviceToHost, ps));
    HIP_OK(hipMemcpyAsync(s.h_host_idx + s.spec, s.d_host_idx + s.spec, (size_t)(n - s.spec) * 4,
                          hipMemcpyDeviceToHost, ps));
    HIP_OK(hipStreamSynchronize(ps));
  }
  last_host_ = n;
}

// ---------------------------------------------------------------------------- host pre-pass
// One task per file with host events (audit state is per file, cache effects are ops resolved
// on the GPU in line order), run on the engine's worker pool; the per-file op lists are then
// merged by event index and their string buffers concatenated.
void DeviceJoin::host_prepass(int k, const uint8_t* hb, uint32_t n_host, const ParallelFor& parallel,
                              std::vector<HostOp>& hops_out, std::string& hbuf_out) {
  Slot& s = sl_[k];
  hops_out.clear();
  hbuf_out.clear();
  std::unordered_map<int32_t, int> task_of;
  int nt = 0;
  int32_t last_file = -1;
  int last_t = -1;
  for (uint32_t i = 0; i < n_host; ++i) {
    const int32_t file = s.chunk_file[s.h_host_ev[i].chunk];
    if (file == last_file) {  // events come in chunk order: runs of one file
      tasks_[last_t].idx.push_back(i);
      continue;
    }
    auto it = task_of.find(file);
    int t;
    if (it == task_of.end()) {
      t = nt++;
      task_of.emplace(file, t);
      if ((int)tasks_.size() < nt) tasks_.emplace_back();
      PrepassTask& T = tasks_[t];
      T.file = file;
      T.idx.clear(); T.hops.clear(); T.hbuf.clear();
      T.audit_errors = T.invalid_acct = T.pm_host = 0;
    } else {
      t = it->second;
    }
    last_file = file;
    last_t = t;
    tasks_[t].idx.push_back(i);
  }
  auto work = [&](int t) {
    PrepassTask& T = tasks_[t];
    for (uint32_t i : T.idx) host_event(T, s.h_host_ev[i], s.h_host_idx[i], hb);
  };
  if (parallel && nt > 1) parallel(nt, work);
  else for (int t = 0; t < nt; ++t) work(t);
  // merge by event index (each task's list ascends); rebase the host-buffer offsets
  size_t total = 0;
  std::vector<uint32_t> base(nt);
  for (int t = 0; t < nt; ++t) {
    base[t] = (uint32_t)hbuf_out.size();
    hbuf_out += tasks_[t].hbuf;
    total += tasks_[t].hops.size();
    audit_errors_ += tasks_[t].audit_errors;
    host_invalid_acct_ += tasks_[t].invalid_acct;
    host_pm_ += tasks_[t].pm_host;
  }
  hops_out.reserve(total);
  std::vector<size_t> pos(nt, 0);
  for (;;) {
    int best = -1;
    uint32_t bev = UINT32_MAX;
    for (int t = 0; t < nt; ++t)
      if (pos[t] < tasks_[t].hops.size() && tasks_[t].hops[pos[t]].ev < bev) { bev = tasks_[t].hops[pos[t]].ev; best = t; }
    if (best < 0) break;
    HostOp h = tasks_[best].hops[pos[best]++];
    if (h.kind == HOP_AUD) {  // (an AudF in the op's bytes)
      AudF f;
      std::memcpy(&f, &h.op, sizeof(f));
      if (f.flags & AF_SRC_HOST) f.ref += base[best];
      std::memcpy(&h.op, &f, sizeof(f));
    } else {
      if (h.op.flags & JF_LID_HOST) h.op.lid += base[best];
      if (h.op.flags & JF_SVC_HOST) h.op.svc_ref += base[best];
    }
    hops_out.push_back(h);
  }
  host_events_ += n_host;
}

void DeviceJoin::host_event(PrepassTask& T, const Event& e, uint32_t ev, const uint8_t* hb) {
  const int32_t server = (*files_)[T.file].server;
  const std::string_view line((const char*)hb + e.off, e.len);
  if (e.mask & PM_HOST) ++T.pm_host;
  if (e.kind == LK_APP) { on_app(T, e, ev, line); return; }
  HostOp h;
  std::memset(&h, 0, sizeof(h));
  h.ev = ev;
  h.op = blank_op(e, server);
  JOp& op = h.op;
  if (e.kind == LK_SOAP) {  // parseSoapLine (:352-376), fields only: the context scan is on the GPU
    const uint32_t m = e.mask;
    if (m & PM_SOAP_IN) {
      auto toks = js::split_ws(line, 4);
      std::string_view lid;
      bool has = false;
      if (toks.size() > 1) {
        const std::string_view t1 = toks[1];
        const size_t eq = t1.find('=');
        if (eq != std::string_view::npos) {
          const size_t eq2 = t1.find('=', eq + 1);
          lid = t1.substr(eq + 1, eq2 == std::string_view::npos ? std::string_view::npos : eq2 - eq - 1);
          has = true;
        }
      }
      h.kind = HOP_SOAP_IN;
      h.lid_hash = has ? hash_bytes(lid.data(), lid.size()) : hash_bytes("undefined", 9);
    } else if (m & PM_SOAP_OUT) {
      h.kind = HOP_SOAP_OUT;
    } else if ((m & PM_SOAP_ACCT) || (!(m & PM_SOAP_KEY) && (m & PM_SOAP_VALUE))) {
      const std::string_view acct = js::trim(angle_field2(line));
      h.kind = (m & PM_SOAP_ACCT) ? HOP_SOAP_ACCT : HOP_SOAP_VALUE;
      if (all_digits(acct)) { op.flags = JF_BAF_VALID; op.num = js::parse_int(acct); }
    } else if (m & PM_SOAP_KEY) {
      h.kind = HOP_SOAP_KEY;
    } else {
      return;
    }
    T.hops.push_back(h);
    return;
  }
  if (e.kind < LK_EJB_ENTRY || e.kind > LK_CT_EXIT) return;
  // EJB / CommonTiming (:378-565): the host split (PM_HOST lines, bracketed logIds, short lines)
  const bool ejb = e.kind <= LK_EJB_EXIT;
  const bool entry = e.kind == LK_EJB_ENTRY || e.kind == LK_CT_ENTRY;
  auto toks = js::split_ws(line, 16);
  auto get = [&](size_t i) { return i < toks.size() ? toks[i] : kUndef; };
  std::string scratch;
  const std::string lid(strip_brackets(toks[0], scratch));
  double ts;
  bool ts_empty = false;
  {
    const std::string tsstr = std::string(get(1)) + " " + std::string(get(2));
    if (!js::convert_date(tsstr, cfg_.tz, ts)) { ts_empty = true; ts = js::nan(); }
  }
  std::string_view name;
  double elapsed = js::nan();
  if (ejb) {
    name = get(entry ? 13 : 9);
    if (!entry && toks.size() > 11) elapsed = js::parse_int(toks[11]);
  } else {
    const auto seg = info_segment_tokens(line);
    name = seg.size() > 1 ? seg[1] : kUndef;
    if (!entry && seg.size() > 5) elapsed = js::parse_int(seg[5]);
  }
  if (entry && lid.empty()) return;  // parseEntry returns before anything else
  op.svc = hash_bytes(name.data(), name.size(), ejb ? kHashSeedEjb : kHashSeed);
  op.flags = JF_HAS_SVC | JF_SVC_HOST | (ejb ? JF_EJB : 0);
  op.svc_ref = T.put(name);
  op.svc_len = (uint16_t)name.size();
  op.ts = ts;
  if (ts_empty) op.flags |= JF_TS_EMPTY;
  if (!lid.empty()) {
    op.lid = T.put(lid);
    op.lid_len = (uint16_t)std::min<size_t>(lid.size(), 0xffff);
    op.flags |= JF_LID_HOST;
    op.gkey = dj::gkey_of(hash_bytes(lid.data(), lid.size()), h_file_skey_[T.file]);
  }
  if (entry) {
    op.op = JOP_ENTRY;
  } else {
    op.num = elapsed;
    if (!ejb) {
      const bool use_baf = (e.mask & PM_HOST) ? baf_match(line) : (e.mask & PM_BAF) != 0;
      if (use_baf) {
        std::string_view t3 = get(3);
        size_t p = std::string_view::npos;
        for (size_t i = 0; i + 1 < t3.size(); ++i) if (t3[i] == ']' && t3[i + 1] == '[') p = i;
        if (p != std::string_view::npos) t3 = t3.substr(p + 2);
        std::string b;
        for (char c : t3) if (c != '[' && c != ']') b.push_back(c);
        const size_t c = b.rfind(':');
        const std::string acct = c == std::string::npos ? b : b.substr(c + 1);
        if (!acct.empty()) {
          op.flags |= JF_BAF;
          op.aux = js::parse_int(acct);
          const std::string_view t = js::trim(acct);
          if (all_digits(t)) { op.flags |= JF_BAF_VALID; op.aux2 = js::parse_int(t); }
        }
      }
    }
    op.op = lid.empty() ? JOP_DIRECT : (ejb ? JOP_EJB_EXIT : JOP_CT_EXIT);
    if (lid.empty()) op.gkey = 0;
  }
  h.kind = HOP_JOIN;
  T.hops.push_back(h);
}

// HOP_AUD: the fields (AudF) of an audit line the GPU could not read alone -- parseAppLine's
// string work (:578-731) with the exact JS helpers; the state machine itself runs on the GPU
// (devjoin.hip k_aud_*).  Mirrors aud_fields() there; strings go to the host op buffer.
void DeviceJoin::on_app(PrepassTask& T, const Event& e, uint32_t ev, std::string_view line) {
  HostOp h;
  std::memset(&h, 0, sizeof(h));
  h.ev = ev;
  h.kind = HOP_AUD;
  AudF f;
  std::memset(&f, 0, sizeof(f));
  f.el = js::nan();
  f.ts = js::nan();
  const uint32_t m = e.mask;
  auto done = [&]() {
    std::memcpy(&h.op, &f, sizeof(f));
    T.hops.push_back(h);
  };
  if (m & PM_AUTR_MAP) {
    auto toks = js::split_ws(line, 8);
    std::string scratch;
    const std::string_view log_id = strip_brackets(toks[0], scratch);
    f.h_sw = hash_bytes(log_id.data(), log_id.size());
    f.len = (uint16_t)std::min<size_t>(log_id.size(), 0xffff);
    f.ref = T.put(log_id.substr(0, f.len));
    f.flags |= AF_SRC_HOST;
    const std::string_view t5 = toks.size() > 5 ? toks[5] : std::string_view();
    const size_t eq = t5.find('=');
    uint64_t ah;
    if (eq != std::string_view::npos) {
      const size_t eq2 = t5.find('=', eq + 1);
      const std::string_view autr = t5.substr(eq + 1, eq2 == std::string_view::npos ? std::string_view::npos : eq2 - eq - 1);
      ah = hash_bytes(autr.data(), autr.size());
    } else {
      ah = hash_bytes("undefined", 9);
    }
    f.h_item = dj::aud_key(ah, h_file_fkey_[T.file]);
    // attemptReadAccountNumberFromBAFInfo -> the block's alt account and saveAcctNum
    if ((e.mask & PM_HOST) ? baf_match(line) : (e.mask & PM_BAF) != 0) {
      std::string_view t3 = toks.size() > 3 ? toks[3] : std::string_view();
      size_t p = std::string_view::npos;
      for (size_t i = 0; i + 1 < t3.size(); ++i) if (t3[i] == ']' && t3[i + 1] == '[') p = i;
      if (p != std::string_view::npos) t3 = t3.substr(p + 2);
      std::string b;
      for (char c : t3) if (c != '[' && c != ']') b.push_back(c);
      const size_t c = b.rfind(':');
      const std::string alt = c == std::string::npos ? b : b.substr(c + 1);
      if (!alt.empty()) {
        f.flags |= AF_ACCT;
        f.el = js::parse_int(alt);
        if (all_digits(js::trim(alt))) f.flags |= AF_ACCT_VALID;
      }
    }
    return done();
  }
  if (m & PM_AUTR_HDR) {  // line.split(':')[1].trim()
    const size_t c1 = line.find(':');
    const size_t c2 = line.find(':', c1 + 1);
    const std::string_view autr = js::trim(line.substr(c1 + 1, c2 == std::string_view::npos ? std::string_view::npos : c2 - c1 - 1));
    f.h_item = dj::aud_key(hash_bytes(autr.data(), autr.size()), h_file_fkey_[T.file]);
    return done();
  }
  {  // item role: service and elapsed of a RequestTrace line
    const size_t c1 = line.find(':');
    const std::string_view service = js::trim(line.substr(0, c1));
    f.h_item = hash_bytes(service.data(), service.size());
    std::string elapsed;
    if (c1 != std::string_view::npos) {
      const size_t c2 = line.find(':', c1 + 1);
      const std::string_view a1 = line.substr(c1 + 1, c2 == std::string_view::npos ? std::string_view::npos : c2 - c1 - 1);
      auto st = js::split_ws(a1, 2);
      for (char ch : st[0]) if (ch != '[' && ch != ']') elapsed.push_back(ch);
    }
    f.el = js::parse_int(elapsed);
  }
  if (m & PM_SW_NAME) {
    const std::string name = xml_inner(line);
    f.len = (uint16_t)std::min<size_t>(name.size(), 0xffff);
    f.ref = T.put(std::string_view(name).substr(0, f.len));
    f.flags |= AF_SRC_HOST;
    f.h_sw = hash_bytes(name.data(), name.size());
    if (!icontains(name, "Provider[")) f.flags |= AF_TO_DB;
  } else if (m & (PM_SW_STARTTS | PM_SW_STOPTS)) {
    double v = js::nan();
    if (js::convert_date(xml_inner(line), cfg_.tz, v)) f.ts = v;
    else f.flags |= AF_TS_EMPTY;
  }
  done();
}

// ---------------------------------------------------------------------------- registration
int32_t DeviceJoin::intern_name(const std::string& s) {
  auto it = name_off_.find(s);
  if (it != name_off_.end()) return it->second;
  const int32_t off = (int32_t)names_.size();
  names_ += s;
  name_off_.emplace(s, off);
  return off;
}

void DeviceJoin::register_misses(const uint8_t* hb, uint32_t n_miss, hipStream_t s) {
  if (n_miss > miss_cap_) throw std::runtime_error("device join: service registry miss list overflow");
  HIP_OK(hipMemcpyAsync(h_miss_, d_miss_, (size_t)n_miss * sizeof(RegMiss), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  const int32_t first = n_raw_.load(std::memory_order_relaxed);
  int32_t n = first;
  for (uint32_t i = 0; i < n_miss; ++i) {
    const RegMiss& m = h_miss_[i];
    std::string raw = (m.flags & JF_EJB) ? "S:" : "";
    if (m.flags & JF_SVC_UNDEF) raw += "undefined";
    else if (m.flags & JF_SVC_HOST) raw.append(hbuf_.data() + m.name, m.name_len);
    else if (m.flags & JF_SVC_AUD) {  // a carried stopWatch name (rare: new service, block across batches)
      std::string b(m.name_len, '\0');
      if (m.name_len) HIP_OK(hipMemcpy(&b[0], aud_gen_[aud_cur_].txt + m.name, m.name_len, hipMemcpyDeviceToHost));
      raw += b;
    }
    else raw.append((const char*)hb + m.name, m.name_len);
    const std::string norm = normalize_service(raw);
    if ((uint32_t)n >= cfg_.max_raw) throw std::runtime_error("device join: more raw services than gpu.maxRawServices");
    const int32_t nid = dict_->service_id(norm);
    raw_info_.push_back(RawInfo{m.server, nid, m.svc});
    RawSvc& r = h_rawtab_[n];
    r.srv_off = intern_name((*servers_)[m.server]);
    r.srv_len = (int32_t)(*servers_)[m.server].size();
    r.norm_off = intern_name(norm);
    r.norm_len = (int32_t)norm.size();
    r.toplevel = norm.size() >= 2 && norm[0] == 'S' && norm[1] == ':';
    r.pad = 0;
    h_reg_fill_[2 * i] = m.slot;
    h_reg_fill_[2 * i + 1] = n;
    ++n;
  }
  if (names_.size() > names_cap_) {
    const size_t cap = std::max<size_t>(names_.size() * 2, 1 << 20);
    char* p = nullptr;
    HIP_OK(hipMalloc((void**)&p, cap));
    if (d_names_) {
      HIP_OK(hipMemcpyAsync(p, d_names_, names_uploaded_, hipMemcpyDeviceToDevice, s));
      HIP_OK(hipStreamSynchronize(s));
      HIP_OK(hipFree(d_names_));
      device_bytes_ -= names_cap_;
    }
    d_names_ = p;
    names_cap_ = cap;
    device_bytes_ += cap;
  }
  if (names_.size() > names_uploaded_) {
    HIP_OK(hipMemcpyAsync(d_names_ + names_uploaded_, names_.data() + names_uploaded_, names_.size() - names_uploaded_,
                          hipMemcpyHostToDevice, s));
    HIP_OK(hipStreamSynchronize(s));  // names_ may reallocate on the next registration
    names_uploaded_ = names_.size();
  }
  HIP_OK(hipMemcpyAsync(d_rawtab_ + first, h_rawtab_ + first, (size_t)(n - first) * sizeof(RawSvc), hipMemcpyHostToDevice, s));
  HIP_OK(hipMemcpyAsync(d_reg_fill_, h_reg_fill_, (size_t)n_miss * 8, hipMemcpyHostToDevice, s));
  apm_dj_reg_fill(d_reg_, d_reg_fill_, n_miss, s);
  n_raw_.store(n, std::memory_order_release);
}

// ---------------------------------------------------------------------------- ring
uint64_t DeviceJoin::ring_reserve(uint64_t bytes) {
  std::lock_guard<std::mutex> g(ring_mu_);
  const uint64_t cap = cfg_.ring_bytes;
  if (bytes > cap / 4) throw std::runtime_error("device join: one batch of tx text exceeds a quarter of gpu.txTextRingMB");
  uint64_t base = ring_head_.load(std::memory_order_relaxed);
  if ((base & (cap - 1)) + bytes > cap) base = (base + cap - 1) & ~(cap - 1);  // keep the region contiguous
  const uint64_t low = ring_low_.load(std::memory_order_acquire);
  if (base + bytes > low + cap)
    throw std::runtime_error("device join: tx text ring exhausted (pending released-tx lines span more than "
                             "gpu.txTextRingMB; raise it)");
  ring_head_.store(base + bytes, std::memory_order_release);
  return base;
}

void DeviceJoin::set_ring_low(uint64_t low) {
  uint64_t cur = ring_low_.load(std::memory_order_relaxed);
  while (low > cur && !ring_low_.compare_exchange_weak(cur, low)) {
  }
}

// ---------------------------------------------------------------------------- batch
void DeviceJoin::release_slot(int k, hipStream_t stats_stream) {
  HIP_OK(hipEventRecord(sl_[k].free_ev, stats_stream));
  sl_[k].used = true;
}

void DeviceJoin::ensure_tmp() {
  const uint32_t E = std::max<uint32_t>(cfg_.max_events, 1024);
  const size_t need = std::max(apm_dj_tmp_bytes(E, out_cap_, table_bits_), apm_dj_tmp_bytes(cfg_.arena_cap, out_cap_, table_bits_));
  if (need <= tmp_bytes_ && d_tmp_) return;
  if (d_tmp_) {
    HIP_OK(hipStreamSynchronize(stream_));
    dfree(d_tmp_, tmp_bytes_);
  }
  tmp_bytes_ = need;
  d_tmp_ = dmalloc(tmp_bytes_);
}

// Reinsert the live keys (acct / record not expired, or a live need entry) into a clean table of
// `new_cap` slots.  Same size: the spare buffer (no allocation on the ingest path).
void DeviceJoin::rebuild_table(double now, uint32_t new_cap) {
  hipStream_t st = stream_;
  KeyState* fresh;
  const bool same = new_cap == table_cap_;
  if (same && !rebuild_copy()) {  // in place (apm_dj_rebuild_inplace), then wait for the count
    rebuild_inplace(now);
    sync_keys();
    HIP_OK(hipMemcpyAsync(h_live_, d_live_, 8, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    keys_live_ = *h_live_;
    keys_since_rebuild_ = 0;
    live_pending_ = false;
    ++table_rebuilds_;
    return;
  }
  if (same && d_table_spare_) fresh = d_table_spare_;
  else fresh = (KeyState*)dmalloc((size_t)new_cap * sizeof(KeyState));
  HIP_OK(hipMemsetAsync(fresh, 0, (size_t)new_cap * sizeof(KeyState), st));
  HIP_OK(hipMemsetAsync(d_live_, 0, 8, st));
  apm_dj_rebuild(d_table_, table_cap_, fresh, new_cap - 1, d_arena_, cfg_.arena_cap, now, d_counts_, d_live_, d_pool_,
                 d_pool_ring_, pool_n_ - 1, st);
  HIP_OK(hipMemcpyAsync(h_live_, d_live_, 8, hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  if (same) {
    d_table_spare_ = d_table_;
    spare_clean_ = false;
  } else {
    dfree(d_table_, (size_t)table_cap_ * sizeof(KeyState));
    if (d_table_spare_) dfree(d_table_spare_, (size_t)table_cap_ * sizeof(KeyState));
    d_table_spare_ = nullptr;
    ++table_grows_;
  }
  d_table_ = fresh;
  table_cap_ = new_cap;
  table_bits_ = 0;
  while ((1u << table_bits_) < table_cap_) ++table_bits_;
  keys_live_ = *h_live_;
  keys_since_rebuild_ = 0;
  live_pending_ = false;
  ++table_rebuilds_;
  ensure_tmp();  // the grouping sort's key width follows the table
  sync_keys();
}

// Dense key array (k_claim's probe target) from the table, on the join stream.
void DeviceJoin::sync_keys() {
  if (keys_cap_ != table_cap_) {
    if (d_keys_) {
      HIP_OK(hipStreamSynchronize(stream_));
      dfree(d_keys_, (size_t)keys_cap_ * 8);
    }
    d_keys_ = (uint64_t*)dmalloc((size_t)table_cap_ * 8);
    keys_cap_ = table_cap_;
  }
  apm_dj_keys_sync(d_table_, table_cap_, d_keys_, stream_);
  keys_stale_ = false;
}

// The same-size rebuild in stream order, without waiting for it: the live count arrives in h_live_
// with the batch's own syncs and is read at the next capacity check.  (A synchronous rebuild
// stalled the ingest thread ~0.5 ms every ~32 batches at the headline rate: the p99 step.)  It
// compacts the table's clusters in place (apm_dj_rebuild_inplace): no second table to zero and
// fill.  APM_REBUILD_COPY=1 keeps the reinsert-into-the-spare form (A/B).
bool DeviceJoin::rebuild_copy() {
  static const bool copy = [] { const char* e = std::getenv("APM_REBUILD_COPY"); return e && e[0] == '1'; }();
  return copy;
}

void DeviceJoin::rebuild_inplace(double now) {
  const size_t need = apm_dj_rebuild_scratch_bytes(table_cap_);
  if (need > rb_scratch_bytes_) {
    if (d_rb_scratch_) dfree(d_rb_scratch_, rb_scratch_bytes_);
    d_rb_scratch_ = (uint32_t*)dmalloc(need);
    rb_scratch_bytes_ = need;
  }
  HIP_OK(hipMemsetAsync(d_live_, 0, 8, stream_));
  apm_dj_rebuild_inplace(d_table_, table_cap_, d_rb_scratch_, d_arena_, cfg_.arena_cap, now, d_counts_, d_live_,
                         d_pool_, d_pool_ring_, pool_n_ - 1, stream_);
}

void DeviceJoin::rebuild_table_async(double now) {
  hipStream_t st = stream_;
  if (rebuild_copy()) {
    HIP_OK(hipMemsetAsync(d_live_, 0, 8, st));
    KeyState* fresh = d_table_spare_;
    if (!fresh) fresh = (KeyState*)dmalloc((size_t)table_cap_ * sizeof(KeyState));  // (zeroed)
    else if (!spare_clean_) HIP_OK(hipMemsetAsync(fresh, 0, (size_t)table_cap_ * sizeof(KeyState), st));
    apm_dj_rebuild(d_table_, table_cap_, fresh, table_cap_ - 1, d_arena_, cfg_.arena_cap, now, d_counts_, d_live_,
                   d_pool_, d_pool_ring_, pool_n_ - 1, st);
    d_table_spare_ = d_table_;  // (zeroed later, in an idle gap of the join stream)
    spare_clean_ = false;
    d_table_ = fresh;
  } else {
    rebuild_inplace(now);
  }
  sync_keys();  // (the join stream's idle gap, with the rebuild)
  HIP_OK(hipMemcpyAsync(h_live_, d_live_, 8, hipMemcpyDeviceToHost, st));
  if (!live_ev_) HIP_OK(hipEventCreateWithFlags(&live_ev_, hipEventDisableTiming));
  HIP_OK(hipEventRecord(live_ev_, st));
  keys_since_rebuild_ = 0;
  live_pending_ = true;
  ++table_rebuilds_;
}

// After a batch's last sync the join stream idles while the host finishes the batch (hand-off,
// clocks) and starts the next one: the key table's upkeep runs there instead of in front of the
// next batch's kernels -- the rebuild when the next batch (estimated as large as this one) would
// trigger it, else zeroing the spare table so a later rebuild skips its memset.  The clock is
// this batch's: only entries expired at it are dropped (later expiries are checked by the kernels).
void DeviceJoin::idle_upkeep(double now, uint32_t n_next) {
  static const int mode = [] {  // APM_IDLE_UPKEEP: 0 off, 1 spare zeroing only, 2 (default) + rebuild
    const char* e = std::getenv("APM_IDLE_UPKEEP");
    return e ? std::atoi(e) : 2;
  }();
  if (mode == 0 || live_pending_) return;  // (a rebuild's count is still unread)
  if (mode >= 2 && (keys_live_ + keys_since_rebuild_ + n_next) * 2 > table_cap_ && table_rebuilds_ > 0 &&
      async_rebuild_fits(n_next)) {
    rebuild_table_async(now);
  } else if (rebuild_copy() && d_table_spare_ && !spare_clean_) {
    HIP_OK(hipMemsetAsync(d_table_spare_, 0, (size_t)table_cap_ * sizeof(KeyState), stream_));
    spare_clean_ = true;
  }
}

// Need entries at virtual [lo, arena_head_) move to the same virtual slots of a bigger ring; the
// table's `need` links follow them (through NeedEnt::vidx).
void DeviceJoin::grow_arena(uint32_t new_cap, uint64_t lo) {
  hipStream_t st = stream_;
  NeedEnt* fresh = (NeedEnt*)dmalloc((size_t)new_cap * sizeof(NeedEnt));
  apm_dj_arena_grow(d_arena_, cfg_.arena_cap, fresh, new_cap, lo, arena_head_, d_table_, table_cap_, st);
  HIP_OK(hipStreamSynchronize(st));
  dfree(d_arena_, (size_t)cfg_.arena_cap * sizeof(NeedEnt));
  d_arena_ = fresh;
  // expiry scratch is sized by the arena
  for (void* p : {(void*)d_exp_key_, (void*)d_exp_key_sorted_}) dfree(p, ((size_t)exp_cap_ + 1) * 8);
  for (void* p : {(void*)d_exp_idx_, (void*)d_exp_idx_sorted_, (void*)d_exp_cnt_, (void*)d_exp_pos_})
    dfree(p, ((size_t)exp_cap_ + 1) * 4);
  cfg_.arena_cap = new_cap;
  exp_cap_ = new_cap;
  d_exp_key_ = (uint64_t*)dmalloc(((size_t)exp_cap_ + 1) * 8);
  d_exp_key_sorted_ = (uint64_t*)dmalloc(((size_t)exp_cap_ + 1) * 8);
  d_exp_idx_ = (uint32_t*)dmalloc(((size_t)exp_cap_ + 1) * 4);
  d_exp_idx_sorted_ = (uint32_t*)dmalloc(((size_t)exp_cap_ + 1) * 4);
  d_exp_cnt_ = (uint32_t*)dmalloc(((size_t)exp_cap_ + 1) * 4);
  d_exp_pos_ = (uint32_t*)dmalloc(((size_t)exp_cap_ + 1) * 4);
  ensure_tmp();
  ++arena_grows_;
}

// Capacity of an audit carry generation about to be written (its contents are not kept): every
// array grows to twice the bound so growth is rare; frees wait for the join stream.
void DeviceJoin::aud_reserve(AudGen& g, uint32_t autr, uint32_t items, uint64_t txt) {
  if (txt >= (1ull << 31)) throw std::runtime_error("device join: audit carry text beyond 2 GB");
  const bool grow = autr > g.cap_autr || items > g.cap_items || txt > g.cap_txt;
  if (!grow) return;
  HIP_OK(hipStreamSynchronize(stream_));
  if (autr > g.cap_autr) {
    dfree(g.autr, (size_t)g.cap_autr * sizeof(AutrEnt));
    g.cap_autr = std::max<uint32_t>(autr * 2, 4096);
    g.autr = (AutrEnt*)dmalloc((size_t)g.cap_autr * sizeof(AutrEnt));
  }
  if (items > g.cap_items) {
    dfree(g.items, (size_t)g.cap_items * sizeof(AudItem));
    g.cap_items = std::max<uint32_t>(items * 2, 16384);
    g.items = (AudItem*)dmalloc((size_t)g.cap_items * sizeof(AudItem));
  }
  if (txt > g.cap_txt) {
    dfree(g.txt, g.cap_txt);
    g.cap_txt = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(txt * 2, 1u << 20), (1ull << 32) - 1);
    g.txt = (char*)dmalloc(g.cap_txt);
  }
}

uint64_t DeviceJoin::pool_avail(bool exact) {
  if (exact) {
    HIP_OK(hipMemcpyAsync(h_counts_, d_counts_, sizeof(JoinCounts), hipMemcpyDeviceToHost, stream_));
    HIP_OK(hipStreamSynchronize(stream_));
  }
  return h_counts_->pool_tail - h_counts_->pool_head;
}

void DeviceJoin::grow_pool(uint64_t need_free) {
  hipStream_t st = stream_;
  const uint64_t avail = pool_avail(true);
  uint64_t n = pool_n_;
  while (avail + (n - pool_n_) < need_free) n *= 2;
  if (n >= (1ull << 31)) throw std::runtime_error("device join: chain pool beyond 2^31 blocks");
  uint8_t* pool = (uint8_t*)dmalloc((size_t)n * CHAIN_BLK);
  uint32_t* ring = (uint32_t*)dmalloc((size_t)n * 4);
  HIP_OK(hipMemcpyAsync(pool, d_pool_, (size_t)pool_n_ * CHAIN_BLK, hipMemcpyDeviceToDevice, st));
  apm_dj_pool_grow(d_pool_ring_, pool_n_ - 1, ring, pool_n_, (uint32_t)n, d_counts_, st);
  HIP_OK(hipStreamSynchronize(st));
  dfree(d_pool_, (size_t)pool_n_ * CHAIN_BLK);
  dfree(d_pool_ring_, (size_t)pool_n_ * 4);
  d_pool_ = pool;
  d_pool_ring_ = ring;
  pool_n_ = (uint32_t)n;
  pool_avail(true);
  ++pool_grows_;
}

void DeviceJoin::ensure_capacity(uint32_t n_ev, uint64_t bytes, double now) {
  // key table: every op of the batch may claim a new key
  if (live_pending_) {  // the in-order rebuild's count (queued at the previous batch's end)
    HIP_OK(hipEventSynchronize(live_ev_));
    keys_live_ = *h_live_;
    live_pending_ = false;
  }
  if ((keys_live_ + keys_since_rebuild_ + n_ev) * 2 > table_cap_) {
    // steady state: every key the queued rebuild may keep (the live count after the previous
    // rebuild plus the keys claimed since) and this batch's ops keep the table at most 5/8 full
    // -- rebuild in stream order; otherwise (growth may be due) wait for the count.  (A table a
    // little past half full only probes longer; the count read at the next check grows it if the
    // live keys really grew.)
    if (table_rebuilds_ > 0 && async_rebuild_fits(n_ev)) {
      rebuild_table_async(now);
      return ensure_rest(n_ev, bytes);
    }
    rebuild_table(now, table_cap_);
    uint64_t cap = table_cap_;
    while ((keys_live_ + n_ev) * 2 > cap) cap *= 2;
    if (cap >= (1ull << 31)) throw std::runtime_error("device join: key table beyond 2^31 slots");
    if (cap != table_cap_) rebuild_table(now, (uint32_t)cap);
  }
  ensure_rest(n_ev, bytes);
}

void DeviceJoin::ensure_rest(uint32_t n_ev, uint64_t bytes) {
  // need arena: every op may open one entry; entries of the regions expiring in this batch stay
  // untouched until k_write printed their logIds
  {
    const uint64_t low = regions_.empty() ? arena_head_ : regions_.front().lo;
    const uint64_t used = arena_head_ - low;
    uint64_t cap = cfg_.arena_cap;
    while (cap - used < n_ev) cap *= 2;
    if (cap >= (1ull << 31)) throw std::runtime_error("device join: need arena beyond 2^31 entries");
    if (cap != cfg_.arena_cap) grow_arena((uint32_t)cap, low);
  }
  // chain pool: one block per op (a partial or a parked record) + the logId bytes of new entries
  const uint64_t need = 2ull * n_ev + bytes / LBLK_N + 64;
  if (pool_avail(false) < need && pool_avail(true) < need) grow_pool(need);
}

void DeviceJoin::prepass_ahead(int k, const uint8_t* hb, const ParallelFor& parallel) {
  if (ahead_k_ >= 0) throw std::runtime_error("device join: a pre-pass is already ahead");
  // hops_ / hbuf_ hold the running batch's ops (register_misses reads hbuf_ after sync A)
  host_prepass(k, hb, sl_[k].h_n_host->host, parallel, hops_ahead_, hbuf_ahead_);
  ahead_k_ = k;
}

void DeviceJoin::run(int k, const uint8_t* hb, uint32_t n_ev, uint64_t n_bytes, double now, uint64_t batch_no,
                     bool want_tx, bool want_db, DevJoinBatch& out, const ParallelFor& parallel,
                     const std::function<void()>* meanwhile) {
  Slot& s = sl_[k];
  hipStream_t st = stream_;
  if (n_ev > cfg_.max_events) throw std::runtime_error("device join: more events than maxLinesPerBatch");
  events_ += n_ev;
  phase_t[0] = clock_ms();
  // ---- host pre-pass (audit blocks, PM_HOST lines)
  if (ahead_k_ == k) {  // done by prepass_ahead while the previous batch's kernels ran
    std::swap(hops_, hops_ahead_);
    std::swap(hbuf_, hbuf_ahead_);
    ahead_k_ = -1;
  } else {
    if (ahead_k_ >= 0) throw std::runtime_error("device join: pre-pass ahead for another slot");
    host_prepass(k, hb, s.h_n_host->host, parallel, hops_, hbuf_);
  }
  phase_t[1] = clock_ms();
  spans.clear();
  double sp = phase_t[1];
  auto span = [&](const char* name) { const double t = clock_ms(); spans.push_back({name, {sp, t}}); sp = t; };
  if (hops_.size() > h_hops_cap_) {
    if (h_hops_) HIP_OK(hipHostFree(h_hops_));
    h_hops_cap_ = hops_.size() * 2 + 65536;
    HIP_OK(hipHostMalloc((void**)&h_hops_, h_hops_cap_ * sizeof(HostOp), host_flags_()));
    HIP_OK(hipHostGetDevicePointer((void**)&hd_hops_, h_hops_, 0));
  }
  if (hbuf_.size() > h_hbuf_cap_) {
    if (h_hbuf_) HIP_OK(hipHostFree(h_hbuf_));
    h_hbuf_cap_ = hbuf_.size() * 2 + (4 << 20);
    HIP_OK(hipHostMalloc((void**)&h_hbuf_, h_hbuf_cap_, host_flags_()));
    HIP_OK(hipHostGetDevicePointer((void**)&hd_hbuf_, h_hbuf_, 0));
  }
  span("u.hostgrow");
  if (hops_.size() > d_hops_cap_) {
    d_hops_cap_ = hops_.size() * 2 + 65536;
    HostOp* p = nullptr;
    HIP_OK(hipMalloc((void**)&p, d_hops_cap_ * sizeof(HostOp)));
    allocs_.push_back(p);
    d_hops_ = p;  // the old buffer stays allocated (rare growth)
  }
  if (hbuf_.size() > d_hbuf_cap_) {
    d_hbuf_cap_ = hbuf_.size() * 2 + (4 << 20);
    uint8_t* p = nullptr;
    HIP_OK(hipMalloc((void**)&p, d_hbuf_cap_));
    allocs_.push_back(p);
    d_hbuf_ = p;
  }
  span("u.devgrow");
  // The host ops (~160 KB a batch) are read by a kernel over the host link (apm_copy on the join
  // stream).  A DMA copy queues behind the next batch's 22 MB of log bytes on the copy engine: on
  // its own stream it cost 1.44-1.50 vs 1.20-1.23 ms per step (round-3 A/B, 60 steps), and a fifth
  // stream for it shares the 4 hardware queues -- so no separate upload stream exists.
  if (!hops_.empty()) {
    std::memcpy(h_hops_, hops_.data(), hops_.size() * sizeof(HostOp));
    span("u.hops.memcpy");
    apm_copy(d_hops_, hd_hops_, hops_.size() * sizeof(HostOp), st);
    span("u.hops.h2d");
  }
  if (!hbuf_.empty()) {
    std::memcpy(h_hbuf_, hbuf_.data(), hbuf_.size());
    span("u.hbuf.memcpy");
    apm_copy(d_hbuf_, hd_hbuf_, hbuf_.size(), st);
    span("u.hbuf.h2d");
  }
  // ---- file -> server table (and the files' keys, normally synced by the parse's select_host)
  sync_file_keys();
  if (files_->size() > files_uploaded_) {
    if (files_->size() > soap_cap_) throw std::runtime_error("device join: too many files");
    std::vector<int32_t> fs(files_->size() - files_uploaded_);
    for (size_t i = files_uploaded_; i < files_->size(); ++i) fs[i - files_uploaded_] = (*files_)[i].server;
    HIP_OK(hipMemcpyAsync(d_file_server_ + files_uploaded_, fs.data(), fs.size() * 4, hipMemcpyHostToDevice, st));
    HIP_OK(hipStreamSynchronize(st));
    files_uploaded_ = files_->size();
  }
  ensure_capacity(n_ev, n_bytes + hbuf_.size(), now);
  span("u.capacity");
  const uint64_t arena_low = regions_.empty() ? arena_head_ : regions_.front().lo;  // before expiry
  const uint32_t arena_limit = (uint32_t)((uint64_t)cfg_.arena_cap - (arena_head_ - arena_low));
  // ---- needNumRecordCache regions whose TTL passed (front of the creation-ordered FIFO)
  uint32_t n_reg = 0, n_exp = 0;
  while (!regions_.empty() && regions_.front().exp < now && n_reg < 4096) {
    h_exp_[n_reg] = regions_.front().lo;
    h_exp_[4096 + n_reg] = regions_.front().hi;
    n_exp += (uint32_t)(regions_.front().hi - regions_.front().lo);
    regions_.pop_front();
    ++n_reg;
  }
  if (n_reg) {
    apm_copy(d_exp_lo_, hd_exp_, (size_t)n_reg * 8, st);
    apm_copy(d_exp_hi_, (const uint64_t*)hd_exp_ + 4096, (size_t)n_reg * 8, st);
  }
  span("u.files+exp");
  // ---- join
  DJArgs& a = a_;
  a = DJArgs{};
  a.ev = s.d_events; a.n_ev = n_ev; a.bytes = s.d_bytes;
  a.chunk_file = s.d_chunk_file; a.chunk_kind = s.d_chunk_kind; a.n_chunks = s.n_chunks;
  a.chunk_next = s.d_chunk_next; a.chunk_first = s.d_chunk_first; a.file_server = d_file_server_;
  a.file_skey = d_file_skey_; a.file_fkey = d_file_fkey_;
  a.hops = d_hops_; a.n_hops = (uint32_t)hops_.size(); a.hbuf = d_hbuf_;
  a.now = now; a.batch_no = batch_no;
  a.rec_ttl = cfg_.record_ttl_ms; a.acct_ttl = cfg_.acct_ttl_ms; a.need_ttl = cfg_.need_ttl_ms;
  a.host_flag = s.host_flag;
  a.ops = d_ops_; a.soap_code = d_soap_code_; a.soap_num = d_soap_num_; a.soap_hash = d_soap_hash_;
  a.chunk_ev_lo = d_chunk_ev_lo_; a.seg_f = d_seg_f_; a.seg_in = d_seg_in_; a.chain_hash = d_chain_hash_;
  a.soap_state = d_soap_;
  a.op_slot = d_op_slot_; a.op_slot_sorted = d_op_slot_sorted_; a.op_idx = d_op_idx_; a.op_idx_sorted = d_op_idx_sorted_;
  a.tmp = d_tmp_; a.tmp_bytes = tmp_bytes_;
  if (!group_sort_ && heads_cap_ != table_cap_) {  // (the join stream is ordered after any rebuild)
    if (d_slot_head_) { HIP_OK(hipStreamSynchronize(st)); dfree(d_slot_head_, (size_t)heads_cap_ * 4); }
    d_slot_head_ = (uint32_t*)dmalloc((size_t)table_cap_ * 4);
    HIP_OK(hipMemsetAsync(d_slot_head_, 0xff, (size_t)table_cap_ * 4, st));
    heads_cap_ = table_cap_;
  }
  a.slot_head = d_slot_head_; a.big = d_big_; a.group_sort = group_sort_ ? 1 : 0;
  if (keys_stale_ || keys_cap_ != table_cap_) sync_keys();
  a.table = d_table_; a.keys = d_keys_; a.table_mask = table_cap_ - 1; a.table_bits = table_bits_;
  a.pool = d_pool_; a.pool_ring = d_pool_ring_; a.pool_mask = pool_n_ - 1;
  a.reg = d_reg_; a.reg_mask = (1u << cfg_.reg_bits) - 1; a.miss = d_miss_; a.miss_cap = miss_cap_;
  a.arena = d_arena_; a.arena_cap = cfg_.arena_cap; a.arena_base = arena_head_; a.arena_limit = arena_limit;
  a.exp_lo = d_exp_lo_; a.exp_hi = d_exp_hi_; a.n_exp_regions = n_reg; a.n_exp_entries = n_exp;
  a.exp_key = d_exp_key_; a.exp_key_sorted = d_exp_key_sorted_; a.exp_idx = d_exp_idx_;
  a.exp_idx_sorted = d_exp_idx_sorted_; a.exp_cnt = d_exp_cnt_; a.exp_pos = d_exp_pos_;
  a.out_cnt = d_out_cnt_; a.out_pos = d_out_pos_; a.stage = d_stage_; a.ovf = d_ovf_;
  a.out = d_out_; a.out_cap = out_cap_; a.counts = d_counts_;
  // ---- audit trail (K5): this batch reads generation aud_cur_, writes the other one
  {
    const SelCount tot = *s.h_n_host;
    AudGen& gin = aud_gen_[aud_cur_];
    AudGen& gout = aud_gen_[aud_cur_ ^ 1];
    aud_reserve(gout, gin.n_autr + tot.mh, gin.n_items + tot.walk, (uint64_t)gin.n_txt + tot.aud_bytes);
    const uint32_t N = gin.n_autr + tot.mh;
    if (N + 1 > aud_key_cap_) {
      HIP_OK(hipStreamSynchronize(st));
      for (void* p : {(void*)d_aud_key_, (void*)d_aud_key_sorted_}) dfree(p, (size_t)aud_key_cap_ * 8);
      for (void* p : {(void*)d_aud_ord_, (void*)d_aud_ord_sorted_}) dfree(p, (size_t)aud_key_cap_ * 4);
      aud_key_cap_ = std::max<uint32_t>(2 * (N + 1), 1u << 14);
      d_aud_key_ = (uint64_t*)dmalloc((size_t)aud_key_cap_ * 8);
      d_aud_key_sorted_ = (uint64_t*)dmalloc((size_t)aud_key_cap_ * 8);
      d_aud_ord_ = (uint32_t*)dmalloc((size_t)aud_key_cap_ * 4);
      d_aud_ord_sorted_ = (uint32_t*)dmalloc((size_t)aud_key_cap_ * 4);
    }
    if (N > std::max<uint32_t>(cfg_.max_events, cfg_.arena_cap)) {  // the key sort's scratch
      const size_t need = apm_dj_tmp_bytes(N, out_cap_, table_bits_);
      if (need > tmp_bytes_) {
        HIP_OK(hipStreamSynchronize(st));
        dfree(d_tmp_, tmp_bytes_);
        tmp_bytes_ = need;
        d_tmp_ = dmalloc(tmp_bytes_);
        a.tmp = d_tmp_; a.tmp_bytes = tmp_bytes_;
      }
    }
    const uint32_t slots = tot.walk + gin.n_items;
    if (slots > aud_slots_cap_) {
      HIP_OK(hipStreamSynchronize(st));
      dfree(d_aud_slots_, (size_t)aud_slots_cap_ * sizeof(AudItem));
      aud_slots_cap_ = std::max<uint32_t>(2 * slots, 1u << 14);
      d_aud_slots_ = (AudItem*)dmalloc((size_t)aud_slots_cap_ * sizeof(AudItem));
    }
    a.n_mh = tot.mh; a.n_walk = tot.walk; a.n_files = (uint32_t)files_->size();
    a.aud = s.d_aud; a.gin = gin; a.gout = gout;
    a.mh_idx = s.d_mh_idx; a.walk_idx = s.d_walk_idx;
    a.aud_key = d_aud_key_; a.aud_key_sorted = d_aud_key_sorted_; a.aud_ord = d_aud_ord_; a.aud_ord_sorted = d_aud_ord_sorted_;
    a.walk_lo = d_walk_lo_; a.file_first_chunk = d_file_first_; a.aud_slots = d_aud_slots_;
  }
  // the stats thread is done with the slot's hand-off arrays (after the capacity upkeep, which
  // may synchronize this stream and must not wait for the stats thread)
  if (s.used) HIP_OK(hipStreamWaitEvent(st, s.free_ev, 0));
  static const bool dbg = std::getenv("APM_DJ_DEBUG") != nullptr;
  if (dbg) {  // (see devjoin.hip dj_check): the uploads before the join kernels
    const hipError_t e = hipStreamSynchronize(st);
    if (e != hipSuccess) { fprintf(stderr, "[devjoin debug] before the join: %s\n", hipGetErrorString(e)); abort(); }
  }
  phase_t[2] = clock_ms();
  if (apm_dj_join(&a, st) != 0) throw std::runtime_error("device join: scan scratch too small");
  HIP_OK(hipMemcpyAsync(h_counts_, d_counts_, sizeof(JoinCounts), hipMemcpyDeviceToHost, st));
  if (meanwhile) (*meanwhile)();
  phase_t[3] = clock_ms();
  HIP_OK(hipStreamSynchronize(st));  // ---- sync A
  phase_t[4] = clock_ms();
  const JoinCounts c = *h_counts_;
  if (c.n_out > out_cap_) throw std::runtime_error("device join: more tx in one batch than the output capacity");
  if (c.aud_pad) throw std::runtime_error("device join: audit carry over capacity (sizing bug)");
  {
    AudGen& gout = aud_gen_[aud_cur_ ^ 1];
    gout.n_autr = c.aud_autr_n; gout.n_items = c.aud_items_n; gout.n_txt = c.aud_txt_n;
  }
  if (c.pad[0] > DJ_OVF_CAP) throw std::runtime_error("device join: output overflow list full");
  if (c.n_need_new) {
    const uint32_t cnt = std::min(c.n_need_new, arena_limit);
    regions_.push_back(Region{arena_head_, arena_head_ + cnt, now + cfg_.need_ttl_ms});
    arena_head_ += cnt;
  }
  keys_since_rebuild_ += c.n_keys_new;
  if (c.n_miss) register_misses(hb, c.n_miss, st);
  phase_t[5] = clock_ms();
  // ---- resolve + plan
  DJFormatArgs& f = f_;
  f = DJFormatArgs{};
  f.out = d_out_; f.n_out = c.n_out; f.reg = d_reg_; f.reg_mask = (1u << cfg_.reg_bits) - 1;
  f.raw = d_rawtab_; f.raw_series = d_raw_series_; f.raw_first = d_raw_first_; f.names = d_names_;
  f.bytes = s.d_bytes; f.hbuf = d_hbuf_; f.aud_txt = aud_gen_[aud_cur_].txt; f.arena = d_arena_; f.arena_cap = cfg_.arena_cap; f.pool = d_pool_;
  f.lens = d_lens_; f.offs = d_offs_; f.ring = d_ring_; f.ring_cap = cfg_.ring_bytes;
  f.tx = s.d_tx; f.tx_raw = s.d_tx_raw; f.tx_gid = s.d_tx_gid; f.tx_bucket = d_bucket_; f.tx_bmax = d_bmax_;
  f.cand = d_cand_; f.cand_bucket = d_cand_bucket_; f.unresolved = d_unres_;
  f.want_tx = want_tx; f.want_db = want_db; f.counts = d_counts_; f.tmp = d_tmp_; f.tmp_bytes = tmp_bytes_;
  // the ring region and the write verdict are decided on the device (k_plan_totals): no sync
  // between the plan and the write pass; the host learns both at sync C
  const uint64_t ring_head = ring_head_.load(std::memory_order_acquire);
  f.ring_head = ring_head;
  f.ring_low = ring_low_.load(std::memory_order_acquire);
  f.ring_pos = d_ring_pos_;
  if (want_tx || want_db) ensure_txt(std::max<size_t>(txt_cap_, 4u << 20));
  f.txt_tx = d_txt_tx_;
  f.txt_db = d_txt_db_;
  f.txt_cap = txt_cap_;
  if (apm_dj_plan(&f, st) != 0) throw std::runtime_error("device join: scan scratch too small");
  phase_t[6] = clock_ms();
  // copy-backs sized before the sizes are known: the previous batch's x 2 (the rest after sync C)
  const uint32_t spec = std::min<uint32_t>(c.n_out, std::max<uint32_t>(2 * last_cands_, 1024));
  const size_t spec_tx = want_tx ? std::min<size_t>(txt_cap_, 2 * (size_t)last_tx_bytes_ + 65536) : 0;
  const size_t spec_db = want_db ? std::min<size_t>(txt_cap_, 2 * (size_t)last_db_bytes_ + 65536) : 0;
  if (spec_tx + spec_db > h_txt_cap_) {
    if (h_txt_) HIP_OK(hipHostFree(h_txt_));
    h_txt_cap_ = (spec_tx + spec_db) * 2 + (4 << 20);
    HIP_OK(hipHostMalloc((void**)&h_txt_, h_txt_cap_, hipHostMallocDefault));
  }
  // the read-back: one kernel writing the host-mapped buffers (a blit per array before: six
  // launches on the join lane's critical path)
  auto mapped = [](void* h) {
    void* d = nullptr;
    HIP_OK(hipHostGetDevicePointer(&d, h, 0));
    return d;
  };
  auto write_and_copy = [&] {
    if (apm_dj_write(&f, st) != 0) throw std::runtime_error("device join: scan scratch too small");
    static const bool seg = [] {  // A/B: APM_DJ_SEGCOPY=0 -> a blit per array
      const char* e = std::getenv("APM_DJ_SEGCOPY");
      return !e || std::atoi(e) != 0;
    }();
    if (!seg) {
      if (spec) {
        HIP_OK(hipMemcpyAsync(h_cand_, d_cand_, (size_t)spec * 4, hipMemcpyDeviceToHost, st));
        HIP_OK(hipMemcpyAsync(h_cand_bucket_, d_cand_bucket_, (size_t)spec * 8, hipMemcpyDeviceToHost, st));
        HIP_OK(hipMemcpyAsync(h_unres_, d_unres_, (size_t)spec * 8, hipMemcpyDeviceToHost, st));
      }
      if (spec_tx) HIP_OK(hipMemcpyAsync(h_txt_, d_txt_tx_, spec_tx, hipMemcpyDeviceToHost, st));
      if (spec_db) HIP_OK(hipMemcpyAsync(h_txt_ + spec_tx, d_txt_db_, spec_db, hipMemcpyDeviceToHost, st));
      HIP_OK(hipMemcpyAsync(h_counts_, d_counts_, sizeof(JoinCounts), hipMemcpyDeviceToHost, st));
      HIP_OK(hipStreamSynchronize(st));  // ---- sync C
      return;
    }
    CopySegs cs;
    if (spec) {
      cs.add(mapped(h_cand_), d_cand_, (size_t)spec * 4);
      cs.add(mapped(h_cand_bucket_), d_cand_bucket_, (size_t)spec * 8);
      cs.add(mapped(h_unres_), d_unres_, (size_t)spec * 8);
    }
    if (spec_tx) cs.add(mapped(h_txt_), d_txt_tx_, spec_tx);
    if (spec_db) cs.add((char*)mapped(h_txt_) + spec_tx, d_txt_db_, spec_db);
    cs.add(mapped(h_counts_), d_counts_, sizeof(JoinCounts));
    apm_copy_segs(&cs, st);
    HIP_OK(hipStreamSynchronize(st));  // ---- sync C
  };
  write_and_copy();
  JoinCounts c3 = *h_counts_;
  if (c3.pad[1] == DJ_WRITE_TXT) {  // the staging grows; the write pass runs again (it wrote nothing)
    ensure_txt(std::max<size_t>(c3.tx_text_bytes, c3.db_text_bytes) * 2 + (16 << 20));
    f.txt_tx = d_txt_tx_;
    f.txt_db = d_txt_db_;
    f.txt_cap = txt_cap_;
    static_assert(DJ_WRITE_OK == 0, "the verdict is cleared by a zero fill");
    HIP_OK(hipMemsetAsync(&d_counts_->pad[1], 0, 4, st));
    ++write_regrows_;
    write_and_copy();
    c3 = *h_counts_;
  }
  if (c3.pad[1] == DJ_WRITE_TOO_BIG)
    throw std::runtime_error("device join: one batch of tx text exceeds a quarter of gpu.txTextRingMB");
  if (c3.pad[1] == DJ_WRITE_RING_FULL)
    throw std::runtime_error("device join: tx text ring exhausted (pending released-tx lines span more than "
                             "gpu.txTextRingMB; raise it)");
  if (c3.pad[1] != DJ_WRITE_OK) throw std::runtime_error("device join: write pass skipped");
  phase_t[7] = clock_ms();
  const uint64_t ring_base = ring_place(ring_head, c3.text_bytes, cfg_.ring_bytes);
  {
    std::lock_guard<std::mutex> g(ring_mu_);
    ring_head_.store(ring_base + c3.text_bytes, std::memory_order_release);
  }
  const uint32_t tx_bytes = want_tx ? c3.tx_text_bytes : 0, db_bytes = want_db ? c3.db_text_bytes : 0;
  if (c3.n_cand > spec || c3.n_unresolved > spec || tx_bytes > spec_tx || db_bytes > spec_db) {
    if (c3.n_cand > spec || c3.n_unresolved > spec) {
      HIP_OK(hipMemcpyAsync(h_cand_, d_cand_, (size_t)c3.n_cand * 4, hipMemcpyDeviceToHost, st));
      HIP_OK(hipMemcpyAsync(h_cand_bucket_, d_cand_bucket_, (size_t)c3.n_cand * 8, hipMemcpyDeviceToHost, st));
      HIP_OK(hipMemcpyAsync(h_unres_, d_unres_, (size_t)c3.n_unresolved * 8, hipMemcpyDeviceToHost, st));
    }
    if (tx_bytes > spec_tx || db_bytes > spec_db) {  // (both streams again, into a larger buffer)
      if ((size_t)tx_bytes + db_bytes > h_txt_cap_) {
        HIP_OK(hipStreamSynchronize(st));
        if (h_txt_) HIP_OK(hipHostFree(h_txt_));
        h_txt_cap_ = ((size_t)tx_bytes + db_bytes) * 2 + (4 << 20);
        HIP_OK(hipHostMalloc((void**)&h_txt_, h_txt_cap_, hipHostMallocDefault));
      }
      if (tx_bytes) HIP_OK(hipMemcpyAsync(h_txt_, d_txt_tx_, tx_bytes, hipMemcpyDeviceToHost, st));
      if (db_bytes) HIP_OK(hipMemcpyAsync(h_txt_ + tx_bytes, d_txt_db_, db_bytes, hipMemcpyDeviceToHost, st));
    }
    HIP_OK(hipStreamSynchronize(st));
  }
  const char* h_tx_txt = h_txt_;
  const char* h_db_txt = h_txt_ + ((tx_bytes > spec_tx || db_bytes > spec_db) ? tx_bytes : spec_tx);
  last_tx_bytes_ = tx_bytes;
  last_db_bytes_ = db_bytes;
  last_cands_ = std::max(c3.n_cand, c3.n_unresolved);
  out.slot = k;
  out.n_out = c3.n_out;
  out.n_stats = c3.n_stats;
  out.n_db = c3.n_db;
  out.n_dropped = c3.n_dropped;
  out.ring_base = ring_base;
  out.d_tx = s.d_tx;
  out.d_raw = s.d_tx_raw;
  out.d_gid = s.d_tx_gid;
  out.cands.resize(c3.n_cand);
  out.max_bucket = INT64_MIN;
  for (uint32_t i = 0; i < c3.n_cand; ++i) {
    out.cands[i] = {h_cand_[i], h_cand_bucket_[i]};
    out.max_bucket = std::max(out.max_bucket, h_cand_bucket_[i]);
  }
  std::sort(out.cands.begin(), out.cands.end());
  out.unresolved.resize(c3.n_unresolved);
  for (uint32_t i = 0; i < c3.n_unresolved; ++i) out.unresolved[i] = {h_unres_[2 * i], (int32_t)h_unres_[2 * i + 1]};
  std::sort(out.unresolved.begin(), out.unresolved.end());
  out.text_tx.clear();
  out.text_db.clear();
  if (want_tx) out.text_tx.assign(h_tx_txt, tx_bytes);
  if (want_db) out.text_db.assign(h_db_txt, db_bytes);
  tx_ += c3.n_out;
  tx_db_ += c3.n_db;
  aud_cur_ ^= 1;  // the next batch reads what this one carried
  idle_upkeep(now, n_ev);
  phase_t[8] = clock_ms();
  {  // APM_DJ_MARKS=1: one span per launch (host time from the previous mark)
    double t[64];
    const char* nm[64];
    const int m = apm_dj_take_marks(t, nm, 64);
    double prev = phase_t[2];
    for (int i = 0; i < m; ++i) {
      spans.push_back({nm[i], {prev, t[i]}});
      prev = t[i];
    }
  }
}

size_t DeviceJoin::trim(double now) {
  hipStream_t st = stream_;
  HIP_OK(hipStreamSynchronize(st));
  if (live_pending_) {
    HIP_OK(hipEventSynchronize(live_ev_));
    keys_live_ = *h_live_;
    live_pending_ = false;
  }
  const size_t before = device_bytes_;
  const uint64_t tg = table_grows_, ag = arena_grows_;  // (a shrink is not a growth event)
  auto pow2_at_least = [](uint64_t v) { uint64_t p = 1; while (p < v) p <<= 1; return p; };
  // key table: an exact live count first (same-size rebuild, expired keys dropped at `now`) --
  // only when the table is above its configured size (else nothing can shrink: no rebuild)
  if (table_cap_ > init_table_cap_) {
    rebuild_table(now, table_cap_);
    const uint64_t want = std::max<uint64_t>(init_table_cap_, pow2_at_least(std::max<uint64_t>(keys_live_ * 4, 8)));
    if (want < table_cap_) rebuild_table(now, (uint32_t)want);  // reinserts into a fresh, smaller table
  }
  if (d_table_spare_) {  // (re-made on demand: checkpoint compaction, APM_REBUILD_COPY)
    dfree(d_table_spare_, (size_t)table_cap_ * sizeof(KeyState));
    d_table_spare_ = nullptr;
    spare_clean_ = false;
  }
  if (d_slot_head_) {  // sized by the table: re-made by the next batch
    dfree(d_slot_head_, (size_t)heads_cap_ * 4);
    d_slot_head_ = nullptr;
    heads_cap_ = 0;
  }
  if (d_rb_scratch_) {  // sized by the table: re-made by the next in-place rebuild
    dfree(d_rb_scratch_, rb_scratch_bytes_);
    d_rb_scratch_ = nullptr;
    rb_scratch_bytes_ = 0;
  }
  // need arena: live entries [lo, head) move into a smaller ring (their virtual indices stay)
  {
    const uint64_t lo = regions_.empty() ? arena_head_ : regions_.front().lo;
    const uint64_t live = arena_head_ - lo;
    const uint64_t acap = std::max<uint64_t>(init_arena_cap_, pow2_at_least(std::max<uint64_t>(live * 4, 1024)));
    if (acap < cfg_.arena_cap) grow_arena((uint32_t)acap, lo);
  }
  // tx / audit text staging of the write pass (re-made by the next batch that needs it)
  if (d_txt_tx_) {
    HIP_OK(hipFree(d_txt_tx_));
    device_bytes_ -= txt_cap_ * 2;
    d_txt_tx_ = d_txt_db_ = nullptr;
    txt_cap_ = 0;
  }
  HIP_OK(hipStreamSynchronize(st));
  table_grows_ = tg;
  arena_grows_ = ag;
  ++trims_;
  return before > device_bytes_ ? before - device_bytes_ : 0;
}

std::vector<uint64_t> DeviceJoin::cache_stats(double now, bool sync) {
  if (!d_cstats_) {
    d_cstats_ = (unsigned long long*)dmalloc(64);
    HIP_OK(hipHostMalloc((void**)&h_cstats_, 64, hipHostMallocDefault));
    HIP_OK(hipEventCreateWithFlags(&cstats_ev_, hipEventDisableTiming));
  }
  // A stat line (sync = false) reads the previous interval's counts when they are ready and
  // queues this interval's count on the join stream -- no host wait on the ingest path; the
  // drained form (sync) counts now and waits.
  if (!sync && cstats_pending_ && hipEventQuery(cstats_ev_) == hipSuccess) {
    std::memcpy(cstats_last_, h_cstats_, sizeof cstats_last_);
    cstats_last_cap_ = cstats_cap_;
    cstats_pending_ = false;
  }
  if (sync || !cstats_pending_) {
    apm_dj_cache_stats(d_table_, table_cap_, now, d_cstats_, stream_);
    HIP_OK(hipMemcpyAsync(h_cstats_, d_cstats_, 5 * 8, hipMemcpyDeviceToHost, stream_));
    HIP_OK(hipEventRecord(cstats_ev_, stream_));
    cstats_cap_ = table_cap_;
    cstats_pending_ = true;
    if (sync || !cstats_have_) {
      HIP_OK(hipEventSynchronize(cstats_ev_));
      std::memcpy(cstats_last_, h_cstats_, sizeof cstats_last_);
      cstats_last_cap_ = cstats_cap_;
      cstats_pending_ = false;
      cstats_have_ = true;
    }
  }
  const unsigned long long* h = cstats_last_;
  return {(uint64_t)cstats_last_cap_, h[0], h[1], h[2], h[3], h[4]};
}

JoinCounters DeviceJoin::counters() const {
  const JoinCounts& c = *h_counts_;
  JoinCounters t;
  t.events = events_;
  t.tx = tx_;
  t.tx_db = tx_db_;
  t.expired_partials = c.expired_partials;
  t.need_expired = c.need_expired;
  t.ejb_exit_unmatched = c.ejb_unmatched;
  t.invalid_acct = c.invalid_acct + host_invalid_acct_;
  t.audit_errors = audit_errors_ + c.audit_errors;
  t.host_fallback = host_pm_;  // lines the parser deferred (and audit lines whose fields the GPU could not read)
  t.partial_overflow = c.partial_overflow;
  t.need_overflow = c.need_overflow;
  t.table_full = c.table_full;
  t.pool_exhausted = c.pool_fail;
  t.chain_partial_blocks = c.chain_parts;
  t.chain_need_blocks = c.chain_items;
  t.chain_logid_blocks = c.chain_lids;
  t.table_slots = table_cap_;
  t.table_grows = table_grows_;
  t.table_rebuilds = table_rebuilds_;
  t.trims = trims_;
  t.need_arena_entries = cfg_.arena_cap;
  t.arena_grows = arena_grows_;
  t.chain_pool_blocks = pool_n_;
  t.pool_grows = pool_grows_;
  t.host_events = host_events_;
  return t;
}

// ---------------------------------------------------------------------------- checkpoint
// Key table (live slots), need arena (live regions) and the chain blocks they reach, into a
// memory writer: vec(live KeyState), arena_cap, arena_head, regions, vec(NeedEnt), vec(blocks)
// -- chain links renumbered 1..n in the file, in place in the writer's buffer.
void DeviceJoin::save_tables(BinWriter& w) {
  hipStream_t st = stream_;
  double sp = clock_ms();
  auto span = [&](const char* name) { const double t = clock_ms(); save_spans.push_back({name, {sp, t}}); sp = t; };
  if (!h_ck_bounce_) HIP_OK(hipHostMalloc((void**)&h_ck_bounce_, kCkBounce, hipHostMallocDefault));
  // live (non-empty) slots, selected on the device
  uint32_t n_live = 0;
  size_t live_off = 0;
  {
    const size_t tb = apm_dj_live_tmp_bytes(table_cap_);
    // the spare table is the compaction target (kept: the in-place rebuild leaves no spare, and a
    // hipMalloc / hipFree of a table-sized buffer per checkpoint costs milliseconds and a device sync)
    if (!d_table_spare_) d_table_spare_ = (KeyState*)dmalloc((size_t)table_cap_ * sizeof(KeyState));
    KeyState* out = d_table_spare_;
    void* tmp = nullptr;
    HIP_OK(hipMalloc(&tmp, tb + 64));
    uint32_t* d_n = (uint32_t*)((char*)tmp + tb);
    apm_dj_live_compact(d_table_, table_cap_, out, d_n, tmp, tb, st);
    HIP_OK(hipMemcpyAsync(&n_live, d_n, 4, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    w.pod<uint64_t>(n_live);
    live_off = w.mem_pos();
    write_dev(w, out, (size_t)n_live * sizeof(KeyState), st, h_ck_bounce_, kCkBounce);
    HIP_OK(hipFree(tmp));
    // (the compaction scratch: only the reinsert rebuild (APM_REBUILD_COPY=1) targets the spare
    // and needs it zeroed again; the in-place rebuild never reads it)
    if (rebuild_copy()) spare_clean_ = false;
  }
  span("ck.j.table");
  // needNumRecordCache regions + their arena entries (arena capacity first: the table's `need`
  // links are physical slots of an arena of that size)
  w.pod(cfg_.arena_cap);
  w.pod(arena_head_);
  w.pod<uint64_t>(regions_.size());
  for (const Region& r : regions_) { w.pod(r.lo); w.pod(r.hi); w.pod(r.exp); }
  const uint64_t lo = regions_.empty() ? arena_head_ : regions_.front().lo;
  const size_t n_ents = (size_t)(arena_head_ - lo);
  w.pod<uint64_t>(n_ents);
  const size_t ents_off = w.mem_pos();
  if (n_ents) {  // the live range of the arena ring in (at most) two copies, not one per entry
    const uint64_t cap = cfg_.arena_cap, first = lo & (cap - 1);
    const uint64_t n1 = std::min<uint64_t>(n_ents, cap - first);
    write_dev(w, d_arena_ + first, (size_t)n1 * sizeof(NeedEnt), st, h_ck_bounce_, kCkBounce);
    if (n_ents > n1) write_dev(w, d_arena_, (size_t)(n_ents - n1) * sizeof(NeedEnt), st, h_ck_bounce_, kCkBounce);
  }
  span("ck.j.arena");
  // chain blocks reachable from the live state, renumbered 1..n in the file.  Only those blocks
  // are read (gathered on the device one chain level at a time): the whole pool is ~256 MB.
  // The chain heads (key partials, entry items / logIds) are read from the device (the snapshot's
  // table and arena bytes may still be on their way: CkDefer holes) and the renumbered heads are
  // written into the blob -- or, while the snapshot defers its reads, recorded as patches the
  // checkpoint writer applies after it filled the holes.
  CkDefer* const defer = ck_defer();
  auto put32 = [&](size_t off, int32_t v) {
    if (defer) defer->patches.push_back({off, v});
    else std::memcpy(w.mem_at(off), &v, 4);
  };
  // the fields gathered on the device into one packed buffer, then one D2H:
  // [pblk x n_live][key (2 words) x n_ents][iblk x n_ents][lblk x n_ents]
  std::vector<int32_t> pblk(n_live), iblk(n_ents), lblk(n_ents);
  std::vector<uint64_t> ekey(n_ents);
  {
    const size_t words = (size_t)n_live + 4 * n_ents;
    uint32_t* d_f = nullptr;
    if (words) HIP_OK(hipMalloc((void**)&d_f, words * 4));
    apm_dj_gather_field((const char*)d_table_spare_ + offsetof(KeyState, pblk), sizeof(KeyState), n_live, 1, d_f, st);
    uint32_t* fk = d_f + n_live;
    uint32_t* fi = fk + 2 * n_ents;
    uint32_t* fl = fi + n_ents;
    if (n_ents) {
      const uint64_t cap = cfg_.arena_cap, first = lo & (cap - 1);
      const uint64_t n1 = std::min<uint64_t>(n_ents, cap - first);
      for (int part = 0; part < 2; ++part) {
        const size_t at = part ? (size_t)n1 : 0, cnt = part ? (size_t)(n_ents - n1) : (size_t)n1;
        const char* src = (const char*)(d_arena_ + (part ? 0 : first));
        apm_dj_gather_field(src + offsetof(NeedEnt, key), sizeof(NeedEnt), (uint32_t)cnt, 2, fk + 2 * at, st);
        apm_dj_gather_field(src + offsetof(NeedEnt, iblk), sizeof(NeedEnt), (uint32_t)cnt, 1, fi + at, st);
        apm_dj_gather_field(src + offsetof(NeedEnt, lblk), sizeof(NeedEnt), (uint32_t)cnt, 1, fl + at, st);
      }
    }
    if (words) {
      std::vector<uint32_t> h(words);
      HIP_OK(hipMemcpyAsync(h.data(), d_f, words * 4, hipMemcpyDeviceToHost, st));
      HIP_OK(hipStreamSynchronize(st));
      HIP_OK(hipFree(d_f));
      std::memcpy(pblk.data(), h.data(), (size_t)n_live * 4);
      std::memcpy(ekey.data(), h.data() + n_live, n_ents * 8);
      std::memcpy(iblk.data(), h.data() + n_live + 2 * n_ents, n_ents * 4);
      std::memcpy(lblk.data(), h.data() + n_live + 3 * n_ents, n_ents * 4);
    }
  }
  struct Blk { uint8_t b[CHAIN_BLK]; };
  std::vector<Blk> blocks;
  {
    std::vector<int32_t> cur;      // pool block numbers (1-based) to fetch
    std::vector<size_t> slot_of;   // level 0: where (writer offset) each head's new number goes
    for (uint32_t i = 0; i < n_live; ++i) {
      const size_t o = live_off + (size_t)i * sizeof(KeyState) + offsetof(KeyState, pblk);
      if (const int32_t b = pblk[i]) { cur.push_back(b); slot_of.push_back(o); }
    }
    for (size_t i = 0; i < n_ents; ++i) {
      const size_t e = ents_off + i * sizeof(NeedEnt);
      const size_t oi = e + offsetof(NeedEnt, iblk), ol = e + offsetof(NeedEnt, lblk);
      if (!ekey[i]) { put32(oi, 0); put32(ol, 0); continue; }
      if (const int32_t b = iblk[i]) { cur.push_back(b); slot_of.push_back(oi); }
      if (const int32_t b = lblk[i]) { cur.push_back(b); slot_of.push_back(ol); }
    }
    std::vector<int32_t> parent(cur.size(), -1);  // index in `blocks` of the predecessor (-1: a head)
    int32_t* d_idx = nullptr;
    uint8_t* d_out = nullptr;
    size_t cap = 0;
    while (!cur.empty()) {
      if (cur.size() > cap) {
        if (d_idx) { HIP_OK(hipFree(d_idx)); HIP_OK(hipFree(d_out)); }
        cap = cur.size() * 2;
        HIP_OK(hipMalloc((void**)&d_idx, cap * 4));
        HIP_OK(hipMalloc((void**)&d_out, cap * CHAIN_BLK));
      }
      HIP_OK(hipMemcpyAsync(d_idx, cur.data(), cur.size() * 4, hipMemcpyHostToDevice, st));
      apm_dj_gather_blocks(d_pool_, d_idx, (uint32_t)cur.size(), d_out, st);
      const size_t base = blocks.size();
      blocks.resize(base + cur.size());
      HIP_OK(hipMemcpyAsync(blocks.data() + base, d_out, cur.size() * CHAIN_BLK, hipMemcpyDeviceToHost, st));
      HIP_OK(hipStreamSynchronize(st));
      std::vector<int32_t> nxt, nparent;
      for (size_t i = 0; i < cur.size(); ++i) {
        const int32_t nb = (int32_t)(base + i + 1);  // new number of this block
        if (parent[i] < 0) put32(slot_of[i], nb);
        else *(int32_t*)blocks[(size_t)parent[i]].b = nb;
        const int32_t next = *(const int32_t*)blocks[base + i].b;
        *(int32_t*)blocks[base + i].b = 0;
        if (next) { nxt.push_back(next); nparent.push_back((int32_t)(base + i)); }
      }
      cur.swap(nxt);
      parent.swap(nparent);
    }
    if (d_idx) { HIP_OK(hipFree(d_idx)); HIP_OK(hipFree(d_out)); }
  }
  span("ck.j.chains");
  w.vec(blocks);
}

void DeviceJoin::save(BinWriter& w) {
  hipStream_t st = stream_;
  save_spans.clear();
  double sp0 = clock_ms();
  auto span = [&](const char* name) { const double t = clock_ms(); save_spans.push_back({name, {sp0, t}}); sp0 = t; };
  HIP_OK(hipStreamSynchronize(st));
  HIP_OK(hipMemcpy(h_counts_, d_counts_, sizeof(JoinCounts), hipMemcpyDeviceToHost));
  w.pod(*h_counts_);
  for (uint64_t v : {events_, tx_, tx_db_, audit_errors_, host_pm_, host_invalid_acct_, host_events_}) w.pod(v);
  // key table, need arena and chain blocks: built straight into a memory writer (the async
  // checkpoint's own; a file writer gets them spliced in), so the ~100 MB of live key slots are
  // copied once (pinned bounce -> snapshot) and the chain numbers are fixed up in place
  if (w.is_memory()) {
    save_tables(w);
  } else {
    BinWriter mw{BinWriter::Memory{}};
    CkDefer* const d = ck_defer();
    ck_defer() = nullptr;  // (a temporary writer: its holes would never be filled)
    save_tables(mw);
    ck_defer() = d;
    const MemBlob b = mw.take_memory();
    w.raw(b.data(), b.size());
  }
  sp0 = clock_ms();
  // SOAP contexts of every file
  {
    std::vector<SoapState> ss(files_->size());
    if (!ss.empty()) HIP_OK(hipMemcpy(ss.data(), d_soap_, ss.size() * sizeof(SoapState), hipMemcpyDeviceToHost));
    w.vec(ss);
  }
  // raw service registry (names are re-derived from the dictionary on load)
  {
    const int32_t n = n_raw();
    std::vector<RawInfo> ri(raw_info_.begin(), raw_info_.begin() + n);
    w.vec(ri);
    std::vector<int32_t> top(n);
    for (int32_t i = 0; i < n; ++i) top[i] = h_rawtab_[i].toplevel;
    w.vec(top);
  }
  span("ck.j.soap+registry");
  // audit trail (K5): the carry generation the next batch reads
  {
    const AudGen& g = aud_gen_[aud_cur_];
    const uint32_t nf = (uint32_t)files_->size();
    std::vector<AudCarry> carry(nf);
    std::vector<AutrEnt> autr(g.n_autr);
    std::vector<AudItem> items(g.n_items);
    std::string txt(g.n_txt, '\0');
    if (nf) HIP_OK(hipMemcpy(carry.data(), g.carry, (size_t)nf * sizeof(AudCarry), hipMemcpyDeviceToHost));
    if (g.n_autr) HIP_OK(hipMemcpy(autr.data(), g.autr, (size_t)g.n_autr * sizeof(AutrEnt), hipMemcpyDeviceToHost));
    if (g.n_items) HIP_OK(hipMemcpy(items.data(), g.items, (size_t)g.n_items * sizeof(AudItem), hipMemcpyDeviceToHost));
    if (g.n_txt) HIP_OK(hipMemcpy(&txt[0], g.txt, g.n_txt, hipMemcpyDeviceToHost));
    w.vec(carry);
    w.vec(autr);
    w.vec(items);
    w.str(txt);
  }
  span("ck.j.audit");
}

void DeviceJoin::load(BinReader& rd) {
  hipStream_t st = stream_;
  JoinCounts c;
  rd.pod(c);
  HIP_OK(hipMemcpy(d_counts_, &c, sizeof(JoinCounts), hipMemcpyHostToDevice));
  *h_counts_ = c;
  for (uint64_t* v : {&events_, &tx_, &tx_db_, &audit_errors_, &host_pm_, &host_invalid_acct_, &host_events_}) rd.pod(*v);
  {
    auto live = rd.vec<KeyState>();
    uint64_t cap = table_cap_;
    while (live.size() * 2 > cap) cap *= 2;  // the saving process may have grown its table
    HIP_OK(hipStreamSynchronize(st));
    if (cap != table_cap_) {
      dfree(d_table_, (size_t)table_cap_ * sizeof(KeyState));
      if (d_table_spare_) dfree(d_table_spare_, (size_t)table_cap_ * sizeof(KeyState));
      d_table_spare_ = nullptr;
      table_cap_ = (uint32_t)cap;
      table_bits_ = 0;
      while ((1u << table_bits_) < table_cap_) ++table_bits_;
      d_table_ = (KeyState*)dmalloc((size_t)table_cap_ * sizeof(KeyState));
      ensure_tmp();
    } else {
      HIP_OK(hipMemsetAsync(d_table_, 0, (size_t)table_cap_ * sizeof(KeyState), st));
    }
    if (!live.empty()) {
      KeyState* tmp = nullptr;
      HIP_OK(hipMalloc((void**)&tmp, live.size() * sizeof(KeyState)));
      HIP_OK(hipMemcpy(tmp, live.data(), live.size() * sizeof(KeyState), hipMemcpyHostToDevice));
      HIP_OK(hipMemsetAsync(d_live_, 0, 8, st));
      // every saved slot is reinserted (now = -inf keeps them all, chains included)
      apm_dj_rebuild(tmp, (uint32_t)live.size(), d_table_, table_cap_ - 1, d_arena_, cfg_.arena_cap, -__builtin_inf(),
                     d_counts_, d_live_, d_pool_, d_pool_ring_, pool_n_ - 1, st);
      HIP_OK(hipStreamSynchronize(st));
      HIP_OK(hipFree(tmp));
    }
    keys_live_ = live.size();
    keys_since_rebuild_ = 0;
    live_pending_ = false;
    sync_keys();
  }
  {
    const uint32_t saved_cap = rd.pod<uint32_t>();
    if (saved_cap != cfg_.arena_cap) {  // the `need` links are slots of the saver's arena size
      HIP_OK(hipStreamSynchronize(st));
      dfree(d_arena_, (size_t)cfg_.arena_cap * sizeof(NeedEnt));
      cfg_.arena_cap = saved_cap;
      d_arena_ = (NeedEnt*)dmalloc((size_t)cfg_.arena_cap * sizeof(NeedEnt));
      for (void* p : {(void*)d_exp_key_, (void*)d_exp_key_sorted_}) dfree(p, ((size_t)exp_cap_ + 1) * 8);
      for (void* p : {(void*)d_exp_idx_, (void*)d_exp_idx_sorted_, (void*)d_exp_cnt_, (void*)d_exp_pos_})
        dfree(p, ((size_t)exp_cap_ + 1) * 4);
      exp_cap_ = saved_cap;
      d_exp_key_ = (uint64_t*)dmalloc(((size_t)exp_cap_ + 1) * 8);
      d_exp_key_sorted_ = (uint64_t*)dmalloc(((size_t)exp_cap_ + 1) * 8);
      d_exp_idx_ = (uint32_t*)dmalloc(((size_t)exp_cap_ + 1) * 4);
      d_exp_idx_sorted_ = (uint32_t*)dmalloc(((size_t)exp_cap_ + 1) * 4);
      d_exp_cnt_ = (uint32_t*)dmalloc(((size_t)exp_cap_ + 1) * 4);
      d_exp_pos_ = (uint32_t*)dmalloc(((size_t)exp_cap_ + 1) * 4);
      ensure_tmp();
    }
  }
  rd.pod(arena_head_);
  regions_.clear();
  for (uint64_t n = rd.pod<uint64_t>(); n; --n) {
    Region r;
    rd.pod(r.lo); rd.pod(r.hi); rd.pod(r.exp);
    regions_.push_back(r);
  }
  {
    auto ents = rd.vec<NeedEnt>();
    const uint64_t lo = regions_.empty() ? arena_head_ : regions_.front().lo;
    if (ents.size() != arena_head_ - lo) throw std::runtime_error("checkpoint: need arena size mismatch");
    // the live range [lo, head) of the ring: at most two bulk copies, split at the wrap point
    // (mirrors save_tables; restore time no longer scales with one copy per entry)
    const uint64_t cap = cfg_.arena_cap;
    if (ents.size() > cap) throw std::runtime_error("checkpoint: need arena larger than the ring");
    // dmalloc zeroes on the join stream; the blocking copies below run on the null stream, which
    // does not order against it -- without this wait a regrown buffer's memset could land after
    // the restored contents (seen: restored logId chain blocks read back as zeros)
    HIP_OK(hipStreamSynchronize(st));
    if (!ents.empty()) {
      const uint64_t first = lo & (cap - 1);
      const uint64_t n1 = std::min<uint64_t>(ents.size(), cap - first);
      HIP_OK(hipMemcpy(d_arena_ + first, ents.data(), n1 * sizeof(NeedEnt), hipMemcpyHostToDevice));
      if (ents.size() > n1)
        HIP_OK(hipMemcpy(d_arena_, ents.data() + n1, (ents.size() - n1) * sizeof(NeedEnt), hipMemcpyHostToDevice));
    }
  }
  {
    // chain blocks: saved 1..n, loaded into blocks 0..n-1 of a fresh pool whose first n ring
    // entries (identity) are taken
    struct Blk { uint8_t b[CHAIN_BLK]; };
    auto blocks = rd.vec<Blk>();
    HIP_OK(hipStreamSynchronize(st));
    uint64_t n = pool_n_;
    while (n < 2 * blocks.size() + (1u << 16)) n *= 2;
    if (n != pool_n_) {
      dfree(d_pool_, (size_t)pool_n_ * CHAIN_BLK);
      dfree(d_pool_ring_, (size_t)pool_n_ * 4);
      pool_n_ = (uint32_t)n;
      d_pool_ = (uint8_t*)dmalloc((size_t)pool_n_ * CHAIN_BLK);
      d_pool_ring_ = (uint32_t*)dmalloc((size_t)pool_n_ * 4);
      HIP_OK(hipStreamSynchronize(st));  // (the zeroing before the null-stream copy, as above)
    }
    if (!blocks.empty())
      HIP_OK(hipMemcpy(d_pool_, blocks.data(), blocks.size() * CHAIN_BLK, hipMemcpyHostToDevice));
    apm_dj_pool_init(d_pool_ring_, pool_n_, d_counts_, st);
    const unsigned long long taken = blocks.size();
    HIP_OK(hipMemcpyAsync((uint8_t*)d_counts_ + offsetof(JoinCounts, pool_head), &taken, 8, hipMemcpyHostToDevice, st));
    HIP_OK(hipStreamSynchronize(st));
    pool_avail(true);
  }
  {
    auto ss = rd.vec<SoapState>();
    if (ss.size() > soap_cap_) throw std::runtime_error("checkpoint: too many files");
    if (!ss.empty()) HIP_OK(hipMemcpy(d_soap_, ss.data(), ss.size() * sizeof(SoapState), hipMemcpyHostToDevice));
  }
  {
    auto ri = rd.vec<RawInfo>();
    auto top = rd.vec<int32_t>();
    if (ri.size() > cfg_.max_raw) throw std::runtime_error("checkpoint: more raw services than gpu.maxRawServices");
    const uint32_t rmask = (1u << cfg_.reg_bits) - 1;
    std::vector<RegSlot> reg((size_t)rmask + 1);
    for (auto& r : reg) { r.key = 0; r.raw = RAW_EMPTY; r.pad = 0; }
    raw_info_.clear();
    for (size_t i = 0; i < ri.size(); ++i) {
      raw_info_.push_back(ri[i]);
      RawSvc& r = h_rawtab_[i];
      const std::string& srv = (*servers_)[ri[i].server];
      const std::string norm = dict_->service_name(ri[i].norm_id);
      r.srv_off = intern_name(srv);
      r.srv_len = (int32_t)srv.size();
      r.norm_off = intern_name(norm);
      r.norm_len = (int32_t)norm.size();
      r.toplevel = top[i];
      r.pad = 0;
      const uint64_t k = dj::regkey_of(ri[i].svc, ri[i].server);
      for (uint32_t h = dj::home_of(k, rmask);; h = (h + 1) & rmask)
        if (!reg[h].key) { reg[h].key = k; reg[h].raw = (int32_t)i; break; }
    }
    HIP_OK(hipMemcpy(d_reg_, reg.data(), reg.size() * sizeof(RegSlot), hipMemcpyHostToDevice));
    if (!ri.empty()) HIP_OK(hipMemcpy(d_rawtab_, h_rawtab_, ri.size() * sizeof(RawSvc), hipMemcpyHostToDevice));
    if (names_.size() > names_cap_) {
      names_cap_ = std::max<size_t>(names_.size() * 2, 1 << 20);
      HIP_OK(hipMalloc((void**)&d_names_, names_cap_));
      device_bytes_ += names_cap_;
    }
    if (!names_.empty()) HIP_OK(hipMemcpy(d_names_, names_.data(), names_.size(), hipMemcpyHostToDevice));
    names_uploaded_ = names_.size();
    n_raw_.store((int32_t)ri.size(), std::memory_order_release);
  }
  {
    auto carry = rd.vec<AudCarry>();
    auto autr = rd.vec<AutrEnt>();
    auto items = rd.vec<AudItem>();
    const std::string txt = rd.str();
    if (carry.size() > soap_cap_) throw std::runtime_error("checkpoint: too many files");
    HIP_OK(hipStreamSynchronize(st));
    aud_cur_ = 0;
    AudGen& g = aud_gen_[0];
    aud_reserve(g, (uint32_t)autr.size(), (uint32_t)items.size(), txt.size());
    HIP_OK(hipStreamSynchronize(st));  // (its zeroing before the null-stream copies, as above)
    HIP_OK(hipMemset(g.carry, 0, (size_t)soap_cap_ * sizeof(AudCarry)));
    HIP_OK(hipMemset(aud_gen_[1].carry, 0, (size_t)soap_cap_ * sizeof(AudCarry)));
    if (!carry.empty()) HIP_OK(hipMemcpy(g.carry, carry.data(), carry.size() * sizeof(AudCarry), hipMemcpyHostToDevice));
    if (!autr.empty()) HIP_OK(hipMemcpy(g.autr, autr.data(), autr.size() * sizeof(AutrEnt), hipMemcpyHostToDevice));
    if (!items.empty()) HIP_OK(hipMemcpy(g.items, items.data(), items.size() * sizeof(AudItem), hipMemcpyHostToDevice));
    if (!txt.empty()) HIP_OK(hipMemcpy(g.txt, txt.data(), txt.size(), hipMemcpyHostToDevice));
    g.n_autr = (uint32_t)autr.size();
    g.n_items = (uint32_t)items.size();
    g.n_txt = (uint32_t)txt.size();
  }
  files_uploaded_ = 0;
  HIP_OK(hipStreamSynchronize(st));
}

void DeviceJoin::reset_ring(uint64_t head) {
  std::lock_guard<std::mutex> g(ring_mu_);
  ring_head_.store(head, std::memory_order_release);
  ring_low_.store(0, std::memory_order_release);
}

}  // namespace apm
