#include <cstdlib>
// apm::Engine implementation -- see engine.h.
#include "engine.h"

#include <pthread.h>
#include <sched.h>

#include <cctype>
#include <fstream>

#include <rocprofiler-sdk-roctx/roctx.h>

#include <unistd.h>

#include <cerrno>
#include <cstring>

#include <algorithm>
#include <exception>
#include <chrono>
#include <cmath>
#include <cstring>
#include <queue>
#include <stdexcept>

#include "../kernels/devjoin_api.h"
#include "../kernels/kernel_api.h"
#include "format.h"

namespace apm {
namespace copyenc {
void encode_blob(std::string_view blob, std::string* out, int64_t* counts);  // copyenc.cpp
}
}  // namespace apm

namespace apm {

namespace {
double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

// ----------------------------------------------------------------------------- CPU placement
// Host lanes (join workers, stats thread, output lane) can be pinned to physical cores local to
// the GPU's PCIe root: the pinned batch buffers and the device's DMA live on that NUMA node, and
// a pinned join worker keeps its shard's maps in one core's L2 / one CCD's L3.  Ranks whose GPUs
// share a NUMA node take disjoint slices of its cores (slice = rank among those GPUs).
void pin_current_thread(int cpu) {
  cpu_set_t set;
  CPU_ZERO(&set);
  CPU_SET(cpu, &set);
  pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
}

namespace {
std::vector<int> parse_cpulist(const std::string& s) {
  std::vector<int> out;
  size_t i = 0;
  while (i < s.size()) {
    size_t j = s.find(',', i);
    if (j == std::string::npos) j = s.size();
    const std::string tok = s.substr(i, j - i);
    const size_t dash = tok.find('-');
    try {
      if (dash == std::string::npos) {
        if (!tok.empty() && tok != "\n") out.push_back(std::stoi(tok));
      } else {
        const int a = std::stoi(tok.substr(0, dash)), b = std::stoi(tok.substr(dash + 1));
        for (int c = a; c <= b; ++c) out.push_back(c);
      }
    } catch (...) {
    }
    i = j + 1;
  }
  return out;
}

std::string read_small(const std::string& path) {
  std::ifstream f(path);
  std::string s;
  std::getline(f, s);
  return s;
}

std::string pci_dir(int device) {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) != hipSuccess) return "";
  std::string b(bus);
  for (char& c : b) c = (char)std::tolower((unsigned char)c);
  return "/sys/bus/pci/devices/" + b;
}
}  // namespace

std::vector<int> local_core_slice(int device) {
  const std::string dir = pci_dir(device);
  if (dir.empty()) return {};
  const std::string mine = read_small(dir + "/local_cpulist");
  std::vector<int> local = parse_cpulist(mine);
  cpu_set_t allowed;
  CPU_ZERO(&allowed);
  if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return {};
  std::vector<int> cores;  // one CPU per physical core (the first SMT sibling), allowed for us
  for (int c : local) {
    if (!CPU_ISSET(c, &allowed)) continue;
    const std::vector<int> sib =
        parse_cpulist(read_small("/sys/devices/system/cpu/cpu" + std::to_string(c) + "/topology/thread_siblings_list"));
    if (sib.empty() || sib[0] == c) cores.push_back(c);
  }
  int n_dev = 0;
  if (hipGetDeviceCount(&n_dev) != hipSuccess) n_dev = device + 1;
  int slot = 0, peers = 0;
  for (int d = 0; d < n_dev; ++d) {
    if (read_small(pci_dir(d) + "/local_cpulist") != mine) continue;
    if (d < device) ++slot;
    ++peers;
  }
  peers = std::max(peers, 1);
  const size_t per = cores.size() / (size_t)peers;
  if (per == 0) return {};
  // L3 domains (one CCD each on EPYC: 8 cores, 32 MB).  Ranks sharing the NUMA node take whole
  // CCDs where possible, and inside a slice consecutive lanes go round-robin over its CCDs, so
  // the first join workers each get a private L3 for their shard's maps instead of eight
  // workers sharing one CCD's L3 and its fabric link (CPU numbering interleaves CCDs).
  auto l3_of = [](int c) {
    const std::string id = read_small("/sys/devices/system/cpu/cpu" + std::to_string(c) + "/cache/index3/id");
    try { return id.empty() ? 0 : std::stoi(id); } catch (...) { return 0; }
  };
  std::vector<std::pair<int, int>> keyed;  // (l3 id, cpu)
  for (int c : cores) keyed.push_back({l3_of(c), c});
  std::stable_sort(keyed.begin(), keyed.end());
  std::vector<std::pair<int, int>> mine_sl(keyed.begin() + (ptrdiff_t)(slot * per),
                                           keyed.begin() + (ptrdiff_t)((slot + 1) * per));
  std::vector<std::vector<int>> groups;
  for (size_t i = 0; i < mine_sl.size(); ++i) {
    if (i == 0 || mine_sl[i].first != mine_sl[i - 1].first) groups.emplace_back();
    groups.back().push_back(mine_sl[i].second);
  }
  std::vector<int> out;
  for (size_t r = 0; out.size() < mine_sl.size(); ++r)
    for (auto& g : groups)
      if (r < g.size()) out.push_back(g[r]);
  return out;
}

// ----------------------------------------------------------------------------- thread pool
// Static task placement: task t always runs on worker t % W.  A join shard's working set (its
// TTL maps, several MB) then stays in one core's L2 / one CCD's L3 from batch to batch; with
// first-come task grabbing every batch moved each shard to a cold core (measured: the same
// join ran 2.2x slower per shard inside the engine than alone).
ThreadPool::ThreadPool(int n, const std::vector<int>& cpus) {
  for (int i = 0; i < n; ++i) {
    const int cpu = cpus.empty() ? -1 : cpus[(size_t)i % cpus.size()];
    workers_.emplace_back([this, i, n, cpu]() {
      if (cpu >= 0) pin_current_thread(cpu);
      uint64_t seen = 0;
      for (;;) {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&]() { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        const int n_tasks = n_tasks_;
        const std::function<void(int)>* fn = fn_;
        lk.unlock();
        int mine = 0;
        for (int t = i; t < n_tasks; t += n) { (*fn)(t); ++mine; }
        if (mine) {
          lk.lock();
          done_ += mine;
          if (done_ == n_tasks_) done_cv_.notify_all();
        }
      }
    });
  }
}

ThreadPool::~ThreadPool() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : workers_) t.join();
}

void ThreadPool::run(int n_tasks, const std::function<void(int)>& fn, const std::function<void()>* meanwhile) {
  if (n_tasks <= 0 || workers_.empty() || n_tasks == 1) {
    for (int i = 0; i < n_tasks; ++i) fn(i);
    if (meanwhile) (*meanwhile)();
    return;
  }
  std::unique_lock<std::mutex> lk(mu_);
  fn_ = &fn;
  n_tasks_ = n_tasks;
  done_ = 0;
  ++gen_;
  cv_.notify_all();
  std::exception_ptr err;
  if (meanwhile) {
    lk.unlock();
    try { (*meanwhile)(); } catch (...) { err = std::current_exception(); }
    lk.lock();
  }
  done_cv_.wait(lk, [&]() { return done_ == n_tasks_; });
  fn_ = nullptr;
  lk.unlock();
  if (err) std::rethrow_exception(err);
}

// ----------------------------------------------------------------------------- setup
void* Engine::dmalloc(size_t bytes) {
  void* p = nullptr;
  bytes = (bytes + 255) & ~(size_t)255;
  HIP_OK(hipMalloc(&p, bytes));
  HIP_OK(hipMemset(p, 0, bytes));
  // hipMemset runs on the null stream, which does not order against the engine's non-blocking
  // streams: without this wait, a buffer regrown mid-run could be zeroed *after* the first copy
  // into it on stream_ (seen: K12 names table read back as zeros after a regrow).  The null
  // stream only, not the device: a device-wide sync would also wait for the collective stream
  // (a lock-step all-reduce waiting for a peer rank).
  HIP_OK(hipStreamSynchronize(nullptr));
  std::lock_guard<std::mutex> g(alloc_mu_);  // the stats thread and the rollover lane allocate
  allocations_.push_back(p);
  alloc_bytes_[p] = bytes;
  device_bytes_ += bytes;
  return p;
}

// Optional scratch (checkpoint packing): nullptr instead of a throw when HBM is short, no zeroing
// and no device-wide sync; counted in device_bytes_ and freed by dfree / the destructor.
void* Engine::dmalloc_try(size_t bytes) {
  void* p = nullptr;
  bytes = (bytes + 255) & ~(size_t)255;
  if (hipMalloc(&p, bytes) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  std::lock_guard<std::mutex> g(alloc_mu_);
  allocations_.push_back(p);
  alloc_bytes_[p] = bytes;
  device_bytes_ += bytes;
  return p;
}

Engine::Engine(const EngineConfig& cfg) : cfg_(cfg) {
  check_window(cfg_.window, cfg_.buffer, cfg_.interval_len);
  if (cfg_.n_lags < 1 || cfg_.n_lags > MAX_LAGS)
    throw std::runtime_error("engine: 1.." + std::to_string(MAX_LAGS) + " LAG settings");
  HIP_OK(hipSetDevice(cfg_.device));
  {
    // Ranks sharing one GPU (a rehearsal of the node on one card): host threads that spin in
    // every stream / event wait multiply by the rank count and starve each other of the box's
    // CPU share -- there the waits block instead (APM_BLOCKING_SYNC=1; bench.py sets it when
    // local ranks outnumber the GPUs).  Best effort: the flag cannot change on a device whose
    // runtime state exists already.
    const char* e = std::getenv("APM_BLOCKING_SYNC");
    if (e && e[0] == '1') (void)hipSetDeviceFlags(hipDeviceScheduleBlockingSync);
  }
  {
    // The device join's kernels are the ingest thread's critical chain, and most of them are
    // small, latency-bound grids: sharing every SIMD with the parse / stats / output kernels of
    // the other streams stretched them 5-10x in the bench timeline (k_aud_walk 47 us alone,
    // ~190 us co-running).  APM_CU_RESERVE=N keeps N CUs (every (CUs/N)-th, so spread over the
    // XCDs) out of those streams' CU masks; the join stream keeps all CUs.
    const char* e = std::getenv("APM_CU_RESERVE");
    int n_cu = 0;
    HIP_OK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, cfg_.device));
    const int reserve = e ? std::atoi(e) : 0;
    if (reserve > 0 && reserve < n_cu / 2) {
      const int stride = n_cu / reserve;
      std::vector<uint32_t> mask((size_t)(n_cu + 31) / 32, 0u);
      for (int c = 0; c < n_cu; ++c)
        if (c % stride != stride - 1) mask[(size_t)c / 32] |= 1u << (c % 32);
      for (hipStream_t* s : {&stream_, &parse_stream_, &out_stream_})
        HIP_OK(hipExtStreamCreateWithCUMask(s, (uint32_t)mask.size(), mask.data()));
      cu_reserved_ = reserve;
    } else {
      // The stats stream (rollover chain K8..K11 -> alert candidates) at the join stream's high
      // priority, so a batch's alert decision is not queued behind the next batch's join kernels:
      // 271.2 / 265.4 / 280.3 / 268.0 M against 264.9-267.3 M default-priority runs on the same
      // boxes, p50 ingest -> alert 1.13-1.17 vs 1.17-1.24 ms (profiles/r6_g, r6_q).
      // APM_STATS_PRIO=0: default priority (A/B).
      static const bool sp = [] { const char* x = std::getenv("APM_STATS_PRIO"); return !(x && x[0] == '0'); }();
      int lo = 0, hi = 0;
      HIP_OK(hipDeviceGetStreamPriorityRange(&lo, &hi));
      HIP_OK(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, sp ? hi : 0));
      // APM_PARSE_PRIO=1: the parse stream (the next batch's K1/K2, which the ingest thread waits
      // for at the start of every batch) at high priority too -- A/B
      static const bool pp = [] { const char* x = std::getenv("APM_PARSE_PRIO"); return x && x[0] == '1'; }();
      HIP_OK(hipStreamCreateWithPriority(&parse_stream_, hipStreamNonBlocking, pp ? hi : 0));
      HIP_OK(hipStreamCreateWithFlags(&out_stream_, hipStreamNonBlocking));
    }
  }
  HIP_OK(hipEventCreateWithFlags(&ev_a_, hipEventDisableTiming));
  HIP_OK(hipEventCreateWithFlags(&ev_b_, hipEventDisableTiming));
  const int32_t S = cfg_.max_series;
  // parse
  if (cfg_.device_join) {
    DevJoinConfig dc;
    dc.max_events = cfg_.max_lines;
    dc.max_batch_bytes = cfg_.max_batch_bytes;
    dc.max_chunks = cfg_.max_chunks;
    dc.table_bits = cfg_.join_table_bits;
    dc.max_raw = cfg_.max_raw_services;
    dc.arena_cap = cfg_.need_arena;
    dc.pool_blocks = cfg_.join_chain_blocks;
    dc.ring_bytes = cfg_.tx_ring_bytes;
    dc.record_ttl_ms = cfg_.record_ttl_ms;
    dc.acct_ttl_ms = cfg_.acct_ttl_ms;
    dc.need_ttl_ms = cfg_.need_ttl_ms;
    dc.tz = cfg_.tz;
    dc.device = cfg_.device;
    dj_.reset(new DeviceJoin(dc, &dict_, &files_, &servers_));  // (its bytes: device_bytes())
    d_ring_min_ = (unsigned long long*)dmalloc(64);
    HIP_OK(hipMemset(d_ring_min_, 0xff, 8));  // (the export after each min pass restores it)
    HIP_OK(hipHostMalloc((void**)&h_ring_min_, 64, hipHostMallocDefault));
    HIP_OK(hipHostGetDevicePointer((void**)&hd_ring_min_, h_ring_min_, 0));
    *h_ring_min_ = ~0ULL;
    d_rel_n_ = (int64_t*)dmalloc(64);
    HIP_OK(hipHostMalloc((void**)&h_rel_n_, 64, hipHostMallocDefault));
    HIP_OK(hipHostGetDevicePointer((void**)&hd_rel_n_, h_rel_n_, 0));
    d_rel_lens_ = (uint32_t*)dmalloc(((size_t)cfg_.pool_cap + 2) * 4);
    d_rel_offs_ = (uint32_t*)dmalloc(((size_t)cfg_.pool_cap + 2) * 4);
    d_rel_fb_ = (uint32_t*)dmalloc(4);
    HIP_OK(hipMemset(d_rel_fb_, 0, 4));
    HIP_OK(hipHostMalloc((void**)&h_rel_total_, 64, hipHostMallocDefault));
    HIP_OK(hipHostGetDevicePointer((void**)&hd_rel_total_, h_rel_total_, 0));
    d_unmapped_ = (unsigned long long*)dmalloc(64);
    d_unseen_idx_ = (int32_t*)dmalloc((size_t)cfg_.max_series * 4);
    d_unseen_flag_ = (uint8_t*)dmalloc((size_t)cfg_.max_series);
    HIP_OK(hipHostMalloc((void**)&h_unseen_flag_, (size_t)cfg_.max_series, hipHostMallocDefault));
  } else {
    d_bytes_ = (uint8_t*)dmalloc(cfg_.max_batch_bytes + 256);
  }
  for (int k = 0; k < 2; ++k) {
    ParseSlot& ps = pslot_[k];
    HIP_OK(hipHostMalloc((void**)&ps.h_bytes, cfg_.max_batch_bytes + 256, hipHostMallocDefault));
    HIP_OK(hipHostMalloc((void**)&ps.h_chunk_begin, (cfg_.max_chunks + 2) * 4, hipHostMallocDefault));
    HIP_OK(hipHostMalloc((void**)&ps.h_chunk_kind, cfg_.max_chunks + 2, hipHostMallocDefault));
    HIP_OK(hipHostMalloc((void**)&ps.h_chunk_file, (cfg_.max_chunks + 2) * 4, hipHostMallocDefault));
    d_chunk_begin_[k] = (uint32_t*)dmalloc((cfg_.max_chunks + 2) * 4);
    d_chunk_kind_[k] = (uint8_t*)dmalloc(cfg_.max_chunks + 2);
    d_chunk_file_[k] = (uint32_t*)dmalloc((cfg_.max_chunks + 2) * 4);
    HIP_OK(hipHostMalloc((void**)&ps.h_counts, 16, hipHostMallocDefault));
    HIP_OK(hipHostMalloc((void**)&ps.h_watermark, 8, hipHostMallocDefault));
    if (dev()) continue;  // the device join keeps events on the GPU
    HIP_OK(hipHostMalloc((void**)&ps.h_events, (size_t)cfg_.max_lines * sizeof(Event), hipHostMallocDefault));
    // APM_EVENTS_ZEROCOPY=1: the compaction kernel writes the events straight into this pinned
    // slot (the copy rides along with the prefetched parse) instead of a 15 MB D2H the ingest
    // thread waits for.  Measured A/B on MI355X (tools/ab_env.sh, 4 alternating rounds): -0.3 ms
    // parse but +0.3 ms host join (the join then reads lines the GPU wrote over PCIe), i.e. no
    // net change, so the DMA copy stays the default.
    const char* zc = std::getenv("APM_EVENTS_ZEROCOPY");
    void* dp = nullptr;
    if (zc && std::atoi(zc) != 0 && hipHostGetDevicePointer(&dp, ps.h_events, 0) == hipSuccess)
      ps.d_events_host = (Event*)dp;
  }
  d_parse_ws_ = dmalloc(apm_parse_workspace_bytes(cfg_.max_batch_bytes, cfg_.max_lines, cfg_.max_chunks));
  if (!dev()) d_events_ = (Event*)dmalloc((size_t)cfg_.max_lines * sizeof(Event));
  d_counts_ = (uint32_t*)dmalloc(16);
  d_watermark_ = (unsigned long long*)dmalloc(8);
  d_file_open_ = (uint8_t*)dmalloc(1 << 16);
  // stats
  init_spill_cap_ = cfg_.spill_cap;
  alloc_ring(std::max(cfg_.nslot, ring_slots_for(cfg_.window, cfg_.buffer)));
  for (auto& m : spill_mark_) HIP_OK(hipEventCreateWithFlags(&m.ev, hipEventDisableTiming));
  metrics_.spill_capacity = cfg_.spill_cap;
  d_spill_drop_ = (unsigned long long*)dmalloc(64);
  d_active_ = (uint8_t*)dmalloc(S);
  d_win_ = (WinStat*)dmalloc((size_t)S * sizeof(WinStat));
  d_big_list_ = (int32_t*)dmalloc((size_t)S * 4);
  // per-rollover counters in one block, cleared by one memset: [0] big, [1] nan, [2] alert candidates
  d_big_n_ = (int32_t*)dmalloc(64);
  d_nan_until_ = (int32_t*)dmalloc((size_t)S * 4);
  HIP_OK(hipMemset(d_nan_until_, 0x80, (size_t)S * 4));  // 0x80808080: far below any bucket
  ord_cap_ = std::max<int64_t>(cfg_.max_tx_per_batch, cfg_.max_lines);
  d_ord_list_ = (int32_t*)dmalloc((size_t)ord_cap_ * 4);
  d_ord_n_ = (int32_t*)dmalloc(8);  // [0] ord_n, [1] ordered-append blocks done
  d_nan_list_ = (int32_t*)dmalloc((size_t)S * 4);
  d_nan_n_ = d_big_n_ + 1;
  d_js_scratch_ = (int32_t*)dmalloc((size_t)JS_BLOCKS * kJsCap * 4);
  // z-score
  for (int l = 0; l < cfg_.n_lags; ++l) {
    LagState& L = lag_[l];
    L.ring = dmalloc((size_t)NSTAT * cfg_.lags[l] * S * cfg_.ring_bytes);
    L.len = (int32_t*)dmalloc((size_t)S * 4);
    L.sum = (double*)dmalloc((size_t)NSTAT * S * 8);
    L.comp = (double*)dmalloc((size_t)NSTAT * S * 8);
    L.sumsq = (double*)dmalloc((size_t)NSTAT * S * 8);
    L.sqcomp = (double*)dmalloc((size_t)NSTAT * S * 8);
    L.cnt = (int32_t*)dmalloc((size_t)NSTAT * S * 4);
    L.thr = (double*)dmalloc((size_t)S * 8);
    L.infl = (double*)dmalloc((size_t)S * 8);
    L.out = (ZOut*)dmalloc((size_t)S * sizeof(ZOut));
    L.counter = (int32_t*)dmalloc((size_t)S * 4);
  }
  // rolling-mode resync scratch: one contiguous range of ceil(S / K) series per rollover
  if (cfg_.resync_k > 0 && !cfg_.exact_mean) {
    rs_range_ = (S + cfg_.resync_k - 1) / cfg_.resync_k;
    rs_part_ = (double*)dmalloc((size_t)NSTAT * RS_PARTS * rs_range_ * 4 * 8);
    rs_cnt_ = (int32_t*)dmalloc((size_t)NSTAT * RS_PARTS * rs_range_ * 4);
  }
  {
    const double* sp[MAX_LAGS] = {};
    const double* cp[MAX_LAGS] = {};
    const int32_t* np[MAX_LAGS] = {};
    for (int l = 0; l < cfg_.n_lags; ++l) { sp[l] = lag_[l].sum; cp[l] = lag_[l].comp; np[l] = lag_[l].cnt; }
    d_lag_sum_ptrs_ = dmalloc(sizeof(sp));
    d_lag_comp_ptrs_ = dmalloc(sizeof(cp));
    d_lag_cnt_ptrs_ = dmalloc(sizeof(np));
    HIP_OK(hipMemcpy(d_lag_sum_ptrs_, sp, sizeof(sp), hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_lag_comp_ptrs_, cp, sizeof(cp), hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_lag_cnt_ptrs_, np, sizeof(np), hipMemcpyHostToDevice));
    d_series_service_ = (int32_t*)dmalloc((size_t)S * 4);
  }
  d_hard_max_ = (double*)dmalloc((size_t)S * 8);
  d_suppressed_ = (uint8_t*)dmalloc(S);
  d_cool_t_ = (double*)dmalloc((size_t)S * 8);
  HIP_OK(hipMemsetAsync(d_cool_t_, 0xff, (size_t)S * 8, stream_));  // NaN: no cooldown
  d_emit_key_ = (uint64_t*)dmalloc((size_t)S * 8);
  // K12 formatter
  d_ser_names_ = (int32_t*)dmalloc((size_t)S * 16);
  d_perm_ = (int32_t*)dmalloc((size_t)S * 4);
  d_series_server_ = (int32_t*)dmalloc((size_t)S * 4);
  // st lengths/offsets [S + 1], then fs per (series, LAG) line [S * MAX_LAGS + 1]
  d_fmt_len_ = (uint32_t*)dmalloc(((size_t)(S + 1) + (size_t)S * MAX_LAGS + 1) * 4);
  d_fmt_off_ = (uint32_t*)dmalloc(((size_t)(S + 1) + (size_t)S * MAX_LAGS + 1) * 4);
  d_fmt_fallback_ = (int32_t*)dmalloc(4);
  fmt_tmp_bytes_ = apm_format_tmp_bytes((int32_t)((size_t)S * MAX_LAGS + 1));
  d_fmt_tmp_ = dmalloc(fmt_tmp_bytes_);
  HIP_OK(hipHostMalloc((void**)&h_fmt_meta_, 64, hipHostMallocDefault));
  HIP_OK(hipHostGetDevicePointer((void**)&hd_fmt_meta_, h_fmt_meta_, 0));
  {
    const char* e = std::getenv("APM_FMT_HOST");
    fmt_host_ = e && e[0] == '1';
    const char* f = std::getenv("APM_TXCOPY_FORCE_FALLBACK");
    txcopy_force_fb_ = f && f[0] == '1';
    const char* d = std::getenv("APM_D2H_KERNEL");
    d2h_kernel_ = d && d[0] == '1';
    const char* rl = std::getenv("APM_REL_LANE");
    rel_lane_on_ = !(rl && rl[0] == '0');
    const char* sp = std::getenv("APM_D2H_SPLIT");
    d2h_split_ = sp ? std::max(1, std::atoi(sp)) : 1;
    const char* sd = std::getenv("APM_D2H_SDMA");
    d2h_sdma_ = sd && sd[0] == '1';
    const char* b = std::getenv("APM_D2H_BLOCKS");
    d2h_blocks_ = b ? (uint32_t)std::max(1, std::atoi(b)) : 32u;
  }
  // alerts
  d_alerts_ = (AlertRec*)dmalloc((size_t)cfg_.max_alerts * sizeof(AlertRec));
  d_n_alerts_ = d_big_n_ + 2;
  HIP_OK(hipHostMalloc((void**)&h_alerts_, (size_t)cfg_.max_alerts * sizeof(AlertRec), hipHostMallocDefault));
  HIP_OK(hipHostMalloc((void**)&h_alert_win_, (size_t)cfg_.max_alerts * sizeof(WinStat), hipHostMallocDefault));
  HIP_OK(hipHostMalloc((void**)&h_alert_z_, (size_t)cfg_.max_alerts * sizeof(ZOut), hipHostMallocDefault));
  HIP_OK(hipHostMalloc((void**)&h_n_alerts_, 16, hipHostMallocDefault));
  HIP_OK(hipHostGetDevicePointer((void**)&hd_alerts_, h_alerts_, 0));
  HIP_OK(hipHostGetDevicePointer((void**)&hd_alert_win_, h_alert_win_, 0));
  HIP_OK(hipHostGetDevicePointer((void**)&hd_alert_z_, h_alert_z_, 0));
  HIP_OK(hipHostGetDevicePointer((void**)&hd_n_alerts_, h_n_alerts_, 0));
  HIP_OK(hipEventCreateWithFlags(&ev_alerts_, hipEventDisableTiming));
  HIP_OK(hipEventCreateWithFlags(&ev_release_, hipEventDisableTiming));
  // tx + release
  d_tx_ = (TxRec*)dmalloc((size_t)cfg_.max_tx_per_batch * sizeof(TxRec));
  HIP_OK(hipHostMalloc((void**)&h_tx_, (size_t)cfg_.max_tx_per_batch * sizeof(TxRec), hipHostMallocDefault));
  d_gid_ = (int64_t*)dmalloc((size_t)cfg_.max_tx_per_batch * 8);
  HIP_OK(hipHostMalloc((void**)&h_gid_, (size_t)cfg_.max_tx_per_batch * 8, hipHostMallocDefault));
  d_tail_end_ = (int64_t*)dmalloc((size_t)cfg_.pool_cap * 8);
  d_tail_gid_ = (int64_t*)dmalloc((size_t)cfg_.pool_cap * 8);
  d_sort_end_ = (int64_t*)dmalloc((size_t)cfg_.pool_cap * 8);
  d_sort_gid_ = (int64_t*)dmalloc((size_t)cfg_.pool_cap * 8);
  for (int i = 0; i < 2; ++i) {
    d_pool_end_[i] = (int64_t*)dmalloc((size_t)cfg_.pool_cap * 8);
    d_pool_gid_[i] = (int64_t*)dmalloc((size_t)cfg_.pool_cap * 8);
  }
  release_tmp_bytes_ = apm_release_tmp_bytes(cfg_.pool_cap);
  if (dev()) release_tmp_bytes_ = std::max(release_tmp_bytes_, apm_dj_tmp_bytes((uint32_t)cfg_.pool_cap + 2, 1024, 8));
  d_release_tmp_ = dmalloc(release_tmp_bytes_);
  for (int k = 0; k < 2; ++k) {
    HIP_OK(hipHostMalloc((void**)&h_release_gid_[k], (size_t)cfg_.pool_cap * 8, hipHostMallocDefault));
    HIP_OK(hipEventCreateWithFlags(&ev_rel_[k], hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&ev_fmt_[k], hipEventDisableTiming));
  }
  // threads
  const char* pin_env = std::getenv("APM_PIN_THREADS");
  if (pin_env ? std::atoi(pin_env) != 0 : cfg_.pin_threads) lane_cpus_ = local_core_slice(cfg_.device);
  int nt = cfg_.join_threads;
  // host join: one worker per JVM shard (up to 16); device join: the pool only runs the audit
  // pre-pass (one task per app log), so 8 threads -- 8 ranks per node stay at ~100 threads
  if (nt <= 0) nt = (int)std::min<unsigned>(cfg_.device_join ? 8 : 16, std::max(1u, std::thread::hardware_concurrency()));
  {
    // join workers take the first cores of the slice; the stats thread and output lane the next two
    std::vector<int> wc(lane_cpus_.begin(), lane_cpus_.begin() + (ptrdiff_t)std::min<size_t>(lane_cpus_.size(), (size_t)std::max(nt, 0)));
    pool_.reset(new ThreadPool(nt > 1 ? nt : 0, wc));
  }
  for (int l = 0; l < MAX_LAGS; ++l) { alias_thr_[l] = cfg_.thr[l]; alias_infl_[l] = cfg_.infl[l]; }
  HIP_OK(hipStreamSynchronize(stream_));
  HIP_OK(hipDeviceSynchronize());
  const int nt_used = std::max(cfg_.join_threads > 0 ? cfg_.join_threads : 0, pool_->size());
  const int st_cpu = (int)lane_cpus_.size() > nt_used ? lane_cpus_[nt_used] : -1;
  const int out_cpu = (int)lane_cpus_.size() > nt_used + 1 ? lane_cpus_[nt_used + 1] : -1;
  // The rollover lane mode is fixed before the first batch: node_round derives its candidate
  // cutoff from it, so every rank must use the same rule from round 0 (and the ingest thread must
  // never read a lane pointer the stats thread creates).  sx rows are decided on the stats thread.
  {
    const char* e = std::getenv("APM_ROLL_LANE");
    roll_lane_mode_ = (!e || e[0] != '0') && !want(OUT_SX);
    if (roll_lane_mode_) roll_lane_.reset(new TaskLane());
  }
  stats_thread_ = std::thread([this, st_cpu]() {
    if (st_cpu >= 0) pin_current_thread(st_cpu);
    hipSetDevice(cfg_.device);
    stats_worker();
  });
  out_thread_ = std::thread([this, out_cpu]() {
    if (out_cpu >= 0) pin_current_thread(out_cpu);
    hipSetDevice(cfg_.device);
    out_worker();
  });
}

Engine::~Engine() {
  if (roll_lane_) {  // a pending rollover half reads buffers freed below
    try { roll_lane_->wait_all(); } catch (...) {}
    roll_lane_.reset();
  }
  ahead_lane_.reset();  // drains a pending next-batch pre-pass before the join state goes
  if (in_stage_stream_) {  // a staged input copy writes a buffer the device join frees
    hipStreamSynchronize(in_stage_stream_);
    hipEventDestroy(in_stage_ev_);
    hipStreamDestroy(in_stage_stream_);
  }
  fb_lane_.reset();     // and a pending fb emission before its buffers
  if (nm_ev_) { hipEventSynchronize(nm_ev_); hipEventDestroy(nm_ev_); }
  if (h_nm_send_) hipHostFree(h_nm_send_);
  if (h_spill_snap_) hipHostFree(h_spill_snap_);
  for (auto& m : spill_mark_) if (m.ev) hipEventDestroy(m.ev);
  if (h_nm_recv_) hipHostFree(h_nm_recv_);
  checkpoint_shutdown();
  {
    std::lock_guard<std::mutex> g(st_mu_);
    st_stop_ = true;
  }
  st_cv_.notify_all();
  if (stats_thread_.joinable()) stats_thread_.join();
  {
    std::lock_guard<std::mutex> g(out_mu_);
    out_stop_ = true;
  }
  out_cv_.notify_all();
  if (out_thread_.joinable()) out_thread_.join();
  if (rel_lane_) {  // pending db releases read the buffers freed below
    try { rel_lane_->wait_all(); } catch (...) {}
    rel_lane_.reset();
  }
  if (coll_) {
    hipStreamSynchronize(coll_stream_);
    coll_.reset();
    if (fb_stream_) hipStreamSynchronize(fb_stream_);
    for (int i = 0; i < 2; ++i) {
      hipEventDestroy(fleet_ev_[i]); hipEventDestroy(pack_ev_[i]);
      if (fb_src_ev_[i]) hipEventDestroy(fb_src_ev_[i]);
      if (fb_ev_[i]) hipEventDestroy(fb_ev_[i]);
    }
    if (h_fb_total_) hipHostFree(h_fb_total_);
    if (fb_stream_) hipStreamDestroy(fb_stream_);
    if (node_ev_) hipEventDestroy(node_ev_);
    if (clock_ev_) hipEventDestroy(clock_ev_);
    for (hipEvent_t e : bucket_ev_)
      if (e) hipEventDestroy(e);
    if (h_node_send_) hipHostFree(h_node_send_);
    if (h_node_recv_) hipHostFree(h_node_recv_);
    hipStreamDestroy(coll_stream_);
  }
  if (h_sync_) hipHostFree(h_sync_);
  hipStreamSynchronize(stream_);
  hipStreamSynchronize(parse_stream_);
  for (void* p : allocations_) hipFree(p);
  for (auto& ps : pslot_) {
    hipHostFree(ps.h_bytes); hipHostFree(ps.h_chunk_begin); hipHostFree(ps.h_chunk_kind); hipHostFree(ps.h_chunk_file);
    if (ps.h_events) hipHostFree(ps.h_events);
    hipHostFree(ps.h_counts); hipHostFree(ps.h_watermark);
  }
  hipHostFree(h_alerts_);
  hipHostFree(h_alert_win_);
  hipHostFree(h_alert_z_);
  if (h_series_service_) hipHostFree(h_series_service_);
  hipHostFree(h_n_alerts_); hipEventDestroy(ev_alerts_); hipEventDestroy(ev_release_); hipHostFree(h_tx_); hipHostFree(h_gid_);
  for (int k = 0; k < 2; ++k) {
    hipHostFree(h_release_gid_[k]);
    {  // the sink's references to the staging buffers (its writers drain them; bounded wait)
      FmtHolds& hs = *fmt_holds_;
      std::unique_lock<std::mutex> lk(hs.mu);
      if (!hs.cv.wait_for(lk, std::chrono::seconds(60), [&] { return hs.n[k] == 0; })) continue;
    }
    if (h_fmt_out_[k]) hipHostFree(h_fmt_out_[k]);
    if (h_fs_off_[k]) hipHostFree(h_fs_off_[k]);
    hipEventDestroy(ev_rel_[k]);
    hipEventDestroy(ev_fmt_[k]);
  }
  for (int r = 0; r < FMT_RING; ++r) {
    FmtHolds& hs = *fmt_holds_;
    std::unique_lock<std::mutex> lk(hs.mu);
    if (!hs.cv.wait_for(lk, std::chrono::seconds(60), [&] { return hs.n[6 + r] == 0; })) continue;
    if (h_fmt_ring_[r]) hipHostFree(h_fmt_ring_[r]);
  }
  if (h_roll_out_) hipHostFree(h_roll_out_);
  if (cool_ev_) { hipEventSynchronize(cool_ev_); hipEventDestroy(cool_ev_); }
  if (h_cool_idx_) { hipHostFree(h_cool_idx_); hipHostFree(h_cool_val_); }
  if (dj_) {
    hipStreamSynchronize(out_stream_);
    hipHostFree(h_ring_min_); hipHostFree(h_rel_n_); hipHostFree(h_rel_total_); hipHostFree(h_unseen_flag_);
    for (int r = 0; r < REL_RING; ++r) {
      {  // zero-copy db rows still referenced by the sink (bounded wait, as for st/fs)
        FmtHolds& hs = *fmt_holds_;
        std::unique_lock<std::mutex> lk(hs.mu);
        if (!hs.cv.wait_for(lk, std::chrono::seconds(60), [&] { return hs.n[6 + FMT_RING + r] == 0; })) continue;
      }
      if (h_rel_text_[r]) hipHostFree(h_rel_text_[r]);
    }
    for (int k = 0; k < 2; ++k)
      if (h_rel_offs_[k]) hipHostFree(h_rel_offs_[k]);

    dj_.reset();
  }
  hipStreamSynchronize(out_stream_);
  hipStreamDestroy(out_stream_);
  if (out_stream2_) { hipStreamSynchronize(out_stream2_); hipStreamDestroy(out_stream2_); }
  if (rel_stream_) { hipStreamSynchronize(rel_stream_); hipStreamDestroy(rel_stream_); }
  hipHostFree(h_fmt_meta_);
  for (int k = 0; k < kStage; ++k) {
    if (h_stage_[k]) hipHostFree(h_stage_[k]);
    if (stage_ev_[k]) hipEventDestroy(stage_ev_[k]);
  }
  hipEventDestroy(ev_a_); hipEventDestroy(ev_b_);
  for (int k = 0; k < 2; ++k) {
    if (tail_csr_ev_[k]) hipEventDestroy(tail_csr_ev_[k]);
    if (h_tail_csr_[k]) hipHostFree(h_tail_csr_[k]);
  }
  hipStreamDestroy(stream_); hipStreamDestroy(parse_stream_);
}

int32_t Engine::add_server(const std::string& name) {
  flush();
  auto it = server_ids_.find(name);
  if (it != server_ids_.end()) return it->second;
  const int32_t id = (int32_t)servers_.size();
  servers_.push_back(name);
  server_ids_[name] = id;
  server_rank_.push_back(-1);
  server_next_service_.push_back(0);
  server_gidx_.push_back(id);
  server_first_batch_.push_back(-1);
  JoinConfig jc;
  jc.record_ttl_ms = cfg_.record_ttl_ms;
  jc.acct_ttl_ms = cfg_.acct_ttl_ms;
  jc.need_ttl_ms = cfg_.need_ttl_ms;
  jc.tz = cfg_.tz;
  shards_.emplace_back(new JoinShard(jc, &dict_, &files_, &servers_));
  return id;
}

int32_t Engine::add_file(const std::string& path, int kind, const std::string& server) {
  flush();
  const int32_t sid = add_server(server);
  files_.push_back(FileInfo{path, sid, (uint8_t)kind});
  if (files_.size() > (1 << 16)) throw std::runtime_error("too many files");
  return (int32_t)files_.size() - 1;
}

void Engine::set_override(const std::string& service, const ServiceOverride& o) {
  flush();
  overrides_[service] = o;
}
void Engine::clear_overrides() {
  flush();
  overrides_.clear();
}

// ----------------------------------------------------------------------------- series
void Engine::compute_series_settings(int32_t s, double* thr, double* infl, double& hard_max, uint8_t& suppressed) {
  const std::string& svc = dict_.service_name(series_[s].service);
  auto it = overrides_.find(svc);
  // z-score settings (stream_calc_z_score.js:106-150); with Q4 emulation the override is
  // written into the shared defaults and leaks into every later lookup.
  double* base_thr = cfg_.emulate_aliasing ? alias_thr_ : cfg_.thr;
  double* base_infl = cfg_.emulate_aliasing ? alias_infl_ : cfg_.infl;
  double t[MAX_LAGS], f[MAX_LAGS];
  for (int l = 0; l < cfg_.n_lags; ++l) { t[l] = base_thr[l]; f[l] = base_infl[l]; }
  if (it != overrides_.end()) {
    for (int l = 0; l < cfg_.n_lags; ++l) {
      if (it->second.has_thr[l] && (!cfg_.emulate_aliasing || it->second.thr[l] != 0)) t[l] = it->second.thr[l];
      if (it->second.has_infl[l] && (!cfg_.emulate_aliasing || it->second.infl[l] != 0)) f[l] = it->second.infl[l];
    }
    if (cfg_.emulate_aliasing)
      for (int l = 0; l < cfg_.n_lags; ++l) { alias_thr_[l] = t[l]; alias_infl_[l] = f[l]; }
  }
  for (int l = 0; l < cfg_.n_lags; ++l) { thr[l] = t[l]; infl[l] = f[l]; }
  hard_max = cfg_.hard_max_ms;
  suppressed = 0;
  if (it != overrides_.end()) {
    if (it->second.hard_max != 0) hard_max = it->second.hard_max;
    suppressed = it->second.suppressed ? 1 : 0;
  }
}

int32_t Engine::series_for(int32_t server, int32_t service) {
  // hot path (every tx of every batch): a dense per-server row indexed by the service id
  // (servers x services ints, a few hundred KB that stay in cache) in front of the hash map
  if ((size_t)server < ser_tab_.size() && (size_t)service < ser_tab_[server].size()) {
    const int32_t hit = ser_tab_[server][service];
    if (hit >= 0) return hit;
  }
  const uint64_t key = ((uint64_t)(uint32_t)(server + 1) << 32) | (uint32_t)service;  // never 0 (FlatMap)
  int32_t* slot = series_map_.find(key);
  if (slot) {
    ser_tab_put(server, service, *slot - 1);
    return *slot - 1;
  }
  if (n_series_ >= cfg_.max_series) return -1;
  const int32_t s = n_series_++;
  series_map_[key] = s + 1;
  ser_tab_put(server, service, s);
  if (server_rank_[server] < 0) {
    server_rank_[server] = next_server_rank_++;
    server_first_batch_[server] = (int64_t)stats_seq_;
  }
  const uint64_t ek = ((uint64_t)server_rank_[server] << 24) | (uint64_t)(server_next_service_[server]++);
  {
    std::lock_guard<std::mutex> g(series_mu_);
    series_.push_back(SeriesInfo{server, service, ek});
    cool_series_[cool_key_of(s)].push_back(s);
  }
  h_emit_key_.push_back(ek);
  {
    if ((int32_t)server_name_off_.size() <= server) server_name_off_.resize(server + 1, -1);
    if ((int32_t)service_name_off_.size() <= service) service_name_off_.resize(service + 1, -1);
    if (server_name_off_[server] < 0) server_name_off_[server] = intern_name(servers_[server]);
    if (service_name_off_[service] < 0) service_name_off_[service] = intern_name(dict_.service_name(service));
    h_ser_names_.push_back(server_name_off_[server]);
    h_ser_names_.push_back((int32_t)servers_[server].size());
    h_ser_names_.push_back(service_name_off_[service]);
    h_ser_names_.push_back((int32_t)dict_.service_name(service).size());
    perm_dirty_ = true;
  }
  h_thr_.resize((size_t)n_series_ * MAX_LAGS);
  h_infl_.resize((size_t)n_series_ * MAX_LAGS);
  h_hard_max_.push_back(cfg_.hard_max_ms);
  h_suppressed_.push_back(0);
  zscore_seen_.push_back(0);
  h_active_.push_back(0);
  max_name_len_ = std::max(max_name_len_, servers_[server].size() + dict_.service_name(service).size());
  if (cfg_.emulate_aliasing) {
    // Q4 emulation: settings depend on the order in which the z-score stage first sees series
    // (their first st), resolved at the rollover that makes them visible
    unseen_.push_back(s);
  } else {
    // order-independent settings: resolved now, uploaded with the batch's new series
    apply_series_settings(s);
    zscore_seen_[s] = 1;
  }
  return s;
}

// Series settings are resolved when the z-score stage first sees the series (its first `st`),
// in emission order -- which is what makes Q4 emulation reproduce the reference exactly.
void Engine::apply_series_settings(int32_t s) {
  double thr[MAX_LAGS], infl[MAX_LAGS];
  double hm;
  uint8_t sup;
  compute_series_settings(s, thr, infl, hm, sup);
  for (int l = 0; l < MAX_LAGS; ++l) { h_thr_[(size_t)s * MAX_LAGS + l] = thr[l]; h_infl_[(size_t)s * MAX_LAGS + l] = infl[l]; }
  h_hard_max_[s] = hm;
  h_suppressed_[s] = sup;
}

void Engine::refresh_series_settings() {
  flush();
  // config hot reload (updateAllServiceSettings, stream_calc_z_score.js:152-167)
  for (int l = 0; l < MAX_LAGS; ++l) { alias_thr_[l] = cfg_.thr[l]; alias_infl_[l] = cfg_.infl[l]; }
  std::vector<int32_t> order(n_series_);
  for (int32_t i = 0; i < n_series_; ++i) order[i] = i;
  std::sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return series_[a].emit_key < series_[b].emit_key; });
  for (int32_t s : order) if (zscore_seen_[s]) apply_series_settings(s);
  upload_series_tables(0);
}

void Engine::upload_series_tables(int32_t lo) {
  const int32_t n = n_series_;
  if (lo < 0) lo = 0;
  if (n <= lo) return;
  const size_t m = (size_t)(n - lo);
  // one pinned staging area: [thr, infl] per LAG, hard max, emit key (8 B each), suppressed
  const int L = cfg_.n_lags;
  char* st = stage(m * (8 * (2 * L + 2) + 1));
  double* col = (double*)st;
  for (int l = 0; l < L; ++l) {
    double* t = col + (size_t)(2 * l) * m;
    double* f = col + (size_t)(2 * l + 1) * m;
    for (size_t i = 0; i < m; ++i) {
      t[i] = h_thr_[(size_t)(lo + i) * MAX_LAGS + l];
      f[i] = h_infl_[(size_t)(lo + i) * MAX_LAGS + l];
    }
    h2d(lag_[l].thr + lo, t, m * 8, stream_);
    h2d(lag_[l].infl + lo, f, m * 8, stream_);
  }
  double* hm = col + (size_t)(2 * L) * m;
  uint64_t* ek = (uint64_t*)(col + (size_t)(2 * L + 1) * m);
  uint8_t* sp = (uint8_t*)(col + (size_t)(2 * L + 2) * m);
  std::memcpy(hm, h_hard_max_.data() + lo, m * 8);
  std::memcpy(ek, h_emit_key_.data() + lo, m * 8);
  std::memcpy(sp, h_suppressed_.data() + lo, m);
  h2d(d_hard_max_ + lo, hm, m * 8, stream_);
  h2d(d_emit_key_ + lo, ek, m * 8, stream_);
  h2d(d_suppressed_ + lo, sp, m, stream_);
  stage_done();
}

std::vector<uint64_t> Engine::cache_stats(bool drain) {
  if (drain) flush();
  if (dj_) {
    if (drain) HIP_OK(hipStreamSynchronize(parse_stream_));
    return dj_->cache_stats(watermark_, drain);  // (ordered on the join stream; a stat line does not wait)
  }
  return {};
}

JoinCounters Engine::join_counters() const {
  if (dj_) return dj_->counters();
  JoinCounters t;
  for (auto& s : shards_) {
    const JoinCounters& c = s->counters;
    t.events += c.events; t.tx += c.tx; t.tx_db += c.tx_db; t.expired_partials += c.expired_partials;
    t.need_expired += c.need_expired; t.ejb_exit_unmatched += c.ejb_exit_unmatched;
    t.invalid_acct += c.invalid_acct; t.audit_errors += c.audit_errors; t.host_fallback += c.host_fallback;
  }
  return t;
}

// ----------------------------------------------------------------------------- batch
// Stage a batch into a parse slot (canonical chunk order, pinned staging if needed) and enqueue
// H2D + K1/K2 on the parse stream.  Nothing waits here.
void Engine::launch_parse(ParseSlot& ps, const uint8_t* host_bytes, uint64_t n_bytes, const std::vector<Chunk>& chunks_in,
                          bool speculative) {
  const double t0 = now_ms();
  if (n_bytes > cfg_.max_batch_bytes) throw std::runtime_error("batch larger than max_batch_bytes");
  if (chunks_in.size() > cfg_.max_chunks) throw std::runtime_error("too many chunks in batch");
  // Canonical order: chunks grouped by server (shard) then file, keeping the caller's order
  // otherwise; the batch is re-laid out contiguously in that order in pinned memory.
  std::vector<size_t> order(chunks_in.size());
  for (size_t i = 0; i < order.size(); ++i) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) {
    return files_[chunks_in[a].file].server < files_[chunks_in[b].file].server;
  });
  ps.chunk_file.assign(chunks_in.size(), 0);
  uint64_t off = 0;
  // Fast path: chunks already canonical and contiguous from 0 (bench corpus, tailer output) ->
  // no host copy; the H2D reads the caller's (ideally pinned) buffer directly.
  bool canonical = true;
  for (size_t k = 0; k < order.size(); ++k) {
    const Chunk& c = chunks_in[k];
    if (order[k] != k || c.begin != off) { canonical = false; break; }
    off = c.end;
  }
  canonical = canonical && off == n_bytes && n_bytes + 64 <= cfg_.max_batch_bytes + 256;
  ps.hb = ps.h_bytes;
  if (canonical) {
    ps.hb = host_bytes;
    for (size_t k = 0; k < order.size(); ++k) {
      const Chunk& c = chunks_in[k];
      if (c.end > c.begin && host_bytes[c.end - 1] != '\n') throw std::runtime_error("chunk must end with a newline");
      ps.h_chunk_begin[k] = (uint32_t)c.begin;
      ps.h_chunk_kind[k] = files_[c.file].kind;
      ps.h_chunk_file[k] = (uint32_t)c.file;
      ps.chunk_file[k] = c.file;
    }
  } else {
    off = 0;
    const bool in_place = host_bytes == ps.h_bytes;
    std::vector<uint8_t> tmp_copy;
    const uint8_t* src = host_bytes;
    if (in_place) {  // caller filled our staging buffer: copy aside before re-layout
      tmp_copy.assign(host_bytes, host_bytes + n_bytes);
      src = tmp_copy.data();
    }
    for (size_t k = 0; k < order.size(); ++k) {
      const Chunk& c = chunks_in[order[k]];
      const uint64_t len = c.end - c.begin;
      if (len > 0 && src[c.end - 1] != '\n') throw std::runtime_error("chunk must end with a newline");
      std::memcpy(ps.h_bytes + off, src + c.begin, len);
      ps.h_chunk_begin[k] = (uint32_t)off;
      ps.h_chunk_kind[k] = files_[c.file].kind;
      ps.h_chunk_file[k] = (uint32_t)c.file;
      ps.chunk_file[k] = c.file;
      off += len;
    }
    std::memset(ps.h_bytes + off, 0, 64);
  }
  const uint32_t n_chunks = (uint32_t)order.size();
  ps.h_chunk_begin[n_chunks] = (uint32_t)off;
  ps.n_bytes = off;
  ps.src = host_bytes;
  ps.src_n = n_bytes;
  metrics_.bytes += off;
  ++metrics_.batches;

  // ---- K1/K2 on the GPU.  Host join: d_bytes_ / d_events_ are free (the previous parse was
  // finished -- its events copied to its own host slot -- before this launch).  Device join: the
  // slot's own device buffers (the other slot's batch may still be joined on the join stream).
  const int k = (int)(&ps - pslot_);
  // the input already copied by stage_batch (two batches ahead): take its buffer
  bool staged = false;
  if (dev() && canonical && in_stage_src_ == host_bytes && in_stage_n_ == n_bytes && in_stage_ev_) {
    HIP_OK(hipStreamWaitEvent(parse_stream_, in_stage_ev_, 0));
    dj_->swap_stage(k);
    staged = true;
    ++metrics_.staged_batches;
  }
  in_stage_src_ = nullptr;
  in_stage_n_ = 0;
  uint8_t* dbytes = dev() ? dj_->d_bytes(k) : d_bytes_;
  Event* devents = dev() ? dj_->d_events(k) : (ps.d_events_host ? ps.d_events_host : d_events_);
  if (!staged) HIP_OK(hipMemcpyAsync(dbytes, ps.hb, off, hipMemcpyHostToDevice, parse_stream_));
  // (apm_parse_batch zeroes the 64 bytes after the batch inside its first kernel)
  h2d(d_chunk_begin_[k], ps.h_chunk_begin, (n_chunks + 1) * 4, parse_stream_);
  h2d(d_chunk_kind_[k], ps.h_chunk_kind, n_chunks + 1, parse_stream_);
  h2d(d_chunk_file_[k], ps.h_chunk_file, (n_chunks + 1) * 4, parse_stream_);
  if (apm_parse_batch(dbytes, off, d_chunk_begin_[k], d_chunk_kind_[k], d_chunk_file_[k], n_chunks, d_parse_ws_,
                      cfg_.max_lines, devents, d_counts_, d_counts_ + 1, d_watermark_, d_file_open_, &cfg_.tz,
                      parse_stream_) != 0)
    throw std::runtime_error("parse workspace too small");
  if (dev()) {
    dj_->set_chunks(k, ps.chunk_file, d_chunk_file_[k], d_chunk_kind_[k], parse_stream_);
    dj_->select_host(k, d_counts_, cfg_.max_lines, parse_stream_);
  }
  d2h(ps.h_counts, d_counts_, 8, parse_stream_);
  d2h(ps.h_watermark, d_watermark_, 8, parse_stream_);
  // Prefetched parse: the event count is only known on the device, so copy a guess (the last
  // batch's count + 25 %) right behind the kernels.  The DMA then runs during the current
  // batch's host join instead of on the ingest thread's critical path (15 MB, ~0.3 ms), and
  // finish_parse copies only what the guess missed.
  ps.spec_copied = 0;
  if (speculative && !dev() && !ps.d_events_host && spec_events_) {
    ps.spec_copied = std::min<uint32_t>(spec_events_, cfg_.max_lines);
    HIP_OK(hipMemcpyAsync(ps.h_events, d_events_, (size_t)ps.spec_copied * sizeof(Event), hipMemcpyDeviceToHost,
                          parse_stream_));
  }
  ps.pending = true;
  metrics_.t_parse_ms += now_ms() - t0;
}

void Engine::stage_batch(const uint8_t* host_bytes, uint64_t n_bytes) {
  if (!dev() || !host_bytes || n_bytes == 0 || n_bytes > cfg_.max_batch_bytes) return;
  const double t0 = now_ms();
  if (!in_stage_stream_) {
    HIP_OK(hipStreamCreateWithFlags(&in_stage_stream_, hipStreamNonBlocking));
    HIP_OK(hipEventCreateWithFlags(&in_stage_ev_, hipEventDisableTiming));
  }
  // The staging buffer is free: it is either fresh, the buffer an unconsumed earlier stage wrote
  // (ordered behind that copy on this stream), or -- after a swap -- the parse slot buffer of the
  // batch two back, whose join finished before the current process_batch returned.
  HIP_OK(hipMemcpyAsync(dj_->d_stage(), host_bytes, n_bytes, hipMemcpyHostToDevice, in_stage_stream_));
  HIP_OK(hipEventRecord(in_stage_ev_, in_stage_stream_));
  in_stage_src_ = host_bytes;
  in_stage_n_ = n_bytes;
  trace_event("stage H2D (launch)", t0, now_ms(), 0);
}

// Wait for a launched parse and copy its events into the slot's pinned host buffer.
void Engine::finish_parse(ParseSlot& ps) {
  const double t0 = now_ms();
  HIP_OK(hipStreamSynchronize(parse_stream_));
  ps.n_events = ps.h_counts[0];
  ps.n_lines = ps.h_counts[1];
  if (ps.n_lines > cfg_.max_lines) throw std::runtime_error("batch has more lines than max_lines");
  metrics_.lines += ps.n_lines;
  metrics_.events += ps.n_events;
  if (dev()) {
    dj_->finish_select((int)(&ps - pslot_), parse_stream_);
  } else if (ps.n_events > ps.spec_copied && !ps.d_events_host) {
    const uint32_t lo = ps.spec_copied;
    HIP_OK(hipMemcpyAsync(ps.h_events + lo, d_events_ + lo, (size_t)(ps.n_events - lo) * sizeof(Event),
                          hipMemcpyDeviceToHost, parse_stream_));
    HIP_OK(hipStreamSynchronize(parse_stream_));
  }
  ps.spec_copied = 0;
  spec_events_ = ps.n_events + ps.n_events / 4 + 1024;
  ps.pending = false;
  last_slot_ = (int)(&ps - pslot_);
  metrics_.t_parse_ms += now_ms() - t0;
}

// Merge the shard outputs into the reference's single-stream order.  Cache-expiry emissions
// (seq bit 63 clear, keyed by creation) precede every line emission and may interleave across
// shards: k-way merge (rare).  Line emissions are keyed by the global line index, and each
// shard's lines form one contiguous range (chunks are grouped by server), so those parts are
// concatenated in range order; `multi` (a server with several line ranges in the batch) sorts
// the line part by its (line, sub) key instead.
static void merge_shard_outputs(const std::vector<std::vector<TxOut>>& outs, bool multi, std::vector<TxOut>& txs) {
  txs.clear();
  const int ns = (int)outs.size();
  size_t total = 0;
  std::vector<size_t> split(ns, 0);
  for (int k = 0; k < ns; ++k) {
    auto& v = outs[k];
    total += v.size();
    size_t p = 0;
    while (p < v.size() && !(v[p].seq >> 63)) ++p;
    split[k] = p;
  }
  txs.reserve(total);
  using Item = std::pair<uint64_t, std::pair<int, size_t>>;
  std::priority_queue<Item, std::vector<Item>, std::greater<Item>> pq;
  for (int k = 0; k < ns; ++k)
    if (split[k] > 0) pq.push({outs[k][0].seq, {k, 0}});
  while (!pq.empty()) {
    auto it = pq.top();
    pq.pop();
    auto& v = outs[it.second.first];
    txs.push_back(v[it.second.second]);
    const size_t nx = it.second.second + 1;
    if (nx < split[it.second.first]) pq.push({v[nx].seq, {it.second.first, nx}});
  }
  std::vector<int> order;
  for (int k = 0; k < ns; ++k)
    if (split[k] < outs[k].size()) order.push_back(k);
  std::sort(order.begin(), order.end(), [&](int a, int b) { return outs[a][split[a]].seq < outs[b][split[b]].seq; });
  const size_t line_part = txs.size();
  for (int k : order) txs.insert(txs.end(), outs[k].begin() + (ptrdiff_t)split[k], outs[k].end());
  if (multi)
    std::stable_sort(txs.begin() + (ptrdiff_t)line_part, txs.end(),
                     [](const TxOut& a, const TxOut& b) { return a.seq < b.seq; });
}

void Engine::process_batch(const uint8_t* host_bytes, uint64_t n_bytes, const std::vector<Chunk>& chunks_in,
                           double now_override, const uint8_t* next_bytes, uint64_t next_n,
                           const std::vector<Chunk>* next_chunks) {
  const double t0 = now_ms();
  roctxRangePushA("apm.parse");
  ParseSlot& ps = pslot_[cur_slot_];
  if (prefetched_) {
    // the previous call already launched this batch's parse: it must be the same batch
    if (ps.src != host_bytes || ps.src_n != n_bytes) throw std::runtime_error("batch differs from the prefetched one");
    prefetched_ = false;
  } else {
    launch_parse(ps, host_bytes, n_bytes, chunks_in);
  }
  if (ahead_task_) {  // the previous call finished this batch's parse (+ pre-pass) on the lane
    const uint64_t t = ahead_task_;
    ahead_task_ = 0;
    ahead_lane_->wait(t);
  }
  if (ps.pending) finish_parse(ps);
  if (dev()) {
    process_batch_dev_tail(ps, t0, now_override, next_bytes, next_n, next_chunks);
    return;
  }
  // Pipelining: the next batch's H2D + parse kernels run on the GPU while this batch is joined.
  // Their host side (chunk table, ~15 launches, copies: ~0.3 ms) is issued by this thread while
  // the join workers run, instead of ahead of them on the critical path.
  ParseSlot& next_ps = pslot_[cur_slot_ ^ 1];
  const bool launch_next = next_bytes && next_chunks;
  const std::function<void()> launch_next_parse = [&]() {
    launch_parse(next_ps, next_bytes, next_n, *next_chunks, /*speculative=*/true);
    prefetched_ = true;
  };
  cur_slot_ ^= 1;
  const uint8_t* hb = ps.hb;
  const std::vector<int32_t>& chunk_file = ps.chunk_file;
  const uint32_t n_events = ps.n_events;
  const Event* h_events = ps.h_events;
  last_n_events_ = n_events;
  const double t1 = now_ms();
  roctxRangePop();
  roctxRangePushA("apm.join");
  trace_event("parse", t0, t1, 0);

  // ---- join on the host, one task per server shard
  const double clock = now_override >= 0 ? now_override : watermark_;
  if (lockstep_) lockstep_issue(batch_watermark(ps));
  // Event ranges per shard without walking the events (15 MB of freshly DMA'd records): events
  // are in chunk order, so each run of same-server chunks maps to one binary-searched range.
  std::vector<std::vector<std::pair<uint32_t, uint32_t>>> shard_range(shards_.size());
  {
    auto first_event_of_chunk = [&](uint32_t c) {
      uint32_t lo = 0, hi = n_events;
      while (lo < hi) {
        const uint32_t mid = lo + (hi - lo) / 2;
        if (h_events[mid].chunk < c) lo = mid + 1; else hi = mid;
      }
      return lo;
    };
    const uint32_t nc = (uint32_t)chunk_file.size();
    uint32_t c = 0;
    while (c < nc) {
      const int32_t srv = files_[chunk_file[c]].server;
      uint32_t d = c + 1;
      while (d < nc && files_[chunk_file[d]].server == srv) ++d;
      const uint32_t lo = first_event_of_chunk(c), hi = first_event_of_chunk(d);
      if (hi > lo) shard_range[srv].push_back({lo, hi});
      c = d;
    }
  }
  shard_ms_.assign(shards_.size() * 16, 0.0);  // one cache line per shard
  shard_maxb_.assign(shards_.size() * 8, INT64_MIN);
  pool_->run((int)shards_.size(), [&](int s) {
    const double ts0 = now_ms();
    JoinShard& sh = *shards_[s];
    sh.out().clear();
    sh.begin_batch(clock, batch_no_);
    for (const auto& r : shard_range[s]) sh.process(h_events + r.first, r.second - r.first, hb, chunk_file);
    if (lockstep_) {  // newest 10 s bucket of this shard's tx, for the lock-step clock (scanned in parallel here)
      int64_t b = INT64_MIN;
      for (const TxOut& t : sh.out()) {
        if (t.to_db || !(t.end_ms == t.end_ms) || t.end_ms < 10000) continue;
        const int64_t tb = (int64_t)t.end_ms / 10000;
        if (tb > b) b = tb;
      }
      shard_maxb_[(size_t)s * 8] = b;
    }
    const double ts1 = now_ms();
    shard_ms_[(size_t)s * 16] = ts1 - ts0;
    trace_event("shard", ts0, ts1, 2 + s);
  }, launch_next ? &launch_next_parse : nullptr);
  const double t1b = now_ms();
  metrics_.t_join_shards_ms += t1b - t1;
  {
    double sum = 0, mx = 0;
    for (size_t s = 0; s < shards_.size(); ++s) { sum += shard_ms_[s * 16]; mx = std::max(mx, shard_ms_[s * 16]); }
    metrics_.t_shard_busy_ms += shards_.empty() ? 0 : sum / shards_.size();
    metrics_.t_shard_max_ms += mx;
  }
  // Hand the shard outputs over as they are (swapped out, the shards get recycled vectors back):
  // the stats thread merges them into the single-stream order (merge_shard_outputs), which
  // takes ~0.15 ms of copying off this thread's critical path.
  std::vector<std::vector<TxOut>> outs(shards_.size());
  {
    std::lock_guard<std::mutex> g(out_pool_mu_);
    for (size_t k = 0; k < shards_.size(); ++k) {
      outs[k].swap(shards_[k]->out());
      if (!out_pool_.empty()) {
        shards_[k]->out().swap(out_pool_.back());
        out_pool_.pop_back();
      }
    }
  }
  bool multi = false;
  for (auto& r : shard_range) multi |= r.size() > 1;
  const double t2 = now_ms();
  metrics_.t_join_ms += t2 - t1;
  metrics_.t_merge_ms += t2 - t1b;
  roctxRangePop();
  trace_event("join", t1, t1b, 0);
  trace_event("handoff", t1b, t2, 0);

  // advance the watermark clock (max leading timestamp seen so far); lock-step: the node-wide
  // watermark (cache clock of the next batch) and the newest-bucket exchange
  int sync_slot = -1;
  if (lockstep_) {
    int64_t bmax = INT64_MIN;
    for (size_t k = 0; k < shards_.size(); ++k) bmax = std::max(bmax, shard_maxb_[k * 8]);
    sync_slot = lockstep_collect(bmax);
  } else {
    watermark_ = batch_watermark(ps);
  }

  // ---- stats / z-score / alerts: handed to the stats thread, overlapping the next batch's
  // H2D + parse (parse stream) and host join (pool) with this batch's GPU stats work.
  const double tp0 = now_ms();
  post_stats(std::move(outs), multi, t0, sync_slot);
  const double tp1 = now_ms();
  trace_event("post", tp0, tp1, 0);
  // post_stats returned: the stats thread finished (and packed) every earlier batch
  if (coll_) fleet_exchange_upto(fleet_posted_ - 1);
  trace_event("fleet.exchange", tp1, now_ms(), 0);
  metrics_.t_total_ms += now_ms() - t0;
  ++batch_no_;
}

// Device join (K4/K6 on the GPU): the next batch's parse is launched first (parse stream), then
// this batch is joined on the join stream while it runs; the stats thread gets device arrays.
void Engine::process_batch_dev_tail(ParseSlot& ps, double t0, double now_override, const uint8_t* next_bytes,
                                    uint64_t next_n, const std::vector<Chunk>* next_chunks) {
  const int k = (int)(&ps - pslot_);
  if (next_bytes && next_chunks) {
    launch_parse(pslot_[k ^ 1], next_bytes, next_n, *next_chunks, /*speculative=*/true);
    prefetched_ = true;
  }
  cur_slot_ = k ^ 1;
  last_n_events_ = ps.n_events;
  const double t1 = now_ms();
  roctxRangePop();
  roctxRangePushA("apm.join");
  trace_event("parse", t0, t1, 0);
  const double clock = now_override >= 0 ? now_override : watermark_;
  // lock-step (1/2): this batch's clocks go out before its join kernels (see lockstep_issue)
  if (lockstep_) lockstep_issue(batch_watermark(ps));
  DevJoinBatch b;
  const DeviceJoin::ParallelFor par = [this](int n, const std::function<void(int)>& fn) { pool_->run(n, fn); };
  // once this batch's join kernels are queued, a lane thread finishes the next batch's parse and
  // does its host pre-pass (audit blocks) while this thread completes the batch (join waits,
  // clocks, hand-off): both leave the next batch's critical path
  const std::function<void()> ahead = [this, k, par]() {
    if (!ahead_lane_) ahead_lane_.reset(new TaskLane());
    ahead_task_ = ahead_lane_->post([this, k, par]() {
      ParseSlot& nx = pslot_[k ^ 1];
      const double ta = now_ms();
      finish_parse(nx);
      dj_->prepass_ahead(k ^ 1, nx.hb, par);
      trace_event("next parse+prepass", ta, now_ms(), 3);
    });
  };
  static const bool ahead_on = [] { const char* e = std::getenv("APM_PREPASS_AHEAD"); return !e || e[0] != '0'; }();
  // while this batch's join kernels run: the next batch's parse / pre-pass (ahead lane) and the
  // previous batches' fleet exchange (collective, enqueued on the coll stream in round order --
  // before this batch's lock-step all-reduce, as when it ran after the previous hand-off)
  const bool do_ahead = prefetched_ && ahead_on;
  const std::function<void()> meanwhile = [this, &ahead, do_ahead]() {
    if (do_ahead) ahead();
    if (coll_ && fleet_due_ > fleet_rounds_) {
      const double tf = now_ms();
      fleet_exchange_upto(fleet_due_);
      trace_event("fleet.exchange", tf, now_ms(), 0);
    }
  };
  dj_->run(k, ps.hb, ps.n_events, ps.n_bytes, clock, batch_no_, want(OUT_TRANSACTIONS), want(OUT_AUDIT_DB), b, par,
           &meanwhile);
  const double t2 = now_ms();
  metrics_.t_join_ms += t2 - t1;
  metrics_.t_join_shards_ms += t2 - t1;
  metrics_.t_shard_max_ms += t2 - t1;
  metrics_.t_shard_busy_ms += t2 - t1;
  roctxRangePop();
  trace_event("join (GPU)", t1, t2, 0);
  if (trace_on_) {
    static const char* names[DeviceJoin::kPhases] = {"dj.prepass", "dj.upload", "dj.launch", "dj.syncA",
                                                     "dj.register", "dj.plan", "dj.write+syncC", "dj.tail"};
    for (int i = 0; i < DeviceJoin::kPhases; ++i) trace_event(names[i], dj_->phase_t[i], dj_->phase_t[i + 1], 2);
    for (const auto& sp : dj_->spans) trace_event(sp.first, sp.second.first, sp.second.second, 2);
  }
  // lock-step (2/2): collect the clocks, send the newest bucket (the stats thread waits for it)
  const int sync_slot = lockstep_ ? lockstep_collect(b.max_bucket) : -1;
  if (!lockstep_) watermark_ = batch_watermark(ps);
  const double tp0 = now_ms();
  post_stats_dev(std::move(b), t0, sync_slot);
  const double tp1 = now_ms();
  trace_event("post", tp0, tp1, 0);
  if (coll_) fleet_due_ = fleet_posted_ - 1;  // exchanged during the next batch's join (see above)
  metrics_.t_total_ms += now_ms() - t0;
  ++batch_no_;
}

// Transactions from a reference parser stage (the `transactions` queue, entries.js TxEntry
// CSV) enter at the stats stage: one TxOut per line in arrival order, the line itself kept as the
// pending tx text for the release (db stream).  Host-join mode only (the shards' text arenas
// carry the lines; the device join has no such input).
void Engine::process_tx_lines(const std::string& blob, double now) {
  if (dev()) throw std::runtime_error("process_tx_lines needs gpu.joinOnDevice = false");
  const double t0 = now_ms();
  std::vector<std::vector<TxOut>> outs(shards_.size());
  uint64_t line = 0;
  size_t i = 0;
  while (i < blob.size()) {
    size_t j = blob.find('\n', i);
    if (j == std::string::npos) j = blob.size();
    const std::string_view ln(blob.data() + i, j - i);
    i = j + 1;
    if (ln.size() < 3 || ln.compare(0, 3, "tx|") != 0) continue;
    std::string_view f[9];
    int nf = 0;
    size_t a = 0;
    while (nf < 9) {
      const size_t b = ln.find('|', a);
      f[nf++] = ln.substr(a, b == std::string_view::npos ? std::string_view::npos : b - a);
      if (b == std::string_view::npos) break;
      a = b + 1;
    }
    if (nf < 8) { ++metrics_.tx_dropped; continue; }
    const std::string srv(f[1]);
    const auto known = server_ids_.find(srv);
    const int32_t sid = known != server_ids_.end() ? known->second : add_server(srv);
    if ((size_t)sid >= outs.size()) outs.resize(shards_.size());
    const int32_t svc = dict_.service_id(f[2]);
    std::string& arena = shards_[sid]->text();
    TxOut t{};
    t.seq = (1ULL << 63) | (line++ << 12);
    t.server = sid;
    t.service = svc;
    t.raw_svc = svc;
    t.end_ms = js::parse_int(f[6]);
    t.elapsed = js::parse_int(f[7]);
    t.line_off = (uint32_t)arena.size();
    t.line_len = (uint32_t)ln.size();
    t.to_db = false;
    t.toplevel = nf > 8 && f[8] == "Y";
    arena.append(ln.data(), ln.size());
    arena += '\n';
    outs[sid].push_back(t);
  }
  if (now >= 0 && now > watermark_) watermark_ = now;
  outs.resize(shards_.size());
  metrics_.lines += line;
  post_stats(std::move(outs), /*multi=*/true, t0, /*sync_slot=*/-1);
  metrics_.t_total_ms += now_ms() - t0;
  ++batch_no_;
}

void Engine::trace_event(const char* name, double t0, double t1, int tid) {
  if (!trace_on_) return;
  std::lock_guard<std::mutex> g(trace_mu_);
  if (trace_.size() < 1000000) trace_.push_back(TraceEvent{name, t0, t1, tid, batch_no_});
}

std::vector<TraceEvent> Engine::take_trace() {
  flush();
  std::lock_guard<std::mutex> g(trace_mu_);
  std::vector<TraceEvent> r;
  r.swap(trace_);
  return r;
}

void Engine::recycle_arena(std::string&& a) {
  a.clear();
  std::lock_guard<std::mutex> g(arena_mu_);
  if (arena_pool_.size() < 4 * shards_.size() + 8) arena_pool_.push_back(std::move(a));
}

void Engine::stats_worker() {
  StatsJob job;
  for (;;) {
    {
      std::unique_lock<std::mutex> lk(st_mu_);
      st_cv_.wait(lk, [&]() { return st_stop_ || st_has_job_; });
      if (st_stop_ && !st_has_job_) return;
      job.outs.swap(st_job_.outs);
      job.multi = st_job_.multi;
      job.text.swap(st_job_.text);
      job.t0 = st_job_.t0;
      job.sync_slot = st_job_.sync_slot;
      job.dev = st_job_.dev;
      job.seq = st_job_.seq;
      job.round = st_job_.round;
      std::swap(job.dj, st_job_.dj);
      st_has_job_ = false;
    }
    const double t = now_ms();
    roctxRangePushA("apm.stats");
    try {
      stats_seq_ = job.seq;
      stats_round_ = job.round;
      apply_ctx_pending(job.seq);
      apply_reconfig_pending(job.seq);
      node_take_text();  // al rows decided by the rollover lane / the node rounds
      trace_event("st.pre", t, now_ms(), 1);
      if (job.dev) {
        stats_for_batch_dev(job.dj, job.t0);
      } else {
        cur_text_ = &job.text;
        const double tm = now_ms();
        merge_shard_outputs(job.outs, job.multi, job.txs);
        trace_event("merge", tm, now_ms(), 1);
        {  // the shard vectors go back to the ingest thread with their capacity
          std::lock_guard<std::mutex> g(out_pool_mu_);
          for (auto& v : job.outs) {
            v.clear();
            if (out_pool_.size() < 2 * shards_.size() + 4) out_pool_.push_back(std::move(v));
          }
          job.outs.clear();
        }
        stats_for_batch(job.txs, job.t0);
      }
      const double ta = now_ms();
      if (job.sync_slot >= 0) apply_latest_locked(lockstep_latest(job.sync_slot), job.t0);
      trace_event("st.apply_latest", ta, now_ms(), 1);
      fleet_pack_locked();
      if (roll_pending_) finish_rollover();  // (a rollover the lane does not take: decided here)
      if (node_mode_) {
        // round marker: every rollover of this batch has queued its alert candidates once the
        // lane (FIFO) got here -- the ingest thread's node round waits for it (wait_roll_round)
        const int64_t r = (int64_t)job.round;
        auto mark = [this, r]() {
          {
            std::lock_guard<std::mutex> g(roll_mu_);
            roll_done_round_ = std::max(roll_done_round_, r);
          }
          roll_cv_.notify_all();
        };
        if (roll_lane_) roll_lane_->post(mark);
        else mark();
      }
      const double td = now_ms();
      drain_sinks(~kLaneKinds);
      trace_event("st.drain", td, now_ms(), 1);
    } catch (const std::exception& e) {
      std::lock_guard<std::mutex> g(st_mu_);
      st_error_ = e.what();
    }
    roctxRangePop();
    trace_event("stats", t, now_ms(), 1);
    {
      std::lock_guard<std::mutex> g(st_mu_);
      metrics_.t_stats_ms += now_ms() - t;
      st_busy_ = false;
    }
    st_cv_.notify_all();
  }
}

void Engine::post_stats(std::vector<std::vector<TxOut>>&& outs, bool multi, double t0, int sync_slot) {
  std::unique_lock<std::mutex> lk(st_mu_);
  st_cv_.wait(lk, [&]() { return !st_busy_; });
  if (!st_error_.empty()) { std::string e = st_error_; st_error_.clear(); throw std::runtime_error(e); }
  {
    std::lock_guard<std::mutex> g(out_mu_);
    if (!out_error_.empty()) { std::string e = out_error_; out_error_.clear(); throw std::runtime_error(e); }
  }
  st_job_.outs = std::move(outs);
  st_job_.multi = multi;
  // hand the shards' formatted tx lines to the stats thread; the shards get the previous
  // batch's (consumed) arenas back and reuse their capacity
  st_job_.text.resize(shards_.size());
  for (size_t i = 0; i < shards_.size(); ++i) {
    st_job_.text[i].swap(shards_[i]->text());
    // the returned string may be empty (its arena became a release block): hand the shard a
    // recycled arena so the join workers never page-fault fresh memory
    if (shards_[i]->text().capacity() < (1u << 20)) {
      std::lock_guard<std::mutex> g(arena_mu_);
      if (!arena_pool_.empty()) { shards_[i]->text().swap(arena_pool_.back()); arena_pool_.pop_back(); }
    }
  }
  st_job_.t0 = t0;
  st_job_.sync_slot = sync_slot;
  st_job_.seq = batch_no_;
  st_job_.round = fleet_posted_;
  if (coll_) ++fleet_posted_;
  st_has_job_ = true;
  st_busy_ = true;
  lk.unlock();
  st_cv_.notify_all();
  if (!cfg_.async_stats) flush();
}

void Engine::post_stats_dev(DevJoinBatch&& b, double t0, int sync_slot) {
  std::unique_lock<std::mutex> lk(st_mu_);
  st_cv_.wait(lk, [&]() { return !st_busy_; });
  if (!st_error_.empty()) { std::string e = st_error_; st_error_.clear(); throw std::runtime_error(e); }
  {
    std::lock_guard<std::mutex> g(out_mu_);
    if (!out_error_.empty()) { std::string e = out_error_; out_error_.clear(); throw std::runtime_error(e); }
  }
  st_job_.dev = true;
  st_job_.dj = std::move(b);
  st_job_.t0 = t0;
  st_job_.sync_slot = sync_slot;
  st_job_.seq = batch_no_;
  st_job_.round = fleet_posted_;
  if (coll_) ++fleet_posted_;
  st_has_job_ = true;
  st_busy_ = true;
  lk.unlock();
  st_cv_.notify_all();
  if (!cfg_.async_stats) flush();
}

void Engine::flush() {
  std::unique_lock<std::mutex> lk(st_mu_);
  st_cv_.wait(lk, [&]() { return !st_busy_; });
  // the stats thread is idle: complete its last rollover (lane), then no new output-lane task
  // can appear
  try {
    finish_rollover();
  } catch (const std::exception& e) {
    if (st_error_.empty()) st_error_ = e.what();
  }
  out_wait_idle();
  if (fb_lane_) fb_lane_->wait_all();
  {
    std::lock_guard<std::mutex> g(out_mu_);
    metrics_.t_out_ms += t_out_ms_;
    t_out_ms_ = 0;
    metrics_.formatted_bytes += formatted_bytes_lane_;
    formatted_bytes_lane_ = 0;
    if (!out_error_.empty()) { std::string e = out_error_; out_error_.clear(); throw std::runtime_error(e); }
  }
  if (!st_error_.empty()) { std::string e = st_error_; st_error_.clear(); throw std::runtime_error(e); }
  apply_ctx_pending(UINT64_MAX);  // the stats thread is idle
  apply_reconfig_pending(UINT64_MAX);  // (tags >= batch_no_: no job of an earlier batch is left)
  node_take_text();  // decided alerts (rollover lane / node rounds) -> the al stream
  drain_kind(OUT_AL);
  if (node_mode_) {
    metrics_.alerts += node_alerts_;
    node_alerts_ = 0;
  }
  {
    // one export kernel into the spare words of the pinned format meta block ([8, 15)): three
    // pageable hipMemcpyAsync round trips were part of every drain
    unsigned long long u[3] = {0, 0, 0};
    int32_t fb = 0;
    ExportArgs ex{};
    if (dev()) ex.add(d_unmapped_, hd_fmt_meta_ + 8, 8);
    ex.add(d_spill_drop_, hd_fmt_meta_ + 10, 8);
    ex.add(d_spill_drop_ + 1, hd_fmt_meta_ + 12, 8);
    ex.add(d_fmt_fallback_, hd_fmt_meta_ + 14, 4);
    apm_export(&ex, stream_);
    HIP_OK(hipStreamSynchronize(stream_));
    if (dev()) std::memcpy(&u[0], h_fmt_meta_ + 8, 8);
    std::memcpy(&u[1], h_fmt_meta_ + 10, 16);
    std::memcpy(&fb, h_fmt_meta_ + 14, 4);
    metrics_.series_overflow_tx = u[0];
    metrics_.spill_dropped = u[1];
    metrics_.nan_windows_clipped = u[2];
    metrics_.format_fallbacks = (uint64_t)fb;
  }
}

std::string Engine::last_events() const {
  if (!dj_) return std::string((const char*)pslot_[last_slot_].h_events, (size_t)last_n_events_ * sizeof(Event));
  std::string out((size_t)last_n_events_ * sizeof(Event), '\0');
  if (last_n_events_)
    HIP_OK(hipMemcpy(&out[0], const_cast<DeviceJoin&>(*dj_).d_events(last_slot_), out.size(), hipMemcpyDeviceToHost));
  return out;
}

// ----------------------------------------------------------------------------- output lane
// The stats thread enqueues "wait for this D2H, then emit" tasks and moves on to the next
// rollover / batch; the lane runs them in order.  It owns the db (released tx), st and fs
// streams, so those blobs and sinks are only touched here (or with both lanes idle).
void Engine::out_worker() {
  for (;;) {
    std::function<void()> fn;
    {
      std::unique_lock<std::mutex> lk(out_mu_);
      out_cv_.wait(lk, [&]() { return out_stop_ || !out_q_.empty(); });
      if (out_q_.empty()) return;  // stop requested and nothing left
      fn = std::move(out_q_.front());
      out_q_.pop_front();
    }
    const double t = now_ms();
    std::string err;
    try {
      fn();
    } catch (const std::exception& e) {
      err = e.what();
    }
    {
      std::lock_guard<std::mutex> g(out_mu_);
      t_out_ms_ += now_ms() - t;
      if (!err.empty() && out_error_.empty()) out_error_ = err;
      ++out_done_;
    }
    out_cv_.notify_all();
  }
}

TaskLane::TaskLane() {
  th_ = std::thread([this]() {
    for (;;) {
      std::function<void()> fn;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&]() { return stop_ || !q_.empty(); });
        if (q_.empty()) return;
        fn = std::move(q_.front());
        q_.pop_front();
      }
      std::string err;
      try {
        fn();
      } catch (const std::exception& e) {
        err = e.what();
      }
      std::lock_guard<std::mutex> g(mu_);
      if (!err.empty() && err_.empty()) err_ = err;
      ++done_;
      cv_.notify_all();
    }
  });
}

TaskLane::~TaskLane() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
    cv_.notify_all();
  }
  th_.join();
}

uint64_t TaskLane::post(std::function<void()> fn) {
  std::lock_guard<std::mutex> g(mu_);
  q_.push_back(std::move(fn));
  cv_.notify_all();
  return ++posted_;
}

void TaskLane::wait_all() {
  uint64_t id;
  {
    std::lock_guard<std::mutex> g(mu_);
    id = posted_;
  }
  wait(id);
}

void TaskLane::wait(uint64_t id) {
  std::unique_lock<std::mutex> lk(mu_);
  cv_.wait(lk, [&]() { return done_ >= id; });
  if (!err_.empty()) {
    const std::string e = err_;
    err_.clear();
    throw std::runtime_error(e);
  }
}

uint64_t Engine::post_out(std::function<void()> fn) {
  std::lock_guard<std::mutex> g(out_mu_);
  out_q_.push_back(std::move(fn));
  const uint64_t id = ++out_posted_;
  out_cv_.notify_all();
  return id;
}

uint64_t Engine::post_rel(std::function<void()> fn) {
  if (!rel_lane_on_) return post_out(std::move(fn));
  if (!rel_lane_) {
    rel_lane_.reset(new TaskLane());
    HIP_OK(hipStreamCreateWithFlags(&rel_stream_, hipStreamNonBlocking));
  }
  return rel_lane_->post(std::move(fn));
}

void Engine::rel_wait(uint64_t task) {
  if (!rel_lane_on_) { out_wait(task); return; }
  if (rel_lane_ && task) rel_lane_->wait(task);
}

void Engine::out_wait(uint64_t task) {
  std::unique_lock<std::mutex> lk(out_mu_);
  out_cv_.wait(lk, [&]() { return out_done_ >= task; });
}

void Engine::out_wait_idle() {
  if (rel_lane_) rel_lane_->wait_all();
  std::unique_lock<std::mutex> lk(out_mu_);
  out_cv_.wait(lk, [&]() { return out_done_ >= out_posted_; });
}

// Released tx lines, in pool (endTs) order, gathered from the zero-copy line blocks.
void Engine::release_gather(int k, int64_t released) {
  HIP_OK(hipEventSynchronize(ev_rel_[k]));
  const int64_t* gids = h_release_gid_[k];
  std::string& out = blob_[OUT_DB];
  uint32_t cur_id = UINT32_MAX;
  LineBlock* cur = nullptr;
  // Released lines arrive in endTs order, so consecutive ones hop between the blocks of every
  // shard and batch still pending (32 shards x ~20 batches for the firehose shard).  A
  // direct-mapped cache of block pointers keeps the locked map lookup to once per block per
  // release instead of once per line (60k lock + find per batch made this lane the bottleneck).
  struct BlockSlot { uint32_t id = UINT32_MAX; LineBlock* b = nullptr; };
  std::vector<BlockSlot> cache(1024);
  for (int64_t i = 0; i < released; ++i) {
    const uint64_t g = (uint64_t)gids[i];
    const uint32_t id = (uint32_t)(g >> 44);
    if (id != cur_id) {
      BlockSlot& sl = cache[id & 1023u];
      if (sl.id != id) {
        std::lock_guard<std::mutex> lk(blocks_mu_);
        auto it = line_blocks_.find(id);
        sl.b = it == line_blocks_.end() ? nullptr : &it->second;  // element references survive rehash
        sl.id = id;
      }
      cur = sl.b;
      cur_id = id;
    }
    if (!cur) continue;
    const size_t off = (size_t)((g >> 12) & 0xffffffffu);
    size_t len = (size_t)(g & 0xfff);
    if (len == 4095) len = cur->data.find('\n', off) - off;  // long line: scan to its end
    out.append(cur->data, off, len + 1);  // the arena stores each line with its '\n'
    if (--cur->live == 0) {
      std::string data;
      {
        std::lock_guard<std::mutex> lk(blocks_mu_);
        data.swap(cur->data);
        line_blocks_.erase(cur_id);
      }
      recycle_arena(std::move(data));
      cache[cur_id & 1023u] = BlockSlot{};
      cur = nullptr;
      cur_id = UINT32_MAX;
    }
  }
  drain_kind(OUT_DB);
}

// The per-batch tx staging (host pinned + device) doubles instead of failing the batch; the
// `keep` tx already staged are carried over.  Runs on the stats thread between batches' copies.
void Engine::grow_tx_capacity(uint32_t need, uint32_t keep) {
  int64_t cap = std::max<int64_t>(cfg_.max_tx_per_batch, 1024);
  while (cap < (int64_t)need) cap *= 2;
  HIP_OK(hipStreamSynchronize(stream_));  // no copy / kernel still reads the old buffers
  TxRec* h_tx = nullptr;
  int64_t* h_gid = nullptr;
  HIP_OK(hipHostMalloc((void**)&h_tx, (size_t)cap * sizeof(TxRec), hipHostMallocDefault));
  HIP_OK(hipHostMalloc((void**)&h_gid, (size_t)cap * 8, hipHostMallocDefault));
  std::memcpy(h_tx, h_tx_, (size_t)keep * sizeof(TxRec));
  std::memcpy(h_gid, h_gid_, (size_t)keep * 8);
  hipHostFree(h_tx_);
  hipHostFree(h_gid_);
  h_tx_ = h_tx;
  h_gid_ = h_gid;
  dfree(d_tx_);
  dfree(d_gid_);
  d_tx_ = (TxRec*)dmalloc((size_t)cap * sizeof(TxRec));
  d_gid_ = (int64_t*)dmalloc((size_t)cap * 8);
  if (cap > std::max<int64_t>(ord_cap_, 0)) {
    dfree(d_ord_list_);
    d_ord_list_ = (int32_t*)dmalloc((size_t)cap * 4);
    ord_cap_ = cap;
  }
  cfg_.max_tx_per_batch = (int32_t)cap;
  ++metrics_.tx_capacity_grows;
}

StatsState Engine::stats_state() const {
  StatsState st{d_counts_cells_, d_cells_, d_spill_n_, d_spill_series_, d_spill_val_, d_active_,
                cfg_.cell_cap, cfg_.spill_cap, cfg_.max_series};
  st.spill_drop = d_spill_drop_;
  st.nan_until = d_nan_until_;
  st.ord_list = d_ord_list_;
  st.ord_n = d_ord_n_;
  st.ord_done = (uint32_t*)(d_ord_n_ + 1);
  st.keep = (int32_t)(cfg_.window + cfg_.buffer);
  st.spill_snap = hd_spill_snap_;
  st.nslot = nslot_;
  return st;
}

// ---- spill sizing: the reference window is unbounded (stream_calc_stats.js:127-131), so an
// append never starts unless every live slot's list can take all of its samples.
void Engine::spill_reserve(uint32_t n) {
  if (n == 0) return;
  // newest completed snapshot (the K7 kernel wrote h_spill_snap_ at or after that point; the
  // values only grow until a clear, and clears after the mark are handled by spill_clear_at_)
  const SpillMark* mk = nullptr;
  for (int i = 0; i < kSpillMarks; ++i) {
    const SpillMark& m = spill_mark_[(spill_mark_k_ + kSpillMarks - 1 - i) % kSpillMarks];
    if (!m.live) continue;
    if (hipEventQuery(m.ev) == hipSuccess) { mk = &m; break; }
  }
  int64_t worst = 0;
  for (int s = 0; s < nslot_; ++s) {
    if (slot_bucket_[s] == NO_BUCKET) continue;
    int64_t b = (int64_t)(spill_added_ - spill_clear_at_[s]);
    if (mk && spill_clear_at_[s] <= mk->added) b = std::min<int64_t>(b, (int64_t)h_spill_snap_[s] + (int64_t)(spill_added_ - mk->added));
    worst = std::max(worst, b);
  }
  if (worst + (int64_t)n <= cfg_.spill_cap) return;
  // the bound is too loose: read the exact levels (stream drain, rare), then grow if needed
  spill_resync();
  worst = 0;
  for (int s = 0; s < nslot_; ++s)
    if (slot_bucket_[s] != NO_BUCKET) worst = std::max<int64_t>(worst, h_spill_snap_[s]);
  if (worst + (int64_t)n <= cfg_.spill_cap) return;
  int64_t cap = cfg_.spill_cap;
  while (worst + (int64_t)n > cap) cap *= 2;
  if (cap > INT32_MAX / nslot_) throw std::runtime_error("bucket spill lists beyond 2^31 entries");
  grow_spill((int32_t)cap);
}

// exact fill levels now (drains the stats stream): the newest snapshot, every older one retired
void Engine::spill_resync() {
  HIP_OK(hipStreamSynchronize(stream_));
  std::vector<int32_t> exact(nslot_);
  HIP_OK(hipMemcpy(exact.data(), d_spill_n_, (size_t)nslot_ * 4, hipMemcpyDeviceToHost));
  for (auto& m : spill_mark_) m.live = false;
  std::memcpy(h_spill_snap_, exact.data(), (size_t)nslot_ * 4);
  spill_mark_[0].added = spill_added_;
  spill_mark_[0].live = true;
  HIP_OK(hipEventRecord(spill_mark_[0].ev, stream_));
  HIP_OK(hipEventSynchronize(spill_mark_[0].ev));
  spill_mark_k_ = 1;
  for (int s = 0; s < nslot_; ++s) spill_clear_at_[s] = std::min(spill_clear_at_[s], spill_added_);
}

// after an append's kernels were queued: its snapshot point
void Engine::spill_marked() {
  SpillMark& m = spill_mark_[spill_mark_k_];
  m.added = spill_added_;
  m.live = true;
  HIP_OK(hipEventRecord(m.ev, stream_));
  spill_mark_k_ = (spill_mark_k_ + 1) % kSpillMarks;
}

int32_t ring_slots_for(int window, int buffer) { return std::max<int32_t>(NSLOT_MIN, window + buffer + 1); }

// The bucket ring at `nslot` slots: cells, counts, spill lists (+ their sort targets), the
// host's fill snapshot and slot table.  Fresh (every slot free).
void Engine::alloc_ring(int32_t nslot) {
  const int32_t S = cfg_.max_series;
  nslot_ = nslot;
  d_counts_cells_ = (int32_t*)dmalloc((size_t)nslot * S * 4);
  d_cells_ = (int32_t*)dmalloc((size_t)nslot * S * cfg_.cell_cap * 4);
  d_spill_n_ = (int32_t*)dmalloc((size_t)nslot * 4);
  d_spill_series_ = (int32_t*)dmalloc((size_t)nslot * cfg_.spill_cap * 4);
  d_spill_val_ = (int32_t*)dmalloc((size_t)nslot * cfg_.spill_cap * 4);
  d_spill_series_alt_ = (int32_t*)dmalloc((size_t)nslot * cfg_.spill_cap * 4);
  d_spill_val_alt_ = (int32_t*)dmalloc((size_t)nslot * cfg_.spill_cap * 4);
  spill_tmp_bytes_ = apm_spill_sort_tmp_bytes(cfg_.spill_cap, S, nslot);
  d_spill_tmp_ = dmalloc(spill_tmp_bytes_);
  d_win_slots_ = (int32_t*)dmalloc((size_t)nslot * 4);
  HIP_OK(hipHostMalloc((void**)&h_spill_snap_, (size_t)nslot * 4, hipHostMallocDefault));
  HIP_OK(hipHostGetDevicePointer((void**)&hd_spill_snap_, h_spill_snap_, 0));
  std::memset(h_spill_snap_, 0, (size_t)nslot * 4);
  slot_bucket_.assign((size_t)nslot, NO_BUCKET);
  spill_clear_at_.assign((size_t)nslot, 0);
}

// A reload to a window the ring cannot hold (stream_calc_stats.js:228-261 takes any size): the
// ring is re-made at `nslot` slots and every live bucket's cells, counts and spill list move to
// slot b % nslot.  Stats thread, between rollovers (the stream is drained first).
void Engine::grow_ring(int32_t nslot) {
  if (nslot <= nslot_) return;
  HIP_OK(hipStreamSynchronize(stream_));
  const int32_t S = cfg_.max_series, cap = cfg_.cell_cap, sc = cfg_.spill_cap;
  int32_t* o_counts = d_counts_cells_;
  int32_t* o_cells = d_cells_;
  int32_t* o_sn = d_spill_n_;
  int32_t* o_ss = d_spill_series_;
  int32_t* o_sv = d_spill_val_;
  const std::vector<int64_t> o_bucket = slot_bucket_;
  const std::vector<uint64_t> o_clear = spill_clear_at_;
  std::vector<int32_t> o_snap(h_spill_snap_, h_spill_snap_ + nslot_);
  for (void* p : {(void*)d_spill_series_alt_, (void*)d_spill_val_alt_, d_spill_tmp_, (void*)d_win_slots_}) dfree(p);
  HIP_OK(hipHostFree(h_spill_snap_));
  if (d_ck_slots_) { dfree(d_ck_slots_); d_ck_slots_ = nullptr; }  // (sized by the ring: re-made on demand)
  const int32_t o_n = nslot_;
  alloc_ring(nslot);
  for (int32_t s = 0; s < o_n; ++s) {
    const int64_t b = o_bucket[(size_t)s];
    if (b == NO_BUCKET) continue;
    const int32_t t = (int32_t)(((b % nslot) + nslot) % nslot);
    HIP_OK(hipMemcpyAsync(d_counts_cells_ + (size_t)t * S, o_counts + (size_t)s * S, (size_t)S * 4,
                          hipMemcpyDeviceToDevice, stream_));
    HIP_OK(hipMemcpyAsync(d_cells_ + (size_t)t * S * cap, o_cells + (size_t)s * S * cap, (size_t)S * cap * 4,
                          hipMemcpyDeviceToDevice, stream_));
    HIP_OK(hipMemcpyAsync(d_spill_n_ + t, o_sn + s, 4, hipMemcpyDeviceToDevice, stream_));
    HIP_OK(hipMemcpyAsync(d_spill_series_ + (size_t)t * sc, o_ss + (size_t)s * sc, (size_t)sc * 4,
                          hipMemcpyDeviceToDevice, stream_));
    HIP_OK(hipMemcpyAsync(d_spill_val_ + (size_t)t * sc, o_sv + (size_t)s * sc, (size_t)sc * 4,
                          hipMemcpyDeviceToDevice, stream_));
    slot_bucket_[(size_t)t] = b;
    spill_clear_at_[(size_t)t] = o_clear[(size_t)s];
    h_spill_snap_[t] = o_snap[(size_t)s];
  }
  HIP_OK(hipStreamSynchronize(stream_));
  for (void* p : {(void*)o_counts, (void*)o_cells, (void*)o_sn, (void*)o_ss, (void*)o_sv}) dfree(p);
  spill_resync();  // fill levels at the new slots
  ++ring_grows_;
}

// Every slot list keeps its entries at the same positions of a longer row.
void Engine::grow_spill(int32_t cap) {
  resize_spill(cap);
  ++metrics_.spill_grows;
}

void Engine::resize_spill(int32_t cap) {
  HIP_OK(hipStreamSynchronize(stream_));
  const size_t old = (size_t)cfg_.spill_cap;
  const size_t w = std::min(old, (size_t)cap) * 4;  // (a shrink keeps every slot's fill: cap >= it)
  int32_t* ser = (int32_t*)dmalloc((size_t)nslot_ * cap * 4);
  int32_t* val = (int32_t*)dmalloc((size_t)nslot_ * cap * 4);
  HIP_OK(hipMemcpy2DAsync(ser, (size_t)cap * 4, d_spill_series_, old * 4, w, nslot_, hipMemcpyDeviceToDevice, stream_));
  HIP_OK(hipMemcpy2DAsync(val, (size_t)cap * 4, d_spill_val_, old * 4, w, nslot_, hipMemcpyDeviceToDevice, stream_));
  HIP_OK(hipStreamSynchronize(stream_));
  dfree(d_spill_series_);
  dfree(d_spill_val_);
  dfree(d_spill_series_alt_);
  dfree(d_spill_val_alt_);
  dfree(d_spill_tmp_);
  d_spill_series_ = ser;
  d_spill_val_ = val;
  d_spill_series_alt_ = (int32_t*)dmalloc((size_t)nslot_ * cap * 4);
  d_spill_val_alt_ = (int32_t*)dmalloc((size_t)nslot_ * cap * 4);
  cfg_.spill_cap = cap;
  spill_tmp_bytes_ = apm_spill_sort_tmp_bytes(cfg_.spill_cap, cfg_.max_series, nslot_);
  d_spill_tmp_ = dmalloc(spill_tmp_bytes_);
  metrics_.spill_capacity = cap;
}

std::pair<size_t, size_t> Engine::trim_device_memory() {
  checkpoint_wait();  // the writer reads the staging buffer
  flush();            // the stats thread, rollover lane and output lane idle
  const size_t before = device_bytes();
  HIP_OK(hipStreamSynchronize(stream_));
  if (dj_) dj_->trim(watermark_);
  // spill lists: back to max(configured, 2x the fullest slot)
  {
    std::vector<int32_t> fill(nslot_);
    HIP_OK(hipMemcpy(fill.data(), d_spill_n_, (size_t)nslot_ * 4, hipMemcpyDeviceToHost));
    int32_t mx = 0;
    for (int32_t f : fill) mx = std::max(mx, std::min(f, cfg_.spill_cap));
    const int32_t want = std::max<int32_t>(init_spill_cap_, ((2 * mx + 1023) / 1024) * 1024);
    if (want < cfg_.spill_cap) resize_spill(want);
  }
  // checkpoint packing scratch and the incremental checkpoint's staging (re-made by the next one;
  // a staging allocation that then fails falls back to the synchronous writer)
  for (void** q : {(void**)&d_ck_lens_, (void**)&d_ck_offs_, (void**)&d_ck_packed_, &d_ck_ptmp_}) {
    dfree(*q);
    *q = nullptr;
  }
  ck_pack_n_ = 0;
  ck_ptmp_bytes_ = 0;
  for (int k = 0; k < 2; ++k) {
    dfree(d_ck_text_[k]);
    d_ck_text_[k] = nullptr;
    ck_text_cap_[k] = 0;
  }
  dfree(d_ck_gids_);
  d_ck_gids_ = nullptr;
  ck_gids_cap_ = 0;
  // the snapshot staging is kept at what the last snapshot needed (re-allocating it at the next
  // checkpoint would stall that checkpoint and put HBM back over the threshold): freed only when
  // it is more than twice that
  if (ck_stage_bytes_ > 2 * ck_last_need_) free_ck_stage();
  if (d_ck_defer_ && ck_defer_cap_ > 2 * std::max<size_t>(ck_defer_want_, (size_t)1 << 30)) {
    // the deferred small-section staging (the writer is idle: checkpoint_wait)
    HIP_OK(hipFree(d_ck_defer_));
    d_ck_defer_ = nullptr;
    std::lock_guard<std::mutex> g(alloc_mu_);
    device_bytes_ -= ck_defer_cap_;
    ck_defer_cap_ = 0;
  }
  HIP_OK(hipStreamSynchronize(stream_));
  return {before, device_bytes()};
}

// before K8: each slot's list sorted by series (stable), the live and sort buffers swapped
void Engine::spill_sort() {
  StatsState st = stats_state();
  if (apm_spill_sort(&st, d_spill_series_alt_, d_spill_val_alt_, d_spill_tmp_, spill_tmp_bytes_, stream_) != 0)
    throw std::runtime_error("spill sort scratch too small");
  std::swap(d_spill_series_, d_spill_series_alt_);
  std::swap(d_spill_val_, d_spill_val_alt_);
}

void Engine::ensure_bucket_slot(int64_t b) {
  const int slot = (int)(((b % nslot_) + nslot_) % nslot_);
  if (slot_bucket_[slot] == b) return;
  if (slot_bucket_[slot] != NO_BUCKET) {
    StatsState st = stats_state();
    apm_stats_clear_slot(&st, slot, stream_);
  }
  spill_clear_at_[slot] = spill_added_;
  slot_bucket_[slot] = b;
}

void Engine::stats_for_batch(std::vector<TxOut>& txs, double batch_t0) {
  const double ts0 = now_ms();
  const int32_t n_series_at_start = n_series_;
  const int64_t latest_at_start = latest_;
  const bool w_tx = want(OUT_TRANSACTIONS), w_audit = want(OUT_AUDIT_DB), w_db = want(OUT_DB);
  std::vector<std::string>& text = *cur_text_;
  // Each shard's text arena of this batch becomes a release block (zero copy): the pool payload
  // of a pending tx addresses its line inside the arena, gid = block << 44 | offset << 12 | len.
  const size_t n_arena = text.size();
  std::vector<uint32_t> blk_id(n_arena, 0);
  std::vector<int64_t> blk_live(n_arena, 0);
  if (w_db)
    for (size_t a = 0; a < n_arena; ++a) blk_id[a] = (line_block_seq_++) & 0xFFFFFu;
  // split: audit non-Provider records go straight to db_insert (Q18)
  std::vector<std::pair<uint32_t, int64_t>> triggers;  // (index in upload, new latest)
  uint32_t n = 0;
  int64_t agg_b = INT64_MIN, agg_n = 0, agg_e = 0;
  for (uint32_t i = 0; i < txs.size(); ++i) {
    TxOut& t = txs[i];
    ++metrics_.tx;
    if (t.to_db) {
      ++metrics_.tx_db;
      if (w_audit) {
        blob_[OUT_AUDIT_DB].append(text[t.server], t.line_off, t.line_len + 1);  // with its '\n'
      }
      continue;
    }
    if (w_tx) {
      blob_[OUT_TRANSACTIONS].append(text[t.server], t.line_off, t.line_len + 1);
    }
    // NaN / short endTs would wedge the reference's heap forever: dropped and counted (fix)
    if (!(t.end_ms == t.end_ms) || t.end_ms < 10000) { ++metrics_.tx_dropped; continue; }
    const int64_t end = (int64_t)t.end_ms;
    const int64_t b = end / 10000;
    // a tx with a newer bucket triggers the rollover *before* it is added (:348-370)
    if (b > latest_) { triggers.push_back({n, b}); latest_ = b; }
    if (n >= (uint32_t)cfg_.max_tx_per_batch) grow_tx_capacity(n + 1, n);  // e.g. a burst of need-cache expiries
    int32_t s;
    {
      if ((size_t)t.server >= ser_raw_.size()) ser_raw_.resize((size_t)t.server + 1);
      auto& row = ser_raw_[t.server];
      if ((size_t)t.raw_svc >= row.size()) row.resize(std::max<size_t>((size_t)t.raw_svc + 1, row.size() * 2), -1);
      s = row[t.raw_svc];
      if (s < 0) {
        s = series_for(t.server, t.service);
        row[t.raw_svc] = s;  // -1 (series table full) stays uncached
      }
    }
    TxRec r;
    r.end_ms = end;
    r.series = s;
    const double e = t.elapsed;
    r.elapsed = (e == e && e >= -2147483647.0 && e <= 2147483647.0) ? (int32_t)e : ELAPSED_NAN;
    h_tx_[n] = r;
    int64_t gid = next_gid_++;
    if (w_db) {
      gid = (int64_t)(((uint64_t)blk_id[t.server] << 44) | ((uint64_t)t.line_off << 12) |
                      (uint64_t)std::min<uint32_t>(t.line_len, 4095));
      ++blk_live[t.server];
    }
    h_gid_[n] = gid;
    if (b != agg_b) { if (agg_n) { pool_bucket_count_[agg_b] += agg_n; pool_exact_edge_[agg_b] += agg_e; } agg_b = b; agg_n = agg_e = 0; }
    ++agg_n;
    if (end == b * 10000) ++agg_e;
    ++n;
  }
  if (agg_n) { pool_bucket_count_[agg_b] += agg_n; pool_exact_edge_[agg_b] += agg_e; }
  if (n_series_ > n_series_at_start && !cfg_.emulate_aliasing) upload_series_tables(n_series_at_start);
  for (size_t a = 0; a < n_arena; ++a)
    if (blk_live[a] > 0) {
      std::lock_guard<std::mutex> lk(blocks_mu_);
      if (line_blocks_.count(blk_id[a])) throw std::runtime_error("release block id wrapped while still live");
      LineBlock& b = line_blocks_[blk_id[a]];
      b.data.swap(text[a]);  // the arena moves into the block; the job keeps an empty string
      b.live = blk_live[a];
    }
  for (auto it = pool_exact_edge_.begin(); it != pool_exact_edge_.end();) {
    if (it->second == 0) it = pool_exact_edge_.erase(it); else ++it;
  }
  metrics_.t_stats_tx_ms += now_ms() - ts0;
  trace_event("tx loop", ts0, now_ms(), 1);
  if (n == 0) return;
  HIP_OK(hipMemcpyAsync(d_tx_, h_tx_, (size_t)n * sizeof(TxRec), hipMemcpyHostToDevice, stream_));
  HIP_OK(hipMemcpyAsync(d_gid_, h_gid_, (size_t)n * 8, hipMemcpyHostToDevice, stream_));
  {
    StatsState st = stats_state();
    apm_nan_mark(d_tx_, n, &st, stream_);
  }
  const int64_t keep_iv = cfg_.window + cfg_.buffer;
  auto append = [&](uint32_t lo, uint32_t hi, int64_t lat) {
    if (hi <= lo) return;
    const int64_t min_live = lat - keep_iv;
    int64_t seen[8];
    int nseen = 0;
    for (uint32_t i = lo; i < hi; ++i) {
      const TxRec& r = h_tx_[i];
      if (r.series >= 0 && r.series < (int32_t)h_active_.size()) h_active_[r.series] = 1;
      const int64_t b = r.end_ms / 10000;
      if (b < min_live) continue;
      bool dup = false;
      for (int k = 0; k < nseen; ++k) dup |= seen[k] == b;
      if (dup) continue;
      ensure_bucket_slot(b);
      if (nseen < 8) seen[nseen++] = b;
    }
    spill_reserve(hi - lo);
    StatsState st = stats_state();
    apm_bucket_append(d_tx_, lo, hi, &st, min_live, stream_);
    spill_added_ += hi - lo;
    spill_marked();
    apm_pool_append(d_tx_, lo, hi, d_gid_, d_tail_end_, d_tail_gid_, tail_n_, stream_);
    tail_n_ += hi - lo;
  };
  uint32_t seg_lo = 0;
  int64_t cur_latest = latest_at_start;
  for (auto& tr : triggers) {
    append(seg_lo, tr.first, cur_latest);
    do_rollover(tr.second, batch_t0);
    cur_latest = tr.second;
    seg_lo = tr.first;
  }
  append(seg_lo, n, cur_latest);
}

// Device join: the batch's tx are already on the GPU (TxRec / raw service id / ring gid in the
// join slot, in single-stream order).  The host only resolves series for raw services seen for the
// first time (first-appearance order = the reference's object insertion order) and splits the
// batch at the rollover triggers.
void Engine::stats_for_batch_dev(DevJoinBatch& b, double batch_t0) {
  const double ts0 = now_ms();
  cur_dj_ = &b;
  metrics_.tx += b.n_out;
  metrics_.tx_db += b.n_db;
  metrics_.tx_dropped += b.n_dropped;
  if (want(OUT_TRANSACTIONS)) blob_[OUT_TRANSACTIONS] += b.text_tx;
  if (want(OUT_AUDIT_DB)) blob_[OUT_AUDIT_DB] += b.text_db;
  if (!b.unresolved.empty()) {
    const int32_t n_before = n_series_;
    std::vector<std::pair<int32_t, int32_t>> upd;
    for (const auto& u : b.unresolved) {
      const int32_t raw = u.second;
      if ((size_t)raw >= h_raw_series_.size()) h_raw_series_.resize((size_t)raw + 1, -1);
      if (h_raw_series_[raw] >= 0) continue;  // resolved meanwhile (the join read a stale -1)
      const int32_t sr = series_for(dj_->raw_server(raw), dj_->raw_service(raw));
      if (sr >= 0) { h_raw_series_[raw] = sr; upd.push_back({raw, sr}); }
    }
    if (!upd.empty()) {
      int32_t* hp = pinned_pairs(upd.size() * 2);
      for (size_t i = 0; i < upd.size(); ++i) { hp[2 * i] = upd[i].first; hp[2 * i + 1] = upd[i].second; }
      h2d(d_pairs_, hp, upd.size() * 8, stream_);
      pinned_pairs_done();
      apm_dj_scatter_i32(dj_->d_raw_series(), d_pairs_, (uint32_t)upd.size(), stream_);
    }
    apm_dj_fill_series(b.d_tx, b.d_raw, b.n_stats, dj_->d_raw_series(), d_unmapped_, stream_);
    if (n_series_ > n_before && !cfg_.emulate_aliasing) upload_series_tables(n_before);
  }
  const int64_t latest_at_start = latest_;
  std::vector<std::pair<uint32_t, int64_t>> triggers;  // a tx with a newer bucket rolls over first
  for (const auto& c : b.cands)
    if (c.second > latest_) { triggers.push_back(c); latest_ = c.second; }
  metrics_.t_stats_tx_ms += now_ms() - ts0;
  trace_event("tx loop", ts0, now_ms(), 1);
  {
    StatsState st = stats_state();
    apm_nan_mark(b.d_tx, b.n_stats, &st, stream_);
  }
  const int64_t keep_iv = cfg_.window + cfg_.buffer;
  auto append = [&](uint32_t lo, uint32_t hi, int64_t lat) {
    if (hi <= lo) return;
    const double ta = now_ms();
    struct Span { Engine* e; double t; ~Span() { e->trace_event("st.append", t, now_ms(), 1); } } span{this, ta};
    const int64_t min_live = lat - keep_iv;
    // every live bucket slot is (re)bound: a slot still holding a bucket older than the window is
    // cleared exactly as the first tx of a new bucket would clear it
    for (int64_t bk = min_live; bk <= lat; ++bk) ensure_bucket_slot(bk);
    if (tail_n_ + (int64_t)(hi - lo) > cfg_.pool_cap) throw std::runtime_error("release pool overflow");
    spill_reserve(hi - lo);
    StatsState st = stats_state();
    apm_bucket_append(b.d_tx, lo, hi, &st, min_live, stream_);
    spill_added_ += hi - lo;
    spill_marked();
    apm_pool_append(b.d_tx, lo, hi, b.d_gid, d_tail_end_, d_tail_gid_, tail_n_, stream_);
    tail_n_ += hi - lo;
  };
  uint32_t seg_lo = 0;
  int64_t cur_latest = latest_at_start;
  for (auto& tr : triggers) {
    append(seg_lo, tr.first, cur_latest);
    do_rollover(tr.second, batch_t0);
    cur_latest = tr.second;
    seg_lo = tr.first;
  }
  append(seg_lo, b.n_stats, cur_latest);
  const double trs = now_ms();
  dj_->release_slot(b.slot, stream_);
  trace_event("st.release_slot", trs, now_ms(), 1);
  cur_dj_ = nullptr;
}

// Small per-batch transfers between device memory and pinned (hipHostMalloc) host buffers run
// as kernel copies over the host link (apm_copy): hipMemcpyAsync of a few KB from pinned memory
// held the calling thread for up to 0.6 ms on this pool (trace span u.hops.h2d), a launch never
// does.  Bulk transfers (batch bytes, st/fs text) stay on the DMA engines.
void Engine::h2d(void* d, const void* h, size_t n, hipStream_t s) {
  if (n == 0) return;
  void* hv = nullptr;
  HIP_OK(hipHostGetDevicePointer(&hv, const_cast<void*>(h), 0));
  apm_copy(d, hv, n, s);
}

void Engine::lane_d2h(void* h, const void* d, size_t n, hipStream_t s) {
  if (!n) return;
  if (s && s != out_stream_) {  // the release lane's stream: one blit copy
    HIP_OK(hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, s));
    return;
  }
  if (d2h_split_ > 1 && n >= ((size_t)4 << 20)) {
    // APM_D2H_SPLIT=N: N pieces over two streams, so two copies run at once on the host link
    if (!out_stream2_) HIP_OK(hipStreamCreateWithFlags(&out_stream2_, hipStreamNonBlocking));
    const size_t piece = ((n + d2h_split_ - 1) / d2h_split_ + 4095) & ~(size_t)4095;
    int i = 0;
    for (size_t off = 0; off < n; off += piece, ++i) {
      const size_t m = std::min(piece, n - off);
      HIP_OK(hipMemcpyAsync((char*)h + off, (const char*)d + off, m, hipMemcpyDeviceToHost,
                            (i & 1) ? out_stream2_ : out_stream_));
    }
    return;
  }
  if (d2h_kernel_) {
    void* hv = nullptr;
    HIP_OK(hipHostGetDevicePointer(&hv, h, 0));
    apm_copy_capped(hv, d, n, d2h_blocks_, out_stream_);
  } else if (d2h_sdma_) {  // a copy engine instead of ROCclr's blit kernel (A/B)
    HIP_OK(hipMemcpyAsync(h, d, n, hipMemcpyDeviceToDeviceNoCU, out_stream_));
  } else {
    HIP_OK(hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, out_stream_));
  }
}

void Engine::lane_sync() {
  HIP_OK(hipStreamSynchronize(out_stream_));
  if (out_stream2_) HIP_OK(hipStreamSynchronize(out_stream2_));
}

void Engine::d2h(void* h, const void* d, size_t n, hipStream_t s) {
  if (n == 0) return;
  void* hv = nullptr;
  HIP_OK(hipHostGetDevicePointer(&hv, h, 0));
  apm_copy(hv, d, n, s);
}

// Pinned staging for the stats thread's small H2D uploads (raw -> series pairs, unseen series
// ids): two buffers used alternately, each reused only after its previous copy completed, so
// the upload never waits for the whole stats stream.
char* Engine::stage(size_t bytes) {
  const int k = stage_k_;
  if (stage_ev_[k]) HIP_OK(hipEventSynchronize(stage_ev_[k]));
  else HIP_OK(hipEventCreateWithFlags(&stage_ev_[k], hipEventDisableTiming));
  if (bytes > h_stage_cap_[k]) {
    // slots rotate over uploads of very different sizes (80k-series permutation vs a JMX row):
    // grow each to the largest request seen so far, so the ring stops reallocating (a pinned
    // free + alloc costs ~1 ms) after one pass instead of after every slot met every size
    stage_max_ = std::max(stage_max_, bytes);
    if (h_stage_[k]) HIP_OK(hipHostFree(h_stage_[k]));
    h_stage_cap_[k] = std::max<size_t>(stage_max_ * 2, 1 << 20);
    HIP_OK(hipHostMalloc((void**)&h_stage_[k], h_stage_cap_[k], hipHostMallocDefault));
  }
  return h_stage_[k];
}

void Engine::stage_done() {
  HIP_OK(hipEventRecord(stage_ev_[stage_k_], stream_));
  stage_k_ = (stage_k_ + 1) % kStage;
}

int32_t* Engine::pinned_pairs(size_t n_ints) {
  if (n_ints * 4 > pairs_bytes_) d_pairs_ = (int32_t*)regrow(d_pairs_, pairs_bytes_, n_ints * 8 + 65536);
  return (int32_t*)stage(n_ints * 4);
}

// K8 needs the z-score settings of series that became visible before this rollover: with the
// device join the host never sees individual tx, so the `active` flags of the still-unseen series
// are read back (only while the series set grows).
void Engine::refresh_unseen_active() {
  if (unseen_.empty()) return;
  const uint32_t n = (uint32_t)unseen_.size();
  int32_t* hp = pinned_pairs(n);
  std::memcpy(hp, unseen_.data(), (size_t)n * 4);
  h2d(d_unseen_idx_, hp, (size_t)n * 4, stream_);
  pinned_pairs_done();
  apm_dj_gather_u8(d_active_, d_unseen_idx_, n, d_unseen_flag_, stream_);
  d2h(h_unseen_flag_, d_unseen_flag_, n, stream_);
  HIP_OK(hipStreamSynchronize(stream_));
  for (uint32_t i = 0; i < n; ++i)
    if (h_unseen_flag_[i]) h_active_[unseen_[i]] = 1;
}

void Engine::do_rollover(int64_t L, double batch_t0) {
  finish_rollover();  // a previous rollover of this job still owns the candidate buffers
  const int64_t keep_iv = cfg_.window + cfg_.buffer;
  // the decision's clock, fixed before K11 so its cooldown pre-filter and the host decide alike
  roll_now_ = cfg_.alert_clock_entry ? (double)((L - cfg_.buffer - 1) * 10000)
                                     : (double)std::chrono::duration_cast<std::chrono::milliseconds>(
                                           std::chrono::system_clock::now().time_since_epoch()).count();
  ++metrics_.rollovers;
  // removeOldBuckets(36): drop every bucket < L - 36
  for (int i = 0; i < nslot_; ++i) {
    if (slot_bucket_[i] != NO_BUCKET && slot_bucket_[i] < L - keep_iv) {
      StatsState st = stats_state();
      apm_stats_clear_slot(&st, i, stream_);
      slot_bucket_[i] = NO_BUCKET;
      spill_clear_at_[i] = spill_added_;
    }
  }
  const int64_t edge_ts = (L - cfg_.buffer - 1) * 10000;
  last_edge_ts_ = edge_ts;
  const double tr0 = now_ms();
  // ---- K9 release: merge the sorted pool with the sorted tail, hand out endTs <= edge (the
  // device form is queued after K8-K11 and the alert gather, below: the alert candidates do not
  // wait for it on the stream)
  if (dev()) {
  } else {
    int64_t released = 0;
    for (auto it = pool_bucket_count_.begin(); it != pool_bucket_count_.end();) {
      if (it->first * 10000 + 9999 <= edge_ts) { released += it->second; it = pool_bucket_count_.erase(it); }
      else break;
    }
    const int64_t eb = edge_ts / 10000;
    auto ex = pool_exact_edge_.find(eb);
    if (ex != pool_exact_edge_.end()) {
      released += ex->second;
      pool_bucket_count_[eb] -= ex->second;
      if (pool_bucket_count_[eb] == 0) pool_bucket_count_.erase(eb);
      pool_exact_edge_.erase(ex);
    }
    for (auto it = pool_exact_edge_.begin(); it != pool_exact_edge_.end();) {
      if (it->first < eb) it = pool_exact_edge_.erase(it); else break;
    }
    const int nxt = pool_cur_ ^ 1;
    if (pool_n_ + tail_n_ > cfg_.pool_cap) throw std::runtime_error("release pool overflow");
    if (apm_release_merge(d_pool_end_[pool_cur_] + pool_off_, d_pool_gid_[pool_cur_] + pool_off_, pool_n_,
                          d_tail_end_, d_tail_gid_, tail_n_, d_sort_end_, d_sort_gid_, d_pool_end_[nxt],
                          d_pool_gid_[nxt], d_release_tmp_, release_tmp_bytes_, stream_) != 0)
      throw std::runtime_error("release tmp too small");
    pool_cur_ = nxt;
    pool_n_ = pool_n_ + tail_n_;
    tail_n_ = 0;
    if (released > pool_n_) released = pool_n_;
    if (want(OUT_DB) && released > 0) {
      // the D2H of the released ids is queued behind the merge; the output lane waits for it and
      // gathers the lines while this thread continues with K8/K10/K11
      const int k = rel_k_;
      rel_k_ ^= 1;
      rel_wait(rel_task_[k]);  // the buffer's previous reader is done
      HIP_OK(hipMemcpyAsync(h_release_gid_[k], d_pool_gid_[pool_cur_], (size_t)released * 8, hipMemcpyDeviceToHost,
                            stream_));
      HIP_OK(hipEventRecord(ev_rel_[k], stream_));
      rel_task_[k] = post_rel([this, k, released]() { release_gather(k, released); });
    }
    metrics_.released += released;
    pool_off_ = released;
    pool_n_ -= released;
    // the remaining pool now starts at pool_off_ inside the current buffer
  }
  const double tr1 = now_ms();
  metrics_.t_release_ms += tr1 - tr0;
  // ---- first st for newly visible series: resolve their z-score settings in emission order
  if (dev()) refresh_unseen_active();
  const double tu = now_ms();
  trace_event("ro.unseen", tr1, tu, 1);
  {
    std::vector<int32_t> fresh;
    std::vector<int32_t> still;
    for (int32_t s : unseen_) { if (h_active_[s]) fresh.push_back(s); else still.push_back(s); }
    unseen_.swap(still);
    // a series is visible iff it had a tx before this rollover: all created series qualify except
    // those whose first tx is the trigger or later -- the device `active` flag is authoritative;
    // settings for not-yet-active series are computed now and harmlessly recomputed later.
    std::sort(fresh.begin(), fresh.end(), [&](int32_t a, int32_t b) { return series_[a].emit_key < series_[b].emit_key; });
    if (!fresh.empty()) {
      int32_t lo = INT32_MAX;
      for (int32_t s : fresh) {
        zscore_seen_[s] = 1;
        apply_series_settings(s);
        lo = std::min(lo, s);
      }
      upload_series_tables(lo);
    }
  }
  const double tsp = now_ms();
  trace_event("ro.fresh", tu, tsp, 1);
  // ---- K8 window statistics over buckets [L-36, L-6]
  spill_sort();
  trace_event("ro.spill_sort", tsp, now_ms(), 1);
  WindowArgs wa;
  wa.st = stats_state();
  wa.n_win = (int32_t)(keep_iv - cfg_.buffer + 1);
  wa.win_slots_ext = nullptr;
  {
    std::vector<int32_t> ws((size_t)std::max<int32_t>(wa.n_win, K8_INLINE_SLOTS), -1);
    for (int r = 0; r < wa.n_win; ++r) {
      const int64_t b = L - keep_iv + r;
      const int slot = (int)(((b % nslot_) + nslot_) % nslot_);
      ws[(size_t)r] = slot_bucket_[slot] == b ? slot : -1;
    }
    for (int r = 0; r < K8_INLINE_SLOTS; ++r) wa.win_slots[r] = ws[(size_t)r];
    if (wa.n_win > K8_INLINE_SLOTS) {
      // a window longer than the argument block (> 10 min): the whole slot list from a device
      // array, rewritten once the previous rollover's K8 (the array's last reader) has finished
      HIP_OK(hipStreamSynchronize(stream_));
      HIP_OK(hipMemcpy(d_win_slots_, ws.data(), (size_t)wa.n_win * 4, hipMemcpyHostToDevice));
      wa.win_slots_ext = d_win_slots_;
    }
  }
  wa.tpm_div = (double)cfg_.window * cfg_.interval_len / 60.0;
  {
    // APM_K8_LDS=1: the LDS bitonic for every window; =2: only the two-series kernel's windows
    // of 33-512 samples (A/B of its register network)
    static const int lds = [] { const char* e = std::getenv("APM_K8_LDS"); return e && (e[0] == '1' || e[0] == '2') ? e[0] - '0' : 0; }();
    wa.lds_sort = lds;
  }
  wa.out = d_win_;
  wa.big_list = d_big_list_;
  wa.big_n = d_big_n_;
  wa.nan_list = d_nan_list_;
  wa.nan_n = d_nan_n_;
  wa.js_scratch = d_js_scratch_;
  wa.js_cap = kJsCap;
  wa.n_series = n_series_;
  HIP_OK(hipMemsetAsync(d_big_n_, 0, 12, stream_));  // big / nan windows, alert candidates
  apm_window_stats(&wa, stream_);
  // ---- K10 z-score per LAG, K11 alert eval (a streamed checkpoint's rows first: copy-before-overwrite)
  ck_guard_rollover(rollover_idx_);
  for (int l = 0; l < cfg_.n_lags; ++l) {
    LagState& LS = lag_[l];
    ZArgs za;
    za.ring = LS.ring; za.len = LS.len; za.sum = LS.sum; za.comp = LS.comp; za.cnt = LS.cnt;
    za.sumsq = LS.sumsq; za.sqcomp = LS.sqcomp; za.thr = LS.thr; za.infl = LS.infl; za.win = d_win_;
    za.out = LS.out; za.S = cfg_.max_series; za.n_series = n_series_; za.lag = cfg_.lags[l];
    za.head = (int32_t)(rollover_idx_ % cfg_.lags[l]);
    za.exact = cfg_.exact_mean; za.sigma_stddev = cfg_.sigma_stddev; za.resync_k = cfg_.resync_k;
    za.rollover_idx = rollover_idx_;
    za.rs_lo = 0; za.rs_n = 0; za.rs_parts = RS_PARTS; za.rs_part = rs_part_; za.rs_cnt = rs_cnt_;
    za.rs_mfma = cfg_.resync_mfma ? 1 : 0;
    if (rs_range_ > 0) {
      za.rs_lo = (int32_t)((rollover_idx_ % cfg_.resync_k) * rs_range_);
      za.rs_n = std::max(0, std::min(rs_range_, n_series_ - za.rs_lo));
    }
    apm_zscore(&za, cfg_.ring_bytes, stream_);
    AlertArgs aa;
    aa.win = d_win_; aa.z = LS.out; aa.counter = LS.counter; aa.hard_max = d_hard_max_;
    aa.suppressed = d_suppressed_; aa.emit_key = d_emit_key_; aa.out = d_alerts_; aa.n_out = d_n_alerts_;
    aa.n_series = n_series_; aa.lag_idx = l; aa.n_lags = cfg_.n_lags; aa.lag_suppressed = cfg_.lag_suppressed[l];
    aa.window = cfg_.alert_window; aa.threshold = cfg_.alert_threshold; aa.hard_min_ms = cfg_.hard_min_ms;
    aa.hard_min_tpm = cfg_.hard_min_tpm; aa.both_only = cfg_.both_only; aa.max_out = cfg_.max_alerts;
    aa.cool_t = d_cool_t_; aa.now = roll_now_; aa.cool_s = cfg_.cooldown_ms / 1000.0;
    apm_alert_eval(&aa, stream_);
  }
  ++rollover_idx_;
  if (want(OUT_SX)) server_rollup(edge_ts);
  // the candidates go straight to pinned host memory; the st/fs formatting is queued behind them
  // and runs on the GPU while this thread waits for the candidates only and decides the alerts
  {
    const ZOut* zl[MAX_LAGS] = {};
    for (int l = 0; l < cfg_.n_lags; ++l) zl[l] = lag_[l].out;
    apm_alert_gather(d_alerts_, d_n_alerts_, cfg_.max_alerts, d_win_, zl, cfg_.n_lags, want(OUT_AL) ? 1 : 0,
                     hd_alerts_, hd_alert_win_, hd_alert_z_, hd_n_alerts_, stream_);
    HIP_OK(hipEventRecord(ev_alerts_, stream_));
  }
  if (dev()) {
    const double tq = now_ms();
    release_device(edge_ts);
    HIP_OK(hipEventRecord(ev_release_, stream_));
    metrics_.t_release_ms += now_ms() - tq;
    trace_event("release (device)", tq, now_ms(), 1);
  }
  const double tr2 = now_ms();
  trace_event("ro.K8-K11 launch", tsp, tr2, 1);
  if (want(OUT_ST) || want(OUT_FS)) format_rollover_text(edge_ts);
  const double tr3 = now_ms();
  metrics_.t_rollover_ms += tr2 - tr1;
  metrics_.t_format_ms += tr3 - tr2;
  trace_event("release", tr0, tr1, 1);
  trace_event("window+zscore+alerts", tr1, tr2, 1);
  trace_event("format (launch)", tr2, tr3, 1);
  roll_pending_ = true;
  roll_edge_ts_ = edge_ts;
  roll_batch_t0_ = batch_t0;
  roll_round_ = stats_round_;
  roll_ring_base_ = cur_dj_ ? cur_dj_->ring_base : (dj_ ? dj_->ring_head() : 0);
  // The decision runs on the rollover lane as soon as the GPU chain is done, while this thread
  // goes on (APM_ROLL_LANE=0: decide right here, the previous behaviour; sx rows always here).
  if (roll_lane_mode_) {
    roll_pending_ = false;
    roll_posted_ = true;
    roll_task_ = roll_lane_->post([this]() { finish_rollover_body(); });
  } else {
    finish_rollover();
  }
}

// Second half of a rollover, once its GPU chain has produced the candidates and the released
// count: queue the released lines' gather, decide the alerts, format the sx rows.
void Engine::finish_rollover() {
  if (roll_posted_) {
    const double t0 = now_ms();
    roll_lane_->wait(roll_task_);
    roll_posted_ = false;
    trace_event("roll.lane wait", t0, now_ms(), 1);
    return;
  }
  if (!roll_pending_) return;
  roll_pending_ = false;
  finish_rollover_body();
}

// Node mode: the ingest thread exchanges round q's alert candidates only once the lane queued them.
void Engine::wait_roll_round(uint64_t round) {
  std::unique_lock<std::mutex> lk(roll_mu_);
  roll_cv_.wait(lk, [&]() { return roll_done_round_ >= (int64_t)round; });
}

void Engine::finish_rollover_body() {
  const double t0 = now_ms();
  HIP_OK(hipEventSynchronize(ev_alerts_));
  const double t1 = now_ms();
  metrics_.t_rollover_ms += t1 - t0;
  trace_event("rollover wait", t0, t1, 1);
  metrics_.rollover_latency_ms.push_back(t1 - roll_batch_t0_);
  // the alerts first (they need only the candidates), then the release queued behind them
  flush_alerts(roll_edge_ts_);
  const double t2 = now_ms();
  trace_event("alerts", t1, t2, 1);
  if (dev()) {
    HIP_OK(hipEventSynchronize(ev_release_));
    release_device_finish();
  }
  trace_event("release finish", t2, now_ms(), 1);
  if (want(OUT_SX)) format_server_rollup(roll_edge_ts_);
  metrics_.t_format_ms += now_ms() - t1;
}

// K9 with the device join, part 1 (before K8): merge the tail into the sorted pool, count the
// released prefix (endTs <= edge) and plan its gather -- all on the stats stream, no host wait.
void Engine::release_device(int64_t edge_ts) {
  const int nxt = pool_cur_ ^ 1;
  if (pool_n_ + tail_n_ > cfg_.pool_cap) throw std::runtime_error("release pool overflow");
  if (apm_release_merge(d_pool_end_[pool_cur_] + pool_off_, d_pool_gid_[pool_cur_] + pool_off_, pool_n_, d_tail_end_,
                        d_tail_gid_, tail_n_, d_sort_end_, d_sort_gid_, d_pool_end_[nxt], d_pool_gid_[nxt],
                        d_release_tmp_, release_tmp_bytes_, stream_) != 0)
    throw std::runtime_error("release tmp too small");
  pool_cur_ = nxt;
  pool_off_ = 0;
  pool_n_ += tail_n_;
  tail_n_ = 0;
  apm_dj_count_le(d_pool_end_[pool_cur_], pool_n_, edge_ts, d_rel_n_, stream_);
  ExportArgs ex{};
  ex.add(d_rel_n_, hd_rel_n_, 8);
  if (want(OUT_DB) && pool_n_ > 0) {
    rel_copy_ = db_copy_;
    const int rc = rel_copy_
                       ? apm_dj_txcopy_plan(d_pool_gid_[pool_cur_], pool_n_, d_rel_n_, dj_->ring(), dj_->ring_cap(),
                                            d_rel_lens_, d_rel_offs_, d_rel_fb_, d_release_tmp_, release_tmp_bytes_,
                                            stream_)
                       : apm_dj_gather_plan(d_pool_gid_[pool_cur_], pool_n_, d_rel_n_, d_rel_lens_, d_rel_offs_,
                                            d_release_tmp_, release_tmp_bytes_, stream_);
    if (rc != 0) throw std::runtime_error("release tmp too small");
    ex.add(d_rel_offs_ + pool_n_, hd_rel_total_, 4);
    if (rel_copy_) ex.add(d_rel_fb_, hd_rel_total_ + 1, 4, true, 0);  // read and reset
  }
  apm_export(&ex, stream_);
}

// Part 2 (after the rollover's stream sync): the released count is known; gather the lines out
// of the HBM text ring into one blob, D2H it on the output lane, and publish the lowest ring
// position still referenced so the ingest thread may reuse the ring below it.
void Engine::release_device_finish() {
  const int64_t released = std::min<int64_t>(*h_rel_n_, pool_n_);
  if (want(OUT_DB) && released > 0) {
    size_t total = *h_rel_total_;
    bool copy = rel_copy_;
    bool host_enc = false;
    if (copy && (h_rel_total_[1] != 0 || txcopy_force_fb_)) {
      // a released line outside the GPU encoder's domain (txcopy.hip): this release goes out as
      // wire lines and is encoded on the host, row for row as the sink's encoder would
      copy = false;
      host_enc = true;
      ++metrics_.db_copy_fallbacks;
      if (apm_dj_gather_plan(d_pool_gid_[pool_cur_], pool_n_, d_rel_n_, d_rel_lens_, d_rel_offs_, d_release_tmp_,
                             release_tmp_bytes_, stream_) != 0)
        throw std::runtime_error("release tmp too small");
      uint32_t wire_total = 0;
      HIP_OK(hipMemcpyAsync(&wire_total, d_rel_offs_ + pool_n_, 4, hipMemcpyDeviceToHost, stream_));
      HIP_OK(hipStreamSynchronize(stream_));
      total = wire_total;
    }
    if (copy) metrics_.db_copy_rows += (uint64_t)released;
    const int k = rel_k_;
    rel_k_ ^= 1;
    const double tw = now_ms();
    rel_wait(rel_task_[k]);  // the buffer's previous reader is done
    trace_event("rel.wait_lane", tw, now_ms(), 1);
    if (total + 64 > rel_text_cap_[k]) d_rel_text_[k] = (char*)regrow(d_rel_text_[k], rel_text_cap_[k], total + 64);
    if (copy)
      apm_dj_txcopy_write(d_pool_gid_[pool_cur_], released, dj_->ring(), dj_->ring_cap(), d_rel_offs_, d_rel_text_[k],
                          stream_);
    else
      apm_dj_gather_copy(d_pool_gid_[pool_cur_], released, dj_->ring(), dj_->ring_cap(), d_rel_offs_, d_rel_text_[k],
                         total, stream_);
    // a COPY sink cuts its flushes from the row offsets (d_rel_offs_ is rewritten by the next
    // release: copied here, in stream order)
    const bool rows = byte_sink_[OUT_DB] != nullptr && !host_enc;
    if (rows) {
      if ((size_t)released + 1 > h_rel_offs_cap_[k]) {
        if (h_rel_offs_[k]) HIP_OK(hipHostFree(h_rel_offs_[k]));
        h_rel_offs_cap_[k] = ((size_t)released + 1) * 2;
        HIP_OK(hipHostMalloc((void**)&h_rel_offs_[k], h_rel_offs_cap_[k] * 4, hipHostMallocDefault));
      }
      d2h(h_rel_offs_[k], d_rel_offs_, ((size_t)released + 1) * 4, stream_);
    }
    HIP_OK(hipEventRecord(ev_rel_[k], stream_));
    const int rk = rel_ring_k_;
    rel_ring_k_ = (rel_ring_k_ + 1) % REL_RING;
    rel_task_[k] = post_rel([this, k, rk, total, rows, released, host_enc]() {
      const double tw0 = now_ms();
      HIP_OK(hipEventSynchronize(ev_rel_[k]));
      const double tw1 = now_ms();
      wait_fmt_holds(6 + FMT_RING + rk);  // the sink still writes from this slot (zero-copy COPY rows)
      trace_event("lane db wait gather", tw0, tw1, 4);
      trace_event("lane db wait sink", tw1, now_ms(), 4);
      char*& h = h_rel_text_[rk];
      if (total > h_rel_text_cap_[rk]) {
        if (h) HIP_OK(hipHostFree(h));
        h_rel_text_cap_[rk] = total * 2 + (4 << 20);  // (a pinned allocation costs ms: 2x headroom)
        HIP_OK(hipHostMalloc((void**)&h, h_rel_text_cap_[rk], hipHostMallocDefault));
      }
      const double tl0 = now_ms();
      if (rel_lane_on_) {
        lane_d2h(h, d_rel_text_[k], total, rel_stream_);
        HIP_OK(hipStreamSynchronize(rel_stream_));
      } else {
        lane_d2h(h, d_rel_text_[k], total);
        lane_sync();
      }
      const double tl1 = now_ms();
      if (host_enc) {
        std::string enc[5];
        int64_t counts[5] = {0, 0, 0, 0, 0};
        copyenc::encode_blob(std::string_view(h, total), enc, counts);
        emit_bytes(OUT_DB, enc[0].data(), enc[0].size());
      } else if (rows) {
        emit_bytes_held(OUT_DB, h, total, 6 + FMT_RING + rk, h_rel_offs_[k], (size_t)released);
      } else {
        emit_bytes(OUT_DB, h, total);
      }
      trace_event("lane db D2H", tl0, tl1, 4);
      trace_event("lane db emit", tl1, now_ms(), 4);
    });
  }
  metrics_.released += released;
  pool_off_ = released;
  pool_n_ -= released;
  // ring reuse bound: min position of the pool as of the previous rollover (its D2H is done)
  // and the ring base of the batch being processed then
  const uint64_t prev_min = *h_ring_min_;
  const uint64_t low = std::min<uint64_t>(prev_min, ring_low_pending_);
  if (low != UINT64_MAX) dj_->set_ring_low(low);
  // d_ring_min_ is UINT64_MAX here: the export below resets it after reading
  apm_dj_min_pos(d_pool_gid_[pool_cur_] + pool_off_, pool_n_, d_ring_min_, stream_);
  ExportArgs ex{};
  ex.add(d_ring_min_, hd_ring_min_, 8, /*reset=*/true, ~0ull);
  apm_export(&ex, stream_);
  ring_low_pending_ = roll_ring_base_;
}

void Engine::flush_alerts(int64_t edge_ts) {
  const int32_t na = h_n_alerts_[0];  // apm_alert_gather's clamped count (ev_alerts_ has completed)
  metrics_.alert_candidates += na;
  if (h_n_alerts_[1] > na) metrics_.alert_candidates_dropped += (uint64_t)(h_n_alerts_[1] - na);
  if (na <= 0) return;
  const bool need_rows = want(OUT_AL);
  // one sequential copy out of the GPU-written pinned buffers before the sort's random reads
  std::vector<AlertRec> alerts(h_alerts_, h_alerts_ + na);
  std::vector<WinStat> awin;
  std::vector<ZOut> az;
  if (need_rows) {
    awin.assign(h_alert_win_, h_alert_win_ + na);
    az.assign(h_alert_z_, h_alert_z_ + na);
  }
  // candidate i's rows are win_of(i) / z_of(i) in device order; decide in emission order
  std::vector<int32_t> ord((size_t)na);
  for (int32_t i = 0; i < na; ++i) ord[i] = i;
  std::sort(ord.begin(), ord.end(), [&](int32_t a, int32_t b) { return alerts[a].order < alerts[b].order; });
  // per-(service|series) cooldown, first candidate in emission order wins (:436-468)
  const double now = cfg_.alert_clock_entry ? (double)edge_ts : roll_now_;
  std::unique_lock<std::mutex> sg(series_mu_);  // series_ may grow on the stats thread meanwhile
  if (node_mode_) {
    // node-wide cooldown: queue the candidates (decided by the ingest thread, node_resolve)
    std::lock_guard<std::mutex> g(node_mu_);
    for (int32_t j = 0; j < na; ++j) {
      const int32_t i = ord[j];
      const AlertRec& r = alerts[i];
      const SeriesInfo& si = series_[r.series];
      const std::string& svc = dict_.service_name(si.service);
      NodePayload p;
      p.seq_batch = roll_round_;
      p.c = NodeCand{};
      p.c.edge_ts = edge_ts;
      p.c.first_batch = server_first_batch_[si.server];
      p.c.gidx = server_gidx_[si.server];
      p.c.seq = (uint32_t)(si.emit_key & 0xffffffu);
      p.c.lag_idx = r.lag_idx;
      p.c.causes = r.causes;
      uint64_t h = hash_bytes((const uint8_t*)svc.data(), svc.size());
      if (!cfg_.cooldown_by_service) {
        const std::string& sv = servers_[si.server];
        h = hash_mix(h, hash_bytes((const uint8_t*)sv.data(), sv.size()));
      }
      p.c.key = h;
      p.c.now = now;
      p.c.rank = coll_->rank();
      p.c.local_id = node_next_id_++;
      p.series = r.series;
      if (need_rows) { p.w = awin[i]; p.z = az[i]; }
      p.lag = cfg_.lags[r.lag_idx];
      node_q_.push_back(std::move(p));
    }
    return;
  }
  std::string text;
  std::vector<std::pair<uint64_t, double>> wins;
  for (int32_t j = 0; j < na; ++j) {
    const int32_t i = ord[j];
    const AlertRec& r = alerts[i];
    const SeriesInfo& si = series_[r.series];
    std::string key = dict_.service_name(si.service);
    if (!cfg_.cooldown_by_service) key = servers_[si.server] + '\x01' + key;
    auto it = last_alert_.find(key);
    if (it != last_alert_.end() && !((now - it->second) / 1000.0 > cfg_.cooldown_ms / 1000.0)) continue;
    last_alert_[key] = now;
    wins.push_back({cool_key_of(r.series), now});
    ++metrics_.alerts;
    if (need_rows) {
      const std::string fs = fmt::fs_line(edge_ts, servers_[si.server], dict_.service_name(si.service),
                                          cfg_.lags[r.lag_idx], awin[i], az[i]);
      text += fmt::al_line(now, edge_ts, servers_[si.server], dict_.service_name(si.service), r.causes, fs);
      text += '\n';
    }
  }
  sg.unlock();
  if (!wins.empty()) cool_mark(wins, stream_);
  if (!text.empty()) {  // (possibly the rollover lane) -> the al stream via node_text_
    std::lock_guard<std::mutex> g(node_mu_);
    node_text_ += text;
  }
}

uint64_t Engine::cool_key_of(int32_t s) const {
  const SeriesInfo& si = series_[s];
  const std::string& svc = dict_.service_name(si.service);
  uint64_t h = hash_bytes((const uint8_t*)svc.data(), svc.size());
  if (!cfg_.cooldown_by_service) {
    const std::string& sv = servers_[si.server];
    h = hash_mix(h, hash_bytes((const uint8_t*)sv.data(), sv.size()));
  }
  return h;
}

// Alerts decided (key, time): every local series of the key gets the time in d_cool_t_ (a scatter
// reading the pinned staging directly).  Called by the one thread that decides alerts.
void Engine::cool_mark(const std::vector<std::pair<uint64_t, double>>& wins, hipStream_t st) {
  std::vector<std::pair<int32_t, double>> upd;
  {
    std::lock_guard<std::mutex> g(series_mu_);
    for (const auto& w : wins) {
      auto it = cool_series_.find(w.first);
      if (it == cool_series_.end()) continue;
      for (int32_t s : it->second) upd.push_back({s, w.second});
    }
  }
  if (upd.empty()) return;
  if (!cool_ev_) HIP_OK(hipEventCreateWithFlags(&cool_ev_, hipEventDisableTiming));
  else HIP_OK(hipEventSynchronize(cool_ev_));  // the previous scatter read the staging
  if (upd.size() > cool_cap_) {
    if (h_cool_idx_) { HIP_OK(hipHostFree(h_cool_idx_)); HIP_OK(hipHostFree(h_cool_val_)); }
    cool_cap_ = std::max<size_t>(upd.size() * 2, 4096);
    HIP_OK(hipHostMalloc((void**)&h_cool_idx_, cool_cap_ * 4, hipHostMallocDefault));
    HIP_OK(hipHostMalloc((void**)&h_cool_val_, cool_cap_ * 8, hipHostMallocDefault));
  }
  for (size_t i = 0; i < upd.size(); ++i) { h_cool_idx_[i] = upd[i].first; h_cool_val_[i] = upd[i].second; }
  int32_t* di = nullptr;
  double* dv = nullptr;
  HIP_OK(hipHostGetDevicePointer((void**)&di, h_cool_idx_, 0));
  HIP_OK(hipHostGetDevicePointer((void**)&dv, h_cool_val_, 0));
  apm_scatter_f64(d_cool_t_, di, dv, (int32_t)upd.size(), st);
  HIP_OK(hipEventRecord(cool_ev_, st));
}

// After a restore / cooldown import: the key map and d_cool_t_ from series_ and both maps.
void Engine::rebuild_cool() {
  std::vector<double> t((size_t)std::max(n_series_, 1), std::nan(""));
  {
    std::lock_guard<std::mutex> g(series_mu_);
    cool_series_.clear();
    for (int32_t s = 0; s < n_series_; ++s) {
      const uint64_t k = cool_key_of(s);
      cool_series_[k].push_back(s);
      auto nc = node_cool_.find(k);
      if (nc != node_cool_.end()) t[s] = nc->second;
      const SeriesInfo& si = series_[s];
      std::string key = dict_.service_name(si.service);
      if (!cfg_.cooldown_by_service) key = servers_[si.server] + '\x01' + key;
      auto la = last_alert_.find(key);
      if (la != last_alert_.end() && !(la->second <= t[s])) t[s] = la->second;
    }
  }
  HIP_OK(hipMemsetAsync(d_cool_t_, 0xff, (size_t)cfg_.max_series * 8, stream_));
  if (n_series_ > 0) HIP_OK(hipMemcpyAsync(d_cool_t_, t.data(), (size_t)n_series_ * 8, hipMemcpyHostToDevice, stream_));
  HIP_OK(hipStreamSynchronize(stream_));
}

int32_t Engine::intern_name(const std::string& name) {
  auto it = name_off_.find(name);
  if (it != name_off_.end()) return it->second;
  const int32_t off = (int32_t)h_names_.size();
  h_names_ += name;
  name_off_.emplace(name, off);
  return off;
}

// Frees a dmalloc'd buffer and forgets it (the destructor frees what is still listed).
void Engine::dfree(void* p) {
  if (!p) return;
  HIP_OK(hipFree(p));
  std::lock_guard<std::mutex> g(alloc_mu_);
  allocations_.erase(std::remove(allocations_.begin(), allocations_.end(), p), allocations_.end());
  auto it = alloc_bytes_.find(p);
  if (it != alloc_bytes_.end()) {
    device_bytes_ -= it->second;
    alloc_bytes_.erase(it);
  }
}

void* Engine::regrow(void* old, size_t& cap, size_t need) {
  if (need <= cap && old) return old;
  // 2x headroom: a regrow syncs the stream and hipFree waits for the device (a few ms of one
  // batch), so the per-batch buffers must stop growing during the warm-up
  size_t nc = std::max<size_t>(2 * need, 4 << 20);
  // The old buffer is retired, not freed: kernels still in flight on any stream may read it, and
  // hipFree would wait for the whole device (the collective stream included).  Retired buffers
  // stay listed in allocations_ (and counted) until the engine goes away; with 2x growth they
  // add up to less than the live buffer.
  (void)old;
  cap = nc;
  void* p = nullptr;
  const size_t bytes = (nc + 255) & ~(size_t)255;
  HIP_OK(hipMalloc(&p, bytes));
  // zeroed in order on the stats stream; the sync orders it for the other streams' later work
  // without waiting for them (dmalloc's device-wide sync is for construction time)
  HIP_OK(hipMemsetAsync(p, 0, bytes, stream_));
  HIP_OK(hipStreamSynchronize(stream_));
  std::lock_guard<std::mutex> g(alloc_mu_);
  allocations_.push_back(p);
  alloc_bytes_[p] = bytes;
  device_bytes_ += bytes;
  return p;
}

void Engine::sync_format_tables() {
  // uploads go through the pinned stager: nothing here waits for the stats stream
  if (names_uploaded_ < h_names_.size()) {
    if (h_names_.size() > names_cap_) {
      // grow: re-upload everything into the bigger buffer
      d_names_ = (char*)regrow(d_names_, names_cap_, h_names_.size());
      names_uploaded_ = 0;
    }
    const size_t nb = h_names_.size() - names_uploaded_;
    char* st = stage(nb);
    std::memcpy(st, h_names_.data() + names_uploaded_, nb);
    h2d(d_names_ + names_uploaded_, st, nb, stream_);
    stage_done();
    names_uploaded_ = h_names_.size();
  }
  if (ser_names_uploaded_ < n_series_) {
    const int32_t lo = ser_names_uploaded_;
    const size_t nb = (size_t)(n_series_ - lo) * 16;
    char* st = stage(nb);
    std::memcpy(st, h_ser_names_.data() + (size_t)lo * 4, nb);
    h2d(d_ser_names_ + (size_t)lo * 4, st, nb, stream_);
    stage_done();
    ser_names_uploaded_ = n_series_;
  }
  if (perm_dirty_) {
    // Emission order of the series.  h_perm_ already holds the first h_perm_.size() series in
    // order (emit keys never change, h_perm_key_ holds them in that order), so only the new ones
    // are sorted and merged in from the back: O(new + moved) with sequential key reads, and only
    // the suffix from the first insertion point is uploaded (a std::merge over all 80k series
    // with random key lookups cost ~0.2 ms of the stats thread per batch with one new series).
    const int32_t old_n = std::min<int32_t>((int32_t)h_perm_.size(), n_series_);
    std::vector<std::pair<uint64_t, int32_t>> fresh;
    for (int32_t i = old_n; i < n_series_; ++i) fresh.push_back({h_emit_key_[i], i});
    std::sort(fresh.begin(), fresh.end());
    h_perm_.resize(old_n);
    h_perm_key_.resize(old_n);
    size_t first = (size_t)old_n;
    if (!fresh.empty()) {
      first = (size_t)(std::lower_bound(h_perm_key_.begin(), h_perm_key_.end(), fresh.front().first) -
                       h_perm_key_.begin());
      h_perm_.resize(n_series_);
      h_perm_key_.resize(n_series_);
      int64_t a = old_n - 1, w = n_series_ - 1, b = (int64_t)fresh.size() - 1;
      while (b >= 0) {  // backward merge; keys are distinct
        if (a >= 0 && h_perm_key_[a] > fresh[b].first) {
          h_perm_key_[w] = h_perm_key_[a];
          h_perm_[w] = h_perm_[a];
          --a;
        } else {
          h_perm_key_[w] = fresh[b].first;
          h_perm_[w] = fresh[b].second;
          --b;
        }
        --w;
      }
    }
    if (perm_uploaded_ < (int64_t)first) first = (size_t)std::max<int64_t>(perm_uploaded_, 0);
    const size_t nb = ((size_t)n_series_ - first) * 4;
    if (nb) {
      char* st = stage(nb);
      std::memcpy(st, h_perm_.data() + first, nb);
      h2d(d_perm_ + first, st, nb, stream_);
      stage_done();
    }
    perm_uploaded_ = n_series_;
    perm_dirty_ = false;
  }
}

// ms since the epoch -> Postgres COPY timestamp text 'YYYY-MM-DD HH:MM:SS.mmm+00' (copyenc.cpp
// c_ts); returns the length written to out (>= 27 bytes)
int Engine::pg_timestamp(int64_t ms, char* out) {
  int64_t days = ms / 86400000, rem = ms % 86400000;
  if (rem < 0) { rem += 86400000; --days; }
  days += 719468;
  const int64_t era = (days >= 0 ? days : days - 146096) / 146097;
  const unsigned doe = (unsigned)(days - era * 146097);
  const unsigned yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  const unsigned doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  const unsigned mp = (5 * doy + 2) / 153;
  const unsigned d = doy - (153 * mp + 2) / 5 + 1;
  const unsigned m = mp < 10 ? mp + 3 : mp - 9;
  const int y = (int)(yoe + era * 400) + (m <= 2);
  return std::snprintf(out, 32, "%04d-%02u-%02u %02d:%02d:%02d.%03d+00", y, m, d, (int)(rem / 3600000),
                       (int)(rem / 60000 % 60), (int)(rem / 1000 % 60), (int)(rem % 1000));
}

void Engine::set_fs_copy(bool on) {
  flush();
  fs_copy_ = on;
}

bool Engine::set_db_copy(bool on) {
  flush();
  db_copy_ = on && dj_ != nullptr;
  return db_copy_;
}

void Engine::emit_bytes(int kind, const char* p, size_t n) {
  if (!n) return;
  if (byte_sink_[kind]) {
    drain_kind(kind);
    byte_sink_[kind]->write_bytes(kind, p, n);
    sink_bytes_[kind] += n;
    return;
  }
  if (sink_fd_[kind] >= 0) {
    // keep stream order: whatever is buffered goes first, then straight from the staging buffer
    drain_kind(kind);
    while (n) {
      const ssize_t w = ::write(sink_fd_[kind], p, n);
      if (w < 0) {
        if (errno == EINTR) continue;
        throw std::runtime_error(std::string("sink write failed: ") + std::strerror(errno));
      }
      p += w;
      n -= (size_t)w;
      sink_bytes_[kind] += (size_t)w;
    }
    return;
  }
  blob_[kind].append(p, n);
}

void Engine::emit_bytes_held(int kind, const char* p, size_t n, int k, const uint32_t* row_off, size_t nrows) {
  if (!n) return;
  if (!byte_sink_[kind]) { emit_bytes(kind, p, n); return; }
  drain_kind(kind);
  std::shared_ptr<FmtHolds> hs = fmt_holds_;
  {
    std::lock_guard<std::mutex> g(hs->mu);
    ++hs->n[k];
  }
  std::shared_ptr<const void> hold(p, [hs, k](const void*) {
    {
      std::lock_guard<std::mutex> g(hs->mu);
      --hs->n[k];
    }
    hs->cv.notify_all();
  });
  if (row_off) byte_sink_[kind]->write_rows_held(kind, p, n, row_off, nrows, std::move(hold));
  else byte_sink_[kind]->write_bytes_held(kind, p, n, std::move(hold));
  sink_bytes_[kind] += n;
}

void Engine::wait_fmt_holds(int k) {
  FmtHolds& hs = *fmt_holds_;
  std::unique_lock<std::mutex> lk(hs.mu);
  hs.cv.wait(lk, [&] { return hs.n[k] == 0; });
}

void Engine::format_rollover_text(int64_t edge_ts) {
  const int32_t n = n_series_;
  if (n == 0) return;
  const double tf0 = now_ms();
  sync_format_tables();
  trace_event("fmt.tables", tf0, now_ms(), 1);
  const int32_t S = cfg_.max_series;
  FormatArgs fa{};
  fa.perm = d_perm_;
  fa.win = d_win_;
  for (int l = 0; l < cfg_.n_lags; ++l) { fa.z[l] = lag_[l].out; fa.lag_value[l] = cfg_.lags[l]; }
  std::vector<int> lag_order(cfg_.n_lags);
  for (int l = 0; l < cfg_.n_lags; ++l) lag_order[l] = l;
  std::sort(lag_order.begin(), lag_order.end(), [&](int a, int b) { return cfg_.lags[a] < cfg_.lags[b]; });
  for (int l = 0; l < cfg_.n_lags; ++l) fa.lag_order[l] = lag_order[l];
  fa.series_names = reinterpret_cast<const int4*>(d_ser_names_);
  fa.names = d_names_;
  fa.edge_ts = edge_ts;
  fa.n = n;
  fa.n_lags = cfg_.n_lags;
  fa.want_st = want(OUT_ST);
  fa.want_fs = want(OUT_FS);
  fa.fs_copy = fs_copy_ ? 1 : 0;
  if (fs_copy_) fa.ts_copy_len = pg_timestamp(edge_ts, fa.ts_copy);
  fa.ts_wire_len = std::snprintf(fa.ts_wire, sizeof fa.ts_wire, "%lld|", (long long)edge_ts);
  fa.st_len = d_fmt_len_;
  fa.fs_len = d_fmt_len_ + (S + 1);
  fa.st_off = d_fmt_off_;
  fa.fs_off = d_fmt_off_ + (S + 1);
  fa.fallback = d_fmt_fallback_;
  // Output bound from the name lengths (numbers are at most ~25 characters), so nothing waits
  // for the length pass: the output lane reads the real totals after the event.
  const int k = fmt_k_;
  fmt_k_ ^= 1;
  const double tf1 = now_ms();
  out_wait(fmt_task_[k]);  // slot k's previous D2H + emission is done
  trace_event("fmt.wait_lane", tf1, now_ms(), 1);
  const size_t st_cap = fa.want_st ? (size_t)n * (176 + max_name_len_) : 0;
  const size_t fs_cap = fa.want_fs ? (size_t)n * cfg_.n_lags * (fs_copy_ ? 720 + 2 * max_name_len_ : 560 + max_name_len_) : 0;
  if (fmt_host_) {
    // the kernel writes into the pinned buffer itself: the sink must be done with its contents
    const double th = now_ms();
    wait_fmt_holds(k);
    trace_event("fmt.wait_holds", th, now_ms(), 1);
    if (st_cap + fs_cap + 64 > h_fmt_cap_[k]) {
      if (h_fmt_out_[k]) HIP_OK(hipHostFree(h_fmt_out_[k]));
      h_fmt_cap_[k] = (st_cap + fs_cap + 64) * 5 / 4;
      HIP_OK(hipHostMalloc((void**)&h_fmt_out_[k], h_fmt_cap_[k], hipHostMallocDefault));
      HIP_OK(hipHostGetDevicePointer((void**)&hd_fmt_out_[k], h_fmt_out_[k], 0));
    }
    fa.st_out = hd_fmt_out_[k];
    fa.fs_out = hd_fmt_out_[k] + st_cap;
  } else {
    if (st_cap + fs_cap + 64 > fmt_out_cap_[k]) d_fmt_out_[k] = (char*)regrow(d_fmt_out_[k], fmt_out_cap_[k], st_cap + fs_cap + 64);
    fa.st_out = d_fmt_out_[k];
    fa.fs_out = d_fmt_out_[k] + st_cap;
  }
  const double tpl = now_ms();
  if (apm_format_plan(&fa, d_fmt_tmp_, fmt_tmp_bytes_, stream_) != 0) throw std::runtime_error("format scan failed");
  const double tpw = now_ms();
  trace_event("fmt.len+scans", tpl, tpw, 1);
  fa.stage_hint = fmt_block_bytes_.load(std::memory_order_relaxed);
  apm_format_write(&fa, stream_);
  trace_event("fmt.write", tpw, now_ms(), 1);
  {
    ExportArgs ex{};
    ex.add(fa.st_off + n, hd_fmt_meta_ + 4 * k + 0, 4);
    ex.add(fa.fs_off + (size_t)n * cfg_.n_lags, hd_fmt_meta_ + 4 * k + 1, 4);
    apm_export(&ex, stream_);
  }
  fs_rows_[k] = 0;
  if (fa.want_fs && byte_sink_[OUT_FS]) {
    // the row offsets for the sink's flush cuts (slot k's lane is done with the previous ones)
    const size_t rows = (size_t)n * cfg_.n_lags;
    if (rows + 1 > h_fs_off_cap_[k]) {
      if (h_fs_off_[k]) HIP_OK(hipHostFree(h_fs_off_[k]));
      h_fs_off_cap_[k] = (rows + 1) * 5 / 4;
      HIP_OK(hipHostMalloc((void**)&h_fs_off_[k], h_fs_off_cap_[k] * 4, hipHostMallocDefault));
    }
    d2h(h_fs_off_[k], fa.fs_off, (rows + 1) * 4, stream_);
    fs_rows_[k] = rows;
  }
  HIP_OK(hipEventRecord(ev_fmt_[k], stream_));
  trace_event("fmt.plan", tf0, now_ms(), 1);
  char* dst = d_fmt_out_[k];
  const size_t n_st = fa.want_st ? (size_t)n : 0, n_fs = fa.want_fs ? (size_t)n * cfg_.n_lags : 0;
  if (fmt_host_) {
    fmt_task_[k] = post_out([this, k, st_cap, n_st, n_fs]() {
      const double tl0 = now_ms();
      HIP_OK(hipEventSynchronize(ev_fmt_[k]));  // the text is in host memory once K12 completed
      const size_t st_total = h_fmt_meta_[4 * k], fs_total = h_fmt_meta_[4 * k + 1];
      note_fmt_block(st_total, n_st, fs_total, n_fs);
      {
        std::lock_guard<std::mutex> g(out_mu_);
        formatted_bytes_lane_ += st_total + fs_total;
      }
      const double tl1 = now_ms();
      emit_bytes(OUT_ST, h_fmt_out_[k], st_total);
      emit_bytes_held(OUT_FS, h_fmt_out_[k] + st_cap, fs_total, k, fs_rows_[k] ? h_fs_off_[k] : nullptr, fs_rows_[k]);
      trace_event("lane st/fs wait (direct)", tl0, tl1, 4);
      trace_event("lane st/fs emit", tl1, now_ms(), 4);
    });
    return;
  }
  const int hk = fmt_ring_k_;
  fmt_ring_k_ = (fmt_ring_k_ + 1) % FMT_RING;
  fmt_task_[k] = post_out([this, k, hk, dst, st_cap, n_st, n_fs]() {
    const double tw0 = now_ms();
    HIP_OK(hipEventSynchronize(ev_fmt_[k]));
    const size_t st_total = h_fmt_meta_[4 * k], fs_total = h_fmt_meta_[4 * k + 1];
    note_fmt_block(st_total, n_st, fs_total, n_fs);
    const double tw1 = now_ms();
    wait_fmt_holds(6 + hk);  // the sink still writes from this ring slot (zero-copy COPY rows)
    trace_event("lane st/fs wait format", tw0, tw1, 4);
    trace_event("lane st/fs wait sink", tw1, now_ms(), 4);
    if (st_total + fs_total > h_fmt_ring_cap_[hk]) {
      if (h_fmt_ring_[hk]) HIP_OK(hipHostFree(h_fmt_ring_[hk]));
      h_fmt_ring_cap_[hk] = (st_total + fs_total) * 5 / 4 + (4 << 20);
      HIP_OK(hipHostMalloc((void**)&h_fmt_ring_[hk], h_fmt_ring_cap_[hk], hipHostMallocDefault));
    }
    char* h = h_fmt_ring_[hk];
    const double tl0 = now_ms();
    if (st_total) lane_d2h(h, dst, st_total);
    if (fs_total) lane_d2h(h + st_total, dst + st_cap, fs_total);
    lane_sync();
    {
      std::lock_guard<std::mutex> g(out_mu_);
      formatted_bytes_lane_ += st_total + fs_total;
    }
    const double tl1 = now_ms();
    emit_bytes(OUT_ST, h, st_total);
    emit_bytes_held(OUT_FS, h + st_total, fs_total, 6 + hk, fs_rows_[k] ? h_fs_off_[k] : nullptr, fs_rows_[k]);
    trace_event("lane st/fs D2H", tl0, tl1, 4);
    trace_event("lane st/fs emit", tl1, now_ms(), 4);
  });
}

// Ingest (caller) thread: the sample applies from the next processed batch on.
bool Engine::set_server_context(const std::string& server, double ts_ms, const std::vector<double>& gauges,
                                double host_load) {
  auto it = server_ids_.find(server);
  if (it == server_ids_.end()) return false;
  CtxUpdate u;
  u.batch = batch_no_;
  u.server = it->second;
  u.row[0] = ts_ms;
  for (int k = 0; k < 16; ++k) u.row[1 + k] = k < (int)gauges.size() ? gauges[k] : apm_nan();
  u.row[17] = host_load;
  std::lock_guard<std::mutex> g(ctx_mu_);
  ctx_pending_.push_back(u);
  return true;
}

// Stats thread (or a caller with the stats thread idle): fold the samples of batches <= upto.
void Engine::apply_ctx_pending(uint64_t upto) {
  std::lock_guard<std::mutex> g(ctx_mu_);
  size_t k = 0;
  for (const CtxUpdate& u : ctx_pending_) {
    if (u.batch > upto) break;  // tags ascend
    const int32_t v = u.server;
    if (h_ctx_.size() < (size_t)(v + 1) * CTX_FIELDS) h_ctx_.resize((size_t)(v + 1) * CTX_FIELDS, 0.0);
    std::copy(u.row, u.row + CTX_FIELDS, h_ctx_.data() + (size_t)v * CTX_FIELDS);
    ctx_dirty_ = true;
    ++k;
  }
  ctx_pending_.erase(ctx_pending_.begin(), ctx_pending_.begin() + (ptrdiff_t)k);
}

void Engine::server_rollup(int64_t edge_ts) {
  const int32_t nsv = (int32_t)servers_.size();
  if (nsv == 0) return;
  if ((size_t)nsv > roll_cap_) {  // grow (rare: new servers)
    size_t cap = std::max<size_t>(64, (size_t)nsv * 2), c1 = 0, c2 = 0, c3 = 0;
    d_ctx_ = (double*)regrow(d_ctx_, c1 = roll_cap_ * CTX_FIELDS * 8, cap * CTX_FIELDS * 8);
    d_roll_acc_ = (unsigned long long*)regrow(d_roll_acc_, c2 = roll_cap_ * ROLLUP_ACC * 8, cap * ROLLUP_ACC * 8);
    d_roll_out_ = (double*)regrow(d_roll_out_, c3 = roll_cap_ * ROLLUP_OUT * 8, cap * ROLLUP_OUT * 8);
    if (h_roll_out_) HIP_OK(hipHostFree(h_roll_out_));
    HIP_OK(hipHostMalloc((void**)&h_roll_out_, cap * ROLLUP_OUT * 8, hipHostMallocDefault));
    roll_cap_ = cap;
    ctx_dirty_ = true;
  }
  if (series_server_uploaded_ < n_series_) {  // new series: pinned stager, no stream sync
    const int32_t lo = series_server_uploaded_;
    int32_t* sv = reinterpret_cast<int32_t*>(stage((size_t)(n_series_ - lo) * 4));
    for (int32_t s = lo; s < n_series_; ++s) sv[s - lo] = series_[s].server;
    h2d(d_series_server_ + lo, sv, (size_t)(n_series_ - lo) * 4, stream_);
    stage_done();
    series_server_uploaded_ = n_series_;
  }
  if (ctx_dirty_) {  // (a JMX sample per server per batch: pinned staging, no stream sync)
    const size_t nb = (size_t)nsv * CTX_FIELDS * 8;
    double* full = reinterpret_cast<double*>(stage(nb));
    std::fill(full, full + (size_t)nsv * CTX_FIELDS, 0.0);
    std::copy(h_ctx_.begin(), h_ctx_.begin() + std::min(h_ctx_.size(), (size_t)nsv * CTX_FIELDS), full);
    h2d(d_ctx_, full, nb, stream_);
    stage_done();
    ctx_dirty_ = false;
  }
  RollupArgs ra{};
  ra.win = d_win_;
  ra.series_server = d_series_server_;
  for (int l = 0; l < cfg_.n_lags; ++l) ra.z[l] = lag_[l].out;
  ra.n_lags = cfg_.n_lags;
  ra.n_series = n_series_;
  ra.n_servers = nsv;
  ra.edge_ts = edge_ts;
  ra.tpm_div = (double)cfg_.window * cfg_.interval_len / 60.0;
  ra.ctx = d_ctx_;
  ra.acc = d_roll_acc_;
  ra.out = d_roll_out_;
  apm_server_rollup(&ra, stream_);
  HIP_OK(hipMemcpyAsync(h_roll_out_, d_roll_out_, (size_t)nsv * ROLLUP_OUT * 8, hipMemcpyDeviceToHost, stream_));
}

void Engine::format_server_rollup(int64_t edge_ts) {
  // sx|ts|server|liveSeries|tpm|avg|maxP95|avgSignals|p75Signals|heapUtil|metaUtil|dsUtil|sysLoad|
  //   threads|beanUtil|gaugeAgeS|vmLoad|flags      (NaN prints 'undefined', like nf())
  const int32_t nsv = (int32_t)servers_.size();
  std::string& out = blob_[OUT_SX];
  for (int32_t v = 0; v < nsv; ++v) {
    if (server_rank_[v] < 0) continue;  // no transactions yet
    const double* o = h_roll_out_ + (size_t)v * ROLLUP_OUT;
    out += "sx|";
    out += std::to_string(edge_ts);
    out += '|';
    out += servers_[v];
    static const int fx[ROLLUP_OUT] = {0, 2, 1, 1, 0, 0, 3, 3, 3, 2, 0, 3, 1, 2, 0};
    for (int k = 0; k < ROLLUP_OUT; ++k) {
      out += '|';
      if (fx[k] == 0 && o[k] == o[k]) js::append_num(out, o[k]);
      else out += js::nf(o[k], fx[k]);
    }
    out += '\n';
  }
}

void Engine::format_rollover_text_host(int64_t edge_ts) {
  std::vector<WinStat> win;
  download_winstats(win);
  std::vector<std::vector<ZOut>> z(cfg_.n_lags);
  for (int l = 0; l < cfg_.n_lags; ++l) download_zout(l, z[l]);
  std::vector<int32_t> order;
  for (int32_t s = 0; s < n_series_; ++s) if (win[s].active) order.push_back(s);
  std::sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return series_[a].emit_key < series_[b].emit_key; });
  std::string& st = blob_[OUT_ST];
  std::string& fs = blob_[OUT_FS];
  const bool w_st = want(OUT_ST), w_fs = want(OUT_FS);
  // lag order: ascending LAG value (integer-keyed object iteration in the reference)
  std::vector<int> lag_order(cfg_.n_lags);
  for (int l = 0; l < cfg_.n_lags; ++l) lag_order[l] = l;
  std::sort(lag_order.begin(), lag_order.end(), [&](int a, int b) { return cfg_.lags[a] < cfg_.lags[b]; });
  for (int32_t s : order) {
    const SeriesInfo& si = series_[s];
    if (w_st) { st += fmt::st_line(edge_ts, servers_[si.server], dict_.service_name(si.service), win[s]); st += '\n'; }
    if (w_fs)
      for (int l : lag_order) {
        fs += fmt::fs_line(edge_ts, servers_[si.server], dict_.service_name(si.service), cfg_.lags[l], win[s], z[l][s]);
        fs += '\n';
      }
  }
}

void Engine::download_winstats(std::vector<WinStat>& out) {
  out.resize(std::max(n_series_, 1));
  if (n_series_ == 0) return;
  HIP_OK(hipMemcpyAsync(out.data(), d_win_, (size_t)n_series_ * sizeof(WinStat), hipMemcpyDeviceToHost, stream_));
  HIP_OK(hipStreamSynchronize(stream_));
}

void Engine::download_zout(int l, std::vector<ZOut>& out) {
  out.resize(std::max(n_series_, 1));
  if (n_series_ == 0) return;
  HIP_OK(hipMemcpyAsync(out.data(), lag_[l].out, (size_t)n_series_ * sizeof(ZOut), hipMemcpyDeviceToHost, stream_));
  HIP_OK(hipStreamSynchronize(stream_));
}

const char* out_kind_name(int k) {
  static const char* n[N_OUT] = {"transactions", "audit_db", "db", "st", "fs", "al", "sx", "fb"};
  return n[k];
}

int out_kind_of(const std::string& name) {
  for (int k = 0; k < N_OUT; ++k)
    if (name == out_kind_name(k)) return k;
  throw std::runtime_error("unknown output stream: " + name);
}

std::vector<std::string> Engine::take(const std::string& kind) {
  const std::string b = take_bytes(kind);
  std::vector<std::string> r;
  size_t i = 0;
  while (i < b.size()) {
    size_t j = b.find('\n', i);
    if (j == std::string::npos) j = b.size();
    r.emplace_back(b, i, j - i);
    i = j + 1;
  }
  return r;
}

std::string Engine::take_bytes(const std::string& kind) {
  flush();
  std::string r;
  r.swap(blob_[out_kind_of(kind)]);
  return r;
}

void Engine::set_sink_fd(const std::string& kind, int fd) {
  flush();
  sink_fd_[out_kind_of(kind)] = fd;
}

void Engine::set_byte_sink(const std::string& kind, std::shared_ptr<ByteSink> sink) {
  flush();
  byte_sink_[out_kind_of(kind)] = std::move(sink);
}

void Engine::drain_kind(int k) {
  if (byte_sink_[k] && !blob_[k].empty()) {
    byte_sink_[k]->write_bytes(k, blob_[k].data(), blob_[k].size());
    sink_bytes_[k] += blob_[k].size();
    blob_[k].clear();
    return;
  }
  if (sink_fd_[k] < 0 || blob_[k].empty()) return;
  const char* p = blob_[k].data();
  size_t left = blob_[k].size();
  while (left) {
    const ssize_t w = ::write(sink_fd_[k], p, left);
    if (w < 0) {
      if (errno == EINTR) continue;
      throw std::runtime_error(std::string("sink write failed: ") + std::strerror(errno));
    }
    p += w;
    left -= (size_t)w;
  }
  sink_bytes_[k] += blob_[k].size();
  blob_[k].clear();
}

void Engine::drain_sinks(uint32_t kinds) {
  for (int k = 0; k < N_OUT; ++k)
    if ((kinds >> k) & 1u) drain_kind(k);
}

void Engine::warm_history(uint64_t seed) {
  flush();
  ck_all_dirty_ = true;  // every ring row rewritten: the next checkpoint is a base
  // Use the latest window stats as the per-series baseline; fill every lag ring completely.
  for (int l = 0; l < cfg_.n_lags; ++l) {
    LagState& LS = lag_[l];
    ZArgs za{};
    za.ring = LS.ring; za.len = LS.len; za.sum = LS.sum; za.comp = LS.comp; za.cnt = LS.cnt;
    za.sumsq = LS.sumsq; za.sqcomp = LS.sqcomp; za.S = cfg_.max_series; za.n_series = n_series_;
    za.lag = cfg_.lags[l]; za.head = (int32_t)(rollover_idx_ % cfg_.lags[l]);
    apm_zscore_warm(&za, cfg_.ring_bytes, cfg_.lags[l], seed + l, d_win_, stream_);
  }
  HIP_OK(hipStreamSynchronize(stream_));
}

uintptr_t Engine::alloc_pinned(size_t n) {
  void* p = nullptr;
  HIP_OK(hipHostMalloc(&p, n + 256, hipHostMallocDefault));
  return (uintptr_t)p;
}

void Engine::free_pinned(uintptr_t p) { hipHostFree((void*)p); }

void Engine::pack_moments_locked(double* d_dst, int32_t cap, hipStream_t stream, bool atomic_path) {
  const double tp0 = now_ms();
  if (coll_) {  // node-wide slots: queue new services, adopt the slots the last round assigned
    reg_collect_locked();
    reg_apply_locked();
  }
  trace_event("pack.registry", tp0, now_ms(), 1);
  // series -> service table (grows with the dictionary): upload only the new tail
  if (series_service_uploaded_ < n_series_) {
    // Pinned host mirror of the table: the series list is append-only, so each upload reads a
    // region no earlier (possibly still in-flight) copy reads -- no stream sync on the stats thread.
    const int32_t lo = series_service_uploaded_;
    if (!h_series_service_) {
      void* p = nullptr;
      HIP_OK(hipHostMalloc(&p, (size_t)cfg_.max_series * 4, hipHostMallocDefault));
      h_series_service_ = (int32_t*)p;
    }
    if (lo == 0) HIP_OK(hipStreamSynchronize(stream_));  // table reset (load_state / new slots): rewrite from 0
    for (int32_t s = lo; s < n_series_; ++s) h_series_service_[s] = svc_key(s);
    HIP_OK(hipMemcpyAsync(d_series_service_ + lo, h_series_service_ + lo, (size_t)(n_series_ - lo) * 4,
                          hipMemcpyHostToDevice, stream_));
    series_service_uploaded_ = n_series_;
  }
  // the pack reads the z-score state written on the main stream: order another stream after it
  if (stream != stream_) {
    HIP_OK(hipEventRecord(ev_a_, stream_));
    HIP_OK(hipStreamWaitEvent(stream, ev_a_, 0));
  }
  if (!atomic_path && cfg_.n_lags * NSTAT * 2 + 1 <= 16) {
    // MFMA Gram path (fleet.hip): series listed per service (CSR).  Series added since the CSR
    // snapshot are accumulated by the atomic kernel on top; the CSR is rebuilt (host pass + a
    // stream sync) only when that tail exceeds 1/8 of the table, i.e. O(log n) times while the
    // dictionary grows instead of on every batch that adds a series.
    if (svc_csr_n_ < 0 || svc_csr_cap_ != cap || (int64_t)(n_series_ - svc_csr_n_) * 8 > n_series_) {
      h_svc_off_.assign((size_t)cap + 1, 0);
      for (int32_t s = 0; s < n_series_; ++s) {
        const int32_t v = svc_key(s);
        if (v >= 0 && v < cap) ++h_svc_off_[(size_t)v + 1];
      }
      for (int32_t v = 0; v < cap; ++v) h_svc_off_[(size_t)v + 1] += h_svc_off_[v];
      h_svc_ids_.assign(std::max<size_t>(1, (size_t)h_svc_off_[cap]), 0);
      std::vector<int32_t> pos(h_svc_off_.begin(), h_svc_off_.end() - 1);
      for (int32_t s = 0; s < n_series_; ++s) {
        const int32_t v = svc_key(s);
        if (v >= 0 && v < cap) h_svc_ids_[(size_t)pos[v]++] = s;
      }
      trace_event("fleet.csr", now_ms(), now_ms(), 1);
      // an earlier pack may still read the old lists; on the comm stream that pack can sit
      // behind an all-reduce, so wait with the collective watchdog rather than a bare sync
      HIP_OK(hipEventRecord(ev_a_, stream));
      if (coll_) coll_wait(nullptr, ev_a_, "fleet CSR rebuild");
      else HIP_OK(hipEventSynchronize(ev_a_));
      d_svc_off_ = (int32_t*)regrow(d_svc_off_, svc_off_cap_, h_svc_off_.size() * 4);
      d_svc_ids_ = (int32_t*)regrow(d_svc_ids_, svc_ids_cap_, h_svc_ids_.size() * 4);
      HIP_OK(hipMemcpyAsync(d_svc_off_, h_svc_off_.data(), h_svc_off_.size() * 4, hipMemcpyHostToDevice, stream));
      HIP_OK(hipMemcpyAsync(d_svc_ids_, h_svc_ids_.data(), h_svc_ids_.size() * 4, hipMemcpyHostToDevice, stream));
      svc_csr_n_ = n_series_;
      svc_csr_cap_ = cap;
      tail_csr_for_ = {-1, -1};
      tail_upto_ = -1;  // rows may have moved (registry adoption): the tail is rebuilt from the snapshot
    }
    const double tg0 = now_ms();
    if (apm_service_gram(d_svc_off_, d_svc_ids_, d_active_, cap, cfg_.max_series, cfg_.n_lags,
                         (const double* const*)d_lag_sum_ptrs_, (const double* const*)d_lag_comp_ptrs_,
                         (const int32_t* const*)d_lag_cnt_ptrs_, d_dst, stream) == 0) {
      // series added since the snapshot: a small per-batch CSR of just those series (by service,
      // in series order) accumulated by the same Gram kernel -- the pack stays deterministic
      if (n_series_ > svc_csr_n_ && tail_csr_for_ == std::make_pair(svc_csr_n_, n_series_)) {
        // same tail as the previous pack (no series since): the uploaded lists are still valid
        if (tail_csr_m_)
          apm_service_gram(d_tail_csr_ + tail_csr_m_, d_tail_csr_ + 2 * tail_csr_m_ + 1, d_active_, tail_csr_m_,
                           cfg_.max_series, cfg_.n_lags, (const double* const*)d_lag_sum_ptrs_,
                           (const double* const*)d_lag_comp_ptrs_, (const int32_t* const*)d_lag_cnt_ptrs_, d_dst,
                           stream, d_tail_csr_, 1);
      } else if (n_series_ > svc_csr_n_) {
        // the tail grows with the series table: fold only the series added since the last pack
        if (tail_upto_ < svc_csr_n_) { tail_by_svc_.clear(); tail_upto_ = svc_csr_n_; }
        for (int32_t s = tail_upto_; s < n_series_; ++s) {
          const int32_t v = svc_key(s);
          if (v >= 0 && v < cap) tail_by_svc_[v].push_back(s);
        }
        tail_upto_ = n_series_;
        size_t nt = 0;
        for (const auto& e : tail_by_svc_) nt += e.second.size();
        last_gram_tail_ = (int64_t)nt;
        tail_csr_for_ = {svc_csr_n_, n_series_};
        tail_csr_m_ = 0;
        if (nt) {
          // one pinned block per call: [map m][off m+1][ids nt]; two blocks alternate, so the one
          // written now was last read by the upload two packs ago
          const size_t m = tail_by_svc_.size(), nb = (m + (m + 1) + nt) * 4;
          tail_csr_m_ = (int32_t)m;
          const int k = tail_k_;
          tail_k_ ^= 1;
          if (!tail_csr_ev_[k]) HIP_OK(hipEventCreateWithFlags(&tail_csr_ev_[k], hipEventDisableTiming));
          else HIP_OK(hipEventSynchronize(tail_csr_ev_[k]));
          if (nb > tail_csr_cap_[k]) {
            if (h_tail_csr_[k]) HIP_OK(hipHostFree(h_tail_csr_[k]));
            tail_csr_cap_[k] = nb * 2 + 4096;
            HIP_OK(hipHostMalloc((void**)&h_tail_csr_[k], tail_csr_cap_[k], hipHostMallocDefault));
          }
          if (nb > d_tail_csr_cap_) d_tail_csr_ = (int32_t*)regrow(d_tail_csr_, d_tail_csr_cap_, nb * 2 + 4096);
          int32_t* h = h_tail_csr_[k];
          int32_t* hmap = h;
          int32_t* hoff = h + m;
          int32_t* hids = h + 2 * m + 1;
          size_t r = 0, o = 0;
          for (const auto& e : tail_by_svc_) {
            hmap[r] = e.first;
            hoff[r] = (int32_t)o;
            std::memcpy(hids + o, e.second.data(), e.second.size() * 4);
            o += e.second.size();
            ++r;
          }
          hoff[m] = (int32_t)o;
          HIP_OK(hipMemcpyAsync(d_tail_csr_, h, nb, hipMemcpyHostToDevice, stream));
          HIP_OK(hipEventRecord(tail_csr_ev_[k], stream));
          apm_service_gram(d_tail_csr_ + m, d_tail_csr_ + 2 * m + 1, d_active_, (int32_t)m, cfg_.max_series,
                           cfg_.n_lags, (const double* const*)d_lag_sum_ptrs_, (const double* const*)d_lag_comp_ptrs_,
                           (const int32_t* const*)d_lag_cnt_ptrs_, d_dst, stream, d_tail_csr_, 1);
        }
      }
      trace_event("pack.gram", tg0, now_ms(), 1);
      return;
    }
  }
  apm_service_moments(d_series_service_, d_active_, n_series_, cfg_.max_series, cfg_.n_lags, cap,
                      (const double* const*)d_lag_sum_ptrs_, (const double* const*)d_lag_comp_ptrs_,
                      (const int32_t* const*)d_lag_cnt_ptrs_, d_dst, stream);
}

void Engine::pack_service_moments(double* d_dst, int32_t cap, hipStream_t stream, bool atomic_path) {
  flush();  // series tables are owned by the stats thread
  pack_moments_locked(d_dst, cap, stream, atomic_path);
}

// ---- native fleet exchange + lock-step clocks over RCCL --------------------------------------
// ONE communicator per rank, driven only by the ingest thread on its own stream (coll_stream_).
// Per batch i, every rank issues exactly, in this order:
//   1. (lock-step) all-reduce(MAX) of {watermark, newest bucket} -- 16 B, host waits for it;
//   2. (fleet)     all-reduce(SUM) of the per-service moments of batch i-1 -- async.
// The moments of batch i-1 are packed by the stats thread on the stats stream (pack_ev_), which
// is guaranteed enqueued once post_stats(i) returned.  A single issuing thread per communicator
// and a fixed per-batch sequence make the collective order identical on every rank, whatever
// the thread timing, and no other stream ever waits on a peer (two communicators driven from
// two threads can deadlock once their streams share a hardware queue).  Two device slots: the
// exchange of batch j lands in slot j%2; `fleet_merged` flushes the pending one and reads it.
std::vector<uint8_t> Engine::fleet_unique_id() { return rccl_unique_id(); }

void Engine::fleet_init(const std::vector<uint8_t>& uid, const std::vector<uint8_t>& clock_uid, int nranks, int rank,
                        int32_t cap) {
  flush();
  if (coll_) throw std::runtime_error("fleet_init called twice");
  if (!clock_uid.empty() && clock_uid.size() != uid.size()) throw std::runtime_error("bad unique id size");
  if (cap <= 0) throw std::runtime_error("fleet_init: cap must be > 0");
  HIP_OK(hipSetDevice(cfg_.device));
  coll_ = make_rccl_collective(uid, nranks, rank, cfg_.coll_init_timeout_ms);
  fleet_setup(cap, !clock_uid.empty());
}

void Engine::fleet_init_local(std::shared_ptr<LocalGroup> group, int rank, int32_t cap, bool lockstep) {
  flush();
  if (coll_) throw std::runtime_error("fleet_init called twice");
  if (cap <= 0) throw std::runtime_error("fleet_init: cap must be > 0");
  HIP_OK(hipSetDevice(cfg_.device));
  coll_ = make_local_collective(std::move(group), rank);
  fleet_setup(cap, lockstep);
}

void Engine::fleet_init_host(const std::string& addr, int port, int nranks, int rank, int32_t cap, bool lockstep) {
  flush();
  if (coll_) throw std::runtime_error("fleet_init called twice");
  if (cap <= 0) throw std::runtime_error("fleet_init: cap must be > 0");
  HIP_OK(hipSetDevice(cfg_.device));
  coll_ = make_host_collective(addr, port, nranks, rank, cfg_.coll_timeout_ms);
  fleet_setup(cap, lockstep);
}

void Engine::fleet_setup(int32_t cap, bool lockstep) {
  const int nranks = coll_->nranks();
  // Highest priority: with GPU_MAX_HW_QUEUES = 4 the engine's streams share hardware queues, and
  // the 16-byte clock collective the ingest thread waits for would otherwise queue behind the
  // stats stream's 20 MB st/fs D2H blit.
  int prio_lo = 0, prio_hi = 0;
  HIP_OK(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
  const char* pe = std::getenv("APM_COLL_PRIO");  // diagnostic: 0 = default-priority collective stream
  HIP_OK(hipStreamCreateWithPriority(&coll_stream_, hipStreamNonBlocking, pe && pe[0] == '0' ? prio_lo : prio_hi));
  const char* se = std::getenv("APM_FLEET_SKIP_SOLO");  // diagnostic: skip the one-rank (identity) all-reduce
  fleet_skip_solo_ = nranks == 1 && se && se[0] == '1';
  fleet_nranks_ = nranks;
  lockstep_ = lockstep;
  if (lockstep_) {
    d_sync_ = (double*)dmalloc(64);
    HIP_OK(hipHostMalloc((void**)&h_sync_, 256, hipHostMallocDefault));  // layout: engine.h
    std::memset(h_sync_, 0, 256);
    HIP_OK(hipEventCreateWithFlags(&clock_ev_, hipEventDisableTiming));
    for (hipEvent_t& e : bucket_ev_) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    clock_pending_ = false;
  }
  fleet_cap_ = cap;
  fleet_elems_ = (size_t)cap * MAX_LAGS * NSTAT * 3;  // (capacity: a reload may change the LAG count)
  for (int i = 0; i < 2; ++i) {
    fleet_buf_[i] = (double*)dmalloc(fleet_elems_ * 8);  // zeroed (and synchronised) by dmalloc
    HIP_OK(hipEventCreateWithFlags(&fleet_ev_[i], hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&pack_ev_[i], hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&fb_src_ev_[i], hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&fb_ev_[i], hipEventDisableTiming));
  }
  // fb rows: lowest priority (off every critical path; the output lane drains them)
  HIP_OK(hipStreamCreateWithPriority(&fb_stream_, hipStreamNonBlocking, prio_lo));
  HIP_OK(hipHostMalloc((void**)&h_fb_total_, 16, hipHostMallocDefault));
  fleet_rounds_ = fleet_posted_ = fleet_packed_ = 0;
  if (!lockstep_ && nranks > 1)
    throw std::runtime_error("fleet baseline across ranks needs lock-step rounds (node-wide service registry)");
  d_reg_send_ = (uint8_t*)dmalloc(kRegBlock);
  d_reg_recv_ = (uint8_t*)dmalloc(kRegBlock * (size_t)nranks);
  HIP_OK(hipHostMalloc((void**)&h_reg_send_, kRegBlock, hipHostMallocDefault));
  HIP_OK(hipHostMalloc((void**)&h_reg_recv_, kRegBlock * (size_t)nranks, hipHostMallocDefault));
  fleet_slot_.clear();
  reg_queued_.clear();
  reg_scan_series_ = 0;
  series_service_uploaded_ = 0;  // rows become node-wide slots
  svc_csr_n_ = -1;
  node_mode_ = lockstep_ && cfg_.node_cooldown != 0;
  node_cool_ms_ = cfg_.cooldown_ms;
  if (node_mode_) {
    const size_t per = sizeof(NodeHdr) + (size_t)node_cap_ * sizeof(NodeCand);
    d_node_send_ = (uint8_t*)dmalloc(per);
    d_node_recv_ = (uint8_t*)dmalloc(per * (size_t)nranks);
    HIP_OK(hipHostMalloc((void**)&h_node_send_, per, hipHostMallocDefault));
    HIP_OK(hipHostMalloc((void**)&h_node_recv_, per * (size_t)nranks, hipHostMallocDefault));
    HIP_OK(hipEventCreateWithFlags(&node_ev_, hipEventDisableTiming));
  }
}

// Watchdog for the ingest thread's collectives.  A launch error or an asynchronous RCCL error
// (peer gone, network fault) or a collective still pending after gpu.collectiveTimeoutSeconds
// aborts the communicator (ncclCommAbort unblocks the wedged kernel) and throws: the service
// exits non-zero and the supervisor restarts the whole rank group from its checkpoints, which is
// how the node degrades / recovers instead of hanging every rank forever.
void Engine::coll_wait(hipStream_t s, hipEvent_t ev, const char* what) {
  const double t0 = now_ms();
  for (int spin = 0;; ++spin) {
    const hipError_t e = ev ? hipEventQuery(ev) : hipStreamQuery(s);
    if (e == hipSuccess) return;
    if (e != hipErrorNotReady) HIP_OK(e);
    const std::string ae = coll_->async_error();
    if (!ae.empty()) {
      coll_->abort();
      throw std::runtime_error(std::string("collective ") + what + " failed: " + ae);
    }
    if (now_ms() - t0 > cfg_.coll_timeout_ms) {
      coll_->abort();
      throw std::runtime_error(std::string("RCCL ") + what + ": no completion after " +
                               std::to_string((long long)cfg_.coll_timeout_ms) + " ms (peer rank dead or wedged)");
    }
    // the clock exchange is on the batch's critical path: spin briefly, then back off
    if (spin < 4096) std::this_thread::yield();
    else std::this_thread::sleep_for(std::chrono::microseconds(100));
  }
}

// Lock-step rounds.  Every rank must see the same cache clock per batch (the node-wide
// watermark: the newest leading timestamp any rank has parsed) and roll over on the same batch
// (the node-wide newest bucket of the joined tx), as the single reference parser / stats process
// does (stream_parse_transactions.js:211-239, stream_calc_stats.js:331-371).  Two MAX
// all-reduces per batch on the collective stream, neither of them a barrier on the ingest thread:
//   (1) lockstep_issue, before batch k's join: the watermark through batch k (its parse is done)
//       -- the cache clock of batch k + 1 -- plus "services waiting for a registry slot" and the
//       oldest staged reload.  It runs while the join kernels run; lockstep_collect takes the
//       result after the join, so a peer up to one join behind costs this rank nothing.
//   (2) lockstep_collect, after batch k's join: the newest bucket of batch k's tx.  Only the stats
//       thread waits for it (lockstep_latest, after batch k's bucket appends), right before it
//       decides batch k's rollovers; the ingest thread goes on with batch k + 1.
// The same rounds run at every world size, N = 1 included (MAX over one rank is the identity):
// a one-GPU run pays exactly the per-batch exchanges and waits of each rank of an 8-GPU node.
double Engine::batch_watermark(const ParseSlot& ps) const {
  double w = watermark_;
  const unsigned long long wm = *ps.h_watermark;
  if (wm) {
    const double v = (double)((long long)wm - (1LL << 62));
    if (v > w) w = v;
  }
  return w;
}

void Engine::lockstep_issue(double wm) {
  if (coll_->aborted()) throw std::runtime_error("collective communicator was aborted");
  if (clock_pending_) throw std::runtime_error("lock-step: clock round issued twice");
  // the values travel as kernel arguments: a kernel reading them from pinned memory queues its
  // PCIe read behind the output lane's D2H traffic (tens of us in the bench timeline)
  const double v[4] = {wm, (double)reg_pending_count(), -(double)reconfig_staged_gen(), 0.0};
  apm_set_f64(d_sync_, v, 4, coll_stream_);
  coll_->all_reduce_f64(d_sync_, 4, /*max=*/true, coll_stream_);
  d2h(h_sync_ + 4, d_sync_, 32, coll_stream_);
  HIP_OK(hipEventRecord(clock_ev_, coll_stream_));
  clock_pending_ = true;
}

int Engine::lockstep_collect(int64_t batch_max) {
  const double tl = now_ms();
  if (!clock_pending_) throw std::runtime_error("lock-step: no clock round in flight");
  coll_wait(nullptr, clock_ev_, "lock-step clocks");
  clock_pending_ = false;
  watermark_ = h_sync_[4];  // (>= this rank's own watermark: it was one of the inputs)
  if (h_sync_[6] < 0) reconfig_agree((uint64_t)(-h_sync_[6]));  // every rank has it: same batch everywhere
  if (h_sync_[5] > 0) reg_round();  // every rank sees the same max: all enter the gather
  // the previous batch's node-wide alert gather (issued during this batch's join)
  if (node_round_pending_) {
    coll_wait(nullptr, node_ev_, "node alerts");
    node_resolve();
  }
  const int slot = (int)(batch_no_ & 3);
  const double v[4] = {batch_max == INT64_MIN ? -1.0 : (double)batch_max, 0.0, 0.0, 0.0};  // buckets < 2^53
  apm_set_f64(d_sync_ + 4, v, 4, coll_stream_);
  coll_->all_reduce_f64(d_sync_ + 4, 4, /*max=*/true, coll_stream_);
  d2h(h_sync_ + 8 + 4 * slot, d_sync_ + 4, 32, coll_stream_);
  HIP_OK(hipEventRecord(bucket_ev_[slot], coll_stream_));
  const double te = now_ms();
  metrics_.t_lockstep_ms += te - tl;
  metrics_.t_lockstep_max_ms = std::max(metrics_.t_lockstep_max_ms, te - tl);
  trace_event("lockstep", tl, te, 0);
  return slot;
}

// Stats thread: batch k's node-wide newest bucket (exchange (2) above).
int64_t Engine::lockstep_latest(int slot) {
  const double t0 = now_ms();
  coll_wait(nullptr, bucket_ev_[slot], "lock-step bucket");
  metrics_.t_lockstep_stats_ms += now_ms() - t0;
  const double b = h_sync_[8 + 4 * slot];
  return b >= 0 ? (int64_t)b : INT64_MIN;
}

// Stats thread: every rank rolls over when any rank saw a newer bucket, exactly as the single
// reference stats process rolls over on the first tx of a new bucket from any JVM.
void Engine::apply_latest_locked(int64_t g, double batch_t0) {
  if (g == INT64_MIN || g <= latest_) return;
  latest_ = g;
  ++metrics_.lockstep_rollovers;
  do_rollover(g, batch_t0);
}

// Stats thread: pack this batch's moments into its slot (after the slot's previous all-reduce).
void Engine::fleet_pack_locked() {
  if (!coll_) return;
  const int slot = (int)(fleet_packed_ & 1);
  // The slot's previous all-reduce (batch - 2) has long finished: check it on the host (with the
  // collective watchdog) instead of a device-side wait, so the stats stream never depends on a
  // peer, and pack on the stats stream itself -- a cross-stream wait makes the next enqueue on
  // the waiting stream block the host until the awaited work is done.
  if (fleet_packed_ >= 2) coll_wait(nullptr, fleet_ev_[slot], "fleet slot reuse");
  // a rollover happened since the previous pack: this exchange's merge is that interval's fb
  pack_edge_[slot] = metrics_.rollovers != last_edge_seen_ ? last_edge_ts_ : 0;
  last_edge_seen_ = metrics_.rollovers;
  const double t0 = now_ms();
  // APM_FLEET_ATOMIC=1: the per-series fp64 atomic scatter instead of the MFMA Gram pack (A/B)
  static const bool atomic_pack = [] { const char* x = std::getenv("APM_FLEET_ATOMIC"); return x && x[0] == '1'; }();
  pack_nlags_[slot] = cfg_.n_lags;
  for (int l = 0; l < MAX_LAGS; ++l) pack_lags_[slot][l] = cfg_.lags[l];
  pack_moments_locked(fleet_buf_[slot], fleet_cap_, stream_, atomic_pack);
  trace_event("fleet.pack", t0, now_ms(), 1);
  HIP_OK(hipEventRecord(pack_ev_[slot], stream_));
  ++fleet_packed_;
}

// Ingest thread: all-reduce the packed batches [fleet_rounds_, rounds).
void Engine::fleet_exchange_upto(uint64_t rounds) {
  if (coll_->aborted() && fleet_rounds_ < rounds) throw std::runtime_error("collective communicator was aborted");
  while (fleet_rounds_ < rounds) {
    const int slot = (int)(fleet_rounds_ & 1);
    HIP_OK(hipStreamWaitEvent(coll_stream_, pack_ev_[slot], 0));
    // Only the registered node-wide slots carry moments (identical count on every rank: the
    // registry rounds are collective), not the whole table: 10k services of a 64k-slot table
    // is 1.4 MB on the wire per batch instead of 9.4 MB.
    const size_t per_svc = (size_t)pack_nlags_[slot] * NSTAT * 3;
    const size_t n_red = lockstep_ ? std::min<size_t>(reg_names_.size(), (size_t)fleet_cap_) * per_svc
                                   : (size_t)fleet_cap_ * per_svc;
    if (!fleet_skip_solo_ && n_red) coll_->all_reduce_f64(fleet_buf_[slot], n_red, /*max=*/false, coll_stream_);
    // fb rows: every rank its slice, on the fb stream behind this all-reduce -- the next batch's
    // clock all-reduce on this in-order stream never waits for formatting
    bool fb_queued = false;
    if (pack_edge_[slot] && want(OUT_FB)) {
      HIP_OK(hipEventRecord(fb_src_ev_[slot], coll_stream_));
      fb_queued = fleet_emit_fb(slot);
    }
    // edges are identical on every rank only in lock-step mode (fleet_setup refuses multi-rank
    // without it): the extra all-reduce must never pair with another rank's fleet all-reduce
    if (pack_edge_[slot] && (lockstep_ || fleet_nranks_ == 1)) node_metrics_round();
    // the slot is free again (its next pack may overwrite it) once the all-reduce -- and the fb
    // rows reading it, which wait for the all-reduce -- are done
    HIP_OK(hipEventRecord(fleet_ev_[slot], fb_queued ? fb_stream_ : coll_stream_));
    if (node_mode_) node_round(fleet_rounds_, /*wait=*/false);
    ++fleet_rounds_;
  }
}

void Engine::node_metrics_round() {
  // nm_mu_ is held across harvest and re-launch so node_metrics() never reads h_nm_recv_ while
  // the next copy into it is queued
  std::lock_guard<std::mutex> g(nm_mu_);
  if (!d_nm_) {
    d_nm_ = (double*)dmalloc(kNodeMetrics * 8);
    HIP_OK(hipHostMalloc((void**)&h_nm_send_, kNodeMetrics * 8, hipHostMallocDefault));
    HIP_OK(hipHostMalloc((void**)&h_nm_recv_, kNodeMetrics * 8, hipHostMallocDefault));
    HIP_OK(hipEventCreateWithFlags(&nm_ev_, hipEventDisableTiming));
  } else if (nm_pending_) {
    coll_wait(nullptr, nm_ev_, "node metrics");  // the previous interval's: long done
    node_metrics_.assign(h_nm_recv_, h_nm_recv_ + kNodeMetrics);
    nm_pending_ = false;
  }
  // counters written by other lanes are read as they stand: the element count, not the values,
  // must agree across ranks
  auto ld = [](const uint64_t& x) { return (double)__atomic_load_n(&x, __ATOMIC_RELAXED); };
  const EngineMetrics& m = metrics_;
  const double v[kNodeMetrics] = {1.0, ld(m.batches), ld(m.lines), ld(m.events), ld(m.bytes), ld(m.tx),
                                  ld(m.tx_db), ld(m.released), ld(m.rollovers), ld(m.alert_candidates),
                                  ld(m.alerts), (double)__atomic_load_n(&n_series_, __ATOMIC_RELAXED)};
  std::memcpy(h_nm_send_, v, sizeof v);
  h2d(d_nm_, h_nm_send_, sizeof v, coll_stream_);
  coll_->all_reduce_f64(d_nm_, kNodeMetrics, /*max=*/false, coll_stream_);
  d2h(h_nm_recv_, d_nm_, sizeof v, coll_stream_);
  HIP_OK(hipEventRecord(nm_ev_, coll_stream_));
  nm_pending_ = true;
}

std::vector<double> Engine::node_metrics() {
  std::lock_guard<std::mutex> g(nm_mu_);
  if (nm_pending_ && hipEventQuery(nm_ev_) == hipSuccess) {
    node_metrics_.assign(h_nm_recv_, h_nm_recv_ + kNodeMetrics);
    nm_pending_ = false;
  }
  return node_metrics_;
}

std::vector<double> Engine::fleet_merged() {
  flush();  // every posted batch is packed
  std::vector<double> out;
  if (!coll_) return out;
  fleet_exchange_upto(fleet_posted_);
  if (fleet_rounds_ == 0) return out;
  const int slot = (int)((fleet_rounds_ - 1) & 1);
  coll_wait(nullptr, fleet_ev_[slot], "fleet moments");
  const size_t n = (size_t)fleet_cap_ * pack_nlags_[slot] * NSTAT * 3;  // [cap][n_lags of the pack][NSTAT][3]
  out.resize(n);
  HIP_OK(hipMemcpy(out.data(), fleet_buf_[slot], n * 8, hipMemcpyDeviceToHost));
  return out;
}

// ---- node-wide alert cooldown -------------------------------------------------------------
// The reference has ONE alerts process: a service alerting on two JVMs in the same interval
// yields one alert, the first in the z-score stage's emission order, and the cooldown then
// silences the service everywhere (stream_process_alerts.js:436-468).  With the servers sharded
// over ranks, every rank queues its candidates (flush_alerts) and the ingest thread all-gathers
// them once per exchanged batch (a fixed-size record block per rank, behind the fleet
// all-reduce on the same stream).  A block's header says whether the rank has sent every
// candidate of the batches exchanged so far; once all ranks have, every rank sorts the pooled
// candidates in the global emission order -- (interval edge, server first-batch, node-wide
// server index, service order, LAG) -- and applies the same cooldown map, so all ranks agree and
// each emits the al rows of its own winners.  The gather lands before the next batch's clock
// collective returns (same in-order stream), so the decision costs no extra wait.
void Engine::set_server_index(const std::string& server, int32_t global_index) {
  flush();
  const int32_t id = add_server(server);
  server_gidx_[id] = global_index;
}

void Engine::node_take_text() {
  std::lock_guard<std::mutex> g(node_mu_);
  if (node_text_.empty()) return;
  blob_[OUT_AL] += node_text_;
  node_text_.clear();
}

void Engine::node_round(uint64_t round, bool wait, bool all) {
  if (node_round_pending_) {
    coll_wait(nullptr, node_ev_, "node alerts");
    node_resolve();
  }
  // With the rollover lane a batch's candidates are queued after its stats job: round q carries
  // the candidates of batches <= q - 1 (whose lane work is long done), the drain everything.
  // Every rank uses the same rule, so the pools and decisions stay identical across ranks.
  uint64_t upto = round;
  if (!all && roll_lane_mode_) {
    if (round == 0) upto = UINT64_MAX;  // nothing yet (seq_batch <= -1)
    else upto = round - 1;
  }
  if (upto != UINT64_MAX) wait_roll_round(upto);
  else if (all) wait_roll_round(round);
  const size_t per = sizeof(NodeHdr) + (size_t)node_cap_ * sizeof(NodeCand);
  NodeHdr* hdr = (NodeHdr*)h_node_send_;
  NodeCand* out = (NodeCand*)(h_node_send_ + sizeof(NodeHdr));
  std::memset(hdr, 0, sizeof(NodeHdr));
  {
    std::lock_guard<std::mutex> g(node_mu_);
    int32_t n = 0;
    while (upto != UINT64_MAX && n < node_cap_ && !node_q_.empty() && node_q_.front().seq_batch <= upto) {
      NodePayload& p = node_q_.front();
      out[n++] = p.c;
      if (node_sent_.empty()) node_sent_base_ = p.c.local_id;
      node_sent_.push_back(p);
      node_q_.pop_front();
    }
    hdr->count = n;
    hdr->all_sent = upto == UINT64_MAX || node_q_.empty() || node_q_.front().seq_batch > upto;
  }
  const size_t used = sizeof(NodeHdr) + (size_t)hdr->count * sizeof(NodeCand);
  h2d(d_node_send_, h_node_send_, used, coll_stream_);
  coll_->all_gather(d_node_send_, d_node_recv_, per, coll_stream_);
  // one rank: its own block, of known size (the blocks of other ranks have host-unknown counts:
  // the whole fixed-size block each)
  d2h(h_node_recv_, d_node_recv_, fleet_nranks_ == 1 ? used : per * (size_t)fleet_nranks_, coll_stream_);
  HIP_OK(hipEventRecord(node_ev_, coll_stream_));
  node_round_pending_ = true;
  if (wait) {
    coll_wait(nullptr, node_ev_, "node alerts");
    node_resolve();
  }
}

void Engine::node_resolve() {
  node_round_pending_ = false;
  const size_t per = sizeof(NodeHdr) + (size_t)node_cap_ * sizeof(NodeCand);
  bool all = true;
  for (int r = 0; r < fleet_nranks_; ++r) {
    const NodeHdr* h = (const NodeHdr*)(h_node_recv_ + per * (size_t)r);
    const NodeCand* c = (const NodeCand*)(h_node_recv_ + per * (size_t)r + sizeof(NodeHdr));
    if (h->count < 0 || h->count > node_cap_) throw std::runtime_error("node alerts: corrupt candidate block");
    node_pool_.insert(node_pool_.end(), c, c + h->count);
    all = all && h->all_sent != 0;
  }
  node_all_sent_ = all;
  if (!all) return;  // some rank still holds candidates of an exchanged batch: decide later
  std::sort(node_pool_.begin(), node_pool_.end(), [](const NodeCand& a, const NodeCand& b) {
    if (a.edge_ts != b.edge_ts) return a.edge_ts < b.edge_ts;
    if (a.first_batch != b.first_batch) return a.first_batch < b.first_batch;
    if (a.gidx != b.gidx) return a.gidx < b.gidx;
    if (a.seq != b.seq) return a.seq < b.seq;
    return a.lag_idx < b.lag_idx;
  });
  const int me = coll_->rank();
  std::string text;
  std::vector<const NodePayload*> won;
  std::vector<const NodeCand*> won_c;
  std::vector<std::pair<uint64_t, double>> wins;
  for (const NodeCand& c : node_pool_) {
    auto it = node_cool_.find(c.key);
    if (it != node_cool_.end() && !((c.now - it->second) / 1000.0 > node_cool_ms_ / 1000.0)) continue;
    node_cool_[c.key] = c.now;
    wins.push_back({c.key, c.now});
    if (c.rank != me) continue;
    ++node_alerts_;
    const uint32_t idx = c.local_id - node_sent_base_;
    if (idx >= node_sent_.size()) throw std::runtime_error("node alerts: lost candidate payload");
    won.push_back(&node_sent_[idx]);
    won_c.push_back(&c);
  }
  if (want(OUT_AL) && !won.empty()) {
    std::lock_guard<std::mutex> sg(series_mu_);  // series_ may grow on the stats thread meanwhile
    for (size_t i = 0; i < won.size(); ++i) {
      const NodePayload& q = *won[i];
      const NodeCand& c = *won_c[i];
      const SeriesInfo& si = series_[q.series];
      const std::string& server = servers_[si.server];
      const std::string& service = dict_.service_name(si.service);
      const std::string fs = fmt::fs_line(c.edge_ts, server, service, q.lag, q.w, q.z);
      text += fmt::al_line(c.now, c.edge_ts, server, service, c.causes, fs);
      text += '\n';
    }
  }
  node_pool_.clear();
  node_sent_.clear();  // everything sent so far was in this pool
  if (!wins.empty()) cool_mark(wins, coll_stream_);
  if (!text.empty()) {
    std::lock_guard<std::mutex> g(node_mu_);
    node_text_ += text;
  }
}

void Engine::node_drain() {
  flush();
  if (!coll_ || !node_mode_) return;
  fleet_exchange_upto(fleet_posted_);
  if (node_round_pending_) {
    coll_wait(nullptr, node_ev_, "node alerts");
    node_resolve();
  }
  // every rank computes the same node_all_sent_, so the extra rounds match across ranks
  const uint64_t last = fleet_rounds_ ? fleet_rounds_ - 1 : 0;
  while (!node_all_sent_) node_round(last, /*wait=*/true, /*all=*/true);
  flush();  // folds the decided rows into the al stream
}

}  // namespace apm
