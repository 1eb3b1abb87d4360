// Launch-side API of the CDNA4 kernels: argument structs + host entry points.
// Included by the .hip translation units and by the host runtime (engine.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../apm_types.h"
#include "common.h"

namespace apm {

struct StatsState {
  int32_t* counts;        // [nslot][S]
  int32_t* cells;         // [nslot][S][cap]
  int32_t* spill_n;       // [nslot]
  int32_t* spill_series;  // [nslot][spill_cap]  (sorted by series, stably, before every K8)
  int32_t* spill_val;     // [nslot][spill_cap]
  uint8_t* active;        // [S]
  int32_t cap;
  int32_t spill_cap;
  int32_t S;
  int32_t nslot = NSLOT_MIN;  // bucket ring slots (bucket b lives in slot b % nslot)
  unsigned long long* spill_drop = nullptr;  // [0] samples lost to a full spill list, [1] NaN windows clipped
  // NaN elapsed samples (stream_calc_stats.js:131 pushes parseInt -> NaN): once a series holds one,
  // the JS binaryInsert order of every later sample in its windows matters, so the series' samples
  // are appended in arrival order (not atomic order) while a NaN is live in its window.
  int32_t* nan_until = nullptr;  // [S] last bucket whose window can still see a NaN sample (INT32_MIN = none)
  int32_t* ord_list = nullptr;   // [max_tx] tx indices deferred to the ordered append
  int32_t* ord_n = nullptr;
  uint32_t* ord_done = nullptr;  // blocks of the ordered append finished (the last one resets ord_n)
  int32_t keep = 0;              // windowSz + intervalBufferSz
  // host-mapped pinned [nslot]: spill_n after each append (the host's exact fill level, read once
  // the append's event completed; it sizes the spill area so no sample is ever dropped)
  int32_t* spill_snap = nullptr;
};

struct WindowArgs {
  StatsState st;
  int32_t win_slots[K8_INLINE_SLOTS];  // slot index per window bucket (-1 = bucket absent), n_win <= 64
  const int32_t* win_slots_ext;        // device [n_win] when n_win > K8_INLINE_SLOTS (else null)
  int32_t n_win;          // windowSizeInIntervals (31 in the shipped config)
  double tpm_div;         // windowSz * intervalLen / 60
  WinStat* out;           // [S]
  int32_t* big_list;      // series deferred to the block pass
  int32_t* big_n;
  int32_t* nan_list;      // series whose window holds a NaN sample (JS insertion emulation)
  int32_t* nan_n;
  int32_t* js_scratch;    // [JS_BLOCKS][js_cap] ordered window samples of a NaN series
  int32_t js_cap;
  int32_t n_series;       // ids < n_series may be active
  int32_t lds_sort;       // APM_K8_LDS=1: the LDS bitonic for every window (A/B of the register sort)
};
constexpr int JS_BLOCKS = 8;

struct ZArgs {
  void* ring;              // [NSTAT][LAG][S] of T for this lag
  int32_t* len;            // [S]
  double* sum;             // [NSTAT][S]
  double* comp;            // [NSTAT][S]
  int32_t* cnt;            // [NSTAT][S]
  double* sumsq;           // [NSTAT][S]
  double* sqcomp;          // [NSTAT][S]
  const double* thr;       // [S]
  const double* infl;      // [S]
  const WinStat* win;      // [S]
  ZOut* out;               // [S]
  int32_t S;
  int32_t n_series;
  int32_t lag;
  int32_t head;            // write position this rollover
  int32_t exact;           // 1 = sequential mean every time
  int32_t sigma_stddev;    // 0 = sqrt(mean) quirk, 1 = population sigma
  int32_t resync_k;        // rolling mode: exact resync period (0 = never)
  int64_t rollover_idx;
  // rolling-mode resync range of this rollover (host computes it; rs_n = 0 -> none)
  int32_t rs_lo, rs_n, rs_parts;
  int32_t rs_mfma;         // 1: window re-sum as MFMA tile reductions (k_zscore_resync_mfma)
  double* rs_part;         // [NSTAT][rs_parts][rs_n][4] partial (sum, comp, sumsq, sqcomp)
  int32_t* rs_cnt;         // [NSTAT][rs_parts][rs_n]
};

// K14 per-JVM rollup fused with exogenous gauges (context.hip)
constexpr int ROLLUP_ACC = 6;    // live series, window tx, window elapsed sum, max p95 bits, #avg sig, #p75 sig
constexpr int ROLLUP_OUT = 15;   // see k_server_fuse
constexpr int CTX_FIELDS = 18;   // [0] gauge ts (ms), [1..16] JmxEntry gauges, [17] VM load
struct RollupArgs {
  const WinStat* win;
  const int32_t* series_server;
  const ZOut* z[MAX_LAGS];
  int32_t n_lags;
  int32_t n_series;
  int32_t n_servers;
  int64_t edge_ts;
  double tpm_div;
  const double* ctx;              // [n_servers][CTX_FIELDS]
  unsigned long long* acc;        // [n_servers][ROLLUP_ACC]
  double* out;                    // [n_servers][ROLLUP_OUT]
};

// apm_copy_segs: up to 8 device -> device / host-mapped copies in one launch (stats.hip)
struct CopySeg {
  void* dst;
  const void* src;
  size_t bytes;
};
struct CopySegs {
  CopySeg seg[8];
  int32_t n = 0;
  void add(void* d, const void* s, size_t b) {
    if (b) seg[n++] = CopySeg{d, s, b};
  }
};

// apm_export: device scalars -> pinned host memory (stats.hip)
struct ExportArgs {
  static constexpr int kMax = 8;
  void* src[kMax];  // device scalars
  void* dst[kMax];  // device views of pinned host memory
  uint64_t reset_val[kMax];
  uint8_t bytes[kMax];  // 4 or 8
  uint8_t reset[kMax];
  int32_t n;
  void add(void* s, void* d, int nb, bool rst = false, uint64_t rv = 0) {
    src[n] = s; dst[n] = d; bytes[n] = (uint8_t)nb; reset[n] = rst ? 1 : 0; reset_val[n] = rv; ++n;
  }
};

// K12 st/fs encoding (format.hip)
struct FormatArgs {
  const int32_t* perm;          // [n] series in emission order
  const WinStat* win;           // [S]
  const ZOut* z[MAX_LAGS];      // [S] per lag
  const int4* series_names;     // [S] {server off, len, service off, len} into `names`
  const char* names;
  int64_t edge_ts;
  int32_t n;
  int32_t n_lags;
  int32_t lag_order[MAX_LAGS];  // ascending LAG value
  int32_t lag_value[MAX_LAGS];
  int32_t want_st, want_fs;
  // fs as Postgres COPY rows (the DB sink's K13 encoding fused into K12): the fs stream then
  // carries `timestamp \t server \t service \t tpm \t lag \t stats-json` rows (copyenc.cpp)
  int32_t fs_copy;
  uint32_t stage_hint;  // bytes of an average 64-line block of the longer stream (previous batch); 0 = unknown
  int32_t ts_copy_len;
  char ts_copy[32];        // edge_ts as 'YYYY-MM-DD HH:MM:SS.mmm+00'
  int32_t ts_wire_len;
  char ts_wire[24];        // "<edge_ts>|" as the wire lines' second field (printed once, on the host)
  uint32_t *st_len, *fs_len, *st_off, *fs_off;  // st [n + 1], fs per (series, LAG) line [n * n_lags + 1]
  char *st_out, *fs_out;
  int32_t* fallback;
};

// fb rows: the fleet-merged per-service baseline (all ranks' series of a service), one row per
// (service slot, LAG) with a baseline, after the moments all-reduce (format.hip).  Every rank
// formats the rows of its own slice of the slots [slot_lo, slot_lo + n_slots).
struct FleetFormatArgs {
  const double* moments;   // [cap][n_lags][NSTAT][3] {n, sum of means, sum of squared means}
  const int2* names;       // [all slots] {offset, length} into chars
  const char* chars;
  int32_t slot_lo, n_slots, n_lags;
  int32_t lag_order[MAX_LAGS], lag_value[MAX_LAGS];
  int64_t edge_ts;
  int32_t copy;            // 1: Postgres COPY rows (apm_fleet_stats), 0: fb wire lines
  int32_t ts_len;
  char ts[32];
  unsigned long long* status;  // [blocks] each 64-row wave's byte total (k_fleet_len)
  uint32_t* total;         // bytes written (device)
  char* out;
  int32_t* fallback;
};
struct AlertArgs {
  const WinStat* win;         // [S]
  const ZOut* z;              // [S] for this lag
  int32_t* counter;           // [S] leaky counter for this lag
  const double* hard_max;     // [S] per-series effective hardMaxMsAlertThreshold
  const uint8_t* suppressed;  // [S] service in suppressedServices
  const uint64_t* emit_key;   // [S]
  AlertRec* out;
  int32_t* n_out;
  int32_t n_series;
  int32_t lag_idx;
  int32_t n_lags;
  int32_t lag_suppressed;
  int32_t window;             // rollingAlertWindowSizeInIntervals
  int32_t threshold;          // requiredNumberBadIntervalsInAlertWindowToTrigger
  double hard_min_ms;
  double hard_min_tpm;
  int32_t both_only;
  int32_t max_out;
  // Device-side cooldown pre-filter: time of the latest alert of the series' cooldown key (NaN:
  // none).  A candidate the host's cooldown would certainly suppress -- same expression, same
  // `now` -- is not emitted (cooldown times only grow, so a stale value can only let through a
  // candidate the host then suppresses).  An alert storm otherwise ships ~20k candidates per
  // rollover to the host decision.
  const double* cool_t;       // [S] or nullptr
  double now;
  double cool_s;              // cooldown in seconds (perServiceAlertCooldownInMinutes * 60)
};

}  // namespace apm

extern "C" {
// parse.hip
size_t apm_parse_workspace_bytes(uint64_t max_bytes, uint32_t max_lines, uint32_t max_chunks);
int apm_parse_batch(const uint8_t* d_bytes, uint64_t n_bytes, const uint32_t* d_chunk_begin,
                    const uint8_t* d_chunk_kind, const uint32_t* d_chunk_file, uint32_t n_chunks,
                    void* d_ws, uint32_t max_lines, apm::Event* d_events, uint32_t* d_n_events,
                    uint32_t* d_n_lines, unsigned long long* d_watermark, uint8_t* d_file_open,
                    const apm::TzTable* tz, hipStream_t stream);
// stats.hip
// checkpoint: occupied cells of k bucket slots packed on the device (entry i * n + s = slot
// d_slots[i], series s); offs[k * n] = total cells.  lens / offs: k * n + 1 entries.
size_t apm_ck_pack_tmp_bytes(uint64_t n_entries);
int apm_ck_pack_cells(const int32_t* counts, const int32_t* cells, const int32_t* d_slots, int k, int32_t n, int32_t S,
                      int32_t cap, uint32_t* lens, uint32_t* offs, void* tmp, size_t tmp_bytes, int32_t* packed,
                      hipStream_t s);
void apm_stats_clear_slot(apm::StatsState* st, int slot, hipStream_t stream);
void apm_bucket_append(const apm::TxRec* d_tx, uint32_t lo, uint32_t hi, apm::StatsState* st,
                       int64_t min_live_bucket, hipStream_t stream);
// marks series with a NaN elapsed sample in tx[0, n) (before any of the batch is appended)
void apm_nan_mark(const apm::TxRec* d_tx, uint32_t n, apm::StatsState* st, hipStream_t stream);
void apm_window_stats(apm::WindowArgs* a, hipStream_t stream);
// before K8: every slot's spill list [slot * cap, + spill_n[slot]) sorted by series, stably (a
// series' samples keep their arrival order), into (series_out, val_out); the caller swaps buffers
size_t apm_spill_sort_tmp_bytes(int32_t spill_cap, int32_t S, int32_t nslot);
int apm_spill_sort(const apm::StatsState* st, int32_t* series_out, int32_t* val_out, void* tmp, size_t tmp_bytes,
                   hipStream_t stream);
void apm_pool_append(const apm::TxRec* d_tx, uint32_t lo, uint32_t hi, const int64_t* d_gid, int64_t* tail_end,
                     int64_t* tail_gid, int64_t base, hipStream_t stream);
size_t apm_release_tmp_bytes(int64_t cap);
int apm_release_merge(const int64_t* pool_end, const int64_t* pool_gid, int64_t n_pool, const int64_t* tail_end,
                      const int64_t* tail_gid, int64_t n_tail, int64_t* sort_end, int64_t* sort_gid,
                      int64_t* out_end, int64_t* out_gid, void* tmp, size_t tmp_bytes, hipStream_t stream);
// device scalars (4 or 8 bytes) -> host-mapped pinned memory, optional device reset afterwards
void apm_export(const apm::ExportArgs* a, hipStream_t stream);
// copy by a kernel (src / dst may be device views of pinned host memory): ordered on `stream`,
// never blocks the calling thread
void apm_copy(void* dst, const void* src, size_t bytes, hipStream_t stream);
// the same on at most `max_blocks` workgroups of 256 (a host-link copy that leaves the CUs to
// the kernels running beside it)
void apm_copy_capped(void* dst, const void* src, size_t bytes, uint32_t max_blocks, hipStream_t stream);
void apm_copy_segs(const apm::CopySegs* c, hipStream_t stream);
// up to 8 doubles -> device memory, passed as kernel arguments (nothing read over the host link)
void apm_set_f64(double* dst, const double* vals, int n, hipStream_t stream);
// zscore.hip
void apm_zscore(apm::ZArgs* a, int dtype_bytes, hipStream_t stream);
void apm_zscore_warm(apm::ZArgs* a, int dtype_bytes, int fill, uint64_t seed, const apm::WinStat* base,
                     hipStream_t stream);
void apm_server_rollup(apm::RollupArgs* a, hipStream_t stream);
size_t apm_format_tmp_bytes(int32_t n_max);
void apm_format_fixed_batch(const double* d_x, int n, int f, char* d_out, hipStream_t stream);
int apm_format_plan(apm::FormatArgs* a, void* tmp, size_t tmp_bytes, hipStream_t stream);
void apm_format_write(apm::FormatArgs* a, hipStream_t stream);
void apm_alert_eval(apm::AlertArgs* a, hipStream_t stream);
// dst[idx[i]] = val[i]; idx / val may be device views of pinned host memory
void apm_scatter_f64(double* dst, const int32_t* idx, const double* val, int32_t n, hipStream_t stream);
// blocks of the one-pass fb formatter for `n_rows` rows (the status array's length)
uint32_t apm_fleet_format_blocks(int32_t n_rows);
void apm_fleet_format(apm::FleetFormatArgs* a, hipStream_t stream);
// after K11: the candidate count (clamped to max_n), the candidates and -- rows != 0 -- their window
// stats and candidate-LAG z-score rows, written into host-mapped pinned buffers (device pointers
// of hipHostMalloc memory) in candidate order
void apm_alert_gather(const apm::AlertRec* alerts, const int32_t* n_dev, int32_t max_n, const apm::WinStat* win,
                      const apm::ZOut* const* z_by_lag, int32_t n_lags, int32_t rows, apm::AlertRec* alerts_out,
                      apm::WinStat* win_out, apm::ZOut* z_out, int32_t* n_out, hipStream_t stream);
// fleet.hip
void apm_service_moments(const int32_t* series_service, const uint8_t* active, int32_t n_series, int32_t S,
                         int32_t n_lags, int32_t n_services_cap, const double* const* sums, const double* const* comps,
                         const int32_t* const* cnts, double* dst, hipStream_t stream);
void apm_service_moments_tail(const int32_t* series_service, const uint8_t* active, int32_t s_lo, int32_t n_series,
                              int32_t S, int32_t n_lags, int32_t n_services_cap, const double* const* sums,
                              const double* const* comps, const int32_t* const* cnts, double* dst,
                              hipStream_t stream);
int apm_service_gram(const int32_t* svc_off, const int32_t* svc_ids, const uint8_t* active, int32_t n_services,
                     int32_t S, int32_t n_lags, const double* const* sums, const double* const* comps,
                     const int32_t* const* cnts, double* dst, hipStream_t stream, const int32_t* svc_map = nullptr,
                     int32_t accumulate = 0);
}
