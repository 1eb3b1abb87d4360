// K7 bucket append, K8 window statistics, K9 ordered release.
//
// Reference behaviour: stream_calc_stats.js addData (:115-134), removeOldBuckets (:103-113),
// generateAllStatsToQueue (:157-203) with util_methods.js calcPercentile (:112-142), and the
// min-heap release writeHeapToQueue (:136-155) / binary_heap.js popAllLessOrEqualToScore.
//
// Layout (MI355X): samples live in a per-series ring of `nslot` ten-second bucket cells (config-
// sized, >= window + buffer + 1; 40 by default), cells[slot][series][CAP] (int32 elapsed ms) +
// counts[slot][series]; a live bucket b sits in slot b % nslot (at most window + buffer + 1
// buckets are live, so slots never alias).  Appends are one atomicAdd
// per sample into the cell (overflow beyond CAP goes to a per-slot spill list).  At a rollover
// every active series is reduced by one wave: the 31 window cells are gathered into LDS, summed,
// bitonic-sorted in LDS and the two percentile ranks read out with the reference index rule.
// Series too large for a wave's LDS tile are deferred to a block-wide pass.
// Spill lists: the reference window is an unbounded array (stream_calc_stats.js:127-131), so the
// host sizes the spill area from the device's exact fill levels before every append and never
// lets a sample be lost; before K8 every list is sorted by series (stable, rocprim segmented
// radix sort), so a series' spilled samples are one contiguous run found by binary search
// instead of a scan of the whole list per series.
#include "kernel_api.h"

#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <cstdlib>

namespace apm {

constexpr int WS_WAVES = 4;              // waves per block in the window kernel
constexpr int WS_TILE = 1024;            // samples per wave held in LDS
constexpr int BIG_TILE = 16384;          // samples per block in the large-series pass (64 KiB)

// slot of window bucket r (kernel arguments for the first K8_INLINE_SLOTS, then a device array)
__device__ __forceinline__ int win_slot(const WindowArgs& a, int r) {
  return r < K8_INLINE_SLOTS ? a.win_slots[r] : a.win_slots_ext[r];
}


// --------------------------------------------------------------------------------- K7
// Appends tx[lo, hi) to their bucket cells. `slot_of` maps (bucket - slot_base) -> slot or -1
// (bucket already deleted: the sample is dropped but the series still becomes active, as in
// the reference where the late bucket is re-created and deleted at the next rollover).
__global__ void k_bucket_append(const TxRec* __restrict__ tx, uint32_t lo, uint32_t hi, StatsState st,
                                int64_t min_live_bucket) {
  const uint32_t i = lo + blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= hi) return;
  const TxRec r = tx[i];
  if (r.series < 0 || r.series >= st.S) return;
  st.active[r.series] = 1;
  const int64_t b = r.end_ms / 10000;  // endTs string minus its last 4 digits
  if (b < min_live_bucket) return;
  // NaN samples are kept (sentinel ELAPSED_NAN): they count toward tpm and poison the average
  if (st.nan_until && b <= (int64_t)st.nan_until[r.series]) {
    st.ord_list[atomicAdd(st.ord_n, 1)] = (int32_t)i;  // arrival order matters: ordered pass
    return;
  }
  const int slot = (int)(b % st.nslot);
  const size_t cidx = (size_t)slot * st.S + r.series;
  const int k = atomicAdd(&st.counts[cidx], 1);
  if (k < st.cap) {
    st.cells[cidx * st.cap + k] = r.elapsed;
  } else {
    const int j = atomicAdd(&st.spill_n[slot], 1);
    if (j < st.spill_cap) {
      st.spill_series[(size_t)slot * st.spill_cap + j] = r.series;
      st.spill_val[(size_t)slot * st.spill_cap + j] = r.elapsed;
    } else {
      // spill list full: the sample is lost -- take it back out of the cell count, so the
      // count K8 trusts stays the number of stored samples (never reads unwritten positions)
      atomicSub(&st.counts[cidx], 1);
      if (st.spill_drop) atomicAdd(st.spill_drop, 1ULL);
    }
  }
}

__global__ void k_nan_mark(const TxRec* __restrict__ tx, uint32_t n, StatsState st) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const TxRec r = tx[i];
  if (r.elapsed != ELAPSED_NAN || r.series < 0 || r.series >= st.S) return;
  atomicMax(&st.nan_until[r.series], (int32_t)(r.end_ms / 10000) + st.keep);
}

// Ordered append of the deferred tx (series with a live NaN): one block sorts the deferred
// entries by (cell, tx index) in LDS, so every cell receives its samples in arrival order and
// the spill entries of one run are reserved contiguously.  Entries are taken in tx-index ranges
// that hold at most ORD_TILE of them (indices are unique), processed in index order.
constexpr int ORD_TILE = 4096;
__global__ __launch_bounds__(1024) void k_bucket_append_ordered(const TxRec* __restrict__ tx, uint32_t lo, uint32_t hi,
                                                               StatsState st) {
  __shared__ unsigned long long key[ORD_TILE];
  __shared__ int32_t pos[ORD_TILE];
  __shared__ int32_t sp0[ORD_TILE];
  __shared__ int m_sh;
  // Cells are partitioned over the blocks (cell % gridDim.x): a cell's samples, their order and
  // their spill run all belong to one block, so the blocks sort and place independently (one
  // block for every cell cost 60-70 us a call -- a serial tail on the stats stream).
  const int n_ord = *st.ord_n;
  if (n_ord == 0) {
    // every append of this call is done (stream order): publish the fill levels to the host
    if (blockIdx.x == 0 && st.spill_snap)
      for (int k = threadIdx.x; k < st.nslot; k += blockDim.x) st.spill_snap[k] = st.spill_n[k];
    return;
  }
  const uint32_t G = gridDim.x, blk = blockIdx.x;
  const uint32_t span = hi - lo;
  // this block's entries: all in one pass when they fit the LDS tile (nearly always: ~n_ord / G),
  // else in tx-index ranges of ORD_TILE (a range holds at most ORD_TILE entries)
  if (threadIdx.x == 0) m_sh = 0;
  __syncthreads();
  {
    int mine = 0;
    for (int j = threadIdx.x; j < n_ord; j += blockDim.x) {
      const TxRec r = tx[st.ord_list[j]];
      const uint32_t cell = (uint32_t)((r.end_ms / 10000) % st.nslot) * (uint32_t)st.S + (uint32_t)r.series;
      mine += cell % G == blk;
    }
    if (mine) atomicAdd(&m_sh, mine);
  }
  __syncthreads();
  const uint32_t R = m_sh <= ORD_TILE ? span : (uint32_t)ORD_TILE;
  __syncthreads();
  for (uint32_t r0 = 0; r0 < span; r0 += R) {
    if (threadIdx.x == 0) m_sh = 0;
    __syncthreads();
    for (int j = threadIdx.x; j < n_ord; j += blockDim.x) {
      const uint32_t i = (uint32_t)st.ord_list[j];
      if (i - lo >= r0 && i - lo < r0 + R) {
        const TxRec r = tx[i];
        const uint32_t cell = (uint32_t)((r.end_ms / 10000) % st.nslot) * (uint32_t)st.S + (uint32_t)r.series;
        if (cell % G == blk) key[atomicAdd(&m_sh, 1)] = ((unsigned long long)cell << 32) | i;
      }
    }
    __syncthreads();
    const int m = m_sh;
    if (m == 0) continue;  // uniform
    int np2 = 1;
    while (np2 < m) np2 <<= 1;
    for (int k = m + threadIdx.x; k < np2; k += blockDim.x) key[k] = ~0ULL;
    __syncthreads();
    for (int k = 2; k <= np2; k <<= 1)
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = threadIdx.x; i < np2; i += blockDim.x) {
          const int ixj = i ^ j;
          if (ixj > i) {
            const unsigned long long x = key[i], y = key[ixj];
            if ((x > y) == ((i & k) == 0)) { key[i] = y; key[ixj] = x; }
          }
        }
        __syncthreads();
      }
    // position of every entry = cell count before this range + rank inside its run
    for (int k = threadIdx.x; k < m; k += blockDim.x) {
      const uint32_t cell = (uint32_t)(key[k] >> 32);
      int a = 0, b = k;  // first index of the run
      while (a < b) { const int mid = (a + b) >> 1; if ((uint32_t)(key[mid] >> 32) < cell) a = mid + 1; else b = mid; }
      pos[k] = st.counts[cell] + (k - a);
    }
    __syncthreads();
    // run heads publish the new count and reserve the run's spill entries in one piece
    for (int k = threadIdx.x; k < m; k += blockDim.x) {
      const uint32_t cell = (uint32_t)(key[k] >> 32);
      if (k > 0 && (uint32_t)(key[k - 1] >> 32) == cell) continue;
      int a = k, b = m;  // one past the run
      while (a < b) { const int mid = (a + b) >> 1; if ((uint32_t)(key[mid] >> 32) <= cell) a = mid + 1; else b = mid; }
      const int base = pos[k], end = base + (a - k);
      st.counts[cell] = end;
      const int first_sp = max(base, st.cap);
      sp0[k] = end > first_sp ? atomicAdd(&st.spill_n[cell / (uint32_t)st.S], end - first_sp) - first_sp : 0;
      // a full spill list drops the run's tail (spill index sp0 + p >= spill_cap): the cell keeps
      // the count of the samples actually stored (see k_bucket_append)
      if (end > first_sp) {
        const int stored_end = max(first_sp, min(end, st.spill_cap - sp0[k]));
        if (stored_end < end) st.counts[cell] = stored_end;
      }
    }
    __syncthreads();
    for (int k = threadIdx.x; k < m; k += blockDim.x) {
      const uint32_t cell = (uint32_t)(key[k] >> 32);
      const uint32_t i = (uint32_t)key[k];
      const int p = pos[k];
      const int32_t v = tx[i].elapsed;
      if (p < st.cap) {
        st.cells[(size_t)cell * st.cap + p] = v;
      } else {
        int a = 0, b = k;
        while (a < b) { const int mid = (a + b) >> 1; if ((uint32_t)(key[mid] >> 32) < cell) a = mid + 1; else b = mid; }
        const int slot = (int)(cell / (uint32_t)st.S);
        const int j = sp0[a] + p;
        if (j < st.spill_cap) {
          st.spill_series[(size_t)slot * st.spill_cap + j] = (int32_t)(cell % (uint32_t)st.S);
          st.spill_val[(size_t)slot * st.spill_cap + j] = v;
        } else if (st.spill_drop) {
          atomicAdd(st.spill_drop, 1ULL);
        }
      }
    }
    __threadfence();
    __syncthreads();
  }
  // the last block to finish resets the count for the next append and publishes the fill levels
  __shared__ bool last;
  if (threadIdx.x == 0) {
    __threadfence();
    last = atomicAdd(st.ord_done, 1u) == G - 1;
  }
  __syncthreads();
  if (!last) return;
  if (threadIdx.x == 0) {
    *st.ord_n = 0;
    *st.ord_done = 0;
  }
  if (st.spill_snap)
    for (int k = threadIdx.x; k < st.nslot; k += blockDim.x) st.spill_snap[k] = atomicAdd(&st.spill_n[k], 0);
}

__global__ void k_clear_slot(StatsState st, int slot) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < (uint32_t)st.S) st.counts[(size_t)slot * st.S + i] = 0;
  if (i == 0) st.spill_n[slot] = 0;
}

// --------------------------------------------------------------------------------- K8
// first position of series s in a slot's sorted spill list [0, n)
__device__ __forceinline__ int spill_lower(const int32_t* keys, int n, int32_t s) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (keys[mid] < s) lo = mid + 1; else hi = mid;
  }
  return lo;
}
// the run of series s's spilled samples in slot sl: [*first, *first + cnt - cap)
__device__ __forceinline__ const int32_t* spill_run(const StatsState& st, int sl, int s) {
  const size_t base = (size_t)sl * st.spill_cap;
  const int ns = min(st.spill_n[sl], st.spill_cap);
  return st.spill_val + base + spill_lower(st.spill_series + base, ns, s);
}

__device__ __forceinline__ void percentile_ranks(int n, int pct, int& lo, int& hi) {
  // calcPercentile: idx = p/100*n - 1; integral -> a[idx]; else ceil, last -> a[last],
  // otherwise (a[i] + a[i+1]) / 2.  Computed in double exactly as JS does.
  if (n <= 0) { lo = hi = -1; return; }
  const double idx = ((double)pct / 100.0) * (double)n - 1.0;
  if (n == 1 || idx == floor(idx)) { lo = hi = (int)idx; return; }
  const int i = (int)ceil(idx);
  lo = i;
  hi = (i == n - 1) ? i : i + 1;
}

__device__ __forceinline__ double pct_value(const int32_t* a, int lo, int hi) {
  if (lo < 0) return apm_nan();
  if (lo == hi) return (double)a[lo];
  return ((double)a[lo] + (double)a[hi]) / 2.0;
}

// Bitonic sort of n (power of two) ints in LDS by the lanes of one wave.
__device__ inline void wave_bitonic(int32_t* a, int n, int lane) {
  for (int k = 2; k <= n; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = lane; i < n; i += APM_WAVE) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const int32_t x = a[i], y = a[ixj];
          const bool up = (i & k) == 0;
          if ((x > y) == up) { a[i] = y; a[ixj] = x; }
        }
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    }
  }
}

__device__ __forceinline__ void finish_series(const WindowArgs& a, int s, int n, long long sum,
                                              const int32_t* sorted) {
  WinStat w;
  w.n = n;
  w.active = 1;
  w.tpm = js_round_fixed((double)n / a.tpm_div, 2);
  if (n > 0) {
    int lo, hi;
    w.avg = js_round_fixed((double)sum / (double)n, 1);
    percentile_ranks(n, 75, lo, hi);
    w.p75 = js_round_fixed(pct_value(sorted, lo, hi), 1);
    percentile_ranks(n, 95, lo, hi);
    w.p95 = js_round_fixed(pct_value(sorted, lo, hi), 1);
  } else {
    w.avg = w.p75 = w.p95 = apm_nan();
  }
  a.out[s] = w;
}

__global__ __launch_bounds__(WS_WAVES * APM_WAVE) void k_window_stats(WindowArgs a) {
  __shared__ int32_t tile[WS_WAVES][WS_TILE];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int s = blockIdx.x * WS_WAVES + wv;
  if (s >= a.n_series) return;
  if (!a.st.active[s]) {
    if (lane == 0) { WinStat w{}; w.active = 0; w.n = 0; a.out[s] = w; }
    return;
  }
  if (a.n_win > APM_WAVE) {  // a window longer than the wave (> 640 s): the block pass loops over its buckets
    if (lane == 0) { const int j = atomicAdd(a.big_n, 1); a.big_list[j] = s; }
    return;
  }
  // per-window-bucket counts (lane r handles window bucket r)
  int cnt = 0, slot = -1;
  if (lane < a.n_win) {
    slot = a.win_slots[lane];
    if (slot >= 0) cnt = a.st.counts[(size_t)slot * a.st.S + s];
  }
  const int inl = min(cnt, a.st.cap);
  const int spill = cnt - inl;
  // exclusive prefix of inline counts across lanes
  int pre = inl;
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(pre, o, 64);
    if (lane >= o) pre += v;
  }
  const int total_inl = __shfl(pre, 63, 64);
  int total_spill = spill;
  for (int o = 32; o > 0; o >>= 1) total_spill += __shfl_xor(total_spill, o, 64);
  const int n = total_inl + total_spill;
  if (n > WS_TILE) {
    if (lane == 0) { const int j = atomicAdd(a.big_n, 1); a.big_list[j] = s; }
    return;
  }
  int32_t* t = tile[wv];
  pre -= inl;
  long long sum = 0;
  // gather inline samples: every lane copies its own cell (contiguous CAP run)
  int nan = 0;
  if (inl > 0) {
    const int32_t* cell = a.st.cells + ((size_t)slot * a.st.S + s) * a.st.cap;
    for (int k = 0; k < inl; ++k) { const int32_t v = cell[k]; t[pre + k] = v; sum += v; nan += v == ELAPSED_NAN; }
  }
  // spilled samples: each window bucket's run in its slot's sorted spill list (binary search by
  // the lane owning the bucket), copied by the whole wave
  if (total_spill > 0) {
    const int32_t* run = spill > 0 ? spill_run(a.st, slot, s) : nullptr;
    int spre = spill;
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(spre, o, 64);
      if (lane >= o) spre += v;
    }
    spre -= spill;
    __builtin_amdgcn_wave_barrier();
    unsigned long long todo = __ballot(spill > 0);
    while (todo) {
      const int r = __ffsll((long long)todo) - 1;
      todo &= todo - 1;
      const int m = __shfl(spill, r, 64);
      const int off = total_inl + __shfl(spre, r, 64);
      const uintptr_t rp = (uintptr_t)__shfl((long long)(uintptr_t)run, r, 64);
      const int32_t* src = (const int32_t*)rp;
      for (int k = lane; k < m; k += 64) {
        const int32_t v = src[k];
        t[off + k] = v;
        sum += v;
        nan += v == ELAPSED_NAN;
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
  for (int o = 32; o > 0; o >>= 1) nan += __shfl_xor(nan, o, 64);
  if (nan > 0) {  // NaN in the window: JS insertion order decides the percentiles
    if (lane == 0) a.nan_list[atomicAdd(a.nan_n, 1)] = s;
    return;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  if (n <= APM_WAVE && !a.lds_sort) {
    // The usual window (~20 samples): one sample per lane, a bitonic network over the lanes in
    // registers -- 21 shuffle + min/max steps, no LDS round trips or wave barriers (the LDS
    // network padded every series to 64 and cost 21 LDS passes; profiles/r4_pm: 100 us per
    // rollover at 19 % L2 hit).  The percentile ranks are read back by shuffles.
    int32_t v = lane < n ? t[lane] : 0x7fffffff;
#pragma unroll
    for (int k = 2; k <= APM_WAVE; k <<= 1) {
#pragma unroll
      for (int j = k >> 1; j > 0; j >>= 1) {
        const int32_t o = __shfl_xor(v, j, APM_WAVE);
        const bool keep_min = ((lane & j) == 0) == ((lane & k) == 0);
        v = keep_min ? min(v, o) : max(v, o);
      }
    }
    int l75, h75, l95, h95;
    percentile_ranks(n, 75, l75, h75);
    percentile_ranks(n, 95, l95, h95);
    const int32_t a75 = __shfl(v, max(l75, 0), APM_WAVE), b75 = __shfl(v, max(h75, 0), APM_WAVE);
    const int32_t a95 = __shfl(v, max(l95, 0), APM_WAVE), b95 = __shfl(v, max(h95, 0), APM_WAVE);
    if (lane == 0) {
      WinStat w;
      w.n = n;
      w.active = 1;
      w.tpm = js_round_fixed((double)n / a.tpm_div, 2);
      if (n > 0) {
        w.avg = js_round_fixed((double)sum / (double)n, 1);
        w.p75 = js_round_fixed(l75 == h75 ? (double)a75 : ((double)a75 + (double)b75) / 2.0, 1);
        w.p95 = js_round_fixed(l95 == h95 ? (double)a95 : ((double)a95 + (double)b95) / 2.0, 1);
      } else {
        w.avg = w.p75 = w.p95 = apm_nan();
      }
      a.out[s] = w;
    }
    return;
  }
  // pad to a power of two and sort in LDS
  int np2 = 64;
  while (np2 < n) np2 <<= 1;
  for (int i = n + lane; i < np2; i += 64) t[i] = 0x7fffffff;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  if (n > 1) wave_bitonic(t, np2, lane);
  if (lane == 0) finish_series(a, s, n, sum, t);
}

// K8 for windows of at most 32 buckets (the shipped config: window 31 -> 32 window buckets): two
// series per wave, one per 32-lane half.  Lane r of each half owns window bucket r, so the two
// halves' count and cell loads of a bucket hit adjacent series -- the same cache line -- and the
// prefix scans / sorting network run 32 lanes wide (5 + 15 shuffle steps instead of 6 + 21, each
// step serving two series).  Windows of at most 32 samples (nearly all) are sorted in registers;
// up to 512 by the half in LDS; larger ones go to the block pass, NaN windows to the JS pass.
// APM_K8_H2=0 keeps the one-series-per-wave kernel (A/B).
constexpr int HW = 32;                 // lanes per series
constexpr int H2_TILE = WS_TILE / 2;   // samples per half in LDS

// Cross-lane moves inside a 32-lane half without the LDS crossbar (ds_bpermute): DPP where the
// pattern stays inside a 16-lane row (quad permutes for xor 1 / 2, a quad reversal then
// row_half_mirror for xor 4, row_ror:8 for xor 8, row shifts and row_bcast:15 for scans), and
// ds_swizzle (no LDS bank access, no address VGPR) only for xor 16, the one move between rows.
template <int CTRL, int ROWS = 0xF>
__device__ __forceinline__ int dpp(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, ROWS, 0xF, false); }
template <int J>
__device__ __forceinline__ int32_t half_xor(int32_t v) {
  if constexpr (J == 1) return dpp<0xB1>(v);          // quad_perm [1,0,3,2]
  else if constexpr (J == 2) return dpp<0x4E>(v);     // quad_perm [2,3,0,1]
  else if constexpr (J == 8) return dpp<0x128>(v);    // row_ror:8 == xor 8 inside a row
  else if constexpr (J == 4) return dpp<0x141>(dpp<0x1B>(v));  // quad_perm [3,2,1,0], row_half_mirror: i^3^7
  else return __builtin_amdgcn_ds_swizzle(v, 0x401F);         // BitMode xor 16
}
// inclusive prefix sum over each 32-lane half
__device__ __forceinline__ int half_scan(int x) {
  x += dpp<0x111>(x);        // row_shr:1
  x += dpp<0x112>(x);        // row_shr:2
  x += dpp<0x114>(x);        // row_shr:4
  x += dpp<0x118>(x);        // row_shr:8
  x += dpp<0x142, 0xA>(x);   // row_bcast:15 -> rows 1, 3
  return x;
}
// the same for doubles (exact sums of integers below 2^53): the two words move together
template <int CTRL, int ROWS = 0xF>
__device__ __forceinline__ double dpp_f64(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = dpp<CTRL, ROWS>((int)(b & 0xffffffffll));
  const int hi = dpp<CTRL, ROWS>((int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double half_scan_f64(double x) {
  x += dpp_f64<0x111>(x);
  x += dpp_f64<0x112>(x);
  x += dpp_f64<0x114>(x);
  x += dpp_f64<0x118>(x);
  x += dpp_f64<0x142, 0xA>(x);
  return x;
}
// lane 31 of this half (a half's total after half_scan): two readlanes, no crossbar
__device__ __forceinline__ int half_last(int x, int half) {
  const int a = __builtin_amdgcn_readlane(x, 31), b = __builtin_amdgcn_readlane(x, 63);
  return half ? b : a;
}
__device__ __forceinline__ double half_last_f64(double x, int half) {
  const long long v = __double_as_longlong(x);
  const int lo = half_last((int)(v & 0xffffffffll), half), hi = half_last((int)(v >> 32), half);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
template <int K, int J>
__device__ __forceinline__ int32_t bitonic_step(int32_t v, int hl) {
  const int32_t o = half_xor<J>(v);
  const bool keep_min = ((hl & J) == 0) == ((hl & K) == 0);
  return keep_min ? min(v, o) : max(v, o);
}
template <int K>
__device__ __forceinline__ int32_t bitonic_merge(int32_t v, int hl) {
  if constexpr (K >= 32) v = bitonic_step<K, 16>(v, hl);
  if constexpr (K >= 16) v = bitonic_step<K, 8>(v, hl);
  if constexpr (K >= 8) v = bitonic_step<K, 4>(v, hl);
  if constexpr (K >= 4) v = bitonic_step<K, 2>(v, hl);
  return bitonic_step<K, 1>(v, hl);
}

// Register bitonic sort of a 32-lane half's N = 32 E samples, E per lane.  Index bits 0-3 are the
// lane's position in its 16-lane row (DPP moves), bits 4 .. 3 + log2 E the element (moves inside
// the lane), and the top bit the row (ds_swizzle xor 16): the top bit is compared in one stage
// only, so the network makes E swizzles in all and no LDS access (the LDS form below made ~20
// loads / stores per stage for a 256-sample window).
template <int E>
__device__ __forceinline__ void reg_bitonic(int32_t (&v)[E], int hl) {
  constexpr int N = 32 * E;
  const int base = (hl >> 4) * (16 * E) + (hl & 15);
#pragma unroll
  for (int k = 2; k <= N; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (j >= 16 && j < 16 * E) {
        const int je = j >> 4;
#pragma unroll
        for (int e = 0; e < E; ++e) {
          if (e & je) continue;
          const bool up = ((base + e * 16) & k) == 0;
          const int32_t x = v[e], y = v[e | je];
          v[e] = up ? min(x, y) : max(x, y);
          v[e | je] = up ? max(x, y) : min(x, y);
        }
      } else {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const int i = base + e * 16;
          int32_t o;
          if (j == 1) o = half_xor<1>(v[e]);
          else if (j == 2) o = half_xor<2>(v[e]);
          else if (j == 4) o = half_xor<4>(v[e]);
          else if (j == 8) o = half_xor<8>(v[e]);
          else o = half_xor<16>(v[e]);
          const bool keep_min = ((i & j) == 0) == ((i & k) == 0);
          v[e] = keep_min ? min(v[e], o) : max(v[e], o);
        }
      }
    }
  }
}

// Sorts the half's n (<= 32 E) samples in t[0, n) in place (t holds at least 32 E entries).
template <int E>
__device__ __forceinline__ void half_sort_regs(int32_t* t, int n, int hl) {
  const int base = (hl >> 4) * (16 * E) + (hl & 15);
  int32_t v[E];
#pragma unroll
  for (int e = 0; e < E; ++e) v[e] = base + e * 16 < n ? t[base + e * 16] : 0x7fffffff;
  reg_bitonic<E>(v, hl);
#pragma unroll
  for (int e = 0; e < E; ++e) t[base + e * 16] = v[e];
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
}

__device__ inline void half_bitonic(int32_t* a, int n, int hl) {
  for (int k = 2; k <= n; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = hl; i < n; i += HW) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const int32_t x = a[i], y = a[ixj];
          const bool up = (i & k) == 0;
          if ((x > y) == up) { a[i] = y; a[ixj] = x; }
        }
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    }
  }
}

__global__ __launch_bounds__(WS_WAVES * APM_WAVE) void k_window_stats_h2(WindowArgs a) {
  __shared__ int32_t tile[WS_WAVES * 2][H2_TILE];
  const int lane = threadIdx.x & 63;
  const int half = lane >> 5, hl = lane & (HW - 1);
  const int wv = threadIdx.x >> 6;
  const int s = (blockIdx.x * WS_WAVES + wv) * 2 + half;
  // no early return per half: the shuffles below are 32 lanes wide, and both halves run them
  const bool valid = s < a.n_series;
  const bool active = valid && a.st.active[s];
  if (valid && !active && hl == 0) { WinStat w{}; w.active = 0; w.n = 0; a.out[s] = w; }
  int cnt = 0, slot = -1;
  if (active && hl < a.n_win) {
    slot = a.win_slots[hl];
    if (slot >= 0) cnt = a.st.counts[(size_t)slot * a.st.S + s];
  }
  const int inl = min(cnt, a.st.cap);
  const int spill = cnt - inl;
  int pre = half_scan(inl);
  const int total_inl = half_last(pre, half);
  const int total_spill = half_last(half_scan(spill), half);
  const int n = total_inl + total_spill;
  const bool big = active && n > H2_TILE;
  if (big && hl == 0) { const int j = atomicAdd(a.big_n, 1); a.big_list[j] = s; }
  const bool go = active && !big;
  int32_t* t = tile[wv * 2 + half];
  pre -= inl;
  long long sum = 0;
  int nan = 0;
  if (go && inl > 0) {
    const int32_t* cell = a.st.cells + ((size_t)slot * a.st.S + s) * a.st.cap;
    for (int k = 0; k < inl; ++k) { const int32_t v = cell[k]; t[pre + k] = v; sum += v; nan += v == ELAPSED_NAN; }
  }
  // spilled samples: each window bucket's run found by its lane, copied by the half
  const unsigned long long any_spill = __ballot(go && total_spill > 0);
  if (any_spill) {
    const int32_t* run = go && spill > 0 ? spill_run(a.st, slot, s) : nullptr;
    int spre = half_scan(go ? spill : 0);
    spre -= go ? spill : 0;
    const unsigned long long all = __ballot(go && spill > 0);
    unsigned int todo = (unsigned int)(half ? (all >> 32) : (all & 0xffffffffull));
    __builtin_amdgcn_wave_barrier();
    // (both halves run the loop the larger number of times; a half with nothing left idles)
    const unsigned int other = (unsigned int)(half ? (all & 0xffffffffull) : (all >> 32));
    const int iters = max(__popc(todo), __popc(other));
    for (int it = 0; it < iters; ++it) {
      const int r = todo ? __ffs((int)todo) - 1 : 0;
      const bool mine = todo != 0;
      todo &= todo - 1;
      const int m = __shfl(spill, r, HW);
      const int off = total_inl + __shfl(spre, r, HW);
      const uintptr_t rp = (uintptr_t)__shfl((long long)(uintptr_t)run, r, HW);
      if (mine) {
        const int32_t* src = (const int32_t*)rp;
        for (int k = hl; k < m; k += HW) {
          const int32_t v = src[k];
          t[off + k] = v;
          sum += v;
          nan += v == ELAPSED_NAN;
        }
      }
    }
  }
  // (window sums of int32 samples, at most 512 per half: exact in a double)
  const long long total_sum = (long long)half_last_f64(half_scan_f64((double)sum), half);
  nan = half_last(half_scan(nan), half);
  sum = total_sum;
  const bool has_nan = go && nan > 0;
  if (has_nan && hl == 0) a.nan_list[atomicAdd(a.nan_n, 1)] = s;
  const bool ok = go && !has_nan;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  // register network for n <= 32 (every lane runs it: the shuffles need both halves)
  int32_t v = ok && n <= HW && hl < n ? t[hl] : 0x7fffffff;
  v = bitonic_merge<2>(v, hl);
  v = bitonic_merge<4>(v, hl);
  v = bitonic_merge<8>(v, hl);
  v = bitonic_merge<16>(v, hl);
  v = bitonic_merge<32>(v, hl);
  int l75, h75, l95, h95;
  percentile_ranks(ok && n <= HW ? n : 1, 75, l75, h75);
  percentile_ranks(ok && n <= HW ? n : 1, 95, l95, h95);
  const int32_t a75 = __shfl(v, max(l75, 0), HW), b75 = __shfl(v, max(h75, 0), HW);
  const int32_t a95 = __shfl(v, max(l95, 0), HW), b95 = __shfl(v, max(h95, 0), HW);
  if (!ok) return;
  if (n <= HW) {
    if (hl == 0) {
      WinStat w;
      w.n = n;
      w.active = 1;
      w.tpm = js_round_fixed((double)n / a.tpm_div, 2);
      if (n > 0) {
        w.avg = js_round_fixed((double)sum / (double)n, 1);
        w.p75 = js_round_fixed(l75 == h75 ? (double)a75 : ((double)a75 + (double)b75) / 2.0, 1);
        w.p95 = js_round_fixed(l95 == h95 ? (double)a95 : ((double)a95 + (double)b95) / 2.0, 1);
      } else {
        w.avg = w.p75 = w.p95 = apm_nan();
      }
      a.out[s] = w;
    }
    return;
  }
  // 32 < n <= 512: this half sorts its tile in registers (APM_K8_LDS=2: the LDS network, A/B)
  if (a.lds_sort == 2) {
    int np2 = HW;
    while (np2 < n) np2 <<= 1;
    for (int i = n + hl; i < np2; i += HW) t[i] = 0x7fffffff;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    half_bitonic(t, np2, hl);
  } else if (n <= 2 * HW) {
    half_sort_regs<2>(t, n, hl);
  } else if (n <= 4 * HW) {
    half_sort_regs<4>(t, n, hl);
  } else if (n <= 8 * HW) {
    half_sort_regs<8>(t, n, hl);
  } else {
    half_sort_regs<16>(t, n, hl);
  }
  if (hl == 0) finish_series(a, s, n, sum, t);
}

// Every sample of series s in the window (inline cells + spill lists), visited by the block.
template <class F>
__device__ __forceinline__ void for_each_window_sample(const WindowArgs& a, int s, F&& f) {
  for (int r = 0; r < a.n_win; ++r) {
    const int sl = win_slot(a, r);
    if (sl < 0) continue;
    const int cnt = a.st.counts[(size_t)sl * a.st.S + s];
    const int inl = min(cnt, a.st.cap);
    const int32_t* cell = a.st.cells + ((size_t)sl * a.st.S + s) * a.st.cap;
    for (int k = threadIdx.x; k < inl; k += blockDim.x) f(cell[k]);
    if (cnt > inl) {
      const int32_t* run = spill_run(a.st, sl, s);
      for (int k = threadIdx.x; k < cnt - inl; k += blockDim.x) f(run[k]);
    }
  }
}

// Exact k-th smallest samples for windows beyond BIG_TILE: radix select, 8 bits per pass, the
// up to four ranks of the p75 / p95 formula (percentile_ranks) selected together.  `scratch`
// holds 4 x 256 histogram bins (the LDS tile of the caller).
__device__ void window_select(const WindowArgs& a, int s, int n, long long sum, int32_t* scratch) {
  __shared__ uint32_t prefix[4];
  __shared__ int32_t want[4];
  int ranks[4];
  percentile_ranks(n, 75, ranks[0], ranks[1]);
  percentile_ranks(n, 95, ranks[2], ranks[3]);
  uint32_t* hist = reinterpret_cast<uint32_t*>(scratch);
  if (threadIdx.x < 4) { prefix[threadIdx.x] = 0; want[threadIdx.x] = ranks[threadIdx.x]; }
  __syncthreads();
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    const uint32_t hi_mask = pass == 0 ? 0u : ~((1u << (shift + 8)) - 1u);
    for (int i = threadIdx.x; i < 4 * 256; i += blockDim.x) hist[i] = 0;
    __syncthreads();
    uint32_t pf[4];
    for (int r = 0; r < 4; ++r) pf[r] = prefix[r];
    for_each_window_sample(a, s, [&](int32_t v) {
      const uint32_t u = (uint32_t)v ^ 0x80000000u;  // order-preserving unsigned key
      const uint32_t bin = (u >> shift) & 255u;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if ((u & hi_mask) == (pf[r] & hi_mask)) atomicAdd(&hist[r * 256 + bin], 1u);
    });
    __syncthreads();
    if (threadIdx.x < 4) {
      const int r = threadIdx.x;
      int k = want[r];
      uint32_t b = 0;
      for (; b < 256; ++b) {
        const int c = (int)hist[r * 256 + b];
        if (k < c) break;
        k -= c;
      }
      want[r] = k;
      prefix[r] |= (b & 255u) << shift;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    int32_t val[4];
    for (int r = 0; r < 4; ++r) val[r] = (int32_t)(prefix[r] ^ 0x80000000u);
    WinStat w;
    w.n = n;
    w.active = 1;
    w.tpm = js_round_fixed((double)n / a.tpm_div, 2);
    w.avg = js_round_fixed((double)sum / (double)n, 1);
    w.p75 = js_round_fixed(ranks[0] == ranks[1] ? (double)val[0] : ((double)val[0] + (double)val[1]) / 2.0, 1);
    w.p95 = js_round_fixed(ranks[2] == ranks[3] ? (double)val[2] : ((double)val[2] + (double)val[3]) / 2.0, 1);
    a.out[s] = w;
  }
}

// Large series: one 1024-thread block per deferred series, block-wide bitonic in LDS.
__global__ __launch_bounds__(1024) void k_window_stats_big(WindowArgs a) {
  __shared__ int32_t t[BIG_TILE];
  __shared__ long long red[16];
  __shared__ int wpos, wnan;
  const int nb = *a.big_n;
  for (int bi = blockIdx.x; bi < nb; bi += gridDim.x) {
    const int s = a.big_list[bi];
    if (threadIdx.x == 0) { wpos = 0; wnan = 0; }
    __syncthreads();
    long long sum = 0;
    int nan = 0;
    for (int r = 0; r < a.n_win; ++r) {
      const int sl = win_slot(a, r);
      if (sl < 0) continue;
      const int cnt = a.st.counts[(size_t)sl * a.st.S + s];
      const int inl = min(cnt, a.st.cap);
      const int32_t* cell = a.st.cells + ((size_t)sl * a.st.S + s) * a.st.cap;
      for (int k = threadIdx.x; k < inl; k += blockDim.x) {
        const int32_t v = cell[k];
        const int p = atomicAdd(&wpos, 1);
        if (p < BIG_TILE) t[p] = v;
        sum += v;
        nan += v == ELAPSED_NAN;
      }
      if (cnt > inl) {
        const int32_t* run = spill_run(a.st, sl, s);
        for (int k = threadIdx.x; k < cnt - inl; k += blockDim.x) {
          const int32_t v = run[k];
          const int p = atomicAdd(&wpos, 1);
          if (p < BIG_TILE) t[p] = v;
          sum += v;
          nan += v == ELAPSED_NAN;
        }
      }
    }
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sum;
    if (nan) atomicAdd(&wnan, nan);
    __syncthreads();
    const int n_all = wpos;
    if (wnan > 0) {  // uniform: NaN windows go to the JS insertion emulation
      if (threadIdx.x == 0) a.nan_list[atomicAdd(a.nan_n, 1)] = s;
      __syncthreads();
      continue;
    }
    if (n_all > BIG_TILE) {
      // hotter than the LDS tile: the four order statistics the reference percentile formula
      // reads are selected exactly by a 4-pass radix select over the window's samples
      long long tot = 0;
      for (int w = 0; w < 16; ++w) tot += red[w];
      window_select(a, s, n_all, tot, t);
      __syncthreads();
      continue;
    }
    const int n = n_all;
    int np2 = 1;
    while (np2 < n) np2 <<= 1;
    for (int i = n + threadIdx.x; i < np2; i += blockDim.x) t[i] = 0x7fffffff;
    __syncthreads();
    for (int k = 2; k <= np2; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = threadIdx.x; i < np2; i += blockDim.x) {
          const int ixj = i ^ j;
          if (ixj > i) {
            const int32_t x = t[i], y = t[ixj];
            const bool up = (i & k) == 0;
            if ((x > y) == up) { t[i] = y; t[ixj] = x; }
          }
        }
        __syncthreads();
      }
    }
    if (threadIdx.x == 0) {
      long long tot = 0;
      for (int w = 0; w < 16; ++w) tot += red[w];
      finish_series(a, s, n_all, tot, t);
    }
    __syncthreads();
  }
}

// Windows holding a NaN sample: windowSortedElapTimes is built by binaryConcat'ing the window
// buckets in key order (stream_calc_stats.js:172-178); NaN compares 'equal' to everything in the
// binary search (util_methods.js:57-95), so the array stops being sorted and the percentile
// ranks read whatever the insertion order put there.  One block per series replays it exactly:
// samples gathered bucket by bucket in arrival order (inline cell, then the series' spill
// entries), the prefix before the first NaN sorted (any order of it yields the same sorted
// array), the rest inserted one by one with a block-parallel tail shift.  Rare by construction.
__device__ __forceinline__ double js_elem(int32_t v) { return v == ELAPSED_NAN ? apm_nan() : (double)v; }

__global__ __launch_bounds__(1024) void k_window_stats_js(WindowArgs a) {
  __shared__ int32_t lds[BIG_TILE];
  __shared__ int wsum[16], wpos, ins_at, first_nan;
  const int nn = *a.nan_n;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int32_t* const gbuf = a.js_scratch + (size_t)blockIdx.x * a.js_cap;
  for (int bi = blockIdx.x; bi < nn; bi += gridDim.x) {
    const int s = a.nan_list[bi];
    if (threadIdx.x == 0) { wpos = 0; first_nan = INT32_MAX; }
    __syncthreads();
    for (int r = 0; r < a.n_win; ++r) {
      const int sl = win_slot(a, r);
      if (sl < 0) continue;
      const int cnt = a.st.counts[(size_t)sl * a.st.S + s];
      const int inl = min(cnt, a.st.cap);
      const int base = wpos;
      const int32_t* cell = a.st.cells + ((size_t)sl * a.st.S + s) * a.st.cap;
      for (int k = threadIdx.x; k < inl; k += blockDim.x)
        if (base + k < a.js_cap) gbuf[base + k] = cell[k];
      __syncthreads();
      if (threadIdx.x == 0) wpos = base + inl;
      __syncthreads();
      if (cnt > inl) {  // the series' spill run: arrival order (the list sort is stable)
        const int32_t* run = spill_run(a.st, sl, s);
        const int m = cnt - inl;
        for (int k = threadIdx.x; k < m; k += blockDim.x)
          if (base + inl + k < a.js_cap) gbuf[base + inl + k] = run[k];
        __syncthreads();
        if (threadIdx.x == 0) wpos = base + inl + m;
        __syncthreads();
      }
    }
    const int n_all = wpos;
    const int n = min(n_all, a.js_cap);
    if (n_all > a.js_cap && threadIdx.x == 0 && a.st.spill_drop) atomicAdd(a.st.spill_drop + 1, 1ULL);
    int32_t* buf = n <= BIG_TILE ? lds : gbuf;
    if (buf == lds)
      for (int k = threadIdx.x; k < n; k += blockDim.x) lds[k] = gbuf[k];
    __syncthreads();
    for (int k = threadIdx.x; k < n; k += blockDim.x)
      if (buf[k] == ELAPSED_NAN) atomicMin(&first_nan, k);
    __syncthreads();
    const int f = min(first_nan, n);
    // sorted prefix (bitonic in LDS when it fits, else insertion below covers it too)
    int done = 0;
    if (buf == lds && f > 1) {
      int np2 = 1;
      while (np2 < f) np2 <<= 1;
      if (np2 <= BIG_TILE) {
        // pad with +inf past f: the tail [f, n) is parked in gbuf and copied back after the sort
        for (int k = f + threadIdx.x; k < np2; k += blockDim.x) lds[k] = 0x7fffffff;
        __syncthreads();
        for (int k = 2; k <= np2; k <<= 1)
          for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < np2; i += blockDim.x) {
              const int ixj = i ^ j;
              if (ixj > i) {
                const int32_t x = lds[i], y = lds[ixj];
                if ((x > y) == ((i & k) == 0)) { lds[i] = y; lds[ixj] = x; }
              }
            }
            __syncthreads();
          }
        for (int k = f + threadIdx.x; k < n; k += blockDim.x) lds[k] = gbuf[k];
        __syncthreads();
        done = f;
      }
    }
    if (done == 0) done = min(n, 1);
    for (int k = done; k < n; ++k) {
      const int32_t v = buf[k];
      if (threadIdx.x == 0) {
        int lo = 0, hi = k - 1, at = -1;
        const bool vn = v == ELAPSED_NAN;
        while (lo <= hi) {
          const int m = (lo + hi) >> 1;
          const int32_t x = buf[m];
          if (!vn && x != ELAPSED_NAN && x < v) lo = m + 1;
          else if (!vn && x != ELAPSED_NAN && x > v) hi = m - 1;
          else { at = m; break; }
        }
        ins_at = at >= 0 ? at : lo;
      }
      __syncthreads();
      const int at = ins_at;
      // shift buf[at, k) right by one, last chunk first
      for (int c = k - 1; c >= at; c -= (int)blockDim.x) {
        const int idx = c - (int)threadIdx.x;
        int32_t x = 0;
        if (idx >= at) x = buf[idx];
        __syncthreads();
        if (idx >= at) buf[idx + 1] = x;
        __syncthreads();
      }
      if (threadIdx.x == 0) buf[at] = v;
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      WinStat w;
      w.n = n_all;
      w.active = 1;
      w.tpm = js_round_fixed((double)n_all / a.tpm_div, 2);
      w.avg = apm_nan();  // the NaN poisons windowRtTotalSum
      int lo, hi;
      percentile_ranks(n, 75, lo, hi);
      w.p75 = js_round_fixed(lo == hi ? js_elem(buf[lo]) : (js_elem(buf[lo]) + js_elem(buf[hi])) / 2.0, 1);
      percentile_ranks(n, 95, lo, hi);
      w.p95 = js_round_fixed(lo == hi ? js_elem(buf[lo]) : (js_elem(buf[lo]) + js_elem(buf[hi])) / 2.0, 1);
      a.out[s] = w;
    }
    __syncthreads();
  }
}

// --------------------------------------------------------------------------------- K9
// The pending pool is kept sorted by (endTs, arrival gid).  New tx are appended to an unsorted
// tail; at a rollover the tail is radix-sorted (stable, so arrival order breaks endTs ties),
// merged behind the pool, and the released prefix (endTs <= edge) is handed to the sink.  The
// prefix length is known on the host (it counts endTs per bucket as it emits tx), so no device
// synchronisation is needed.
__global__ void k_pool_append(const TxRec* __restrict__ tx, uint32_t lo, uint32_t hi, const int64_t* __restrict__ gid,
                              int64_t* __restrict__ tail_end, int64_t* __restrict__ tail_gid, int64_t base) {
  const uint32_t i = lo + blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= hi) return;
  tail_end[base + (i - lo)] = tx[i].end_ms;
  tail_gid[base + (i - lo)] = gid[i];
}

// Device scalars -> host-mapped pinned memory in one launch (instead of one blit per value);
// entries with a reset flag get their device value rewritten after the read.
__global__ void k_export(ExportArgs a) {
  const int i = threadIdx.x;
  if (i >= a.n) return;
  if (a.bytes[i] == 8) {
    unsigned long long* s = (unsigned long long*)a.src[i];
    *(unsigned long long*)a.dst[i] = *s;
    if (a.reset[i]) *s = a.reset_val[i];
  } else {
    uint32_t* s = (uint32_t*)a.src[i];
    *(uint32_t*)a.dst[i] = *s;
    if (a.reset[i]) *s = (uint32_t)a.reset_val[i];
  }
}

// Plain copy by a kernel, for small per-batch transfers between device memory and host-mapped
// pinned memory (src or dst may be the device view of a hipHostMalloc buffer).  hipMemcpyAsync
// of a few KB from pinned memory held the calling thread for up to 0.6 ms behind other copies
// on this pool (trace span u.hops.h2d, profiles/r3_*); a kernel read over the host link is
// ordered on the stream like any launch and never blocks the host.  W: bytes per lane per step.
template <typename W>
__global__ __launch_bounds__(256) void k_copy(W* __restrict__ dst, const W* __restrict__ src, size_t n,
                                              uint8_t* __restrict__ tdst, const uint8_t* __restrict__ tsrc,
                                              uint32_t tail) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const size_t t0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t i = t0;
  for (; i + 3 * stride < n; i += 4 * stride) {  // four loads in flight per lane (host-link latency)
    const W a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
    dst[i] = a; dst[i + stride] = b; dst[i + 2 * stride] = c; dst[i + 3 * stride] = d;
  }
  for (; i < n; i += stride) dst[i] = src[i];
  if (t0 < tail) tdst[t0] = tsrc[t0];  // the bytes after the last full W (same launch)
}

}  // namespace apm

// ------------------------------------------------------------------------ checkpoint packing
// The occupied cells of the live bucket slots, packed on the device for the checkpoint (the host
// used to copy every slot's full cell array and pack it series by series on the ingest thread).
// Entry i * n + s = (slot[i], series s): lens = min(count, cap), scanned, then gathered.
__global__ void k_ck_lens(const int32_t* __restrict__ counts, const int32_t* __restrict__ slots, int k, int32_t n,
                          int32_t S, int32_t cap, uint32_t* __restrict__ lens) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t N = (uint64_t)k * n;
  if (t > N) return;
  if (t == N) { lens[N] = 0; return; }
  const int i = (int)(t / (uint64_t)n), s = (int)(t % (uint64_t)n);
  const int32_t c = counts[(size_t)slots[i] * S + s];
  lens[t] = (uint32_t)(c < cap ? (c > 0 ? c : 0) : cap);
}

__global__ void k_ck_pack(const int32_t* __restrict__ cells, const int32_t* __restrict__ slots, int k, int32_t n,
                          int32_t S, int32_t cap, const uint32_t* __restrict__ lens, const uint32_t* __restrict__ offs,
                          int32_t* __restrict__ packed) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (uint64_t)k * n) return;
  const int i = (int)(t / (uint64_t)n), s = (int)(t % (uint64_t)n);
  const int32_t* src = cells + ((size_t)slots[i] * S + s) * cap;
  int32_t* dst = packed + offs[t];
  for (uint32_t j = 0; j < lens[t]; ++j) dst[j] = src[j];
}

// Up to 8 copies in one launch (blockIdx.y = the copy): the join's sync-C read-back (counts,
// rollover candidates, unresolved series, audit_db text) into host-mapped pinned memory as one
// kernel instead of a blit per array.
__global__ void k_copy_segs(apm::CopySegs c) {
  const apm::CopySeg& g = c.seg[blockIdx.y];
  if (blockIdx.y >= (unsigned)c.n) return;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uintptr_t al = (uintptr_t)g.dst | (uintptr_t)g.src;
  if ((al & 15) == 0) {
    const size_t n16 = g.bytes / 16;
    for (size_t i = t; i < n16; i += stride) reinterpret_cast<uint4*>(g.dst)[i] = reinterpret_cast<const uint4*>(g.src)[i];
    for (size_t i = n16 * 16 + t; i < g.bytes; i += stride) ((uint8_t*)g.dst)[i] = ((const uint8_t*)g.src)[i];
  } else if ((al & 3) == 0) {
    const size_t n4 = g.bytes / 4;
    for (size_t i = t; i < n4; i += stride) reinterpret_cast<uint32_t*>(g.dst)[i] = reinterpret_cast<const uint32_t*>(g.src)[i];
    for (size_t i = n4 * 4 + t; i < g.bytes; i += stride) ((uint8_t*)g.dst)[i] = ((const uint8_t*)g.src)[i];
  } else {
    for (size_t i = t; i < g.bytes; i += stride) ((uint8_t*)g.dst)[i] = ((const uint8_t*)g.src)[i];
  }
}

// up to 8 doubles from the kernel arguments (no host-memory read on the device side: a small
// H2D that waits behind nothing on the host link)
struct F64x8 {
  double v[8];
};
__global__ void k_set_f64(double* __restrict__ dst, F64x8 v, int n) {
  if ((int)threadIdx.x < n) dst[threadIdx.x] = v.v[threadIdx.x];
}

extern "C" {

using namespace apm;

void apm_copy(void* dst, const void* src, size_t bytes, hipStream_t stream) {
  apm_copy_capped(dst, src, bytes, 1024, stream);
}

void apm_copy_capped(void* dst, const void* src, size_t bytes, uint32_t max_blocks, hipStream_t stream) {
  if (bytes == 0) return;
  const uintptr_t a = (uintptr_t)dst | (uintptr_t)src;
  auto launch = [&](auto* d, const auto* s, size_t w) {
    const size_t n = bytes / w, done = n * w;
    const size_t blocks = std::max<size_t>(1, std::min<size_t>((n + 255) / 256, std::max<uint32_t>(max_blocks, 1)));
    hipLaunchKernelGGL(k_copy, dim3((unsigned)blocks), dim3(256), 0, stream, d, s, n, (uint8_t*)dst + done,
                       (const uint8_t*)src + done, (uint32_t)(bytes - done));
  };
  if ((a & 15) == 0) launch((uint4*)dst, (const uint4*)src, 16);
  else if ((a & 3) == 0) launch((uint32_t*)dst, (const uint32_t*)src, 4);
  else launch((uint8_t*)dst, (const uint8_t*)src, 1);
}

void apm_copy_segs(const CopySegs* c, hipStream_t stream) {
  if (c->n <= 0) return;
  size_t mx = 0;
  for (int i = 0; i < c->n; ++i) mx = std::max(mx, c->seg[i].bytes);
  const unsigned bx = (unsigned)std::max<size_t>(1, std::min<size_t>((mx / 16 + 255) / 256, 64));
  hipLaunchKernelGGL(k_copy_segs, dim3(bx, (unsigned)c->n), dim3(256), 0, stream, *c);
}

void apm_set_f64(double* dst, const double* vals, int n, hipStream_t stream) {
  F64x8 v{};
  n = std::min(std::max(n, 0), 8);
  for (int i = 0; i < n; ++i) v.v[i] = vals[i];
  hipLaunchKernelGGL(k_set_f64, dim3(1), dim3(64), 0, stream, dst, v, n);
}

void apm_export(const ExportArgs* a, hipStream_t stream) {
  if (a->n > 0) hipLaunchKernelGGL(k_export, dim3(1), dim3(64), 0, stream, *a);
}

void apm_stats_clear_slot(StatsState* st, int slot, hipStream_t stream) {
  hipLaunchKernelGGL(k_clear_slot, dim3((st->S + 255) / 256), dim3(256), 0, stream, *st, slot);
}

void apm_bucket_append(const TxRec* d_tx, uint32_t lo, uint32_t hi, StatsState* st, int64_t min_live_bucket,
                       hipStream_t stream) {
  if (hi <= lo) return;
  // ord_n is zero here: k_bucket_append_ordered resets it after reading
  hipLaunchKernelGGL(k_bucket_append, dim3((hi - lo + 255) / 256), dim3(256), 0, stream, d_tx, lo, hi, *st,
                     min_live_bucket);
  if (st->ord_n) hipLaunchKernelGGL(k_bucket_append_ordered, dim3(64), dim3(1024), 0, stream, d_tx, lo, hi, *st);
}

void apm_nan_mark(const TxRec* d_tx, uint32_t n, StatsState* st, hipStream_t stream) {
  if (n == 0 || !st->nan_until) return;
  hipLaunchKernelGGL(k_nan_mark, dim3((n + 255) / 256), dim3(256), 0, stream, d_tx, n, *st);
}

// big_n / nan_n must be zero on entry (the engine clears them with the rollover's other counters)
void apm_window_stats(WindowArgs* a, hipStream_t stream) {
  static const bool h2 = [] { const char* e = std::getenv("APM_K8_H2"); return !(e && e[0] == '0'); }();
  if (h2 && a->n_win <= HW && a->lds_sort != 1) {
    const int blocks2 = (a->n_series + 2 * WS_WAVES - 1) / (2 * WS_WAVES);
    if (blocks2 == 0) return;
    hipLaunchKernelGGL(k_window_stats_h2, dim3(blocks2), dim3(WS_WAVES * APM_WAVE), 0, stream, *a);
  } else {
    const int blocks = (a->n_series + WS_WAVES - 1) / WS_WAVES;
    if (blocks == 0) return;
    hipLaunchKernelGGL(k_window_stats, dim3(blocks), dim3(WS_WAVES * APM_WAVE), 0, stream, *a);
  }
  hipLaunchKernelGGL(k_window_stats_big, dim3(64), dim3(1024), 0, stream, *a);
  hipLaunchKernelGGL(k_window_stats_js, dim3(JS_BLOCKS), dim3(1024), 0, stream, *a);
}

namespace {
// segment [slot * cap, slot * cap + spill_n[slot]) (one functor type for both offset iterators)
struct SpillOff {
  const int32_t* n;  // null: segment begin
  int32_t cap;
  __host__ __device__ int operator()(int slot) const { return slot * cap + (n ? min(n[slot], cap) : 0); }
};
int key_bits(int32_t S) {
  int b = 1;
  while ((1ll << b) < (long long)S) ++b;
  return b;
}
}  // namespace

size_t apm_spill_sort_tmp_bytes(int32_t spill_cap, int32_t S, int32_t nslot) {
  size_t need = 0;
  const auto beg = rocprim::make_transform_iterator(rocprim::make_counting_iterator(0), SpillOff{nullptr, spill_cap});
  const auto end = rocprim::make_transform_iterator(rocprim::make_counting_iterator(0), SpillOff{nullptr, spill_cap});
  HIP_OK(rocprim::segmented_radix_sort_pairs(nullptr, need, (int32_t*)nullptr, (int32_t*)nullptr, (int32_t*)nullptr,
                                             (int32_t*)nullptr, (size_t)nslot * spill_cap, (unsigned)nslot, beg, end, 0,
                                             key_bits(S), (hipStream_t)0));
  return need + 4096;
}

int apm_spill_sort(const StatsState* st, int32_t* series_out, int32_t* val_out, void* tmp, size_t tmp_bytes,
                   hipStream_t stream) {
  size_t need = 0;
  const auto beg = rocprim::make_transform_iterator(rocprim::make_counting_iterator(0), SpillOff{nullptr, st->spill_cap});
  const auto end = rocprim::make_transform_iterator(rocprim::make_counting_iterator(0), SpillOff{st->spill_n, st->spill_cap});
  HIP_OK(rocprim::segmented_radix_sort_pairs(nullptr, need, st->spill_series, series_out, st->spill_val, val_out,
                                             (size_t)st->nslot * st->spill_cap, (unsigned)st->nslot, beg, end, 0, key_bits(st->S),
                                             stream));
  if (need > tmp_bytes) return -1;
  HIP_OK(rocprim::segmented_radix_sort_pairs(tmp, need, st->spill_series, series_out, st->spill_val, val_out,
                                             (size_t)st->nslot * st->spill_cap, (unsigned)st->nslot, beg, end, 0, key_bits(st->S),
                                             stream));
  return 0;
}

void apm_pool_append(const TxRec* d_tx, uint32_t lo, uint32_t hi, const int64_t* d_gid, int64_t* tail_end,
                     int64_t* tail_gid, int64_t base, hipStream_t stream) {
  if (hi <= lo) return;
  hipLaunchKernelGGL(k_pool_append, dim3((hi - lo + 255) / 256), dim3(256), 0, stream, d_tx, lo, hi, d_gid,
                     tail_end, tail_gid, base);
}

size_t apm_release_tmp_bytes(int64_t cap) {
  size_t a = 0, b = 0;
  HIP_OK(rocprim::radix_sort_pairs(nullptr, a, (int64_t*)nullptr, (int64_t*)nullptr, (int64_t*)nullptr,
                                   (int64_t*)nullptr, (size_t)cap, 0, 64, (hipStream_t)0));
  HIP_OK(rocprim::merge(nullptr, b, (int64_t*)nullptr, (int64_t*)nullptr, (int64_t*)nullptr,
                        (int64_t*)nullptr, (int64_t*)nullptr, (int64_t*)nullptr, (size_t)cap, (size_t)cap,
                        rocprim::less<int64_t>(), (hipStream_t)0));
  return std::max(a, b) + 4096;
}

// out = merge(pool[0..n_pool), sort(tail[0..n_tail)))   (stable: pool entries first on ties)
int apm_release_merge(const int64_t* pool_end, const int64_t* pool_gid, int64_t n_pool, const int64_t* tail_end,
                      const int64_t* tail_gid, int64_t n_tail, int64_t* sort_end, int64_t* sort_gid,
                      int64_t* out_end, int64_t* out_gid, void* tmp, size_t tmp_bytes, hipStream_t stream) {
  size_t need = 0;
  if (n_tail > 0) {
    HIP_OK(rocprim::radix_sort_pairs(nullptr, need, tail_end, sort_end, tail_gid, sort_gid, (size_t)n_tail, 0, 64,
                                     stream));
    if (need > tmp_bytes) return -1;
    HIP_OK(rocprim::radix_sort_pairs(tmp, need, tail_end, sort_end, tail_gid, sort_gid, (size_t)n_tail, 0, 64,
                                     stream));
  }
  if (n_pool + n_tail == 0) return 0;
  HIP_OK(rocprim::merge(nullptr, need, pool_end, sort_end, out_end, pool_gid, sort_gid, out_gid, (size_t)n_pool,
                        (size_t)n_tail, rocprim::less<int64_t>(), stream));
  if (need > tmp_bytes) return -1;
  HIP_OK(rocprim::merge(tmp, need, pool_end, sort_end, out_end, pool_gid, sort_gid, out_gid, (size_t)n_pool,
                        (size_t)n_tail, rocprim::less<int64_t>(), stream));
  return 0;
}


size_t apm_ck_pack_tmp_bytes(uint64_t n_entries) {
  size_t b = 0;
  HIP_OK(rocprim::exclusive_scan(nullptr, b, (uint32_t*)nullptr, (uint32_t*)nullptr, 0u, (size_t)n_entries + 1,
                                 rocprim::plus<uint32_t>(), (hipStream_t)0));
  return b;
}

int apm_ck_pack_cells(const int32_t* counts, const int32_t* cells, const int32_t* d_slots, int k, int32_t n, int32_t S,
                      int32_t cap, uint32_t* lens, uint32_t* offs, void* tmp, size_t tmp_bytes, int32_t* packed,
                      hipStream_t s) {
  const uint64_t N = (uint64_t)k * n;
  hipLaunchKernelGGL(k_ck_lens, dim3((unsigned)((N + 1 + 255) / 256)), dim3(256), 0, s, counts, d_slots, k, n, S, cap, lens);
  size_t need = 0;
  HIP_OK(rocprim::exclusive_scan(nullptr, need, lens, offs, 0u, (size_t)N + 1, rocprim::plus<uint32_t>(), s));
  if (need > tmp_bytes) return -1;
  HIP_OK(rocprim::exclusive_scan(tmp, need, lens, offs, 0u, (size_t)N + 1, rocprim::plus<uint32_t>(), s));
  if (N) hipLaunchKernelGGL(k_ck_pack, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, cells, d_slots, k, n, S, cap, lens, offs, packed);
  return 0;
}
}  // extern "C"
