// Stream compaction / exclusive scan over [0, n) where n lives on the device.
//
// The per-batch counts of the parse and join stages (lines, events, ...) are only known on the
// GPU, so their scans used to run over the buffers' capacity (2M entries) with rocprim -- a
// look-back scan, its state-init kernel and a scatter over 8x more entries than a batch has.  Here
// the grid is sized for the capacity but every block past the device-side count exits at its
// first instruction, so the work follows the batch:
//
//   k_ds_reduce  one block per 4096-entry tile: the sum of f(i) over the tile (rocprim block_reduce)
//   k_ds_tiles   one block: exclusive scan of the tile sums (<= 4096 tiles), the total -> *total
//   k_ds_apply   one block per tile: each lane scans its 16 consecutive entries, a block scan of
//                the lane sums gives every entry its exclusive prefix p, and g(i, p) consumes it
//
// f(i) -> T must be cheap (it runs in both passes); g(i, p) writes the outputs (scatter).
#pragma once
#include <rocprim/rocprim.hpp>

#include "common.h"

namespace apm {

constexpr int DS_BLOCK = 256, DS_ITEMS = 16, DS_TILE = DS_BLOCK * DS_ITEMS;
constexpr int DS_TILES_BLOCK = 1024, DS_TILES_ITEMS = 4, DS_MAX_TILES = DS_TILES_BLOCK * DS_TILES_ITEMS;

__device__ __forceinline__ uint32_t ds_count(const uint32_t* d_n, uint32_t cap) {
  const uint32_t n = *d_n;
  return n < cap ? n : cap;
}

template <class T, class F>
__global__ __launch_bounds__(DS_BLOCK) void k_ds_reduce(F f, const uint32_t* __restrict__ d_n, uint32_t cap,
                                                        T* __restrict__ tile_sum) {
  const uint32_t n = ds_count(d_n, cap);
  const uint32_t t0 = blockIdx.x * (uint32_t)DS_TILE;
  if (t0 >= n) return;
  T acc = 0;
#pragma unroll
  for (int k = 0; k < DS_ITEMS; ++k) {  // strided: coalesced reads of f's arrays
    const uint32_t i = t0 + (uint32_t)k * DS_BLOCK + threadIdx.x;
    if (i < n) acc += f(i);
  }
  typedef rocprim::block_reduce<T, DS_BLOCK> R;
  __shared__ typename R::storage_type st;
  T s;
  R().reduce(acc, s, st);
  if (threadIdx.x == 0) tile_sum[blockIdx.x] = s;
}

template <class T>
__global__ __launch_bounds__(DS_TILES_BLOCK) void k_ds_tiles(T* __restrict__ tile_sum, const uint32_t* __restrict__ d_n,
                                                             uint32_t cap, T* __restrict__ total) {
  const uint32_t n = ds_count(d_n, cap);
  const uint32_t nt = (n + DS_TILE - 1) / DS_TILE;
  T v[DS_TILES_ITEMS];
#pragma unroll
  for (int k = 0; k < DS_TILES_ITEMS; ++k) {
    const uint32_t j = threadIdx.x * DS_TILES_ITEMS + k;
    v[k] = j < nt ? tile_sum[j] : T(0);
  }
  typedef rocprim::block_scan<T, DS_TILES_BLOCK> S;
  __shared__ typename S::storage_type st;
  T lane = 0;
#pragma unroll
  for (int k = 0; k < DS_TILES_ITEMS; ++k) lane += v[k];
  T excl, sum;
  S().exclusive_scan(lane, excl, T(0), sum, st);
#pragma unroll
  for (int k = 0; k < DS_TILES_ITEMS; ++k) {
    const uint32_t j = threadIdx.x * DS_TILES_ITEMS + k;
    if (j < nt) tile_sum[j] = excl;  // in place: tile sum -> tile offset
    excl += v[k];
  }
  if (threadIdx.x == 0) *total = sum;
}

template <class T, class F, class G>
__global__ __launch_bounds__(DS_BLOCK) void k_ds_apply(F f, G g, const uint32_t* __restrict__ d_n, uint32_t cap,
                                                       const T* __restrict__ tile_off) {
  const uint32_t n = ds_count(d_n, cap);
  const uint32_t t0 = blockIdx.x * (uint32_t)DS_TILE;
  if (t0 >= n) return;
  const uint32_t i0 = t0 + threadIdx.x * (uint32_t)DS_ITEMS;
  T v[DS_ITEMS];
  T lane = 0;
#pragma unroll
  for (int k = 0; k < DS_ITEMS; ++k) {
    v[k] = i0 + k < n ? f(i0 + k) : T(0);
    lane += v[k];
  }
  typedef rocprim::block_scan<T, DS_BLOCK> S;
  __shared__ typename S::storage_type st;
  T excl;
  S().exclusive_scan(lane, excl, T(0), st);
  T p = tile_off[blockIdx.x] + excl;
#pragma unroll
  for (int k = 0; k < DS_ITEMS; ++k) {
    if (i0 + k < n) g(i0 + k, p);
    p += v[k];
  }
}

// f, g: functors (device operator()); tile_sum: >= ceil(cap / DS_TILE) entries of scratch;
// total: device word receiving sum f(i) over [0, min(*d_n, cap)).  Returns -1 if cap exceeds the
// single-block tile scan (DS_MAX_TILES * DS_TILE = 16.7M entries).
template <class T, class F, class G>
int ds_scan_apply(F f, G g, const uint32_t* d_n, uint32_t cap, T* tile_sum, T* total, hipStream_t s) {
  const uint32_t tiles = (cap + DS_TILE - 1) / DS_TILE;
  if (tiles > (uint32_t)DS_MAX_TILES) return -1;
  if (tiles == 0) return 0;
  hipLaunchKernelGGL((k_ds_reduce<T, F>), dim3(tiles), dim3(DS_BLOCK), 0, s, f, d_n, cap, tile_sum);
  hipLaunchKernelGGL((k_ds_tiles<T>), dim3(1), dim3(DS_TILES_BLOCK), 0, s, tile_sum, d_n, cap, total);
  hipLaunchKernelGGL((k_ds_apply<T, F, G>), dim3(tiles), dim3(DS_BLOCK), 0, s, f, g, d_n, cap, (const T*)tile_sum);
  return 0;
}

}  // namespace apm
