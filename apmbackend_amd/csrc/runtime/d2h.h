// Device -> host copies of checkpoint state through a pinned bounce buffer: the DMA of one half
// of the bounce overlaps the host copy out of the other (a pageable hipMemcpy of ~100 MB held the
// ingest thread for tens of ms per checkpoint).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <memory>
#include <vector>

#include "../kernels/common.h"
#include "binio.h"

namespace apm {

inline void d2h_bounced(void* dst, const void* dev, size_t n, hipStream_t st, char* bounce, size_t bounce_bytes) {
  if (!n) return;
  const size_t half = bounce_bytes / 2;
  HIP_OK(hipMemcpyAsync(bounce, dev, std::min(half, n), hipMemcpyDeviceToHost, st));
  size_t off = 0;
  for (int k = 0; off < n; ++k) {
    const size_t len = std::min(half, n - off);
    HIP_OK(hipStreamSynchronize(st));  // chunk k is in half k & 1
    const size_t next = off + len;
    if (next < n)
      HIP_OK(hipMemcpyAsync(bounce + (size_t)((k + 1) & 1) * half, (const char*)dev + next, std::min(half, n - next),
                            hipMemcpyDeviceToHost, st));
    std::memcpy((char*)dst + off, bounce + (size_t)(k & 1) * half, len);
    off = next;
  }
}

// Deferred device reads of an asynchronous checkpoint (Engine::checkpoint_async): while one is set
// on the thread that serialises the snapshot, write_dev / write_dev_rows into an in-memory writer
// copy the bytes D2D into HBM staging (~TB/s; the snapshot waits for those copies) and leave a hole
// in the blob; the checkpoint writer thread fills the holes (D2H through its bounce) before it
// writes the file.  The ingest thread no longer pays for the host-link reads (the join table,
// window cells, pending-line text: ~36 ms per checkpoint at the production path, profiles/r5_e).
struct CkDefer {
  struct Hole { size_t blob_off, stage_off, len; };
  char* stage = nullptr;   // device staging
  size_t cap = 0, used = 0;
  size_t want = 0;         // bytes the last snapshot would have deferred (sizes the next staging)
  std::vector<Hole> holes;
  std::vector<hipStream_t> streams;  // streams the D2D copies were queued on
  // 4-byte values the writer stores into the blob after it filled the holes (fix-ups of bytes
  // that may sit in a hole: the join's chain block numbers, DeviceJoin::save_tables)
  std::vector<std::pair<size_t, int32_t>> patches;
  bool take(BinWriter& w, const void* dev, size_t pitch, size_t width, size_t rows, hipStream_t st) {
    const size_t n = width * rows;
    want += (n + 255) & ~(size_t)255;
    if (!w.memory() || !stage || used + n > cap) return false;
    if (rows == 1) HIP_OK(hipMemcpyAsync(stage + used, dev, n, hipMemcpyDeviceToDevice, st));
    else HIP_OK(hipMemcpy2DAsync(stage + used, width, dev, pitch, width, rows, hipMemcpyDeviceToDevice, st));
    holes.push_back(Hole{w.hole(n), used, n});
    used += (n + 255) & ~(size_t)255;
    if (std::find(streams.begin(), streams.end(), st) == streams.end()) streams.push_back(st);
    return true;
  }
};
inline CkDefer*& ck_defer() {
  static thread_local CkDefer* d = nullptr;
  return d;
}

// n device bytes appended to the writer in place
inline void write_dev(BinWriter& w, const void* dev, size_t n, hipStream_t st, char* bounce, size_t bounce_bytes) {
  if (!n) return;
  if (CkDefer* d = ck_defer())
    if (d->take(w, dev, n, n, 1, st)) return;
  w.raw_fill(n, [&](char* dst) { d2h_bounced(dst, dev, n, st, bounce, bounce_bytes); });
}

// An array of trivially copyable records without the zero fill of std::vector::resize (the
// snapshot overwrites every byte); written in the BinWriter::vec layout.
template <class T>
struct PodBuf {
  std::unique_ptr<T[]> p;
  size_t n = 0;
  void resize_uninit(size_t k) {
    p.reset(k ? new T[k] : nullptr);
    n = k;
  }
  T* data() { return p.get(); }
  size_t size() const { return n; }
  bool empty() const { return n == 0; }
  T* begin() { return p.get(); }
  T* end() { return p.get() + n; }
  T& operator[](size_t i) { return p[i]; }
};
template <class T>
void write_vec(BinWriter& w, const PodBuf<T>& v) {
  w.pod<uint64_t>(v.n);
  w.raw(v.p.get(), v.n * sizeof(T));
}

}  // namespace apm
