// Device -> host copies of checkpoint state through a pinned bounce buffer: the DMA of one half
// of the bounce overlaps the host copy out of the other (a pageable hipMemcpy of ~100 MB held the
// ingest thread for tens of ms per checkpoint).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <memory>

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

// n device bytes appended to the writer in place
inline void write_dev(BinWriter& w, const void* dev, size_t n, hipStream_t st, char* bounce, size_t bounce_bytes) {
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
