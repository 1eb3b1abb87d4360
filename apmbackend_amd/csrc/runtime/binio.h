// Tiny tagged binary writer/reader for checkpoints (little-endian, host byte order).
//
// A file is: magic "APMCKPT\0", u32 version, then sections {u32 tag, u64 length, payload}.
// Readers check every section tag in order, so a layout change fails loudly instead of
// silently misreading.  Writers go to `<path>.tmp`, fsync, then rename (atomic replace --
// the reference wrote its resume files in place).
#pragma once
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

namespace apm {

// 3: join section carries the join mode (host / GPU); 4: node-wide server order; 5: rings in their own
// trailing section (full or dirty rows, for incremental checkpoints) + NaN horizons + an opaque extra
constexpr uint32_t kCkptVersion = 9;  // 7: device audit-trail carry (K5 on the GPU); 8: 8 LAG slots;
                                      // 9: 16 LAG slots, config-sized bucket ring (slot table as a vector)

// Section tags, in file order (checkpoint.cpp writes / reads them, merge.cpp re-shards them).
enum : uint32_t {
  SEC_CONFIG = 1, SEC_TOPOLOGY, SEC_SERIES, SEC_CLOCK, SEC_JOIN, SEC_PARSE, SEC_BUCKETS, SEC_ZSCORE, SEC_POOL,
  SEC_ALERTS, SEC_OUTPUTS, SEC_METRICS, SEC_RING, SEC_EXTRA, SEC_DUMP = 100, SEC_DUMP_SERIES = 101
};

// A malloc'd byte buffer (no zero-fill on growth), owned and move-only.
struct MemBlob {
  char* p = nullptr;
  size_t n = 0, cap = 0;
  MemBlob() = default;
  MemBlob(const MemBlob&) = delete;
  MemBlob& operator=(const MemBlob&) = delete;
  MemBlob(MemBlob&& o) noexcept : p(o.p), n(o.n), cap(o.cap) { o.p = nullptr; o.n = o.cap = 0; }
  MemBlob& operator=(MemBlob&& o) noexcept {
    if (this != &o) { std::free(p); p = o.p; n = o.n; cap = o.cap; o.p = nullptr; o.n = o.cap = 0; }
    return *this;
  }
  ~MemBlob() { std::free(p); }
  void reserve(size_t c) {
    if (c <= cap) return;
    char* q = (char*)std::realloc(p, c);
    if (!q) throw std::runtime_error("checkpoint: out of host memory");
    p = q;
    cap = c;
  }
  char* grow(size_t k) {  // k more bytes at the end (uninitialised)
    if (n + k > cap) reserve(std::max(n + k, cap + cap / 2 + (1u << 20)));
    char* at = p + n;
    n += k;
    return at;
  }
  const char* data() const { return p; }
  size_t size() const { return n; }
};

class BinWriter {
 public:
  explicit BinWriter(const std::string& path) : path_(path), tmp_(path + ".tmp") {
    f_ = std::fopen(tmp_.c_str(), "wb");
    if (!f_) throw std::runtime_error("checkpoint: cannot open " + tmp_ + ": " + std::strerror(errno));
    std::setvbuf(f_, nullptr, _IOFBF, 1 << 22);
    raw("APMCKPT", 8);
    pod(kCkptVersion);
  }
  // In-memory writer (no header): sections serialised into a byte vector reserved up front
  // (`reserve`: the previous snapshot's size), later spliced into a file by the asynchronous
  // checkpoint writer.  (open_memstream + a copy out cost two extra passes over ~300 MB of
  // state on the ingest thread.)
  struct Memory {};
  explicit BinWriter(Memory, size_t reserve = 0) : mem_(true) { buf_.reserve(reserve); }
  // ... into a previous snapshot's buffer: its pages are already mapped, so the ingest thread's
  // serialisation does not page-fault its way through a fresh ~100 MB allocation
  BinWriter(Memory, MemBlob&& reuse, size_t reserve) : mem_(true), buf_(std::move(reuse)) {
    buf_.n = 0;
    buf_.reserve(reserve);
  }
  MemBlob take_memory() { return std::move(buf_); }
  ~BinWriter() {
    if (f_) {
      std::fclose(f_);
      if (!tmp_.empty()) std::remove(tmp_.c_str());
    }
  }
  bool memory() const { return mem_; }
  // memory mode: n bytes left for a later fill (a deferred device copy, d2h.h); their offset
  size_t hole(size_t n) {
    char* at = buf_.grow(n);
    bytes_ += n;
    return (size_t)(at - buf_.data());
  }
  void raw(const void* p, size_t n) {
    if (mem_) {
      if (n) std::memcpy(buf_.grow(n), p, n);
    } else if (n && std::fwrite(p, 1, n, f_) != n) {
      throw std::runtime_error("checkpoint: write failed");
    }
    bytes_ += n;
  }
  // append n bytes written by `fill(dst)` in place (memory mode; file mode: through a buffer)
  template <class F>
  void raw_fill(size_t n, F&& fill) {
    if (!n) return;
    if (mem_) {
      fill(buf_.grow(n));
      bytes_ += n;
    } else {
      std::vector<char> tmp(n);
      fill(tmp.data());
      raw(tmp.data(), n);
    }
  }
  template <class T>
  void pod(const T& v) {
    static_assert(std::is_trivially_copyable<T>::value, "pod");
    raw(&v, sizeof(T));
  }
  void str(const std::string& s) { pod<uint64_t>(s.size()); raw(s.data(), s.size()); }
  template <class T>
  void vec(const std::vector<T>& v) {
    static_assert(std::is_trivially_copyable<T>::value, "vec");
    pod<uint64_t>(v.size());
    raw(v.data(), v.size() * sizeof(T));
  }
  void strs(const std::vector<std::string>& v) {
    pod<uint64_t>(v.size());
    for (auto& s : v) str(s);
  }
  // section framing: the length is patched in when the section ends
  void begin(uint32_t tag) {
    pod(tag);
    if (mem_) {
      sec_pos_ = (long)buf_.size();
    } else {
      std::fflush(f_);
      sec_pos_ = std::ftell(f_);
    }
    pod<uint64_t>(0);
  }
  void end() {
    if (mem_) {
      const uint64_t len = (uint64_t)((long)buf_.size() - sec_pos_ - 8);
      std::memcpy(buf_.p + sec_pos_, &len, 8);
      return;
    }
    const long here = std::ftell(f_);
    const uint64_t len = (uint64_t)(here - sec_pos_ - 8);
    std::fseek(f_, sec_pos_, SEEK_SET);
    raw(&len, 8);
    bytes_ -= 8;
    std::fseek(f_, here, SEEK_SET);
  }
  void commit() {
    pod<uint32_t>(0xE0Fu);  // end marker
    if (std::fflush(f_) != 0) throw std::runtime_error("checkpoint: flush failed");
    ::fsync(::fileno(f_));
    std::fclose(f_);
    f_ = nullptr;
    if (std::rename(tmp_.c_str(), path_.c_str()) != 0)
      throw std::runtime_error("checkpoint: rename failed: " + std::string(std::strerror(errno)));
  }
  uint64_t bytes() const { return bytes_; }
  // memory mode: current size, and a pointer to an earlier offset (valid until the next write)
  bool is_memory() const { return mem_; }
  size_t mem_pos() const { return buf_.size(); }
  char* mem_at(size_t off) { return buf_.p + off; }

 private:
  std::string path_, tmp_;
  FILE* f_ = nullptr;
  long sec_pos_ = 0;
  uint64_t bytes_ = 0;
  bool mem_ = false;
  MemBlob buf_;
};

class BinReader {
 public:
  explicit BinReader(const std::string& path) {
    f_ = std::fopen(path.c_str(), "rb");
    if (!f_) throw std::runtime_error("checkpoint: cannot open " + path + ": " + std::strerror(errno));
    std::setvbuf(f_, nullptr, _IOFBF, 1 << 22);
    char magic[8];
    raw(magic, 8);
    if (std::memcmp(magic, "APMCKPT", 8) != 0) throw std::runtime_error("checkpoint: bad magic");
    const uint32_t v = pod<uint32_t>();
    if (v != kCkptVersion) throw std::runtime_error("checkpoint: unsupported version " + std::to_string(v));
  }
  ~BinReader() { if (f_) std::fclose(f_); }
  void raw(void* p, size_t n) {
    if (n && std::fread(p, 1, n, f_) != n) throw std::runtime_error("checkpoint: truncated file");
  }
  template <class T>
  T pod() {
    T v;
    raw(&v, sizeof(T));
    return v;
  }
  template <class T>
  void pod(T& v) { raw(&v, sizeof(T)); }
  std::string str() {
    const uint64_t n = pod<uint64_t>();
    std::string s(n, '\0');
    raw(&s[0], n);
    return s;
  }
  template <class T>
  std::vector<T> vec() {
    const uint64_t n = pod<uint64_t>();
    std::vector<T> v(n);
    raw(v.data(), n * sizeof(T));
    return v;
  }
  std::vector<std::string> strs() {
    const uint64_t n = pod<uint64_t>();
    std::vector<std::string> v;
    v.reserve(n);
    for (uint64_t i = 0; i < n; ++i) v.push_back(str());
    return v;
  }
  void begin(uint32_t tag) {
    const uint32_t t = pod<uint32_t>();
    if (t != tag) throw std::runtime_error("checkpoint: expected section " + std::to_string(tag) + ", found " +
                                           std::to_string(t));
    pod<uint64_t>();
  }
  void end() {}
  // Skips whole sections until `tag` (its header consumed), for readers that want one part.
  void skip_to(uint32_t tag) {
    for (;;) {
      const uint32_t t = pod<uint32_t>();
      if (t == 0xE0Fu) throw std::runtime_error("checkpoint: section " + std::to_string(tag) + " not found");
      const uint64_t len = pod<uint64_t>();
      if (t == tag) return;
      if (std::fseek(f_, (long)len, SEEK_CUR) != 0) throw std::runtime_error("checkpoint: seek failed");
    }
  }
  void finish() {
    if (pod<uint32_t>() != 0xE0Fu) throw std::runtime_error("checkpoint: missing end marker");
  }
  void skip(uint64_t n) {
    if (n && std::fseek(f_, (long)n, SEEK_CUR) != 0) throw std::runtime_error("checkpoint: seek failed");
  }

 private:
  FILE* f_ = nullptr;
};

}  // namespace apm
