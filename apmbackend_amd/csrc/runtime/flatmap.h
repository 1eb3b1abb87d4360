// Small containers for the join workers' hot path.
//
// FlatMap<V>: open-addressing hash table keyed by a 64-bit hash (linear probing, power-of-two
// capacity, load <= 1/2, backward-shift deletion so there are no tombstones).  Key 0 marks an
// empty slot, so key 0 is stored as 1 (keys are FNV-1a hashes; see join.h for the collision
// stance).  References returned by find/emplace stay valid until the next insertion into the
// same map.
//
// SmallVec<T, N>: up to N elements inline, spills to the heap beyond that.  The join's partial
// maps hold one or two services per logId, so the common case allocates nothing.
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <utility>
#include <vector>

namespace apm {

template <class V>
class FlatMap {
 public:
  explicit FlatMap(size_t cap = 1024) { alloc(pow2(cap)); }

  size_t size() const { return n_; }
  bool empty() const { return n_ == 0; }

  V* find(uint64_t k) {
    k = fix(k);
    for (size_t i = idx(k);; i = (i + 1) & mask_) {
      if (keys_[i] == k) return &vals_[i];
      if (keys_[i] == 0) return nullptr;
    }
  }

  // Returns (value, inserted).  A new value is value-initialised.
  std::pair<V*, bool> emplace(uint64_t k) {
    k = fix(k);
    if ((n_ + 1) * 2 > keys_.size()) grow();
    size_t i = idx(k);
    for (;; i = (i + 1) & mask_) {
      if (keys_[i] == k) return {&vals_[i], false};
      if (keys_[i] == 0) break;
    }
    keys_[i] = k;
    vals_[i] = V();
    ++n_;
    return {&vals_[i], true};
  }

  V& operator[](uint64_t k) { return *emplace(k).first; }

  bool erase(uint64_t k) {
    k = fix(k);
    size_t i = idx(k);
    for (;; i = (i + 1) & mask_) {
      if (keys_[i] == 0) return false;
      if (keys_[i] == k) break;
    }
    // backward-shift: pull later members of the probe run into the hole
    size_t j = i;
    for (;;) {
      j = (j + 1) & mask_;
      if (keys_[j] == 0) break;
      const size_t home = idx(keys_[j]);
      // can keys_[j] move to i?  yes iff `home` is not cyclically in (i, j]
      const bool between = i <= j ? (home > i && home <= j) : (home > i || home <= j);
      if (between) continue;
      keys_[i] = keys_[j];
      vals_[i] = std::move(vals_[j]);
      i = j;
    }
    keys_[i] = 0;
    vals_[i] = V();
    --n_;
    return true;
  }

  template <class F>
  void for_each(F&& f) {
    for (size_t i = 0; i < keys_.size(); ++i)
      if (keys_[i]) f(keys_[i], vals_[i]);
  }

  void clear() {
    std::fill(keys_.begin(), keys_.end(), 0);
    for (auto& v : vals_) v = V();
    n_ = 0;
  }

 private:
  static size_t pow2(size_t c) {
    size_t p = 16;
    while (p < c) p <<= 1;
    return p;
  }
  static uint64_t fix(uint64_t k) { return k ? k : 1; }
  size_t idx(uint64_t k) const { return (size_t)((k * 0x9E3779B97F4A7C15ULL) >> shift_); }
  void alloc(size_t cap) {
    keys_.assign(cap, 0);
    vals_.clear();
    vals_.resize(cap);
    mask_ = cap - 1;
    int b = 0;
    while (((size_t)1 << b) < cap) ++b;
    shift_ = 64 - b;
    n_ = 0;
  }
  void grow() {
    std::vector<uint64_t> ok;
    std::vector<V> ov;
    ok.swap(keys_);
    ov.swap(vals_);
    alloc(ok.size() * 2);
    for (size_t i = 0; i < ok.size(); ++i) {
      if (!ok[i]) continue;
      size_t j = idx(ok[i]);
      while (keys_[j]) j = (j + 1) & mask_;
      keys_[j] = ok[i];
      vals_[j] = std::move(ov[i]);
      ++n_;
    }
  }

  std::vector<uint64_t> keys_;
  std::vector<V> vals_;
  size_t n_ = 0, mask_ = 0;
  int shift_ = 60;
};

template <class T, int N>
class SmallVec {
 public:
  T* begin() { return spilled() ? ext_.data() : inl_; }
  T* end() { return begin() + size(); }
  size_t size() const { return spilled() ? ext_.size() : n_; }
  bool empty() const { return size() == 0; }
  void push_back(const T& v) {
    if (!spilled()) {
      if (n_ < N) { inl_[n_++] = v; return; }
      ext_.assign(inl_, inl_ + n_);
      n_ = N + 1;  // marks "spilled"
    }
    ext_.push_back(v);
  }
  void erase(T* p) {
    if (spilled()) { ext_.erase(ext_.begin() + (p - ext_.data())); return; }
    for (T* q = p; q + 1 < inl_ + n_; ++q) *q = q[1];
    --n_;
  }
  void clear() { n_ = 0; ext_.clear(); }

 private:
  bool spilled() const { return n_ > N; }
  T inl_[N];
  uint32_t n_ = 0;
  std::vector<T> ext_;
};

}  // namespace apm
