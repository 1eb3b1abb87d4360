// Small containers for the join workers' hot path.
//
// FlatMap<V>: open-addressing hash table keyed by a 64-bit hash (linear probing, power-of-two
// capacity, load <= 1/2, backward-shift deletion so there are no tombstones).  Key 0 marks an
// empty slot, so key 0 is stored as 1 (keys are FNV-1a hashes; see join.h for the collision
// stance).  References returned by find/emplace stay valid until the next insertion into the
// same map.
//
// SmallVec<T, N>: up to N elements inline, spills to the heap beyond that.  The join's partial
// maps hold one or two services per logId, so the common case allocates nothing; the spill is a
// single pointer so a map value stays within one cache line.
//
// Keys are hash_bytes() values (kernels/common.h), shared with the parse kernel.
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <utility>
#include <vector>

#include "../kernels/common.h"

namespace apm {

template <class V>
class FlatMap {
 public:
  explicit FlatMap(size_t cap = 1024) { alloc(pow2(cap)); }

  size_t size() const { return n_; }
  bool empty() const { return n_ == 0; }

  // Touch the home slot of `k` (key and value) ahead of a lookup: the join walks a batch's
  // events with a lookahead so the random map accesses overlap instead of serialising.
  void prefetch(uint64_t k) const {
    const size_t i = idx(fix(k));
    __builtin_prefetch(keys_.data() + i);
    __builtin_prefetch(vals_.data() + i);
  }

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
  SmallVec() = default;
  SmallVec(const SmallVec& o) { for (const T& v : o) push_back(v); }
  SmallVec(SmallVec&& o) noexcept : n_(o.n_), ext_(o.ext_) {
    std::copy(o.inl_, o.inl_ + (o.n_ <= N ? o.n_ : 0), inl_);
    o.n_ = 0;
    o.ext_ = nullptr;
  }
  SmallVec& operator=(const SmallVec& o) {
    if (this != &o) { clear(); for (const T& v : o) push_back(v); }
    return *this;
  }
  SmallVec& operator=(SmallVec&& o) noexcept {
    if (this != &o) {
      delete ext_;
      n_ = o.n_;
      ext_ = o.ext_;
      std::copy(o.inl_, o.inl_ + (o.n_ <= N ? o.n_ : 0), inl_);
      o.n_ = 0;
      o.ext_ = nullptr;
    }
    return *this;
  }
  ~SmallVec() { delete ext_; }

  T* begin() { return spilled() ? ext_->data() : inl_; }
  T* end() { return begin() + size(); }
  const T* begin() const { return spilled() ? ext_->data() : inl_; }
  const T* end() const { return begin() + size(); }
  size_t size() const { return spilled() ? ext_->size() : n_; }
  bool empty() const { return size() == 0; }
  void push_back(const T& v) {
    if (!spilled()) {
      if (n_ < N) { inl_[n_++] = v; return; }
      ext_ = new std::vector<T>(inl_, inl_ + n_);
      n_ = N + 1;  // marks "spilled"
    }
    ext_->push_back(v);
  }
  void erase(T* p) {
    if (spilled()) { ext_->erase(ext_->begin() + (p - ext_->data())); return; }
    for (T* q = p; q + 1 < inl_ + n_; ++q) *q = q[1];
    --n_;
  }
  void clear() {
    delete ext_;
    ext_ = nullptr;
    n_ = 0;
  }

 private:
  bool spilled() const { return n_ > N; }
  T inl_[N];
  uint32_t n_ = 0;
  std::vector<T>* ext_ = nullptr;
};

}  // namespace apm
