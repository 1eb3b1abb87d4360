// Device helpers shared by the CDNA4 kernels (gfx950, wave64).
#pragma once
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "../apm_types.h"

#define APM_WAVE 64

#define HIP_OK(x)                                                                      \
  do {                                                                                 \
    hipError_t _e = (x);                                                               \
    if (_e != hipSuccess) {                                                            \
      fprintf(stderr, "HIP error %s at %s:%d: %s\n", hipGetErrorName(_e), __FILE__,    \
              __LINE__, hipGetErrorString(_e));                                        \
      abort();                                                                         \
    }                                                                                  \
  } while (0)

namespace apm {

__host__ __device__ inline double apm_nan() { return __builtin_nan(""); }

// ECMAScript MakeDay/MakeTime for integral fields (month 0-based, may be out of range).
__host__ __device__ inline int64_t days_from_civil(int64_t y, int64_t m /*1..12*/, int64_t d) {
  y -= m <= 2;
  const int64_t era = (y >= 0 ? y : y - 399) / 400;
  const int64_t yoe = y - era * 400;
  const int64_t mp = (m + 9) % 12;
  const int64_t doy = (153 * mp + 2) / 5 + d - 1;
  const int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + doe - 719468;
}

__host__ __device__ inline int64_t floordiv64(int64_t a, int64_t b) {
  int64_t q = a / b;
  if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
  return q;
}

__host__ __device__ inline int64_t make_date_ms(int64_t y, int64_t mon0, int64_t d, int64_t h,
                                                int64_t mi, int64_t s, int64_t ms) {
  const int64_t ym = y + floordiv64(mon0, 12);
  const int64_t mn = mon0 - floordiv64(mon0, 12) * 12;
  const int64_t day = days_from_civil(ym, mn + 1, 1) + d - 1;
  return day * 86400000LL + ((h * 60 + mi) * 60 + s) * 1000 + ms;
}

// Local -> UTC through a host-built transition table sorted by local start time.
struct TzTable {
  int n;
  int64_t local_start[64];
  int64_t offset_ms[64];
};

__host__ __device__ inline int64_t local_to_utc(const TzTable& tz, int64_t local_ms) {
  int lo = 0, hi = tz.n - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (tz.local_start[mid] <= local_ms) lo = mid; else hi = mid - 1;
  }
  return local_ms - tz.offset_ms[lo];
}

// JS Number.prototype.toFixed(f) followed by parseFloat: the value a downstream stage sees.
// Exact: the rounding decision uses the error-free product x*10^f = p + e (fma), ties to the
// larger n as ECMA-262 requires (on |x|, then the sign is reapplied).
__host__ __device__ inline double js_round_fixed(double x, int f) {
  if (x != x) return x;
  const double scale = f == 0 ? 1.0 : (f == 1 ? 10.0 : (f == 2 ? 100.0 : 1000.0));
  const bool neg = x < 0;
  const double ax = neg ? -x : x;
  if (ax >= 1e21) return x;
  const double p = ax * scale;
  const double e = fma(ax, scale, -p);
  const double q = floor(p);
  const double d = (p - q) - 0.5;
  double n = q;
  if (d > 0 || (d == 0 && e >= 0)) n = q + 1;
  double r = n / scale;
  return neg ? -r : r;
}

// Join-key hash, shared by the parse kernel (which hashes logIds and service names into the
// Event) and the host join / checkpoints: word-at-a-time, one 64x64->128 multiply folded per
// 8 bytes (wyhash-style).  FNV-1a's byte-serial multiply chain cost ~4 cycles per byte.
__host__ __device__ inline uint64_t hash_mix(uint64_t a, uint64_t b) {
  const __uint128_t r = (__uint128_t)a * b;
  return (uint64_t)r ^ (uint64_t)(r >> 64);
}

constexpr uint64_t kHashSeed = 0x243f6a8885a308d3ULL;     // logId keys, plain service names
constexpr uint64_t kHashSeedEjb = 0x13198a2e03707344ULL;  // "S:" + EJB service names

__host__ __device__ inline uint64_t hash_bytes(const void* data, size_t n, uint64_t seed = kHashSeed) {
  const uint8_t* p = static_cast<const uint8_t*>(data);
  uint64_t h = seed ^ hash_mix(n ^ 0xa0761d6478bd642fULL, 0xe7037ed1a0b428dbULL);
  while (n >= 8) {
    uint64_t w;
    memcpy(&w, p, 8);
    h = hash_mix(h ^ w, 0x8ebc6af09c88c6e3ULL);
    p += 8;
    n -= 8;
  }
  if (n) {
    uint64_t w = 0;
    memcpy(&w, p, n);
    h = hash_mix(h ^ w ^ ((uint64_t)n << 59), 0x589965cc75374cc3ULL);
  }
  return hash_mix(h, 0x1d8e4e27c47d124fULL);
}

// 64-bit FNV-1a (host and device agree; used for dictionary keys).
__host__ __device__ inline uint64_t fnv1a64(const uint8_t* p, int n, uint64_t h = 1469598103934665603ULL) {
  for (int i = 0; i < n; ++i) { h ^= p[i]; h *= 1099511628211ULL; }
  return h;
}

}  // namespace apm
