// K12: st / fs record encoding on the GPU (entries.js StatEntry.toCSVString :71-73,
// FullStatEntry.toCSVString :116-118, nf() :116).
//
// Every rollover emits one `st` line per live series and one `fs` line per (series, LAG) -- for
// 80k series and two LAGs that is ~25 MB of text per 10 s interval, far too much to format on
// the host thread that owns the pipeline.  The classic two-pass scheme:
//   pass 1  one lane per series in emission order: line lengths (st, sum over LAGs of fs)
//   scan    exclusive prefix sums (rocprim) -> byte offsets
//   pass 2  same lane re-formats straight into the output at its offset
// Number printing reproduces Number.prototype.toFixed exactly: the rounding decision uses the
// error-free product x*10^f = p + e (fma), ties to the larger n (ECMA-262 21.1.3.3), then the
// integer n is printed with the decimal point inserted f digits from the right.  Magnitudes
// >= 1e13 (where the exact-decision argument needs more care, and JS switches to exponent
// notation at 1e21) set a fallback flag and the host formats that rollover instead.
#include "kernel_api.h"  // (common.h pulls <cstring> in before rocprim)

#include <rocprim/rocprim.hpp>

namespace apm {

namespace {

struct Out {
  char* p;      // nullptr in the length pass
  uint32_t n = 0;
  __device__ __forceinline__ void c(char ch) {
    if (p) p[n] = ch;
    ++n;
  }
  __device__ __forceinline__ void s(const char* src, int len) {
    if (p)
      for (int i = 0; i < len; ++i) p[n + i] = src[i];
    n += len;
  }
  __device__ __forceinline__ void u(uint64_t v) {
    char buf[20];
    int k = 0;
    do { buf[k++] = (char)('0' + v % 10); v /= 10; } while (v);
    if (p)
      for (int i = 0; i < k; ++i) p[n + i] = buf[k - 1 - i];
    n += k;
  }
  __device__ __forceinline__ void i64(int64_t v) {
    if (v < 0) { c('-'); u((uint64_t)(-v)); } else u((uint64_t)v);
  }
  // nf(x, f): 'undefined' for NaN, else x.toFixed(f)
  __device__ __forceinline__ void fixed(double x, int f, bool& fallback) {
    if (x != x) { s("undefined", 9); return; }
    const bool neg = x < 0;
    const double ax = neg ? -x : x;
    if (!(ax < 1e13)) { fallback = true; return; }
    const double scale = f == 1 ? 10.0 : 100.0;
    const double pr = ax * scale;
    const double e = fma(ax, scale, -pr);
    const double q = floor(pr);
    const double d = (pr - q) - 0.5;
    uint64_t nn = (uint64_t)q;
    if (d > 0 || (d == 0 && e >= 0)) ++nn;
    if (neg) c('-');
    const uint64_t sc = f == 1 ? 10 : 100;
    u(nn / sc);
    c('.');
    const uint64_t fr = nn % sc;
    if (f == 2) { c((char)('0' + fr / 10)); c((char)('0' + fr % 10)); }
    else c((char)('0' + fr));
  }
};

__device__ __forceinline__ void head(Out& o, const char* tag, const FormatArgs& a, int32_t s) {
  o.s(tag, 3);
  o.i64(a.edge_ts);
  o.c('|');
  const int4 nm = a.series_names[s];
  o.s(a.names + nm.x, nm.y);
  o.c('|');
  o.s(a.names + nm.z, nm.w);
  o.c('|');
}

template <bool WRITE>
__device__ void format_series(const FormatArgs& a, int32_t i, uint32_t* st_len, uint32_t* fs_len, bool& fb) {
  const int32_t s = a.perm[i];
  const WinStat w = a.win[s];
  Out st{WRITE ? a.st_out + a.st_off[i] : nullptr};
  Out fs{WRITE ? a.fs_out + a.fs_off[i] : nullptr};
  if (w.active) {
    if (a.want_st) {
      head(st, "st|", a, s);
      st.fixed(w.tpm, 2, fb); st.c('|');
      st.fixed(w.avg, 1, fb); st.c('|');
      st.fixed(w.p75, 1, fb); st.c('|');
      st.fixed(w.p95, 1, fb); st.c('\n');
    }
    if (a.want_fs) {
      const double x[NSTAT] = {w.avg, w.p75, w.p95};
      for (int li = 0; li < a.n_lags; ++li) {
        const int l = a.lag_order[li];
        const ZOut z = a.z[l][s];
        head(fs, "fs|", a, s);
        fs.u((uint64_t)a.lag_value[l]);
        fs.c('|');
        fs.fixed(w.tpm, 2, fb);
        for (int k = 0; k < NSTAT; ++k) {
          fs.c('|');
          fs.fixed(x[k], 1, fb); fs.c(':');
          fs.fixed(z.mean[k], 1, fb); fs.c(':');
          fs.fixed(z.lb[k], 1, fb); fs.c(':');
          fs.fixed(z.ub[k], 1, fb); fs.c(':');
          // averageSignal is printed raw, the percentile signals through nf (entries.js:117)
          if (k == 0) fs.i64(z.sig[k]);
          else fs.fixed((double)z.sig[k], 1, fb);
        }
        fs.c('\n');
      }
    }
  }
  if (!WRITE) { st_len[i] = st.n; fs_len[i] = fs.n; }
}

__global__ __launch_bounds__(256) void k_format_len(FormatArgs a) {
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  bool fb = false;
  format_series<false>(a, i, a.st_len, a.fs_len, fb);
  if (fb) atomicOr(a.fallback, 1);
}

__global__ __launch_bounds__(256) void k_format_write(FormatArgs a) {
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  bool fb = false;
  format_series<true>(a, i, nullptr, nullptr, fb);
}

__global__ void k_fixed_batch(const double* x, int n, int f, char* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  bool fb = false;
  Out o{out + (size_t)i * 32};
  o.fixed(x[i], f, fb);
  if (fb) { o.n = 0; o.s("<fallback>", 10); }
  o.c('\0');
}

}  // namespace

}  // namespace apm

extern "C" {
using namespace apm;

size_t apm_format_tmp_bytes(int32_t n_max) {
  size_t b = 0;
  rocprim::exclusive_scan(nullptr, b, (uint32_t*)nullptr, (uint32_t*)nullptr, 0u, (size_t)n_max + 1,
                          rocprim::plus<uint32_t>(), (hipStream_t)0);
  return b;
}

// Lengths + scan: afterwards st_off/fs_off[0..n] hold exclusive offsets, [n] = total bytes.
// The *_len / *_off arrays hold n + 1 entries.
int apm_format_plan(FormatArgs* a, void* tmp, size_t tmp_bytes, hipStream_t stream) {
  if (a->n <= 0) return 0;
  HIP_OK(hipMemsetAsync(a->fallback, 0, 4, stream));
  HIP_OK(hipMemsetAsync(a->st_len + a->n, 0, 4, stream));
  HIP_OK(hipMemsetAsync(a->fs_len + a->n, 0, 4, stream));
  hipLaunchKernelGGL(k_format_len, dim3((a->n + 255) / 256), dim3(256), 0, stream, *a);
  size_t need = tmp_bytes;
  if (rocprim::exclusive_scan(tmp, need, a->st_len, a->st_off, 0u, (size_t)a->n + 1, rocprim::plus<uint32_t>(),
                              stream) != hipSuccess)
    return -1;
  if (rocprim::exclusive_scan(tmp, need, a->fs_len, a->fs_off, 0u, (size_t)a->n + 1, rocprim::plus<uint32_t>(),
                              stream) != hipSuccess)
    return -1;
  return 0;
}

// Test hook: nf(x[i], f) into 32-byte NUL-terminated slots.
void apm_format_fixed_batch(const double* d_x, int n, int f, char* d_out, hipStream_t stream) {
  if (n > 0) hipLaunchKernelGGL(k_fixed_batch, dim3((n + 255) / 256), dim3(256), 0, stream, d_x, n, f, d_out);
}

void apm_format_write(FormatArgs* a, hipStream_t stream) {
  if (a->n <= 0) return;
  hipLaunchKernelGGL(k_format_write, dim3((a->n + 255) / 256), dim3(256), 0, stream, *a);
}

}  // extern "C"
