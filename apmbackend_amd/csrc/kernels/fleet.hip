// Fleet baseline packing: per-service moments of the z-score baselines, for the RCCL all-reduce
// that merges every GPU's (server, service) series into one fleet-wide per-service baseline.
//
// dst[service][lag][stat] = {n_series_with_baseline, sum(mean), sum(mean^2)} where mean is the
// series' current LAG-window mean (the z-score "avg"), read from the O(1) running sums.  The
// layout is a dense fp64 matrix so one all_reduce(SUM) over xGMI merges all ranks; the merged
// per-service mean/variance of baselines is what the survey calls the global merge (§2.4).
// Two implementations: the MFMA Gram kernel (default, deterministic: series added since the
// CSR snapshot go through a second, per-batch tail CSR accumulated by the same kernel) and a
// per-series fp64 atomic scatter (reference / fallback for more than two LAGs).
#include "kernel_api.h"

namespace apm {

__global__ __launch_bounds__(256) void k_service_moments(const int32_t* __restrict__ series_service,
                                                         const uint8_t* __restrict__ active, int32_t s_lo,
                                                         int32_t n_series, int32_t S, int32_t n_lags, int32_t n_services_cap,
                                                         const double* const* __restrict__ sums,
                                                         const double* const* __restrict__ comps,
                                                         const int32_t* const* __restrict__ cnts,
                                                         double* __restrict__ dst) {
  const int s = s_lo + blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_series || !active[s]) return;
  const int svc = series_service[s];
  if (svc < 0 || svc >= n_services_cap) return;
  for (int l = 0; l < n_lags; ++l) {
    for (int k = 0; k < NSTAT; ++k) {
      const int c = cnts[l][k * S + s];
      if (c <= 0) continue;
      const double m = (sums[l][k * S + s] + comps[l][k * S + s]) / (double)c;
      double* o = dst + (((size_t)svc * n_lags + l) * NSTAT + k) * 3;
      atomicAdd(o + 0, 1.0);
      atomicAdd(o + 1, m);
      atomicAdd(o + 2, m * m);
    }
  }
}

// ---- MFMA path: per-service Gram matrices on the matrix cores ---------------------------------
// With the series of each service listed contiguously (CSR, built on the host in series order),
// one wave per service accumulates G = F^T F over its series with v_mfma_f64_16x16x4f64, where
// row s of F holds 16 features of series s:
//   f = 0             1                                  (active series)
//   f = 1 .. P        v_p = 1 if (lag, stat) p has a baseline, else 0
//   f = P+1 .. 2P     x_p = that baseline mean, else 0                (P = n_lags * 3 <= 7)
// so G[v_p][v_p] = #series with a baseline, G[0][x_p] = sum of means, G[x_p][x_p] = sum of
// squared means -- the moments the fleet all-reduce merges -- and the off-diagonal blocks are
// the cross-moments between lags / stats.  One MFMA folds 4 series: lane l holds F[4c + l/16]
// [l % 16], which is both the A (16x4, F^T) and the B (4x16, F) operand.  The summation order
// is fixed by the series order, so the moments are bitwise reproducible (the atomic fallback's
// fp64 atomics are not).
typedef double apm_f64x4 __attribute__((ext_vector_type(4)));
constexpr int GRAM_WAVES = 4;

__global__ __launch_bounds__(GRAM_WAVES * 64) void k_service_gram(const int32_t* __restrict__ svc_off,
                                                                const int32_t* __restrict__ svc_ids,
                                                                const int32_t* __restrict__ svc_map,
                                                                int32_t accumulate,
                                                                const uint8_t* __restrict__ active,
                                                                int32_t n_services, int32_t S, int32_t n_lags,
                                                                const double* const* __restrict__ sums,
                                                                const double* const* __restrict__ comps,
                                                                const int32_t* const* __restrict__ cnts,
                                                                double* __restrict__ dst) {
  __shared__ double g[GRAM_WAVES][16][17];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int svc = blockIdx.x * GRAM_WAVES + wave;
  const int f = lane & 15, kk = lane >> 4;
  const int P = n_lags * NSTAT;
  const int lo = svc < n_services ? svc_off[svc] : 0, hi = svc < n_services ? svc_off[svc + 1] : 0;
  apm_f64x4 acc = {0.0, 0.0, 0.0, 0.0};
  for (int base = lo; base < hi; base += 4) {  // uniform across the wave
    double x = 0.0;
    const int j = base + kk;
    if (j < hi) {
      const int s = svc_ids[j];
      if (active[s]) {
        if (f == 0) {
          x = 1.0;
        } else if (f <= 2 * P) {
          const int p = f <= P ? f - 1 : f - 1 - P;
          const int l = p / NSTAT, k = p % NSTAT;
          const int c = cnts[l][k * S + s];
          if (c > 0) x = f <= P ? 1.0 : (sums[l][k * S + s] + comps[l][k * S + s]) / (double)c;
        }
      }
    }
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x, acc, 0, 0, 0);
  }
  // D[i][j] of v_mfma_f64_16x16x4f64: lane l, accumulator r holds row 4 * r + l / 16, column l % 16
  // (tests/test_engine_gpu.py::test_fleet_moments_mfma_gram_matches_atomic_scatter pins this)
#pragma unroll
  for (int r = 0; r < 4; ++r) g[wave][4 * r + kk][f] = acc[r];
  __syncthreads();
  if (svc < n_services && lane < P) {
    const int p = lane, l = p / NSTAT, k = p % NSTAT;
    const int row = svc_map ? svc_map[svc] : svc;  // tail CSR: entry -> service row
    double* o = dst + (((size_t)row * n_lags + l) * NSTAT + k) * 3;
    if (accumulate) {  // one wave per service, entries in fixed order: still deterministic
      o[0] += g[wave][1 + p][1 + p];
      o[1] += g[wave][0][1 + P + p];
      o[2] += g[wave][1 + P + p][1 + P + p];
    } else {
      o[0] = g[wave][1 + p][1 + p];
      o[1] = g[wave][0][1 + P + p];
      o[2] = g[wave][1 + P + p][1 + P + p];
    }
  }
}

}  // namespace apm

extern "C" int apm_service_gram(const int32_t* svc_off, const int32_t* svc_ids, const uint8_t* active,
                                int32_t n_services, int32_t S, int32_t n_lags, const double* const* sums,
                                const double* const* comps, const int32_t* const* cnts, double* dst,
                                hipStream_t stream, const int32_t* svc_map, int32_t accumulate) {
  using namespace apm;
  if (n_lags * NSTAT * 2 + 1 > 16) return -1;  // more features than one 16x16 Gram holds
  if (n_services <= 0) return 0;
  hipLaunchKernelGGL(k_service_gram, dim3((n_services + GRAM_WAVES - 1) / GRAM_WAVES), dim3(GRAM_WAVES * 64), 0,
                     stream, svc_off, svc_ids, svc_map, accumulate, active, n_services, S, n_lags, sums, comps, cnts,
                     dst);
  return 0;
}

extern "C" void apm_service_moments(const int32_t* series_service, const uint8_t* active, int32_t n_series,
                                    int32_t S, int32_t n_lags, int32_t n_services_cap, const double* const* sums,
                                    const double* const* comps, const int32_t* const* cnts, double* dst,
                                    hipStream_t stream) {
  using namespace apm;
  HIP_OK(hipMemsetAsync(dst, 0, (size_t)n_services_cap * n_lags * NSTAT * 3 * sizeof(double), stream));
  if (n_series <= 0) return;
  hipLaunchKernelGGL(k_service_moments, dim3((n_series + 255) / 256), dim3(256), 0, stream, series_service, active,
                     0, n_series, S, n_lags, n_services_cap, sums, comps, cnts, dst);
}

// Series [s_lo, n_series) added since the Gram kernel's CSR snapshot: atomically accumulated on
// top of the Gram output (no memset), so the CSR is rebuilt only when that tail grows large.
extern "C" void apm_service_moments_tail(const int32_t* series_service, const uint8_t* active, int32_t s_lo,
                                         int32_t n_series, int32_t S, int32_t n_lags, int32_t n_services_cap,
                                         const double* const* sums, const double* const* comps,
                                         const int32_t* const* cnts, double* dst, hipStream_t stream) {
  using namespace apm;
  if (n_series <= s_lo) return;
  hipLaunchKernelGGL(k_service_moments, dim3((n_series - s_lo + 255) / 256), dim3(256), 0, stream, series_service,
                     active, s_lo, n_series, S, n_lags, n_services_cap, sums, comps, cnts, dst);
}
