// Fleet baseline packing: per-service moments of the z-score baselines, for the RCCL all-reduce
// that merges every GPU's (server, service) series into one fleet-wide per-service baseline.
//
// dst[service][lag][stat] = {n_series_with_baseline, sum(mean), sum(mean^2)} where mean is the
// series' current LAG-window mean (the z-score "avg"), read from the O(1) running sums.  The
// layout is a dense fp64 matrix so one all_reduce(SUM) over xGMI merges all ranks; the merged
// per-service mean/variance of baselines is what the survey calls the global merge (§2.4).
#include "kernel_api.h"

namespace apm {

__global__ __launch_bounds__(256) void k_service_moments(const int32_t* __restrict__ series_service,
                                                         const uint8_t* __restrict__ active, int32_t n_series,
                                                         int32_t S, int32_t n_lags, int32_t n_services_cap,
                                                         const double* const* __restrict__ sums,
                                                         const double* const* __restrict__ comps,
                                                         const int32_t* const* __restrict__ cnts,
                                                         double* __restrict__ dst) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
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

}  // namespace apm

extern "C" void apm_service_moments(const int32_t* series_service, const uint8_t* active, int32_t n_series,
                                    int32_t S, int32_t n_lags, int32_t n_services_cap, const double* const* sums,
                                    const double* const* comps, const int32_t* const* cnts, double* dst,
                                    hipStream_t stream) {
  using namespace apm;
  HIP_OK(hipMemsetAsync(dst, 0, (size_t)n_services_cap * n_lags * NSTAT * 3 * sizeof(double), stream));
  if (n_series <= 0) return;
  hipLaunchKernelGGL(k_service_moments, dim3((n_series + 255) / 256), dim3(256), 0, stream, series_service, active,
                     n_series, S, n_lags, n_services_cap, sums, comps, cnts, dst);
}
