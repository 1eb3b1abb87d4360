// K14 (new): per-JVM rollup of the interval's window statistics fused with the JVM's exogenous
// gauges -- the "multi-source join on GPU" of BASELINE.json config 4.
//
// Sources: the JMX poller's jx gauges (pull_jvm_stats.js: datasource pool, heap/metaspace,
// system load, classes, threads, EJB bean pool) and the VM load sampled by the engine host,
// kept per server in a small device table; the transaction side is this interval's K8 window
// statistics and the K10 signals of every series of the server.
//
//   k_server_rollup  one lane per series: integer atomics (deterministic) into per-server
//                    accumulators -- live series, window tx count, exact window elapsed sum
//                    (avg * n of integer samples), series with avg / p75 upper-bound signals,
//                    and an order-independent max of p95 (CAS max on the bit pattern of a
//                    non-negative double).
//   k_server_fuse    one lane per server: rates and means from the accumulators joined with the
//                    gauge row (heap / metaspace / datasource / bean-pool utilisation, load,
//                    threads, gauge age) and pressure flags.
#include "kernel_api.h"

namespace apm {

namespace {

// The accumulators of a server are hit by every one of its series (80k series over 8 JVMs: ~400k
// atomics on 48 words, serialised in the L2 atomic units).  A block first folds its 256 series
// into LDS copies of the accumulators (ds atomics), then adds each non-zero word to global memory
// once: ~300 blocks x 8 servers x 6 words.  All integer (or bit-pattern max): order-independent.
constexpr int RL_LDS_SERVERS = 64;

__device__ __forceinline__ void rollup_series(const RollupArgs& a, int s, unsigned long long* acc) {
  const WinStat w = a.win[s];
  if (!w.active) return;
  atomicAdd(acc + 0, 1ull);
  if (w.n > 0) {
    atomicAdd(acc + 1, (unsigned long long)w.n);
    const double sum = w.avg * (double)w.n;  // integer samples: exact up to 2^53
    atomicAdd(acc + 2, (unsigned long long)(long long)llround(sum));
    if (w.p95 == w.p95 && w.p95 >= 0) atomicMax(acc + 3, (unsigned long long)__double_as_longlong(w.p95));
  }
  bool sa = false, sp = false;
  for (int l = 0; l < a.n_lags; ++l) {
    const ZOut z = a.z[l][s];
    sa |= z.sig[0] > 0;
    sp |= z.sig[1] > 0;
  }
  if (sa) atomicAdd(acc + 4, 1ull);
  if (sp) atomicAdd(acc + 5, 1ull);
}

__global__ __launch_bounds__(256) void k_server_rollup(RollupArgs a) {
  __shared__ unsigned long long lacc[RL_LDS_SERVERS * ROLLUP_ACC];
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  const bool lds = a.n_servers <= RL_LDS_SERVERS;  // uniform
  if (lds) {
    for (int k = threadIdx.x; k < a.n_servers * ROLLUP_ACC; k += blockDim.x) lacc[k] = 0;
    __syncthreads();
  }
  if (s < a.n_series) {
    const int srv = a.series_server[s];
    if (srv >= 0 && srv < a.n_servers)
      rollup_series(a, s, lds ? lacc + (size_t)srv * ROLLUP_ACC : a.acc + (size_t)srv * ROLLUP_ACC);
  }
  if (!lds) return;
  __syncthreads();
  for (int k = threadIdx.x; k < a.n_servers * ROLLUP_ACC; k += blockDim.x) {
    const unsigned long long v = lacc[k];
    if (!v) continue;
    if (k % ROLLUP_ACC == 3) atomicMax(a.acc + k, v);
    else atomicAdd(a.acc + k, v);
  }
}

__global__ void k_server_fuse(RollupArgs a) {
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= a.n_servers) return;
  const unsigned long long* acc = a.acc + (size_t)v * ROLLUP_ACC;
  const double* g = a.ctx + (size_t)v * CTX_FIELDS;  // [0] = gauge timestamp (ms), [1..] gauges
  double* o = a.out + (size_t)v * ROLLUP_OUT;
  const double n = (double)acc[1];
  const double nan = apm_nan();
  o[0] = (double)acc[0];                                   // live series
  o[1] = n / a.tpm_div;                                    // tx per minute over the window
  o[2] = n > 0 ? (double)(long long)acc[2] / n : nan;      // mean elapsed
  o[3] = acc[3] ? __longlong_as_double((long long)acc[3]) : nan;  // max p95
  o[4] = (double)acc[4];
  o[5] = (double)acc[5];
  const bool have = g[0] > 0;
  auto ratio = [&](double num, double den) { return (have && den > 0) ? num / den : nan; };
  // gauge order = JmxEntry fields (entries.js:243-273)
  const double ds_inuse = g[1], ds_avail = g[3], heap_used = g[4], heap_max = g[6], meta_used = g[7],
               meta_committed = g[8], sysload = g[10], threads = g[12], bean_avail = g[14], bean_max = g[16],
               host_load = g[17];
  o[6] = ratio(heap_used, heap_max);
  o[7] = ratio(meta_used, meta_committed);
  o[8] = ratio(ds_inuse, ds_inuse + ds_avail);
  o[9] = have ? sysload : nan;
  o[10] = have ? threads : nan;
  o[11] = have && bean_max > 0 ? 1.0 - bean_avail / bean_max : nan;
  o[12] = have ? (double)(a.edge_ts - (long long)g[0]) / 1000.0 : nan;
  o[13] = host_load;
  unsigned flags = 0;
  if (o[6] == o[6] && o[6] > 0.9) flags |= 1;              // heap pressure
  if (o[8] == o[8] && o[8] > 0.9) flags |= 2;              // datasource pool saturated
  if (o[11] == o[11] && o[11] > 0.9) flags |= 4;           // EJB bean pool exhausted
  if (o[4] > 0 && o[0] > 0 && o[4] / o[0] > 0.25) flags |= 8;  // broad slowdown across services
  o[14] = (double)flags;
}

}  // namespace

}  // namespace apm

extern "C" void apm_server_rollup(apm::RollupArgs* a, hipStream_t stream) {
  using namespace apm;
  if (a->n_servers <= 0) return;
  HIP_OK(hipMemsetAsync(a->acc, 0, (size_t)a->n_servers * ROLLUP_ACC * 8, stream));
  if (a->n_series > 0)
    hipLaunchKernelGGL(k_server_rollup, dim3((a->n_series + 255) / 256), dim3(256), 0, stream, *a);
  hipLaunchKernelGGL(k_server_fuse, dim3((a->n_servers + 63) / 64), dim3(64), 0, stream, *a);
}
