// Microbenchmark: host cost of enqueueing work behind a cross-stream event wait.
// Stream A runs a ~300 us kernel; B waits on an event recorded after it, then enqueues a tiny
// kernel: how long does that enqueue (and the wait call) block the host?
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_spin(int* d, int iters) {
  int v = d[threadIdx.x];
  for (int i = 0; i < iters; ++i) v = v * 1103515245 + 12345;
  d[threadIdx.x] = v;
}
__global__ void k_tiny(int* d) { d[threadIdx.x] += 1; }

static double us_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t).count();
}

int main() {
  int* d = nullptr;
  CK(hipMalloc(&d, 1 << 20));
  CK(hipMemset(d, 0, 1 << 20));
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  hipEvent_t ev, evt;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  CK(hipEventCreate(&evt));
  for (int variant = 0; variant < 4; ++variant) {
    double t_wait = 0, t_launch = 0, t_total = 0;
    const int reps = 20;
    for (int r = 0; r < reps; ++r) {
      CK(hipDeviceSynchronize());
      hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, a, d, 200000);  // long-running on A
      hipEvent_t evx = variant == 3 ? evt : ev;
      CK(hipEventRecord(evx, a));
      auto t0 = std::chrono::steady_clock::now();
      if (variant >= 1) CK(hipStreamWaitEvent(b, evx, 0));
      t_wait += us_since(t0);
      auto t1 = std::chrono::steady_clock::now();
      if (variant == 2) hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, a, d + 4096);  // same stream as the long one
      else hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, b, d + 4096);
      t_launch += us_since(t1);
      t_total += us_since(t0);
      CK(hipDeviceSynchronize());
    }
    auto t2 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, a, d, 200000);
    CK(hipDeviceSynchronize());
    const double spin = us_since(t2);
    std::printf("variant %d (%s): wait %.1f us, launch %.1f us (long kernel %.0f us)\n", variant,
                variant == 0 ? "no wait" : variant == 1 ? "wait, launch on B" : variant == 2 ? "launch on A" : "timing event",
                t_wait / reps, t_launch / reps, spin);
  }
  return 0;
}
