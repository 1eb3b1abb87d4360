// Microbenchmark: does a thread blocked in hipStreamSynchronize / hipEventSynchronize on one
// stream delay another thread's enqueues (hipMemcpyAsync H2D, kernel launch) on another stream?
#include <hip/hip_runtime.h>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <thread>

#define CK(x) do { hipError_t err_ = (x); if (err_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(err_)); std::abort(); } } while (0)

__global__ void k_spin(int* d, int iters) {
  int v = d[threadIdx.x];
  for (int i = 0; i < iters; ++i) v = v * 1103515245 + 12345;
  d[threadIdx.x] = v;
}
__global__ void k_tiny(int* d) { d[threadIdx.x] += 1; }

int main() {
  int *d1 = nullptr, *d2 = nullptr;
  char *h = nullptr, *dd = nullptr;
  CK(hipMalloc(&d1, 4096)); CK(hipMalloc(&d2, 4096));
  CK(hipMemset(d1, 0, 4096)); CK(hipMemset(d2, 0, 4096));
  CK(hipHostMalloc(&h, 1 << 20, hipHostMallocDefault));
  CK(hipMalloc(&dd, 1 << 20));
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  for (int mode = 0; mode < 3; ++mode) {  // 0 no waiter, 1 stream-sync waiter, 2 event-sync waiter
    std::atomic<bool> stop{false};
    std::thread waiter([&] {
      while (!stop.load()) {
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, a, d1, 200000);
        if (mode == 1) CK(hipStreamSynchronize(a));
        else if (mode == 2) { CK(hipEventRecord(ev, a)); CK(hipEventSynchronize(ev)); }
        else { CK(hipStreamSynchronize(a)); }
      }
    });
    double t_copy = 0, t_launch = 0, worst = 0;
    const int reps = 2000;
    if (mode == 0) { stop = true; waiter.join(); }
    for (int r = 0; r < reps; ++r) {
      const auto t0 = std::chrono::steady_clock::now();
      CK(hipMemcpyAsync(dd, h, 1 << 20, hipMemcpyHostToDevice, b));
      const auto t1 = std::chrono::steady_clock::now();
      hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, b, d2);
      const auto t2 = std::chrono::steady_clock::now();
      const double c = std::chrono::duration<double, std::micro>(t1 - t0).count();
      t_copy += c;
      t_launch += std::chrono::duration<double, std::micro>(t2 - t1).count();
      if (c > worst) worst = c;
      if (r % 64 == 0) CK(hipStreamSynchronize(b));
    }
    if (mode != 0) { stop = true; waiter.join(); }
    CK(hipDeviceSynchronize());
    std::printf("waiter=%s: H2D call %.1f us (worst %.0f), launch %.1f us\n",
                mode == 0 ? "none" : mode == 1 ? "streamSync" : "eventSync", t_copy / reps, worst, t_launch / reps);
  }
  return 0;
}
