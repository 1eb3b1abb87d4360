// Microbenchmark: host-side duration of hipMemcpyAsync H2D from pinned memory by size, with the
// stream idle and with the stream busy behind a long kernel.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

#define CK(x) do { hipError_t err_ = (x); if (err_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(err_)); return 1; } } while (0)

__global__ void k_spin(int* d, int iters) {
  int v = d[threadIdx.x];
  for (int i = 0; i < iters; ++i) v = v * 1103515245 + 12345;
  d[threadIdx.x] = v;
}

int main() {
  const size_t maxb = 16u << 20;
  char *h = nullptr, *dd = nullptr;
  int* d = nullptr;
  CK(hipHostMalloc(&h, maxb, hipHostMallocDefault));
  CK(hipMalloc(&dd, maxb));
  CK(hipMalloc(&d, 4096));
  CK(hipMemset(d, 0, 4096));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (int busy = 0; busy < 2; ++busy) {
    for (size_t b = 4096; b <= maxb; b *= 4) {
      double api = 0;
      const int reps = 20;
      for (int r = 0; r < reps; ++r) {
        CK(hipStreamSynchronize(s));
        if (busy) hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, d, 100000);
        const auto t0 = std::chrono::steady_clock::now();
        CK(hipMemcpyAsync(dd, h, b, hipMemcpyHostToDevice, s));
        api += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
      }
      CK(hipStreamSynchronize(s));
      std::printf("%s %8zu B: hipMemcpyAsync H2D host time %.1f us\n", busy ? "busy" : "idle", b, api / reps);
    }
  }
  return 0;
}
