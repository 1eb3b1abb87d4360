// Microbenchmark: GPU-side cost of the small copies / fills the engine issues per batch.
//   variant 0: kernel only
//   variant 1: kernel + 4-byte D2H into pinned memory (hipMemcpyAsync)
//   variant 2: kernel + 8-byte device memset
//   variant 3: kernel writing 4 bytes straight into host-mapped pinned memory
//   variant 4: kernel + 64 KB D2H
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_touch(int* d, int n, int* host_out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) d[i] += 1;
  if (host_out && i == 0) *host_out = d[0];
}

int main() {
  const int n = 1 << 20, iters = 200;
  int *d = nullptr, *h = nullptr, *hd = nullptr, *dm = nullptr;
  CK(hipMalloc(&d, n * 4));
  CK(hipMalloc(&dm, 1 << 16));
  CK(hipMemset(d, 0, n * 4));
  CK(hipHostMalloc(&h, 1 << 16, hipHostMallocDefault));
  CK(hipHostGetDevicePointer((void**)&hd, h, 0));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (int v = 0; v < 5; ++v) {
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipStreamSynchronize(s));
      const auto t0 = std::chrono::steady_clock::now();
      double api = 0;
      for (int it = 0; it < iters; ++it) {
        hipLaunchKernelGGL(k_touch, dim3(n / 256), dim3(256), 0, s, d, n, v == 3 ? hd : nullptr);
        const auto a0 = std::chrono::steady_clock::now();
        if (v == 1) CK(hipMemcpyAsync(h, dm, 4, hipMemcpyDeviceToHost, s));
        if (v == 2) CK(hipMemsetAsync(dm, 0, 8, s));
        if (v == 4) CK(hipMemcpyAsync(h, dm, 1 << 16, hipMemcpyDeviceToHost, s));
        api += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a0).count();
      }
      CK(hipStreamSynchronize(s));
      const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
      if (rep) std::printf("variant %d: %.1f us per iteration (extra-op API call %.1f us)\n", v, us / iters, api / iters);
    }
  }
  return 0;
}
