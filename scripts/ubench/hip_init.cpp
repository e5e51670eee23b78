// Measurement tool: wall time of bringing up the HIP runtime on device 0 (the fixed
// cost any GPU process pays before its first kernel; compare with ./Application).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
int main() {
  auto t0 = std::chrono::steady_clock::now();
  if (hipSetDevice(0) != hipSuccess) return 1;
  void *p = nullptr;
  if (hipMalloc(&p, 1 << 20) != hipSuccess) return 1;
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  auto t1 = std::chrono::steady_clock::now();
  (void)hipFree(p);
  printf("hip init + first alloc: %.3f s\n", std::chrono::duration<double>(t1 - t0).count());
  return 0;
}
