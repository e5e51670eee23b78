// Microbenchmark (measurement tool, not product): the memory pattern of the SCALED
// band tick on MI355X. A "table" slab stream (16 B/lane read + write, NT) plus a
// payload write stream (16 B/lane per 8 cells -> half the table bytes), plus K
// gathered 16 B/lane payload reads per lane from random rows of a region of R rows
// (same column offset), at band width B (lanes per row = B/8).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16; return x;
}

// n rows x B columns per band, nb bands. table [nb][n][B] u32; pay [nb][n][2][B] u16.
template <int B, int K>
__global__ __launch_bounds__(256) void kband(uint32_t *table, uint16_t *pay, int n, int nb, int R, int persistent,
                                             uint32_t *sink) {
  constexpr int LPR = B / 8, RPW = 64 / LPR;
  const int lane = threadIdx.x & 63, sub = lane / LPR, li = lane % LPR;
  const int U = n / RPW, total = U * nb;
  int u = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int W = persistent ? gridDim.x * 4 : total;
  uint32_t acc = 0;
  for (; u < total; u += W) {
    const int band = u / U, r = (u - band * U) * RPW + sub;
    const size_t slab = (size_t)band * n;
    uint32_t *tr = table + (slab + r) * B + li * 8;
    u32x4 a = __builtin_nontemporal_load((const u32x4 *)tr);
    u32x4 b = __builtin_nontemporal_load((const u32x4 *)(tr + 4));
    u32x4 m[K > 0 ? K : 1];
#pragma unroll
    for (int j = 0; j < K; j++) {
      const int sn = (int)(mix(r * 8 + j + band * 131) % (uint32_t)R);
      m[j] = *(const u32x4 *)(pay + ((slab + sn) * 2 + 1) * B + li * 8);
    }
    u32x4 o = a ^ b;
#pragma unroll
    for (int j = 0; j < K; j++) o = __builtin_elementwise_max(o, m[j]);
    a += 1u; b += 1u;
    __builtin_nontemporal_store(a, (u32x4 *)tr);
    __builtin_nontemporal_store(b, (u32x4 *)(tr + 4));
    __builtin_nontemporal_store(o, (u32x4 *)(pay + ((slab + r) * 2 + 0) * B + li * 8));
    acc += o.x;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int B, int K>
float run(uint32_t *table, uint16_t *pay, int n, int nb, int R, int persistent, uint32_t *sink, int reps) {
  int dev, cus, per;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kband<B, K>, 256, 0);
  constexpr int RPW = 64 / (B / 8);
  const int total = (n / RPW) * nb;
  const int grid = persistent ? cus * per : (total + 3) / 4;
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL((kband<B, K>), dim3(grid), dim3(256), 0, 0, table, pay, n, nb, R, persistent, sink);
  hipEventRecord(e0);
  for (int i = 0; i < reps; i++)
    hipLaunchKernelGGL((kband<B, K>), dim3(grid), dim3(256), 0, 0, table, pay, n, nb, R, persistent, sink);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}

int main(int argc, char **argv) {
  const int n = 65536, wp = 65536;
  uint32_t *table; uint16_t *pay; uint32_t *sink;
  hipMalloc(&table, (size_t)n * wp * 4);
  hipMalloc(&pay, (size_t)n * wp * 4);
  hipMalloc(&sink, 64);
  hipMemset(table, 0, (size_t)n * wp * 4);
  hipMemset(pay, 0, (size_t)n * wp * 4);
  const double stream_b = (double)n * wp * 10;  // 4 r + 4 w + 2 w
  auto rep = [&](const char *name, int B, int K, int R, int pers, float ms) {
    const double gath = (double)n * wp * 2 * K;
    printf("%-10s B=%3d K=%d R=%6d pers=%d  %7.2f ms  stream %5.2f TB/s  total(alg) %5.2f TB/s\n", name, B, K, R, pers,
           ms, stream_b / ms / 1e9, (stream_b + gath) / ms / 1e9);
    fflush(stdout);
  };
#define RUN(B, K, R, P) rep("band", B, K, R, P, run<B, K>(table, pay, n, wp / B, R, P, sink, 3))
  for (int P = 0; P < 2; P++) {
    RUN(128, 0, n, P); RUN(512, 0, n, P);
    RUN(128, 5, 64, P); RUN(512, 5, 64, P);
    RUN(128, 5, n, P); RUN(512, 5, n, P);
  }
  RUN(64, 5, n, 1); RUN(256, 5, n, 1);
  RUN(128, 8, n, 1); RUN(128, 3, n, 1);
  return 0;
}
