// Microbenchmark (measurement tool, not product): the band tick's memory pattern
// with 16-bit table cells and 8-bit payload cells, 16 cells per lane: table slab
// stream 32 B/lane read + write (NT), payload write 16 B/lane, K gathered 16 B/lane
// payload reads from random rows of the band's payload slab. Compare with
// stream_gather.hip (32-bit cells, 16-bit payload, 8 cells per lane).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint8_t u8x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16; return x;
}

// table [nb][n][B] u16; pay [nb][n][2][B] u8.  LPR = B/16 lanes per row.
template <int B, int K>
__global__ __launch_bounds__(256) void kband(uint16_t *table, uint8_t *pay, int n, int nb, int R, uint32_t *sink) {
  constexpr int LPR = B / 16, RPW = 64 / LPR;
  const int lane = threadIdx.x & 63, sub = lane / LPR, li = lane % LPR;
  const int U = n / RPW;
  const int u = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (u >= U * nb) return;
  const int band = u / U, r = (u - band * U) * RPW + sub;
  const size_t slab = (size_t)band * n;
  uint16_t *tr = table + (slab + r) * B + li * 16;
  u32x4 a = __builtin_nontemporal_load((const u32x4 *)tr);
  u32x4 b = __builtin_nontemporal_load((const u32x4 *)(tr + 8));
  u32x4 m[K > 0 ? K : 1];
#pragma unroll
  for (int j = 0; j < K; j++) {
    const int sn = (int)(mix(r * 8 + j + band * 131) % (uint32_t)R);
    m[j] = *(const u32x4 *)(pay + ((slab + sn) * 2 + 1) * B + li * 16);
  }
  u8x16 o = __builtin_bit_cast(u8x16, a ^ b);
#pragma unroll
  for (int j = 0; j < K; j++) o = __builtin_elementwise_min(o, __builtin_bit_cast(u8x16, m[j]));
  a += 1u; b += 1u;
  __builtin_nontemporal_store(a, (u32x4 *)tr);
  __builtin_nontemporal_store(b, (u32x4 *)(tr + 8));
  __builtin_nontemporal_store(__builtin_bit_cast(u32x4, o), (u32x4 *)(pay + ((slab + r) * 2 + 0) * B + li * 16));
  if (o[0] == 0x7b && o[5] == 0x11 && r == 3) sink[0] = 1;
}

template <int B, int K>
float run(uint16_t *table, uint8_t *pay, int n, int nb, int R, uint32_t *sink, int reps) {
  constexpr int RPW = 64 / (B / 16);
  const int grid = ((n / RPW) * nb + 3) / 4;
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL((kband<B, K>), dim3(grid), dim3(256), 0, 0, table, pay, n, nb, R, sink);
  hipEventRecord(e0);
  for (int i = 0; i < reps; i++) hipLaunchKernelGGL((kband<B, K>), dim3(grid), dim3(256), 0, 0, table, pay, n, nb, R, sink);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}

int main() {
  const int n = 65536, wp = 65536;
  uint16_t *table; uint8_t *pay; uint32_t *sink;
  hipMalloc(&table, (size_t)n * wp * 2);
  hipMalloc(&pay, (size_t)n * wp * 2);
  hipMalloc(&sink, 64);
  hipMemset(table, 0, (size_t)n * wp * 2);
  hipMemset(pay, 0, (size_t)n * wp * 2);
  const double cells = (double)n * wp;
  auto rep = [&](int B, int K, int R, float ms) {
    printf("narrow B=%3d K=%d R=%6d  %6.2f ms  hbm-min %5.2f TB/s  (%.2f ns per 1k cells)\n", B, K, R, ms,
           cells * 6 / ms / 1e9, ms * 1e6 / (cells / 1000));
    fflush(stdout);
  };
#define RUN(B, K, R) rep(B, K, R, run<B, K>(table, pay, n, wp / B, R, sink, 3))
  RUN(256, 0, n); RUN(512, 0, n);
  RUN(256, 5, 64); RUN(512, 5, 64);
  RUN(128, 5, n); RUN(256, 5, n); RUN(512, 5, n); RUN(1024, 5, n);
  RUN(256, 8, n);
  return 0;
}
