// Microbenchmark (measurement tool, not product): the band tick's memory pattern with
// 16-bit table cells and 4-bit payload nibbles (round-2 layout), 16 cells per lane:
// table slab stream 32 B/lane read + write (NT), payload write 8 B/lane, K gathered
// 8 B/lane payload reads from random rows of the band's payload slab.
//   DEP = 0: sender ids from a hash (no dependent load before the gathers)
//   DEP = 1: sender ids loaded from an inbox array first (the real kernel's chain)
// Prints ms per sweep of an N = 65,536 x 65,536 table; compare with gm_s_band.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16; return x;
}

// table [nb][n][B] u16; pay [nb][n][2][B/2] bytes; inbox [n][8] i32
// XCD = 1: workgroups are dispatched round-robin over the 8 XCDs, so workgroup w runs on
// XCD w % 8; map it to band 8*(j / BPB) + w % 8 (j = w / 8, BPB workgroups per band): every
// XCD sweeps its own bands, and a band's payload slab is gathered through one L2 only
template <int B, int K, int DEP, int XCD = 0>
__global__ __launch_bounds__(256) void kband(uint16_t *table, uint8_t *pay, const int *inbox, int n, int nb,
                                             uint32_t *sink) {
  constexpr int LPR = B / 16, RPW = 64 / LPR;
  const int lane = threadIdx.x & 63, sub = lane / LPR, li = lane % LPR;
  const int U = n / RPW;
  int u = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (XCD) {
    const int bpb = U / 4, w = blockIdx.x, j = w >> 3;
    u = (8 * (j / bpb) + (w & 7)) * U + (j % bpb) * 4 + (threadIdx.x >> 6);
  }
  if (u >= U * nb) return;
  const int band = u / U, r = (u - band * U) * RPW + sub;
  const size_t slab = (size_t)band * n;
  uint16_t *tr = table + (slab + r) * B + li * 16;
  u32x4 a = __builtin_nontemporal_load((const u32x4 *)tr);
  u32x4 b = __builtin_nontemporal_load((const u32x4 *)(tr + 8));
  int snd[8];
  if (DEP) {
    const int4 x = *(const int4 *)(inbox + (size_t)r * 8), y = *(const int4 *)(inbox + (size_t)r * 8 + 4);
    snd[0] = x.x; snd[1] = x.y; snd[2] = x.z; snd[3] = x.w; snd[4] = y.x; snd[5] = y.y; snd[6] = y.z; snd[7] = y.w;
  } else {
#pragma unroll
    for (int j = 0; j < 8; j++) snd[j] = (int)(mix(r * 8 + j + band * 131) % (uint32_t)n);
  }
  u32x2 m[K > 0 ? K : 1];
#pragma unroll
  for (int j = 0; j < K; j++) m[j] = *(const u32x2 *)(pay + (slab + snd[j]) * B + B / 2 + li * 8);
  u16x2 acc = __builtin_bit_cast(u16x2, a.x ^ b.y);
#pragma unroll
  for (int j = 0; j < K; j++) {
    acc = __builtin_elementwise_max(acc, __builtin_bit_cast(u16x2, m[j].x));
    acc = __builtin_elementwise_max(acc, __builtin_bit_cast(u16x2, m[j].y) << (u16x2)(4));
  }
  a += 1u; b += 1u;
  __builtin_nontemporal_store(a, (u32x4 *)tr);
  __builtin_nontemporal_store(b, (u32x4 *)(tr + 8));
  const u32x2 o = {__builtin_bit_cast(uint32_t, acc), a.y};
  __builtin_nontemporal_store(o, (u32x2 *)(pay + (slab + r) * B + li * 8));
  if (acc.x == 0x7b && r == 3) sink[0] = 1;
}

template <int B, int K, int DEP, int XCD = 0>
float run(uint16_t *table, uint8_t *pay, const int *inbox, int n, int nb, uint32_t *sink, int reps) {
  constexpr int RPW = 64 / (B / 16);
  const int grid = ((n / RPW) * nb + 3) / 4;
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL((kband<B, K, DEP, XCD>), dim3(grid), dim3(256), 0, 0, table, pay, inbox, n, nb, sink);
  hipEventRecord(e0);
  for (int i = 0; i < reps; i++)
    hipLaunchKernelGGL((kband<B, K, DEP, XCD>), dim3(grid), dim3(256), 0, 0, table, pay, inbox, n, nb, sink);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}

__global__ void fill_inbox(int *inbox, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n * 8) inbox[i] = (int)(mix(i * 2654435761u) % (uint32_t)n);
}

int main() {
  const int n = 65536, wp = 65536;
  uint16_t *table; uint8_t *pay; int *inbox; uint32_t *sink;
  hipMalloc(&table, (size_t)n * wp * 2);
  hipMalloc(&pay, (size_t)n * wp);
  hipMalloc(&inbox, (size_t)n * 8 * 4);
  hipMalloc(&sink, 64);
  hipMemset(table, 0, (size_t)n * wp * 2);
  hipMemset(pay, 0, (size_t)n * wp);
  hipLaunchKernelGGL(fill_inbox, dim3(n * 8 / 256), dim3(256), 0, 0, inbox, n);
  const double cells = (double)n * wp;
  auto rep = [&](const char *what, int B, int K, float ms) {
    printf("nibble %-8s B=%3d K=%d  %6.3f ms  dram-min %5.2f TB/s\n", what, B, K, ms, cells * 5 / ms / 1e9);
    fflush(stdout);
  };
#define RUN(B, K, D) rep(D ? "inbox" : "hash", B, K, run<B, K, D>(table, pay, inbox, n, wp / B, sink, 3))
#define RUNX(B, K, D) rep(D ? "inbox-xcd" : "hash-xcd", B, K, run<B, K, D, 1>(table, pay, inbox, n, wp / B, sink, 3))
  RUN(1024, 0, 0); RUN(1024, 5, 1); RUN(512, 5, 1); RUN(256, 5, 1); RUN(128, 5, 1); RUN(64, 5, 1);
  RUNX(1024, 5, 1); RUNX(512, 5, 1); RUNX(256, 5, 1); RUNX(128, 5, 1); RUNX(64, 5, 1);
  RUN(128, 0, 0); RUN(64, 0, 0);
  return 0;
}
