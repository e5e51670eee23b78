// Micro-benchmark: throughput of the mt19937 init step v = 1812433253 * (v ^ (v >> 30)) + i on gfx950,
// with the 32-bit multiply as v_mul_lo_u32 (native) against a 24-bit-multiply decomposition.
// Dependent chains of 4096 steps, 64 lanes x many waves; prints ns per step per wave.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint32_t mul_native(uint32_t v) { return 1812433253u * v; }
// 0x6C078965 = hi8 0x6C, lo24 0x078965; (a * b) mod 2^32 = a_lo24 * b_lo24 (low 32 bits) +
// ((a_hi8 * b_lo8 + a_lo8 * b_hi8) mod 256) << 24
__device__ __forceinline__ uint32_t u24(uint32_t a, uint32_t b) {  // v_mul_u32_u24 (the compiler folds __umul24 back)
  uint32_t r;
  asm volatile("v_mul_u32_u24 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ uint32_t mul_u24x(uint32_t a) {
  const uint32_t p0 = u24(a, 0x078965u);
  const uint32_t p1 = u24(a >> 24, 0x65u) + u24(a, 0x6Cu);
  return p0 + (p1 << 24);
}

template <int MODE>
__global__ __launch_bounds__(256) void chain(uint32_t *out, int steps) {
  uint32_t v = blockIdx.x * 256 + threadIdx.x;
  for (int i = 1; i <= steps; i++) {
    const uint32_t x = v ^ (v >> 30);
    v = (MODE == 0 ? mul_native(x) : mul_u24x(x)) + (uint32_t)i;
  }
  out[blockIdx.x * 256 + threadIdx.x] = v;
}

int main() {
  const int blocks = 256 * 8 * 4, steps = 4096;  // 8 waves per SIMD x 1024 SIMDs
  uint32_t *d;
  hipMalloc(&d, sizeof(uint32_t) * blocks * 256);
  uint32_t h0, h1;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int mode = 0; mode < 2; mode++) {
    for (int rep = 0; rep < 3; rep++) {
      hipEventRecord(a);
      if (mode == 0) hipLaunchKernelGGL(chain<0>, dim3(blocks), dim3(256), 0, 0, d, steps);
      else hipLaunchKernelGGL(chain<1>, dim3(blocks), dim3(256), 0, 0, d, steps);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      const double waves = blocks * 4.0;
      printf("mode %s rep %d: %.3f ms, %.2f cycles per step per SIMD-wave at 2.4 GHz\n",
             mode ? "u24x" : "native", rep, ms, ms * 1e-3 * 2.4e9 * 1024 / (waves * steps));
    }
    hipMemcpy(mode ? &h1 : &h0, d + 12345, 4, hipMemcpyDeviceToHost);
  }
  printf("check %s (%u %u)\n", h0 == h1 ? "same" : "DIFFER", h0, h1);
  return h0 == h1 ? 0 : 1;
}
