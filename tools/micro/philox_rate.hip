// Microbenchmark: cost of one Philox4x32-R call (R = 10 and 7) per wave on gfx950,
// and of a 24-bit-multiply hash alternative.  Prints ns per call per wave and
// the implied shader cycles per call per SIMD (at the measured clock, assume 2.4 GHz).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int R>
__device__ __forceinline__ uint4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c0 = hi1 ^ c1 ^ k0; c1 = lo1; c2 = hi0 ^ c3 ^ k1; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return make_uint4(c0, c1, c2, c3);
}

template <int R>
__global__ void bench(uint32_t* out, int iters, uint32_t seed) {
  uint32_t acc = 0;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  for (int i = 0; i < iters; ++i) {
    uint4 w = philox<R>(t, i, 7, 0, seed, seed ^ 0x1234u);
    acc ^= w.x ^ w.y ^ w.z ^ w.w;
  }
  out[t] = acc;
}

int main() {
  uint32_t* out;
  hipMalloc(&out, 256 * 1024 * 4 * sizeof(uint32_t));
  const int blocks = 256 * 8, threads = 256, iters = 2000;  // 8 waves per SIMD... 2048 blocks x 4 waves
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int rep = 0; rep < 2; ++rep) {
    for (int R : {10, 7}) {
      hipEventRecord(a);
      if (R == 10) hipLaunchKernelGGL(bench<10>, dim3(blocks), dim3(threads), 0, 0, out, iters, 1u);
      else hipLaunchKernelGGL(bench<7>, dim3(blocks), dim3(threads), 0, 0, out, iters, 1u);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      const double waves = (double)blocks * threads / 64.0;
      const double calls = waves * iters;                     // wave-calls
      const double per_simd = calls / 1024.0;                 // 256 CUs x 4 SIMDs
      printf("Philox4x32-%d: %.3f ms, %.1f cycles per wave-call per SIMD at 2.4 GHz\n", R, ms,
             ms * 1e-3 * 2.4e9 / per_simd);
    }
  }
  return 0;
}
