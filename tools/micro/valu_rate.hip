// VALU issue-rate probe: cycles per wave-instruction of v_mad_u64_u32, v_bitop3_b32 (xor3) and v_fma_f32,
// 8 independent chains per lane, 8 waves per SIMD (enough to hide latency).
//   hipcc --offload-arch=gfx950 -O3 tools/micro/valu_rate.hip -o /tmp/valu_rate && /tmp/valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int kIters = 4096;

__global__ void __launch_bounds__(256) k_mad(uint32_t* out, uint32_t seed) {
  uint32_t x[8];
  for (int i = 0; i < 8; ++i) x[i] = seed + threadIdx.x * 8 + i;
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint64_t p = (uint64_t)0xD2511F53u * x[i];
      x[i] = (uint32_t)(p >> 32) ^ (uint32_t)p;
    }
  }
  uint32_t r = 0;
  for (int i = 0; i < 8; ++i) r ^= x[i];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

__global__ void __launch_bounds__(256) k_xor3(uint32_t* out, uint32_t seed) {
  uint32_t x[8];
  for (int i = 0; i < 8; ++i) x[i] = seed + threadIdx.x * 8 + i;
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = __builtin_amdgcn_bitop3_b32(x[i], x[(i + 1) & 7], seed + it, 0x96);
  }
  uint32_t r = 0;
  for (int i = 0; i < 8; ++i) r ^= x[i];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

__global__ void __launch_bounds__(256) k_fma(float* out, float seed) {
  float x[8];
  for (int i = 0; i < 8; ++i) x[i] = seed + threadIdx.x + i;
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = __builtin_fmaf(x[i], 0.999f, 0.5f);
  }
  float r = 0;
  for (int i = 0; i < 8; ++i) r += x[i];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <typename F>
float time_it(F f) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) f();
  hipEventRecord(a);
  for (int i = 0; i < 10; ++i) f();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / 10;
}

int main() {
  const int blocks = 256 * 8;  // 8 workgroups of 4 waves per CU -> 8 waves per SIMD
  void* buf;
  hipMalloc(&buf, (size_t)blocks * 256 * 4);
  const double wave_instr_per_simd = (double)blocks * 4 / 1024 * kIters * 8;  // per SIMD
  float t_mad = time_it([&] { hipLaunchKernelGGL(k_mad, dim3(blocks), dim3(256), 0, 0, (uint32_t*)buf, 1u); });
  float t_x = time_it([&] { hipLaunchKernelGGL(k_xor3, dim3(blocks), dim3(256), 0, 0, (uint32_t*)buf, 1u); });
  float t_f = time_it([&] { hipLaunchKernelGGL(k_fma, dim3(blocks), dim3(256), 0, 0, (float*)buf, 1.f); });
  // per wave-instruction of the probed op, in ns per SIMD; at ~2.1-2.4 GHz multiply by the clock for cycles
  printf("mad_u64_u32 (+1 xor): %.3f ms  -> %.2f ns per (mad + xor) wave-pair per SIMD\n", t_mad, t_mad * 1e6 / wave_instr_per_simd);
  printf("bitop3 xor3        : %.3f ms  -> %.2f ns per wave-instr per SIMD\n", t_x, t_x * 1e6 / wave_instr_per_simd);
  printf("fma_f32            : %.3f ms  -> %.2f ns per wave-instr per SIMD\n", t_f, t_f * 1e6 / wave_instr_per_simd);
  hipFree(buf);
  return 0;
}
