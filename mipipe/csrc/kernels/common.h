// Shared device helpers for the mipipe CDNA4 (gfx950) kernels.
//
// * bf16 <-> f32: bf16 is carried as raw uint16 in memory; conversion to f32 is
//   a shift, conversion back is a plain cast to clang's __bf16 (hipcc emits
//   v_cvt_pk_bf16_f32 on gfx950, which rounds to nearest-even and keeps NaNs).
// * wave64 reductions with __shfl_xor (64 lanes: never 32).
// * Philox4x32-10 counter-based RNG keyed by the (seed, offset) that the torch
//   device generator hands out, so dropout masks replay bit-exactly under
//   activation recompute.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mipipe {

typedef uint16_t bf16_t;
typedef __attribute__((ext_vector_type(8))) unsigned short u16x8;
typedef __attribute__((ext_vector_type(4))) unsigned short u16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;

constexpr int kWave = 64;

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}

template <typename T>
struct Io;

template <>
struct Io<float> {
  static __device__ __forceinline__ float load(const float* p) { return *p; }
  static __device__ __forceinline__ void store(float* p, float v) { *p = v; }
  // 8 consecutive elements
  static __device__ __forceinline__ void load8(const float* p, float (&v)[8]) {
    const float4* q = reinterpret_cast<const float4*>(p);
    float4 a = q[0], b = q[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  static __device__ __forceinline__ void store8(float* p, const float (&v)[8]) {
    float4* q = reinterpret_cast<float4*>(p);
    q[0] = make_float4(v[0], v[1], v[2], v[3]);
    q[1] = make_float4(v[4], v[5], v[6], v[7]);
  }
};

template <>
struct Io<bf16_t> {
  static __device__ __forceinline__ float load(const bf16_t* p) { return bf2f(*p); }
  static __device__ __forceinline__ void store(bf16_t* p, float v) { *p = f2bf(v); }
  static __device__ __forceinline__ void load8(const bf16_t* p, float (&v)[8]) {
    u16x8 r = *reinterpret_cast<const u16x8*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = bf2f(r[i]);
  }
  static __device__ __forceinline__ void store8(bf16_t* p, const float (&v)[8]) {
    bf16x8 r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i] = (__bf16)v[i];
    *reinterpret_cast<bf16x8*>(p) = r;
  }
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum of two values (blockDim.x multiple of 64, <= 1024).
// `scratch` must hold 2 * (blockDim.x / 64) floats.
__device__ __forceinline__ void block_sum2(float& a, float& b, float* scratch) {
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
  a = wave_sum(a);
  b = wave_sum(b);
  if (lane == 0) {
    scratch[wid] = a;
    scratch[nw + wid] = b;
  }
  __syncthreads();
  float ta = 0.f, tb = 0.f;
  for (int w = 0; w < nw; ++w) {
    ta += scratch[w];
    tb += scratch[nw + w];
  }
  a = ta;
  b = tb;
  __syncthreads();
}

// ---------------------------------------------------------------- Philox4x32-10
struct Philox {
  uint32_t c0, c1, c2, c3;
  uint32_t k0, k1;

  __device__ __forceinline__ Philox(uint64_t seed, uint64_t subsequence, uint64_t offset) {
    k0 = (uint32_t)seed;
    k1 = (uint32_t)(seed >> 32);
    c0 = (uint32_t)subsequence;
    c1 = (uint32_t)(subsequence >> 32);
    c2 = (uint32_t)offset;
    c3 = (uint32_t)(offset >> 32);
  }

  // Returns 4 uniform 32-bit words for the current counter.
  __device__ __forceinline__ uint4 next4() const {
    uint32_t x0 = c0, x1 = c1, x2 = c2, x3 = c3;
    uint32_t a = k0, b = k1;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
      const uint64_t p0 = (uint64_t)0xD2511F53u * x0;
      const uint64_t p1 = (uint64_t)0xCD9E8D57u * x2;
      const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
      const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
      x0 = __builtin_amdgcn_bitop3_b32(hi1, x1, a, 0x96);  // hi1 ^ x1 ^ a in one v_bitop3_b32 (0x96 = xor3)
      x1 = lo1;
      x2 = __builtin_amdgcn_bitop3_b32(hi0, x3, b, 0x96);
      x3 = lo0;
      a += 0x9E3779B9u;
      b += 0xBB67AE85u;
    }
    return make_uint4(x0, x1, x2, x3);
  }
};

// Keep-mask bits for 4 consecutive elements starting at `group*4` of a tensor:
// element kept iff its uniform word >= p * 2^32.
__device__ __forceinline__ uint32_t dropout_keep4(uint64_t seed, uint64_t offset, uint64_t group, uint32_t threshold) {
  uint4 r = Philox(seed, group, offset).next4();
  return (uint32_t)(r.x >= threshold) | ((uint32_t)(r.y >= threshold) << 1) | ((uint32_t)(r.z >= threshold) << 2) |
         ((uint32_t)(r.w >= threshold) << 3);
}

// 8 consecutive elements starting at a multiple of 8 from ONE Philox block:
// element i draws the 16-bit uniform (word i/2 >> 16*(i&1)) and is kept iff it
// is >= floor(p * 2^16).  The RNG is the VALU cost of a dropout pass (10
// rounds x 4 quarter-rate multiplies per block), so halving the blocks per
// element matters for the memory-bound LayerNorm / embedding kernels; p is
// resolved to 1/65536 (0.2 -> 0.199997).
__device__ __forceinline__ uint32_t dropout_keep8(uint64_t seed, uint64_t offset, uint64_t elem8, uint32_t threshold) {
  if (threshold == 0xFFFFFFFFu) return 0u;  // p >= 1: drop everything
  const uint4 r = Philox(seed, elem8 >> 3, offset).next4();
  const uint32_t t = threshold >> 16;
  const uint32_t w[4] = {r.x, r.y, r.z, r.w};
  uint32_t keep = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    keep |= (uint32_t)((w[i] & 0xFFFFu) >= t) << (2 * i);
    keep |= (uint32_t)((w[i] >> 16) >= t) << (2 * i + 1);
  }
  return keep;
}

// The dropout layout of the GEMM epilogues and the bias + activation kernels
// (fwd, and every backward that regenerates the mask): element (row, col) of
// an [*, ld] activation (ld even) draws the 16-bit half (col & 1) of word
// (row & 3) of Philox block (row / 4) * (ld / 2) + col / 2 -- one block per
// 4 rows x 2 columns, half the blocks of one 32-bit uniform per element (the
// Philox rounds are most of a dropout epilogue's cost: +70 us on an 18432 x
// 6400 output, tools/epilogue_cost_probe.py) -- and is kept iff that uniform
// is >= floor(p * 2^16).
__device__ __forceinline__ uint64_t drop_sub(int64_t row, int64_t col, int64_t ld) {
  return (uint64_t)(row >> 2) * (uint64_t)(ld >> 1) + (uint64_t)(col >> 1);
}
__device__ __forceinline__ bool drop_keep(uint32_t word, int half, uint32_t thr16) {
  return ((word >> (16 * half)) & 0xFFFFu) >= thr16;
}

// Exact-erf GELU with erf from Abramowitz & Stegun 7.1.26 (|error| < 1.5e-7,
// far below the bf16 output rounding): one rcp + one exp and a handful of
// registers, where ocml's erff keeps so many values live that the GEMM's
// 16-value epilogue row blocks spilled (1.2 KB scratch per lane), and costs the
// memory-bound bias + activation kernels their bandwidth.  Shared by the GEMM
// epilogues and elementwise.hip, so fused and separate GELU agree bit for bit.
__device__ __forceinline__ float erf_as(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(1.f + 0.3275911f * ax);
  const float poly = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
  const float y = 1.f - poly * __expf(-ax * ax);
  return copysignf(y, x);
}
__device__ __forceinline__ float gelu_f(float x) { return 0.5f * x * (1.f + erf_as(x * 0.70710678118654752f)); }
// GELU'(x) = Phi(x) + x phi(x).  erf_as(x / sqrt 2)'s exp(-x^2 / 2) is the
// density's exponential: computed once (one transcendental fewer per element).
__device__ __forceinline__ float gelu_grad_f(float x) {
  const float e = __expf(-0.5f * x * x);
  const float ax = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(1.f + 0.3275911f * ax);
  const float poly = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
  const float erf = copysignf(1.f - poly * e, x);
  return 0.5f * (1.f + erf) + x * 0.3989422804014327f * e;
}
__host__ __device__ inline uint32_t dropout_threshold(float p) {
  double t = (double)p * 4294967296.0;
  if (t >= 4294967295.0) return 0xFFFFFFFFu;
  return (uint32_t)t;
}

}  // namespace mipipe
