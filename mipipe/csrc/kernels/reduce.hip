// Second stage of the column reductions (LayerNorm dgamma/dbeta, bias grads).
//
// Stage 1 kernels write fp32 partial rows part[nparts][cols]; this kernel sums
// them per column and either stores the result in the parameter dtype or
// ACCUMULATES it into an fp32 main_grad buffer -- so parameter gradients of
// every micro-batch land in fp32 without a separate add kernel.
//
// Each workgroup owns 16 columns (64-byte row segments) so a 4096-column
// reduction runs on 256 workgroups, each row lane with 4 loads in flight.
#include "common.h"
#include "kernels.h"

namespace mipipe {

namespace {

template <typename TOut>
__global__ void __launch_bounds__(256) reduce_parts_kernel(const float* __restrict__ part_a,
                                                           const float* __restrict__ part_b, int nparts, int cols,
                                                           TOut* __restrict__ out_a, TOut* __restrict__ out_b,
                                                           int accumulate) {
  // 16 columns per workgroup: 4 column lanes x float4 by 64 row lanes, each
  // row lane keeping 4 partial rows in flight; the 64 row sums are folded in LDS.
  __shared__ float sm[2][64][17];
  const int cl = threadIdx.x & 3;
  const int g = threadIdx.x >> 2;
  const int c0 = blockIdx.x * 16 + cl * 4;
  float a[4] = {0.f, 0.f, 0.f, 0.f}, b[4] = {0.f, 0.f, 0.f, 0.f};
  const bool vec = (cols & 3) == 0 && c0 + 3 < cols;
  auto add_row = [&](const float* base, float* acc) {
    if (vec) {
      const float4 v = *reinterpret_cast<const float4*>(base + c0);
      acc[0] += v.x; acc[1] += v.y; acc[2] += v.z; acc[3] += v.w;
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (c0 + i < cols) acc[i] += base[c0 + i];
    }
  };
  int r = g;
  for (; r + 192 < nparts; r += 256) {
    float4 va[4], vb[4];
    if (vec) {
#pragma unroll
      for (int u = 0; u < 4; ++u) va[u] = *reinterpret_cast<const float4*>(part_a + (size_t)(r + 64 * u) * cols + c0);
      if (part_b != nullptr) {
#pragma unroll
        for (int u = 0; u < 4; ++u) vb[u] = *reinterpret_cast<const float4*>(part_b + (size_t)(r + 64 * u) * cols + c0);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a[0] += va[u].x; a[1] += va[u].y; a[2] += va[u].z; a[3] += va[u].w;
        if (part_b != nullptr) { b[0] += vb[u].x; b[1] += vb[u].y; b[2] += vb[u].z; b[3] += vb[u].w; }
      }
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        add_row(part_a + (size_t)(r + 64 * u) * cols, a);
        if (part_b != nullptr) add_row(part_b + (size_t)(r + 64 * u) * cols, b);
      }
    }
  }
  for (; r < nparts; r += 64) {
    add_row(part_a + (size_t)r * cols, a);
    if (part_b != nullptr) add_row(part_b + (size_t)r * cols, b);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    sm[0][g][cl * 4 + i] = a[i];
    sm[1][g][cl * 4 + i] = b[i];
  }
  __syncthreads();
  if (threadIdx.x < 32) {
    const int which = threadIdx.x >> 4;  // 0: a, 1: b
    const int cc = threadIdx.x & 15;
    const int c = blockIdx.x * 16 + cc;
    TOut* out = which == 0 ? out_a : out_b;
    if (out != nullptr && c < cols) {
      float s = 0.f;
#pragma unroll 16
      for (int k = 0; k < 64; ++k) s += sm[which][k][cc];
      if (accumulate) s += Io<TOut>::load(out + c);
      Io<TOut>::store(out + c, s);
    }
  }
}

}  // namespace

void reduce_parts(const float* part_a, const float* part_b, int nparts, int cols, void* out_a, void* out_b,
                  bool out_f32, bool accumulate, hipStream_t s) {
  if (cols == 0) return;
  const dim3 grid((cols + 15) / 16), block(256);
  if (out_f32) {
    hipLaunchKernelGGL((reduce_parts_kernel<float>), grid, block, 0, s, part_a, part_b, nparts, cols,
                       static_cast<float*>(out_a), static_cast<float*>(out_b), accumulate ? 1 : 0);
  } else {
    hipLaunchKernelGGL((reduce_parts_kernel<bf16_t>), grid, block, 0, s, part_a, part_b, nparts, cols,
                       static_cast<bf16_t*>(out_a), static_cast<bf16_t*>(out_b), accumulate ? 1 : 0);
  }
}

}  // namespace mipipe
