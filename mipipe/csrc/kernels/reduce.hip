// Second stage of the column reductions (LayerNorm dgamma/dbeta, bias grads).
//
// Stage 1 kernels write fp32 partial rows part[nparts][cols]; this kernel sums
// them per column and either stores the result in the parameter dtype or
// ACCUMULATES it into an fp32 main_grad buffer -- so parameter gradients of
// every micro-batch land in fp32 without a separate add kernel.
//
// Each workgroup owns 64 columns: 16 row-groups x 16 lanes x float4, so the
// partial reads are 256-byte coalesced segments and a 4096-column reduction
// runs on 64 workgroups instead of 16 long serial loops.
#include "common.h"
#include "kernels.h"

namespace mipipe {

namespace {

template <typename TOut>
__global__ void __launch_bounds__(256) reduce_parts_kernel(const float* __restrict__ part_a,
                                                           const float* __restrict__ part_b, int nparts, int cols,
                                                           TOut* __restrict__ out_a, TOut* __restrict__ out_b,
                                                           int accumulate) {
  __shared__ float sm[2][16][65];
  const int lane16 = threadIdx.x & 15;
  const int g = threadIdx.x >> 4;
  const int c0 = blockIdx.x * 64 + lane16 * 4;
  float a[4] = {0.f, 0.f, 0.f, 0.f}, b[4] = {0.f, 0.f, 0.f, 0.f};
  const bool vec = (cols & 3) == 0 && c0 + 3 < cols;
  for (int r = g; r < nparts; r += 16) {
    const float* pa = part_a + (size_t)r * cols;
    const float* pb = part_b != nullptr ? part_b + (size_t)r * cols : nullptr;
    if (vec) {
      const float4 va = *reinterpret_cast<const float4*>(pa + c0);
      a[0] += va.x; a[1] += va.y; a[2] += va.z; a[3] += va.w;
      if (pb != nullptr) {
        const float4 vb = *reinterpret_cast<const float4*>(pb + c0);
        b[0] += vb.x; b[1] += vb.y; b[2] += vb.z; b[3] += vb.w;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (c0 + i < cols) {
          a[i] += pa[c0 + i];
          if (pb != nullptr) b[i] += pb[c0 + i];
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    sm[0][g][lane16 * 4 + i] = a[i];
    sm[1][g][lane16 * 4 + i] = b[i];
  }
  __syncthreads();
  if (threadIdx.x < 128) {
    const int which = threadIdx.x >> 6;  // 0: a, 1: b
    const int cl = threadIdx.x & 63;
    const int c = blockIdx.x * 64 + cl;
    TOut* out = which == 0 ? out_a : out_b;
    if (out != nullptr && c < cols) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k) s += sm[which][k][cl];
      if (accumulate) s += Io<TOut>::load(out + c);
      Io<TOut>::store(out + c, s);
    }
  }
}

}  // namespace

void reduce_parts(const float* part_a, const float* part_b, int nparts, int cols, void* out_a, void* out_b,
                  bool out_f32, bool accumulate, hipStream_t s) {
  if (cols == 0) return;
  const dim3 grid((cols + 63) / 64), block(256);
  if (out_f32) {
    hipLaunchKernelGGL((reduce_parts_kernel<float>), grid, block, 0, s, part_a, part_b, nparts, cols,
                       static_cast<float*>(out_a), static_cast<float*>(out_b), accumulate ? 1 : 0);
  } else {
    hipLaunchKernelGGL((reduce_parts_kernel<bf16_t>), grid, block, 0, s, part_a, part_b, nparts, cols,
                       static_cast<bf16_t*>(out_a), static_cast<bf16_t*>(out_b), accumulate ? 1 : 0);
  }
}

}  // namespace mipipe
