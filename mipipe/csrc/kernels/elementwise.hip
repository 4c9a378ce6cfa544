// Fused bias + activation + dropout, and column sums.
//
//   fwd:  y  = dropout(act(x + bias))
//   bwd:  dx = act'(x + bias) * mask * dy / (1-p)       (dbias = colsum(dx))
//
// For ReLU / identity the backward reads the *output* y (for kept elements
// y > 0 <=> pre-activation > 0), which the next GEMM saves anyway, so the op
// stores nothing extra.  GELU (erf form, torch's default) reads the
// pre-activation.  Memory-bound: 16-byte vectors, grid-stride, mask from
// Philox, never stored.
#include "common.h"
#include "kernels.h"

namespace mipipe {

namespace {

__device__ __forceinline__ float gelu_f(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }

__device__ __forceinline__ float gelu_grad(float x) {
  const float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752f));
  const float pdf = 0.3989422804014327f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

template <typename T, int ACT>
__global__ void __launch_bounds__(256) bias_act_fwd_kernel(const T* __restrict__ x, const T* __restrict__ bias,
                                                           T* __restrict__ y, int64_t nvec, int cols, float p,
                                                           uint32_t threshold, uint64_t seed, uint64_t offset) {
  const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = v * 8;
    float a[8];
    Io<T>::load8(x + e, a);
    if (bias != nullptr) {
      float b[8];
      Io<T>::load8(bias + (int)(e % cols), b);
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] += b[i];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (ACT == kActRelu) a[i] = fmaxf(a[i], 0.f);
      if (ACT == kActGelu) a[i] = gelu_f(a[i]);
    }
    if (p > 0.f) {
      const uint32_t keep = dropout_keep8(seed, offset, (uint64_t)e, threshold);
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = ((keep >> i) & 1) ? a[i] * scale : 0.f;
    }
    Io<T>::store8(y + e, a);
  }
}

template <typename T, int ACT>
__global__ void __launch_bounds__(256) bias_act_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ saved,
                                                           const T* __restrict__ bias, T* __restrict__ dx,
                                                           int64_t nvec, int cols, float p, uint32_t threshold,
                                                           uint64_t seed, uint64_t offset) {
  const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = v * 8;
    float g[8];
    Io<T>::load8(dy + e, g);
    if (ACT == kActRelu) {
      float s[8];
      Io<T>::load8(saved + e, s);  // the op's output
#pragma unroll
      for (int i = 0; i < 8; ++i) g[i] = s[i] > 0.f ? g[i] : 0.f;
    } else if (ACT == kActGelu) {
      float s[8];
      Io<T>::load8(saved + e, s);  // pre-bias input
      if (bias != nullptr) {
        float b[8];
        Io<T>::load8(bias + (int)(e % cols), b);
#pragma unroll
        for (int i = 0; i < 8; ++i) s[i] += b[i];
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) g[i] *= gelu_grad(s[i]);
    }
    if (p > 0.f) {
      const uint32_t keep = dropout_keep8(seed, offset, (uint64_t)e, threshold);
#pragma unroll
      for (int i = 0; i < 8; ++i) g[i] = ((keep >> i) & 1) ? g[i] * scale : 0.f;
    }
    Io<T>::store8(dx + e, g);
  }
}

// Stage 1 of a column sum: block b sums rows [b*rows_per, (b+1)*rows_per) of
// each column owned by its threads (8 columns per thread, 16-byte loads).
template <typename T>
__global__ void __launch_bounds__(256) colsum_part_kernel(const T* __restrict__ x, int rows, int cols, int rows_per,
                                                          float* __restrict__ part) {
  const int nvec = cols >> 3;
  const int r0 = blockIdx.y * rows_per;
  const int r1 = min(rows, r0 + rows_per);
  for (int vi = blockIdx.x * blockDim.x + threadIdx.x; vi < nvec; vi += gridDim.x * blockDim.x) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int r = r0; r < r1; ++r) {
      float a[8];
      Io<T>::load8(x + (size_t)r * cols + vi * 8, a);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += a[i];
    }
    Io<float>::store8(part + (size_t)blockIdx.y * cols + vi * 8, acc);
  }
}

// Same for widths that are not a multiple of 8 (e.g. a 28,782-word decoder bias):
// one column per thread, consecutive threads on consecutive columns.
template <typename T>
__global__ void __launch_bounds__(256) colsum_part_scalar_kernel(const T* __restrict__ x, int rows, int cols,
                                                                 int rows_per, float* __restrict__ part) {
  const int r0 = blockIdx.y * rows_per;
  const int r1 = min(rows, r0 + rows_per);
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < cols; c += gridDim.x * blockDim.x) {
    float acc = 0.f;
    for (int r = r0; r < r1; ++r) acc += Io<T>::load(x + (size_t)r * cols + c);
    part[(size_t)blockIdx.y * cols + c] = acc;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) colsum_final_kernel(const float* __restrict__ part, int nparts, int cols,
                                                           T* __restrict__ out, int accumulate) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= cols) return;
  float a = accumulate ? Io<T>::load(out + c) : 0.f;
  for (int r = 0; r < nparts; ++r) a += part[(size_t)r * cols + c];
  Io<T>::store(out + c, a);
}

int64_t grid_for(int64_t nvec) {
  int64_t g = (nvec + 255) / 256;
  return g < 2048 ? (g < 1 ? 1 : g) : 2048;
}

}  // namespace

template <typename T>
void bias_act_dropout_fwd(const T* x, const T* bias, T* y, int64_t rows, int cols, int act, float p, uint64_t seed,
                          uint64_t offset, hipStream_t s) {
  const int64_t nvec = rows * cols / 8;
  if (nvec == 0) return;
  const dim3 grid((unsigned)grid_for(nvec)), block(256);
  const uint32_t thr = dropout_threshold(p);
  switch (act) {
    case kActNone: hipLaunchKernelGGL((bias_act_fwd_kernel<T, kActNone>), grid, block, 0, s, x, bias, y, nvec, cols, p, thr, seed, offset); break;
    case kActRelu: hipLaunchKernelGGL((bias_act_fwd_kernel<T, kActRelu>), grid, block, 0, s, x, bias, y, nvec, cols, p, thr, seed, offset); break;
    case kActGelu: hipLaunchKernelGGL((bias_act_fwd_kernel<T, kActGelu>), grid, block, 0, s, x, bias, y, nvec, cols, p, thr, seed, offset); break;
  }
}

template <typename T>
void bias_act_dropout_bwd(const T* dy, const T* saved, const T* bias, T* dx, int64_t rows, int cols, int act, float p,
                          uint64_t seed, uint64_t offset, hipStream_t s) {
  const int64_t nvec = rows * cols / 8;
  if (nvec == 0) return;
  const dim3 grid((unsigned)grid_for(nvec)), block(256);
  const uint32_t thr = dropout_threshold(p);
  switch (act) {
    case kActNone: hipLaunchKernelGGL((bias_act_bwd_kernel<T, kActNone>), grid, block, 0, s, dy, saved, bias, dx, nvec, cols, p, thr, seed, offset); break;
    case kActRelu: hipLaunchKernelGGL((bias_act_bwd_kernel<T, kActRelu>), grid, block, 0, s, dy, saved, bias, dx, nvec, cols, p, thr, seed, offset); break;
    case kActGelu: hipLaunchKernelGGL((bias_act_bwd_kernel<T, kActGelu>), grid, block, 0, s, dy, saved, bias, dx, nvec, cols, p, thr, seed, offset); break;
  }
}

int colsum_parts(int64_t rows) {
  // ~64 rows per part keeps stage 1 latency-friendly and stage 2 short.
  int64_t parts = (rows + 63) / 64;
  return (int)(parts < 1 ? 1 : (parts > 256 ? 256 : parts));
}

template <typename T>
void column_sum(const T* x, int64_t rows, int cols, float* part, int nparts, T* out, bool accumulate, hipStream_t s) {
  if (rows == 0 || cols == 0) return;
  const int rows_per = (int)((rows + nparts - 1) / nparts);
  if (cols % 8 == 0) {
    const int nvec = cols / 8;
    dim3 g1((unsigned)((nvec + 255) / 256), (unsigned)nparts);
    hipLaunchKernelGGL((colsum_part_kernel<T>), g1, dim3(256), 0, s, x, (int)rows, cols, rows_per, part);
  } else {
    dim3 g1((unsigned)((cols + 255) / 256), (unsigned)nparts);
    hipLaunchKernelGGL((colsum_part_scalar_kernel<T>), g1, dim3(256), 0, s, x, (int)rows, cols, rows_per, part);
  }
  hipLaunchKernelGGL((colsum_final_kernel<T>), dim3((cols + 255) / 256), dim3(256), 0, s, part, nparts, cols, out,
                     accumulate ? 1 : 0);
}

template void bias_act_dropout_fwd<float>(const float*, const float*, float*, int64_t, int, int, float, uint64_t, uint64_t, hipStream_t);
template void bias_act_dropout_fwd<bf16_t>(const bf16_t*, const bf16_t*, bf16_t*, int64_t, int, int, float, uint64_t, uint64_t, hipStream_t);
template void bias_act_dropout_bwd<float>(const float*, const float*, const float*, float*, int64_t, int, int, float, uint64_t, uint64_t, hipStream_t);
template void bias_act_dropout_bwd<bf16_t>(const bf16_t*, const bf16_t*, const bf16_t*, bf16_t*, int64_t, int, int, float, uint64_t, uint64_t, hipStream_t);
template void column_sum<float>(const float*, int64_t, int, float*, int, float*, bool, hipStream_t);
template void column_sum<bf16_t>(const bf16_t*, int64_t, int, float*, int, bf16_t*, bool, hipStream_t);

}  // namespace mipipe
