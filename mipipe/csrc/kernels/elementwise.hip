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

__device__ __forceinline__ float gelu_grad(float x) { return gelu_grad_f(x); }  // common.h (erf_as)

// Dropout mask layout shared with the GEMM epilogues (common.h drop_sub):
// element (row, col) draws half (col & 1) of word (row & 3) of Philox block
// (row / 4) * (cols / 2) + col / 2.  Each thread owns a 4-row x 8-column tile:
// 4 Philox calls produce exactly its 32 16-bit uniforms.
template <typename T, int ACT, bool BWD>
__global__ void __launch_bounds__(256) bias_act_kernel(const T* __restrict__ in, const T* __restrict__ saved,
                                                       const T* __restrict__ bias, T* __restrict__ out,
                                                       int64_t rows, int cols, float p, uint32_t threshold,
                                                       uint64_t seed, uint64_t offset) {
  const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const int cvec = cols >> 3;
  const int64_t quads = (rows + 3) >> 2;
  const int64_t ntiles = quads * cvec;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < ntiles; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t q = t / cvec;
    const int c0 = (int)(t - q * cvec) * 8;
    float b[8];
    if (bias != nullptr) {
      Io<T>::load8(bias + c0, b);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) b[i] = 0.f;
    }
    uint32_t w[4][4];  // [column pair][row]
    const uint32_t thr16 = threshold >> 16;
    if (p > 0.f) {
      const uint64_t sub = drop_sub(q * 4, c0, cols);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint4 r = Philox(seed, sub + i, offset).next4();
        w[i][0] = r.x; w[i][1] = r.y; w[i][2] = r.z; w[i][3] = r.w;
      }
    }
    // Activation backward: every load of the tile first (4 rows x 2 tensors, 16
    // bytes each), then the math and the stores -- GELU' 153 -> 141 us at
    // 18432 x 6400.  The one-tensor kernels (forward, dropout-only backward) load
    // row by row: all-loads-first cost the dropout backward 92 -> 100 us
    // (tools/bias_act_ab.py).
    constexpr bool kAhead = BWD && ACT != kActNone;
    const int nr = (int)(rows - q * 4 < 4 ? rows - q * 4 : 4);
    float a[4][8], sv[4][8];
    if (kAhead) {
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        if (rr < nr) {
          const int64_t e = (q * 4 + rr) * cols + c0;
          Io<T>::load8(in + e, a[rr]);
          Io<T>::load8(saved + e, sv[rr]);
        }
      }
    }
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      if (rr >= nr) break;
      if (!kAhead) Io<T>::load8(in + (q * 4 + rr) * cols + c0, a[rr]);
      if (!BWD) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          float v = a[rr][i] + b[i];
          if (ACT == kActRelu) v = fmaxf(v, 0.f);
          if (ACT == kActGelu) v = gelu_f(v);
          if (p > 0.f) v = drop_keep(w[i >> 1][rr], i & 1, thr16) ? v * scale : 0.f;
          a[rr][i] = v;
        }
      } else {
        if (ACT != kActNone) {
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            if (ACT == kActRelu) a[rr][i] = sv[rr][i] > 0.f ? a[rr][i] : 0.f;   // saved = the op's output
            if (ACT == kActGelu) a[rr][i] *= gelu_grad(sv[rr][i] + b[i]);  // saved = pre-bias input
            if (ACT == kActSavedGrad) a[rr][i] *= sv[rr][i];              // saved = act'(pre) itself
          }
        }
        if (p > 0.f) {
#pragma unroll
          for (int i = 0; i < 8; ++i) a[rr][i] = drop_keep(w[i >> 1][rr], i & 1, thr16) ? a[rr][i] * scale : 0.f;
        }
      }
      Io<T>::store8(out + (q * 4 + rr) * cols + c0, a[rr]);
    }
  }
}

// Stage 1 of a column sum.  A block owns a 64-column strip of rows
// [blockIdx.y * rows_per, ...): 8 column lanes x 8 columns (16-byte loads, a
// wave reads 8 rows x 128 contiguous bytes) by 32 row lanes, each row lane
// summing every 32nd row with 4 loads in flight; the 32 row sums of each
// column are folded through LDS and the block writes ONE partial row.  Parts
// cover >= 256 rows each, so the partial image stays small (<= 64 rows) and
// the second stage (reduce_parts) is a launch, not a second pass.
// blockIdx.z picks one of up to kColsumSegs equally shaped inputs (the
// micro-batch gradients of a deferred bias), each owning gridDim.y part rows:
// all segments of a step run in ONE launch.
template <typename T>
__global__ void __launch_bounds__(256) colsum_part_kernel(ColsumSegs segs, int rows, int cols, int rows_per,
                                                          float* __restrict__ part) {
  __shared__ float sm[32][65];
  const T* __restrict__ x = reinterpret_cast<const T*>(segs.p[blockIdx.z]);
  part += (size_t)blockIdx.z * gridDim.y * cols;
  const int cx = threadIdx.x & 7, ry = threadIdx.x >> 3;
  const int c0 = blockIdx.x * 64 + cx * 8;
  const int r0 = blockIdx.y * rows_per;
  const int r1 = min(rows, r0 + rows_per);
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c0 < cols) {
    int r = r0 + ry;
    // 8 independent 16-byte loads in flight per lane (a pure read stream:
    // latency hiding comes from loads in flight, not from occupancy)
    for (; r + 224 < r1; r += 256) {
      float a[8][8];
#pragma unroll
      for (int u = 0; u < 8; ++u) Io<T>::load8(x + (size_t)(r + 32 * u) * cols + c0, a[u]);
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] += a[u][i];
    }
    for (; r < r1; r += 32) {
      float a[8];
      Io<T>::load8(x + (size_t)r * cols + c0, a);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += a[i];
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) sm[ry][cx * 8 + i] = acc[i];
  __syncthreads();
  if (threadIdx.x < 64) {
    const int c = blockIdx.x * 64 + threadIdx.x;
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 32; ++k) s += sm[k][threadIdx.x];
    if (c < cols) part[(size_t)blockIdx.y * cols + c] = s;
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

int64_t grid_for(int64_t nvec) {
  int64_t g = (nvec + 255) / 256;
  return g < 2048 ? (g < 1 ? 1 : g) : 2048;
}

}  // namespace

template <typename T, bool BWD>
void launch_bias_act(const T* in, const T* saved, const T* bias, T* out, int64_t rows, int cols, int act, float p,
                     uint64_t seed, uint64_t offset, hipStream_t s) {
  const int64_t ntiles = ((rows + 3) / 4) * (cols / 8);
  if (ntiles == 0) return;
  const dim3 grid((unsigned)grid_for(ntiles)), block(256);
  const uint32_t thr = dropout_threshold(p);
  switch (act) {
    case kActNone: hipLaunchKernelGGL((bias_act_kernel<T, kActNone, BWD>), grid, block, 0, s, in, saved, bias, out, rows, cols, p, thr, seed, offset); break;
    case kActRelu: hipLaunchKernelGGL((bias_act_kernel<T, kActRelu, BWD>), grid, block, 0, s, in, saved, bias, out, rows, cols, p, thr, seed, offset); break;
    case kActGelu: hipLaunchKernelGGL((bias_act_kernel<T, kActGelu, BWD>), grid, block, 0, s, in, saved, bias, out, rows, cols, p, thr, seed, offset); break;
    case kActSavedGrad:
      if constexpr (BWD) hipLaunchKernelGGL((bias_act_kernel<T, kActSavedGrad, BWD>), grid, block, 0, s, in, saved, bias, out, rows, cols, p, thr, seed, offset);
      break;
  }
}

template <typename T>
void bias_act_dropout_fwd(const T* x, const T* bias, T* y, int64_t rows, int cols, int act, float p, uint64_t seed,
                          uint64_t offset, hipStream_t s) {
  launch_bias_act<T, false>(x, nullptr, bias, y, rows, cols, act, p, seed, offset, s);
}

template <typename T>
void bias_act_dropout_bwd(const T* dy, const T* saved, const T* bias, T* dx, int64_t rows, int cols, int act, float p,
                          uint64_t seed, uint64_t offset, hipStream_t s) {
  launch_bias_act<T, true>(dy, saved, bias, dx, rows, cols, act, p, seed, offset, s);
}

int colsum_parts(int64_t rows, int64_t cols) {
  if (cols % 8 != 0) {
    // scalar path: ~16 rows per part keeps enough one-column threads in flight
    int64_t parts = (rows + 15) / 16;
    return (int)(parts < 1 ? 1 : (parts > 512 ? 512 : parts));
  }
  // 2-D tiled path: >= 256 rows per part and >= ~1024 blocks when the shape
  // allows it (4096 x 4096 -> 64 strips x 16 parts).
  const int64_t strips = (cols + 63) / 64;
  int64_t parts = (rows + 255) / 256;
  const int64_t want = (1024 + strips - 1) / strips;
  if (parts > want) parts = want;
  return (int)(parts < 1 ? 1 : (parts > 64 ? 64 : parts));
}

template <typename T>
void column_sum_partial(const T* x, int64_t rows, int cols, float* part, int nparts, hipStream_t s) {
  if (rows == 0 || cols == 0) return;
  const int rows_per = (int)((rows + nparts - 1) / nparts);
  if (cols % 8 == 0) {
    dim3 g1((unsigned)((cols + 63) / 64), (unsigned)nparts);
    ColsumSegs segs;
    segs.p[0] = x;
    hipLaunchKernelGGL((colsum_part_kernel<T>), g1, dim3(256), 0, s, segs, (int)rows, cols, rows_per, part);
  } else {
    dim3 g1((unsigned)((cols + 255) / 256), (unsigned)nparts);
    hipLaunchKernelGGL((colsum_part_scalar_kernel<T>), g1, dim3(256), 0, s, x, (int)rows, cols, rows_per, part);
  }
}

template <typename T>
bool column_sum_partial_multi(const ColsumSegs& segs, int nseg, int64_t rows, int cols, float* part, int nparts,
                              hipStream_t s) {
  if (cols % 8 != 0 || nseg < 1 || nseg > kColsumSegs) return false;
  if (rows == 0 || cols == 0) return true;
  const int rows_per = (int)((rows + nparts - 1) / nparts);
  dim3 g1((unsigned)((cols + 63) / 64), (unsigned)nparts, (unsigned)nseg);
  hipLaunchKernelGGL((colsum_part_kernel<T>), g1, dim3(256), 0, s, segs, (int)rows, cols, rows_per, part);
  return true;
}

template <typename T>
void column_sum(const T* x, int64_t rows, int cols, float* part, int nparts, void* out, bool out_f32, bool accumulate,
                hipStream_t s) {
  if (rows == 0 || cols == 0) return;
  const int rows_per = (int)((rows + nparts - 1) / nparts);
  if (cols % 8 == 0) {
    dim3 g1((unsigned)((cols + 63) / 64), (unsigned)nparts);
    ColsumSegs segs;
    segs.p[0] = x;
    hipLaunchKernelGGL((colsum_part_kernel<T>), g1, dim3(256), 0, s, segs, (int)rows, cols, rows_per, part);
  } else {
    dim3 g1((unsigned)((cols + 255) / 256), (unsigned)nparts);
    hipLaunchKernelGGL((colsum_part_scalar_kernel<T>), g1, dim3(256), 0, s, x, (int)rows, cols, rows_per, part);
  }
  reduce_parts(part, nullptr, nparts, cols, out, nullptr, out_f32, accumulate, s);
}

template void bias_act_dropout_fwd<float>(const float*, const float*, float*, int64_t, int, int, float, uint64_t, uint64_t, hipStream_t);
template void bias_act_dropout_fwd<bf16_t>(const bf16_t*, const bf16_t*, bf16_t*, int64_t, int, int, float, uint64_t, uint64_t, hipStream_t);
template void bias_act_dropout_bwd<float>(const float*, const float*, const float*, float*, int64_t, int, int, float, uint64_t, uint64_t, hipStream_t);
template void bias_act_dropout_bwd<bf16_t>(const bf16_t*, const bf16_t*, const bf16_t*, bf16_t*, int64_t, int, int, float, uint64_t, uint64_t, hipStream_t);
template void column_sum_partial<float>(const float*, int64_t, int, float*, int, hipStream_t);
template void column_sum_partial<bf16_t>(const bf16_t*, int64_t, int, float*, int, hipStream_t);
template bool column_sum_partial_multi<float>(const ColsumSegs&, int, int64_t, int, float*, int, hipStream_t);
template bool column_sum_partial_multi<bf16_t>(const ColsumSegs&, int, int64_t, int, float*, int, hipStream_t);
template void column_sum<float>(const float*, int64_t, int, float*, int, void*, bool, bool, hipStream_t);
template void column_sum<bf16_t>(const bf16_t*, int64_t, int, float*, int, void*, bool, bool, hipStream_t);

}  // namespace mipipe
