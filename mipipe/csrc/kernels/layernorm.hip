// Fused residual + dropout + LayerNorm, forward and backward.
//
//   z = residual + dropout(x)          (residual optional, dropout optional)
//   y = (z - mean(z)) * rstd(z) * gamma + beta
//
// The post-norm TransformerEncoderLayer's two "Add & Norm" steps, and the
// pre-norm GPT-2 LayerNorms (no residual / no dropout), are each ONE pass over
// HBM: one row per 256-thread workgroup, the row held in registers (16-byte
// vector loads, Guideline 13), statistics in fp32, wave64 shuffles + one LDS
// exchange for the row reduction.  The dropout mask is never stored: backward
// regenerates it from the same Philox (seed, offset).
//
// Backward computes dz (= grad of the residual input), dx = dz * mask / (1-p)
// and per-workgroup partial dgamma/dbeta that a second small kernel reduces,
// so there are no float atomics (Guideline 12) and results are reproducible.
#include "common.h"
#include "kernels.h"

namespace mipipe {

namespace {

constexpr int kThreads = 256;

template <typename T, int MAXV>
__global__ void __launch_bounds__(kThreads) ln_fwd_kernel(
    const T* __restrict__ x, const T* __restrict__ res, const T* __restrict__ gamma, const T* __restrict__ beta,
    T* __restrict__ y, T* __restrict__ z, float* __restrict__ mean_out, float* __restrict__ rstd_out, int cols,
    float eps, float p, uint32_t threshold, uint64_t seed, uint64_t offset) {
  __shared__ float scratch[2 * (kThreads / 64)];
  const int row = blockIdx.x;
  const size_t base = (size_t)row * cols;
  const int nvec = cols >> 3;
  const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;

  float v[MAXV][8];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = threadIdx.x + k * kThreads;
    if (vi < nvec) {
      const size_t e = base + (size_t)vi * 8;
      Io<T>::load8(x + e, v[k]);
      if (p > 0.f) {
        const uint32_t keep = dropout_keep8(seed, offset, e, threshold);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[k][i] = ((keep >> i) & 1) ? v[k][i] * scale : 0.f;
      }
      if (res != nullptr) {
        float r[8];
        Io<T>::load8(res + e, r);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[k][i] += r[i];
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) s1 += v[k][i];
    }
  }
  // Two-pass statistics from registers: mean first, then centred variance.
  float dummy = 0.f;
  block_sum2(s1, dummy, scratch);
  const float mean = s1 / (float)cols;
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = threadIdx.x + k * kThreads;
    if (vi < nvec) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float d = v[k][i] - mean;
        s2 += d * d;
      }
    }
  }
  block_sum2(s2, dummy, scratch);
  const float rstd = rsqrtf(s2 / (float)cols + eps);
  if (threadIdx.x == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = threadIdx.x + k * kThreads;
    if (vi < nvec) {
      const size_t e = base + (size_t)vi * 8;
      if (z != nullptr) Io<T>::store8(z + e, v[k]);
      float g[8], b[8], o[8];
      Io<T>::load8(gamma + vi * 8, g);
      Io<T>::load8(beta + vi * 8, b);
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = (v[k][i] - mean) * rstd * g[i] + b[i];
      Io<T>::store8(y + e, o);
    }
  }
}

template <typename T, int MAXV>
__global__ void __launch_bounds__(kThreads) ln_bwd_kernel(
    const T* __restrict__ dy, const T* __restrict__ z, const float* __restrict__ mean_in,
    const float* __restrict__ rstd_in, const T* __restrict__ gamma, T* __restrict__ dz, T* __restrict__ dx,
    float* __restrict__ dgamma_part, float* __restrict__ dbeta_part, int rows, int cols, float p,
    uint32_t threshold, uint64_t seed, uint64_t offset) {
  __shared__ float scratch[2 * (kThreads / 64)];
  const int nvec = cols >> 3;
  const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;

  float g[MAXV][8];
  float dg[MAXV][8], db[MAXV][8];
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = threadIdx.x + k * kThreads;
#pragma unroll
    for (int i = 0; i < 8; ++i) dg[k][i] = db[k][i] = 0.f;
    if (vi < nvec) Io<T>::load8(gamma + vi * 8, g[k]);
  }

  // Rows are software-pipelined: the next row's z / dy loads are in flight
  // while this row's reductions and stores run (a block walks rows/grid rows).
  float zn[MAXV][8], dn[MAXV][8];
  auto load_row = [&](int row) {
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int vi = threadIdx.x + k * kThreads;
      if (vi < nvec) {
        const size_t e = (size_t)row * cols + (size_t)vi * 8;
        Io<T>::load8(z + e, zn[k]);
        Io<T>::load8(dy + e, dn[k]);
      }
    }
  };
  constexpr bool kPrefetch = MAXV <= 2;  // wider rows: the extra row would spill
  if (kPrefetch && blockIdx.x < rows) load_row(blockIdx.x);
  for (int row = blockIdx.x; row < rows; row += gridDim.x) {
    const size_t base = (size_t)row * cols;
    const float mean = mean_in[row];
    const float rstd = rstd_in[row];
    if (!kPrefetch) load_row(row);
    float zc[MAXV][8], dc[MAXV][8];
#pragma unroll
    for (int k = 0; k < MAXV; ++k)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        zc[k][i] = zn[k][i];
        dc[k][i] = dn[k][i];
      }
    if (kPrefetch && row + (int)gridDim.x < rows) load_row(row + gridDim.x);
    float xh[MAXV][8], gy[MAXV][8];
    float a = 0.f, b = 0.f;  // sum(g*dy), sum(g*dy*xhat)
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int vi = threadIdx.x + k * kThreads;
      if (vi < nvec) {
        const float* zz = zc[k];
        const float* d = dc[k];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          xh[k][i] = (zz[i] - mean) * rstd;
          gy[k][i] = d[i] * g[k][i];
          dg[k][i] += d[i] * xh[k][i];
          db[k][i] += d[i];
          a += gy[k][i];
          b += gy[k][i] * xh[k][i];
        }
      }
    }
    block_sum2(a, b, scratch);
    const float inv_n = 1.f / (float)cols;
    a *= inv_n;
    b *= inv_n;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int vi = threadIdx.x + k * kThreads;
      if (vi < nvec) {
        const size_t e = base + (size_t)vi * 8;
        float o[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = rstd * (gy[k][i] - a - xh[k][i] * b);
        Io<T>::store8(dz + e, o);
        if (dx != nullptr) {
          const uint32_t keep = dropout_keep8(seed, offset, e, threshold);
#pragma unroll
          for (int i = 0; i < 8; ++i) o[i] = ((keep >> i) & 1) ? o[i] * scale : 0.f;
          Io<T>::store8(dx + e, o);
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = threadIdx.x + k * kThreads;
    if (vi < nvec) {
      const size_t o = (size_t)blockIdx.x * cols + vi * 8;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        dgamma_part[o + i] = dg[k][i];
        dbeta_part[o + i] = db[k][i];
      }
    }
  }
}

template <typename T, int MAXV>
void launch_fwd(const LnArgs<T>& a, hipStream_t s) {
  hipLaunchKernelGGL((ln_fwd_kernel<T, MAXV>), dim3(a.rows), dim3(kThreads), 0, s, a.x, a.res, a.gamma, a.beta,
                     a.y, a.z, a.mean, a.rstd, a.cols, a.eps, a.p, dropout_threshold(a.p), a.seed, a.offset);
}

template <typename T, int MAXV>
void launch_bwd(const LnBwdArgs<T>& a, hipStream_t s) {
  hipLaunchKernelGGL((ln_bwd_kernel<T, MAXV>), dim3(a.nparts), dim3(kThreads), 0, s, a.dy, a.z, a.mean, a.rstd,
                     a.gamma, a.dz, a.dx, a.dgamma_part, a.dbeta_part, a.rows, a.cols, a.p,
                     dropout_threshold(a.p), a.seed, a.offset);
  reduce_parts(a.dgamma_part, a.dbeta_part, a.nparts, a.cols, a.dgamma, a.dbeta, a.out_f32, a.accumulate, s);
}

}  // namespace

int ln_max_vec(int cols) {
  const int per = kThreads * 8;
  if (cols <= per) return 1;
  if (cols <= 2 * per) return 2;
  if (cols <= 4 * per) return 4;
  if (cols <= 8 * per) return 8;
  return -1;
}

int ln_bwd_parts(int rows) { return rows < 512 ? rows : 512; }

template <typename T>
void layernorm_fwd(const LnArgs<T>& a, hipStream_t s) {
  switch (ln_max_vec(a.cols)) {
    case 1: launch_fwd<T, 1>(a, s); break;
    case 2: launch_fwd<T, 2>(a, s); break;
    case 4: launch_fwd<T, 4>(a, s); break;
    case 8: launch_fwd<T, 8>(a, s); break;
    default: break;
  }
}

template <typename T>
void layernorm_bwd(const LnBwdArgs<T>& a, hipStream_t s) {
  switch (ln_max_vec(a.cols)) {
    case 1: launch_bwd<T, 1>(a, s); break;
    case 2: launch_bwd<T, 2>(a, s); break;
    case 4: launch_bwd<T, 4>(a, s); break;
    case 8: launch_bwd<T, 8>(a, s); break;
    default: break;
  }
}

template void layernorm_fwd<float>(const LnArgs<float>&, hipStream_t);
template void layernorm_fwd<bf16_t>(const LnArgs<bf16_t>&, hipStream_t);
template void layernorm_bwd<float>(const LnBwdArgs<float>&, hipStream_t);
template void layernorm_bwd<bf16_t>(const LnBwdArgs<bf16_t>&, hipStream_t);

}  // namespace mipipe
