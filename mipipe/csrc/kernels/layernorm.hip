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

// Sum over the 256-thread block through its own scratch: ONE barrier (each
// reduction of a row has a separate buffer, so none is rewritten while read).
__device__ __forceinline__ float block_sum_once(float a, float* scratch) {
  a = wave_sum(a);
  if ((threadIdx.x & 63) == 0) scratch[threadIdx.x >> 6] = a;
  __syncthreads();
  return scratch[0] + scratch[1] + scratch[2] + scratch[3];
}

template <typename T, int MAXV>
__global__ void __launch_bounds__(kThreads) ln_fwd_kernel(
    const T* __restrict__ x, const T* __restrict__ res, const T* __restrict__ gamma, const T* __restrict__ beta,
    T* __restrict__ y, T* __restrict__ z, float* __restrict__ mean_out, float* __restrict__ rstd_out, int cols,
    float eps, float p, uint32_t threshold, uint64_t seed, uint64_t offset) {
  static_assert(kThreads == 256, "block_sum_once folds 4 waves");
  __shared__ float scratch[2][kThreads / 64];
  const int row = blockIdx.x;
  const size_t base = (size_t)row * cols;
  const int nvec = cols >> 3;
  const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;

  // gamma / beta are loaded with the row (L2-resident, but read after the two
  // reductions they were a dependent round trip at the end of every row:
  // 8192 x 4096 bf16 48.9 -> 47.2 us); rows over 4096 wide and fp32 rows load
  // them at the end (registers: fp32 4096-wide rows measured 114 -> 117 us)
  constexpr bool kEarly = MAXV <= 2 && sizeof(T) == 2;
  float v[MAXV][8], g[MAXV][8], bt[MAXV][8];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = threadIdx.x + k * kThreads;
    if (vi < nvec) {
      const size_t e = base + (size_t)vi * 8;
      Io<T>::load8(x + e, v[k]);
      if (kEarly) {
        Io<T>::load8(gamma + vi * 8, g[k]);
        Io<T>::load8(beta + vi * 8, bt[k]);
      }
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
  const float mean = block_sum_once(s1, scratch[0]) / (float)cols;
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
  const float rstd = rsqrtf(block_sum_once(s2, scratch[1]) / (float)cols + eps);
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
      if (!kEarly) {
        Io<T>::load8(gamma + vi * 8, g[k]);
        Io<T>::load8(beta + vi * 8, bt[k]);
      }
      float o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = (v[k][i] - mean) * rstd * g[k][i] + bt[k][i];
      Io<T>::store8(y + e, o);
    }
  }
}

// Row reduction of a pair over one 256-thread row group of a G-group block
// (every thread of the block calls it: the barrier is block-wide).  Callers
// alternate two scratch buffers by row parity, so one barrier per row is
// enough: a buffer is written again two rows later, behind the next row's
// barrier, which a thread reaches only after reading this row's sums.
template <int G>
__device__ __forceinline__ void group_sum2(float& a, float& b, float (*scratch)[8], int grp, int t) {
  const int lane = t & 63, wid = t >> 6;
  a = wave_sum(a);
  b = wave_sum(b);
  if (lane == 0) {
    scratch[grp][wid] = a;
    scratch[grp][4 + wid] = b;
  }
  __syncthreads();
  a = scratch[grp][0] + scratch[grp][1] + scratch[grp][2] + scratch[grp][3];
  b = scratch[grp][4] + scratch[grp][5] + scratch[grp][6] + scratch[grp][7];
}

// 8 elements kept as loaded (bf16: 4 registers instead of 8), converted on use.
template <typename T> struct Raw8;
template <> struct Raw8<float> {
  float v[8];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = 0.f;
  }
  __device__ __forceinline__ void load(const float* p) { Io<float>::load8(p, v); }
  __device__ __forceinline__ float get(int i) const { return v[i]; }
};
template <> struct Raw8<bf16_t> {
  u16x8 v;
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = 0;
  }
  __device__ __forceinline__ void load(const bf16_t* p) { v = *reinterpret_cast<const u16x8*>(p); }
  __device__ __forceinline__ float get(int i) const { return bf2f(v[i]); }
};

// G row groups of 256 threads per block, each on its own row; the groups'
// dgamma/dbeta partials are folded through LDS so a block writes ONE partial
// row pair (G = 2 halves the partial image the second stage re-reads).
template <typename T, int MAXV, int G>
__global__ void __launch_bounds__(kThreads * G) ln_bwd_kernel(
    const T* __restrict__ dy, const T* __restrict__ z, const float* __restrict__ mean_in,
    const float* __restrict__ rstd_in, const T* __restrict__ gamma, T* __restrict__ dz, T* __restrict__ dx,
    float* __restrict__ dgamma_part, float* __restrict__ dbeta_part, int rows, int cols, float p,
    uint32_t threshold, uint64_t seed, uint64_t offset, const T* __restrict__ addend) {
  __shared__ float scratch[2][G][8];
  __shared__ float fold[G > 1 ? 2 * MAXV * 8 * kThreads : 1];
  const int grp = threadIdx.x / kThreads, t = threadIdx.x % kThreads;
  const int nvec = cols >> 3;
  const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const float inv_n = 1.f / (float)cols;

  float g[MAXV][8];
  float dg[MAXV][8], db[MAXV][8];
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = t + k * kThreads;
#pragma unroll
    for (int i = 0; i < 8; ++i) dg[k][i] = db[k][i] = g[k][i] = 0.f;
    if (vi < nvec) Io<T>::load8(gamma + vi * 8, g[k]);
  }

  const int stride = gridDim.x * G;
  const int iters = (rows + stride - 1) / stride;  // uniform over the block (barriers inside)
  auto row_of = [&](int it) { return it * stride + blockIdx.x * G + grp; };
  const bool has_add = addend != nullptr;
  // A row as loaded -- z, dy and the fan-out addend kept raw (bf16: 4 registers
  // per 8 elements, converted on use), its mean and rstd -- so rows can be
  // loaded ahead without the conversion waiting on the load.
  struct RowBuf {
    Raw8<T> z[MAXV], d[MAXV], a[MAXV];
    float mean, rstd;
  };
  auto load_row = [&](int row, RowBuf& r) {
    const bool valid = row < rows;
    r.mean = valid ? mean_in[row] : 0.f;
    r.rstd = valid ? rstd_in[row] : 0.f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int vi = t + k * kThreads;
      r.z[k].zero();
      r.d[k].zero();
      r.a[k].zero();
      if (vi < nvec && valid) {
        const size_t e = (size_t)row * cols + (size_t)vi * 8;
        r.z[k].load(z + e);
        r.d[k].load(dy + e);
        if (has_add) r.a[k].load(addend + e);
      }
    }
  };
  auto process = [&](int it, const RowBuf& r) {
    const int row = row_of(it);
    float xh[MAXV][8], gy[MAXV][8];
    float a = 0.f, b = 0.f;  // sum(g*dy), sum(g*dy*xhat)
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float dv = r.d[k].get(i);
        xh[k][i] = (r.z[k].get(i) - r.mean) * r.rstd;
        gy[k][i] = dv * g[k][i];
        dg[k][i] += dv * xh[k][i];
        db[k][i] += dv;
        a += gy[k][i];
        b += gy[k][i] * xh[k][i];
      }
    }
    group_sum2<G>(a, b, scratch[it & 1], grp, t);
    a *= inv_n;
    b *= inv_n;
    if (row < rows) {
#pragma unroll
      for (int k = 0; k < MAXV; ++k) {
        const int vi = t + k * kThreads;
        if (vi < nvec) {
          const size_t e = (size_t)row * cols + (size_t)vi * 8;
          float o[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) o[i] = r.rstd * (gy[k][i] - a - xh[k][i] * b) + r.a[k].get(i);
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
  };
  if constexpr (MAXV <= 2) {
    // Two rows in flight per group while one is reduced and stored: the loop is
    // unrolled by two over two named buffers (a copy between buffers would wait
    // for the loads in flight).  The mean / rstd loads travel with their row:
    // read at the top of the row's iteration they were a dependent HBM round
    // trip per row.
    RowBuf b0, b1;
    load_row(row_of(0), b0);
    load_row(row_of(1), b1);
    for (int it = 0; it < iters; it += 2) {
      process(it, b0);
      if (it + 2 < iters) load_row(row_of(it + 2), b0);
      if (it + 1 < iters) {
        process(it + 1, b1);
        if (it + 3 < iters) load_row(row_of(it + 3), b1);
      }
    }
  } else {  // wider rows: one row at a time (a second buffer would spill)
    RowBuf b0;
    for (int it = 0; it < iters; ++it) {
      load_row(row_of(it), b0);
      process(it, b0);
    }
  }
  if constexpr (G > 1) {
    // groups 1..G-1 hand their partials to group 0 through LDS, one at a time
#pragma unroll
    for (int src = 1; src < G; ++src) {
      if (grp == src) {
#pragma unroll
        for (int k = 0; k < MAXV; ++k)
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            fold[((0 * MAXV + k) * 8 + i) * kThreads + t] = dg[k][i];
            fold[((1 * MAXV + k) * 8 + i) * kThreads + t] = db[k][i];
          }
      }
      __syncthreads();
      if (grp == 0) {
#pragma unroll
        for (int k = 0; k < MAXV; ++k)
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            dg[k][i] += fold[((0 * MAXV + k) * 8 + i) * kThreads + t];
            db[k][i] += fold[((1 * MAXV + k) * 8 + i) * kThreads + t];
          }
      }
      __syncthreads();
    }
  }
  if (grp == 0) {
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int vi = t + k * kThreads;
      if (vi < nvec) {
        const size_t o = (size_t)blockIdx.x * cols + vi * 8;
        Io<float>::store8(dgamma_part + o, dg[k]);
        Io<float>::store8(dbeta_part + o, db[k]);
      }
    }
  }
}

// ---- wave-per-row variants for rows up to 2048 wide (GPT-2-XL's 1600,
// ref_main's 2048) --------------------------------------------------------------
// One wave per row, kRowWaves rows per block, reductions by wave shuffles only
// (no LDS, no barriers in the row loop): at 1600 columns the one-row-per-
// 256-thread kernels above leave 56 threads idle and pay two block barriers
// per row with only 2 KB of row data in flight (latency-bound: ~3 TB/s).
// Lane l holds 16-byte vectors l, l + 64, l + 128, l + 192 of its row.
constexpr int kRowWaves = 8;
constexpr int kRowNV = 4;

template <typename T>
__global__ void __launch_bounds__(64 * kRowWaves) ln_fwd_rows_kernel(
    const T* __restrict__ x, const T* __restrict__ res, const T* __restrict__ gamma, const T* __restrict__ beta,
    T* __restrict__ y, T* __restrict__ z, float* __restrict__ mean_out, float* __restrict__ rstd_out, int rows,
    int cols, float eps, float p, uint32_t threshold, uint64_t seed, uint64_t offset) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * kRowWaves + (threadIdx.x >> 6);
  if (row >= rows) return;  // whole waves: no barriers below
  const size_t base = (size_t)row * cols;
  const int nvec = cols >> 3;
  const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  float v[kRowNV][8];
  float s1 = 0.f;
#pragma unroll
  for (int k = 0; k < kRowNV; ++k) {
    const int vi = lane + 64 * k;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[k][i] = 0.f;
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
  const float mean = wave_sum(s1) / (float)cols;
  float s2 = 0.f;
#pragma unroll
  for (int k = 0; k < kRowNV; ++k)
    if (lane + 64 * k < nvec)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float d = v[k][i] - mean;
        s2 += d * d;
      }
  const float rstd = rsqrtf(wave_sum(s2) / (float)cols + eps);
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
#pragma unroll
  for (int k = 0; k < kRowNV; ++k) {
    const int vi = lane + 64 * k;
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

// Backward: gridDim.x = nparts blocks, waves stride over the rows; each lane
// keeps its columns' dgamma / dbeta sums, folded over the block's waves through
// LDS in wave order (deterministic) into the block's partial row.
template <typename T>
__global__ void __launch_bounds__(64 * kRowWaves) ln_bwd_rows_kernel(
    const T* __restrict__ dy, const T* __restrict__ z, const float* __restrict__ mean_in,
    const float* __restrict__ rstd_in, const T* __restrict__ gamma, T* __restrict__ dz, T* __restrict__ dx,
    float* __restrict__ dgamma_part, float* __restrict__ dbeta_part, int rows, int cols, float p,
    uint32_t threshold, uint64_t seed, uint64_t offset, const T* __restrict__ addend) {
  __shared__ float fold[2 * kRowNV * 8 * 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nvec = cols >> 3;
  const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const float inv_n = 1.f / (float)cols;
  // gamma is re-read per row (an L1/L2 hit): held in registers next to the
  // row data and the dgamma / dbeta sums, it spilled
  float dg[kRowNV][8], db[kRowNV][8];
#pragma unroll
  for (int k = 0; k < kRowNV; ++k)
#pragma unroll
    for (int i = 0; i < 8; ++i) dg[k][i] = db[k][i] = 0.f;
  const int stride = gridDim.x * kRowWaves;
  for (int row = blockIdx.x * kRowWaves + wave; row < rows; row += stride) {
    const size_t base = (size_t)row * cols;
    const float mean = mean_in[row], rstd = rstd_in[row];
    float xh[kRowNV][8], gy[kRowNV][8];
    Raw8<T> ad[kRowNV];
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int k = 0; k < kRowNV; ++k) {
      const int vi = lane + 64 * k;
      float zz[8], d[8], g[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) zz[i] = d[i] = g[i] = 0.f;
      ad[k].zero();
      if (vi < nvec) {
        const size_t e = base + (size_t)vi * 8;
        Io<T>::load8(z + e, zz);
        Io<T>::load8(dy + e, d);
        Io<T>::load8(gamma + vi * 8, g);
        if (addend != nullptr) ad[k].load(addend + e);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        xh[k][i] = (zz[i] - mean) * rstd;
        gy[k][i] = d[i] * g[i];
        dg[k][i] += d[i] * xh[k][i];
        db[k][i] += d[i];
        a += gy[k][i];
        b += gy[k][i] * xh[k][i];
      }
    }
    a = wave_sum(a) * inv_n;
    b = wave_sum(b) * inv_n;
#pragma unroll
    for (int k = 0; k < kRowNV; ++k) {
      const int vi = lane + 64 * k;
      if (vi < nvec) {
        const size_t e = base + (size_t)vi * 8;
        float o[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = rstd * (gy[k][i] - a - xh[k][i] * b) + ad[k].get(i);
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
  // fold the waves' partials into wave 0, one wave at a time (fixed order)
  for (int src = 1; src < kRowWaves; ++src) {
    if (wave == src) {
#pragma unroll
      for (int k = 0; k < kRowNV; ++k)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          fold[((0 * kRowNV + k) * 8 + i) * 64 + lane] = dg[k][i];
          fold[((1 * kRowNV + k) * 8 + i) * 64 + lane] = db[k][i];
        }
    }
    __syncthreads();
    if (wave == 0) {
#pragma unroll
      for (int k = 0; k < kRowNV; ++k)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          dg[k][i] += fold[((0 * kRowNV + k) * 8 + i) * 64 + lane];
          db[k][i] += fold[((1 * kRowNV + k) * 8 + i) * 64 + lane];
        }
    }
    __syncthreads();
  }
  if (wave == 0) {
#pragma unroll
    for (int k = 0; k < kRowNV; ++k) {
      const int vi = lane + 64 * k;
      if (vi < nvec) {
        const size_t o = (size_t)blockIdx.x * cols + vi * 8;
        Io<float>::store8(dgamma_part + o, dg[k]);
        Io<float>::store8(dbeta_part + o, db[k]);
      }
    }
  }
}

// MIPIPE_LN_ROWS=0: the one-row-per-block kernels at every width (A/B runs).
int g_ln_rows = -1;
bool ln_rows_variant(int cols) {
  if (g_ln_rows < 0) {
    const char* e = getenv("MIPIPE_LN_ROWS");
    g_ln_rows = e ? atoi(e) : 1;
  }
  return g_ln_rows != 0 && cols <= 64 * kRowNV * 8;
}

template <typename T, int MAXV>
void launch_fwd(const LnArgs<T>& a, hipStream_t s) {
  hipLaunchKernelGGL((ln_fwd_kernel<T, MAXV>), dim3(a.rows), dim3(kThreads), 0, s, a.x, a.res, a.gamma, a.beta,
                     a.y, a.z, a.mean, a.rstd, a.cols, a.eps, a.p, dropout_threshold(a.p), a.seed, a.offset);
}

template <typename T, int MAXV>
void launch_bwd(const LnBwdArgs<T>& a, hipStream_t s) {
  // one partial row pair per block (a.nparts blocks, see ln_bwd_parts)
  constexpr int G = MAXV <= 2 ? 2 : 1;
  hipLaunchKernelGGL((ln_bwd_kernel<T, MAXV, G>), dim3(a.nparts), dim3(kThreads * G), 0, s, a.dy, a.z, a.mean,
                     a.rstd, a.gamma, a.dz, a.dx, a.dgamma_part, a.dbeta_part, a.rows, a.cols, a.p,
                     dropout_threshold(a.p), a.seed, a.offset, a.addend);
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

int ln_bwd_parts(int rows, int cols) {
  // blocks of 2 x 256 threads for rows up to 4096 wide (2048 waves in flight
  // at 256 blocks), single-group blocks of 256 beyond
  const int cap = ln_max_vec(cols) <= 2 ? 256 : 512;
  return rows < cap ? (rows < 1 ? 1 : rows) : cap;
}

template <typename T>
void layernorm_fwd(const LnArgs<T>& a, hipStream_t s) {
  if (ln_rows_variant(a.cols)) {
    hipLaunchKernelGGL((ln_fwd_rows_kernel<T>), dim3((a.rows + kRowWaves - 1) / kRowWaves), dim3(64 * kRowWaves), 0, s,
                       a.x, a.res, a.gamma, a.beta, a.y, a.z, a.mean, a.rstd, a.rows, a.cols, a.eps, a.p,
                       dropout_threshold(a.p), a.seed, a.offset);
    return;
  }
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
  if (ln_rows_variant(a.cols)) {
    hipLaunchKernelGGL((ln_bwd_rows_kernel<T>), dim3(a.nparts), dim3(64 * kRowWaves), 0, s, a.dy, a.z, a.mean, a.rstd,
                       a.gamma, a.dz, a.dx, a.dgamma_part, a.dbeta_part, a.rows, a.cols, a.p, dropout_threshold(a.p),
                       a.seed, a.offset, a.addend);
    reduce_parts(a.dgamma_part, a.dbeta_part, a.nparts, a.cols, a.dgamma, a.dbeta, a.out_f32, a.accumulate, s);
    return;
  }
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
