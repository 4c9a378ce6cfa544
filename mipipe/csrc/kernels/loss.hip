// Fused cross-entropy (log-softmax + NLL), forward and backward.
//
// One 256-thread workgroup per row.  Forward streams the row once with an
// online (running max, running sum) reduction and writes only the per-row loss
// and log-sum-exp -- the log-probabilities are never materialised.  Backward
// streams the row once more and writes dlogits = scale * (softmax - onehot),
// where `scale` (= dL / n_valid) is read from device memory so no host sync is
// needed.  Vocabularies need not be multiples of 8 (28,782 in the reference
// driver): rows of a padded-vocabulary buffer are 16-byte aligned, so the
// body of each row is read with 16-byte vectors and only the V % 8 tail is scalar.
#include "common.h"
#include "kernels.h"

namespace mipipe {

namespace {

constexpr int kT = 256;

// Online (max, sum-of-exp) update with one value.
__device__ __forceinline__ void lse_push(float& m, float& s, float v) {
  if (v > m) {
    s = s * __expf(m - v) + 1.f;
    m = v;
  } else {
    s += __expf(v - m);
  }
}

// Rows whose base and stride are 16-byte aligned run a vector path: 8 values
// per 16-byte load, ONE rescale per chunk (chunk max first), scalar tail for
// V % 8.  4,096 x 28,782 bf16 logits: 1 scalar 2-byte load per element
// streamed at ~0.9 TB/s; the vector path is HBM-bound.
template <typename T>
__device__ __forceinline__ bool row_vec_ok(const T* p, int64_t ld) {
  return (reinterpret_cast<uintptr_t>(p) % 16 == 0) && ((ld * (int64_t)sizeof(T)) % 16 == 0);
}

// Row log-sum-exp of x[0, V) by one kT-thread block, returned to every thread
// (sm: 2 * kT / 64 + 1 floats of LDS).
template <typename T>
__device__ __forceinline__ float block_row_lse(const T* __restrict__ x, int64_t V, bool vec, float* sm) {
  float m = -INFINITY, s = 0.f;
  int64_t c0 = 0;
  if (vec) {
    const int64_t nv = V >> 3;
    for (int64_t vi = threadIdx.x; vi < nv; vi += kT) {
      float a[8];
      Io<T>::load8(x + vi * 8, a);
      float cm = a[0];
#pragma unroll
      for (int i = 1; i < 8; ++i) cm = fmaxf(cm, a[i]);
      if (cm > m) {
        s *= __expf(m - cm);
        m = cm;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) s += __expf(a[i] - m);
    }
    c0 = nv << 3;
  }
  for (int64_t c = c0 + threadIdx.x; c < V; c += kT) lse_push(m, s, Io<T>::load(x + c));
  // combine (m, s) across the wave, then the block
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64);
    const float os = __shfl_xor(s, o, 64);
    const float nm = fmaxf(m, om);
    s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + (om == -INFINITY ? 0.f : os * __expf(om - nm));
    m = nm;
  }
  if (lane == 0) {
    sm[wid] = m;
    sm[kT / 64 + wid] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = -INFINITY;
    for (int w = 0; w < kT / 64; ++w) M = fmaxf(M, sm[w]);
    float S = 0.f;
    for (int w = 0; w < kT / 64; ++w) S += sm[w] == -INFINITY ? 0.f : sm[kT / 64 + w] * __expf(sm[w] - M);
    sm[2 * (kT / 64)] = M + __logf(S);
  }
  __syncthreads();
  return sm[2 * (kT / 64)];
}

// t_offset: the logits are vocabulary columns [t_offset, t_offset + V) of a
// larger vocabulary (the split decoder): a target t counts as t - t_offset when
// it falls in the slice and as "no target here" (loss 0) otherwise.
template <typename T>
__global__ void __launch_bounds__(kT) ce_fwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ target,
                                                    int64_t V, int64_t ld, int64_t ignore_index,
                                                    float* __restrict__ loss, float* __restrict__ lse_out,
                                                    int64_t t_offset) {
  __shared__ float sm[2 * (kT / 64) + 1];
  const int64_t row = blockIdx.x;
  const T* x = logits + row * ld;
  const float lse = block_row_lse(x, V, row_vec_ok(logits, ld), sm);
  if (threadIdx.x == 0) {
    lse_out[row] = lse;
    const int64_t t0 = target[row], t = t0 - t_offset;
    if (t0 == ignore_index || t < 0 || t >= V) {
      loss[row] = 0.f;
    } else {
      loss[row] = lse - Io<T>::load(x + t);
    }
  }
}

// ---------------------------------------------------------------- split decoder
// (mipipe/models/vocab_split.py).  A packed message row is [h (E values) |
// statistic slots]: the slots hold `nslot` fp32 words (bit-cast into the
// activation dtype), words 0 and 1 used, the rest zero.

// Head forward: out[row] = [x[row] | lse(logits[row]), logits[row, t] (0 when
// the target is outside [0, V)), 0...] -- the pack and the statistics in one pass.
template <typename T>
__global__ void __launch_bounds__(kT) vsplit_head_fwd_kernel(const T* __restrict__ logits, int64_t ld, int64_t V,
                                                             const int64_t* __restrict__ target,
                                                             const T* __restrict__ x, int64_t ldx, int64_t E,
                                                             T* __restrict__ out, int64_t ldo, int nslot) {
  __shared__ float sm[2 * (kT / 64) + 1];
  const int64_t row = blockIdx.x;
  // the pack first: its loads overlap the row reduction's
  const int64_t nvec = E * (int64_t)sizeof(T) / 16;
  const uint4* src = reinterpret_cast<const uint4*>(x + row * ldx);
  uint4* dst = reinterpret_cast<uint4*>(out + row * ldo);
  for (int64_t i = threadIdx.x; i < nvec; i += kT) dst[i] = src[i];
  const T* l = logits + row * ld;
  const float lse = block_row_lse(l, V, row_vec_ok(logits, ld), sm);
  float* st = reinterpret_cast<float*>(out + row * ldo + E);
  if (threadIdx.x < nslot) {
    float v = 0.f;
    if (threadIdx.x == 0) {
      v = lse;
    } else if (threadIdx.x == 1) {
      const int64_t t = target[row];
      v = (t >= 0 && t < V) ? Io<T>::load(l + t) : 0.f;
    }
    st[threadIdx.x] = v;
  }
}

// Tail forward, per row: the slice [t_offset, t_offset + V)'s log-sum-exp is
// merged with the head's (slot word 0) into the full lse; the target logit
// comes from this slice or the head (slot word 1).  Writes lse, the row loss
// and the row's validity (1 / 0) -- vsplit_mean_kernel reduces them.
template <typename T>
__global__ void __launch_bounds__(kT) vsplit_tail_fwd_kernel(const T* __restrict__ logits, int64_t ld, int64_t V,
                                                             const int64_t* __restrict__ target, int64_t t_offset,
                                                             int64_t ignore_index, const float* __restrict__ stats,
                                                             int64_t ld_st, float* __restrict__ lse_out,
                                                             float* __restrict__ loss_row,
                                                             float* __restrict__ valid_row) {
  __shared__ float sm[2 * (kT / 64) + 1];
  const int64_t row = blockIdx.x;
  const T* l = logits + row * ld;
  const float lse_b = block_row_lse(l, V, row_vec_ok(logits, ld), sm);
  if (threadIdx.x == 0) {
    const float lse_a = stats[row * ld_st], t_a = stats[row * ld_st + 1];
    const float mx = fmaxf(lse_a, lse_b);
    const float lse = mx == -INFINITY ? mx : mx + __logf(__expf(lse_a - mx) + __expf(lse_b - mx));
    const int64_t t = target[row], tb = t - t_offset;
    const bool valid = t != ignore_index && t >= 0 && t < t_offset + V;
    const float tl = (tb >= 0 && tb < V) ? Io<T>::load(l + tb) : t_a;
    lse_out[row] = lse;
    loss_row[row] = valid ? lse - tl : 0.f;
    valid_row[row] = valid ? 1.f : 0.f;
  }
}

// One block: loss = sum(loss_row) / max(sum(valid), 1); then valid_row[r] is
// turned into the row weight valid / count in place (dloss_row / dloss).
// A fixed-order reduction: the loss is bitwise reproducible.
constexpr int kMeanT = 1024;
__global__ void __launch_bounds__(kMeanT) vsplit_mean_kernel(const float* __restrict__ loss_row,
                                                             float* __restrict__ valid_row, int64_t rows,
                                                             float* __restrict__ loss) {
  __shared__ float sl[kMeanT / 64], sc[kMeanT / 64], tot[2];
  float a = 0.f, c = 0.f;
  for (int64_t r = threadIdx.x; r < rows; r += kMeanT) {
    a += loss_row[r];
    c += valid_row[r];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    c += __shfl_xor(c, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    sl[threadIdx.x >> 6] = a;
    sc[threadIdx.x >> 6] = c;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float A = 0.f, C = 0.f;
    for (int w = 0; w < kMeanT / 64; ++w) {
      A += sl[w];
      C += sc[w];
    }
    C = fmaxf(C, 1.f);
    tot[0] = A / C;
    tot[1] = 1.f / C;
    loss[0] = tot[0];
  }
  __syncthreads();
  const float inv = tot[1];
  for (int64_t r = threadIdx.x; r < rows; r += kMeanT) valid_row[r] *= inv;
}

// row_scale (optional): per-row dL/dloss_row; then a target outside [0, V)
// means "no one-hot term in this vocabulary slice" (the row still gets its
// softmax term) -- the vocabulary-split decoder's backward.
// zero_to > V: columns [V, zero_to) of dlogits are written with zeros (the
// padded-vocabulary gradient handed straight to the decoder GEMM).
// lse / row_scale may be strided (ld_lse, ld_rs floats): the statistics can be
// read straight out of the packed slots of a split-decoder message.  Both
// scale_p and row_scale given: the row's scale is their product.
// stat_out (optional): the row's (lse, scale) go to slot words 0 / 1 of a
// split-decoder gradient message (nslot words per row, stride ld_stat floats).
template <typename T>
__global__ void __launch_bounds__(kT) ce_bwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ target,
                                                    const float* __restrict__ lse_in, const float* __restrict__ scale_p,
                                                    const float* __restrict__ row_scale, int64_t V, int64_t ld,
                                                    int64_t ld_out, int64_t ignore_index, T* __restrict__ dlogits,
                                                    int64_t zero_to, int64_t t_offset, int64_t ld_lse, int64_t ld_rs,
                                                    float* __restrict__ stat_out, int64_t ld_stat, int nslot) {
  const int64_t row = blockIdx.x;
  const T* x = logits + row * ld;
  T* d = dlogits + row * ld_out;
  const int64_t t0 = target[row];
  const bool valid = !(t0 == ignore_index || t0 - t_offset < 0 || t0 - t_offset >= V);
  const int64_t t = valid ? t0 - t_offset : -1;  // the one-hot column (none: -1)
  const float scale = row_scale != nullptr ? row_scale[row * ld_rs] * (scale_p != nullptr ? *scale_p : 1.f)
                                           : (valid ? *scale_p : 0.f);
  const float lse = lse_in[row * ld_lse];
  if (stat_out != nullptr && threadIdx.x < nslot)
    stat_out[row * ld_stat + threadIdx.x] = threadIdx.x == 0 ? lse : threadIdx.x == 1 ? scale : 0.f;
  int64_t c0 = 0;
  if (row_vec_ok(logits, ld) && row_vec_ok(dlogits, ld_out)) {
    const int64_t nv = V >> 3;
    for (int64_t vi = threadIdx.x; vi < nv; vi += kT) {
      float a[8];
      Io<T>::load8(x + vi * 8, a);
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = (__expf(a[i] - lse) - (vi * 8 + i == t ? 1.f : 0.f)) * scale;
      Io<T>::store8(d + vi * 8, a);
    }
    c0 = nv << 3;
  }
  for (int64_t c = c0 + threadIdx.x; c < V; c += kT) {
    const float pr = __expf(Io<T>::load(x + c) - lse);
    Io<T>::store(d + c, (pr - (c == t ? 1.f : 0.f)) * scale);
  }
  for (int64_t c = V + threadIdx.x; c < zero_to; c += kT) Io<T>::store(d + c, 0.f);
}

// Plain CE mean: loss = sum(loss_row) / max(#valid targets, 1) with valid =
// (t != ignore_index and 0 <= t < V); weight[r] = valid / count (the rows'
// dL/dloss_row for dL/dloss = 1, read by the backward as its row scale).  One
// block, fixed-order reduction (bitwise reproducible).  A target outside
// [0, V) that is not ignore_index (nn.CrossEntropyLoss raises on it) makes
// the loss and the row weights NaN: loud, without a host sync, where
// leaving the row out would silently re-weight the mean.
__global__ void __launch_bounds__(kMeanT) ce_mean_kernel(const float* __restrict__ loss_row,
                                                         const int64_t* __restrict__ target, int64_t rows, int64_t V,
                                                         int64_t ignore_index, float* __restrict__ weight,
                                                         float* __restrict__ loss) {
  __shared__ float sl[kMeanT / 64], sc[kMeanT / 64], tot;
  float a = 0.f, c = 0.f, bad = 0.f;
  for (int64_t r = threadIdx.x; r < rows; r += kMeanT) {
    const int64_t t = target[r];
    a += loss_row[r];
    c += (t != ignore_index && t >= 0 && t < V) ? 1.f : 0.f;
    bad += (t != ignore_index && (t < 0 || t >= V)) ? 1.f : 0.f;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    c += __shfl_xor(c, o, 64);
    bad += __shfl_xor(bad, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    sl[threadIdx.x >> 6] = a;
    sc[threadIdx.x >> 6] = c + (bad > 0.f ? 1e30f : 0.f);  // any bad target poisons the count
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float A = 0.f, C = 0.f;
    for (int w = 0; w < kMeanT / 64; ++w) {
      A += sl[w];
      C += sc[w];
    }
    const bool poisoned = C >= 1e30f;
    C = fmaxf(C, 1.f);
    loss[0] = poisoned ? __builtin_nanf("") : A / C;
    tot = poisoned ? __builtin_nanf("") : 1.f / C;
  }
  __syncthreads();
  const float inv = tot;
  for (int64_t r = threadIdx.x; r < rows; r += kMeanT) {
    const int64_t t = target[r];
    weight[r] = (t != ignore_index && t >= 0 && t < V) ? inv : 0.f;
  }
}

}  // namespace

template <typename T>
void cross_entropy_mean_fwd(const T* logits, const int64_t* target, int64_t rows, int64_t V, int64_t ld,
                            int64_t ignore_index, float* loss_row, float* lse, float* weight, float* loss,
                            hipStream_t s) {
  if (rows == 0) return;
  hipLaunchKernelGGL((ce_fwd_kernel<T>), dim3((unsigned)rows), dim3(kT), 0, s, logits, target, V, ld, ignore_index,
                     loss_row, lse, (int64_t)0);
  hipLaunchKernelGGL(ce_mean_kernel, dim3(1), dim3(kMeanT), 0, s, loss_row, target, rows, V, ignore_index, weight,
                     loss);
}
template void cross_entropy_mean_fwd<float>(const float*, const int64_t*, int64_t, int64_t, int64_t, int64_t, float*, float*, float*, float*, hipStream_t);
template void cross_entropy_mean_fwd<bf16_t>(const bf16_t*, const int64_t*, int64_t, int64_t, int64_t, int64_t, float*, float*, float*, float*, hipStream_t);

template <typename T>
void cross_entropy_fwd(const T* logits, const int64_t* target, int64_t rows, int64_t V, int64_t ld,
                       int64_t ignore_index, float* loss, float* lse, hipStream_t s, int64_t t_offset) {
  if (rows == 0) return;
  hipLaunchKernelGGL((ce_fwd_kernel<T>), dim3((unsigned)rows), dim3(kT), 0, s, logits, target, V, ld, ignore_index,
                     loss, lse, t_offset);
}

template <typename T>
void cross_entropy_bwd(const T* logits, const int64_t* target, const float* lse, const float* scale,
                       const float* row_scale, int64_t rows, int64_t V, int64_t ld, int64_t ld_out,
                       int64_t ignore_index, T* dlogits, int64_t zero_to, hipStream_t s, int64_t t_offset,
                       int64_t ld_lse, int64_t ld_rs, float* stat_out, int64_t ld_stat, int nslot) {
  if (rows == 0) return;
  hipLaunchKernelGGL((ce_bwd_kernel<T>), dim3((unsigned)rows), dim3(kT), 0, s, logits, target, lse, scale, row_scale,
                     V, ld, ld_out, ignore_index, dlogits, zero_to, t_offset, ld_lse, ld_rs, stat_out, ld_stat, nslot);
}

template <typename T>
void vsplit_head_fwd(const T* logits, int64_t ld, int64_t rows, int64_t V, const int64_t* target, const T* x,
                     int64_t ldx, int64_t E, T* out, int64_t ldo, int nslot, hipStream_t s) {
  if (rows == 0) return;
  hipLaunchKernelGGL((vsplit_head_fwd_kernel<T>), dim3((unsigned)rows), dim3(kT), 0, s, logits, ld, V, target, x, ldx,
                     E, out, ldo, nslot);
}

template <typename T>
void vsplit_tail_fwd(const T* logits, int64_t ld, int64_t rows, int64_t V, const int64_t* target, int64_t t_offset,
                     int64_t ignore_index, const float* stats, int64_t ld_st, float* lse, float* loss_row,
                     float* weight_row, float* loss, hipStream_t s) {
  if (rows == 0) return;
  hipLaunchKernelGGL((vsplit_tail_fwd_kernel<T>), dim3((unsigned)rows), dim3(kT), 0, s, logits, ld, V, target, t_offset,
                     ignore_index, stats, ld_st, lse, loss_row, weight_row);
  hipLaunchKernelGGL(vsplit_mean_kernel, dim3(1), dim3(kMeanT), 0, s, loss_row, weight_row, rows, loss);
}

template void cross_entropy_fwd<float>(const float*, const int64_t*, int64_t, int64_t, int64_t, int64_t, float*, float*, hipStream_t, int64_t);
template void cross_entropy_fwd<bf16_t>(const bf16_t*, const int64_t*, int64_t, int64_t, int64_t, int64_t, float*, float*, hipStream_t, int64_t);
#define MP_CE_INST(T)                                                                                              \
  template void cross_entropy_bwd<T>(const T*, const int64_t*, const float*, const float*, const float*, int64_t,     \
                                     int64_t, int64_t, int64_t, int64_t, T*, int64_t, hipStream_t, int64_t, int64_t,   \
                                     int64_t, float*, int64_t, int);                                                   \
  template void vsplit_head_fwd<T>(const T*, int64_t, int64_t, int64_t, const int64_t*, const T*, int64_t, int64_t,   \
                                   T*, int64_t, int, hipStream_t);                                                    \
  template void vsplit_tail_fwd<T>(const T*, int64_t, int64_t, int64_t, const int64_t*, int64_t, int64_t,             \
                                   const float*, int64_t, float*, float*, float*, float*, hipStream_t);
MP_CE_INST(float)
MP_CE_INST(bf16_t)
#undef MP_CE_INST

}  // namespace mipipe
