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

template <typename T>
__global__ void __launch_bounds__(kT) ce_fwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ target,
                                                    int64_t V, int64_t ld, int64_t ignore_index,
                                                    float* __restrict__ loss, float* __restrict__ lse_out) {
  __shared__ float sm[2 * (kT / 64)];
  const int64_t row = blockIdx.x;
  const T* x = logits + row * ld;
  float m = -INFINITY, s = 0.f;
  int64_t c0 = 0;
  if (row_vec_ok(logits, ld)) {
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
    const float lse = M + __logf(S);
    lse_out[row] = lse;
    const int64_t t = target[row];
    if (t == ignore_index || t < 0 || t >= V) {
      loss[row] = 0.f;
    } else {
      loss[row] = lse - Io<T>::load(x + t);
    }
  }
}

// row_scale (optional): per-row dL/dloss_row; then a target outside [0, V)
// means "no one-hot term in this vocabulary slice" (the row still gets its
// softmax term) -- the vocabulary-split decoder's backward.
// zero_to > V: columns [V, zero_to) of dlogits are written with zeros (the
// padded-vocabulary gradient handed straight to the decoder GEMM).
template <typename T>
__global__ void __launch_bounds__(kT) ce_bwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ target,
                                                    const float* __restrict__ lse_in, const float* __restrict__ scale_p,
                                                    const float* __restrict__ row_scale, int64_t V, int64_t ld,
                                                    int64_t ld_out, int64_t ignore_index, T* __restrict__ dlogits,
                                                    int64_t zero_to) {
  const int64_t row = blockIdx.x;
  const T* x = logits + row * ld;
  T* d = dlogits + row * ld_out;
  const int64_t t = target[row];
  const bool valid = !(t == ignore_index || t < 0 || t >= V);
  const float scale = row_scale != nullptr ? row_scale[row] : (valid ? *scale_p : 0.f);
  const float lse = lse_in[row];
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

}  // namespace

template <typename T>
void cross_entropy_fwd(const T* logits, const int64_t* target, int64_t rows, int64_t V, int64_t ld,
                       int64_t ignore_index, float* loss, float* lse, hipStream_t s) {
  if (rows == 0) return;
  hipLaunchKernelGGL((ce_fwd_kernel<T>), dim3((unsigned)rows), dim3(kT), 0, s, logits, target, V, ld, ignore_index,
                     loss, lse);
}

template <typename T>
void cross_entropy_bwd(const T* logits, const int64_t* target, const float* lse, const float* scale,
                       const float* row_scale, int64_t rows, int64_t V, int64_t ld, int64_t ld_out,
                       int64_t ignore_index, T* dlogits, int64_t zero_to, hipStream_t s) {
  if (rows == 0) return;
  hipLaunchKernelGGL((ce_bwd_kernel<T>), dim3((unsigned)rows), dim3(kT), 0, s, logits, target, lse, scale, row_scale,
                     V, ld, ld_out, ignore_index, dlogits, zero_to);
}

template void cross_entropy_fwd<float>(const float*, const int64_t*, int64_t, int64_t, int64_t, int64_t, float*, float*, hipStream_t);
template void cross_entropy_fwd<bf16_t>(const bf16_t*, const int64_t*, int64_t, int64_t, int64_t, int64_t, float*, float*, hipStream_t);
template void cross_entropy_bwd<float>(const float*, const int64_t*, const float*, const float*, const float*, int64_t, int64_t, int64_t, int64_t, int64_t, float*, int64_t, hipStream_t);
template void cross_entropy_bwd<bf16_t>(const bf16_t*, const int64_t*, const float*, const float*, const float*, int64_t, int64_t, int64_t, int64_t, int64_t, bf16_t*, int64_t, hipStream_t);

}  // namespace mipipe
