// Token embedding: gather x sqrt(E) + positional encoding + dropout
// and its backward scatter-add (K12).
//
// Forward: one workgroup per token row, 16-byte vector gathers of the
// embedding row (whole rows are contiguous, so the gather is coalesced).
// Backward: dW[token] += dout * scale * mask, accumulated in fp32 with
// no-return global float atomics, one dword per lane per instruction and whole
// contiguous rows per wave (the shape the atomic unit serves at full rate,
// Guideline 12).  The fp32 accumulator is the parameter's persistent
// `main_grad` buffer, so no dense [V, E] gradient is materialised per
// micro-batch.
#include "common.h"
#include "kernels.h"

namespace mipipe {

namespace {

template <typename T, typename P>
__global__ void __launch_bounds__(256) embed_fwd_kernel(const int64_t* __restrict__ tokens, const T* __restrict__ weight,
                                                        const P* __restrict__ pe, T* __restrict__ out, int seq_len,
                                                        int E, int64_t V, float scale, float p, uint32_t threshold,
                                                        uint64_t seed, uint64_t offset) {
  const int64_t row = blockIdx.x;  // token index in [B*S]
  const int pos = (int)(row % seq_len);
  int64_t tok = tokens[row];
  tok = tok < 0 ? 0 : (tok >= V ? V - 1 : tok);  // host validates; clamp keeps a bad id from faulting
  const float pscale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  for (int vi = threadIdx.x; vi < E / 8; vi += blockDim.x) {
    float w[8], q[8];
    Io<T>::load8(weight + tok * E + vi * 8, w);
    if (pe != nullptr) {
      Io<P>::load8(pe + (int64_t)pos * E + vi * 8, q);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) q[i] = 0.f;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = w[i] * scale + q[i];
    const int64_t e = row * E + vi * 8;
    if (p > 0.f) {
      const uint32_t keep = dropout_keep8(seed, offset, (uint64_t)e, threshold);
#pragma unroll
      for (int i = 0; i < 8; ++i) w[i] = ((keep >> i) & 1) ? w[i] * pscale : 0.f;
    }
    Io<T>::store8(out + e, w);
  }
}

// Scatter-add of one token row per workgroup into the fp32 table gradient.
// The row is read with 16-byte loads (8 consecutive elements per lane, the
// dropout mask's 8-element granule), bounced through LDS, and added back with
// lane-contiguous float atomics: one 256-byte request per wave-instruction
// (memory-side atomics run at ~1.3 TB/s of added bytes; a lane stride of 32 B
// would cut that 8x).  Rows of E <= 8192 elements.
// dpe (optional): the learned position table's fp32 gradient -- the same
// masked row (without the token scale) is added at the row's position, so
// GPT-2's position embedding needs no separate reduction over the batch.
template <typename T>
__global__ void __launch_bounds__(256) embed_bwd_kernel(const int64_t* __restrict__ tokens, const T* __restrict__ dout,
                                                        float* __restrict__ dweight, float* __restrict__ dpe,
                                                        int seq_len, int E, int64_t V, float scale, float p,
                                                        uint32_t threshold, uint64_t seed, uint64_t offset) {
  __shared__ float rowbuf[8192];
  const int64_t row = blockIdx.x;
  const int64_t tok = tokens[row];
  const bool tok_ok = tok >= 0 && tok < V;
  if (!tok_ok && dpe == nullptr) return;
  const float pscale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  for (int vi = threadIdx.x; vi < E / 8; vi += blockDim.x) {
    float g[8];
    const int64_t e = row * E + vi * 8;
    Io<T>::load8(dout + e, g);
    uint32_t keep = 0xFFu;
    if (p > 0.f) keep = dropout_keep8(seed, offset, (uint64_t)e, threshold);
#pragma unroll
    for (int i = 0; i < 8; ++i) rowbuf[vi * 8 + i] = ((keep >> i) & 1) ? g[i] * pscale : 0.f;
  }
  __syncthreads();
  if (tok_ok) {
    float* dst = dweight + tok * E;
    for (int c = threadIdx.x; c < E; c += blockDim.x) atomicAdd(dst + c, rowbuf[c] * scale);
  }
  if (dpe != nullptr) {
    float* dst = dpe + (row % seq_len) * E;
    for (int c = threadIdx.x; c < E; c += blockDim.x) atomicAdd(dst + c, rowbuf[c]);
  }
}

}  // namespace

template <typename T>
void embedding_fwd(const int64_t* tokens, const T* weight, const void* pe, bool pe_f32, T* out, int64_t rows,
                   int seq_len, int E, int64_t V, float scale, float p, uint64_t seed, uint64_t offset, hipStream_t s) {
  if (rows == 0) return;
  if (pe_f32 || pe == nullptr)
    hipLaunchKernelGGL((embed_fwd_kernel<T, float>), dim3((unsigned)rows), dim3(256), 0, s, tokens, weight,
                       static_cast<const float*>(pe), out, seq_len, E, V, scale, p, dropout_threshold(p), seed, offset);
  else  // a table in the model dtype (GPT-2's learned positions in a bf16 model): read as stored
    hipLaunchKernelGGL((embed_fwd_kernel<T, T>), dim3((unsigned)rows), dim3(256), 0, s, tokens, weight,
                       static_cast<const T*>(pe), out, seq_len, E, V, scale, p, dropout_threshold(p), seed, offset);
}

template <typename T>
void embedding_bwd(const int64_t* tokens, const T* dout, float* dweight, int64_t rows, int E, int64_t V, float scale,
                   float p, uint64_t seed, uint64_t offset, hipStream_t s, float* dpe, int seq_len) {
  if (rows == 0 || E > 8192) return;  // callers check embedding_supported
  hipLaunchKernelGGL((embed_bwd_kernel<T>), dim3((unsigned)rows), dim3(256), 0, s, tokens, dout, dweight, dpe,
                     seq_len > 0 ? seq_len : 1, E, V, scale, p, dropout_threshold(p), seed, offset);
}

template void embedding_fwd<float>(const int64_t*, const float*, const void*, bool, float*, int64_t, int, int, int64_t, float, float, uint64_t, uint64_t, hipStream_t);
template void embedding_fwd<bf16_t>(const int64_t*, const bf16_t*, const void*, bool, bf16_t*, int64_t, int, int, int64_t, float, float, uint64_t, uint64_t, hipStream_t);
template void embedding_bwd<float>(const int64_t*, const float*, float*, int64_t, int, int64_t, float, float, uint64_t, uint64_t, hipStream_t, float*, int);
template void embedding_bwd<bf16_t>(const int64_t*, const bf16_t*, float*, int64_t, int, int64_t, float, float, uint64_t, uint64_t, hipStream_t, float*, int);

}  // namespace mipipe
