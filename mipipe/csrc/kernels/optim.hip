// Optimizer kernels over FLAT parameter buffers.
//
// Each pipeline stage keeps its parameters in one contiguous buffer (bf16
// model copy + fp32 master copy), its gradients in one contiguous fp32
// `main_grad` buffer and Adam's moments in two more.  The whole optimizer step
// is then two launches regardless of the parameter count:
//   1. sumsq   -- global ||g||^2 of this stage (partials + final, no atomics);
//      the pipeline all-reduces the one float across stages (clip_grad_norm_).
//   2. adam    -- reads the clip coefficient from device memory, updates m, v,
//      the fp32 master and writes the bf16 model copy; 16-byte vectors.
// No host sync anywhere: the norm never leaves the device.
#include "common.h"
#include "kernels.h"

namespace mipipe {

namespace {

__global__ void __launch_bounds__(256) sumsq_partial_kernel(const float* __restrict__ g, int64_t n,
                                                            float* __restrict__ partial) {
  __shared__ float sm[8];
  float acc = 0.f;
  const int64_t nvec = n / 4;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 v = g4[i];
    acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  if (blockIdx.x == 0) {
    for (int64_t i = nvec * 4 + threadIdx.x; i < n; i += blockDim.x) acc += g[i] * g[i];
  }
  float dummy = 0.f;
  block_sum2(acc, dummy, sm);
  if (threadIdx.x == 0) partial[blockIdx.x] = acc;
}

__global__ void __launch_bounds__(256) sumsq_final_kernel(const float* __restrict__ partial, int nparts,
                                                          float* __restrict__ out) {
  __shared__ float sm[8];
  float acc = 0.f;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) acc += partial[i];
  float dummy = 0.f;
  block_sum2(acc, dummy, sm);
  if (threadIdx.x == 0) out[0] = acc;
}

template <typename M>
__global__ void __launch_bounds__(256) adam_kernel(float* __restrict__ master, M* __restrict__ model,
                                                   const float* __restrict__ grad, float* __restrict__ m,
                                                   float* __restrict__ v, int64_t n, AdamHyper h,
                                                   const float* __restrict__ sumsq) {
  float coef = 1.f;
  if (sumsq != nullptr && h.max_norm > 0.f) {
    const float norm = sqrtf(*sumsq);
    coef = fminf(1.f, h.max_norm / (norm + 1e-6f));
  }
  const float step_size = h.lr / h.bias_correction1;
  const float inv_bc2_sqrt = 1.f / sqrtf(h.bias_correction2);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float p = master[i];
    float g = grad[i] * coef;
    if (h.weight_decay != 0.f) {
      if (h.adamw) {
        p -= h.lr * h.weight_decay * p;
      } else {
        g += h.weight_decay * p;
      }
    }
    float mi = h.beta1 * m[i] + (1.f - h.beta1) * g;
    float vi = h.beta2 * v[i] + (1.f - h.beta2) * g * g;
    m[i] = mi;
    v[i] = vi;
    p -= step_size * mi / (sqrtf(vi) * inv_bc2_sqrt + h.eps);
    master[i] = p;
    if (model != nullptr) Io<M>::store(model + i, p);
  }
}

}  // namespace

int sumsq_parts(int64_t n) {
  int64_t b = (n / 4 + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 1024 ? 1024 : b));
}

void sumsq(const float* g, int64_t n, float* partial, int nparts, float* out, hipStream_t s) {
  hipLaunchKernelGGL(sumsq_partial_kernel, dim3(nparts), dim3(256), 0, s, g, n, partial);
  hipLaunchKernelGGL(sumsq_final_kernel, dim3(1), dim3(256), 0, s, partial, nparts, out);
}

template <typename M>
void adam_step(float* master, M* model, const float* grad, float* m, float* v, int64_t n, const AdamHyper& h,
               const float* sumsq_ptr, hipStream_t s) {
  if (n == 0) return;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL((adam_kernel<M>), dim3((unsigned)blocks), dim3(256), 0, s, master, model, grad, m, v, n, h,
                     sumsq_ptr);
}

template void adam_step<float>(float*, float*, const float*, float*, float*, int64_t, const AdamHyper&, const float*, hipStream_t);
template void adam_step<bf16_t>(float*, bf16_t*, const float*, float*, float*, int64_t, const AdamHyper&, const float*, hipStream_t);

}  // namespace mipipe
