// Optimizer kernels over FLAT parameter buffers.
//
// Each pipeline stage keeps its parameters in one contiguous buffer (bf16
// model copy + fp32 master copy), its gradients in one contiguous fp32
// `main_grad` buffer and Adam's moments in two more.  The whole optimizer step
// is then two launches regardless of the parameter count:
//   1. sumsq   -- global ||g||^2 of this stage (partials + final, no atomics);
//      the pipeline all-reduces the one float across stages (clip_grad_norm_).
//   2. adam    -- reads the clip coefficient from device memory, updates m, v,
//      the fp32 master and writes the bf16 model copy; 16-byte vectors (4
//      parameters per thread per iteration).
// No host sync anywhere: the norm never leaves the device.
#include "common.h"
#include "kernels.h"

#include <stdlib.h>

namespace mipipe {

namespace {

// Streaming 16-byte loads (nt bit): the builtins take native vector types.
typedef __attribute__((ext_vector_type(4))) float f32x4;
__device__ __forceinline__ float4 nt_load(const float4* p) {
  const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
  return make_float4(v[0], v[1], v[2], v[3]);
}

// NT: streaming loads (default) or regular ones (MIPIPE_SUMSQ_NT=0, for A/B runs:
// profiles/optim_nt_pp8_ab.txt).
template <bool NT>
__global__ void __launch_bounds__(256) sumsq_partial_kernel(const float* __restrict__ g, int64_t n,
                                                            float* __restrict__ partial) {
  __shared__ float sm[8];
  float acc = 0.f;
  const int64_t nvec = n / 4;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 v = NT ? nt_load(g4 + i) : g4[i];
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

struct AdamScalars {
  float coef, step_size, inv_bc2_sqrt;
};

__device__ __forceinline__ float adam_one(float& p, float g, float& mi, float& vi, const AdamHyper& h,
                                          const AdamScalars& c) {
  g *= c.coef;
  if (h.weight_decay != 0.f) {
    if (h.adamw) {
      p -= h.lr * h.weight_decay * p;
    } else {
      g += h.weight_decay * p;
    }
  }
  mi = h.beta1 * mi + (1.f - h.beta1) * g;
  vi = h.beta2 * vi + (1.f - h.beta2) * g * g;
  p -= c.step_size * mi / (sqrtf(vi) * c.inv_bc2_sqrt + h.eps);
  return p;
}

// 4 elements per thread per iteration: 16-byte loads/stores of master, grad,
// m and v, an 8-byte store of 4 bf16 model values (30 B/parameter of HBM
// traffic, the whole step's floor); scalar tail for n % 4.
template <typename M>
__global__ void __launch_bounds__(256) adam_kernel(float* __restrict__ master, M* __restrict__ model,
                                                   const float* __restrict__ grad, float* __restrict__ m,
                                                   float* __restrict__ v, int64_t n, AdamHyper h,
                                                   const float* __restrict__ sumsq) {
  AdamScalars c;
  c.coef = 1.f;
  if (sumsq != nullptr && h.max_norm > 0.f) {
    const float norm = sqrtf(*sumsq);
    c.coef = fminf(1.f, h.max_norm / (norm + 1e-6f));
  }
  c.step_size = h.lr / h.bias_correction1;
  c.inv_bc2_sqrt = 1.f / sqrtf(h.bias_correction2);
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t tid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  float4* P = reinterpret_cast<float4*>(master);
  const float4* G = reinterpret_cast<const float4*>(grad);
  float4* Mo = reinterpret_cast<float4*>(m);
  float4* V = reinterpret_cast<float4*>(v);
  // master, m and v are read once per step here; main_grad was read once
  // before, by sumsq_partial_kernel (grad-norm), also with streaming loads.
  // Streaming (non-temporal) loads measured faster at enc12 PP=1, where the
  // gradients (GBs) are far larger than L2 + MALL; a PP=8 slice (~180M
  // parameters) could keep main_grad cache-resident between the two passes --
  // see profiles/optim_nt_pp8_ab.txt.  Stores stay regular (nt stores
  // measured 3% slower on MI355X).
  // U vectors per thread per iteration, all 4U loads issued before any math:
  // one vector's loads alone left HBM underfed (4.9 TB/s of 30 B/param).
  constexpr int U = 2;
  auto update = [&](int64_t i, float4 p, float4 mm, float4 vv, const float4 g) {
    adam_one(p.x, g.x, mm.x, vv.x, h, c);
    adam_one(p.y, g.y, mm.y, vv.y, h, c);
    adam_one(p.z, g.z, mm.z, vv.z, h, c);
    adam_one(p.w, g.w, mm.w, vv.w, h, c);
    P[i] = p;
    Mo[i] = mm;
    V[i] = vv;
    if (model != nullptr) {
      if constexpr (sizeof(M) == 2) {
        bf16x4 o;
        o[0] = (__bf16)p.x; o[1] = (__bf16)p.y; o[2] = (__bf16)p.z; o[3] = (__bf16)p.w;
        *reinterpret_cast<bf16x4*>(model + 4 * i) = o;
      } else {
        reinterpret_cast<float4*>(model)[i] = p;
      }
    }
  };
  int64_t i = tid;
  for (; i + (U - 1) * stride < n4; i += U * stride) {
    float4 p[U], mm[U], vv[U], g[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      p[u] = nt_load(P + i + u * stride);
      mm[u] = nt_load(Mo + i + u * stride);
      vv[u] = nt_load(V + i + u * stride);
      g[u] = nt_load(G + i + u * stride);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) update(i + u * stride, p[u], mm[u], vv[u], g[u]);
  }
  for (; i < n4; i += stride) update(i, nt_load(P + i), nt_load(Mo + i), nt_load(V + i), nt_load(G + i));
  for (int64_t i = n4 * 4 + tid; i < n; i += stride) {
    float p = master[i], mi = m[i], vi = v[i];
    adam_one(p, grad[i], mi, vi, h, c);
    m[i] = mi;
    v[i] = vi;
    master[i] = p;
    if (model != nullptr) Io<M>::store(model + i, p);
  }
}

// One-shot variant (no grid-stride loop): each thread owns U consecutive-by-
// stride vectors of one block-sized tile; 4U loads in flight, then the math
// and the stores.  adam_set_variant(1) (round 3): 7.24 vs 8.01 ms for the
// 1.44B-parameter enc12 group, 5.99 vs 5.41 TB/s at 30 B/param (tools/adam_ab.py).
__device__ __forceinline__ void nt_store(float4* p, const float4 v) {
  f32x4 x;
  x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
  __builtin_nontemporal_store(x, reinterpret_cast<f32x4*>(p));
}

template <typename M, int U, bool NTS = false>
__global__ void __launch_bounds__(256) adam_tile_kernel(float* __restrict__ master, M* __restrict__ model,
                                                        const float* __restrict__ grad, float* __restrict__ m,
                                                        float* __restrict__ v, int64_t n, AdamHyper h,
                                                        const float* __restrict__ sumsq) {
  AdamScalars c;
  c.coef = 1.f;
  if (sumsq != nullptr && h.max_norm > 0.f) {
    const float norm = sqrtf(*sumsq);
    c.coef = fminf(1.f, h.max_norm / (norm + 1e-6f));
  }
  c.step_size = h.lr / h.bias_correction1;
  c.inv_bc2_sqrt = 1.f / sqrtf(h.bias_correction2);
  const int64_t n4 = n >> 2;
  const int64_t base = (int64_t)blockIdx.x * (256 * U) + threadIdx.x;
  float4* P = reinterpret_cast<float4*>(master);
  const float4* G = reinterpret_cast<const float4*>(grad);
  float4* Mo = reinterpret_cast<float4*>(m);
  float4* V = reinterpret_cast<float4*>(v);
  float4 p[U], mm[U], vv[U], g[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = min(base + u * 256, n4 - 1);  // clamped: loads stay in bounds, stores are masked
    p[u] = nt_load(P + i);
    mm[u] = nt_load(Mo + i);
    vv[u] = nt_load(V + i);
    g[u] = nt_load(G + i);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * 256;
    if (i >= n4) break;
    adam_one(p[u].x, g[u].x, mm[u].x, vv[u].x, h, c);
    adam_one(p[u].y, g[u].y, mm[u].y, vv[u].y, h, c);
    adam_one(p[u].z, g[u].z, mm[u].z, vv[u].z, h, c);
    adam_one(p[u].w, g[u].w, mm[u].w, vv[u].w, h, c);
    if constexpr (NTS) {
      nt_store(P + i, p[u]);
      nt_store(Mo + i, mm[u]);
      nt_store(V + i, vv[u]);
    } else {
      P[i] = p[u];
      Mo[i] = mm[u];
      V[i] = vv[u];
    }
    if (model != nullptr) {
      if constexpr (sizeof(M) == 2) {
        bf16x4 o;
        o[0] = (__bf16)p[u].x; o[1] = (__bf16)p[u].y; o[2] = (__bf16)p[u].z; o[3] = (__bf16)p[u].w;
        if constexpr (NTS) __builtin_nontemporal_store(o, reinterpret_cast<bf16x4*>(model + 4 * i));
        else *reinterpret_cast<bf16x4*>(model + 4 * i) = o;
      } else {
        reinterpret_cast<float4*>(model)[i] = p[u];
      }
    }
  }
  if (blockIdx.x == 0) {  // scalar tail (n % 4)
    for (int64_t i = n4 * 4 + threadIdx.x; i < n; i += 256) {
      float pp = master[i], mi = m[i], vi = v[i];
      adam_one(pp, grad[i], mi, vi, h, c);
      m[i] = mi;
      v[i] = vi;
      master[i] = pp;
      if (model != nullptr) Io<M>::store(model + i, pp);
    }
  }
}

// 2 (default since round 5): the tile kernel with streaming (nt) stores as well -- 6.80 vs 7.06 ms for the
// 1.44B-parameter enc12 group on one box, 6.37 vs 6.14 TB/s at 30 B/param, interleaved (tools/adam_ab.py,
// profiles/adam_r5.txt); a plain torch copy_ reaches 5.16 TB/s on that box.
int g_adam_variant = 2;

}  // namespace

void adam_set_variant(int v) { g_adam_variant = v; }

int sumsq_parts(int64_t n) {
  int64_t b = (n / 4 + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 1024 ? 1024 : b));
}

void sumsq(const float* g, int64_t n, float* partial, int nparts, float* out, hipStream_t s) {
  static const bool nt = [] {
    const char* e = getenv("MIPIPE_SUMSQ_NT");
    return e == nullptr || atoi(e) != 0;
  }();
  if (nt) hipLaunchKernelGGL(sumsq_partial_kernel<true>, dim3(nparts), dim3(256), 0, s, g, n, partial);
  else hipLaunchKernelGGL(sumsq_partial_kernel<false>, dim3(nparts), dim3(256), 0, s, g, n, partial);
  hipLaunchKernelGGL(sumsq_final_kernel, dim3(1), dim3(256), 0, s, partial, nparts, out);
}

template <typename M>
void adam_step(float* master, M* model, const float* grad, float* m, float* v, int64_t n, const AdamHyper& h,
               const float* sumsq_ptr, hipStream_t s) {
  if (n == 0) return;
  if ((g_adam_variant == 1 || g_adam_variant == 2) && n >= 4) {
    constexpr int U = 4;
    const int64_t tiles = (n / 4 + 256 * U - 1) / (256 * U);
    if (g_adam_variant == 2)  // streaming (nt) stores too: A/B (tools/adam_ab.py)
      hipLaunchKernelGGL((adam_tile_kernel<M, U, true>), dim3((unsigned)tiles), dim3(256), 0, s, master, model, grad,
                         m, v, n, h, sumsq_ptr);
    else
      hipLaunchKernelGGL((adam_tile_kernel<M, U>), dim3((unsigned)tiles), dim3(256), 0, s, master, model, grad, m, v,
                         n, h, sumsq_ptr);
    return;
  }
  int64_t blocks = (n / 4 + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 4096) blocks = 4096;  // 16 blocks (64 waves) per CU queued; each thread loops
  hipLaunchKernelGGL((adam_kernel<M>), dim3((unsigned)blocks), dim3(256), 0, s, master, model, grad, m, v, n, h,
                     sumsq_ptr);
}

template void adam_step<float>(float*, float*, const float*, float*, float*, int64_t, const AdamHyper&, const float*, hipStream_t);
template void adam_step<bf16_t>(float*, bf16_t*, const float*, float*, float*, int64_t, const AdamHyper&, const float*, hipStream_t);

}  // namespace mipipe
