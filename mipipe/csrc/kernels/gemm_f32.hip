// fp32 MFMA GEMM for gfx950 with the same fused epilogues as the bf16 kernel
// (SURVEY §2.3 K1/K4/K6/K8/K10/K13 in the reference's own precision, fp32).
//
//   C[M, N] = A[M, K] . B[K, N]      (fp32 operands, fp32 accumulation)
//
// gfx950 has no xf32/TF32: the matrix path for fp32 is v_mfma_f32_32x32x2_f32,
// exact fp32 (one rounding per product, k-ordered), 64 FLOP/clk/SIMD -- 1/16
// of bf16 MFMA, the same rate as packed fp32 FMA on the VALU, but it needs one
// VGPR per operand per lane and leaves the VALU to the epilogue.  At that rate
// the kernel is compute-bound for any tile >= 64x64, so the design goal is
// only to keep one MFMA chain per accumulator issuing back to back:
//
// * 256 threads = 4 waves (2 x 2), each wave TM x TN tiles of 32x32 (block
//   tile 64..128 x 64..128), BK = 32, two LDS buffers, register-staged
//   global loads one K-tile ahead (fp32 rows are 16-byte float4 loads).
// * The MFMA sums over k, so k may be permuted inside a K-tile as long as A
//   and B agree: in k-step s lane half h (= lane >> 5) uses physical k =
//   16h + 4(s >> 2) + (s & 3).  Then a K-contiguous operand hands each lane 4
//   consecutive k-steps in ONE ds_read_b128 (row-pair XOR swizzle: the 16
//   lanes of a read phase hit 16 distinct 16-byte bank groups), and an
//   I-contiguous operand is one ds_read_b32 per step whose two lane halves
//   (rows k and k + 16) are 128 bytes apart after an XOR of the chunk index
//   (all 64 banks distinct).
// * Two blocks per CU (2 x 64 KiB LDS): while one block waits at its barrier
//   the other's MFMAs run.
// * Epilogues as gemm.hip: bias + ReLU/GELU + dropout (same Philox
//   column-quad mask layout as the elementwise backward) + residual addend +
//   pre-activation aux output, all fp32; fp32 += (weight gradients into
//   main_grad, K-segmented for deferred wgrad); fp32 store.
// The operand layouts are the bf16 kernel's: forward (KC, KC), dgrad (KC, IC),
// wgrad (IC, IC).  M, N multiples of 4, K a multiple of 32.
#include "common.h"
#include "kernels.h"

namespace mipipe {

namespace {

constexpr int BK = 32;
constexpr int kThreads = 256;

// K-contiguous image [rows][32 floats]: 128-byte rows, 16-byte chunk c of row
// r stored at chunk c ^ ((r >> 1) & 7).
__device__ __forceinline__ int kc_off(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

// I-contiguous image [32 k][ROWS floats]: chunk c (4 floats) of row k stored at
// chunk c ^ (8 * ((k >> 4) & 1)).
template <int ROWS>
__device__ __forceinline__ int ic_off(int k, int c) { return k * ROWS * 4 + ((c ^ (((k >> 4) & 1) << 3)) << 4); }

__device__ __forceinline__ float gelu_f(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }

// Bijective XCD-aware block remap + groups of 8 tile rows (as gemm.hip).
__device__ __forceinline__ void tile_coords(int tiles_m, int tiles_n, int& tm, int& tn) {
  const int nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  int wg = bid;
  if (nwg > 8) {
    const int xcd = bid & 7, local = bid >> 3;
    const int q = nwg >> 3, r = nwg & 7;
    wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + local;
  }
  constexpr int G = 8;
  const int group = wg / (G * tiles_n);
  const int first_m = group * G;
  const int gsize = min(tiles_m - first_m, G);
  const int in_group = wg % (G * tiles_n);
  tm = first_m + in_group % gsize;
  tn = in_group / gsize;
}

__device__ __forceinline__ const float* seg_base(const GemmArgs& g, bool is_a, int k0, int& kl) {
  if (g.seg_k == 0) {
    kl = k0;
    return reinterpret_cast<const float*>(is_a ? g.A : g.B);
  }
  const int s = k0 / g.seg_k;
  kl = k0 - s * g.seg_k;
  return reinterpret_cast<const float*>(is_a ? g.a_seg[s] : g.b_seg[s]);
}

// Register staging of one operand tile (ROWS x 32 of the operand's M or N rows).
template <int ROWS, bool KC>
struct Stage {
  static constexpr int kN = ROWS * BK / 4 / kThreads;  // float4s per thread
  f32x4 v[kN];  // native vector type: HIP's float4 struct copies become memcpys that pin the array in scratch
  __device__ __forceinline__ void load(const float* base, int64_t ld, int i0, int lim, int k0, int tid) {
#pragma unroll
    for (int u = 0; u < kN; ++u) {
      const int id = tid + u * kThreads;
      const float* p;
      if (KC) {
        const int r = id >> 3, c = id & 7;
        const int gi = min(i0 + r, lim - 1);  // edge rows clamp (masked at the store)
        p = base + (int64_t)gi * ld + k0 + 4 * c;
      } else {
        constexpr int CPR = ROWS / 4;  // chunks per k-row
        const int k = id / CPR, c = id % CPR;
        const int gi = min(i0 + 4 * c, lim - 4);
        p = base + (int64_t)(k0 + k) * ld + gi;
      }
      v[u] = *reinterpret_cast<const f32x4*>(p);
    }
  }
  __device__ __forceinline__ void store(char* tile, int tid) const {
#pragma unroll
    for (int u = 0; u < kN; ++u) {
      const int id = tid + u * kThreads;
      int off;
      if (KC) {
        off = kc_off(id >> 3, id & 7);
      } else {
        constexpr int CPR = ROWS / 4;
        off = ic_off<ROWS>(id / CPR, id % CPR);
      }
      *reinterpret_cast<f32x4*>(tile + off) = v[u];
    }
  }
};

// The 4 k-steps 4q..4q+3 of rows [ib, ib+32): element e = k-step 4q + e.
template <int ROWS, bool KC>
__device__ __forceinline__ float4 frag4(const char* tile, int ib, int q, int lane) {
  const int i = ib + (lane & 31), h = lane >> 5;
  if (KC) return *reinterpret_cast<const float4*>(tile + kc_off(i, 4 * h + q));
  float4 r;
  const int k0 = 16 * h + 4 * q;
  const int c = i >> 2, w = (i & 3) * 4;
  r.x = *reinterpret_cast<const float*>(tile + ic_off<ROWS>(k0 + 0, c) + w);
  r.y = *reinterpret_cast<const float*>(tile + ic_off<ROWS>(k0 + 1, c) + w);
  r.z = *reinterpret_cast<const float*>(tile + ic_off<ROWS>(k0 + 2, c) + w);
  r.w = *reinterpret_cast<const float*>(tile + ic_off<ROWS>(k0 + 3, c) + w);
  return r;
}

__device__ __forceinline__ float f4(const float4& v, int e) { return e == 0 ? v.x : (e == 1 ? v.y : (e == 2 ? v.z : v.w)); }

template <int TM, int TN, bool A_KC, bool B_KC, int EPI, int ACT>
__global__ void __launch_bounds__(kThreads, 2) gemm_f32_kernel(GemmArgs g) {
  constexpr int BM = 2 * 32 * TM, BN = 2 * 32 * TN;
  constexpr int kA = BM * BK * 4, kB = BN * BK * 4, kBuf = kA + kB;
  __shared__ __attribute__((aligned(16))) char smem[2 * kBuf];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  int tm, tn;
  tile_coords((g.M + BM - 1) / BM, (g.N + BN - 1) / BN, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int t = 0; t < TM; ++t)
#pragma unroll
    for (int u = 0; u < TN; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][u][r] = 0.f;

  Stage<BM, A_KC> sa;
  Stage<BN, B_KC> sb;
  const int nk = g.K / BK;
  {
    int kl;
    const float* A = seg_base(g, true, 0, kl);
    sa.load(A, g.lda, m0, g.M, kl, tid);
    const float* B = seg_base(g, false, 0, kl);
    sb.load(B, g.ldb, n0, g.N, kl, tid);
  }
  sa.store(smem, tid);
  sb.store(smem + kA, tid);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const char* cur = smem + (kt & 1) * kBuf;
    // Next tile's loads, unconditionally (the last iteration reloads its own
    // tile into the idle buffer): staging registers written under a branch
    // are demoted to scratch by the compiler.
    {
      const int kn = min(kt + 1, nk - 1) * BK;
      int kl;
      const float* A = seg_base(g, true, kn, kl);
      sa.load(A, g.lda, m0, g.M, kl, tid);
      const float* B = seg_base(g, false, kn, kl);
      sb.load(B, g.ldb, n0, g.N, kl, tid);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float4 af[TM], bf[TN];
#pragma unroll
      for (int t = 0; t < TM; ++t) af[t] = frag4<BM, A_KC>(cur, wm * 32 * TM + 32 * t, q, lane);
#pragma unroll
      for (int u = 0; u < TN; ++u) bf[u] = frag4<BN, B_KC>(cur + kA, wn * 32 * TN + 32 * u, q, lane);
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int t = 0; t < TM; ++t)
#pragma unroll
          for (int u = 0; u < TN; ++u)
            acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4(af[t], e), f4(bf[u], e), acc[t][u], 0, 0, 0);
    }
    char* nxt = smem + ((kt + 1) & 1) * kBuf;
    sa.store(nxt, tid);
    sb.store(nxt + kA, tid);
    __syncthreads();
  }

  // ---- epilogue: acc[t][u] register r holds (row (r&3) + 8(r>>2) + 4h, col lane&31) ----
  const int h = lane >> 5, cl = lane & 31;
  const float pscale = g.p > 0.f ? 1.f / (1.f - g.p) : 1.f;
  float* C = reinterpret_cast<float*>(g.C);
#pragma unroll
  for (int t = 0; t < TM; ++t) {
#pragma unroll
    for (int u = 0; u < TN; ++u) {
      const int col = n0 + wn * 32 * TN + 32 * u + cl;
      const bool col_ok = col < g.N;
      const float b = (EPI == kEpiStoreAct && g.bias != nullptr && col_ok)
                          ? reinterpret_cast<const float*>(g.bias)[col] : 0.f;
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int row0 = m0 + wm * 32 * TM + 32 * t + 8 * gq + 4 * h;
        if (EPI == kEpiStoreAct) {
          uint32_t ws[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
          if (g.p > 0.f) {
            // column-quad mask layout: subsequence (row/4) * N + col, word row & 3
            const uint64_t sub = (uint64_t)(row0 >> 2) * (uint64_t)g.N + (uint64_t)col;
            const uint4 w = Philox(g.seed, sub, g.offset).next4();
            ws[0] = w.x; ws[1] = w.y; ws[2] = w.z; ws[3] = w.w;
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = row0 + r;
            const float pre = acc[t][u][4 * gq + r] + b;
            float out = ACT == kActRelu ? fmaxf(pre, 0.f) : (ACT == kActGelu ? gelu_f(pre) : pre);
            if (g.p > 0.f) out = ws[r] >= g.threshold ? out * pscale : 0.f;
            if (col_ok && row < g.M) {
              const int64_t o = (int64_t)row * g.ldc + col;
              if (g.res != nullptr) out += reinterpret_cast<const float*>(g.res)[o];
              C[o] = out;
              if (g.aux != nullptr) reinterpret_cast<float*>(g.aux)[o] = pre;
            }
          }
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = row0 + r;
            if (col_ok && row < g.M) {
              float* p = C + (int64_t)row * g.ldc + col;
              if (EPI == kEpiAccumF32) *p += acc[t][u][4 * gq + r];
              else *p = acc[t][u][4 * gq + r];
            }
          }
        }
      }
    }
  }
}

template <int TM, int TN>
int tiles(const GemmArgs& g) {
  return ((g.M + 64 * TM - 1) / (64 * TM)) * ((g.N + 64 * TN - 1) / (64 * TN));
}

template <int TM, int TN, bool A_KC, bool B_KC, int EPI, int ACT>
void launch_tile(const GemmArgs& g, hipStream_t s) {
  hipLaunchKernelGGL((gemm_f32_kernel<TM, TN, A_KC, B_KC, EPI, ACT>), dim3(tiles<TM, TN>(g)), dim3(kThreads), 0, s, g);
}

// Largest tile that still gives >= 256 workgroups (one per CU; two fit per
// CU): 128x128, then 64x128, then 64x64.
template <bool A_KC, bool B_KC, int EPI, int ACT>
void launch(const GemmArgs& g, hipStream_t s) {
  if (tiles<2, 2>(g) >= 256) launch_tile<2, 2, A_KC, B_KC, EPI, ACT>(g, s);
  else if (tiles<1, 2>(g) >= 256) launch_tile<1, 2, A_KC, B_KC, EPI, ACT>(g, s);
  else launch_tile<1, 1, A_KC, B_KC, EPI, ACT>(g, s);
}

template <bool A_KC, bool B_KC, int EPI>
void launch_act(const GemmArgs& g, hipStream_t s) {
  if constexpr (EPI != kEpiStoreAct) {
    launch<A_KC, B_KC, EPI, kActNone>(g, s);
    return;
  }
  switch (g.act) {
    case kActRelu: launch<A_KC, B_KC, EPI, kActRelu>(g, s); break;
    case kActGelu: launch<A_KC, B_KC, EPI, kActGelu>(g, s); break;
    default: launch<A_KC, B_KC, EPI, kActNone>(g, s); break;
  }
}

template <int EPI>
void launch_layout(const GemmArgs& g, hipStream_t s) {
  if (g.a_kc && g.b_kc) launch_act<true, true, EPI>(g, s);
  else if (g.a_kc && !g.b_kc) launch_act<true, false, EPI>(g, s);
  else if (!g.a_kc && !g.b_kc) launch_act<false, false, EPI>(g, s);
  else launch_act<false, true, EPI>(g, s);
}

}  // namespace

bool gemm_f32_supported(int64_t M, int64_t N, int64_t K) {
  return M >= 4 && N >= 4 && K > 0 && M % 4 == 0 && N % 4 == 0 && K % BK == 0 && M < (1LL << 30) &&
         N < (1LL << 30) && K < (1LL << 30);
}

void gemm_f32(const GemmArgs& gi, hipStream_t s) {
  GemmArgs g = gi;
  g.threshold = dropout_threshold(g.p);
  if (g.epi == kEpiStoreAct) launch_layout<kEpiStoreAct>(g, s);
  else if (g.epi == kEpiAccumF32) launch_layout<kEpiAccumF32>(g, s);
  else launch_layout<kEpiStoreF32>(g, s);
}

}  // namespace mipipe
