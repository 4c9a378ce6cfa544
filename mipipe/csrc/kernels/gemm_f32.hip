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
// * 8 waves per block, each TM x TN tiles of 32x32: 128x128 blocks (waves of
//   32x64) for grids that fill the chip, 64x128 / 128x64 blocks (waves of
//   32x32) for the T = 1024 shapes of the reference config; BK = 32, two LDS
//   buffers, and two sets of staging registers, so a K-tile's global loads
//   (16-byte float4s) are issued two K-tiles before they are needed;
//   fragments are read one k-quad ahead of the MFMAs.
// * The MFMA sums over k, so k may be permuted inside a K-tile as long as A
//   and B agree: in k-step s lane half h (= lane >> 5) uses physical k =
//   16h + 4(s >> 2) + (s & 3).  Then a K-contiguous operand hands each lane 4
//   consecutive k-steps in ONE ds_read_b128 (row-pair XOR swizzle: the 16
//   lanes of a read phase hit 16 distinct 16-byte bank groups), and an
//   I-contiguous operand is one ds_read_b32 per step whose two lane halves
//   (rows k and k + 16) are 128 bytes apart after an XOR of the chunk index
//   (all 64 banks distinct).
// * Two or three blocks per CU (LDS 48-64 KiB each): while one block waits
//   at its barrier the others' MFMAs run.
// * Epilogues as gemm.hip: bias + ReLU/GELU + dropout (same Philox
//   column-quad mask layout as the elementwise backward) + residual addend +
//   pre-activation aux output, all fp32; fp32 += (weight gradients into
//   main_grad, K-segmented for deferred wgrad); fp32 store.
// The operand layouts are the bf16 kernel's: forward (KC, KC), dgrad (KC, IC),
// wgrad (IC, IC).  M, N multiples of 4, K a multiple of 32.
#include "common.h"
#include "kernels.h"

#include <stdlib.h>

namespace mipipe {

namespace {

constexpr int BK = 32;

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

// Register staging of one operand tile (ROWS x 32 of the operand's M or N rows)
// by NT threads.
template <int ROWS, bool KC, int NT>
struct Stage {
  static constexpr int kN = ROWS * BK / 4 / NT;  // float4s per thread
  static_assert(kN >= 1 && ROWS * BK / 4 % NT == 0, "tile / thread count mismatch");
  f32x4 v[kN];  // native vector type: HIP's float4 struct copies become memcpys that pin the array in scratch
  __device__ __forceinline__ void load(const float* base, int64_t ld, int i0, int lim, int k0, int tid) {
#pragma unroll
    for (int u = 0; u < kN; ++u) {
      const int id = tid + u * NT;
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
      const int id = tid + u * NT;
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
__device__ __forceinline__ f32x4 frag4(const char* tile, int ib, int q, int lane) {
  const int i = ib + (lane & 31), h = lane >> 5;
  if (KC) return *reinterpret_cast<const f32x4*>(tile + kc_off(i, 4 * h + q));
  f32x4 r;
  const int k0 = 16 * h + 4 * q;
  const int c = i >> 2, w = (i & 3) * 4;
#pragma unroll
  for (int e = 0; e < 4; ++e) r[e] = *reinterpret_cast<const float*>(tile + ic_off<ROWS>(k0 + e, c) + w);
  return r;
}

// WM x WN waves, each TM x TN tiles of 32x32: block tile (32 WM TM) x (32 WN TN).
template <int WM, int WN, int TM, int TN>
struct Cfg {
  static constexpr int kWaves = WM * WN, kThreads = 64 * WM * WN;
  static constexpr int BM = 32 * WM * TM, BN = 32 * WN * TN;
  static constexpr int kLds = 2 * (BM + BN) * BK * 4;
  // blocks per CU the LDS admits (160 KiB), capped by 8 waves per SIMD
  static constexpr int kBlocksPerCu = (160 * 1024 / kLds) < (32 / kWaves) ? (160 * 1024 / kLds) : (32 / kWaves);
};

template <int WM, int WN, int TM, int TN, bool A_KC, bool B_KC, int EPI, int ACT>
__global__ void __launch_bounds__(64 * WM * WN, (Cfg<WM, WN, TM, TN>::kBlocksPerCu)) gemm_f32_kernel(GemmArgs g) {
  using C_ = Cfg<WM, WN, TM, TN>;
  constexpr int NT = C_::kThreads, BM = C_::BM, BN = C_::BN;
  constexpr int kA = BM * BK * 4, kB = BN * BK * 4, kBuf = kA + kB;
  __shared__ __attribute__((aligned(16))) char smem[2 * kBuf];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;

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

  // Two register staging sets: the global loads of tile kt+2 are issued
  // while tile kt computes and tile kt+1 waits in registers, so a load has
  // two K-tiles of MFMA time (>= 4000 cycles) to return from L2 / MALL.
  Stage<BM, A_KC, NT> sa0, sa1;
  Stage<BN, B_KC, NT> sb0, sb1;
  const int nk = g.K / BK;
  auto gload = [&](int kt, Stage<BM, A_KC, NT>& sa, Stage<BN, B_KC, NT>& sb) {
    const int kn = min(kt, nk - 1) * BK;  // clamped: past the end reloads the last tile (unused)
    int kl;
    const float* A = seg_base(g, true, kn, kl);
    sa.load(A, g.lda, m0, g.M, kl, tid);
    const float* B = seg_base(g, false, kn, kl);
    sb.load(B, g.ldb, n0, g.N, kl, tid);
  };
  auto compute = [&](const char* cur) {
    // Fragments one k-quad ahead: the reads of quad q+1 are in flight while
    // the MFMAs of quad q issue.
    f32x4 af[2][TM], bf[2][TN];
#pragma unroll
    for (int t = 0; t < TM; ++t) af[0][t] = frag4<BM, A_KC>(cur, (wm * TM + t) * 32, 0, lane);
#pragma unroll
    for (int u = 0; u < TN; ++u) bf[0][u] = frag4<BN, B_KC>(cur + kA, (wn * TN + u) * 32, 0, lane);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int cq = q & 1;
      if (q < 3) {
#pragma unroll
        for (int t = 0; t < TM; ++t) af[cq ^ 1][t] = frag4<BM, A_KC>(cur, (wm * TM + t) * 32, q + 1, lane);
#pragma unroll
        for (int u = 0; u < TN; ++u) bf[cq ^ 1][u] = frag4<BN, B_KC>(cur + kA, (wn * TN + u) * 32, q + 1, lane);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int t = 0; t < TM; ++t)
#pragma unroll
          for (int u = 0; u < TN; ++u)
            acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[cq][t][e], bf[cq][u][e], acc[t][u], 0, 0, 0);
    }
  };
  gload(0, sa0, sb0);
  gload(1, sa1, sb1);
  sa0.store(smem, tid);
  sb0.store(smem + kA, tid);
  __syncthreads();
  for (int kt = 0; kt < nk; kt += 2) {
    // even tile kt in buffer 0, tile kt+1 in registers set 1
    gload(kt + 2, sa0, sb0);
    compute(smem);
    sa1.store(smem + kBuf, tid);
    sb1.store(smem + kBuf + kA, tid);
    __syncthreads();
    if (kt + 1 >= nk) break;
    // odd tile kt+1 in buffer 1, tile kt+2 in registers set 0
    gload(kt + 3, sa1, sb1);
    compute(smem + kBuf);
    sa0.store(smem, tid);
    sb0.store(smem + kA, tid);
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
      const int col = n0 + (wn * TN + u) * 32 + cl;
      const bool col_ok = col < g.N;
      const float b = (EPI == kEpiStoreAct && g.bias != nullptr && col_ok)
                          ? reinterpret_cast<const float*>(g.bias)[col] : 0.f;
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int row0 = m0 + (wm * TM + t) * 32 + 8 * gq + 4 * h;
        if (EPI == kEpiStoreAct) {
          uint32_t ws[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
          if (g.p > 0.f) {
            // the dropout layout (common.h drop_sub): word row & 3, half col & 1
            const uint4 w = Philox(g.seed, drop_sub(row0, col, g.N), g.offset).next4();
            ws[0] = w.x; ws[1] = w.y; ws[2] = w.z; ws[3] = w.w;
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = row0 + r;
            const float pre = acc[t][u][4 * gq + r] + b;
            float out = ACT == kActRelu ? fmaxf(pre, 0.f) : (ACT == kActGelu ? gelu_f(pre) : pre);
            if (g.p > 0.f) out = drop_keep(ws[r], col & 1, g.threshold >> 16) ? out * pscale : 0.f;
            if (col_ok && row < g.M) {
              const int64_t o = (int64_t)row * g.ldc + col;
              if (g.res != nullptr) out += reinterpret_cast<const float*>(g.res)[(int64_t)row * g.ldr + col];
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

template <int WM, int WN, int TM, int TN>
int tiles(const GemmArgs& g) {
  using C_ = Cfg<WM, WN, TM, TN>;
  return ((g.M + C_::BM - 1) / C_::BM) * ((g.N + C_::BN - 1) / C_::BN);
}

// Share of the CU slots (256 CUs x resident blocks) the grid keeps busy over
// its whole run: a grid of 384 tiles on 512 slots leaves a quarter idle.
template <int WM, int WN, int TM, int TN>
double fill(const GemmArgs& g) {
  const int slots = 256 * Cfg<WM, WN, TM, TN>::kBlocksPerCu;
  const int t = tiles<WM, WN, TM, TN>(g);
  const int rounds = (t + slots - 1) / slots;
  return (double)t / ((double)rounds * slots);
}

template <int WM, int WN, int TM, int TN, bool A_KC, bool B_KC, int EPI, int ACT>
void launch_cfg(const GemmArgs& g, hipStream_t s) {
  hipLaunchKernelGGL((gemm_f32_kernel<WM, WN, TM, TN, A_KC, B_KC, EPI, ACT>), dim3(tiles<WM, WN, TM, TN>(g)),
                     dim3(64 * WM * WN), 0, s, g);
}

// MIPIPE_GEMM_F32_CFG: 0 auto; 1: 128x128 (4 waves, 2x2 tiles each); 2: 64x128
// (8 waves, 1 tile each); 3: 128x64 (8 waves); 4: 64x128 (4 waves, 1x2 tiles);
// 5: 128x128 (8 waves, 1x2 tiles); 6: 128x128 (8 waves, 2x1); 7: 256x128 and
// 8: 128x256 (8 waves, 2x2 tiles).
int g_f32_cfg = -1;

int f32_cfg() {
  if (g_f32_cfg < 0) {
    const char* e = getenv("MIPIPE_GEMM_F32_CFG");
    g_f32_cfg = e ? atoi(e) : 0;
  }
  return g_f32_cfg;
}

template <bool A_KC, bool B_KC, int EPI, int ACT>
void launch(const GemmArgs& g, hipStream_t s) {
  int c = f32_cfg();
  if (c == 0) {
    // the big tile when it fills the machine as well as the small ones (fewer
    // operand bytes per FLOP), else the best-filling 64-row / 64-column tile
    // (profiles/gemm_f32_vs_hipblaslt.txt: 128x128 with 8 waves of 32x64 is the
    // best big tile; 64x128 / 128x64 with 8 waves of 32x32 the best small ones)
    const double f5 = fill<4, 2, 1, 2>(g), f2 = fill<2, 4, 1, 1>(g), f3 = fill<4, 2, 1, 1>(g);
    if (f5 >= 0.95 * f2 && f5 >= 0.95 * f3) c = 5;
    else c = f2 >= f3 ? 2 : 3;
  }
  switch (c) {
    case 2: launch_cfg<2, 4, 1, 1, A_KC, B_KC, EPI, ACT>(g, s); break;
    case 3: launch_cfg<4, 2, 1, 1, A_KC, B_KC, EPI, ACT>(g, s); break;
    case 4: launch_cfg<2, 2, 1, 2, A_KC, B_KC, EPI, ACT>(g, s); break;
    case 5: launch_cfg<4, 2, 1, 2, A_KC, B_KC, EPI, ACT>(g, s); break;
    case 6: launch_cfg<2, 4, 2, 1, A_KC, B_KC, EPI, ACT>(g, s); break;
    case 7: launch_cfg<4, 2, 2, 2, A_KC, B_KC, EPI, ACT>(g, s); break;
    case 8: launch_cfg<2, 4, 2, 2, A_KC, B_KC, EPI, ACT>(g, s); break;
    default: launch_cfg<2, 2, 2, 2, A_KC, B_KC, EPI, ACT>(g, s); break;
  }
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
  if (g.ldr == 0) g.ldr = g.ldc;
  if (g.epi == kEpiStoreAct) launch_layout<kEpiStoreAct>(g, s);
  else if (g.epi == kEpiAccumF32) launch_layout<kEpiAccumF32>(g, s);
  else launch_layout<kEpiStoreF32>(g, s);
}

}  // namespace mipipe
