// bf16 MFMA GEMM for gfx950 with fused epilogues.
//
//   C[M, N] = A[M, K] . B[K, N]      (bf16 operands, fp32 accumulation)
//
// Every Transformer linear runs on this one kernel template, in three
// operand layouts:
//   forward  Y  = X  . W^T   A = X  [T, K] (K-contiguous)  B = W  [N, K] (K-contiguous)
//   dgrad    dX = dY . W     A = dY [T, N] (K-contiguous)  B = W  [N, K] read as [K, N] (N-contiguous)
//   wgrad    dW += dY^T . X  A = dY read as [K=T, M] (M-contiguous), B = X [K=T, N] (N-contiguous)
// Operand tiles are staged into LDS in their memory layout (16-byte loads,
// coalesced); K-contiguous fragments are read with ds_read_b128 and K-strided
// ones with the gfx950 transposing read ds_read_b64_tr_b16, so no layout ever
// needs a transpose pass in HBM.  Both LDS images are XOR-swizzled so the
// lane groups of a read hit distinct banks (T2/T10).
//
// Main kernel (big::gemm256_kernel): 256x256x64 block tile, 8 waves (2 M x 4 N,
// 128x64 per wave as 8x4 v_mfma_f32_16x16x32_bf16 tiles), operand tiles staged
// by LDS-DMA (global_load_lds_dwordx4, SADDR form with loop-invariant per-lane
// offsets) into two 64 KiB buffers, and either a ping-pong main loop (the two
// wave groups one barrier interval apart: one group's 16-MFMA cluster runs
// while the other reads its fragments) or one barrier per K-tile.  Edge tiles
// (M, N any multiple of 8) are clamped on load and masked on store; K may be
// split into segments living in different buffers (deferred weight gradients).
// Block ids are remapped so consecutive tiles of an 8-row group share an XCD's
// L2 (T1, bijective form).  Grids that would leave CUs idle get a 256x128 block
// (big_width) or, with a long K, split-K: 2-8 blocks per tile writing fp32
// partials that one reduction adds (gemm_splitk_factor).  A 128x128
// register-staged kernel serves small exact-multiple grids.
// Epilogues (all results leave through LDS as 16-byte row stores, staged_store):
//   kEpiStoreBf16 -- + bias, activation (ReLU/GELU), dropout (Philox mask in
//                    the "column-quad" layout shared with the elementwise
//                    backward), optional pre-activation aux output, optional
//                    bf16 addend `res` (a fan-out's other gradient: the
//                    autograd add kernel folded into the dgrad), bf16 store;
//   kEpiAccumF32  -- C(fp32) += acc  (weight gradients straight into main_grad);
//   kEpiStoreF32  -- fp32 store (first write of a step, split-K partials).
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace mipipe {

namespace {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int kThreads = 256;
constexpr int kTileBytes = BM * BK * 2;  // 16 KiB per operand tile (BM == BN)
constexpr int kBufBytes = 2 * kTileBytes;  // A + B
constexpr int kSmemBytes = 2 * kBufBytes;  // double buffered = 64 KiB

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// ---- LDS images --------------------------------------------------------------
// K-contiguous tile [128 rows (i)][64 k]: 128-byte rows, 16-byte chunk c of
// row r stored at chunk c ^ ((r >> 1) & 7).
__device__ __forceinline__ int kc_off(int r, int c16) { return r * 128 + ((c16 ^ ((r >> 1) & 7)) << 4); }

// I-contiguous tile [64 rows (k)][128 i]: 256-byte rows, 8-byte chunk c of row
// r stored at chunk c ^ (4 * rk(r)), rk(r) = (r & 3) | (((r >> 3) & 1) << 2).
__device__ __forceinline__ int ic_rk(int r) { return (r & 3) | (((r >> 3) & 1) << 2); }
__device__ __forceinline__ int ic_off(int r, int c8) { return r * 256 + ((c8 ^ (ic_rk(r) << 2)) << 3); }

// ---- global -> registers -> LDS staging ------------------------------------------
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

template <bool KC>
struct Stager {
  u32x4 v[4];  // native vector: HIP's uint4 struct copies become memcpys that pin the array in scratch
  // Loads the tile whose first element is (i0, k0) of an operand of leading
  // dimension ld.
  __device__ __forceinline__ void load(const bf16_t* __restrict__ base, int64_t ld, int i0, int k0, int tid) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int id = tid + u * kThreads;
      const bf16_t* p;
      if (KC) {
        const int r = id >> 3, c = id & 7;
        p = base + (int64_t)(i0 + r) * ld + k0 + c * 8;
      } else {
        const int r = id >> 4, c = id & 15;
        p = base + (int64_t)(k0 + r) * ld + i0 + c * 8;
      }
      v[u] = *reinterpret_cast<const u32x4*>(p);
    }
  }
  __device__ __forceinline__ void store(char* tile, int tid) const {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int id = tid + u * kThreads;
      int off;
      if (KC) {
        off = kc_off(id >> 3, id & 7);
      } else {
        off = ic_off(id >> 4, (id & 15) * 2);
      }
      *reinterpret_cast<u32x4*>(tile + off) = v[u];
    }
  }
};

// ---- LDS -> fragment ---------------------------------------------------------------
// Fragment of the 16x16x32 operand for rows/cols [ib, ib+16) and k-step s:
// lane l holds element (i = ib + (l & 15), k = 32 s + 8 (l >> 4) + j), j = 0..7.
template <bool KC>
__device__ __forceinline__ bf16x8 read_frag(const char* tile, int ib, int s, int lane) {
  if (KC) {
    const int r = ib + (lane & 15);
    const int c = 4 * s + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(tile + kc_off(r, c));
  } else {
    const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
    const int r0 = 32 * s + 8 * g + q;
    const int c8 = (ib >> 2) + p;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(tile + ic_off(r0, c8)));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(tile + ic_off(r0 + 4, c8)));
    const s16x8 both = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, both);
  }
}

// act'(s) for the activation-backward epilogue (GemmArgs::dact): ReLU's from its
// output, GELU's from the pre-activation, or s itself (kActSavedGrad: the forward
// stored GELU'(pre) -- one multiply, like ReLU's sign test).
__device__ __forceinline__ float dact_f(int dact, float s) {
  return dact == kActRelu ? (s > 0.f ? 1.f : 0.f) : (dact == kActSavedGrad ? s : gelu_grad_f(s));
}

// Bijective XCD-aware remap + grouped (8 tile-rows) ordering.
__device__ __forceinline__ void tile_coords(int tiles_m, int tiles_n, int& tm, int& tn, int G = 8) {
  const int nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  int wg = bid;
  if (nwg > 8) {
    const int xcd = bid & 7, local = bid >> 3;
    const int q = nwg >> 3, r = nwg & 7;
    wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + local;
  }
  const int group = wg / (G * tiles_n);
  const int first_m = group * G;
  const int gsize = min(tiles_m - first_m, G);
  const int in_group = wg % (G * tiles_n);
  tm = first_m + in_group % gsize;
  tn = in_group / gsize;
}

template <bool A_KC, bool B_KC, int EPI, int ACT>
__global__ void __launch_bounds__(kThreads) gemm_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  int tm, tn;
  tile_coords(g.M / BM, g.N / BN, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;

  const bf16_t* A = reinterpret_cast<const bf16_t*>(g.A);
  const bf16_t* B = reinterpret_cast<const bf16_t*>(g.B);

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  Stager<A_KC> sa;
  Stager<B_KC> sb;
  const int nk = g.K / BK;

  sa.load(A, g.lda, m0, 0, tid);
  sb.load(B, g.ldb, n0, 0, tid);
  sa.store(smem, tid);
  sb.store(smem + kTileBytes, tid);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    char* cur = smem + (kt & 1) * kBufBytes;
    const bool more = kt + 1 < nk;
    if (more) {
      sa.load(A, g.lda, m0, (kt + 1) * BK, tid);
      sb.load(B, g.ldb, n0, (kt + 1) * BK, tid);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) af[t] = read_frag<A_KC>(cur, wm * 64 + 16 * t, s, lane);
#pragma unroll
      for (int t = 0; t < 4; ++t) bfr[t] = read_frag<B_KC>(cur + kTileBytes, wn * 64 + 16 * t, s, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      char* nxt = smem + ((kt + 1) & 1) * kBufBytes;
      sa.store(nxt, tid);
      sb.store(nxt + kTileBytes, tid);
    }
    __syncthreads();
  }

  // ---- epilogue ----
  const int quad = lane >> 4, col_in = lane & 15;
  const float pscale = g.p > 0.f ? 1.f / (1.f - g.p) : 1.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row0 = m0 + wm * 64 + 16 * i + 4 * quad;  // rows row0 .. row0+3
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = n0 + wn * 64 + 16 * j + col_in;
      f32x4 v = acc[i][j];
      if (EPI == kEpiAccumF32) {
        float* C = reinterpret_cast<float*>(g.C);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float* p = C + (int64_t)(row0 + r) * g.ldc + col;
          *p += v[r];
        }
      } else if (EPI == kEpiStoreF32) {
        float* C = reinterpret_cast<float*>(g.C);
#pragma unroll
        for (int r = 0; r < 4; ++r) C[(int64_t)(row0 + r) * g.ldc + col] = v[r];
      } else {
        bf16_t* C = reinterpret_cast<bf16_t*>(g.C);
        const float b = g.bias != nullptr ? bf2f(reinterpret_cast<const bf16_t*>(g.bias)[col]) : 0.f;
        float pre[4], out[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          pre[r] = v[r] + b;
          out[r] = ACT == kActRelu ? fmaxf(pre[r], 0.f) : (ACT == kActGelu ? gelu_f(pre[r]) : pre[r]);
        }
        if (g.p > 0.f) {
          // the dropout layout (common.h drop_sub): word row & 3, half col & 1
          const uint4 w = Philox(g.seed, drop_sub(row0, col, g.N), g.offset).next4();
          const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
          for (int r = 0; r < 4; ++r) out[r] = drop_keep(ws[r], col & 1, g.threshold >> 16) ? out[r] * pscale : 0.f;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (g.dact_in != nullptr && g.dact == kActReluBits)
            out[r] *= (reinterpret_cast<const uint8_t*>(g.dact_in)[(int64_t)(row0 + r) * g.ldd + (col >> 3)] >> (col & 7)) & 1
                          ? g.dact_scale : 0.f;
          else if (g.dact_in != nullptr)
            out[r] *= g.dact_scale *
                      dact_f(g.dact, bf2f(reinterpret_cast<const bf16_t*>(g.dact_in)[(int64_t)(row0 + r) * g.ldd + col]));
          if (g.res != nullptr) out[r] += bf2f(reinterpret_cast<const bf16_t*>(g.res)[(int64_t)(row0 + r) * g.ldr + col]);
          C[(int64_t)(row0 + r) * g.ldc + col] = f2bf(out[r]);
          if (g.aux != nullptr)
            reinterpret_cast<bf16_t*>(g.aux)[(int64_t)(row0 + r) * g.ldc + col] =
                f2bf(g.aux_grad ? gelu_grad_f(pre[r]) : pre[r]);
        }
      }
    }
  }
}

// ============================================================================
// Large-tile variant: 256x256x64, 8 waves (2 M x 4 N, 128x64 per wave as 8x4
// MFMA tiles), operand tiles staged by LDS-DMA (global_load_lds_dwordx4: no
// VGPR round trip, no ds_write), two 64 KiB LDS buffers, one barrier per K-tile.
// LDS images are lane-linear per wave-instruction (1 KiB), so the bank swizzle
// is applied to the per-lane *source* address and undone on the read (rule 21).
namespace big {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int kThreads = 512;
constexpr int kTileBytes = BM * BK * 2;      // 32 KiB per operand tile
constexpr int kSmemBytes = 128 * 260 * 4;    // 130 KiB: 2 x 64 KiB operand buffers, reused by the epilogue

// The PP == 4 loop keeps an I-contiguous B operand in THREE buffers (A in two;
// see the loop): 2 (A + B) + B = 160 KiB at W = 256, all of the CU's LDS.
template <bool B_KC, int PP, int W>
constexpr int smem_bytes() {
  constexpr int b3 = 2 * (kTileBytes + W * BK * 2) + W * BK * 2;
  return PP == 4 && !B_KC && b3 > kSmemBytes ? b3 : kSmemBytes;
}

// I-contiguous image with 2W-byte rows (W = 256 or 128 i values; the B tile of
// the 256x128 variant is 128 wide).
template <int W>
__device__ __forceinline__ int ic_off_w(int r, int c8) { return r * (2 * W) + ((c8 ^ (ic_rk(r) << 2)) << 3); }

// LDS-DMA staging (global_load_lds_dwordx4: 16 bytes per lane, lane-linear
// 1 KiB per wave-instruction; the bank swizzle is applied to the per-lane
// SOURCE address).
//
// Loop-invariant per-lane byte offsets of the W/64 pieces a wave stages per
// W-wide operand tile; the K position lives in the scalar base, so each LDS-DMA is
// issued in SADDR form (SGPR base + 32-bit VGPR offset) with no per-tile
// address arithmetic.  gemm_supported() keeps rows * ld * 2 bytes < 4 GiB.
// Edge tiles: i indices past `lim` (M for A, N for B) are clamped onto the last
// valid row / 8-column chunk, so every DMA reads mapped memory; the garbage
// they produce lands only in accumulator rows/columns the epilogue masks off.
template <bool KC, int W>
__device__ __forceinline__ void stage_offsets(int64_t ld, int i0, int lim, int wave, int lane, uint32_t (&off)[W / 64]) {
  constexpr int NU = W / 64, LPR = W / 8;  // DMAs per wave; 16-byte chunks per I-contiguous row
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int inst = wave * NU + u;
    if (KC) {
      const int row = 8 * inst + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      const int gi = min(i0 + row, lim - 1);
      off[u] = (uint32_t)(((int64_t)gi * ld + 8 * c) * 2);
    } else {
      const int row = (64 / LPR) * inst + lane / LPR;
      const int c16 = (lane % LPR) ^ (ic_rk(row) << 1);
      const int gi = min(i0 + 8 * c16, lim - 8);
      off[u] = (uint32_t)(((int64_t)row * ld + gi) * 2);
    }
  }
}

// The I-contiguous A tile of the PP == 4 loop is kept as two 128-wide halves
// (i 0-127, then 128-255; 16 KiB each, the W = 128 image), so each half is read
// by one wave group only.  Share s (0-7) stages rows 16 (s & 3) .. +16 of half
// s >> 2 -- the same LDS pieces stage_fast gives share s (4 KiB at 4 s KiB).
__device__ __forceinline__ void stage_offsets_halves(int64_t ld, int i0, int lim, int share, int lane,
                                                     uint32_t (&off)[4]) {
  const int half = share >> 2;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int row = 4 * (4 * (share & 3) + u) + (lane >> 4);
    const int c16 = (lane & 15) ^ (ic_rk(row) << 1);
    const int gi = min(i0 + 128 * half + 8 * c16, lim - 8);
    off[u] = (uint32_t)(((int64_t)row * ld + gi) * 2);
  }
}

// Issued from inline asm on purpose: the compiler cannot prove that a DMA into
// one LDS buffer does not alias the ds_reads of the other, and after a
// __builtin_amdgcn_global_load_lds it inserts s_waitcnt vmcnt(0) before EVERY
// following ds_read -- each phase would wait for the next tile's DMA to land.
// Hidden from the waitcnt pass, the DMA is ordered only by the kernel's own
// counted waits (vmcnt before the barrier that precedes the read).
__device__ __forceinline__ void glds16_saddr(const char* base, uint32_t off, const char* lds_dst) {
  const uint32_t m0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) const char*)lds_dst);
  asm volatile(
      "s_mov_b32 m0, %0\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %2"
      :
      : "s"(m0), "v"(off), "s"(base)
      : "memory", "m0");
}

// s_waitcnt vmcnt(N): all but the N most recently issued vector-memory ops done.
template <int N>
__device__ __forceinline__ void vmcnt_keep() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <bool KC, int W>
__device__ __forceinline__ void stage_fast(const bf16_t* base, int64_t ld, int k0, const uint32_t (&off)[W / 64],
                                           char* tile, int wave) {
  constexpr int NU = W / 64;
  const char* b = reinterpret_cast<const char*>(base) + (KC ? (int64_t)k0 * 2 : (int64_t)k0 * ld * 2);
#pragma unroll
  for (int u = 0; u < NU; ++u) glds16_saddr(b, off[u], tile + (wave * NU + u) * 1024);
}

// Operand base and local k of K-tile k0 (K-segmented operands, GemmArgs::seg_k).
__device__ __forceinline__ const bf16_t* seg_base(const GemmArgs& g, bool is_a, int k0, int& kl) {
  if (g.seg_k == 0) {
    kl = k0;
    return reinterpret_cast<const bf16_t*>(is_a ? g.A : g.B);
  }
  const int s = k0 / g.seg_k;
  kl = k0 - s * g.seg_k;
  return reinterpret_cast<const bf16_t*>(is_a ? g.a_seg[s] : g.b_seg[s]);
}

template <bool KC, int W>
__device__ __forceinline__ bf16x8 frag(const char* tile, int ib, int s, int lane) {
  if (KC) {
    const int r = ib + (lane & 15);
    const int c = 4 * s + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(tile + kc_off(r, c));
  } else {
    const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
    const int r0 = 32 * s + 8 * g + q;
    const int c8 = (ib >> 2) + p;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(tile + ic_off_w<W>(r0, c8)));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(tile + ic_off_w<W>(r0 + 4, c8)));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  }
}

// Epilogue parameters as plain values, read from the kernel arguments once
// (through a GemmArgs reference the fields were re-loaded -- an s_load plus
// its wait -- after every store that might alias them).
struct EpiParams {
  uint64_t seed, offset;
  int N;
  float p, pscale;
  uint32_t threshold;
  int mask_row0, mask_col0, mask_ld;  // launch chunk -> full-matrix mask coordinates
};

// Register-phase bf16 epilogue of accumulator row block i (16 rows x 16 NJ
// cols of the wave's tile): bias, activation, dropout, in place.  One instantiation per i: as a loop, the Philox-heavy body is not
// unrolled and a runtime i demotes the whole accumulator array to scratch.
// Predicated throughout (no continue/break, for the same reason).
// EXTRA = false: bias + activation only (no dropout) -- straight-line code;
// with the dropout and aux-store branches merely present, the compiler's
// per-element control flow cost ~5 us per 256x256 tile round (K = 64 sweep).
template <int I, int ACT, int NJ, bool EXTRA>
__device__ __forceinline__ void epi_rows(const EpiParams ep, f32x4 (&acc)[8][NJ], int nrow, int ncol,
                                         const float (&bias)[NJ]) {
  if constexpr (!EXTRA) {
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float pre = acc[I][j][r] + bias[j];
        acc[I][j][r] = ACT == kActRelu ? fmaxf(pre, 0.f) : (ACT == kActGelu ? gelu_f(pre) : pre);
      }
    return;
  }
  const int row0 = nrow + 16 * I;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int col = ncol + 16 * j;
    const float b = bias[j];
    uint32_t ws[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    if (ep.p > 0.f) {
      const uint4 w = Philox(ep.seed, drop_sub(row0 + ep.mask_row0, col + ep.mask_col0, ep.mask_ld), ep.offset).next4();
      ws[0] = w.x; ws[1] = w.y; ws[2] = w.z; ws[3] = w.w;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float pre = acc[I][j][r] + b;
      float out = ACT == kActRelu ? fmaxf(pre, 0.f) : (ACT == kActGelu ? gelu_f(pre) : pre);
      if (ep.p > 0.f) out = drop_keep(ws[r], (col + ep.mask_col0) & 1, ep.threshold >> 16) ? out * ep.pscale : 0.f;
      acc[I][j][r] = out;
    }
  }
}

// Writes the block's result through LDS (two halves: waves wm = 0, then 1):
// each wave spills its 128 x W/4 accumulator tile into a [128][W+4] fp32
// image (the 4-float row pad keeps the scattered 4-byte writes conflict-free),
// then all 512 threads stream whole rows out with 16-byte accesses -- 8 bf16
// per store (+ the bf16 addend `res`, read as 16-byte row chunks), fp32
// read-modify-write (kEpiAccumF32) or fp32 stores.  Starts with the LDS free,
// ends with a barrier (so it can run twice: aux, then the output).
// NJ: 16-wide accumulator tiles per wave (W / 64 for the 8-wave kernel, whose
// wave tile is 128 x W/4; 8 for the 4-wave kernel's 128 x 128), kT: threads.
// ROWSPLIT (the 4-wave kernel): pass p stages accumulator rows i = 4p..4p+3 of
// EVERY wave (all waves share the LDS writes) instead of all rows of the waves
// with wm == p; image row R is then tile row 128 (R >> 6) + 64 p + (R & 63).
template <int EPI, int W, int NJ = W / 64, int kT = 512, bool ROWSPLIT = false>
__device__ __forceinline__ void staged_store(char* smem, const f32x4 (&acc)[8][NJ], int wm, int wn, int lane,
                                             int tid, int m0, int n0, int M, int N, int64_t ldc, void* out,
                                             const bf16_t* res, int64_t ldr = 0, const bf16_t* dact_in = nullptr,
                                             int64_t ldd = 0, int dact = 0, float dact_scale = 1.f,
                                             bool trans = false, bool dgelu = false) {
  constexpr int WN = 16 * NJ, kStride = W + 4;
  const int quad = lane >> 4, col_in = lane & 15;
  float* stg = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    if (ROWSPLIT) {
#pragma unroll
      for (int ii = 0; ii < 4; ++ii)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            stg[(64 * wm + 16 * ii + 4 * quad + r) * kStride + wn * WN + 16 * j + col_in] = acc[4 * pass + ii][j][r];
    } else if (wm == pass) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            stg[(16 * i + 4 * quad + r) * kStride + wn * WN + 16 * j + col_in] = acc[i][j][r];
    }
    __syncthreads();
    const int rbase = m0 + pass * 128;
    // tile row of image row R (R's 4-row quads never straddle a 64-row block)
    auto grow = [&](int R) { return ROWSPLIT ? m0 + ((R >> 6) << 7) + 64 * pass + (R & 63) : rbase + R; };
    if (EPI == kEpiStoreBf16) {
      bf16_t* C = reinterpret_cast<bf16_t*>(out);
      constexpr int CPR = W / 8;  // 128 rows x W/8 chunks of 8 columns
#pragma unroll
      for (int u = 0; u < 128 * CPR / kT; ++u) {
        const int idx = tid + u * kT;
        const int row = idx / CPR, c8 = idx % CPR;
        if (grow(row) >= M || n0 + 8 * c8 >= N) continue;
        const f32x4 lo = *reinterpret_cast<const f32x4*>(stg + row * kStride + 8 * c8);
        const f32x4 hi = *reinterpret_cast<const f32x4*>(stg + row * kStride + 8 * c8 + 4);
        const int64_t at = (int64_t)grow(row) * ldc + n0 + 8 * c8;
        float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        if (dgelu) {  // GELU'(pre) for the backward instead of pre (GemmArgs::aux_grad)
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = gelu_grad_f(v[e]);
        }
        if (dact_in != nullptr && dact == kActReluBits) {  // the ReLU (+ dropout) mask as bits: one byte
          const uint32_t mb =
              reinterpret_cast<const uint8_t*>(dact_in)[(int64_t)grow(row) * ldd + ((n0 + 8 * c8) >> 3)];
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] *= (mb >> e) & 1 ? dact_scale : 0.f;
        } else if (dact_in != nullptr) {  // activation backward: x act'(saved)
          const bf16x8 sv = *reinterpret_cast<const bf16x8*>(dact_in + (int64_t)grow(row) * ldd + n0 + 8 * c8);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] *= dact_scale * dact_f(dact, (float)sv[e]);
        }
        if (res != nullptr) {
          const bf16x8 rv = *reinterpret_cast<const bf16x8*>(res + (int64_t)grow(row) * ldr + n0 + 8 * c8);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += (float)rv[e];
        }
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (__bf16)v[e];
        *reinterpret_cast<bf16x8*>(C + at) = o;
      }
    } else if (trans) {
      // C^T: element (row m, col n) to C[n * ldc + m].  Item (mq, n): rows
      // 4 mq .. 4 mq + 3 of column n, one 16-byte store; 8 consecutive items
      // are 8 row quads of one column (128 contiguous output bytes).
      float* C = reinterpret_cast<float*>(out);
#pragma unroll 4
      for (int u = 0; u < 32 * W / kT; ++u) {
        const int idx = tid + u * kT;
        const int mq = (idx & 7) + 8 * (idx / (8 * W)), n = (idx >> 3) % W;
        if (grow(4 * mq) >= M || n0 + n >= N) continue;
        const float* sp = stg + 4 * mq * kStride + n;
        const float4 v = make_float4(sp[0], sp[kStride], sp[2 * kStride], sp[3 * kStride]);
        float4* dst = reinterpret_cast<float4*>(C + (int64_t)(n0 + n) * ldc + grow(4 * mq));
        if (EPI == kEpiAccumF32) {
          const float4 o = *dst;
          *dst = make_float4(o.x + v.x, o.y + v.y, o.z + v.z, o.w + v.w);
        } else {
          *dst = v;
        }
      }
    } else {
      float* C = reinterpret_cast<float*>(out);
      constexpr int CPR = W / 4;  // 128 rows x W/4 chunks of 4 columns
#pragma unroll
      for (int u = 0; u < 128 * CPR / kT; ++u) {
        const int idx = tid + u * kT;
        const int row = idx / CPR, c4 = idx % CPR;
        if (grow(row) >= M || n0 + 4 * c4 >= N) continue;
        const float4 v = *reinterpret_cast<const float4*>(stg + row * kStride + 4 * c4);
        float4* dst = reinterpret_cast<float4*>(C + (int64_t)grow(row) * ldc + n0 + 4 * c4);
        if (EPI == kEpiAccumF32) {
          const float4 o = *dst;
          *dst = make_float4(o.x + v.x, o.y + v.y, o.z + v.z, o.w + v.w);
        } else {
          *dst = v;
        }
      }
    }
    __syncthreads();
  }
}

// The EXTRA epilogue (dropout and / or the aux output) in the STAGED layout:
// the pre-activation (acc + bias) goes through the LDS image once, and each
// thread then owns 4-row x 8-column blocks of it -- the 8 Philox calls of a
// block give exactly its 32 mask words (the (row / 4, col) layout of
// epi_rows and bias_act), and the block's rows leave as 16-byte stores of the
// output AND of the aux tensor (pre or GELU'(pre)).  In the register layout
// the aux tensor needed a staging pass of its own and the activation /
// dropout ran on the accumulator registers: GPT-2-XL's fc1 forward
// (18432 x 6400 x 1600, GELU, p 0.1, pre saved) cost 542 us against 358 plain
// (tools/epilogue_cost_probe.py).  Also the activation backward of a dgrad
// whose forward had dropout (dact_in with the mask regenerated).
template <int ACT, int W, int NJ = W / 64, int kT = 512, bool ROWSPLIT = false>
__device__ __forceinline__ void staged_store_act(char* smem, const f32x4 (&acc)[8][NJ], int wm, int wn,
                                                 int lane, int tid, int m0, int n0, const GemmArgs& g) {
  constexpr int WN = 16 * NJ, kStride = W + 4, CB = W / 8;
  const int quad = lane >> 4, col_in = lane & 15;
  float* stg = reinterpret_cast<float*>(smem);
  bf16_t* C = reinterpret_cast<bf16_t*>(g.C);
  bf16_t* aux = reinterpret_cast<bf16_t*>(g.aux);
  const bf16_t* res = reinterpret_cast<const bf16_t*>(g.res);
  const bf16_t* dact_in = reinterpret_cast<const bf16_t*>(g.dact_in);
  const int64_t ldr = g.ldr > 0 ? g.ldr : g.ldc;
  const bool drop = g.p > 0.f;
  const float pscale = drop ? 1.f / (1.f - g.p) : 1.f;
  const int64_t mask_ld = g.mask_ld > 0 ? g.mask_ld : g.N;
  const uint32_t thr16 = g.threshold >> 16;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    if (ROWSPLIT) {
#pragma unroll
      for (int ii = 0; ii < 4; ++ii)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            stg[(64 * wm + 16 * ii + 4 * quad + r) * kStride + wn * WN + 16 * j + col_in] = acc[4 * pass + ii][j][r];
    } else if (wm == pass) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            stg[(16 * i + 4 * quad + r) * kStride + wn * WN + 16 * j + col_in] = acc[i][j][r];
    }
    __syncthreads();
    const int rbase = m0 + pass * 128;
#pragma unroll
    for (int u = 0; u < 32 * CB / kT; ++u) {
      const int idx = tid + u * kT;
      const int rq = idx / CB, c8 = idx % CB;  // consecutive lanes on consecutive 8-column chunks
      const int col = n0 + 8 * c8;
      const int row0 = ROWSPLIT ? m0 + (((4 * rq) >> 6) << 7) + 64 * pass + ((4 * rq) & 63) : rbase + 4 * rq;
      if (col >= g.N || row0 >= g.M) continue;
      uint32_t wd[4][4];  // [column pair][row]: two 16-bit uniforms per word
      if (drop) {
        const uint64_t sub = drop_sub(row0 + g.mask_row0, col + g.mask_col0, mask_ld);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint4 w = Philox(g.seed, sub + e, g.offset).next4();
          wd[e][0] = w.x; wd[e][1] = w.y; wd[e][2] = w.z; wd[e][3] = w.w;
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + r;
        if (row >= g.M) break;
        const float* sp = stg + (4 * rq + r) * kStride + 8 * c8;
        const f32x4 lo = *reinterpret_cast<const f32x4*>(sp);
        const f32x4 hi = *reinterpret_cast<const f32x4*>(sp + 4);
        const float pre[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        if (aux != nullptr) {
          bf16x8 a;
#pragma unroll
          for (int e = 0; e < 8; ++e) a[e] = (__bf16)(ACT == kActGelu && g.aux_grad ? gelu_grad_f(pre[e]) : pre[e]);
          *reinterpret_cast<bf16x8*>(aux + (int64_t)row * g.ldc + col) = a;
        }
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float o = ACT == kActRelu ? fmaxf(pre[e], 0.f) : (ACT == kActGelu ? gelu_f(pre[e]) : pre[e]);
          if (drop) o = drop_keep(wd[e >> 1][r], e & 1, thr16) ? o * pscale : 0.f;
          v[e] = o;
        }
        if (dact_in != nullptr) {
          const bf16x8 sv = *reinterpret_cast<const bf16x8*>(dact_in + (int64_t)row * g.ldd + col);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] *= g.dact_scale * dact_f(g.dact, (float)sv[e]);
        }
        if (res != nullptr) {
          const bf16x8 rv = *reinterpret_cast<const bf16x8*>(res + (int64_t)row * ldr + col);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += (float)rv[e];
        }
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (__bf16)v[e];
        *reinterpret_cast<bf16x8*>(C + (int64_t)row * g.ldc + col) = o;
        if (g.bits != nullptr) {  // the output's nonzeros, for the consumer's dgrad (kActReluBits)
          uint32_t mb = 0;
#pragma unroll
          for (int e = 0; e < 8; ++e) mb |= (v[e] != 0.f ? 1u : 0u) << e;
          reinterpret_cast<uint8_t*>(g.bits)[(int64_t)row * g.ldbits + (col >> 3)] = (uint8_t)mb;
        }
      }
    }
    __syncthreads();
  }
}

// Ping-pong main loop (PP = true).  The two wave groups (wm = 0: waves 0-3,
// wm = 1: waves 4-7; each SIMD hosts one wave of each) run one barrier
// interval apart, so in every interval one wave per SIMD issues its 16-MFMA
// cluster while its partner issues the LDS fragment reads (and LDS-DMA
// staging) for its next cluster -- the LDS latency of one group hides behind
// the other's MFMAs instead of stalling both (guide: 256^2 8-phase template,
// T5 s_setprio).  A K-tile is 4 phases, one per 64x32 quadrant of the wave's
// 128x64 tile, in the order (0,0) (0,1) (1,1) (1,0): A fragments are read in
// phases 0 and 2, B in phases 0 and 1 and kept, phase 3 reads nothing.
// Buffer hand-off (intervals counted from group 0's first phase of tile u,
// group 1 one behind):
//   * tile u+1 is DMA'd into the other buffer in phases 0/1 (A/B) of tile u:
//     that buffer (tile u-1) was last read in tile u-1's phase 2, retired by
//     the lgkmcnt(0) of phase 2's MFMA interval, behind >= 1 barrier;
//   * each wave drains its own DMA (vmcnt(0)) before the barrier that ends
//     the last interval of tile u -- group 0 after its phase-3 MFMAs, group 1
//     in its phase-3 load interval -- so every wave's reads of tile u+1 start
//     after a barrier all DMAs of the tile have landed behind.
//
// 3 / 4 (default): as 2 / 1 with the B operand staged two K-tiles ahead (PP = 2).
// 0: one barrier per K-tile everywhere, 1: ping-pong everywhere, 2:
// ping-pong except the weight-gradient layout (both operands I-contiguous),
// where the per-tile loop measured 1-4 % faster (profiles/gemm_saddr_ab.txt).
// (A piece-staged variant -- each half-tile re-staged as soon as its own last
// reader was 2 phases behind, 6 phases of DMA lead, counted vmcnt -- measured
// 1-8 % slower than ping-pong: profiles/gemm_schedules_ab.txt.)
// Default 4: the B lead measured +3-7 % on the KC-layout forward / dgrad GEMMs
// (enc12 qkv fwd 1313 -> 1365 TF/s, dec dgrad 1297 -> 1388, GPT-2-XL dgrads
// +3-4 %; profiles/gemm_sched_ab.txt), and with it the ping-pong loop beats
// the per-tile one on the weight-gradient layout as well (+3-5 % at the sizes
// of a step's flush: profiles/wgrad_flush_sched.txt).
// 5: half-tile ping-pong (PP = 3: 2 phases of 32 MFMAs per K-tile), 6: 5 on the
// KC layouts and 4 on the weight-gradient layout, 7 (DEFAULT, round 3): whole-
// tile ping-pong (PP = 4: one 64-MFMA interval per K-tile and wave, 236-242
// VGPRs, no scratch).  Fewer, longer intervals pay the two barriers of a phase
// less often: enc12 qkv fwd 1369 -> 1438 TF/s, dec dgrad 1387 -> 1500, the
// enc12 PP=1 bench 139.0k -> 143.8k tok/s (same box, arms alternated;
// profiles/gemm_sched_ab.txt).
// Only schedule 7 is compiled into the product build (launch_big_w); the
// others need -DMIPIPE_GEMM_AB.
int g_gemm_sched = -1;  // -1: MIPIPE_GEMM_SCHED (default 7) not read yet
int gemm_sched() {
  if (g_gemm_sched < 0) {
#ifdef MIPIPE_GEMM_AB
    const char* e = getenv("MIPIPE_GEMM_SCHED");
    g_gemm_sched = e ? atoi(e) : 7;
#else
    g_gemm_sched = 7;
#endif
  }
  return g_gemm_sched;
}

// W: block tile width along N -- 256, or 128 for grids where 256x256 tiles
// would leave CUs idle (256x128 block, 128x32 per wave).
// EXTRA: the bf16 epilogue also applies dropout and/or stores the
// pre-activation (otherwise it is branch-free bias + activation).
// PP: 0 = one barrier per K-tile, 1 = ping-pong, 2 = ping-pong with the B
// operand staged two K-tiles ahead (below).
// X: main-loop extras, 0 none, kXEmit the A^T emission (GemmArgs::at), kXColsum
// the B-side bias fold (GemmArgs::colsum) -- separate instantiations, so the
// plain kernels keep their register allocation.
constexpr int kXEmit = 1, kXColsum = 2;

template <bool A_KC, bool B_KC, int EPI, int ACT, int PP, int W, bool EXTRA, int X = 0>
__global__ void __launch_bounds__(kThreads, 1) gemm256_kernel(GemmArgs g) {
  constexpr int NJ = W / 64;          // 16-wide MFMA column tiles per wave
  constexpr int JJ = NJ / 2;          // ... per ping-pong quadrant
  constexpr int WN = W / 4;           // wave tile width
  constexpr int kBuf = kTileBytes + W * BK * 2;  // A + B tile
  constexpr bool AH = PP == 4 && !A_KC;          // A tile as two 128-wide halves (stage_offsets_halves)
  constexpr bool B3 = PP == 4 && !B_KC;          // B tiles in three buffers (smem_bytes)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;

  int tm, tn;
  tile_coords((g.M + BM - 1) / BM, (g.N + W - 1) / W, tm, tn, g.group_m);
  tm = __builtin_amdgcn_readfirstlane(tm);  // block-uniform: scalar registers, not two VGPRs
  tn = __builtin_amdgcn_readfirstlane(tn);
  const int m0 = tm * BM, n0 = tn * W;
  f32x4 acc[8][NJ];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fused bias gradient (GemmArgs::rowsum): group-0 thread t sums the 4 rows
  // [16 tn + 4 (t & 3), +4) of K-row t >> 2 of every A tile (I-contiguous image)
  const bool rsum = g.rowsum != nullptr && tn < 16 && !A_KC;
  float rs[4] = {0.f, 0.f, 0.f, 0.f};
  auto rowsum_step = [&](const char* tile) {
    if (rsum && wm == 0) {
      const int r = tid >> 2, c8 = 4 * tn + (tid & 3);
      const s16x4 v = *reinterpret_cast<const s16x4*>(
          AH ? tile + (tn >> 3) * (kTileBytes / 2) + ic_off_w<128>(r, c8 & 31) : tile + ic_off_w<256>(r, c8));
#pragma unroll
      for (int e = 0; e < 4; ++e) rs[e] += __uint_as_float((uint32_t)(uint16_t)v[e] << 16);
    }
  };
  // fused bias gradient on the B side (GemmArgs::colsum): the tile column is cut
  // into slices of 16 cm columns spread over its tile rows -- block tm, wave
  // group wm sums slice tm + tiles_m wm; cm (1, 2, 4, 8) is the smallest that
  // lets the 2 tiles_m slices cover all W columns (gemm_colsum_ok).  Group-local
  // thread t sums the 4 columns [16 cm s + 4 q, +4), q = t mod 4 cm, of the
  // cm K-rows t / (4 cm) + j 64 / cm of every B tile it reads.  Four
  // accumulators per lane whatever cm is: more (two slices per lane) spilled
  // the main loop's DMA offsets.
  const int tiles_m = (g.M + BM - 1) / BM;
  const int cm_log = __builtin_amdgcn_readfirstlane(2 * tiles_m * 16 >= W ? 0 : 2 * tiles_m * 32 >= W ? 1
                                                    : 2 * tiles_m * 64 >= W ? 2 : 3);
  const int csl = tm + tiles_m * wm;  // this group's slice
  const bool csum = X == kXColsum && !B_KC && g.colsum != nullptr && csl < (W / 16 >> cm_log);
  float cs[4] = {0.f, 0.f, 0.f, 0.f};
  auto colsum_step = [&](const char* btile) {
    if (csum) {
      const int t = tid & 255;
      const int q = t & ((4 << cm_log) - 1), r0 = t >> (2 + cm_log);
      for (int j = 0; j < (1 << cm_log); ++j) {
        const s16x4 v = *reinterpret_cast<const s16x4*>(
            btile + ic_off_w<W>(r0 + (j << (6 - cm_log)), (4 << cm_log) * csl + q));
#pragma unroll
        for (int e = 0; e < 4; ++e) cs[e] += __uint_as_float((uint32_t)(uint16_t)v[e] << 16);
      }
    }
  };
  // A^T emission is spread evenly: K-tile kt's 32 pieces (wave w, j = 0..3:
  // tile rows [8 (4 w + j), +8)) go to the tile-row's blocks in rotation --
  // piece (w, j) by block tn = (4 w + j + kt) mod tiles_n -- so a wave emits
  // at most one piece per K-tile (2 transposing reads, their wait, 1 store)
  // instead of one block stalling on all 32: few extra registers (the dropout
  // variant's main loop did not fit them otherwise) and no long stall.
  const int ntn = (g.N + W - 1) / W;
  const int ewb = __builtin_amdgcn_readfirstlane((4 * wave) % ntn);  // scalar: no VGPR held across the loop
  // A piece: two transposing reads issued BEFORE the fragment reads and one
  // store issued AFTER them, so its wait retires only the oldest reads and
  // hides behind the fragment loads (waiting right after the reads exposed
  // their latency in every load interval: +8-17 % on the forward GEMMs).
  auto emit_reads = [&](const char* atile, int j, s16x4& a, s16x4& b) {
    const int q = (lane & 15) >> 2, p = lane & 3, gq = lane >> 4;
    const int c16 = 2 * gq + (p >> 1);
    const int r = 8 * (4 * wave + j) + q;
    const int lo = r * 128 + ((c16 ^ ((r >> 1) & 7)) << 4) + 8 * (p & 1);
    const int hi = (r + 4) * 128 + ((c16 ^ (((r + 4) >> 1) & 7)) << 4) + 8 * (p & 1);
    a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(atile + lo));
    b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(atile + hi));
  };
  auto emit_store = [&](int kt, int j, const s16x4& a, const s16x4& b) {
    const int rb = 4 * wave + j;
    bf16_t* at = reinterpret_cast<bf16_t*>(g.at) + (int64_t)(kt * BK + 16 * (lane >> 4) + (lane & 15)) * g.ldat + m0 +
                 8 * rb;
    if (m0 + 8 * rb < g.M) *reinterpret_cast<s16x8*>(at) = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  };
  int kt0 = 0, nk = g.K / BK;
  if (g.k_splits > 1) {  // this block's share of the K-tiles
    const int total = nk;
    kt0 = (int)blockIdx.y * total / g.k_splits;
    nk = ((int)blockIdx.y + 1) * total / g.k_splits - kt0;
  }
  // Staging shares of the PP == 4 schedule (see its loop): the waves of group 1
  // (which restage the buffer their siblings are still reading) take bytes no
  // sibling reads -- A rows 0-127 (group 0's half: share of "wave" w ^ 4; for
  // an I-contiguous A the tile is kept as two halves for this) and, for a
  // K-contiguous B, the first 32 of the 64 rows the wave itself reads (share
  // 2 wn; group 0 the other 32: 2 wn + 1).  An I-contiguous B (every wave
  // reads every k-row) rotates through three buffers instead and keeps the
  // per-wave k-row shares.
  const int shA = PP == 4 ? wave ^ 4 : wave;
  const int shB = PP == 4 && B_KC ? 2 * wn + (wm == 0 ? 1 : 0) : wave;
  uint32_t offA[4], offB[NJ];
  if constexpr (AH) stage_offsets_halves(g.lda, m0, g.M, shA, lane, offA);
  else stage_offsets<A_KC, 256>(g.lda, m0, g.M, shA, lane, offA);
  stage_offsets<B_KC, W>(g.ldb, n0, g.N, shB, lane, offB);
  // PP == 2 (LEADB): the B tile of K-tile u+2 is staged in phase 3 of tile u,
  // into the buffer tile u is being computed from -- its B region is dead by
  // then (B fragments are read in phases 0/1 and kept in registers; group 1's
  // last B read of tile u, phase 1, retired two barriers earlier).  B thus has
  // ~1.5 K-tiles to land instead of ~2 phases; the tile-end waits become
  // vmcnt(NB): all but the B DMAs just issued (loads retire in order).
  constexpr bool LEADB = PP == 2 || PP == 3 || PP == 4;
  constexpr int NB = W / 64;  // B DMAs per wave per K-tile
  constexpr int NA = 4;       // A DMAs per wave per K-tile
  {
    int kl;
    const bf16_t* A = seg_base(g, true, kt0 * BK, kl);
    stage_fast<A_KC, 256>(A, g.lda, kl, offA, smem, shA);
    const bf16_t* B = seg_base(g, false, kt0 * BK, kl);
    stage_fast<B_KC, W>(B, g.ldb, kl, offB, smem + kTileBytes, shB);
    if ((PP == 2 || PP == 3) && nk > 1) {
      B = seg_base(g, false, (kt0 + 1) * BK, kl);
      stage_fast<B_KC, W>(B, g.ldb, kl, offB, smem + kBuf + kTileBytes, wave);
    }
    if (PP == 3 && wm == 1 && nk > 1) {  // group 1 stages its A share one tile earlier (below)
      A = seg_base(g, true, (kt0 + 1) * BK, kl);
      stage_fast<A_KC, 256>(A, g.lda, kl, offA, smem + kBuf, wave);
    }
    if (PP == 4 && wm == 1 && nk > 1) {  // group 1 stages whole tiles one tile earlier (below)
      A = seg_base(g, true, (kt0 + 1) * BK, kl);
      stage_fast<A_KC, 256>(A, g.lda, kl, offA, smem + kBuf, shA);
      B = seg_base(g, false, (kt0 + 1) * BK, kl);
      stage_fast<B_KC, W>(B, g.ldb, kl, offB, smem + kBuf + kTileBytes, shB);
    }
  }

  if constexpr (PP == 4) {
    // Whole-tile ping-pong: one load and one MFMA interval per K-tile and wave
    // (64 MFMAs: the wave's whole 128x64 tile), barriers paid once per 1024
    // MFMA cycles.  Group 0 loads tile u in interval 2u, group 1 in 2u+1
    // (global count).  Tile u+1 goes into tile u-1's buffer, last read by
    // group 1 in 2u-1: group 1 stages its share right after those reads
    // (program order), group 0 in its load interval 2u.  Group 1's DMA into
    // tile u's buffer may land while a SIBLING wave still has reads of it
    // queued (no barrier separates the waves of a group; a sibling delayed by
    // its A^T emission piece was seen to read the next tile's rows once), so
    // group 1 restages only bytes none of its siblings reads: A rows 0-127
    // (shA above; an I-contiguous A is kept as two 128-row halves for that)
    // and, for a K-contiguous B, half of the i-rows the wave itself reads
    // (shB).  An I-contiguous B has no such share (every wave reads every
    // k-row of its columns), so its tiles rotate through three buffers: tile
    // u+2 goes into tile u-1's B buffer, whose last reads (group 1, interval
    // 2u-1) retired before the barrier ending that interval.  Tile u+1 must
    // have landed by the barrier ending 2u+1: group 0 drains after its MFMAs
    // (vmcnt(0)), group 1 in its load interval 2u+1 after staging tile u+2
    // (vmcnt(NA + NB)).
    if (wm == 1 && nk > 1) vmcnt_keep<NA + NB>();
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (wm == 1) __builtin_amdgcn_s_barrier();  // stagger group 1 by one interval
    bf16x8 af[8][2], bq[NJ][2];
    int ekt = kt0 % ntn;  // (kt0 + u) mod tiles_n (A^T emission rotation)
    // B3: B buffer of slot s (tiles kt0, kt0 + 1 were staged into slots 0, 1)
    auto bslot = [&](int s) { return s == 2 ? smem + 2 * kBuf : smem + s * kBuf + kTileBytes; };
    int bs = 0;  // B3: slot of tile u (u mod 3)
    for (int u = 0; u < nk; ++u) {
      char* cur = smem + (u & 1) * kBuf;
      char* nxt = smem + ((u + 1) & 1) * kBuf;
      char* bcur = B3 ? bslot(bs) : cur + kTileBytes;
      // emission first: its reads precede this wave's DMA that may restage
      // `cur`, and its stores (waiting for those reads) precede the fragment
      // reads, so its 16 data registers are dead before the fragments load
      // this wave's A^T piece of K-tile kt0 + u, if any: j with (4 wave + j + kt) mod tiles_n == tn
      // (grids under 4 tile columns give a wave several pieces of a K-tile:
      // those are read and stored one after the other, here)
      int ej = -1;
      if (X == kXEmit && A_KC) {
        int e = ewb + ekt;
        while (e >= ntn) e -= ntn;
        ej = tn - e;  // first piece index (the wrap: tn + ntn - e)
        if (ej < 0) ej += ntn;
        if (ntn < 4) {
          for (int j = ej; j < 4; j += ntn) {
            s16x4 a, b;
            emit_reads(cur, j, a, b);
            emit_store(kt0 + u, j, a, b);
          }
          ej = -1;
        } else if (ej > 3) {
          ej = -1;
        }
      }
      s16x4 ea, eb;
      if (X == kXEmit && A_KC && ej >= 0) emit_reads(cur, ej, ea, eb);
#pragma unroll
      for (int ii = 0; ii < 8; ++ii)
#pragma unroll
        for (int s = 0; s < 2; ++s)
          af[ii][s] = AH ? frag<false, 128>(cur + wm * (kTileBytes / 2), 16 * ii, s, lane)
                         : frag<A_KC, 256>(cur, wm * 128 + 16 * ii, s, lane);
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int s = 0; s < 2; ++s) bq[j][s] = frag<B_KC, W>(bcur, wn * WN + 16 * j, s, lane);
      rowsum_step(cur);
      colsum_step(bcur);
      if (X == kXEmit && A_KC && ej >= 0) emit_store(kt0 + u, ej, ea, eb);
      ekt = ekt + 1 == ntn ? 0 : ekt + 1;
      const int ahead = wm == 0 ? 1 : 2;  // the tile this group stages now
      if (u + ahead < nk) {
        int kl;
        char* dst = wm == 0 ? nxt : cur;
        const bf16_t* A = seg_base(g, true, (kt0 + u + ahead) * BK, kl);
        stage_fast<A_KC, 256>(A, g.lda, kl, offA, dst, shA);
        const bf16_t* B = seg_base(g, false, (kt0 + u + ahead) * BK, kl);
        int bn = bs + ahead;
        if (bn >= 3) bn -= 3;
        stage_fast<B_KC, W>(B, g.ldb, kl, offB, B3 ? bslot(bn) : dst + kTileBytes, shB);
      }
      bs = bs == 2 ? 0 : bs + 1;
      if (wm == 1) {
        if (u + 2 < nk) vmcnt_keep<NA + NB>();
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      // Retire this interval's LDS reads BEFORE the barrier: right after it the
      // other group restages the buffer just read (group 0 DMAs tile u+1 over
      // tile u-1, group 1 tile u+2 over tile u), and a read still queued in
      // the LDS when that DMA lands returns the new tile -- an intermittent
      // wrong accumulator (tools/gemm_round_screen.py caught it: ~1 launch in
      // 3 of one shape).  Guide rule: restage one phase after a read only when
      // an lgkmcnt before the reading phase's barrier retired it.
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int ii = 0; ii < 8; ++ii)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[ii][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ii][s], bq[j][s], acc[ii][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      if (wm == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
    if (wm == 0) __builtin_amdgcn_s_barrier();  // equalise the barrier count
  } else

  if constexpr (PP == 3) {
    // Half-tile ping-pong: as PP = 2, but a K-tile is 2 phases of 32 MFMAs
    // (one 64-row half of the wave's 128x64 tile each, all NJ column tiles:
    // A fragments read in both phases, B in phase 0 and kept), so the two
    // barriers of a phase are paid once per 512 MFMA cycles instead of 256.
    // Intervals (global count, group 1 one behind): group 0 loads in 4u and
    // 4u+2, group 1 in 4u+1 and 4u+3.  A read issued before a DMA into the
    // same bytes returns the old bytes (same wave: program order; another
    // wave: a barrier between), so a region may be restaged by a DMA issued
    // after the barrier that follows its last read's ISSUE:
    //   * the A region of tile u-1's buffer is last read by group 1 in 4u-1
    //     (its phase-1 load): group 1 restages it with A(u+1) right there,
    //     after its own reads (tile u+1 = tile u-1's buffer), group 0 in 4u;
    //   * the B region of tile u's buffer is last read by group 1 in 4u+1:
    //     both groups stage B(u+2) into it in their phase-1 loads (4u+2/4u+3).
    // Every wave drains what tile u+1 needs before the barrier ending 4u+3:
    // group 0 after its phase-1 MFMAs (vmcnt(NB): B(u+2) may be in flight),
    // group 1 in its phase-1 load (vmcnt(NA + NB): A(u+2) and B(u+2)).
    // DMA budget: 4-6 intervals (~2-3k cycles) per piece.
    if (nk > 1) {
      if (wm == 1) vmcnt_keep<NA + NB>();
      else vmcnt_keep<NB>();
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    if (wm == 1) __builtin_amdgcn_s_barrier();  // stagger group 1 by one interval
    bf16x8 af[4][2], bq[NJ][2];
    for (int u = 0; u < nk; ++u) {
      char* cur = smem + (u & 1) * kBuf;
      char* nxt = smem + ((u + 1) & 1) * kBuf;
      const bool more = u + 1 < nk, lead = u + 2 < nk;
#pragma unroll
      for (int ph = 0; ph < 2; ++ph) {
        // ---- load interval ----
#pragma unroll
        for (int ii = 0; ii < 4; ++ii)
#pragma unroll
          for (int s = 0; s < 2; ++s) af[ii][s] = frag<A_KC, 256>(cur, wm * 128 + ph * 64 + 16 * ii, s, lane);
        if (ph == 0) rowsum_step(cur);
        if (ph == 0) {
#pragma unroll
          for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int s = 0; s < 2; ++s) bq[j][s] = frag<B_KC, W>(cur + kTileBytes, wn * WN + 16 * j, s, lane);
          if (wm == 0 && more) {
            int kl;
            const bf16_t* A = seg_base(g, true, (kt0 + u + 1) * BK, kl);
            stage_fast<A_KC, 256>(A, g.lda, kl, offA, nxt, wave);
          }
        } else if (lead) {
          int kl;
          if (wm == 1) {
            const bf16_t* A = seg_base(g, true, (kt0 + u + 2) * BK, kl);
            stage_fast<A_KC, 256>(A, g.lda, kl, offA, cur, wave);
          }
          const bf16_t* B = seg_base(g, false, (kt0 + u + 2) * BK, kl);
          stage_fast<B_KC, W>(B, g.ldb, kl, offB, cur + kTileBytes, wave);
        }
        if (ph == 1 && wm == 1) {
          if (lead) vmcnt_keep<NA + NB>();
          else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        // ---- MFMA interval ----
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int ii = 0; ii < 4; ++ii)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
              acc[ph * 4 + ii][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ii][s], bq[j][s], acc[ph * 4 + ii][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        if (ph == 1 && wm == 0) {
          if (lead) vmcnt_keep<NB>();
          else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if (wm == 0) __builtin_amdgcn_s_barrier();  // equalise the barrier count
  } else if constexpr (PP) {
    if (LEADB && nk > 1) vmcnt_keep<NB>();
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (wm == 1) __builtin_amdgcn_s_barrier();  // stagger group 1 by one interval
    bf16x8 af[4][2], bf[2][JJ][2];
    for (int u = 0; u < nk; ++u) {
      const char* cur = smem + (u & 1) * kBuf;
      char* nxt = smem + ((u + 1) & 1) * kBuf;
      const bool more = u + 1 < nk;
#pragma unroll
      for (int ph = 0; ph < 4; ++ph) {
        const int qm = ph >= 2 ? 1 : 0;
        const int qn = (ph == 1 || ph == 2) ? 1 : 0;
        // ---- load interval: this cluster's fragments, then staging DMA ----
        if (ph == 0 || ph == 2) {
#pragma unroll
          for (int ii = 0; ii < 4; ++ii)
#pragma unroll
            for (int s = 0; s < 2; ++s) af[ii][s] = frag<A_KC, 256>(cur, wm * 128 + qm * 64 + 16 * ii, s, lane);
        }
        if (ph == 0) rowsum_step(cur);
        if (ph == 0 || ph == 1) {
#pragma unroll
          for (int jj = 0; jj < JJ; ++jj)
#pragma unroll
            for (int s = 0; s < 2; ++s)
              bf[qn][jj][s] = frag<B_KC, W>(cur + kTileBytes, wn * WN + qn * (WN / 2) + 16 * jj, s, lane);
        }
        if (ph == 0 && more) {
          int kl;
          const bf16_t* A = seg_base(g, true, (kt0 + u + 1) * BK, kl);
          stage_fast<A_KC, 256>(A, g.lda, kl, offA, nxt, wave);
        }
        if (!LEADB && ph == 1 && more) {
          int kl;
          const bf16_t* B = seg_base(g, false, (kt0 + u + 1) * BK, kl);
          stage_fast<B_KC, W>(B, g.ldb, kl, offB, nxt + kTileBytes, wave);
        }
        const bool lead = LEADB && u + 2 < nk;  // a B DMA two tiles ahead is issued this tile
        if (ph == 3 && lead) {
          int kl;
          const bf16_t* B = seg_base(g, false, (kt0 + u + 2) * BK, kl);
          stage_fast<B_KC, W>(B, g.ldb, kl, offB, const_cast<char*>(cur) + kTileBytes, wave);
        }
        if (ph == 3 && wm == 1) {
          if (lead) vmcnt_keep<NB>();
          else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        // ---- MFMA interval ----
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int ii = 0; ii < 4; ++ii)
#pragma unroll
            for (int jj = 0; jj < JJ; ++jj)
              acc[qm * 4 + ii][qn * JJ + jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                  af[ii][s], bf[qn][jj][s], acc[qm * 4 + ii][qn * JJ + jj], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        if (ph == 3 && wm == 0) {
          if (lead) vmcnt_keep<NB>();
          else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if (wm == 0) __builtin_amdgcn_s_barrier();  // equalise the barrier count
  } else {
  for (int kt = 0; kt < nk; ++kt) {
    // Tile kt has landed (every wave drained its own DMA) and every wave is
    // done reading the buffer the next prefetch overwrites.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kt + 1 < nk) {
      char* nxt = smem + ((kt + 1) & 1) * kBuf;
      int kl;
      const bf16_t* A = seg_base(g, true, (kt0 + kt + 1) * BK, kl);
      stage_fast<A_KC, 256>(A, g.lda, kl, offA, nxt, wave);
      const bf16_t* B = seg_base(g, false, (kt0 + kt + 1) * BK, kl);
      stage_fast<B_KC, W>(B, g.ldb, kl, offB, nxt + kTileBytes, wave);
    }
    const char* cur = smem + (kt & 1) * kBuf;
    rowsum_step(cur);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 bfr[NJ];
#pragma unroll
      for (int t = 0; t < NJ; ++t) bfr[t] = frag<B_KC, W>(cur + kTileBytes, wn * WN + 16 * t, s, lane);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const bf16x8 af = frag<A_KC, 256>(cur, wm * 128 + 16 * i, s, lane);
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[j], acc[i][j], 0, 0, 0);
      }
    }
  }
  }

  if (rsum) {  // K-rows -> one sum per row: lanes (xor over the K-row bits), then the 4 group-0 waves through LDS
    __syncthreads();  // every wave is done reading the operand buffers
    float* red = reinterpret_cast<float*>(smem);
    if (wm == 0) {
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int o = 4; o < 64; o <<= 1) rs[e] += __shfl_xor(rs[e], o, 64);
      if (lane < 4)
#pragma unroll
        for (int e = 0; e < 4; ++e) red[wave * 16 + 4 * lane + e] = rs[e];
    }
    __syncthreads();
    if (tid < 16) {
      const float v = red[tid] + red[16 + tid] + red[32 + tid] + red[48 + tid];
      const int row = m0 + 16 * tn + tid;
      if (row < g.M) g.rowsum[row] += v;
    }
  }
  if (X == kXColsum && g.colsum != nullptr) {  // the same reduction for the B-side column sums, per group
    __syncthreads();
    const int sw = 16 << cm_log;  // slice width
    float* red = reinterpret_cast<float*>(smem) + 64;  // [8 waves][sw columns]
#pragma unroll
    for (int e = 0; e < 4; ++e)
      for (int o = 4 << cm_log; o < 64; o <<= 1) cs[e] += __shfl_xor(cs[e], o, 64);
    if (lane < (4 << cm_log))
#pragma unroll
      for (int e = 0; e < 4; ++e) red[wave * sw + 4 * lane + e] = cs[e];
    __syncthreads();
    if (tid < 2 * sw) {
      const int gq = tid >> (4 + cm_log), c = tid & (sw - 1);
      const int sl = tm + tiles_m * gq;
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) v += red[(4 * gq + w) * sw + c];
      const int col = n0 + sw * sl + c;
      if (sl < (W / 16 >> cm_log) && col < g.N) {
        if (g.k_splits > 1) g.colsum[(int64_t)blockIdx.y * g.N + col] = v;  // split-K: a partial per split
        else g.colsum[col] += v;
      }
    }
  }
  // ---- epilogue ----
  // 1) element-wise epilogue in registers (accumulator layout): bias,
  //    activation, dropout (the mask is tied to this layout); with an aux
  //    output, the pre-activation (acc + bias) is first written out through
  //    the same staged path;
  // 2) staged_store: LDS-staged 16-byte row stores (+ residual addend), fp32
  //    read-modify-write for an accumulated weight gradient, fp32 stores for
  //    the first write of a step or a split-K partial.
  //    (The earlier direct 2-byte bf16 stores cost ~5 us per 256x256 tile at
  //    K = 64 more than this path: tools/gemm_k_sweep.py.)
  const int quad = lane >> 4, col_in = lane & 15;
  __syncthreads();  // every wave is done reading the operand buffers
  if (EPI == kEpiStoreBf16 && EXTRA) {  // dropout and / or aux: the staged-layout epilogue does it all
    const int ncol = n0 + wn * WN + col_in;
    if (g.bias != nullptr) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const float b = ncol + 16 * j < g.N ? bf2f(reinterpret_cast<const bf16_t*>(g.bias)[ncol + 16 * j]) : 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i][j] += b;
      }
    }
    staged_store_act<ACT, W>(smem, acc, wm, wn, lane, tid, m0, n0, g);
    return;
  }
  if (EPI == kEpiStoreBf16 && (ACT != kActNone || g.bias != nullptr)) {
    const int ncol = n0 + wn * WN + col_in, nrow = m0 + wm * 128 + 4 * quad;
    const float pscale = g.p > 0.f ? 1.f / (1.f - g.p) : 1.f;
    const EpiParams ep{g.seed, g.offset, g.N, g.p, pscale, g.threshold, g.mask_row0, g.mask_col0,
                       g.mask_ld > 0 ? g.mask_ld : g.N};
    float bias[NJ];  // the lane's NJ columns: loaded once, all in flight together
#pragma unroll
    for (int j = 0; j < NJ; ++j)
      bias[j] = (g.bias != nullptr && ncol + 16 * j < g.N) ? bf2f(reinterpret_cast<const bf16_t*>(g.bias)[ncol + 16 * j]) : 0.f;
    epi_rows<0, ACT, NJ, EXTRA>(ep, acc, nrow, ncol, bias);
    epi_rows<1, ACT, NJ, EXTRA>(ep, acc, nrow, ncol, bias);
    epi_rows<2, ACT, NJ, EXTRA>(ep, acc, nrow, ncol, bias);
    epi_rows<3, ACT, NJ, EXTRA>(ep, acc, nrow, ncol, bias);
    epi_rows<4, ACT, NJ, EXTRA>(ep, acc, nrow, ncol, bias);
    epi_rows<5, ACT, NJ, EXTRA>(ep, acc, nrow, ncol, bias);
    epi_rows<6, ACT, NJ, EXTRA>(ep, acc, nrow, ncol, bias);
    epi_rows<7, ACT, NJ, EXTRA>(ep, acc, nrow, ncol, bias);
  }
  void* out = EPI == kEpiStoreBf16 ? g.C
                                   : reinterpret_cast<void*>(reinterpret_cast<float*>(g.C) +
                                                             (int64_t)blockIdx.y * g.M * g.ldc);  // split-K partial y
  if (EPI == kEpiStoreBf16 && g.dact_in != nullptr)
    staged_store<EPI, W>(smem, acc, wm, wn, lane, tid, m0, n0, g.M, g.N, g.ldc, out,
                         reinterpret_cast<const bf16_t*>(g.res), g.ldr, reinterpret_cast<const bf16_t*>(g.dact_in),
                         g.ldd, g.dact, g.dact_scale);
  else if (EPI != kEpiStoreBf16 && g.trans_c && g.k_splits <= 1)
    staged_store<EPI, W>(smem, acc, wm, wn, lane, tid, m0, n0, g.M, g.N, g.ldc, out, nullptr, 0, nullptr, 0, 0, 1.f,
                         true);
  else
    staged_store<EPI, W>(smem, acc, wm, wn, lane, tid, m0, n0, g.M, g.N, g.ldc, out,
                         EPI == kEpiStoreBf16 ? reinterpret_cast<const bf16_t*>(g.res) : nullptr, g.ldr);
}

#ifdef MIPIPE_GEMM_AB
// ============================================================================
// 4-wave variant: the same 256x256x64 block tile, LDS
// images, staging offsets and epilogues, computed by 4 waves instead of 8 --
// 2 M x 2 N, a 128x128 tile per wave (8x8 v_mfma_f32_16x16x32_bf16
// accumulators: 256 registers, AGPRs), ONE wave per SIMD.  Per k32-step a
// wave reads 16 fragments (8 A + 8 B) for 64 MFMAs, 256 B of LDS per MFMA
// against the 8-wave kernel's 384 (128x64 wave tile): a third less LDS
// traffic and issue.  With no partner wave on the SIMD, the LDS latency is
// hidden inside the wave: the fragments of the next k32-step are read
// between the MFMAs of this one (one read after every 4th MFMA), and the
// K-tile two ahead is staged by LDS-DMA in the same stream (one 1 KiB piece
// after every 4th MFMA of the second k-step).  One barrier per K-tile,
// between its two k-steps:
//   k-step 0 of tile u:  MFMAs on fragments (u, 0); reads of (u, 1) from cur
//   wait: this wave's DMAs of tile u+1 landed, its reads of cur retired
//   barrier            -> cur is free for restaging, tile u+1 readable
//   k-step 1 of tile u:  MFMAs on (u, 1); reads of (u+1, 0) from nxt; DMA of
//                        tile u+2 into cur
// Past the last tiles the DMA restages the last tile and the reads read the
// other buffer (both harmless: nothing reads them), so the stream has no
// branches.  Compiler scheduling is pinned by sched_barriers between the
// MFMA groups.  A^T emission is not supported (launch_big_w keeps those on
// the 8-wave kernel).
template <bool A_KC, bool B_KC, int EPI, int ACT, bool EXTRA, int X = 0>
__global__ void __launch_bounds__(256, 1) gemm4w_kernel(GemmArgs g) {
  constexpr int W = 256, NJ = 8, WN = 128;
  constexpr int kBuf = 2 * kTileBytes;  // A + B tile
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  int tm, tn;
  tile_coords((g.M + BM - 1) / BM, (g.N + W - 1) / W, tm, tn, g.group_m);
  tm = __builtin_amdgcn_readfirstlane(tm);
  tn = __builtin_amdgcn_readfirstlane(tn);
  const int m0 = tm * BM, n0 = tn * W;
  f32x4 acc[8][NJ];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fused bias gradient, A side (GemmArgs::rowsum): as the 8-wave kernel's
  // group 0, with all 256 threads
  const bool rsum = g.rowsum != nullptr && tn < 16 && !A_KC;
  float rs[4] = {0.f, 0.f, 0.f, 0.f};
  auto rowsum_step = [&](const char* tile) {
    if (rsum) {
      const int r = tid >> 2, c8 = 4 * tn + (tid & 3);
      const s16x4 v = *reinterpret_cast<const s16x4*>(tile + ic_off_w<256>(r, c8));
#pragma unroll
      for (int e = 0; e < 4; ++e) rs[e] += __uint_as_float((uint32_t)(uint16_t)v[e] << 16);
    }
  };
  // fused bias gradient, B side (GemmArgs::colsum): the 8-wave kernel's two
  // group slices, both summed by these 256 threads
  const int tiles_m = (g.M + BM - 1) / BM;
  const int cm_log = __builtin_amdgcn_readfirstlane(2 * tiles_m * 16 >= W ? 0 : 2 * tiles_m * 32 >= W ? 1
                                                    : 2 * tiles_m * 64 >= W ? 2 : 3);
  const bool csum0 = X == kXColsum && !B_KC && g.colsum != nullptr && tm < (W / 16 >> cm_log);
  const bool csum1 = X == kXColsum && !B_KC && g.colsum != nullptr && tm + tiles_m < (W / 16 >> cm_log);
  float cs[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  auto colsum_step = [&](const char* btile) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      if (q == 0 ? csum0 : csum1) {
        const int csl = tm + tiles_m * q;
        const int qq = tid & ((4 << cm_log) - 1), r0 = tid >> (2 + cm_log);
        for (int j = 0; j < (1 << cm_log); ++j) {
          const s16x4 v = *reinterpret_cast<const s16x4*>(
              btile + ic_off_w<W>(r0 + (j << (6 - cm_log)), (4 << cm_log) * csl + qq));
#pragma unroll
          for (int e = 0; e < 4; ++e) cs[q][e] += __uint_as_float((uint32_t)(uint16_t)v[e] << 16);
        }
      }
    }
  };

  int kt0 = 0, nk = g.K / BK;
  if (g.k_splits > 1) {
    const int total = nk;
    kt0 = (int)blockIdx.y * total / g.k_splits;
    nk = ((int)blockIdx.y + 1) * total / g.k_splits - kt0;
  }
  // staging: wave w takes the 8-wave shares w and w + 4 of each operand tile
  uint32_t offA0[4], offA1[4], offB0[4], offB1[4];
  stage_offsets<A_KC, 256>(g.lda, m0, g.M, wave, lane, offA0);
  stage_offsets<A_KC, 256>(g.lda, m0, g.M, wave + 4, lane, offA1);
  stage_offsets<B_KC, W>(g.ldb, n0, g.N, wave, lane, offB0);
  stage_offsets<B_KC, W>(g.ldb, n0, g.N, wave + 4, lane, offB1);
  // Operand bases of K-tile kt (scalar).  Every GemmArgs field the loop needs
  // is read into a local first: the DMA asm clobbers "memory", and a field
  // read after it is re-loaded from the kernel arguments -- an s_load whose
  // s_waitcnt lgkmcnt(0) also drains every LDS read in flight (that cost the
  // first version of this kernel 20 %).  The bases of the tile staged in k-step
  // 1 are computed at the top of the iteration, before any DMA of it.
  const int64_t lda = g.lda, ldb = g.ldb;
  const int seg_k = g.seg_k;
  const char* const gA = reinterpret_cast<const char*>(g.A);
  const char* const gB = reinterpret_cast<const char*>(g.B);
  auto tile_bases = [&](int kt, const char*& bA, const char*& bB) {
    int kl = (kt0 + kt) * BK;
    const char *a = gA, *b = gB;
    if (seg_k > 0) {  // segmented operands: the segment's pointers (the only scalar loads in the loop)
      const int sg = kl / seg_k;
      kl -= sg * seg_k;
      a = reinterpret_cast<const char*>(g.a_seg[sg]);
      b = reinterpret_cast<const char*>(g.b_seg[sg]);
    }
    bA = a + (A_KC ? (int64_t)kl * 2 : (int64_t)kl * lda * 2);
    bB = b + (B_KC ? (int64_t)kl * 2 : (int64_t)kl * ldb * 2);
  };
  // piece d (0-15) of a K-tile into buffer buf: A shares (d 0-7), then B
  auto stage_piece = [&](const char* bA, const char* bB, char* buf, int d) {
    if (d < 8) {
      const int sh = d < 4 ? wave : wave + 4;
      glds16_saddr(bA, d < 4 ? offA0[d & 3] : offA1[d & 3], buf + (sh * 4 + (d & 3)) * 1024);
    } else {
      const int sh = d < 12 ? wave : wave + 4;
      glds16_saddr(bB, d < 12 ? offB0[d & 3] : offB1[d & 3], buf + kTileBytes + (sh * 4 + (d & 3)) * 1024);
    }
  };
  const char *bA, *bB;
  tile_bases(0, bA, bB);
  const char *bA1 = bA, *bB1 = bB;
  if (nk > 1) tile_bases(1, bA1, bB1);
#pragma unroll
  for (int d = 0; d < 16; ++d) stage_piece(bA, bB, smem, d);
  if (nk > 1) {
#pragma unroll
    for (int d = 0; d < 16; ++d) stage_piece(bA1, bB1, smem + kBuf, d);
    vmcnt_keep<16>();
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  bf16x8 fa[2][8], fb[2][8];  // [k-step][tile]
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    fa[0][i] = frag<A_KC, 256>(smem, wm * 128 + 16 * i, 0, lane);
    fb[0][i] = frag<B_KC, W>(smem + kTileBytes, wn * WN + 16 * i, 0, lane);
  }
  for (int u = 0; u < nk; ++u) {
    char* cur = smem + (u & 1) * kBuf;
    char* nxt = smem + ((u + 1) & 1) * kBuf;
    __builtin_amdgcn_sched_barrier(0);
    // ---- k-step 0: MFMAs on (u, 0), fragment reads of (u, 1) ----
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0][i], fb[0][j], acc[i][j], 0, 0, 0);
        // read q after MFMA 3 q: all 16 issued by MFMA 45, so they have landed by
        // the k-step's end (the wait before the barrier, and the compiler's wait
        // at the top of the next k-step, find them retired)
        const int gi = NJ * i + j;
        if (gi % 3 == 0 && gi / 3 < 16) {
          const int q = gi / 3;  // read order A0, B0-B7, A1-A7: the order the MFMAs use them
          const int ia = q == 0 ? 0 : q - 8;
          if (q == 0 || q > 8) fa[1][ia] = frag<A_KC, 256>(cur, wm * 128 + 16 * ia, 1, lane);
          else fb[1][q - 1] = frag<B_KC, W>(cur + kTileBytes, wn * WN + 16 * (q - 1), 1, lane);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    rowsum_step(cur);
    colsum_step(cur + kTileBytes);
    // Bases of tile u+2 (past the end: the last tile again), whose scalar
    // loads (segmented operands) the wait below drains with the LDS reads: no
    // scalar load is ever pending where the compiler counts LDS reads, so its
    // own waits stay counted (lgkmcnt(N)) rather than lgkmcnt(0).
    __builtin_amdgcn_sched_barrier(0);
    const char *sA, *sB;
    tile_bases(u + 2 < nk ? u + 2 : nk - 1, sA, sB);
    // this wave's DMAs of tile u+1 have landed and its reads of cur retired;
    // after the barrier cur may be restaged and nxt read
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // ---- k-step 1: MFMAs on (u, 1), reads of (u+1, 0), DMA of tile u+2 ----
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[1][i], fb[1][j], acc[i][j], 0, 0, 0);
        const int gi = NJ * i + j;
        // DMA piece after every 4th MFMA from 1, fragment read after every 4th from 3
        // (harness schedule 2: tools/micro/gemm4w.hip, profiles/gemm4w_r5.txt)
        if ((gi & 3) == 1) stage_piece(sA, sB, cur, gi >> 2);
        if ((gi & 3) == 3) {
          const int q = gi >> 2, ia = q == 0 ? 0 : q - 8;
          if (q == 0 || q > 8) fa[0][ia] = frag<A_KC, 256>(nxt, wm * 128 + 16 * ia, 0, lane);
          else fb[0][q - 1] = frag<B_KC, W>(nxt + kTileBytes, wn * WN + 16 * (q - 1), 0, lane);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");

  if (rsum) {  // K-rows -> one sum per row: lanes (xor over the K-row bits), then the 4 waves through LDS
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int o = 4; o < 64; o <<= 1) rs[e] += __shfl_xor(rs[e], o, 64);
    if (lane < 4)
#pragma unroll
      for (int e = 0; e < 4; ++e) red[wave * 16 + 4 * lane + e] = rs[e];
    __syncthreads();
    if (tid < 16) {
      const float v = red[tid] + red[16 + tid] + red[32 + tid] + red[48 + tid];
      const int row = m0 + 16 * tn + tid;
      if (row < g.M) g.rowsum[row] += v;
    }
  }
  if (X == kXColsum && g.colsum != nullptr) {  // the 8-wave kernel's reduction, slice q in place of group q
    __syncthreads();
    const int sw = 16 << cm_log;
    float* red = reinterpret_cast<float*>(smem) + 64;  // [2 slices x 4 waves][sw columns]
#pragma unroll
    for (int q = 0; q < 2; ++q) {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        for (int o = 4 << cm_log; o < 64; o <<= 1) cs[q][e] += __shfl_xor(cs[q][e], o, 64);
      if (lane < (4 << cm_log))
#pragma unroll
        for (int e = 0; e < 4; ++e) red[(4 * q + wave) * sw + 4 * lane + e] = cs[q][e];
    }
    __syncthreads();
    for (int t = tid; t < 2 * sw; t += 256) {
      const int gq = t >> (4 + cm_log), c = t & (sw - 1);
      const int sl = tm + tiles_m * gq;
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) v += red[(4 * gq + w) * sw + c];
      const int col = n0 + sw * sl + c;
      if (sl < (W / 16 >> cm_log) && col < g.N) {
        if (g.k_splits > 1) g.colsum[(int64_t)blockIdx.y * g.N + col] = v;
        else g.colsum[col] += v;
      }
    }
  }
  // ---- epilogue (as the 8-wave kernel's, on the 128x128 wave layout) ----
  const int quad = lane >> 4, col_in = lane & 15;
  __syncthreads();
  if (EPI == kEpiStoreBf16 && EXTRA) {
    const int ncol = n0 + wn * WN + col_in;
    if (g.bias != nullptr) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const float b = ncol + 16 * j < g.N ? bf2f(reinterpret_cast<const bf16_t*>(g.bias)[ncol + 16 * j]) : 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i][j] += b;
      }
    }
    staged_store_act<ACT, W, NJ, 256, true>(smem, acc, wm, wn, lane, tid, m0, n0, g);
    return;
  }
  if (EPI == kEpiStoreBf16 && (ACT != kActNone || g.bias != nullptr)) {
    const int ncol = n0 + wn * WN + col_in, nrow = m0 + wm * 128 + 4 * quad;
    const float pscale = g.p > 0.f ? 1.f / (1.f - g.p) : 1.f;
    const EpiParams ep{g.seed, g.offset, g.N, g.p, pscale, g.threshold, g.mask_row0, g.mask_col0,
                       g.mask_ld > 0 ? g.mask_ld : g.N};
    float bias[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
      bias[j] = (g.bias != nullptr && ncol + 16 * j < g.N) ? bf2f(reinterpret_cast<const bf16_t*>(g.bias)[ncol + 16 * j]) : 0.f;
    epi_rows<0, ACT, NJ, EXTRA>(ep, acc, nrow, ncol, bias);
    epi_rows<1, ACT, NJ, EXTRA>(ep, acc, nrow, ncol, bias);
    epi_rows<2, ACT, NJ, EXTRA>(ep, acc, nrow, ncol, bias);
    epi_rows<3, ACT, NJ, EXTRA>(ep, acc, nrow, ncol, bias);
    epi_rows<4, ACT, NJ, EXTRA>(ep, acc, nrow, ncol, bias);
    epi_rows<5, ACT, NJ, EXTRA>(ep, acc, nrow, ncol, bias);
    epi_rows<6, ACT, NJ, EXTRA>(ep, acc, nrow, ncol, bias);
    epi_rows<7, ACT, NJ, EXTRA>(ep, acc, nrow, ncol, bias);
  }
  void* out = EPI == kEpiStoreBf16 ? g.C
                                   : reinterpret_cast<void*>(reinterpret_cast<float*>(g.C) +
                                                             (int64_t)blockIdx.y * g.M * g.ldc);
  if (EPI == kEpiStoreBf16 && g.dact_in != nullptr)
    staged_store<EPI, W, NJ, 256, true>(smem, acc, wm, wn, lane, tid, m0, n0, g.M, g.N, g.ldc, out,
                                  reinterpret_cast<const bf16_t*>(g.res), g.ldr,
                                  reinterpret_cast<const bf16_t*>(g.dact_in), g.ldd, g.dact, g.dact_scale);
  else if (EPI != kEpiStoreBf16 && g.trans_c && g.k_splits <= 1)
    staged_store<EPI, W, NJ, 256, true>(smem, acc, wm, wn, lane, tid, m0, n0, g.M, g.N, g.ldc, out, nullptr, 0, nullptr, 0,
                                  0, 1.f, true);
  else
    staged_store<EPI, W, NJ, 256, true>(smem, acc, wm, wn, lane, tid, m0, n0, g.M, g.N, g.ldc, out,
                                  EPI == kEpiStoreBf16 ? reinterpret_cast<const bf16_t*>(g.res) : nullptr, g.ldr);
}
#endif  // MIPIPE_GEMM_AB (the 4-wave kernel: A/B builds only, profiles/gemm4w_r5.txt)

}  // namespace big

int big_tiles(const GemmArgs& g, int w) { return ((g.M + big::BM - 1) / big::BM) * ((g.N + w - 1) / w); }

// The 256-row kernel handles every shape (edge tiles masked); the 128x128 one
// only exact multiples of 128, where it is kept for grids too small to fill
// the 256 CUs with 256x256 tiles.
// Chunks of a per-round launch stay on it too: the last chunk of e.g.
// GPT-2-XL's fc1 forward (18432 x 6400, 7 rounds + 2 tile rows) ran on the
// 128x128 kernel at ~250 TF/s.
bool use_big(const GemmArgs& g) {
  return g.round_chunk || g.seg_k > 0 || g.at != nullptr || g.trans_c || g.colsum != nullptr || g.rowsum != nullptr ||
         g.M % BM != 0 || g.N % BN != 0 || big_tiles(g, 256) >= 128;
}

// Block width of the 256-row kernel: 256, or 128 when the grid of 256x256
// tiles quantises badly onto the 256 CUs -- rounds of 256 tiles, a round of
// 256x128 tiles costing ~0.73 of a 256x256 round (measured, 2048 x 12288 x
// 4096).  E.g. T = 2048: 2048 x 4096 is 128 256x256 tiles, half the chip
// idle, or 256 256x128 tiles (1.2x faster, profiles/gemm_vs_hipblaslt.txt).
// gemm_set_width(128 / 256) or MIPIPE_GEMM_W forces one (A/B, tests).
int g_gemm_width = -1;  // -1: not read from the environment yet, 0: auto
int g_gemm_rounds = -1;  // MIPIPE_GEMM_ROUNDS: 0 one launch, 1 per round at K >= 4096 (default), 2 per round; -1 unread

int big_width(const GemmArgs& g) {
  if (g_gemm_width < 0) {
    const char* e = getenv("MIPIPE_GEMM_W");
    g_gemm_width = e ? atoi(e) : 0;
  }
  if (g_gemm_width == 128 || g_gemm_width == 256) return g_gemm_width;
  if (g.width == 128 || g.width == 256) return g.width;
  if (g.k_splits > 1) return 256;
  const int r256 = (big_tiles(g, 256) + 255) / 256, r128 = (big_tiles(g, 128) + 255) / 256;
  return 0.75 * r128 < 1.0 * r256 ? 128 : 256;
}

template <bool A_KC, bool B_KC, int EPI, int ACT, int PP, int W, bool EXTRA, int X = 0>
void launch_big(const GemmArgs& g, hipStream_t s) {
  constexpr int smem = big::smem_bytes<B_KC, PP, W>();
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(
        reinterpret_cast<const void*>(&big::gemm256_kernel<A_KC, B_KC, EPI, ACT, PP, W, EXTRA, X>),
        hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr_set = true;
  }
  hipLaunchKernelGGL((big::gemm256_kernel<A_KC, B_KC, EPI, ACT, PP, W, EXTRA, X>), dim3(big_tiles(g, W), g.k_splits),
                     dim3(big::kThreads), smem, s, g);
}

// The product build instantiates the default main loop only (schedule 7, the
// whole-tile ping-pong).  The A/B schedules 0-6 are compiled in only with
// -DMIPIPE_GEMM_AB (python -m mipipe.build --gemm-ab), for tools/gemm_sched_ab.py
// and the like; without it gemm_set_schedule() accepts 7 alone.
// 256-wide blocks: the 4-wave kernel (gemm4w_kernel, -DMIPIPE_GEMM_AB builds
// only: 2-11 % slower at the power cap, profiles/gemm4w_r5.txt) or the 8-wave
// one.  gemm_set_waves(4 / 8) or MIPIPE_GEMM_WAVES picks in an A/B build; the
// product build has the 8-wave kernel alone.
int g_gemm_waves = -1;
int gemm_waves() {
#ifdef MIPIPE_GEMM_AB
  if (g_gemm_waves < 0) {
    const char* e = getenv("MIPIPE_GEMM_WAVES");
    g_gemm_waves = e ? atoi(e) : 0;
  }
  return g_gemm_waves == 4 ? 4 : 8;
#else
  return 8;
#endif
}

#ifdef MIPIPE_GEMM_AB
template <bool A_KC, bool B_KC, int EPI, int ACT, bool EXTRA, int X = 0>
void launch_4w(const GemmArgs& g, hipStream_t s) {
  constexpr int smem = big::kSmemBytes;  // the epilogue's staging image (130 KiB); the main loop uses 128 KiB
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&big::gemm4w_kernel<A_KC, B_KC, EPI, ACT, EXTRA, X>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr_set = true;
  }
  hipLaunchKernelGGL((big::gemm4w_kernel<A_KC, B_KC, EPI, ACT, EXTRA, X>), dim3(big_tiles(g, 256), g.k_splits),
                     dim3(256), smem, s, g);
}
#endif

template <bool A_KC, bool B_KC, int EPI, int ACT, bool EXTRA>
void launch_big_w(const GemmArgs& g, hipStream_t s) {
  const bool narrow = big_width(g) == 128;
#ifdef MIPIPE_GEMM_AB
  if (!narrow && g.at == nullptr && gemm_waves() == 4) {
    if constexpr (A_KC && !B_KC && EPI != kEpiStoreBf16 && !EXTRA) {
      if (g.colsum != nullptr) {
        launch_4w<A_KC, B_KC, EPI, ACT, EXTRA, big::kXColsum>(g, s);
        return;
      }
    }
    launch_4w<A_KC, B_KC, EPI, ACT, EXTRA>(g, s);
    return;
  }
#endif
  if constexpr (A_KC && B_KC && EPI == kEpiStoreBf16 && !(ACT == kActGelu && EXTRA)) {
    if (g.at != nullptr) {  // forward GEMM that also writes A^T (gemm_emit_ok)
      if (narrow) launch_big<A_KC, B_KC, EPI, ACT, 4, 128, EXTRA, big::kXEmit>(g, s);
      else launch_big<A_KC, B_KC, EPI, ACT, 4, 256, EXTRA, big::kXEmit>(g, s);
      return;
    }
  }
  if constexpr (A_KC && !B_KC && EPI != kEpiStoreBf16 && !EXTRA) {
    if (g.colsum != nullptr) {  // transposed weight gradient with the bias fold
      if (narrow) launch_big<A_KC, B_KC, EPI, ACT, 4, 128, EXTRA, big::kXColsum>(g, s);
      else launch_big<A_KC, B_KC, EPI, ACT, 4, 256, EXTRA, big::kXColsum>(g, s);
      return;
    }
  }
#ifndef MIPIPE_GEMM_AB
  if (narrow) launch_big<A_KC, B_KC, EPI, ACT, 4, 128, EXTRA>(g, s);
  else launch_big<A_KC, B_KC, EPI, ACT, 4, 256, EXTRA>(g, s);
#else
  const int sc = big::gemm_sched();
  const bool pp = sc == 1 || sc == 4 || sc == 6 || ((sc == 2 || sc == 3) && (A_KC || B_KC));
  const bool lead = sc == 3 || sc == 4 || sc == 6;
  const bool half = sc == 5 || (sc == 6 && (A_KC || B_KC));
  if (sc == 7 && narrow) launch_big<A_KC, B_KC, EPI, ACT, 4, 128, EXTRA>(g, s);
  else if (sc == 7) launch_big<A_KC, B_KC, EPI, ACT, 4, 256, EXTRA>(g, s);
  else if (half && narrow) launch_big<A_KC, B_KC, EPI, ACT, 3, 128, EXTRA>(g, s);
  else if (half) launch_big<A_KC, B_KC, EPI, ACT, 3, 256, EXTRA>(g, s);
  else if (pp && lead && narrow) launch_big<A_KC, B_KC, EPI, ACT, 2, 128, EXTRA>(g, s);
  else if (pp && lead) launch_big<A_KC, B_KC, EPI, ACT, 2, 256, EXTRA>(g, s);
  else if (pp && narrow) launch_big<A_KC, B_KC, EPI, ACT, 1, 128, EXTRA>(g, s);
  else if (pp) launch_big<A_KC, B_KC, EPI, ACT, 1, 256, EXTRA>(g, s);
  else if (narrow) launch_big<A_KC, B_KC, EPI, ACT, 0, 128, EXTRA>(g, s);
  else launch_big<A_KC, B_KC, EPI, ACT, 0, 256, EXTRA>(g, s);
#endif
}

int g_gemm_group = -1;  // MIPIPE_GEMM_G: tile-rows per ordering group (A/B); -1 unread, 0 default

template <bool A_KC, bool B_KC, int EPI, int ACT>
void launch(const GemmArgs& gi, hipStream_t s) {
  if (g_gemm_group < 0) {
    const char* e = getenv("MIPIPE_GEMM_G");
    g_gemm_group = e ? atoi(e) : 0;
  }
  GemmArgs g = gi;
  if (g_gemm_group > 0) g.group_m = g_gemm_group;
  if (use_big(g)) {
    if constexpr (EPI == kEpiStoreBf16) {
      if (g.p > 0.f || g.aux != nullptr) {
        launch_big_w<A_KC, B_KC, EPI, ACT, true>(g, s);
        return;
      }
    }
    launch_big_w<A_KC, B_KC, EPI, ACT, false>(g, s);
    return;
  }
  const int blocks = (g.M / BM) * (g.N / BN);
  hipLaunchKernelGGL((gemm_kernel<A_KC, B_KC, EPI, ACT>), dim3(blocks), dim3(kThreads), kSmemBytes, s, g);
}

// C[M, N] (bf16, row stride ldc) = sum of the k_splits fp32 partials [s][M][N]
// (+ res): 8 columns per thread, 16-byte loads and stores.
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const float* __restrict__ ws, int splits, int M, int N,
                                                            int64_t ldc, const bf16_t* __restrict__ res, int64_t ldr,
                                                            bf16_t* __restrict__ C) {
  const int64_t chunks = (int64_t)M * (N / 8);
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= chunks) return;
  const int row = (int)(c / (N / 8)), col = (int)(c % (N / 8)) * 8;
  const int64_t at = (int64_t)row * N + col;
  f32x4 lo = *reinterpret_cast<const f32x4*>(ws + at);
  f32x4 hi = *reinterpret_cast<const f32x4*>(ws + at + 4);
  for (int s = 1; s < splits; ++s) {
    lo += *reinterpret_cast<const f32x4*>(ws + (int64_t)s * M * N + at);
    hi += *reinterpret_cast<const f32x4*>(ws + (int64_t)s * M * N + at + 4);
  }
  float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  const int64_t out = (int64_t)row * ldc + col;
  if (res != nullptr) {
    const bf16x8 r = *reinterpret_cast<const bf16x8*>(res + (int64_t)row * ldr + col);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += (float)r[e];
  }
  bf16x8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = (__bf16)v[e];
  *reinterpret_cast<bf16x8*>(C + out) = o;
}

// C[M, N] (fp32, row stride ldc) (+)= sum of the k_splits fp32 partials: the
// split-K reduction of a weight gradient (accumulate: into main_grad).
// trans: C[n * ldc + m] (+)= the partials' (m, n) -- a thread reduces rows
// 4 m' .. 4 m' + 3 of one column n (consecutive threads: consecutive n, so the
// partials are read in coalesced rows) and writes them as one 16-byte chunk.
__global__ void __launch_bounds__(256) splitk_reduce_f32_kernel(const float* __restrict__ ws, int splits, int M, int N,
                                                                int64_t ldc, bool accumulate, bool trans,
                                                                float* __restrict__ C) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (trans) {
    if (c >= (int64_t)(M / 4) * N) return;
    const int m = (int)(c / N) * 4, n = (int)(c % N);
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < splits; ++s) {
      const float* p = ws + (int64_t)s * M * N + (int64_t)m * N + n;
      v += f32x4{p[0], p[N], p[2 * (int64_t)N], p[3 * (int64_t)N]};
    }
    f32x4* dst = reinterpret_cast<f32x4*>(C + (int64_t)n * ldc + m);
    if (accumulate) v += *dst;
    *dst = v;
    return;
  }
  const int64_t chunks = (int64_t)M * (N / 4);
  if (c >= chunks) return;
  const int row = (int)(c / (N / 4)), col = (int)(c % (N / 4)) * 4;
  const int64_t at = (int64_t)row * N + col;
  f32x4 v = *reinterpret_cast<const f32x4*>(ws + at);
  for (int s = 1; s < splits; ++s) v += *reinterpret_cast<const f32x4*>(ws + (int64_t)s * M * N + at);
  f32x4* dst = reinterpret_cast<f32x4*>(C + (int64_t)row * ldc + col);
  if (accumulate) v += *dst;
  *dst = v;
}

// colsum[n] += the k_splits per-split column sums ws[s][n] (fixed order: deterministic).
__global__ void __launch_bounds__(256) colsum_splits_kernel(const float* __restrict__ ws, int splits, int N,
                                                            float* __restrict__ colsum) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float v = 0.f;
  for (int s = 0; s < splits; ++s) v += ws[(int64_t)s * N + n];
  colsum[n] += v;
}

int g_gemm_splitk = -1;  // MIPIPE_GEMM_SPLITK: 0 off, 1 auto (default), n >= 2 forced n ways (A/B); -1 unread

template <bool A_KC, bool B_KC, int EPI>
void launch_act(const GemmArgs& g, hipStream_t s) {
  switch (g.act) {
    case kActRelu: launch<A_KC, B_KC, EPI, kActRelu>(g, s); break;
    case kActGelu: launch<A_KC, B_KC, EPI, kActGelu>(g, s); break;
    default: launch<A_KC, B_KC, EPI, kActNone>(g, s); break;
  }
}

}  // namespace

bool gemm_set_schedule(int mode) {
#ifndef MIPIPE_GEMM_AB
  if (mode != 7) return false;
#else
  if (mode < 0 || mode > 7) return false;
#endif
  big::g_gemm_sched = mode;
  return true;
}
bool gemm_ab_build() {
#ifdef MIPIPE_GEMM_AB
  return true;
#else
  return false;
#endif
}
void gemm_set_width(int w) { g_gemm_width = w; }
void gemm_set_rounds(int on) { g_gemm_rounds = on; }
void gemm_set_waves(int w) { g_gemm_waves = w; }  // 4 takes effect in -DMIPIPE_GEMM_AB builds only
int gemm_get_waves() { return gemm_waves(); }
void gemm_set_splitk(int n) { g_gemm_splitk = n; }
int gemm_get_schedule() { return big::gemm_sched(); }

bool gemm_rowsum_ok(const GemmArgs& g) {
  return !g.a_kc && (g.epi == kEpiAccumF32 || g.epi == kEpiStoreF32) && use_big(g) && gemm_splitk_factor(g) <= 1 &&
         (g.N + big_width(g) - 1) / big_width(g) >= 16;
}

// The A^T emission is compiled into every forward variant but the GELU one
// with an extra epilogue (dropout / pre-activation output): that one would
// spill its main loop's registers (scratch reloads inside the K loop).
bool gemm_bits_ok(const GemmArgs& g) {
  // the staged EXTRA epilogue of the 256-row kernel (dropout), one launch or per-round chunks of whole tiles
  return g.epi == kEpiStoreBf16 && g.act == kActRelu && g.p > 0.f && g.k_splits <= 1 && g.N % 8 == 0 && use_big(g);
}

bool gemm_emit_ok(int act, float p, bool aux) { return !(act == kActGelu && (p > 0.f || aux)); }

bool gemm_colsum_ok(const GemmArgs& g) {
  if (g.b_kc || !g.a_kc || !(g.epi == kEpiAccumF32 || g.epi == kEpiStoreF32)) return false;
  GemmArgs b = g;
  b.k_splits = gemm_splitk_factor(g);  // as launched (split-K: per-split partials, reduced after)
  const int w = big_width(b);
  return 2 * ((g.M + big::BM - 1) / big::BM) * 128 >= w;  // 2 slices of <= 128 columns per block
}

bool gemm_supported(int64_t M, int64_t N, int64_t K) {
  // 16-byte operand chunks along M/N (I-contiguous layouts) and whole 64-deep K tiles.
  // ... and 32-bit per-lane staging offsets: a K-contiguous operand spans < 4 GiB.
  return M >= 8 && N >= 8 && K > 0 && M % 8 == 0 && N % 8 == 0 && K % BK == 0 && M < (1LL << 30) &&
         N < (1LL << 30) && M * K < (1LL << 31) && N * K < (1LL << 31);
}

// Split-K for grids that leave CUs idle while K is long: the T = 2048 LM-head
// dgrad (2048 x 4096 x 28928 = 128 256x256 tiles), GPT-2-XL's weight
// gradients (1600 x 1600 = 49 tiles, 6400 x 1600 = 175, K = 4 x 8192).
// s blocks per tile, each a contiguous share of the K-tiles, write fp32
// partials; one reduction adds them (+ the residual / into main_grad).  s
// minimises rounds(tiles * s) / s of the tile time (a round = 256 blocks, one
// per CU; a 256x256 tile at ~4.5 TFLOP/s per CU) plus the partials' HBM
// traffic, (2 s + 1) * 4 * M * N bytes at ~4 TB/s.  Plain bf16 output (no
// bias / activation / dropout / aux: those stay in the GEMM epilogue) or an
// fp32 weight gradient.
int gemm_splitk_factor(const GemmArgs& g) {
  if (g_gemm_splitk < 0) {
    const char* e = getenv("MIPIPE_GEMM_SPLITK");
    g_gemm_splitk = e ? atoi(e) : 1;
  }
  if (g_gemm_splitk == 0) return 1;
  const bool plain_bf16 = g.epi == kEpiStoreBf16 && g.act == kActNone && g.bias == nullptr && g.p <= 0.f &&
                          g.aux == nullptr && g.dact_in == nullptr;
  const bool f32_out = g.epi == kEpiAccumF32 || g.epi == kEpiStoreF32;
  if (!(plain_bf16 || f32_out) || !use_big(g) || g.K < 8192) return 1;
  const int tiles = big_tiles(g, 256);
  const int kt = g.K / BK;
  if (g_gemm_splitk >= 2) return std::max(1, std::min(g_gemm_splitk, kt / 16));  // forced (gemm_set_splitk, A/B)
  const double t_tile = 2.0 * 256 * 256 * (double)g.K / 4.5e12;
  const double mn = (double)g.M * g.N;
  int best = 1;
  double best_t = (double)((tiles + 255) / 256) * t_tile;
  for (int sp = 2; sp <= 8 && kt / sp >= 16; ++sp) {
    const double t = (double)((tiles * sp + 255) / 256) * t_tile / sp + (2.0 * sp + 1.0) * 4.0 * mn / 4.0e12;
    if (t < 0.97 * best_t) {
      best = sp;
      best_t = t;
    }
  }
  return best;
}

// Grids of several rounds whose last round is at most half full -- and whose
// K is >= 4096 (below) -- are launched one round of tiles at a time: the LM head (4096 x 28928 x 4096, 1808 tiles =
// 7 rounds + 16 tiles) 812 -> 786 us, 2048 x 12288 x 4096 (384 tiles) 176 ->
// 167 us (hipBLASLt's time).  Whole rounds (4096 x 12288: 768 tiles, 292 vs
// 296 us) and a last round over half full (2048 x 28928: 904 tiles, 407 vs
// 415 us) stay one launch (tools/gemm_rounds_probe.py, warm clocks, arms
// alternated).  The grid is cut along its longer tile dimension into chunks of
// floor(256 / other) tiles.

static const char* byte_off(const void* p, int64_t bytes) {
  return p == nullptr ? nullptr : reinterpret_cast<const char*>(p) + bytes;
}

template <typename F>
bool launch_by_rounds(const GemmArgs& g, F&& run) {
  if (g_gemm_rounds < 0) {
    const char* e = getenv("MIPIPE_GEMM_ROUNDS");
    g_gemm_rounds = e ? atoi(e) : 1;
  }
  if (g_gemm_rounds == 0 || g.k_splits > 1 || !use_big(g) || big_width(g) != 256) return false;
  // short main loops (K < 4096: GPT-2-XL's K = 1600 GEMMs) go as ONE launch: a CU
  // that finishes its tile starts the next round's while the others store, so
  // the fixed per-tile prologue / epilogue overlaps across rounds (GPT-2-XL PP=1
  // 64.7-64.8k -> 66.2-66.3k tok/s on one box; enc12, all K = 4096: unchanged)
  if (g_gemm_rounds == 1 && g.K < 4096) return false;
  const int tm = (g.M + 255) / 256, tn = (g.N + 255) / 256;
  // only when the last round is at most half full (see above)
  if (tm * tn <= 256 || (tm * tn) % 256 == 0 || (tm * tn) % 256 > 128) return false;
  const bool along_n = tn >= tm;
  if (along_n && g.rowsum != nullptr) return false;  // the row slices need every tile column of a tile row
  if (!along_n && g.colsum != nullptr) return false;  // the column slices need every tile row of a tile column
  const int other = along_n ? tm : tn, along = along_n ? tn : tm;
  const int per = 256 / other;  // tiles of the split dimension per launch
  if (per < 1 || (along + per - 1) / per > 16) return false;
  const int cbytes = g.epi == kEpiStoreBf16 ? 2 : 4;
  for (int t0 = 0; t0 < along; t0 += per) {
    GemmArgs c = g;
    c.round_chunk = true;
    c.width = 256;  // the full grid's width: the rowsum fold's slices assume its tile-column count
    const int lo = t0 * 256, hi = std::min((t0 + per) * 256, along_n ? g.N : g.M);
    c.mask_ld = g.mask_ld > 0 ? g.mask_ld : g.N;
    if (along_n) {
      c.N = hi - lo;
      c.mask_col0 = g.mask_col0 + lo;
      const int64_t boff = (g.b_kc ? (int64_t)lo * g.ldb : (int64_t)lo) * 2;
      c.B = byte_off(g.B, boff);
      for (int i = 0; i < GemmArgs::kMaxSegs; ++i) c.b_seg[i] = byte_off(g.b_seg[i], boff);
      c.C = const_cast<char*>(byte_off(g.C, (g.trans_c ? (int64_t)lo * g.ldc : (int64_t)lo) * cbytes));
      if (g.colsum != nullptr) c.colsum = g.colsum + lo;
      if (t0 > 0) c.at = nullptr;  // every chunk holds the whole A: the first one emits A^T
      c.bias = byte_off(g.bias, (int64_t)lo * 2);
      c.aux = const_cast<char*>(byte_off(g.aux, (int64_t)lo * 2));
      c.res = byte_off(g.res, (int64_t)lo * 2);
      c.dact_in = byte_off(g.dact_in, g.dact == kActReluBits ? (int64_t)lo / 8 : (int64_t)lo * 2);
      c.bits = const_cast<char*>(byte_off(g.bits, (int64_t)lo / 8));
    } else {
      c.M = hi - lo;
      c.mask_row0 = g.mask_row0 + lo;
      if (g.rowsum != nullptr) c.rowsum = g.rowsum + lo;
      const int64_t aoff = (g.a_kc ? (int64_t)lo * g.lda : (int64_t)lo) * 2;
      c.A = byte_off(g.A, aoff);
      for (int i = 0; i < GemmArgs::kMaxSegs; ++i) c.a_seg[i] = byte_off(g.a_seg[i], aoff);
      c.C = const_cast<char*>(byte_off(g.C, (g.trans_c ? (int64_t)lo : (int64_t)lo * g.ldc) * cbytes));
      c.at = const_cast<char*>(byte_off(g.at, (int64_t)lo * 2));  // A^T columns of this chunk's rows
      c.aux = const_cast<char*>(byte_off(g.aux, (int64_t)lo * g.ldc * 2));
      c.res = byte_off(g.res, (int64_t)lo * g.ldr * 2);
      c.dact_in = byte_off(g.dact_in, (int64_t)lo * g.ldd * (g.dact == kActReluBits ? 1 : 2));
      c.bits = const_cast<char*>(byte_off(g.bits, (int64_t)lo * g.ldbits));
    }
    run(c);
  }
  return true;
}

void gemm_bf16(const GemmArgs& gi, hipStream_t s) {
  GemmArgs g = gi;
  g.threshold = dropout_threshold(g.p);
  if (g.ldr == 0) g.ldr = g.ldc;
  if (g.ldd == 0) g.ldd = g.ldc;
  if (g.k_splits > 1) {
    // fp32 partials into the caller's workspace, then one reduction (+ res)
    GemmArgs p = g;
    p.epi = kEpiStoreF32;
    p.C = g.ws;
    p.ldc = g.N;
    p.res = nullptr;
    p.trans_c = false;  // partials row-major; the reduction transposes
    p.rowsum = nullptr;
    p.colsum = g.colsum != nullptr ? g.colsum_ws : nullptr;  // per-split column sums [k_splits][N]
    if (p.a_kc && p.b_kc) launch<true, true, kEpiStoreF32, kActNone>(p, s);
    else if (p.a_kc && !p.b_kc) launch<true, false, kEpiStoreF32, kActNone>(p, s);
    else if (!p.a_kc && !p.b_kc) launch<false, false, kEpiStoreF32, kActNone>(p, s);
    else launch<false, true, kEpiStoreF32, kActNone>(p, s);
    if (g.epi == kEpiStoreBf16) {
      const int64_t chunks = (int64_t)g.M * (g.N / 8);
      hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((chunks + 255) / 256)), dim3(256), 0, s, g.ws,
                         g.k_splits, g.M, g.N, g.ldc, reinterpret_cast<const bf16_t*>(g.res), g.ldr,
                         reinterpret_cast<bf16_t*>(g.C));
    } else {
      const int64_t chunks = (int64_t)g.M * (g.N / 4);  // = (M / 4) * N items when transposed
      hipLaunchKernelGGL(splitk_reduce_f32_kernel, dim3((unsigned)((chunks + 255) / 256)), dim3(256), 0, s, g.ws,
                         g.k_splits, g.M, g.N, g.ldc, g.epi == kEpiAccumF32, g.trans_c,
                         reinterpret_cast<float*>(g.C));
      if (g.colsum != nullptr)
        hipLaunchKernelGGL(colsum_splits_kernel, dim3((unsigned)((g.N + 255) / 256)), dim3(256), 0, s, g.colsum_ws,
                           g.k_splits, g.N, g.colsum);
    }
    return;
  }
  auto dispatch = [s](const GemmArgs& g) {
    if (g.epi == kEpiStoreBf16) {
      if (g.a_kc && g.b_kc) launch_act<true, true, kEpiStoreBf16>(g, s);
      else if (g.a_kc && !g.b_kc) launch_act<true, false, kEpiStoreBf16>(g, s);
      else if (!g.a_kc && !g.b_kc) launch_act<false, false, kEpiStoreBf16>(g, s);
      else launch_act<false, true, kEpiStoreBf16>(g, s);
    } else if (g.epi == kEpiAccumF32) {
      if (g.a_kc && g.b_kc) launch<true, true, kEpiAccumF32, kActNone>(g, s);
      else if (g.a_kc && !g.b_kc) launch<true, false, kEpiAccumF32, kActNone>(g, s);
      else if (!g.a_kc && !g.b_kc) launch<false, false, kEpiAccumF32, kActNone>(g, s);
      else launch<false, true, kEpiAccumF32, kActNone>(g, s);
    } else {
      if (g.a_kc && g.b_kc) launch<true, true, kEpiStoreF32, kActNone>(g, s);
      else if (g.a_kc && !g.b_kc) launch<true, false, kEpiStoreF32, kActNone>(g, s);
      else if (!g.a_kc && !g.b_kc) launch<false, false, kEpiStoreF32, kActNone>(g, s);
      else launch<false, true, kEpiStoreF32, kActNone>(g, s);
    }
  };
  if (!launch_by_rounds(g, dispatch)) dispatch(g);
}

}  // namespace mipipe
