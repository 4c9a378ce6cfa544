// Experimental 4-wave GEMM main loop: a 256x256x64
// block tile computed by 4 waves, one per SIMD, each owning a 128x128 output
// tile (8x8 v_mfma_f32_16x16x32_bf16 accumulators, 256 registers -- AGPRs),
// against the product kernel's 8 waves x 128x64 (two waves per SIMD in
// ping-pong).  LDS bytes read per MFMA: (128+128)/(128*128) vs (128+64)/(128*64)
// of the k extent -- a third less.  LDS latency is hidden inside the wave by
// software pipelining: the fragments of the next 32-deep k-step are read while
// the 64 MFMAs of this one issue; operand tiles are staged by LDS-DMA two
// K-tiles ahead; one barrier per K-tile.
//
// Forward layout only (A [M, K], B [N, K], both K-contiguous; C = A B^T bf16).
// Standalone harness: correctness on sampled elements vs a CPU fp32 dot
// product, then a K sweep (time per K-tile round = main-loop rate) against the
// same sweep of a one-barrier 8-wave reference written the same way.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/micro/gemm4w.hip -o tools/micro/bin/gemm4w
//   tools/micro/bin/gemm4w [M N]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <vector>
#include <string.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1); } } while (0)

typedef uint16_t bf16_t;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int kTile = BM * BK * 2;  // 32 KiB per operand tile
constexpr int kBuf = 2 * kTile;     // A + B

// K-contiguous image [256 rows][64 k]: 128-byte rows, 16-byte chunk c of row r
// at chunk c ^ ((r >> 1) & 7).
__device__ __forceinline__ int kc_off(int r, int c16) { return r * 128 + ((c16 ^ ((r >> 1) & 7)) << 4); }

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

__device__ __forceinline__ void glds16(const char* base, uint32_t off, const char* lds_dst) {
  const uint32_t m0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) const char*)lds_dst);
  asm volatile(
      "s_mov_b32 m0, %0\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %2"
      :
      : "s"(m0), "v"(off), "s"(base)
      : "memory", "m0");
}

// Per-lane source offsets of piece p (rows 8p..8p+7 of a K-contiguous tile).
__device__ __forceinline__ uint32_t piece_off(int64_t ld, int i0, int lim, int p, int lane) {
  const int row = 8 * p + (lane >> 3);
  const int c = (lane & 7) ^ ((row >> 1) & 7);
  const int gi = min(i0 + row, lim - 1);
  return (uint32_t)(((int64_t)gi * ld + 8 * c) * 2);
}

// I-contiguous image [64 rows (k)][256 i]: 512-byte rows, 8-byte chunk c of row
// r at chunk c ^ (4 rk(r)), rk(r) = (r & 3) | (((r >> 3) & 1) << 2).
__device__ __forceinline__ int ic_rk(int r) { return (r & 3) | (((r >> 3) & 1) << 2); }
__device__ __forceinline__ int ic_off(int r, int c8) { return r * 512 + ((c8 ^ (ic_rk(r) << 2)) << 3); }

// Per-lane source offsets of piece p of an I-contiguous tile (2 k-rows of 256).
__device__ __forceinline__ uint32_t piece_off_ic(int64_t ld, int i0, int lim, int p, int lane) {
  const int row = 2 * p + (lane >> 5);
  const int c16 = (lane & 31) ^ (ic_rk(row) << 1);
  const int gi = min(i0 + 8 * c16, lim - 8);
  return (uint32_t)(((int64_t)row * ld + gi) * 2);
}

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

template <bool KC>
__device__ __forceinline__ bf16x8 frag(const char* tile, int ib, int s, int lane) {
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
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  }
}

#define SB() __builtin_amdgcn_sched_barrier(0)

// Interleave pattern of the interleaved schedules (all but 1): k-step 0 issues
// fragment read q after MFMA R0 q + O0; k-step 1 issues DMA d after MFMA D1 d + OD
// and read q after MFMA R1 q + O1 (MFMAs numbered 0-63 per k-step).
template <int S> struct Sch { static constexpr int R0 = 4, O0 = 3, R1 = 4, O1 = 3, D1 = 4, OD = 1; };
template <> struct Sch<2> { static constexpr int R0 = 3, O0 = 0, R1 = 4, O1 = 3, D1 = 4, OD = 1; };
template <> struct Sch<3> { static constexpr int R0 = 3, O0 = 0, R1 = 3, O1 = 1, D1 = 4, OD = 0; };
template <> struct Sch<4> { static constexpr int R0 = 2, O0 = 0, R1 = 4, O1 = 2, D1 = 4, OD = 0; };

// ---------------------------------------------------------------------------
// 4 waves, 128x128 per wave.  SCHED selects the interleave pattern.
template <int SCHED, bool B_KC>
__global__ void __launch_bounds__(256, 1) gemm4w(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                 bf16_t* __restrict__ C, int M, int N, int K) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  int tm, tn;
  tile_coords(M / BM, N / BN, tm, tn);
  tm = __builtin_amdgcn_readfirstlane(tm);
  tn = __builtin_amdgcn_readfirstlane(tn);
  const int m0 = tm * BM, n0 = tn * BN;
  // 64 pieces of 1 KiB per K-tile (32 A, 32 B); wave w stages A pieces 8w..8w+7 and B pieces 8w..8w+7
  uint32_t offA[8], offB[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    offA[u] = piece_off(K, m0, M, 8 * wave + u, lane);
    offB[u] = B_KC ? piece_off(K, n0, N, 8 * wave + u, lane) : piece_off_ic(N, n0, N, 8 * wave + u, lane);
  }
  const char* Ab = reinterpret_cast<const char*>(A);
  const char* Bb = reinterpret_cast<const char*>(B);
  auto stageA = [&](int kt, char* buf, int u) { glds16(Ab + (int64_t)kt * BK * 2, offA[u], buf + (8 * wave + u) * 1024); };
  auto stageB = [&](int kt, char* buf, int u) {
    glds16(Bb + (B_KC ? (int64_t)kt * BK * 2 : (int64_t)kt * BK * N * 2), offB[u], buf + kTile + (8 * wave + u) * 1024);
  };
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = K / BK;
  // prologue: tiles 0 and 1
#pragma unroll
  for (int u = 0; u < 8; ++u) { stageA(0, smem, u); stageB(0, smem, u); }
  if (nk > 1) {
#pragma unroll
    for (int u = 0; u < 8; ++u) { stageA(1, smem + kBuf, u); stageB(1, smem + kBuf, u); }
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  bf16x8 fa[2][8], fb[2][8];  // [k-step parity][tile]
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    fa[0][i] = frag<true>(smem, wm * 128 + 16 * i, 0, lane);
    fb[0][i] = frag<B_KC>(smem + kTile, wn * 128 + 16 * i, 0, lane);
  }
  for (int u = 0; u < nk; ++u) {
    char* cur = smem + (u & 1) * kBuf;
    char* nxt = smem + ((u + 1) & 1) * kBuf;
    // ---- k-step 0: MFMAs on fa/fb[0], reads of k-step 1 of this tile ----
    SB();
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0][i], fb[0][j], acc[i][j], 0, 0, 0);
        if (SCHED != 1) {
          // fragment read q after MFMA R0 q + O0 (Sch<SCHED>)
          const int g = 8 * i + j;
          if (g % Sch<SCHED>::R0 == Sch<SCHED>::O0 && g / Sch<SCHED>::R0 < 16) {
            const int q = g / Sch<SCHED>::R0;  // 0..15: A0, B0-B7, A1-A7
            const int ia = q == 0 ? 0 : q - 8;
            if (q == 0 || q > 8) fa[1][ia] = frag<true>(cur, wm * 128 + 16 * ia, 1, lane);
            else fb[1][q - 1] = frag<B_KC>(cur + kTile, wn * 128 + 16 * (q - 1), 1, lane);
          }
          SB();
        }
      }
    }
    if (SCHED == 1) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        fa[1][q] = frag<true>(cur, wm * 128 + 16 * q, 1, lane);
        fb[1][q] = frag<B_KC>(cur + kTile, wn * 128 + 16 * q, 1, lane);
      }
    }
    // all reads of `cur` retired and this wave's DMAs of tile u+1 landed, then
    // the barrier: after it `cur` may be restaged and `nxt` read
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    SB();
    __builtin_amdgcn_s_barrier();
    SB();
    const bool more = u + 1 < nk, lead = u + 2 < nk;
    const int kl2 = lead ? u + 2 : nk - 1;
    // ---- k-step 1: MFMAs on fa/fb[1], reads of k-step 0 of tile u+1, DMA of tile u+2 ----
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[1][i], fb[1][j], acc[i][j], 0, 0, 0);
        if (SCHED != 1) {
          const int g = 8 * i + j;  // 0..63
          if (g % Sch<SCHED>::D1 == Sch<SCHED>::OD && g / Sch<SCHED>::D1 < 16) {  // 16 DMAs (past the last tile: a harmless restage)
            const int d = g / Sch<SCHED>::D1;
            if (d < 8) stageA(kl2, cur, d);
            else stageB(kl2, cur, d - 8);
          }
          if (g % Sch<SCHED>::R1 == Sch<SCHED>::O1 && g / Sch<SCHED>::R1 < 16) {  // 16 reads (past the last tile: harmless)
            const int q = g / Sch<SCHED>::R1, ia = q == 0 ? 0 : q - 8;
            if (q == 0 || q > 8) fa[0][ia] = frag<true>(nxt, wm * 128 + 16 * ia, 0, lane);
            else fb[0][q - 1] = frag<B_KC>(nxt + kTile, wn * 128 + 16 * (q - 1), 0, lane);
          }
          SB();
        }
      }
    }
    if (SCHED == 1) {
      if (lead) {
#pragma unroll
        for (int d = 0; d < 8; ++d) { stageA(u + 2, cur, d); stageB(u + 2, cur, d); }
      }
      if (more) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          fa[0][q] = frag<true>(nxt, wm * 128 + 16 * q, 0, lane);
          fb[0][q] = frag<B_KC>(nxt + kTile, wn * 128 + 16 * q, 0, lane);
        }
      }
    }
    SB();
  }
  // epilogue: bf16 through LDS, [256][256] image (no pad), 16-byte row stores
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  bf16_t* img = reinterpret_cast<bf16_t*>(smem);
  const int quad = lane >> 4, col = lane & 15;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * 128 + 16 * i + 4 * quad + r, c = wn * 128 + 16 * j + col;
        const __bf16 v = (__bf16)acc[i][j][r];
        img[row * 256 + c] = __builtin_bit_cast(bf16_t, v);
      }
  __syncthreads();
#pragma unroll 4
  for (int u = 0; u < 256 * 32 / 256; ++u) {
    const int idx = tid + 256 * u;
    const int row = idx >> 5, c8 = idx & 31;
    *reinterpret_cast<uint4*>(C + (int64_t)(m0 + row) * N + n0 + 8 * c8) =
        *reinterpret_cast<const uint4*>(img + row * 256 + 8 * c8);
  }
}

// ---------------------------------------------------------------------------
static float bf2f(bf16_t v) {
  uint32_t u = (uint32_t)v << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}
static bf16_t f2bf(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  u += 0x7FFF + ((u >> 16) & 1);
  return (bf16_t)(u >> 16);
}

template <int SCHED, bool B_KC>
static float run(const bf16_t* dA, const bf16_t* dB, bf16_t* dC, int M, int N, int K, int iters) {
  auto kern = gemm4w<SCHED, B_KC>;
  CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * kBuf));
  dim3 grid((M / BM) * (N / BN)), block(256);
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(kern, grid, block, 2 * kBuf, 0, dA, dB, dC, M, N, K);
  CK(hipGetLastError());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  for (int w = 0; w < iters; ++w) hipLaunchKernelGGL(kern, grid, block, 2 * kBuf, 0, dA, dB, dC, M, N, K);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3f / iters;
}

template <int SCHED, bool B_KC>
static bool check(const std::vector<bf16_t>& hA, const std::vector<bf16_t>& hB, const bf16_t* dA, const bf16_t* dB,
                  bf16_t* dC, int M, int N, int K) {
  run<SCHED, B_KC>(dA, dB, dC, M, N, K, 1);
  CK(hipDeviceSynchronize());
  std::vector<bf16_t> hC((size_t)M * N);
  CK(hipMemcpy(hC.data(), dC, hC.size() * 2, hipMemcpyDeviceToHost));
  srand(7);
  double worst = 0;
  int bad = 0;
  for (int t = 0; t < 4000; ++t) {
    const int i = (t < 16) ? (t * 97) % M : rand() % M, j = (t < 16) ? (t * 131) % N : rand() % N;
    double ref = 0;
    for (int k = 0; k < K; ++k)
      ref += (double)bf2f(hA[(size_t)i * K + k]) * bf2f(B_KC ? hB[(size_t)j * K + k] : hB[(size_t)k * N + j]);
    const double got = bf2f(hC[(size_t)i * N + j]);
    const double err = fabs(got - ref) / (fabs(ref) + 1.0);
    if (err > worst) worst = err;
    if (err > 2e-2) {
      if (bad < 5) printf("  mismatch (%d,%d): got %f ref %f\n", i, j, got, ref);
      ++bad;
    }
  }
  printf("check sched %d B_%s %dx%dx%d: %s (worst rel err %.2e)\n", SCHED, B_KC ? "KC" : "IC", M, N, K,
         bad ? "FAIL" : "ok", worst);
  return bad == 0;
}

// arm v: schedule {0, 2, 3, 4}[v % 4], B K-contiguous for v < 4 (forward layout) else I-contiguous (dgrad)
static const int kSched[4] = {0, 2, 3, 4};
static float run_arm(int v, const bf16_t* dA, const bf16_t* dB, bf16_t* dC, int M, int N, int K, int it) {
  switch (v) {
    case 0: return run<0, true>(dA, dB, dC, M, N, K, it);
    case 1: return run<2, true>(dA, dB, dC, M, N, K, it);
    case 2: return run<3, true>(dA, dB, dC, M, N, K, it);
    case 3: return run<4, true>(dA, dB, dC, M, N, K, it);
    case 4: return run<0, false>(dA, dB, dC, M, N, K, it);
    case 5: return run<2, false>(dA, dB, dC, M, N, K, it);
    case 6: return run<3, false>(dA, dB, dC, M, N, K, it);
    default: return run<4, false>(dA, dB, dC, M, N, K, it);
  }
}

int main(int argc, char** argv) {
  const int M = argc > 2 ? atoi(argv[1]) : 8192, N = argc > 2 ? atoi(argv[2]) : 4096;

  const int Kmax = 8192;
  std::vector<bf16_t> hA((size_t)M * Kmax), hB((size_t)N * Kmax);
  srand(1);
  for (auto& v : hA) v = f2bf((rand() / (float)RAND_MAX - 0.5f));
  for (auto& v : hB) v = f2bf((rand() / (float)RAND_MAX - 0.5f));
  bf16_t *dA, *dB, *dC;
  CK(hipMalloc(&dA, hA.size() * 2));
  CK(hipMalloc(&dB, hB.size() * 2));
  CK(hipMalloc(&dC, (size_t)M * N * 2));
  CK(hipMemcpy(dA, hA.data(), hA.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, hB.data(), hB.size() * 2, hipMemcpyHostToDevice));
  if (argc > 4) {  // gemm4w M N <variant 0-3> <K> [iters]: one arm only (PMC runs)
    const int v = atoi(argv[3]), K = atoi(argv[4]), it = argc > 5 ? atoi(argv[5]) : 50;
    const float t = run_arm(v, dA, dB, dC, M, N, K, it);
    printf("variant %d %dx%dx%d: %.1f us (%.0f TF/s)\n", v, M, N, K, t, 2.0 * M * N * K / t / 1e6);
    return 0;
  }
  // correctness at K = 4096: A [M][K]; B [N][K] (KC) or [K][N] (IC) -- the first N*K elements either way
  bool ok = true;
  {
    const int K = 4096;
    std::vector<bf16_t> a((size_t)M * K), b((size_t)N * K);
    for (size_t i = 0; i < a.size(); ++i) a[i] = hA[i];
    for (size_t i = 0; i < b.size(); ++i) b[i] = hB[i];
    ok &= check<0, true>(a, b, dA, dB, dC, M, N, K);
    ok &= check<2, true>(a, b, dA, dB, dC, M, N, K);
    ok &= check<3, true>(a, b, dA, dB, dC, M, N, K);
    ok &= check<4, true>(a, b, dA, dB, dC, M, N, K);
    ok &= check<0, false>(a, b, dA, dB, dC, M, N, K);
    ok &= check<2, false>(a, b, dA, dB, dC, M, N, K);
    ok &= check<3, false>(a, b, dA, dB, dC, M, N, K);
    ok &= check<4, false>(a, b, dA, dB, dC, M, N, K);
  }
  if (!ok) return 1;
  const int rounds = (M / BM) * (N / BN) / 256;
  printf("%dx%d (%d tiles, %d rounds of 256): us per launch (TF/s)\n", M, N, (M / BM) * (N / BN), rounds);
  printf("   K");
  for (int v = 0; v < 8; ++v) printf("   %s s%d", v < 4 ? "fwd" : "dgr", kSched[v % 4]);
  printf("   (us per launch)\n");
  float t[8][4];
  int ks[4] = {1024, 2048, 4096, 8192};
  for (int r = 0; r < 4; ++r) {
    const int K = ks[r];
    for (int v = 0; v < 8; ++v) t[v][r] = run_arm(v, dA, dB, dC, M, N, K, 20);
    printf("%5d", K);
    for (int v = 0; v < 8; ++v) printf("  %8.1f", t[v][r]);
    printf("\n");
  }
  for (int v = 0; v < 8; ++v) {
    double sx = 0, sy = 0, sxx = 0, sxy = 0;
    for (int r = 0; r < 4; ++r) {
      const double x = ks[r] / 1024.0, y = t[v][r];
      sx += x; sy += y; sxx += x * x; sxy += x * y;
    }
    const double slope = (4 * sxy - sx * sy) / (4 * sxx - sx * sx), icpt = (sy - slope * sx) / 4;
    printf("%s sched%d fit: fixed %.1f us + %.2f us per 1k K (%.2f per round)  main loop %.0f TF/s\n",
           v < 4 ? "fwd  " : "dgrad", kSched[v % 4], icpt, slope, slope / (rounds > 0 ? rounds : 1),
           2.0 * M * N * 1024 / slope / 1e6);
  }
  return 0;
}
