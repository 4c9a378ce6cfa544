// fp32 flash attention for gfx950 on v_mfma_f32_32x32x2_f32 (SURVEY §2.3 K2/K3
// in the reference's own precision: main.py runs fp32, S = 128, head dim 64).
//
// Everything is built around the 32x32 accumulator layout of the MFMA:
// register r of lane l holds (row (r&3) + 8(r>>2) + 4(l>>5), column l&31), and
// a following MFMA can take an accumulator tile directly as its B operand
// when it sums over the tile's ROW index (k-step s of lane half h <-> row
// (s&3) + 8(s>>2) + 4h): no LDS round trip for P.  So each kernel picks the
// orientation in which the next product reduces over rows:
//
//   forward (per 32 queries):   S^T = K Q^T  (rows keys, cols queries)
//                               O^T += V^T P^T            (reduces over keys)
//   dQ      (per 32 queries):   S^T, dP^T = V dO^T, dS^T, dQ^T += K^T dS^T
//   dK, dV  (per 32 keys):      S = Q K^T   (rows queries, cols keys)
//                               dV^T += dO^T P,  dK^T += Q^T dS   (reduce over queries)
//
// Softmax statistics live per lane (forward / dQ: the query is the column)
// or are broadcast from LDS (dK/dV).  The running max / sum of a query
// combine the two lane halves with one cross-half shuffle.
//
// Operands are staged in LDS as [32 rows][D] fp32 blocks with chunk c of row
// r at c ^ ((r & 15) ^ 8 * ((r >> 2) & 1)): the float4 "row" reads (16 lanes
// of a phase on 16 rows, same chunk) and the float "column" reads (lanes
// 0-31 on row k, 32-63 on row k + 4) are both bank-conflict free.
//
// Dropout: Philox (seed, offset) from the torch generator, "key-quad" layout:
// the uniform of (query q, key k) of head bh is word (k & 3) of counter
// (bh * S/4 + k/4) * S + q -- one Philox block per 4 keys of a query in the
// forward and dQ kernels.  Masks are regenerated in backward, so activation
// recompute replays them bit-exactly.
//
// Key-length bound: with AttnArgs::kv_len = L < S (a sequence of L tokens
// zero-padded to S, the reference's short tail window) keys >= L get no
// weight (score -inf in the forward, P = 0 in the backward) and the key loops
// stop at the last block holding a valid key.
//
// Supported: fp32, S % 32 == 0, D = 64 or 128, causal or not.
#include "common.h"
#include "kernels.h"

namespace mipipe {

namespace {

constexpr int kThreads = 256;  // 4 waves, 32 rows each
constexpr float kLog2e = 1.4426950408889634f;

__device__ __forceinline__ int swz(int r) { return (r & 15) ^ (((r >> 2) & 1) << 3); }

// byte offset of float4 chunk c of row r in a [32][D] block
template <int D>
__device__ __forceinline__ int boff(int r, int c) { return (r * (D / 4) + (c ^ swz(r))) * 16; }

// accumulator row of register r in lane half h (also the k index of MFMA step r)
__device__ __forceinline__ int arow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ float f4(const float4& v, int e) { return e == 0 ? v.x : (e == 1 ? v.y : (e == 2 ? v.z : v.w)); }

__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int r = 0; r < 16; ++r) z[r] = 0.f;
  return z;
}

// Register staging of one [32 tokens][D] block (token stride ld) into LDS.
template <int D>
struct BlockStage {
  static constexpr int kN = 32 * D / 4 / kThreads;
  f32x4 v[kN];  // native vector type: HIP's float4 struct copies become memcpys that pin the array in scratch
  __device__ __forceinline__ void load(const float* base, int64_t ld, int t0, int tid) {
#pragma unroll
    for (int u = 0; u < kN; ++u) {
      const int id = tid + u * kThreads;
      const int r = id / (D / 4), c = id % (D / 4);
      v[u] = *reinterpret_cast<const f32x4*>(base + (int64_t)(t0 + r) * ld + 4 * c);
    }
  }
  __device__ __forceinline__ void store(char* blk, int tid) const {
#pragma unroll
    for (int u = 0; u < kN; ++u) {
      const int id = tid + u * kThreads;
      *reinterpret_cast<f32x4*>(blk + boff<D>(id / (D / 4), id % (D / 4))) = v[u];
    }
  }
};

// Row-operand fragments (the MFMA K index runs over d) of token `row` of a
// global [tokens][D] tensor: step s of half h holds element
// d = 32(s>>4) + 16h + 4((s>>2)&3) + (s&3).
template <int D>
__device__ __forceinline__ void load_row_frags(const float* base, int64_t ld, int row, int h, float mul,
                                               float (&f)[D / 2]) {
#pragma unroll
  for (int co = 0; co < D / 32; ++co)
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      const float4 v = *reinterpret_cast<const float4*>(base + (int64_t)row * ld + 32 * co + 16 * h + 4 * qq);
      f[16 * co + 4 * qq + 0] = v.x * mul;
      f[16 * co + 4 * qq + 1] = v.y * mul;
      f[16 * co + 4 * qq + 2] = v.z * mul;
      f[16 * co + 4 * qq + 3] = v.w * mul;
    }
}

// acc += A . B over d, A from the LDS block by rows (row li), B = frags.
template <int D>
__device__ __forceinline__ f32x16 rows_times_frags(const char* blk, int li, int h, const float (&f)[D / 2], f32x16 acc) {
#pragma unroll
  for (int co = 0; co < D / 32; ++co)
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      const float4 a = *reinterpret_cast<const float4*>(blk + boff<D>(li, 8 * co + 4 * h + qq));
#pragma unroll
      for (int e = 0; e < 4; ++e) acc = mfma(f4(a, e), f[16 * co + 4 * qq + e], acc);
    }
  return acc;
}

// out[t] += blk^T[32t + li][k] . P[k][col] over the 32 block rows k (P: an
// accumulator tile whose rows are k).
template <int D>
__device__ __forceinline__ void colsT_times_acc(const char* blk, int li, int h, const f32x16& p, f32x16 (&out)[D / 32]) {
#pragma unroll
  for (int t = 0; t < D / 32; ++t) {
    const int d = 32 * t + li;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const float a = *reinterpret_cast<const float*>(blk + boff<D>(arow(s, h), d >> 2) + (d & 3) * 4);
      out[t] = mfma(a, p[s], out[t]);
    }
    // D = 128: keep the scheduler from hoisting all D/32 x 16 LDS loads ahead
    // of the MFMAs (64 live values pushed the dK/dV kernel into scratch)
    if constexpr (D > 64) __builtin_amdgcn_sched_barrier(0);
  }
}

// Writes out^T tiles ([d rows][token cols]) as token rows of a [tokens][D] tensor.
template <int D>
__device__ __forceinline__ void store_T(float* base, int64_t ld, int token, int h, const f32x16 (&acc)[D / 32],
                                        float mul) {
#pragma unroll
  for (int t = 0; t < D / 32; ++t)
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      const int d0 = 32 * t + 8 * gq + 4 * h;
      *reinterpret_cast<float4*>(base + (int64_t)token * ld + d0) =
          make_float4(acc[t][4 * gq] * mul, acc[t][4 * gq + 1] * mul, acc[t][4 * gq + 2] * mul, acc[t][4 * gq + 3] * mul);
    }
}

// ------------------------------------------------------------------ forward
template <int D, bool CAUSAL>
__global__ void __launch_bounds__(kThreads, D <= 64 ? 2 : 1) attn_f32_fwd_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) char lds[2 * 32 * D * 4];
  char* ldsK = lds;
  char* ldsV = lds + 32 * D * 4;
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, li = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: branches on it stay scalar
  const int bh = blockIdx.y, b = bh / a.H, hh = bh % a.H;
  const int q0 = blockIdx.x * 128 + 32 * w;
  const bool active = q0 < a.S;
  const int q = min(q0 + li, a.S - 1);
  const int64_t hoff = (int64_t)b * a.sb_qkv + (int64_t)hh * a.sh_qkv;
  const float* Qb = reinterpret_cast<const float*>(a.q) + hoff;
  const float* Kb = reinterpret_cast<const float*>(a.k) + hoff;
  const float* Vb = reinterpret_cast<const float*>(a.v) + hoff;
  const float sl = a.scale * kLog2e;

  float qf[D / 2];
  load_row_frags<D>(Qb, a.ld_qkv, q, h, sl, qf);
  f32x16 o[D / 32];
#pragma unroll
  for (int t = 0; t < D / 32; ++t) o[t] = zero16();
  float m = -INFINITY, l = 0.f;
  const float pscale = a.p > 0.f ? 1.f / (1.f - a.p) : 1.f;

  const int kl = a.kv_len > 0 ? a.kv_len : a.S;  // valid keys
  const int kend = min(CAUSAL ? min(a.S, (int)blockIdx.x * 128 + 128) : a.S, (kl + 31) & ~31);
  const int nkb = kend / 32;
  BlockStage<D> sk, sv;
  sk.load(Kb, a.ld_qkv, 0, tid);
  sv.load(Vb, a.ld_qkv, 0, tid);
  sk.store(ldsK, tid);
  sv.store(ldsV, tid);
  __syncthreads();
  for (int kb = 0; kb < nkb; ++kb) {
    // unconditional (clamped) prefetch: staging registers written under a
    // branch would be demoted to scratch
    sk.load(Kb, a.ld_qkv, 32 * min(kb + 1, nkb - 1), tid);
    sv.load(Vb, a.ld_qkv, 32 * min(kb + 1, nkb - 1), tid);
    if (active && !(CAUSAL && 32 * kb > q0 + 31)) {
      f32x16 s = rows_times_frags<D>(ldsK, li, h, qf, zero16());
      float mx = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (CAUSAL && 32 * kb + arow(r, h) > q0 + li) s[r] = -INFINITY;
        if (32 * kb + arow(r, h) >= kl) s[r] = -INFINITY;  // padded key
        mx = fmaxf(mx, s[r]);
      }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mnew = fmaxf(m, mx);  // finite: key 0 is valid for every query and seen first
      const float alpha = __builtin_amdgcn_exp2f(m - mnew);
      float psum = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        s[r] = __builtin_amdgcn_exp2f(s[r] - mnew);
        psum += s[r];
      }
      psum += __shfl_xor(psum, 32, 64);
      l = l * alpha + psum;
      m = mnew;
#pragma unroll
      for (int t = 0; t < D / 32; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[t][r] *= alpha;
      if (a.p > 0.f) {
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          const int key0 = 32 * kb + 8 * gq + 4 * h;
          const uint64_t sub = ((uint64_t)bh * (uint64_t)(a.S / 4) + (uint64_t)(key0 >> 2)) * (uint64_t)a.S + (uint64_t)(q0 + li);
          const uint4 wv = Philox(a.seed, sub, a.offset).next4();
          const uint32_t ws[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) s[4 * gq + j] = ws[j] >= a.threshold ? s[4 * gq + j] * pscale : 0.f;
        }
      }
      colsT_times_acc<D>(ldsV, li, h, s, o);
    }
    __syncthreads();
    sk.store(ldsK, tid);  // the last iteration rewrites its own block: harmless, branch-free
    sv.store(ldsV, tid);
    __syncthreads();
  }
  if (active) {
    float* Ob = reinterpret_cast<float*>(a.o) + (int64_t)b * a.sb_o + (int64_t)hh * a.sh_o;
    store_T<D>(Ob, a.ld_o, q0 + li, h, o, 1.f / l);
    if (h == 0) a.lse[(int64_t)bh * a.S + q0 + li] = (m + log2f(l)) / kLog2e;
  }
}

// ------------------------------------------------------------------ delta = rowsum(dO * O)
template <int D>
__global__ void attn_f32_delta_kernel(AttnArgs a) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // over (b, h, s)
  if (idx >= (int64_t)a.B * a.H * a.S) return;
  const int s = (int)(idx % a.S);
  const int bh = (int)(idx / a.S);
  const int b = bh / a.H, hh = bh % a.H;
  const int64_t off = (int64_t)b * a.sb_o + (int64_t)hh * a.sh_o + (int64_t)s * a.ld_o;
  const float* O = reinterpret_cast<const float*>(a.o) + off;
  const float* dO = reinterpret_cast<const float*>(a.dout) + off;
  float acc = 0.f;
#pragma unroll
  for (int c = 0; c < D / 4; ++c) {
    const float4 x = *reinterpret_cast<const float4*>(O + 4 * c);
    const float4 y = *reinterpret_cast<const float4*>(dO + 4 * c);
    acc += x.x * y.x + x.y * y.y + x.z * y.z + x.w * y.w;
  }
  a.delta[idx] = acc;
}

// ------------------------------------------------------------------ dQ
template <int D, bool CAUSAL>
__global__ void __launch_bounds__(kThreads, 1) attn_f32_dq_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) char lds[2 * 32 * D * 4];
  char* ldsK = lds;
  char* ldsV = lds + 32 * D * 4;
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, li = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: branches on it stay scalar
  const int bh = blockIdx.y, b = bh / a.H, hh = bh % a.H;
  const int q0 = blockIdx.x * 128 + 32 * w;
  const bool active = q0 < a.S;
  const int q = min(q0 + li, a.S - 1);
  const int64_t hoff = (int64_t)b * a.sb_qkv + (int64_t)hh * a.sh_qkv;
  const int64_t ooff = (int64_t)b * a.sb_o + (int64_t)hh * a.sh_o;
  const float* Qb = reinterpret_cast<const float*>(a.q) + hoff;
  const float* Kb = reinterpret_cast<const float*>(a.k) + hoff;
  const float* Vb = reinterpret_cast<const float*>(a.v) + hoff;
  const float sl = a.scale * kLog2e;

  float qf[D / 2], of[D / 2];
  load_row_frags<D>(Qb, a.ld_qkv, q, h, sl, qf);
  load_row_frags<D>(reinterpret_cast<const float*>(a.dout) + ooff, a.ld_o, q, h, 1.f, of);
  const float lse2 = a.lse[(int64_t)bh * a.S + q] * kLog2e;
  const float dlt = a.delta[(int64_t)bh * a.S + q];
  const float pscale = a.p > 0.f ? 1.f / (1.f - a.p) : 1.f;
  f32x16 dq[D / 32];
#pragma unroll
  for (int t = 0; t < D / 32; ++t) dq[t] = zero16();

  const int kl = a.kv_len > 0 ? a.kv_len : a.S;  // valid keys
  const int kend = min(CAUSAL ? min(a.S, (int)blockIdx.x * 128 + 128) : a.S, (kl + 31) & ~31);
  const int nkb = kend / 32;
  BlockStage<D> sk, sv;
  sk.load(Kb, a.ld_qkv, 0, tid);
  sv.load(Vb, a.ld_qkv, 0, tid);
  sk.store(ldsK, tid);
  sv.store(ldsV, tid);
  __syncthreads();
  for (int kb = 0; kb < nkb; ++kb) {
    // unconditional (clamped) prefetch: staging registers written under a
    // branch would be demoted to scratch
    sk.load(Kb, a.ld_qkv, 32 * min(kb + 1, nkb - 1), tid);
    sv.load(Vb, a.ld_qkv, 32 * min(kb + 1, nkb - 1), tid);
    if (active && !(CAUSAL && 32 * kb > q0 + 31)) {
      f32x16 s = rows_times_frags<D>(ldsK, li, h, qf, zero16());
      f32x16 dp = rows_times_frags<D>(ldsV, li, h, of, zero16());
      uint32_t ws[16];
      if (a.p > 0.f) {
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          const int key0 = 32 * kb + 8 * gq + 4 * h;
          const uint64_t sub = ((uint64_t)bh * (uint64_t)(a.S / 4) + (uint64_t)(key0 >> 2)) * (uint64_t)a.S + (uint64_t)(q0 + li);
          const uint4 wv = Philox(a.seed, sub, a.offset).next4();
          ws[4 * gq] = wv.x; ws[4 * gq + 1] = wv.y; ws[4 * gq + 2] = wv.z; ws[4 * gq + 3] = wv.w;
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float pr = __builtin_amdgcn_exp2f(s[r] - lse2);
        if (CAUSAL && 32 * kb + arow(r, h) > q0 + li) pr = 0.f;
        if (32 * kb + arow(r, h) >= kl) pr = 0.f;  // padded key
        float d = dp[r];
        if (a.p > 0.f) d = ws[r] >= a.threshold ? d * pscale : 0.f;
        s[r] = pr * (d - dlt);  // dS^T
      }
      colsT_times_acc<D>(ldsK, li, h, s, dq);
    }
    __syncthreads();
    sk.store(ldsK, tid);  // the last iteration rewrites its own block: harmless, branch-free
    sv.store(ldsV, tid);
    __syncthreads();
  }
  if (active) {
    float* dQb = reinterpret_cast<float*>(a.dq) + hoff;
    store_T<D>(dQb, a.ld_qkv, q0 + li, h, dq, a.scale);
  }
}

// ------------------------------------------------------------------ dK, dV
// PART 0: dK and dV in one kernel (D = 64).  D = 128 runs PART 1 (dV) and
// PART 2 (dK) as two kernels: resident K and V fragments plus both
// accumulator sets exceed a lane's 512 registers (the one-kernel form spilled
// 356 B/lane); the split recomputes S = Q K^T once more instead.
template <int D, bool CAUSAL, int PART>
__global__ void __launch_bounds__(kThreads, 1) attn_f32_dkdv_kernel(AttnArgs a) {
  constexpr bool kDV = PART != 2, kDK = PART != 1;
  __shared__ __attribute__((aligned(16))) char lds[2 * 32 * D * 4 + 2 * 32 * 4];
  char* ldsQ = lds;
  char* ldsO = lds + 32 * D * 4;  // dO block
  float* ldsL = reinterpret_cast<float*>(lds + 2 * 32 * D * 4);  // lse2[32], delta[32]
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, li = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: branches on it stay scalar
  const int bh = blockIdx.y, b = bh / a.H, hh = bh % a.H;
  const int k0 = blockIdx.x * 128 + 32 * w;
  const bool active = k0 < a.S;
  const int key = min(k0 + li, a.S - 1);
  const int64_t hoff = (int64_t)b * a.sb_qkv + (int64_t)hh * a.sh_qkv;
  const int64_t ooff = (int64_t)b * a.sb_o + (int64_t)hh * a.sh_o;
  const float* Qb = reinterpret_cast<const float*>(a.q) + hoff;
  const float* dOb = reinterpret_cast<const float*>(a.dout) + ooff;
  const float sl = a.scale * kLog2e;

  float kf[D / 2], vf[kDK ? D / 2 : 1];
  load_row_frags<D>(reinterpret_cast<const float*>(a.k) + hoff, a.ld_qkv, key, h, sl, kf);
  if constexpr (kDK) load_row_frags<D>(reinterpret_cast<const float*>(a.v) + hoff, a.ld_qkv, key, h, 1.f, vf);
  const float pscale = a.p > 0.f ? 1.f / (1.f - a.p) : 1.f;
  f32x16 dk[kDK ? D / 32 : 1], dv[kDV ? D / 32 : 1];
#pragma unroll
  for (int t = 0; t < D / 32; ++t) {
    if constexpr (kDK) dk[t] = zero16();
    if constexpr (kDV) dv[t] = zero16();
  }

  const int kl = a.kv_len > 0 ? a.kv_len : a.S;  // valid keys
  const int qb0 = CAUSAL ? (int)blockIdx.x * 4 : 0;  // first query block that sees any of these keys
  const int nqb = a.S / 32;
  BlockStage<D> sq, so;
  float st_l = 0.f;
  auto gload = [&](int qb) {
    sq.load(Qb, a.ld_qkv, 32 * qb, tid);
    so.load(dOb, a.ld_o, 32 * qb, tid);
    const int qq = 32 * qb + (tid & 31);
    const float* src = (tid & 32) ? a.delta : a.lse;  // threads 0-31 lse, 32-63 delta (others unused)
    st_l = src[(int64_t)bh * a.S + qq] * ((tid & 32) ? 1.f : kLog2e);
  };
  auto lstore = [&]() {
    sq.store(ldsQ, tid);
    so.store(ldsO, tid);
    if (tid < 64) ldsL[tid] = st_l;
  };
  if (qb0 < nqb) {
    gload(qb0);
    lstore();
  }
  __syncthreads();
  for (int qb = qb0; qb < nqb; ++qb) {
    gload(min(qb + 1, nqb - 1));
    if (active && !(CAUSAL && 32 * qb + 31 < k0)) {
      f32x16 s = rows_times_frags<D>(ldsQ, li, h, kf, zero16());   // S[q][k] (log2 domain)
      f32x16 dp;                                                   // dP[q][k]
      if constexpr (kDK) dp = rows_times_frags<D>(ldsO, li, h, vf, zero16());
      f32x16 pd;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int qr = arow(r, h);
        const int qg = 32 * qb + qr;
        float pr = __builtin_amdgcn_exp2f(s[r] - ldsL[qr]);
        if (CAUSAL && k0 + li > qg) pr = 0.f;
        if (k0 + li >= kl) pr = 0.f;  // padded key: no weight, no gradient
        float keep = 1.f;
        if (a.p > 0.f) {
          const int kk = k0 + li;
          const uint64_t sub = ((uint64_t)bh * (uint64_t)(a.S / 4) + (uint64_t)(kk >> 2)) * (uint64_t)a.S + (uint64_t)qg;
          const uint4 wv = Philox(a.seed, sub, a.offset).next4();
          const int j = kk & 3;
          const uint32_t word = j == 0 ? wv.x : (j == 1 ? wv.y : (j == 2 ? wv.z : wv.w));
          keep = word >= a.threshold ? pscale : 0.f;
        }
        if constexpr (kDV) pd[r] = pr * keep;
        if constexpr (kDK) s[r] = pr * (dp[r] * keep - ldsL[32 + qr]);  // dS
      }
      if constexpr (kDV) colsT_times_acc<D>(ldsO, li, h, pd, dv);  // dV^T += dO^T P_drop
      if constexpr (kDK) colsT_times_acc<D>(ldsQ, li, h, s, dk);   // dK^T += Q^T dS
    }
    __syncthreads();
    lstore();
    __syncthreads();
  }
  if (active) {
    if constexpr (kDK) store_T<D>(reinterpret_cast<float*>(a.dk) + hoff, a.ld_qkv, k0 + li, h, dk, a.scale);
    if constexpr (kDV) store_T<D>(reinterpret_cast<float*>(a.dv) + hoff, a.ld_qkv, k0 + li, h, dv, 1.f);
  }
}

template <int D, bool CAUSAL>
void run_fwd(const AttnArgs& a, hipStream_t s) {
  const dim3 grid((a.S + 127) / 128, a.B * a.H);
  hipLaunchKernelGGL((attn_f32_fwd_kernel<D, CAUSAL>), grid, dim3(kThreads), 0, s, a);
}

template <int D, bool CAUSAL>
void run_bwd(const AttnArgs& a, hipStream_t s) {
  const int64_t rows = (int64_t)a.B * a.H * a.S;
  hipLaunchKernelGGL((attn_f32_delta_kernel<D>), dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, s, a);
  const dim3 grid((a.S + 127) / 128, a.B * a.H);
  hipLaunchKernelGGL((attn_f32_dq_kernel<D, CAUSAL>), grid, dim3(kThreads), 0, s, a);
  if constexpr (D > 64) {
    hipLaunchKernelGGL((attn_f32_dkdv_kernel<D, CAUSAL, 1>), grid, dim3(kThreads), 0, s, a);
    hipLaunchKernelGGL((attn_f32_dkdv_kernel<D, CAUSAL, 2>), grid, dim3(kThreads), 0, s, a);
  } else {
    hipLaunchKernelGGL((attn_f32_dkdv_kernel<D, CAUSAL, 0>), grid, dim3(kThreads), 0, s, a);
  }
}

}  // namespace

// D = 64 (the reference's head dim, and GPT-2's) and D = 128 (dV and dK as two kernels).
bool attention_f32_supported(int S, int D) { return S >= 32 && S % 32 == 0 && (D == 64 || D == 128); }

void attention_f32_fwd(const AttnArgs& ai, hipStream_t s) {
  AttnArgs a = ai;
  a.threshold = dropout_threshold(a.p);
  if (a.D == 128) {
    if (a.causal) run_fwd<128, true>(a, s); else run_fwd<128, false>(a, s);
  } else {
    if (a.causal) run_fwd<64, true>(a, s); else run_fwd<64, false>(a, s);
  }
}

void attention_f32_bwd(const AttnArgs& ai, hipStream_t s) {
  AttnArgs a = ai;
  a.threshold = dropout_threshold(a.p);
  if (a.D == 128) {
    if (a.causal) run_bwd<128, true>(a, s); else run_bwd<128, false>(a, s);
  } else {
    if (a.causal) run_bwd<64, true>(a, s); else run_bwd<64, false>(a, s);
  }
}

}  // namespace mipipe
