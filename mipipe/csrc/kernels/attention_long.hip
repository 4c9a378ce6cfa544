// Long-sequence flash attention for gfx950, head dim 64, bf16 (SURVEY §2.3
// K2/K3 at GPT-2-XL's shape: B 8, H 25, S 1024, D 64, causal, dropout 0.1).
//
// Built on v_mfma_f32_32x32x16_bf16 and its accumulator layout: register r of
// lane l holds (row (r&3) + 8(r>>2) + 4(l>>5), column l&31), and an
// accumulator tile is directly the A or B operand of a following MFMA that
// sums over its ROW index (k-step half h, element j <-> row 8t + j of the
// tile's k-step t; the other operand reads its k index in that same order).
// So no probability or gradient tile ever goes through LDS:
//
//   forward (a wave = 64 queries):  S^T = K Q^T   (keys in registers, query on the lane)
//                                   O  += P V     (P^T registers are the A operand)
//   dK, dV  (a wave = 64 keys; the default 8-wave kernel: 32): S = Q K^T, dP = dO V^T (key on the lane)
//                                   dV^T += dO^T P_drop,  dK^T += Q^T dS
//   dQ      (a wave = 64 queries):  S^T, dP^T = V dO^T, dQ += dS K
//
// Each wave owns two 32-row blocks of its own dimension, so every K/V (Q/dO)
// fragment read from LDS feeds two MFMAs.  64-row operand tiles are staged in
// LDS ([64][64] bf16, 128-byte rows) through registers one tile ahead, with
// 16-byte chunk c of row r at c ^ f(r), f(r) = 4((r>>1)&1) | ((r>>2)&3): the
// row reads (ds_read_b128, 16 lanes on 16 rows) and the transposing column
// reads (ds_read_b64_tr_b16, 32 lanes on 4 rows x 4 chunks) are both free of
// bank conflicts.
//
// Softmax: exp2 with the scale folded into one FMA; the running max is only
// raised when a tile's max exceeds it by more than 2^8 (then O and l are
// rescaled: a lane's query sits in the registers of the O layout, so the
// rescale factors move by ds_bpermute -- rare, not per tile); l is a per-lane
// partial sum reduced once.
//
// Dropout: the keep bits are made by their own kernel (pure VALU at full
// occupancy: the RNG no longer competes with the softmax for issue slots in
// the MFMA kernels) and stored as one 32-bit word per (head, 32-query block,
// key), bit = query % 32.  Philox4x32-10 with 16-bit uniforms: the uniform of
// (q, key) of head bh is the signed 16-bit half (q % 32) / 16 of word q % 4 of
// the block for counter ((bh * S/32 + q/32) * S + key) * 4 + (q % 16) / 4.  Forward,
// dQ and dK/dV read the bits; checkpoint recompute regenerates them.
#include "common.h"
#include "kernels.h"

namespace mipipe {

namespace {

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int D = 64;
constexpr int kThreads = 256;   // 4 waves
constexpr int kWaveRows = 64;   // rows of its own dimension per wave
constexpr int kBlockRows = 256; // per workgroup
constexpr int kTile = 64;       // streamed tile rows
constexpr int kImg = kTile * D * 2;  // 8 KiB per [64][64] bf16 image
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kRescale = 8.f;  // log2 headroom before the running max is raised

__device__ __forceinline__ int swz(int r) { return (((r >> 1) & 1) << 2) | ((r >> 2) & 3); }
__device__ __forceinline__ int ioff(int r, int c16) { return r * 128 + ((c16 ^ swz(r)) << 4); }
__device__ __forceinline__ int arow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

// Register staging of a [64][64] bf16 tile (token stride ld): 2 x 16 B per thread.
struct Stage {
  u32x4 v0, v1;
  __device__ __forceinline__ void load(const bf16_t* base, int64_t ld, int t0, int tid) {
    const int r0 = tid >> 3, c = tid & 7;
    v0 = *reinterpret_cast<const u32x4*>(base + (int64_t)(t0 + r0) * ld + 8 * c);
    v1 = *reinterpret_cast<const u32x4*>(base + (int64_t)(t0 + r0 + 32) * ld + 8 * c);
  }
  __device__ __forceinline__ void store(char* img, int tid) const {
    const int r0 = tid >> 3, c = tid & 7;
    *reinterpret_cast<u32x4*>(img + ioff(r0, c)) = v0;
    *reinterpret_cast<u32x4*>(img + ioff(r0 + 32, c)) = v1;
  }
};

// Row operand (A or B) of a 32x32x16 MFMA whose k index is d: row `row` of
// the image, k-step s (d = 16 s + 8 h + 0..7).
__device__ __forceinline__ bf16x8 row_frag(const char* img, int row, int s, int h) {
  return *reinterpret_cast<const bf16x8*>(img + ioff(row, 2 * s + h));
}

// Column operand whose k index runs over image rows: column `col` (= d),
// rows r0 + (j & 3) + 8 (j >> 2), j = 0..7 (r0 = block row + 16 t + 4 h):
// two transposing reads of 4 rows x 16 columns per 16-lane group.
__device__ __forceinline__ bf16x8 col_frag(const char* img, int r0, int col0, int lane) {
  const int i = lane & 15;
  const int row = r0 + (i >> 2);
  const int col = col0 + 4 * (i & 3);  // the 16-lane group's column base + this lane's 4-column piece
  const int o0 = ioff(row, col >> 3) + (col & 7) * 2;
  const int o1 = ioff(row + 8, col >> 3) + (col & 7) * 2;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + o0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + o1));
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

__device__ __forceinline__ f32x16 mfma(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int r = 0; r < 16; ++r) z[r] = 0.f;
  return z;
}

// 8 registers of an accumulator tile (k-step t) as a bf16 operand.
__device__ __forceinline__ bf16x8 pack8(const f32x16& v, int t) {
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (__bf16)v[8 * t + j];
  return o;
}

// The 16 keep words of the keys a lane holds in the query-on-lane layout (keys
// kk0 + arow(r, h)): 4 runs of 4 consecutive words.
__device__ __forceinline__ void load_keep_words(const uint32_t* mw, uint32_t (&wds)[16]) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const u32x4 w4 = *reinterpret_cast<const u32x4*>(mw + 8 * g);
    wds[4 * g] = w4[0]; wds[4 * g + 1] = w4[1]; wds[4 * g + 2] = w4[2]; wds[4 * g + 3] = w4[3];
  }
}

// x if bit `bit` of `word` is set, else +0: a sign-extended one-bit field is an
// all-ones / all-zeros mask (v_bfe_i32 + v_and_b32 -- no compare, no select).
__device__ __forceinline__ float keep_or_zero(float x, uint32_t word, int bit) {
  return __builtin_bit_cast(float, __builtin_bit_cast(int, x) & __builtin_amdgcn_sbfe((int)word, bit, 1));
}

__device__ __forceinline__ float bperm(float v, int src_lane) {
  return __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src_lane << 2, __builtin_bit_cast(int, v)));
}

// ------------------------------------------------------------------ keep bits
// One thread per (head, 32-query block, key) word; causal: only words with a
// query >= the key somewhere in the block.  Grid (S / 256, S / 32, B * H): no
// 64-bit division in the index math.
//
// The 32 uniforms of a word are the 16-bit halves of the 16 words r_j of four
// Philox blocks (counter 4 idx + j/4, word j%4), read as SIGNED 16-bit s: query
// bit q takes half q/16 of r_{q%16} and is dropped iff s < t - 2^15 (the same
// probability t / 2^16 as unsigned u < t).  One saturating v_pk_sub_i16 per r_j
// puts both drop flags in its sign bits 15 and 31, a rotate by 15 - j moves them
// to bits j and 16 + j, and one v_bitop3 merges them: 3 instructions per 2 bits.
typedef __attribute__((ext_vector_type(2))) short s16x2;

// Keep word `idx` = (bh * S/32 + query block) * S + key.
__device__ __forceinline__ uint32_t keep_word(const AttnArgs& a, int64_t idx) {
  const short ts = (short)((int)(a.threshold >> 16) - 32768);
  const s16x2 t2 = {ts, ts};
  uint32_t dropped = 0;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const uint4 w = Philox(a.seed, (uint64_t)idx * 4 + (uint64_t)c, a.offset).next4();
    const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = 4 * c + i;
      const uint32_t d = __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(__builtin_bit_cast(s16x2, ws[i]), t2));
      const uint32_t rot = __builtin_amdgcn_alignbit(d, d, 15 - j);  // rotate right: bit 15 -> j, bit 31 -> 16 + j
      dropped |= rot & ((1u << j) | (1u << (16 + j)));
    }
  }
  return ~dropped;
}

// Stand-alone form (attention_long_set_fused_rng(false)): the forward then reads the words.
template <bool CAUSAL>
__global__ void __launch_bounds__(256) attn_long_mask_kernel(AttnArgs a) {
  const int key = blockIdx.x * 256 + threadIdx.x;
  const int qblk = blockIdx.y;
  if (CAUSAL && (int)blockIdx.x * 256 > 32 * qblk + 31) return;  // whole block above the diagonal
  if (key >= a.S || (CAUSAL && key > 32 * qblk + 31)) return;
  const int64_t idx = ((int64_t)blockIdx.z * gridDim.y + qblk) * a.S + key;
  a.dmask[idx] = keep_word(a, idx);
}

// ------------------------------------------------------------------ forward
// Per 64-key tile: two 32-key sub-tiles, each S^T (both query blocks share the
// K fragments), softmax, P V (both share the V fragments).  K/V tiles are
// double-buffered in LDS and staged through registers one tile ahead: one
// barrier per tile.
// DM: 0 no dropout, 1 keep words read (made by attn_long_mask_kernel), 2 made here.
template <bool CAUSAL, int DM>
__global__ void __launch_bounds__(kThreads, 2) attn_long_fwd_kernel(AttnArgs a) {
  constexpr bool RNG = DM == 2;
  // K, V double-buffered + each wave's Q image + (RNG) one 128-word keep-word exchange slot per wave
  __shared__ __attribute__((aligned(16))) char lds[2 * 2 * kImg + 4 * kImg + (RNG ? 4 * 128 * 4 : 0)];
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, li = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // grid (B*H, query tiles): the query tile is the SLOW grid dimension, so under
  // causal masking every head's longest tile is dispatched before any shorter one
  const int nqt = (a.S + kBlockRows - 1) / kBlockRows;
  const int qt = CAUSAL ? nqt - 1 - (int)blockIdx.y : (int)blockIdx.y;
  const int bh = blockIdx.x, b = bh / a.H, hh = bh % a.H;
  const int q0w = qt * kBlockRows + wave * kWaveRows;  // this wave's queries q0w .. q0w + 63
  const bool active = q0w < a.S;
  const int64_t hoff = (int64_t)b * a.sb_qkv + (int64_t)hh * a.sh_qkv;
  const bf16_t* Q = reinterpret_cast<const bf16_t*>(a.q) + hoff;
  const bf16_t* K = reinterpret_cast<const bf16_t*>(a.k) + hoff;
  const bf16_t* V = reinterpret_cast<const bf16_t*>(a.v) + hoff;
  constexpr bool drop = DM != 0;
  const float pscale = drop ? 1.f / (1.f - a.p) : 1.f;
  const float sl2 = a.scale * kLog2e;

  // Q^T fragments (B operand of S^T = K Q^T): query q0w + 32 qb + li, d = 16 s + 8 h + j
  // as an LDS image of the wave's 64 queries (row = 32 qb + li), read per use: the
  // 32 registers the fragments would hold for the whole kernel go to the S tiles of
  // both key sub-tiles instead
  char* qimg_w = lds + 4 * kImg + wave * kImg;
  {
    const bf16_t* qr = Q + (int64_t)min(q0w + lane, a.S - 1) * a.ld_qkv;
#pragma unroll
    for (int c = 0; c < 8; ++c) *reinterpret_cast<u32x4*>(qimg_w + ioff(lane, c)) = *reinterpret_cast<const u32x4*>(qr + 8 * c);
  }
  f32x16 o[2][2];
  float m[2], l[2];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    o[qb][0] = zero16();
    o[qb][1] = zero16();
    m[qb] = -INFINITY;
    l[qb] = 0.f;
  }

  const int kend = CAUSAL ? min(a.S, (qt + 1) * kBlockRows) : a.S;
  const int ntiles = kend / kTile;
  Stage sk, sv;
  sk.load(K, a.ld_qkv, 0, tid);
  sv.load(V, a.ld_qkv, 0, tid);
  sk.store(lds, tid);
  sv.store(lds + kImg, tid);
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const char* kimg = lds + (t & 1) * 2 * kImg;
    const char* vimg = kimg + kImg;
    const int k0 = t * kTile;
    {  // next tile in flight (clamped: the last iteration reloads its own tile, unused)
      const int tn = min(t + 1, ntiles - 1) * kTile;
      sk.load(K, a.ld_qkv, tn, tid);
      sv.load(V, a.ld_qkv, tn, tid);
    }
    if (active && !(CAUSAL && k0 > q0w)) {  // wave-uniform: the tile meets this wave's queries
      const bool diag = CAUSAL && k0 == q0w;  // this wave's diagonal tile (k0, q0w multiples of 64)
      // S^T of both 32-key sub-tiles first: the second one's MFMAs run under the first
      // one's softmax, the first one's P V MFMAs under the second one's softmax
      f32x16 st[2][2];  // [kb][qb]: rows keys, columns queries
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        st[kb][0] = st[kb][1] = zero16();
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const bf16x8 kf = row_frag(kimg, 32 * kb + li, s, h);
#pragma unroll
          for (int qb = 0; qb < 2; ++qb) st[kb][qb] = mfma(kf, row_frag(qimg_w, 32 * qb + li, s, h), st[kb][qb]);
        }
      }
      uint32_t* wx = reinterpret_cast<uint32_t*>(lds + 8 * kImg) + wave * 128;
      if (RNG) {
        // Keep words made here, beside the S MFMAs (pure VALU, no branch between them):
        // lane (h, li) makes the word of query block q0w/32 + h and key kk0 + li, stores
        // it for the backward pass and passes it through LDS to the lanes that apply it.
        // Words above the diagonal are made but neither stored nor read.
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          const int kk0 = k0 + 32 * kb;
          const int64_t idx = ((int64_t)bh * (a.S >> 5) + (q0w >> 5) + h) * a.S + kk0 + li;
          const uint32_t w = keep_word(a, idx);
          if (!(CAUSAL && kk0 > q0w + 32 * h + 31)) a.dmask[idx] = w;
          wx[64 * kb + lane] = w;
        }
      }
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        const int kk0 = k0 + 32 * kb;
        bf16x8 pf[2][2];  // [qb][k-step]
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
          const int qrow = q0w + 32 * qb;  // block's first query
          const int q = qrow + li;
          if (diag && kb > qb) {  // wholly above this block's diagonal: P = 0
            pf[qb][0] = bf16x8{};
            pf[qb][1] = bf16x8{};
            continue;
          }
          uint32_t wds[16] = {};
          if (drop) {
            if (RNG) load_keep_words(wx + 64 * kb + 32 * qb + 4 * h, wds);
            else load_keep_words(a.dmask + ((int64_t)bh * (a.S >> 5) + (qrow >> 5)) * a.S + kk0 + 4 * h, wds);
          }
          if (diag && kb == qb) {  // diagonal sub-tile (wave-uniform branch): mask keys > query
#pragma unroll
            for (int r = 0; r < 16; ++r)
              if (kk0 + arow(r, h) > q) st[kb][qb][r] = -INFINITY;
          }
          float mx = -INFINITY;
#pragma unroll
          for (int r = 0; r < 16; ++r) mx = fmaxf(mx, st[kb][qb][r]);
          mx = fmaxf(mx, __shfl_xor(mx, 32, 64)) * sl2;
          if (__ballot(mx > m[qb] + kRescale)) {
            // raise the running max; rescale O (queries in registers there) and l
            const float mn = fmaxf(m[qb], mx);
            const float alpha = m[qb] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m[qb] - mn);
            m[qb] = mn;
            l[qb] *= alpha;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const float ar = bperm(alpha, arow(r, h));
              o[qb][0][r] *= ar;
              o[qb][1][r] *= ar;
            }
          }
          const float mq = m[qb];
          float ps = 0.f;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            float p = __builtin_amdgcn_exp2f(fmaf(st[kb][qb][r], sl2, -mq));
            ps += p;
            // dropped -> 0; the 1/(1-p) scale is applied once to O at the end
            if (drop) p = keep_or_zero(p, wds[r], li);
            st[kb][qb][r] = p;
          }
          l[qb] += ps;
          pf[qb][0] = pack8(st[kb][qb], 0);
          pf[qb][1] = pack8(st[kb][qb], 1);
        }
        // ---- O += P V for this 32-key sub-tile
#pragma unroll
        for (int st_ = 0; st_ < 2; ++st_)
#pragma unroll
          for (int dt = 0; dt < 2; ++dt) {
            const bf16x8 vf = col_frag(vimg, 32 * kb + 16 * st_ + 4 * h, 32 * dt + 16 * ((lane >> 4) & 1), lane);
#pragma unroll
            for (int qb = 0; qb < 2; ++qb) o[qb][dt] = mfma(pf[qb][st_], vf, o[qb][dt]);
          }
      }
    }
    char* nxt = lds + ((t + 1) & 1) * 2 * kImg;
    sk.store(nxt, tid);
    sv.store(nxt + kImg, tid);
    __syncthreads();
  }
  if (!active) return;
  bf16_t* O = reinterpret_cast<bf16_t*>(a.o) + (int64_t)b * a.sb_o + (int64_t)hh * a.sh_o;
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const float lt = l[qb] + __shfl_xor(l[qb], 32, 64);
    const float inv = lt > 0.f ? pscale / lt : 0.f;  // dropout scale folded into the normalisation
    const int qrow = q0w + 32 * qb;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float ir = bperm(inv, arow(r, h));
      const int q = qrow + arow(r, h);
      O[(int64_t)q * a.ld_o + li] = f2bf(o[qb][0][r] * ir);
      O[(int64_t)q * a.ld_o + 32 + li] = f2bf(o[qb][1][r] * ir);
    }
    if (h == 0) a.lse[(int64_t)bh * a.S + qrow + li] = (m[qb] + log2f(lt > 0.f ? lt : 1.f)) / kLog2e;
  }
}

// ------------------------------------------------------------------ delta = rowsum(dO * O)
__global__ void __launch_bounds__(256) attn_long_delta_kernel(AttnArgs a) {
  // 8 lanes per row (8 bf16 each)
  const int64_t row = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 3;  // over (b, s, h)
  const int part = threadIdx.x & 7;
  const int64_t rows = (int64_t)a.B * a.S * a.H;
  float acc = 0.f;
  int64_t bh_s = 0;
  if (row < rows) {
    const int hh = (int)(row % a.H);
    const int64_t bs = row / a.H;
    const int s = (int)(bs % a.S), b = (int)(bs / a.S);
    const int64_t off = (int64_t)b * a.sb_o + (int64_t)hh * a.sh_o + (int64_t)s * a.ld_o + 8 * part;
    const bf16x8 x = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const bf16_t*>(a.o) + off);
    const bf16x8 y = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const bf16_t*>(a.dout) + off);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += (float)x[j] * (float)y[j];
    bh_s = ((int64_t)b * a.H + hh) * a.S + s;
  }
  acc += __shfl_xor(acc, 1, 64);
  acc += __shfl_xor(acc, 2, 64);
  acc += __shfl_xor(acc, 4, 64);
  if (row < rows && part == 0) a.delta[bh_s] = acc;
}

// ------------------------------------------------------------------ dK, dV
template <bool CAUSAL, bool DROP>
__global__ void __launch_bounds__(kThreads, 1) attn_long_dkdv_kernel(AttnArgs a) {
  // Q, dO (x2) + lse2, delta (x2) + this workgroup's K and V (one [64][64] image per wave each)
  __shared__ __attribute__((aligned(16))) char lds[2 * 2 * kImg + 2 * 2 * kTile * 4 + 2 * 4 * kImg];
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, li = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nkt = (a.S + kBlockRows - 1) / kBlockRows;
  // grid (B*H, key tiles), key tile slow: under causal masking the first key
  // tiles see the most queries and are dispatched first
  const int kt = (int)blockIdx.y;
  const int bh = blockIdx.x, b = bh / a.H, hh = bh % a.H;
  const int k0w = kt * kBlockRows + wave * kWaveRows;  // this wave's keys
  const bool active = k0w < a.S;
  const int64_t hoff = (int64_t)b * a.sb_qkv + (int64_t)hh * a.sh_qkv;
  const int64_t ooff = (int64_t)b * a.sb_o + (int64_t)hh * a.sh_o;
  const bf16_t* Q = reinterpret_cast<const bf16_t*>(a.q) + hoff;
  const bf16_t* dO = reinterpret_cast<const bf16_t*>(a.dout) + ooff;
  constexpr bool drop = DROP;
  const float pscale = drop ? 1.f / (1.f - a.p) : 1.f;
  const float sl2 = a.scale * kLog2e;
  (void)nkt;

  // This wave's 64 keys of K and V as LDS images (row = key): the B operands of
  // S = Q K^T and dP = dO V^T are read from there per use rather than held in 64
  // registers for the whole kernel -- the register file then holds dK/dV in the
  // accumulator registers without copies between the two register files.
  char* kimg_w = lds + 4 * kImg + 4 * kTile * 4 + wave * 2 * kImg;
  char* vimg_w = kimg_w + kImg;
  {
    const int key = min(k0w + lane, a.S - 1);
    const bf16_t* kr = reinterpret_cast<const bf16_t*>(a.k) + hoff + (int64_t)key * a.ld_qkv;
    const bf16_t* vr = reinterpret_cast<const bf16_t*>(a.v) + hoff + (int64_t)key * a.ld_qkv;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      *reinterpret_cast<u32x4*>(kimg_w + ioff(lane, c)) = *reinterpret_cast<const u32x4*>(kr + 8 * c);
      *reinterpret_cast<u32x4*>(vimg_w + ioff(lane, c)) = *reinterpret_cast<const u32x4*>(vr + 8 * c);
    }
  }
  f32x16 dk[2][2], dv[2][2];  // [kb][dt]: rows d, columns keys
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      dk[kb][dt] = zero16();
      dv[kb][dt] = zero16();
    }

  const int qstart = CAUSAL ? (kt * kBlockRows) / kTile : 0;  // first query tile with q >= the block's first key
  const int ntiles = a.S / kTile;
  Stage sq, so;
  float st_l = 0.f;
  auto gload = [&](int t) {
    sq.load(Q, a.ld_qkv, t * kTile, tid);
    so.load(dO, a.ld_o, t * kTile, tid);
    if (tid < 2 * kTile) {
      const int64_t i = (int64_t)bh * a.S + t * kTile + (tid & (kTile - 1));
      st_l = tid < kTile ? a.lse[i] * kLog2e : a.delta[i];
    }
  };
  auto lstore = [&](int buf) {
    char* base = lds + buf * 2 * kImg;
    sq.store(base, tid);
    so.store(base + kImg, tid);
    if (tid < 2 * kTile) reinterpret_cast<float*>(lds + 4 * kImg)[buf * 2 * kTile + tid] = st_l;
  };
  if (qstart < ntiles) {
    gload(qstart);
    lstore(0);
  }
  __syncthreads();
  // Tiles wholly before this wave's keys (causal; all of them for an inactive
  // wave) are only staged for the others.  Splitting them into their own loop
  // leaves the compute loop without a branch around the dK/dV accumulation, so
  // those accumulators stay in the accumulator registers across iterations.
  const int tw = !active ? ntiles : (CAUSAL ? max(qstart, k0w / kTile) : qstart);
  for (int t = qstart; t < tw; ++t) {
    gload(min(t + 1, ntiles - 1));
    lstore(((t - qstart) & 1) ^ 1);
    __syncthreads();
  }
  for (int t = tw; t < ntiles; ++t) {
    const int buf = (t - qstart) & 1;
    const char* qimg = lds + buf * 2 * kImg;
    const char* oimg = qimg + kImg;
    const float* lse2 = reinterpret_cast<const float*>(lds + 4 * kImg) + buf * 2 * kTile;
    const float* dlt = lse2 + kTile;
    const int q0 = t * kTile;
    gload(min(t + 1, ntiles - 1));
    {
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        // q0 >= k0w here (both multiples of 64): no query block of the tile lies wholly before the keys
        const int qrow = q0 + 32 * qb;
        f32x16 sacc[2], dpacc[2];
        sacc[0] = sacc[1] = dpacc[0] = dpacc[1] = zero16();
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const bf16x8 qa = row_frag(qimg, 32 * qb + li, s, h);
          const bf16x8 oa = row_frag(oimg, 32 * qb + li, s, h);
#pragma unroll
          for (int kb = 0; kb < 2; ++kb) {
            sacc[kb] = mfma(qa, row_frag(kimg_w, 32 * kb + li, s, h), sacc[kb]);
            dpacc[kb] = mfma(oa, row_frag(vimg_w, 32 * kb + li, s, h), dpacc[kb]);
          }
        }
        bf16x8 pb[2][2], sb[2][2];  // [kb][step]
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          const int key = k0w + 32 * kb + li;
          uint32_t word = 0xFFFFFFFFu;
          if (drop) word = a.dmask[((int64_t)bh * (a.S >> 5) + (qrow >> 5)) * a.S + key];
          // row constants (lse, delta) of the 16 query rows this lane holds: LDS broadcasts
          float lr[16], dr[16];
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const f32x4 lv = *reinterpret_cast<const f32x4*>(lse2 + 32 * qb + 8 * g + 4 * h);
            const f32x4 dv4 = *reinterpret_cast<const f32x4*>(dlt + 32 * qb + 8 * g + 4 * h);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              lr[4 * g + j] = lv[j];
              dr[4 * g + j] = dv4[j];
            }
          }
          float pr[16];
#pragma unroll
          for (int r = 0; r < 16; ++r) pr[r] = __builtin_amdgcn_exp2f(fmaf(sacc[kb][r], sl2, -lr[r]));
          if (CAUSAL && k0w + 32 * kb + 31 > qrow) {  // diagonal sub-tile (wave-uniform branch)
#pragma unroll
            for (int r = 0; r < 16; ++r)
              if (key > qrow + arow(r, h)) pr[r] = 0.f;
          }
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            // kept: P (for dV; the 1/(1-p) is applied to dV once at the end) and
            // dS = P (dP / (1-p) - delta); dropped: P -> 0, dS = -P delta
            const float dsel = drop ? keep_or_zero(dpacc[kb][r], word, arow(r, h)) : dpacc[kb][r];
            sacc[kb][r] = drop ? keep_or_zero(pr[r], word, arow(r, h)) : pr[r];
            dpacc[kb][r] = pr[r] * (drop ? fmaf(dsel, pscale, -dr[r]) : dsel - dr[r]);
          }
          pb[kb][0] = pack8(sacc[kb], 0);
          pb[kb][1] = pack8(sacc[kb], 1);
          sb[kb][0] = pack8(dpacc[kb], 0);
          sb[kb][1] = pack8(dpacc[kb], 1);
        }
#pragma unroll
        for (int st_ = 0; st_ < 2; ++st_)
#pragma unroll
          for (int dt = 0; dt < 2; ++dt) {
            const int r0 = 32 * qb + 16 * st_ + 4 * h, c0 = 32 * dt + 16 * ((lane >> 4) & 1);
            const bf16x8 oc = col_frag(oimg, r0, c0, lane);
            const bf16x8 qc = col_frag(qimg, r0, c0, lane);
#pragma unroll
            for (int kb = 0; kb < 2; ++kb) {
              dv[kb][dt] = mfma(oc, pb[kb][st_], dv[kb][dt]);
              dk[kb][dt] = mfma(qc, sb[kb][st_], dk[kb][dt]);
            }
          }
      }
    }
    lstore(buf ^ 1);  // the other buffer: every wave left it behind the previous barrier
    __syncthreads();
  }
  if (!active) return;
  // dK^T / dV^T tiles: register r = d (32 dt + arow(r, h)), lane = key -> 4 consecutive d per 8-byte store
#pragma unroll
  for (int kb = 0; kb < 2; ++kb) {
    const int key = k0w + 32 * kb + li;
    bf16_t* dK = reinterpret_cast<bf16_t*>(a.dk) + hoff + (int64_t)key * a.ld_qkv;
    bf16_t* dV = reinterpret_cast<bf16_t*>(a.dv) + hoff + (int64_t)key * a.ld_qkv;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d0 = 32 * dt + 8 * g + 4 * h;
        bf16x4 kv, vv;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          kv[j] = (__bf16)(dk[kb][dt][4 * g + j] * a.scale);
          vv[j] = (__bf16)(dv[kb][dt][4 * g + j] * pscale);  // dropout scale of P, folded here
        }
        *reinterpret_cast<bf16x4*>(dK + d0) = kv;
        *reinterpret_cast<bf16x4*>(dV + d0) = vv;
      }
  }
}

// ------------------------------------------------------------------ dK, dV, 8 waves
// The same computation with 8 waves of 32 keys per 256-key block (512
// threads): half the accumulators per wave (dK / dV 64 registers, S / dP 32),
// so two waves share each SIMD -- the 4-wave kernel's one wave per SIMD (256
// VGPRs + ~200 AGPRs) leaves its MFMA and VALU issue mostly idle, waiting on
// its own dependency chains.  Same LDS: the Q / dO tiles double-buffered and
// each wave's [32][64] K and V images.  Query blocks wholly before a wave's
// keys (causal) are skipped.
constexpr int kThreads8 = 512;
constexpr int kImg32 = 32 * D * 2;  // [32][64] bf16

template <bool CAUSAL, bool DROP>
__global__ void __launch_bounds__(kThreads8, 2) attn_long_dkdv8_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) char lds[2 * 2 * kImg + 2 * 2 * kTile * 4 + 8 * 2 * kImg32];
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, li = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kt = (int)blockIdx.y;
  const int bh = blockIdx.x, b = bh / a.H, hh = bh % a.H;
  const int k0w = kt * kBlockRows + wave * 32;  // this wave's keys k0w .. k0w + 31
  const bool active = k0w < a.S;
  const int64_t hoff = (int64_t)b * a.sb_qkv + (int64_t)hh * a.sh_qkv;
  const int64_t ooff = (int64_t)b * a.sb_o + (int64_t)hh * a.sh_o;
  const bf16_t* Q = reinterpret_cast<const bf16_t*>(a.q) + hoff;
  const bf16_t* dO = reinterpret_cast<const bf16_t*>(a.dout) + ooff;
  constexpr bool drop = DROP;
  const float pscale = drop ? 1.f / (1.f - a.p) : 1.f;
  const float sl2 = a.scale * kLog2e;

  char* kimg_w = lds + 4 * kImg + 4 * kTile * 4 + wave * 2 * kImg32;
  char* vimg_w = kimg_w + kImg32;
  {
    const int key = min(k0w + li, a.S - 1);
    const bf16_t* kr = reinterpret_cast<const bf16_t*>(a.k) + hoff + (int64_t)key * a.ld_qkv;
    const bf16_t* vr = reinterpret_cast<const bf16_t*>(a.v) + hoff + (int64_t)key * a.ld_qkv;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = 4 * h + j;
      *reinterpret_cast<u32x4*>(kimg_w + ioff(li, c)) = *reinterpret_cast<const u32x4*>(kr + 8 * c);
      *reinterpret_cast<u32x4*>(vimg_w + ioff(li, c)) = *reinterpret_cast<const u32x4*>(vr + 8 * c);
    }
  }
  f32x16 dk[2], dv[2];  // [dt]: rows d, columns keys
#pragma unroll
  for (int dt = 0; dt < 2; ++dt) {
    dk[dt] = zero16();
    dv[dt] = zero16();
  }

  const int qstart = CAUSAL ? (kt * kBlockRows) / kTile : 0;
  const int ntiles = a.S / kTile;
  u32x4 sq, so;  // one 16-byte piece of the Q / dO tile per thread
  float st_l = 0.f;
  const int sr = tid >> 3, sc = tid & 7;
  auto gload = [&](int t) {
    sq = *reinterpret_cast<const u32x4*>(Q + (int64_t)(t * kTile + sr) * a.ld_qkv + 8 * sc);
    so = *reinterpret_cast<const u32x4*>(dO + (int64_t)(t * kTile + sr) * a.ld_o + 8 * sc);
    if (tid < 2 * kTile) {
      const int64_t i = (int64_t)bh * a.S + t * kTile + (tid & (kTile - 1));
      st_l = tid < kTile ? a.lse[i] * kLog2e : a.delta[i];
    }
  };
  auto lstore = [&](int buf) {
    char* base = lds + buf * 2 * kImg;
    *reinterpret_cast<u32x4*>(base + ioff(sr, sc)) = sq;
    *reinterpret_cast<u32x4*>(base + kImg + ioff(sr, sc)) = so;
    if (tid < 2 * kTile) reinterpret_cast<float*>(lds + 4 * kImg)[buf * 2 * kTile + tid] = st_l;
  };
  if (qstart < ntiles) {
    gload(qstart);
    lstore(0);
  }
  __syncthreads();
  const int tw = !active ? ntiles : (CAUSAL ? max(qstart, k0w / kTile) : qstart);
  for (int t = qstart; t < tw; ++t) {
    gload(min(t + 1, ntiles - 1));
    lstore(((t - qstart) & 1) ^ 1);
    __syncthreads();
  }
  for (int t = tw; t < ntiles; ++t) {
    const int buf = (t - qstart) & 1;
    const char* qimg = lds + buf * 2 * kImg;
    const char* oimg = qimg + kImg;
    const float* lse2 = reinterpret_cast<const float*>(lds + 4 * kImg) + buf * 2 * kTile;
    const float* dlt = lse2 + kTile;
    const int q0 = t * kTile;
    gload(min(t + 1, ntiles - 1));
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      const int qrow = q0 + 32 * qb;
      if (CAUSAL && qrow + 31 < k0w) continue;  // every query of the block is before the wave's keys
      f32x16 sacc = zero16(), dpacc = zero16();
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bf16x8 kb_ = row_frag(kimg_w, li, s, h);
        const bf16x8 vb_ = row_frag(vimg_w, li, s, h);
        sacc = mfma(row_frag(qimg, 32 * qb + li, s, h), kb_, sacc);
        dpacc = mfma(row_frag(oimg, 32 * qb + li, s, h), vb_, dpacc);
      }
      const int key = k0w + li;
      uint32_t word = 0xFFFFFFFFu;
      if (drop) word = a.dmask[((int64_t)bh * (a.S >> 5) + (qrow >> 5)) * a.S + key];
      float pr[16];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 lv = *reinterpret_cast<const f32x4*>(lse2 + 32 * qb + 8 * g + 4 * h);
#pragma unroll
        for (int j = 0; j < 4; ++j) pr[4 * g + j] = __builtin_amdgcn_exp2f(fmaf(sacc[4 * g + j], sl2, -lv[j]));
      }
      if (CAUSAL && k0w + 31 > qrow) {  // diagonal block (wave-uniform branch)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (key > qrow + arow(r, h)) pr[r] = 0.f;
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 dv4 = *reinterpret_cast<const f32x4*>(dlt + 32 * qb + 8 * g + 4 * h);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = 4 * g + j;
          const float dsel = drop ? keep_or_zero(dpacc[r], word, arow(r, h)) : dpacc[r];
          sacc[r] = drop ? keep_or_zero(pr[r], word, arow(r, h)) : pr[r];
          dpacc[r] = pr[r] * (drop ? fmaf(dsel, pscale, -dv4[j]) : dsel - dv4[j]);
        }
      }
      const bf16x8 pb0 = pack8(sacc, 0), pb1 = pack8(sacc, 1);
      const bf16x8 sb0 = pack8(dpacc, 0), sb1 = pack8(dpacc, 1);
#pragma unroll
      for (int st_ = 0; st_ < 2; ++st_)
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const int r0 = 32 * qb + 16 * st_ + 4 * h, c0 = 32 * dt + 16 * ((lane >> 4) & 1);
          dv[dt] = mfma(col_frag(oimg, r0, c0, lane), st_ ? pb1 : pb0, dv[dt]);
          dk[dt] = mfma(col_frag(qimg, r0, c0, lane), st_ ? sb1 : sb0, dk[dt]);
        }
    }
    lstore(buf ^ 1);
    __syncthreads();
  }
  if (!active) return;
  const int key = k0w + li;
  if (key >= a.S) return;
  bf16_t* dK = reinterpret_cast<bf16_t*>(a.dk) + hoff + (int64_t)key * a.ld_qkv;
  bf16_t* dV = reinterpret_cast<bf16_t*>(a.dv) + hoff + (int64_t)key * a.ld_qkv;
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d0 = 32 * dt + 8 * g + 4 * h;
      bf16x4 kv, vv;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        kv[j] = (__bf16)(dk[dt][4 * g + j] * a.scale);
        vv[j] = (__bf16)(dv[dt][4 * g + j] * pscale);
      }
      *reinterpret_cast<bf16x4*>(dK + d0) = kv;
      *reinterpret_cast<bf16x4*>(dV + d0) = vv;
    }
}

// ------------------------------------------------------------------ dQ
template <bool CAUSAL, bool DROP>
__global__ void __launch_bounds__(kThreads, 2) attn_long_dq_kernel(AttnArgs a) {
  // K, V double-buffered + each wave's dO image
  __shared__ __attribute__((aligned(16))) char lds[2 * 2 * kImg + 4 * kImg];
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, li = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // grid (B*H, query tiles): the query tile is the SLOW grid dimension, so under
  // causal masking every head's longest tile is dispatched before any shorter one
  const int nqt = (a.S + kBlockRows - 1) / kBlockRows;
  const int qt = CAUSAL ? nqt - 1 - (int)blockIdx.y : (int)blockIdx.y;
  const int bh = blockIdx.x, b = bh / a.H, hh = bh % a.H;
  const int q0w = qt * kBlockRows + wave * kWaveRows;
  const bool active = q0w < a.S;
  const int64_t hoff = (int64_t)b * a.sb_qkv + (int64_t)hh * a.sh_qkv;
  const int64_t ooff = (int64_t)b * a.sb_o + (int64_t)hh * a.sh_o;
  const bf16_t* K = reinterpret_cast<const bf16_t*>(a.k) + hoff;
  const bf16_t* V = reinterpret_cast<const bf16_t*>(a.v) + hoff;
  constexpr bool drop = DROP;
  const float pscale = drop ? 1.f / (1.f - a.p) : 1.f;
  const float sl2 = a.scale * kLog2e;

  // dO of the wave's 64 queries as an LDS image (row = 32 qb + li), read per use
  // (32 registers fewer than holding the fragments: no scratch)
  char* oimg_w = lds + 4 * kImg + wave * kImg;
  {
    const bf16_t* orow = reinterpret_cast<const bf16_t*>(a.dout) + ooff + (int64_t)min(q0w + lane, a.S - 1) * a.ld_o;
#pragma unroll
    for (int c = 0; c < 8; ++c)
      *reinterpret_cast<u32x4*>(oimg_w + ioff(lane, c)) = *reinterpret_cast<const u32x4*>(orow + 8 * c);
  }
  bf16x8 qf[2][4];
  float lse2[2], dlt[2];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int q = min(q0w + 32 * qb + li, a.S - 1);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      qf[qb][s] = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const bf16_t*>(a.q) + hoff +
                                                   (int64_t)q * a.ld_qkv + 16 * s + 8 * h);
    }
    lse2[qb] = a.lse[(int64_t)bh * a.S + q] * kLog2e;
    dlt[qb] = a.delta[(int64_t)bh * a.S + q];
  }
  f32x16 dq[2][2];  // [qb][dt]: rows = queries, columns = d
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    dq[qb][0] = zero16();
    dq[qb][1] = zero16();
  }

  const int kend = CAUSAL ? min(a.S, (qt + 1) * kBlockRows) : a.S;
  const int ntiles = kend / kTile;
  Stage sk, sv;
  sk.load(K, a.ld_qkv, 0, tid);
  sv.load(V, a.ld_qkv, 0, tid);
  sk.store(lds, tid);
  sv.store(lds + kImg, tid);
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const char* kimg = lds + (t & 1) * 2 * kImg;
    const char* vimg = kimg + kImg;
    const int k0 = t * kTile;
    {
      const int tn = min(t + 1, ntiles - 1) * kTile;
      sk.load(K, a.ld_qkv, tn, tid);
      sv.load(V, a.ld_qkv, tn, tid);
    }
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      const int kk0 = k0 + 32 * kb;
      if (!active || (CAUSAL && kk0 > q0w + kWaveRows - 1)) continue;  // wave-uniform
      f32x16 st[2] = {zero16(), zero16()}, dpt[2] = {zero16(), zero16()};  // [qb]: rows keys, columns queries
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bf16x8 kf = row_frag(kimg, 32 * kb + li, s, h);
        const bf16x8 vfr = row_frag(vimg, 32 * kb + li, s, h);
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
          st[qb] = mfma(kf, qf[qb][s], st[qb]);
          dpt[qb] = mfma(vfr, row_frag(oimg_w, 32 * qb + li, s, h), dpt[qb]);
        }
      }
      bf16x8 sb[2][2];  // [qb][k-step]: dS^T as the A operand of dQ += dS K
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        const int qrow = q0w + 32 * qb;
        const int q = qrow + li;
        if (CAUSAL && kk0 > qrow + 31) {
          sb[qb][0] = bf16x8{};
          sb[qb][1] = bf16x8{};
          continue;
        }
        uint32_t wds[16] = {};
        if (drop) load_keep_words(a.dmask + ((int64_t)bh * (a.S >> 5) + (qrow >> 5)) * a.S + kk0 + 4 * h, wds);
#pragma unroll
        for (int r = 0; r < 16; ++r) st[qb][r] = __builtin_amdgcn_exp2f(fmaf(st[qb][r], sl2, -lse2[qb]));
        if (CAUSAL && kk0 + 31 > qrow) {  // diagonal sub-tile (wave-uniform branch)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (kk0 + arow(r, h) > q) st[qb][r] = 0.f;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float d = drop ? keep_or_zero(dpt[qb][r], wds[r], li) : dpt[qb][r];
          st[qb][r] *= drop ? fmaf(d, pscale, -dlt[qb]) : d - dlt[qb];  // dS = P (dP / (1-p) - delta), dropped: -P delta
        }
        sb[qb][0] = pack8(st[qb], 0);
        sb[qb][1] = pack8(st[qb], 1);
      }
#pragma unroll
      for (int st_ = 0; st_ < 2; ++st_)
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const bf16x8 kc = col_frag(kimg, 32 * kb + 16 * st_ + 4 * h, 32 * dt + 16 * ((lane >> 4) & 1), lane);
#pragma unroll
          for (int qb = 0; qb < 2; ++qb) dq[qb][dt] = mfma(sb[qb][st_], kc, dq[qb][dt]);
        }
    }
    char* nxt = lds + ((t + 1) & 1) * 2 * kImg;
    sk.store(nxt, tid);
    sv.store(nxt + kImg, tid);
    __syncthreads();
  }
  if (!active) return;
  bf16_t* dQ = reinterpret_cast<bf16_t*>(a.dq) + hoff;
#pragma unroll
  for (int qb = 0; qb < 2; ++qb)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int q = q0w + 32 * qb + arow(r, h);
      dQ[(int64_t)q * a.ld_qkv + li] = f2bf(dq[qb][0][r] * a.scale);
      dQ[(int64_t)q * a.ld_qkv + 32 + li] = f2bf(dq[qb][1][r] * a.scale);
    }
}

bool g_fused_rng = true;

template <bool CAUSAL>
void run_fwd(const AttnArgs& a, hipStream_t s) {
  const dim3 grid(a.B * a.H, (a.S + kBlockRows - 1) / kBlockRows);
  if (!(a.p > 0.f)) {
    hipLaunchKernelGGL((attn_long_fwd_kernel<CAUSAL, 0>), grid, dim3(kThreads), 0, s, a);
  } else if (g_fused_rng) {
    hipLaunchKernelGGL((attn_long_fwd_kernel<CAUSAL, 2>), grid, dim3(kThreads), 0, s, a);
  } else {
    hipLaunchKernelGGL((attn_long_mask_kernel<CAUSAL>), dim3((a.S + 255) / 256, a.S / 32, a.B * a.H), dim3(256), 0, s, a);
    hipLaunchKernelGGL((attn_long_fwd_kernel<CAUSAL, 1>), grid, dim3(kThreads), 0, s, a);
  }
}

// dK/dV with 8 waves of 32 keys (1, default: GPT-2-XL's backward 535 -> 441 us, profiles/attn_long_dkdv8_r6.txt)
// or 4 waves of 64 (0); MIPIPE_ATTN_DKDV8 for A/B runs.
const int g_dkdv8 = [] {
  const char* e = getenv("MIPIPE_ATTN_DKDV8");
  return e == nullptr ? 1 : atoi(e);
}();

template <bool CAUSAL>
void run_bwd(const AttnArgs& a, hipStream_t s) {
  const int64_t rows = (int64_t)a.B * a.S * a.H;
  hipLaunchKernelGGL(attn_long_delta_kernel, dim3((unsigned)((rows * 8 + 255) / 256)), dim3(256), 0, s, a);
  const dim3 grid(a.B * a.H, (a.S + kBlockRows - 1) / kBlockRows);
  if (g_dkdv8) {
    if (a.p > 0.f) hipLaunchKernelGGL((attn_long_dkdv8_kernel<CAUSAL, true>), grid, dim3(kThreads8), 0, s, a);
    else hipLaunchKernelGGL((attn_long_dkdv8_kernel<CAUSAL, false>), grid, dim3(kThreads8), 0, s, a);
    if (a.p > 0.f) hipLaunchKernelGGL((attn_long_dq_kernel<CAUSAL, true>), grid, dim3(kThreads), 0, s, a);
    else hipLaunchKernelGGL((attn_long_dq_kernel<CAUSAL, false>), grid, dim3(kThreads), 0, s, a);
    return;
  }
  if (a.p > 0.f) {
    hipLaunchKernelGGL((attn_long_dkdv_kernel<CAUSAL, true>), grid, dim3(kThreads), 0, s, a);
    hipLaunchKernelGGL((attn_long_dq_kernel<CAUSAL, true>), grid, dim3(kThreads), 0, s, a);
  } else {
    hipLaunchKernelGGL((attn_long_dkdv_kernel<CAUSAL, false>), grid, dim3(kThreads), 0, s, a);
    hipLaunchKernelGGL((attn_long_dq_kernel<CAUSAL, false>), grid, dim3(kThreads), 0, s, a);
  }
}

}  // namespace

void attention_long_set_fused_rng(bool on) { g_fused_rng = on; }

bool attention_long_supported(int S, int Dh) { return Dh == D && S >= kBlockRows && S % kTile == 0; }

void attention_long_fwd(const AttnArgs& ai, hipStream_t s) {
  AttnArgs a = ai;
  a.threshold = dropout_threshold(a.p);
  if (a.causal) run_fwd<true>(a, s);
  else run_fwd<false>(a, s);
}

void attention_long_fwd_words(const AttnArgs& ai, hipStream_t s) {
  AttnArgs a = ai;
  a.threshold = dropout_threshold(a.p);
  const dim3 grid(a.B * a.H, (a.S + kBlockRows - 1) / kBlockRows);
  if (a.causal) hipLaunchKernelGGL((attn_long_fwd_kernel<true, 1>), grid, dim3(kThreads), 0, s, a);
  else hipLaunchKernelGGL((attn_long_fwd_kernel<false, 1>), grid, dim3(kThreads), 0, s, a);
}

void attention_long_bwd(const AttnArgs& ai, hipStream_t s) {
  AttnArgs a = ai;
  a.threshold = dropout_threshold(a.p);
  if (a.causal) run_bwd<true>(a, s);
  else run_bwd<false>(a, s);
}

}  // namespace mipipe
