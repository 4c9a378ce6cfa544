// Host-side launch interface of the mipipe HIP kernels.
//
// Kernel translation units include only HIP headers (fast to build); the
// torch-facing bindings (../bindings.cpp) include this header and call the
// launchers with raw pointers and the current HIP stream.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mipipe {

typedef uint16_t bf16_t;

// ------------------------------------------------------------------ LayerNorm
template <typename T>
struct LnArgs {
  const T* x = nullptr;      // branch input (dropout applies here)
  const T* res = nullptr;    // residual input (optional)
  const T* gamma = nullptr;
  const T* beta = nullptr;
  T* y = nullptr;
  T* z = nullptr;            // optional: saved pre-norm sum for backward
  float* mean = nullptr;
  float* rstd = nullptr;
  int rows = 0, cols = 0;
  float eps = 1e-5f;
  float p = 0.f;
  uint64_t seed = 0, offset = 0;
};

template <typename T>
struct LnBwdArgs {
  const T* dy = nullptr;
  const T* z = nullptr;
  const float* mean = nullptr;
  const float* rstd = nullptr;
  const T* gamma = nullptr;
  T* dz = nullptr;           // grad of z (= grad of the residual input)
  const T* addend = nullptr; // optional extra gradient of z, added to dz (fan-out fusion)
  T* dx = nullptr;           // grad of the dropout branch (nullptr if p == 0)
  float* dgamma_part = nullptr;  // [nparts, cols] workspace
  float* dbeta_part = nullptr;
  void* dgamma = nullptr;        // T (store) or fp32 (main_grad, may accumulate)
  void* dbeta = nullptr;
  bool out_f32 = false;
  bool accumulate = false;
  int rows = 0, cols = 0, nparts = 0;
  float p = 0.f;
  uint64_t seed = 0, offset = 0;
};

// out[c] (=|+=) sum over nparts partial rows; out is fp32 (out_f32) or bf16.
void reduce_parts(const float* part_a, const float* part_b, int nparts, int cols, void* out_a, void* out_b,
                  bool out_f32, bool accumulate, hipStream_t s);

int ln_max_vec(int cols);
int ln_bwd_parts(int rows, int cols);
template <typename T> void layernorm_fwd(const LnArgs<T>& a, hipStream_t s);
template <typename T> void layernorm_bwd(const LnBwdArgs<T>& a, hipStream_t s);

// ------------------------------------------------------------------ elementwise
enum Activation : int { kActNone = 0, kActRelu = 1, kActGelu = 2 };
// Backward-only activation code: the saved tensor IS act'(pre) (a GELU forward
// GEMM wrote it with GemmArgs::aux_grad), so the backward is one multiply.
constexpr int kActSavedGrad = 3;
// Backward-only: the saved tensor is a 1-bit mask of a ReLU (+ dropout) output's nonzeros, [M][ld bytes], bit
// (col & 7) of byte col / 8 -- written by the forward GEMM (GemmArgs::bits) so the consumer's dgrad epilogue
// reads 1/16 of the bytes the saved bf16 output costs.
constexpr int kActReluBits = 4;

template <typename T>
void bias_act_dropout_fwd(const T* x, const T* bias, T* y, int64_t rows, int cols, int act, float p, uint64_t seed,
                          uint64_t offset, hipStream_t s);
template <typename T>
void bias_act_dropout_bwd(const T* dy, const T* saved, const T* bias, T* dx, int64_t rows, int cols, int act, float p,
                          uint64_t seed, uint64_t offset, hipStream_t s);
int colsum_parts(int64_t rows, int64_t cols);
// Up to kColsumSegs equally shaped inputs whose stage-1 column sums run as one launch.
constexpr int kColsumSegs = 16;
struct ColsumSegs {
  const void* p[kColsumSegs] = {};
};
template <typename T>
bool column_sum_partial_multi(const ColsumSegs& segs, int nseg, int64_t rows, int cols, float* part, int nparts,
                              hipStream_t s);
// Stage 1 only: per-part column sums of `rows` rows into part[nparts][cols]
// (several inputs can write disjoint part slices and share one reduce_parts).
template <typename T>
void column_sum_partial(const T* x, int64_t rows, int cols, float* part, int nparts, hipStream_t s);
template <typename T>
void column_sum(const T* x, int64_t rows, int cols, float* part, int nparts, void* out, bool out_f32, bool accumulate,
                hipStream_t s);

// ------------------------------------------------------------------ GEMM
// kEpiStoreBf16 / kEpiStoreAct: the activation epilogue (bias, act, dropout,
// residual, aux) stored in the operand dtype (bf16 for gemm_bf16, fp32 for gemm_f32).
enum GemmEpilogue : int { kEpiStoreBf16 = 0, kEpiAccumF32 = 1, kEpiStoreF32 = 2, kEpiStoreAct = 0 };

struct GemmArgs {
  const void* A = nullptr;  // bf16
  const void* B = nullptr;  // bf16
  void* C = nullptr;        // bf16 or fp32 (epilogue)
  const void* bias = nullptr;  // bf16 [N] (kEpiStoreBf16 only)
  void* aux = nullptr;         // bf16 pre-activation output (optional)
  bool aux_grad = false;       // aux holds GELU'(pre) instead of pre (bf16 GEMMs, ACT = GELU)
  const void* res = nullptr;   // bf16 [M, ldr] added to the bf16 output (optional, kEpiStoreBf16)
  int64_t lda = 0, ldb = 0, ldc = 0;
  int64_t ldr = 0;             // row stride of res (0: ldc)
  // Activation backward in the bf16 epilogue (a dgrad GEMM whose output is the
  // gradient of an activation's output): C = acc [x dropout mask (p, seed,
  // offset: the forward's)] x act'(dact_in) x dact_scale.  dact_in is the
  // forward's saved pre-activation (GELU) or output (ReLU: its sign carries the
  // dropout mask too, so p = 0 and dact_scale = 1 / (1 - p)); row stride ldd.
  const void* dact_in = nullptr;
  int dact = 0;
  float dact_scale = 1.f;
  int64_t ldd = 0;
  int M = 0, N = 0, K = 0;
  bool a_kc = true;   // A stored [M, K] (true) or [K, M] (false)
  bool b_kc = true;   // B stored [N, K] (true) or [K, N] (false)
  int epi = kEpiStoreBf16;
  int act = kActNone;
  float p = 0.f;
  uint32_t threshold = 0;
  uint64_t seed = 0, offset = 0;
  int group_m = 8;  // tile-rows per group of the block -> tile order (L2 reuse of B tiles)
  // Split-K (plain bf16 output of an under-filled grid with a long K): the
  // K-tiles are divided among k_splits blocks per output tile, each writing
  // an fp32 partial into ws [k_splits][M][N]; a reduction adds them (+ res).
  int k_splits = 1;
  float* ws = nullptr;
  // Launch chunks of a larger GEMM (one round of tiles each): the chunk's
  // position in the full output, so the dropout mask (Philox counter
  // (row >> 2) * mask_ld + col) is the full matrix's.  mask_ld = 0: N.
  int mask_row0 = 0, mask_col0 = 0, mask_ld = 0;
  bool round_chunk = false;  // a launch_by_rounds chunk: stays on the 256-row kernel even when small
  int width = 0;             // 256-row kernel block width forced by the caller (0: big_width's rule)
  // K-segmented operands (deferred weight gradients: one GEMM over the
  // micro-batches of a step without concatenating them).  seg_k > 0: K-rows
  // [s*seg_k, (s+1)*seg_k) of A / B live at a_seg[s] / b_seg[s] (leading
  // dimensions lda / ldb); seg_k must be a multiple of 64.
  static constexpr int kMaxSegs = 16;
  int seg_k = 0;
  // Fused bias gradient of a weight-gradient GEMM (A = dY read as [K=T, M]):
  // rowsum[m] += sum_k A[k][m], fp32.  The 256 rows of a tile row are split
  // into 16-row slices summed by the blocks tn = 0..15 of that tile row, each
  // over the whole K (one writer per row: deterministic).  Needs
  // ceil(N / block width) >= 16 and k_splits == 1 (gemm_rowsum_ok).
  float* rowsum = nullptr;
  // The same fold on the B side for the transposed weight-gradient GEMM
  // (C^T = X^T . dY, B = dY read as [K=T, N]): colsum[n] += sum_k B[k][n];
  // the W/16 16-column slices of a tile column are spread over its tile
  // rows, 2 per block (gemm_colsum_ok: >= W/32 tile rows); with split-K
  // each split writes colsum_ws and one reduction adds them.
  float* colsum = nullptr;
  float* colsum_ws = nullptr;  // split-K: [k_splits][N] per-split column sums (the caller's workspace)
  // Transposed fp32 output (kEpiAccumF32 / kEpiStoreF32): element (m, n) of
  // the product goes to C[n * ldc + m] -- the weight gradient dW = (X^T dY)^T
  // lands in main_grad's [N_out, K_in] layout.
  bool trans_c = false;
  // A^T emission (forward GEMMs, A K-contiguous): the blocks also write
  // their A tiles transposed, at[k][m] (bf16, row stride ldat, 16-byte
  // aligned, m < M), from the LDS images they compute from -- each K-tile's
  // 8-row pieces shared out in rotation over the blocks of the tile row: X^T
  // for the layer's weight-gradient GEMM without a transposition pass
  // (tools/wgrad_layout_probe.py).
  void* at = nullptr;
  int64_t ldat = 0;
  // Forward ReLU + dropout (the EXTRA epilogue): also write the output's nonzero mask as bits (kActReluBits),
  // [M][ldbits bytes]; gemm_bits_ok(g) says whether this launch can.
  void* bits = nullptr;
  int64_t ldbits = 0;
  const void* a_seg[kMaxSegs] = {};
  const void* b_seg[kMaxSegs] = {};
};
bool gemm_supported(int64_t M, int64_t N, int64_t K);
// True if gemm_bf16 can fold g.rowsum into g (the wgrad layout, no split-K, >= 16 tile columns).
bool gemm_rowsum_ok(const GemmArgs& g);
// True if this forward GEMM (ReLU, dropout, the staged EXTRA epilogue) can write GemmArgs::bits.
bool gemm_bits_ok(const GemmArgs& g);
// True if the forward GEMM with this epilogue can write A^T (GemmArgs::at).
bool gemm_emit_ok(int act, float p, bool aux);
// True if gemm_bf16 can fold g.colsum into g (B I-contiguous, fp32 out, no split-K, >= W/16 tile rows).
bool gemm_colsum_ok(const GemmArgs& g);
// Split-K factor gemm_bf16 would use for g (1 = none); the caller provides
// g.ws with k_splits * M * N floats when it is > 1.
int gemm_splitk_factor(const GemmArgs& g);
// Main-loop schedule of the 256x256 GEMM: 7 (default, the only one in the product build) = whole-tile
// ping-pong.  A -DMIPIPE_GEMM_AB build also has 0 = one barrier per K-tile, 1 = 4-phase ping-pong,
// 2 = 1 except the wgrad layout, 3 / 4 = 2 / 1 with the B operand staged two K-tiles ahead, 5 / 6 =
// half-tile ping-pong (everywhere / on the K-contiguous layouts).  Returns false for a schedule not built.
bool gemm_set_schedule(int mode);
bool gemm_ab_build();
void gemm_set_width(int w);    // 256-row GEMM block width: 0 auto, 128, 256
void gemm_set_rounds(int on);  // 1: multi-round grids launched one round at a time (default), 0: one launch
void gemm_set_waves(int w);   // 256x256 GEMM blocks: 4 (gemm4w_kernel, -DMIPIPE_GEMM_AB builds only) or 8 waves; 0 default
int gemm_get_waves();
void gemm_set_splitk(int n);  // split-K factor: 0 off, 1 auto (gemm_splitk_factor), n >= 2 forced (A/B tools)
int gemm_get_schedule();
void gemm_bf16(const GemmArgs& g, hipStream_t s);
// Same interface with fp32 operands (and fp32 bias / res / aux / C): v_mfma_f32_32x32x2_f32.
bool gemm_f32_supported(int64_t M, int64_t N, int64_t K);
void gemm_f32(const GemmArgs& g, hipStream_t s);

// ------------------------------------------------------------------ attention
struct AttnArgs {
  const void* q = nullptr;  // bf16, element (b, s, h, d) at b*S*ld_qkv + s*ld_qkv + h*D + d
  const void* k = nullptr;
  const void* v = nullptr;
  void* o = nullptr;        // bf16 [B, S, H, D], token stride ld_o
  const void* dout = nullptr;
  void* dq = nullptr;       // same layout as q/k/v (packed dQKV)
  void* dk = nullptr;
  void* dv = nullptr;
  float* lse = nullptr;     // [B, H, S]
  float* delta = nullptr;   // [B, H, S]
  int64_t ld_qkv = 0, ld_o = 0;      // token strides (elements)
  int64_t sb_qkv = 0, sh_qkv = 0;    // batch / head strides of q, k, v (and dq, dk, dv)
  int64_t sb_o = 0, sh_o = 0;        // batch / head strides of o and dout
  int B = 0, H = 0, S = 0, D = 0;
  float scale = 1.f, p = 0.f;
  uint32_t threshold = 0;
  uint64_t seed = 0, offset = 0;
  bool causal = false;
  // valid keys (0 = all S): keys >= kv_len are masked out (a zero-padded
  // non-causal sequence; fp32 kernels)
  int kv_len = 0;
  // long-sequence kernels with dropout: keep bits, one uint32 per (b*h, 32-query
  // block, key) written by the forward and read by the backward
  uint32_t* dmask = nullptr;
};
bool attention_supported(int S, int D);
// S == 128 backward: fused one-pass kernel (1, default) or delta + dK/dV + dQ kernels (0).
void attention_set_fused_bwd(int on);
void attention_fwd(const AttnArgs& a, hipStream_t s);
void attention_bwd(const AttnArgs& a, hipStream_t s);
// fp32 q/k/v/o (v_mfma_f32_32x32x2_f32): S % 32 == 0, D == 64; "key-quad" dropout layout.
bool attention_f32_supported(int S, int D);
// bf16, D == 64, S >= 256, S % 64 == 0 (attention_long.hip): 32x32x16 MFMA, stored dropout bits.
bool attention_long_supported(int S, int D);
// Keep words made inside the forward kernel (default) or by their own kernel first.
void attention_long_set_fused_rng(bool on);
void attention_long_fwd(const AttnArgs& a, hipStream_t s);
// The forward reading keep words already in a.dmask (made by an earlier forward of the same Philox draw:
// a checkpoint recompute) instead of making them.
void attention_long_fwd_words(const AttnArgs& a, hipStream_t s);
void attention_long_bwd(const AttnArgs& a, hipStream_t s);
void attention_f32_fwd(const AttnArgs& a, hipStream_t s);
void attention_f32_bwd(const AttnArgs& a, hipStream_t s);

// ------------------------------------------------------------------ loss
// t_offset: logits are vocabulary columns [t_offset, t_offset + V) (split decoder).
template <typename T>
void cross_entropy_fwd(const T* logits, const int64_t* target, int64_t rows, int64_t V, int64_t ld,
                       int64_t ignore_index, float* loss, float* lse, hipStream_t s, int64_t t_offset = 0);
// Mean CE in two launches (row losses, then a one-block masked mean): loss[0] =
// mean over valid targets; weight[r] = valid / count (the backward's row scale).
template <typename T>
void cross_entropy_mean_fwd(const T* logits, const int64_t* target, int64_t rows, int64_t V, int64_t ld,
                            int64_t ignore_index, float* loss_row, float* lse, float* weight, float* loss,
                            hipStream_t s);
// lse / row_scale read with strides ld_lse / ld_rs (floats); stat_out: (lse,
// scale) written to nslot fp32 words per row (split-decoder gradient slots).
template <typename T>
void cross_entropy_bwd(const T* logits, const int64_t* target, const float* lse, const float* scale,
                       const float* row_scale, int64_t rows, int64_t V, int64_t ld, int64_t ld_out,
                       int64_t ignore_index, T* dlogits, int64_t zero_to, hipStream_t s, int64_t t_offset = 0,
                       int64_t ld_lse = 1, int64_t ld_rs = 1, float* stat_out = nullptr, int64_t ld_stat = 0,
                       int nslot = 0);
// Split-decoder head forward: out[r] = [x[r] (E values) | lse, target logit, 0 ...]
// (nslot fp32 words); E * sizeof(T) % 16 == 0, 16-byte aligned rows.
template <typename T>
void vsplit_head_fwd(const T* logits, int64_t ld, int64_t rows, int64_t V, const int64_t* target, const T* x,
                     int64_t ldx, int64_t E, T* out, int64_t ldo, int nslot, hipStream_t s);
// Split-decoder tail forward: full lse per row from this slice and the head's
// slot statistics (stats: lse_a, t_a at stride ld_st floats), the mean loss
// into loss[0] and per-row weights valid / count.
template <typename T>
void vsplit_tail_fwd(const T* logits, int64_t ld, int64_t rows, int64_t V, const int64_t* target, int64_t t_offset,
                     int64_t ignore_index, const float* stats, int64_t ld_st, float* lse, float* loss_row,
                     float* weight_row, float* loss, hipStream_t s);

// ------------------------------------------------------------------ embedding
// pe (optional): position table [>= seq_len, E], fp32 (pe_f32) or T.
template <typename T>
void embedding_fwd(const int64_t* tokens, const T* weight, const void* pe, bool pe_f32, T* out, int64_t rows,
                   int seq_len, int E, int64_t V, float scale, float p, uint64_t seed, uint64_t offset, hipStream_t s);
// dpe (optional): fp32 [>= seq_len, E] learned-position gradient, += the masked rows by position.
template <typename T>
void embedding_bwd(const int64_t* tokens, const T* dout, float* dweight, int64_t rows, int E, int64_t V, float scale,
                   float p, uint64_t seed, uint64_t offset, hipStream_t s, float* dpe = nullptr, int seq_len = 0);

// ------------------------------------------------------------------ optimizer
struct AdamHyper {
  float lr = 1e-3f, beta1 = 0.9f, beta2 = 0.999f, eps = 1e-8f, weight_decay = 0.f;
  float bias_correction1 = 1.f, bias_correction2 = 1.f;
  float max_norm = 0.f;  // <= 0: no clipping
  int adamw = 0;
};
int sumsq_parts(int64_t n);
void sumsq(const float* g, int64_t n, float* partial, int nparts, float* out, hipStream_t s);
// 0: grid-stride kernel, 2 vectors of loads in flight per thread;
// 1: one-shot tiles of 4 vectors per thread (default, ~10 % faster).
void adam_set_variant(int v);
template <typename M>
void adam_step(float* master, M* model, const float* grad, float* m, float* v, int64_t n, const AdamHyper& h,
               const float* sumsq_ptr, hipStream_t s);

// ------------------------------------------------------------------ misc
void gpu_sleep(int64_t microseconds, hipStream_t s);
// out[c * ldo + r] = x[r * ldx + c], 2-byte elements; rows, cols, ldx, ldo
// multiples of 8 and both pointers 16-byte aligned (the caller checks).
void transpose_b16(const uint16_t* x, int64_t rows, int64_t cols, int64_t ldx, uint16_t* out, int64_t ldo,
                   hipStream_t s);

}  // namespace mipipe
