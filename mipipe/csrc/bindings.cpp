// Python bindings of mipipe._C: the native runtime and the HIP kernels.
//
// Every kernel entry point validates shapes/dtypes/devices on the host before
// launching (a faulting kernel can take down every GPU on the node), allocates
// outputs through the torch caching allocator and launches on the current HIP
// stream of the tensors' device.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <ATen/hip/HIPGeneratorImpl.h>
#include <ATen/core/Generator.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include <mutex>
#include <optional>
#include <tuple>

#include "kernels/kernels.h"
#include "runtime/ipc.h"
#include "runtime/runtime.h"

namespace py = pybind11;
using at::Tensor;

namespace mipipe {
namespace {

#define MP_CHECK(cond, ...) TORCH_CHECK(cond, "mipipe: ", __VA_ARGS__)

hipStream_t cur_stream(const Tensor& t) { return at::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream(); }

// (seed, offset) from the torch device generator; `increment` philox words per
// thread are reserved so successive ops never reuse a counter.
std::pair<uint64_t, uint64_t> philox_draw(const at::Device& dev, uint64_t increment) {
  auto gen = at::get_generator_or_default<at::CUDAGeneratorImpl>(
      std::nullopt, at::cuda::detail::getDefaultCUDAGenerator(dev.index()));
  std::lock_guard<std::mutex> lock(gen->mutex_);
  return gen->philox_engine_inputs(increment);
}

void check_cuda(const Tensor& t, const char* name) {
  MP_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  MP_CHECK(t.is_contiguous(), name, " must be contiguous");
}

void check_same(const Tensor& a, const Tensor& b, const char* an, const char* bn) {
  MP_CHECK(a.device() == b.device(), an, " and ", bn, " must be on the same device");
  MP_CHECK(a.scalar_type() == b.scalar_type(), an, " and ", bn, " must have the same dtype");
}

template <typename T>
T* ptr(const Tensor& t) {
  return reinterpret_cast<T*>(t.data_ptr());
}
template <typename T>
const T* cptr(const Tensor& t) {
  return reinterpret_cast<const T*>(t.data_ptr());
}
template <typename T>
const T* optr(const std::optional<Tensor>& t) {
  return t.has_value() ? reinterpret_cast<const T*>(t->data_ptr()) : nullptr;
}

// ------------------------------------------------------------------ runtime
int64_t py_stream_acquire(int64_t device, int64_t priority) {
  return reinterpret_cast<int64_t>(rt::stream_acquire((int)device, (int)priority));
}

void py_stream_wait(int64_t waiting, int64_t waited, int64_t device) {
  rt::stream_wait(reinterpret_cast<hipStream_t>(waiting), reinterpret_cast<hipStream_t>(waited), (int)device);
}

void py_peer_copy(Tensor dst, Tensor src, int64_t src_stream, int64_t dst_stream, int64_t src_dev, int64_t dst_dev,
                  int64_t engine) {
  MP_CHECK(dst.is_contiguous() && src.is_contiguous(), "peer_copy needs contiguous tensors");
  MP_CHECK(dst.nbytes() == src.nbytes(), "peer_copy size mismatch");
  MP_CHECK(dst.is_cuda() && src.is_cuda(), "peer_copy needs device tensors");
  MP_CHECK(dst.get_device() == dst_dev && src.get_device() == src_dev, "peer_copy device mismatch");
  MP_CHECK(engine == rt::kCopySdma || engine == rt::kCopyBlit, "peer_copy: engine is 0 (sdma) or 1 (blit)");
  rt::peer_copy(dst.data_ptr(), (int)dst_dev, src.data_ptr(), (int)src_dev, src.nbytes(),
                reinterpret_cast<hipStream_t>(src_stream), reinterpret_cast<hipStream_t>(dst_stream), (int)engine);
}

void py_gpu_sleep(int64_t us) { mipipe::gpu_sleep(us, at::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream()); }

// ------------------------------------------------------------------ LayerNorm
std::tuple<Tensor, std::optional<Tensor>, Tensor, Tensor, int64_t, int64_t> py_layernorm_fwd(
    Tensor x, std::optional<Tensor> res, Tensor gamma, Tensor beta, double eps, double p, bool save_z) {
  check_cuda(x, "x");
  check_cuda(gamma, "gamma");
  check_cuda(beta, "beta");
  const int64_t cols = x.size(-1);
  const int64_t rows = x.numel() / cols;
  MP_CHECK(cols % 8 == 0, "layernorm: hidden size must be a multiple of 8, got ", cols);
  MP_CHECK(ln_max_vec((int)cols) > 0, "layernorm: hidden size too large: ", cols);
  MP_CHECK(gamma.numel() == cols && beta.numel() == cols, "layernorm: gamma/beta size mismatch");
  check_same(x, gamma, "x", "gamma");
  check_same(x, beta, "x", "beta");
  if (res.has_value()) {
    check_cuda(*res, "residual");
    check_same(x, *res, "x", "residual");
    MP_CHECK(res->numel() == x.numel(), "layernorm: residual shape mismatch");
  }
  MP_CHECK(p >= 0.0 && p < 1.0, "dropout p must be in [0, 1)");
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto y = at::empty_like(x);
  std::optional<Tensor> z;
  if (save_z) z = at::empty_like(x);
  auto fopt = x.options().dtype(at::kFloat);
  auto mean = at::empty({rows}, fopt);
  auto rstd = at::empty({rows}, fopt);
  uint64_t seed = 0, offset = 0;
  if (p > 0.0) std::tie(seed, offset) = philox_draw(x.device(), 4);
  auto s = cur_stream(x);
  if (rows == 0) return {y, z, mean, rstd, (int64_t)seed, (int64_t)offset};
  if (x.scalar_type() == at::kBFloat16) {
    LnArgs<bf16_t> a;
    a.x = cptr<bf16_t>(x); a.res = optr<bf16_t>(res); a.gamma = cptr<bf16_t>(gamma); a.beta = cptr<bf16_t>(beta);
    a.y = ptr<bf16_t>(y); a.z = z ? ptr<bf16_t>(*z) : nullptr; a.mean = ptr<float>(mean); a.rstd = ptr<float>(rstd);
    a.rows = (int)rows; a.cols = (int)cols; a.eps = (float)eps; a.p = (float)p; a.seed = seed; a.offset = offset;
    layernorm_fwd<bf16_t>(a, s);
  } else if (x.scalar_type() == at::kFloat) {
    LnArgs<float> a;
    a.x = cptr<float>(x); a.res = optr<float>(res); a.gamma = cptr<float>(gamma); a.beta = cptr<float>(beta);
    a.y = ptr<float>(y); a.z = z ? ptr<float>(*z) : nullptr; a.mean = ptr<float>(mean); a.rstd = ptr<float>(rstd);
    a.rows = (int)rows; a.cols = (int)cols; a.eps = (float)eps; a.p = (float)p; a.seed = seed; a.offset = offset;
    layernorm_fwd<float>(a, s);
  } else {
    MP_CHECK(false, "layernorm: unsupported dtype ", x.scalar_type());
  }
  return {y, z, mean, rstd, (int64_t)seed, (int64_t)offset};
}

// With acc_gamma/acc_beta (fp32 main_grad views) the parameter gradients are
// accumulated there and None is returned for them.
std::tuple<Tensor, std::optional<Tensor>, std::optional<Tensor>, std::optional<Tensor>> py_layernorm_bwd(
    Tensor dy, Tensor z, Tensor mean, Tensor rstd, Tensor gamma, double p, int64_t seed, int64_t offset,
    std::optional<Tensor> acc_gamma, std::optional<Tensor> acc_beta, std::optional<Tensor> addend) {
  check_cuda(dy, "dy");
  check_cuda(z, "z");
  check_same(dy, z, "dy", "z");
  check_same(dy, gamma, "dy", "gamma");
  const int64_t cols = dy.size(-1);
  const int64_t rows = dy.numel() / cols;
  MP_CHECK(z.numel() == dy.numel(), "layernorm_bwd: shape mismatch");
  MP_CHECK(mean.numel() == rows && rstd.numel() == rows, "layernorm_bwd: stats size mismatch");
  MP_CHECK(cols % 8 == 0 && ln_max_vec((int)cols) > 0, "layernorm_bwd: bad hidden size");
  if (addend) {
    check_same(dy, *addend, "dy", "addend");
    MP_CHECK(addend->numel() == dy.numel() && addend->is_contiguous(), "layernorm_bwd: addend must match dy");
  }
  at::hip::HIPGuardMasqueradingAsCUDA guard(dy.device());
  auto dz = at::empty_like(dy);
  std::optional<Tensor> dx;
  if (p > 0.0) dx = at::empty_like(dy);
  const bool acc = acc_gamma.has_value();
  MP_CHECK(acc == acc_beta.has_value(), "layernorm_bwd: pass both accumulation targets or neither");
  if (acc) {
    for (auto* t : {&*acc_gamma, &*acc_beta}) {
      MP_CHECK(t->is_cuda() && t->is_contiguous() && t->scalar_type() == at::kFloat && t->numel() == cols,
               "layernorm_bwd: accumulation targets must be contiguous fp32 [cols]");
    }
  }
  Tensor dgamma = acc ? *acc_gamma : at::empty_like(gamma);
  Tensor dbeta = acc ? *acc_beta : at::empty_like(gamma);
  const int nparts = std::max(1, ln_bwd_parts((int)rows, (int)cols));
  auto part = at::empty({2, nparts, cols}, dy.options().dtype(at::kFloat));
  auto s = cur_stream(dy);
  std::optional<Tensor> rg, rb;
  if (!acc) {
    rg = dgamma;
    rb = dbeta;
  }
  if (rows == 0) {
    if (!acc) {
      dgamma.zero_();
      dbeta.zero_();
    }
    return {dz, dx, rg, rb};
  }
  auto fill = [&](auto& a, auto* tag) {
    using T = std::remove_pointer_t<decltype(tag)>;
    a.dy = cptr<T>(dy); a.z = cptr<T>(z); a.mean = cptr<float>(mean); a.rstd = cptr<float>(rstd);
    a.gamma = cptr<T>(gamma); a.dz = ptr<T>(dz); a.dx = dx ? ptr<T>(*dx) : nullptr;
    a.addend = addend ? cptr<T>(*addend) : nullptr;
    a.dgamma_part = ptr<float>(part); a.dbeta_part = ptr<float>(part) + (size_t)nparts * cols;
    a.dgamma = dgamma.data_ptr(); a.dbeta = dbeta.data_ptr();
    a.out_f32 = dgamma.scalar_type() == at::kFloat; a.accumulate = acc;
    a.rows = (int)rows; a.cols = (int)cols; a.nparts = nparts; a.p = (float)p;
    a.seed = (uint64_t)seed; a.offset = (uint64_t)offset;
  };
  if (dy.scalar_type() == at::kBFloat16) {
    LnBwdArgs<bf16_t> a;
    fill(a, (bf16_t*)nullptr);
    layernorm_bwd<bf16_t>(a, s);
  } else if (dy.scalar_type() == at::kFloat) {
    LnBwdArgs<float> a;
    fill(a, (float*)nullptr);
    layernorm_bwd<float>(a, s);
  } else {
    MP_CHECK(false, "layernorm_bwd: unsupported dtype");
  }
  return {dz, dx, rg, rb};
}

// ------------------------------------------------------------------ elementwise
template <typename F>
void dispatch_fb(const Tensor& t, const char* what, F&& f) {
  if (t.scalar_type() == at::kBFloat16) {
    f((bf16_t*)nullptr);
  } else if (t.scalar_type() == at::kFloat) {
    f((float*)nullptr);
  } else {
    MP_CHECK(false, what, ": unsupported dtype ", t.scalar_type());
  }
}

std::tuple<Tensor, int64_t, int64_t> py_bias_act_fwd(Tensor x, std::optional<Tensor> bias, int64_t act, double p) {
  check_cuda(x, "x");
  const int64_t cols = x.size(-1);
  const int64_t rows = x.numel() / std::max<int64_t>(cols, 1);
  MP_CHECK(cols % 8 == 0, "bias_act: last dim must be a multiple of 8");
  MP_CHECK(act >= 0 && act <= 2, "bias_act: bad activation");
  MP_CHECK(p >= 0.0 && p < 1.0, "dropout p must be in [0, 1)");
  if (bias) {
    check_cuda(*bias, "bias");
    check_same(x, *bias, "x", "bias");
    MP_CHECK(bias->numel() == cols, "bias_act: bias size mismatch");
  }
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto y = at::empty_like(x);
  uint64_t seed = 0, offset = 0;
  if (p > 0.0) std::tie(seed, offset) = philox_draw(x.device(), 4);
  auto s = cur_stream(x);
  dispatch_fb(x, "bias_act_fwd", [&](auto* tag) {
    using T = std::remove_pointer_t<decltype(tag)>;
    bias_act_dropout_fwd<T>(cptr<T>(x), optr<T>(bias), ptr<T>(y), rows, (int)cols, (int)act, (float)p, seed, offset, s);
  });
  return {y, (int64_t)seed, (int64_t)offset};
}

Tensor py_column_sum(Tensor x, std::optional<Tensor> out, bool accumulate);

std::tuple<Tensor, std::optional<Tensor>> py_bias_act_bwd(Tensor dy, Tensor saved, std::optional<Tensor> bias,
                                                          int64_t act, double p, int64_t seed, int64_t offset,
                                                          bool need_dbias, std::optional<Tensor> dbias_acc) {
  check_cuda(dy, "dy");
  check_cuda(saved, "saved");
  check_same(dy, saved, "dy", "saved");
  MP_CHECK(dy.numel() == saved.numel(), "bias_act_bwd: shape mismatch");
  const int64_t cols = dy.size(-1);
  const int64_t rows = dy.numel() / std::max<int64_t>(cols, 1);
  MP_CHECK(cols % 8 == 0, "bias_act_bwd: last dim must be a multiple of 8");
  if (bias) MP_CHECK(bias->numel() == cols, "bias_act_bwd: bias size mismatch");
  at::hip::HIPGuardMasqueradingAsCUDA guard(dy.device());
  auto dx = at::empty_like(dy);
  auto s = cur_stream(dy);
  dispatch_fb(dy, "bias_act_bwd", [&](auto* tag) {
    using T = std::remove_pointer_t<decltype(tag)>;
    bias_act_dropout_bwd<T>(cptr<T>(dy), cptr<T>(saved), optr<T>(bias), ptr<T>(dx), rows, (int)cols, (int)act,
                            (float)p, (uint64_t)seed, (uint64_t)offset, s);
  });
  std::optional<Tensor> db;
  if (dbias_acc.has_value()) {
    py_column_sum(dx.view({rows, cols}), dbias_acc, true);  // fp32 main_grad += colsum
  } else if (need_dbias) {
    db = py_column_sum(dx.view({rows, cols}), std::nullopt, false);
  }
  return {dx, db};
}

Tensor py_column_sum(Tensor x, std::optional<Tensor> out, bool accumulate) {
  check_cuda(x, "x");
  const int64_t cols = x.size(-1);
  const int64_t rows = x.numel() / std::max<int64_t>(cols, 1);
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Tensor o = out.has_value() ? *out : at::empty({cols}, x.options());
  MP_CHECK(o.numel() == cols && o.is_contiguous(), "column_sum: bad out");
  const bool out_f32 = o.scalar_type() == at::kFloat;
  MP_CHECK(out_f32 || o.scalar_type() == x.scalar_type(), "column_sum: out must be fp32 or the input dtype");
  if (rows == 0) {
    if (!accumulate) o.zero_();
    return o;
  }
  const int nparts = colsum_parts(rows, cols);
  auto part = at::empty({nparts, cols}, x.options().dtype(at::kFloat));
  auto s = cur_stream(x);
  dispatch_fb(x, "column_sum", [&](auto* tag) {
    using T = std::remove_pointer_t<decltype(tag)>;
    column_sum<T>(cptr<T>(x), rows, (int)cols, ptr<float>(part), nparts, o.data_ptr(), out_f32, accumulate, s);
  });
  return o;
}

// ------------------------------------------------------------------ cross entropy
void check_rows(const Tensor& t, const char* name) {
  MP_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  MP_CHECK(t.dim() == 2 && t.stride(1) == 1 && t.stride(0) >= t.size(1), name, " must be 2-D with unit column stride");
}

std::tuple<Tensor, Tensor> py_ce_fwd(Tensor logits, Tensor target, int64_t ignore_index, int64_t t_offset) {
  check_rows(logits, "logits");
  check_cuda(target, "target");
  MP_CHECK(target.scalar_type() == at::kLong && target.is_contiguous(), "cross_entropy: target must be contiguous int64");
  MP_CHECK(logits.dim() == 2 && target.numel() == logits.size(0), "cross_entropy: expects [N, V] logits and [N] target");
  at::hip::HIPGuardMasqueradingAsCUDA guard(logits.device());
  const int64_t rows = logits.size(0), V = logits.size(1);
  auto fopt = logits.options().dtype(at::kFloat);
  auto loss = at::empty({rows}, fopt);
  auto lse = at::empty({rows}, fopt);
  auto s = cur_stream(logits);
  dispatch_fb(logits, "cross_entropy_fwd", [&](auto* tag) {
    using T = std::remove_pointer_t<decltype(tag)>;
    cross_entropy_fwd<T>(cptr<T>(logits), cptr<int64_t>(target), rows, V, logits.stride(0), ignore_index,
                         ptr<float>(loss), ptr<float>(lse), s, t_offset);
  });
  return {loss, lse};
}

// Mean cross-entropy over the valid targets: (loss [] fp32, lse [N], weight [N] = valid / count).
std::tuple<Tensor, Tensor, Tensor> py_ce_mean_fwd(Tensor logits, Tensor target, int64_t ignore_index) {
  check_rows(logits, "logits");
  check_cuda(target, "target");
  MP_CHECK(target.scalar_type() == at::kLong && target.numel() == logits.size(0),
           "cross_entropy_mean: expects [N, V] logits and [N] int64 target");
  at::hip::HIPGuardMasqueradingAsCUDA guard(logits.device());
  const int64_t rows = logits.size(0), V = logits.size(1);
  auto fopt = logits.options().dtype(at::kFloat);
  auto loss_row = at::empty({rows}, fopt);
  auto lse = at::empty({rows}, fopt);
  auto weight = at::empty({rows}, fopt);
  auto loss = at::empty({}, fopt);
  auto s = cur_stream(logits);
  dispatch_fb(logits, "cross_entropy_mean_fwd", [&](auto* tag) {
    using T = std::remove_pointer_t<decltype(tag)>;
    cross_entropy_mean_fwd<T>(cptr<T>(logits), cptr<int64_t>(target), rows, V, logits.stride(0), ignore_index,
                              ptr<float>(loss_row), ptr<float>(lse), ptr<float>(weight), ptr<float>(loss), s);
  });
  return {loss, lse, weight};
}

// A per-row fp32 vector, possibly strided (a column of a packed message's
// statistic slots): its stride in floats.
int64_t row_vector(const Tensor& t, int64_t rows, const char* name) {
  MP_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.dim() == 1 && t.size(0) == rows, name,
           " must be a [rows] fp32 GPU tensor");
  return rows > 1 ? t.stride(0) : 1;
}

// The statistic slots of a packed split-decoder message: `slots` is the
// [rows, n] column slice after the hidden values, in the activation dtype.
// Returns (fp32 word pointer, row stride in words, words per row).
std::tuple<float*, int64_t, int> stat_slots(const Tensor& slots, int64_t rows, const char* name) {
  MP_CHECK(slots.is_cuda(), name, " must be a GPU tensor");
  MP_CHECK(slots.dim() == 2 && slots.size(0) == rows && slots.stride(1) == 1, name, " must be [rows, n] with unit column stride");
  const int64_t es = slots.element_size();
  const int64_t ld = rows > 1 ? slots.stride(0) : slots.size(1);
  MP_CHECK((ld * es) % 4 == 0 && (slots.size(1) * es) % 4 == 0 && reinterpret_cast<uintptr_t>(slots.data_ptr()) % 4 == 0,
           name, ": slots must hold whole, aligned fp32 words");
  const int nslot = (int)(slots.size(1) * es / 4);
  MP_CHECK(nslot >= 2 && nslot <= 256, name, ": need 2..256 fp32 words per row");
  return {reinterpret_cast<float*>(slots.data_ptr()), ld * es / 4, nslot};
}

// out (optional): [N, >= V] destination with unit column stride (e.g. a
// zero-padded vocabulary buffer); row_scale (optional): per-row scale, see loss.hip.
// zero_pad: columns [V, out.size(1)) of `out` are zeroed (padded-vocabulary gradient).
// lse / row_scale may be strided; scale and row_scale together multiply.
// stat_out (optional): [N, n] slots receiving (lse, row scale) (split decoder).
Tensor py_ce_bwd(Tensor logits, Tensor target, Tensor lse, std::optional<Tensor> scale, int64_t ignore_index,
                 std::optional<Tensor> row_scale, std::optional<Tensor> out, bool zero_pad, int64_t t_offset,
                 std::optional<Tensor> stat_out) {
  check_rows(logits, "logits");
  const int64_t rows = logits.size(0);
  check_cuda(target, "target");
  MP_CHECK(target.scalar_type() == at::kLong && target.is_contiguous() && target.numel() == rows,
           "cross_entropy_bwd: target must be contiguous int64 [N]");
  const int64_t ld_lse = row_vector(lse, rows, "lse");
  MP_CHECK(scale.has_value() || row_scale.has_value(), "cross_entropy_bwd: give scale and/or row_scale");
  if (scale)
    MP_CHECK(scale->scalar_type() == at::kFloat && scale->numel() == 1 && scale->is_cuda(), "cross_entropy_bwd: bad scale");
  const int64_t ld_rs = row_scale ? row_vector(*row_scale, rows, "row_scale") : 1;
  at::hip::HIPGuardMasqueradingAsCUDA guard(logits.device());
  Tensor d;
  if (out) {
    MP_CHECK(out->dim() == 2 && out->size(0) == rows && out->size(1) >= logits.size(1) &&
                 out->stride(1) == 1 && out->scalar_type() == logits.scalar_type() && out->is_cuda(),
             "cross_entropy_bwd: bad out");
    d = *out;
  } else {
    d = at::empty({rows, logits.size(1)}, logits.options());
  }
  float* st = nullptr;
  int64_t ld_st = 0;
  int nslot = 0;
  if (stat_out) std::tie(st, ld_st, nslot) = stat_slots(*stat_out, rows, "stat_out");
  auto s = cur_stream(logits);
  dispatch_fb(logits, "cross_entropy_bwd", [&](auto* tag) {
    using T = std::remove_pointer_t<decltype(tag)>;
    cross_entropy_bwd<T>(cptr<T>(logits), cptr<int64_t>(target), cptr<float>(lse),
                         scale ? cptr<float>(*scale) : nullptr, row_scale ? cptr<float>(*row_scale) : nullptr,
                         rows, logits.size(1), logits.stride(0), d.stride(0), ignore_index, ptr<T>(d),
                         zero_pad ? d.size(1) : logits.size(1), s, t_offset, ld_lse, ld_rs, st, ld_st, nslot);
  });
  return d;
}

// Split-decoder head forward (mipipe/models/vocab_split.py): packs x into
// out[:, :E] and (lse, target logit) into the slots out[:, E:].
void py_vsplit_head_fwd(Tensor logits, Tensor target, Tensor x, Tensor out) {
  check_rows(logits, "logits");
  check_rows(x, "x");
  check_rows(out, "out");
  const int64_t rows = logits.size(0), E = x.size(1);
  MP_CHECK(x.size(0) == rows && out.size(0) == rows && out.size(1) > E, "vsplit_head_fwd: shape mismatch");
  MP_CHECK(x.scalar_type() == logits.scalar_type() && out.scalar_type() == x.scalar_type(), "vsplit_head_fwd: dtypes differ");
  MP_CHECK(target.is_cuda() && target.scalar_type() == at::kLong && target.is_contiguous() && target.numel() == rows,
           "vsplit_head_fwd: target must be contiguous int64 [N]");
  const int64_t es = x.element_size();
  MP_CHECK((E * es) % 16 == 0 && (x.stride(0) * es) % 16 == 0 && (out.stride(0) * es) % 16 == 0 &&
               reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 &&
               reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0,
           "vsplit_head_fwd: x / out rows must be 16-byte aligned");
  auto [st, ld_st, nslot] = stat_slots(out.narrow(1, E, out.size(1) - E), rows, "out slots");
  (void)st;
  (void)ld_st;
  at::hip::HIPGuardMasqueradingAsCUDA guard(logits.device());
  auto s = cur_stream(logits);
  dispatch_fb(logits, "vsplit_head_fwd", [&](auto* tag) {
    using T = std::remove_pointer_t<decltype(tag)>;
    vsplit_head_fwd<T>(cptr<T>(logits), logits.stride(0), rows, logits.size(1), cptr<int64_t>(target), cptr<T>(x),
                       x.stride(0), E, ptr<T>(out), out.stride(0), nslot, s);
  });
}

// Split-decoder tail forward: returns (loss [] fp32, lse [N], weight [N] = valid / count).
std::tuple<Tensor, Tensor, Tensor> py_vsplit_tail_fwd(Tensor logits, Tensor target, int64_t t_offset,
                                                      int64_t ignore_index, Tensor slots) {
  check_rows(logits, "logits");
  const int64_t rows = logits.size(0);
  MP_CHECK(target.is_cuda() && target.scalar_type() == at::kLong && target.is_contiguous() && target.numel() == rows,
           "vsplit_tail_fwd: target must be contiguous int64 [N]");
  auto [st, ld_st, nslot] = stat_slots(slots, rows, "slots");
  (void)nslot;
  at::hip::HIPGuardMasqueradingAsCUDA guard(logits.device());
  auto fopt = logits.options().dtype(at::kFloat);
  auto loss = at::empty({}, fopt);
  auto lse = at::empty({rows}, fopt);
  auto loss_row = at::empty({rows}, fopt);
  auto weight = at::empty({rows}, fopt);
  auto s = cur_stream(logits);
  dispatch_fb(logits, "vsplit_tail_fwd", [&](auto* tag) {
    using T = std::remove_pointer_t<decltype(tag)>;
    vsplit_tail_fwd<T>(cptr<T>(logits), logits.stride(0), rows, logits.size(1), cptr<int64_t>(target), t_offset,
                       ignore_index, st, ld_st, ptr<float>(lse), ptr<float>(loss_row), ptr<float>(weight),
                       ptr<float>(loss), s);
  });
  return {loss, lse, weight};
}

// ------------------------------------------------------------------ embedding
std::tuple<Tensor, int64_t, int64_t> py_embed_fwd(Tensor tokens, Tensor weight, std::optional<Tensor> pe,
                                                  double scale, double p) {
  check_cuda(tokens, "tokens");
  check_cuda(weight, "weight");
  MP_CHECK(tokens.scalar_type() == at::kLong && tokens.dim() == 2, "embedding: tokens must be int64 [B, S]");
  MP_CHECK(weight.dim() == 2 && weight.size(1) % 8 == 0, "embedding: weight must be [V, E] with E % 8 == 0");
  const int64_t S = tokens.size(1), E = weight.size(1), V = weight.size(0);
  if (pe) {
    check_cuda(*pe, "pe");
    MP_CHECK((pe->scalar_type() == at::kFloat || pe->scalar_type() == weight.scalar_type()) && pe->dim() == 2 &&
                 pe->size(1) == E && pe->size(0) >= S && pe->is_contiguous(),
             "embedding: pe must be a contiguous fp32 or weight-dtype [max_len >= S, E]");
  }
  at::hip::HIPGuardMasqueradingAsCUDA guard(weight.device());
  auto out = at::empty({tokens.size(0), S, E}, weight.options());
  uint64_t seed = 0, offset = 0;
  if (p > 0.0) std::tie(seed, offset) = philox_draw(weight.device(), 4);
  auto s = cur_stream(weight);
  dispatch_fb(weight, "embedding_fwd", [&](auto* tag) {
    using T = std::remove_pointer_t<decltype(tag)>;
    embedding_fwd<T>(cptr<int64_t>(tokens), cptr<T>(weight), pe ? pe->data_ptr() : nullptr,
                     pe ? pe->scalar_type() == at::kFloat : true, ptr<T>(out), tokens.numel(), (int)S, (int)E, V,
                     (float)scale, (float)p, seed, offset, s);
  });
  return {out, (int64_t)seed, (int64_t)offset};
}

// dpe (optional): fp32 [max_len, E] gradient of a learned position table, accumulated.
void py_embed_bwd(Tensor tokens, Tensor dout, Tensor dweight, double scale, double p, int64_t seed, int64_t offset,
                  std::optional<Tensor> dpe) {
  check_cuda(dout, "dout");
  check_cuda(dweight, "dweight");
  check_cuda(tokens, "tokens");
  MP_CHECK(tokens.scalar_type() == at::kLong && tokens.dim() == 2, "embedding_bwd: tokens must be int64 [B, S]");
  MP_CHECK(dweight.scalar_type() == at::kFloat && dweight.dim() == 2, "embedding_bwd: dweight must be fp32 [V, E]");
  const int64_t E = dweight.size(1), V = dweight.size(0);
  MP_CHECK(dout.numel() == tokens.numel() * E, "embedding_bwd: shape mismatch");
  MP_CHECK(E % 8 == 0 && E <= 8192, "embedding_bwd: E must be a multiple of 8 and at most 8192");
  if (dpe) {
    check_cuda(*dpe, "dpe");
    MP_CHECK(dpe->scalar_type() == at::kFloat && dpe->dim() == 2 && dpe->size(1) == E &&
                 dpe->size(0) >= tokens.size(1), "embedding_bwd: dpe must be fp32 [>= S, E]");
  }
  at::hip::HIPGuardMasqueradingAsCUDA guard(dout.device());
  auto s = cur_stream(dout);
  dispatch_fb(dout, "embedding_bwd", [&](auto* tag) {
    using T = std::remove_pointer_t<decltype(tag)>;
    embedding_bwd<T>(cptr<int64_t>(tokens), cptr<T>(dout), ptr<float>(dweight), tokens.numel(), (int)E, V,
                     (float)scale, (float)p, (uint64_t)seed, (uint64_t)offset, s, dpe ? ptr<float>(*dpe) : nullptr,
                     (int)tokens.size(1));
  });
}

// ------------------------------------------------------------------ GEMM
// GEMM operands: bf16 (v_mfma_f32_16x16x32_bf16 kernel) or fp32 (v_mfma_f32_32x32x2_f32 kernel).
// Layout (unit column stride, aligned row stride) is checked by row_stride().
void check_gemm_2d(const Tensor& t, const char* name) {
  MP_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  MP_CHECK(t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kFloat, name, " must be bf16 or fp32");
  MP_CHECK(t.dim() == 2, name, " must be 2-D");
  MP_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
}

// Row stride of a 2-D GEMM operand / output: unit column stride and 16-byte
// aligned rows (the tile kernels move 16-byte chunks), so row-strided views
// -- a column slice of a packed activation -- need no copy.
int64_t row_stride(const Tensor& t, const char* name) {
  MP_CHECK(t.dim() == 2 && (t.stride(1) == 1 || t.size(1) == 1), name, " must have unit column stride");
  const int64_t ld = t.size(0) > 1 ? t.stride(0) : t.size(1);
  MP_CHECK(ld >= t.size(1) && (ld * (int64_t)t.element_size()) % 16 == 0, name,
           ": rows must be 16-byte aligned (row stride ", ld, ")");
  return ld;
}

void check_same_dtype(const Tensor& a, const Tensor& b, const char* what) {
  MP_CHECK(a.scalar_type() == b.scalar_type(), what, ": operand dtypes differ");
}

bool gemm_ok(at::ScalarType t, int64_t M, int64_t N, int64_t K) {
  return t == at::kFloat ? gemm_f32_supported(M, N, K) : gemm_supported(M, N, K);
}

void gemm_run(at::ScalarType t, const GemmArgs& g, hipStream_t s) {
  if (t == at::kFloat) gemm_f32(g, s);
  else gemm_bf16(g, s);
}

bool py_gemm_supported(int64_t M, int64_t N, int64_t K) { return gemm_supported(M, N, K); }
bool py_gemm_f32_supported(int64_t M, int64_t N, int64_t K) { return gemm_f32_supported(M, N, K); }

// y[M,N] = act(x[M,K] . w[N,K]^T + bias) with dropout; optional pre-activation.
// xt (optional, bf16 [K, M]): also written with x^T by the same GEMM (its
// blocks transpose the x tiles they stage anyway), the K-contiguous operand of
// the layer's transposed weight-gradient GEMM (linear_wgrad_xt_segments).
std::tuple<Tensor, std::optional<Tensor>, int64_t, int64_t> py_linear_fwd(Tensor x, Tensor w,
                                                                           std::optional<Tensor> bias, int64_t act,
                                                                           double p, bool save_preact,
                                                                           std::optional<Tensor> res,
                                                                           std::optional<Tensor> xt,
                                                                           bool aux_grad,
                                                                           std::optional<Tensor> bits) {
  check_gemm_2d(x, "x");
  check_gemm_2d(w, "w");
  check_same_dtype(x, w, "linear_fwd");
  const auto dt = x.scalar_type();
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  MP_CHECK(w.size(1) == K, "linear_fwd: inner dims differ");
  MP_CHECK(gemm_ok(dt, M, N, K), "linear_fwd: unsupported shape ", M, "x", N, "x", K);
  MP_CHECK(act >= 0 && act <= 2 && p >= 0.0 && p < 1.0, "linear_fwd: bad act/p");
  MP_CHECK(!aux_grad || (act == kActGelu && save_preact && dt == at::kBFloat16),
           "linear_fwd: aux_grad (GELU'(pre) as the saved tensor) needs bf16, GELU and save_preact");
  if (bias) {
    check_cuda(*bias, "bias");
    MP_CHECK(bias->scalar_type() == dt && bias->numel() == N, "linear_fwd: bad bias");
  }
  if (res) {
    check_gemm_2d(*res, "res");
    check_same_dtype(x, *res, "linear_fwd res");
    MP_CHECK(res->size(0) == M && res->size(1) == N, "linear_fwd: res must be [M, N]");
  }
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto y = at::empty({M, N}, x.options());
  std::optional<Tensor> pre;
  if (save_preact) pre = at::empty({M, N}, x.options());
  uint64_t seed = 0, offset = 0;
  if (p > 0.0) std::tie(seed, offset) = philox_draw(x.device(), 4);
  GemmArgs g;
  g.A = x.data_ptr(); g.B = w.data_ptr(); g.C = y.data_ptr();
  g.bias = bias ? bias->data_ptr() : nullptr; g.aux = pre ? pre->data_ptr() : nullptr;
  g.aux_grad = aux_grad;
  if (res) {
    g.res = res->data_ptr();  // y = res + dropout(act(x . w^T + b)): the residual add in the epilogue
    g.ldr = row_stride(*res, "res");
  }
  g.lda = row_stride(x, "x"); g.ldb = row_stride(w, "w"); g.ldc = N; g.M = (int)M; g.N = (int)N; g.K = (int)K;
  g.a_kc = true; g.b_kc = true; g.epi = kEpiStoreAct; g.act = (int)act; g.p = (float)p;
  g.seed = seed; g.offset = offset;
  if (xt) {
    check_gemm_2d(*xt, "xt");
    MP_CHECK(dt == at::kBFloat16 && xt->scalar_type() == dt && xt->size(0) == K && xt->size(1) == M,
             "linear_fwd: xt must be bf16 [K, M]");
    MP_CHECK(gemm_emit_ok((int)act, (float)p, save_preact), "linear_fwd: this epilogue cannot write xt (gemm_emit_ok)");
    g.at = xt->data_ptr();
    g.ldat = row_stride(*xt, "xt");
  }
  if (bits) {  // the output's nonzero mask as bits, for the consumer's dgrad (kActReluBits)
    check_cuda(*bits, "bits");
    MP_CHECK(bits->scalar_type() == at::kByte && bits->dim() == 2 && bits->size(0) == M && bits->size(1) * 8 == N &&
                 bits->stride(1) == 1,
             "linear_fwd: bits must be uint8 [M, N / 8] with unit column stride");
    g.bits = bits->data_ptr();
    g.ldbits = bits->stride(0);
    MP_CHECK(dt == at::kBFloat16 && gemm_bits_ok(g), "linear_fwd: this launch cannot write bits (gemm_bits_ok)");
  }
  gemm_run(dt, g, cur_stream(x));
  return {y, pre, (int64_t)seed, (int64_t)offset};
}

// Split-K (bf16 GEMMs on under-filled grids, gemm_splitk_factor): the fp32
// partials' workspace, from the stream-ordered caching allocator (released
// after the kernels queued on this stream that use it).  Empty when unsplit.
Tensor split_k_workspace(GemmArgs& g, at::ScalarType dt, const Tensor& like) {
  if (dt != at::kBFloat16) return Tensor();
  const int splits = gemm_splitk_factor(g);
  if (splits <= 1) return Tensor();
  Tensor ws = at::empty({splits, (int64_t)g.M, (int64_t)g.N}, like.options().dtype(at::kFloat));
  g.k_splits = splits;
  g.ws = ws.data_ptr<float>();
  return ws;
}

// dx[M,K] = dy[M,N] . w[N,K]
// dx = dy . w (+ res): `res` is the gradient the input receives from its
// other consumer (a residual branch), added in the epilogue.
// act (optional, with `saved`): the output is the gradient of the activation's
// INPUT -- act'(saved) (and the forward's dropout mask: p, seed, offset) applied
// in the epilogue (GELU: saved = the pre-activation; ReLU: saved = the output).
Tensor py_linear_dgrad(Tensor dy, Tensor w, std::optional<Tensor> res, std::optional<Tensor> out, int64_t act,
                       std::optional<Tensor> saved, double p, int64_t seed, int64_t offset) {
  check_gemm_2d(dy, "dy");
  check_gemm_2d(w, "w");
  check_same_dtype(dy, w, "linear_dgrad");
  const auto dt = dy.scalar_type();
  const int64_t M = dy.size(0), N = dy.size(1), K = w.size(1);
  MP_CHECK(w.size(0) == N, "linear_dgrad: inner dims differ");
  MP_CHECK(gemm_ok(dt, M, K, N), "linear_dgrad: unsupported shape");
  if (res) {
    check_gemm_2d(*res, "res");
    check_same_dtype(dy, *res, "linear_dgrad res");
    MP_CHECK(res->size(0) == M && res->size(1) == K, "linear_dgrad: res must be [M, K]");
  }
  MP_CHECK(act == kActNone || act == kActRelu || act == kActGelu || act == kActSavedGrad || act == kActReluBits,
           "linear_dgrad: bad act");
  if (act != kActNone) {
    MP_CHECK(saved.has_value() && dt == at::kBFloat16 && !res, "linear_dgrad: the activation backward needs bf16 "
             "operands, the saved tensor and no residual addend");
    if (act == kActReluBits) {
      check_cuda(*saved, "saved");
      MP_CHECK(saved->scalar_type() == at::kByte && saved->dim() == 2 && saved->size(0) == M &&
                   saved->size(1) * 8 == K && saved->stride(1) == 1,
               "linear_dgrad: the ReLU bit mask must be uint8 [M, K / 8] with unit column stride");
    } else {
      check_gemm_2d(*saved, "saved");
      check_same_dtype(dy, *saved, "linear_dgrad saved");
      MP_CHECK(saved->size(0) == M && saved->size(1) == K, "linear_dgrad: saved must be [M, K]");
    }
    MP_CHECK(p >= 0.0 && p < 1.0, "linear_dgrad: bad p");
  }
  at::hip::HIPGuardMasqueradingAsCUDA guard(dy.device());
  Tensor dx;
  if (out) {  // a (row-strided) destination, e.g. the columns of a packed gradient message
    check_gemm_2d(*out, "out");
    MP_CHECK(out->size(0) == M && out->size(1) == K && out->scalar_type() == dt, "linear_dgrad: bad out");
    dx = *out;
  } else {
    dx = at::empty({M, K}, dy.options());
  }
  GemmArgs g;
  g.A = dy.data_ptr(); g.B = w.data_ptr(); g.C = dx.data_ptr();
  if (res) {
    g.res = res->data_ptr();
    g.ldr = row_stride(*res, "res");
  }
  g.lda = row_stride(dy, "dy"); g.ldb = row_stride(w, "w"); g.ldc = row_stride(dx, "out");
  g.M = (int)M; g.N = (int)K; g.K = (int)N;
  g.a_kc = true; g.b_kc = false; g.epi = kEpiStoreAct;
  if (act != kActNone) {
    g.dact_in = saved->data_ptr();
    g.ldd = act == kActReluBits ? saved->stride(0) : row_stride(*saved, "saved");
    g.dact = (int)act;
    if (act == kActRelu || act == kActReluBits) {  // the saved output's sign (or its bit) is the mask as well
      g.dact_scale = p > 0.0 ? (float)(1.0 / (1.0 - p)) : 1.f;
    } else {
      g.p = (float)p;
      g.seed = (uint64_t)seed;
      g.offset = (uint64_t)offset;
    }
  }
  Tensor ws = split_k_workspace(g, dt, dy);
  gemm_run(dt, g, cur_stream(dy));
  return dx;
}

// main_grad[N,K] (fp32) += dy[T,N]^T . x[T,K]   (= when !accumulate)
void py_linear_wgrad(Tensor dy, Tensor x, Tensor main_grad, bool accumulate) {
  check_gemm_2d(dy, "dy");
  check_gemm_2d(x, "x");
  check_same_dtype(dy, x, "linear_wgrad");
  const auto dt = dy.scalar_type();
  check_cuda(main_grad, "main_grad");
  const int64_t T = dy.size(0), N = dy.size(1), K = x.size(1);
  MP_CHECK(x.size(0) == T, "linear_wgrad: token dims differ");
  MP_CHECK(main_grad.scalar_type() == at::kFloat && main_grad.numel() == N * K, "linear_wgrad: bad main_grad");
  MP_CHECK(gemm_ok(dt, N, K, T), "linear_wgrad: unsupported shape");
  at::hip::HIPGuardMasqueradingAsCUDA guard(dy.device());
  GemmArgs g;
  g.A = dy.data_ptr(); g.B = x.data_ptr(); g.C = main_grad.data_ptr();
  g.lda = row_stride(dy, "dy"); g.ldb = row_stride(x, "x"); g.ldc = K; g.M = (int)N; g.N = (int)K; g.K = (int)T;
  g.a_kc = false; g.b_kc = false; g.epi = accumulate ? kEpiAccumF32 : kEpiStoreF32;
  Tensor ws = split_k_workspace(g, dt, dy);
  gemm_run(dt, g, cur_stream(dy));
}

// Deferred bias gradient over the micro-batches of a step: out (+)= column sums
// of every [rows, cols] input, one stage-1 launch per input into a shared
// partial buffer and ONE reduction.
// x^T of a 2-D bf16/fp16 tensor [R, C] (row stride >= C, unit column stride)
// into a new contiguous [C, R] tensor: the K-contiguous operand of
// linear_wgrad_xt_segments when the flush transposes x itself (ops/linear.py).
Tensor py_transpose_b16(Tensor x) {
  MP_CHECK(x.is_cuda(), "x must be a GPU tensor");
  MP_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.element_size() == 2, "transpose_b16: x must be 2-D, 2-byte, unit column stride");
  const int64_t R = x.size(0), C = x.size(1), ld = x.stride(0);
  MP_CHECK(R % 8 == 0 && C % 8 == 0 && ld % 8 == 0 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
           "transpose_b16: rows, cols and row stride must be multiples of 8, x 16-byte aligned");
  MP_CHECK(C / 256 < 65536, "transpose_b16: too many columns");
  at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto out = at::empty({C, R}, x.options());
  mipipe::transpose_b16(reinterpret_cast<const uint16_t*>(x.data_ptr()), R, C, ld,
                        reinterpret_cast<uint16_t*>(out.data_ptr()), R, cur_stream(x));
  return out;
}

void py_column_sum_segments(std::vector<Tensor> xs, Tensor out, bool accumulate) {
  MP_CHECK(!xs.empty(), "column_sum_segments: empty list");
  check_cuda(out, "out");
  const int64_t cols = xs[0].size(-1);
  MP_CHECK(out.numel() == cols && out.is_contiguous(), "column_sum_segments: bad out");
  const bool out_f32 = out.scalar_type() == at::kFloat;
  MP_CHECK(out_f32 || out.scalar_type() == xs[0].scalar_type(), "column_sum_segments: out must be fp32 or the input dtype");
  std::vector<int64_t> rows(xs.size());
  std::vector<int> parts(xs.size());
  int total = 0;
  for (size_t i = 0; i < xs.size(); ++i) {
    check_cuda(xs[i], "x");
    MP_CHECK(xs[i].is_contiguous() && xs[i].size(-1) == cols && xs[i].scalar_type() == xs[0].scalar_type(),
             "column_sum_segments: inputs must be contiguous with equal width and dtype");
    rows[i] = xs[i].numel() / std::max<int64_t>(cols, 1);
    parts[i] = colsum_parts(rows[i], cols);
    total += parts[i];
  }
  at::hip::HIPGuardMasqueradingAsCUDA guard(out.device());
  auto part = at::empty({total, cols}, xs[0].options().dtype(at::kFloat));
  auto s = cur_stream(out);
  int first = 0;
  bool uniform = true;
  for (size_t i = 1; i < xs.size(); ++i) uniform = uniform && rows[i] == rows[0];
  if (uniform && cols % 8 == 0) {
    // every segment's stage 1 in one launch per kColsumSegs inputs (grid.z = segment)
    for (size_t i0 = 0; i0 < xs.size(); i0 += kColsumSegs) {
      const int n = (int)std::min<size_t>(kColsumSegs, xs.size() - i0);
      ColsumSegs segs;
      for (int j = 0; j < n; ++j) segs.p[j] = xs[i0 + j].data_ptr();
      dispatch_fb(xs[0], "column_sum_segments", [&](auto* tag) {
        using T = std::remove_pointer_t<decltype(tag)>;
        MP_CHECK(column_sum_partial_multi<T>(segs, n, rows[0], (int)cols, ptr<float>(part) + (int64_t)first * cols,
                                             parts[0], s),
                 "column_sum_segments: multi-segment launch refused");
      });
      first += n * parts[0];
    }
    reduce_parts(ptr<float>(part), nullptr, total, (int)cols, out.data_ptr(), nullptr, out_f32, accumulate, s);
    return;
  }
  for (size_t i = 0; i < xs.size(); ++i) {
    dispatch_fb(xs[i], "column_sum_segments", [&](auto* tag) {
      using T = std::remove_pointer_t<decltype(tag)>;
      column_sum_partial<T>(cptr<T>(xs[i]), rows[i], (int)cols, ptr<float>(part) + (int64_t)first * cols, parts[i], s);
    });
    first += parts[i];
  }
  reduce_parts(ptr<float>(part), nullptr, total, (int)cols, out.data_ptr(), nullptr, out_f32, accumulate, s);
}

// Deferred weight gradient over the micro-batches of a step:
//   main_grad[N, K] += sum_i dy_i^T . x_i
// as K-segmented GEMMs (up to GemmArgs::kMaxSegs micro-batches per launch),
// so the fp32 read-modify-write of main_grad happens once per launch instead
// of once per micro-batch and K is long enough to amortise the tile prologue.
// accumulate = false: the FIRST launch overwrites main_grad (its first write of
// the step after a lazy zero_grad), later launches accumulate.
// bias_grad (optional, fp32 [N]): the bias gradient colsum(dy) folded into the
// same GEMMs (GemmArgs::rowsum, accumulated); returns false (nothing added to
// bias_grad) when the shape cannot take the fold -- the caller then reduces it.
bool py_linear_wgrad_segments(std::vector<Tensor> dys, std::vector<Tensor> xs, Tensor main_grad, bool accumulate,
                              std::optional<Tensor> bias_grad) {
  MP_CHECK(!dys.empty() && dys.size() == xs.size(), "linear_wgrad_segments: need matching non-empty lists");
  check_cuda(main_grad, "main_grad");
  const int64_t T = dys[0].size(0), N = dys[0].size(1), K = xs[0].size(1);
  MP_CHECK(main_grad.scalar_type() == at::kFloat && main_grad.numel() == N * K, "linear_wgrad_segments: bad main_grad");
  const auto dt = dys[0].scalar_type();
  for (size_t i = 0; i < dys.size(); ++i) {
    check_gemm_2d(dys[i], "dy");
    check_gemm_2d(xs[i], "x");
    MP_CHECK(dys[i].scalar_type() == dt && xs[i].scalar_type() == dt, "linear_wgrad_segments: mixed dtypes");
    MP_CHECK(dys[i].size(0) == T && dys[i].size(1) == N && xs[i].size(0) == T && xs[i].size(1) == K,
             "linear_wgrad_segments: every micro-batch needs the same [T, N] / [T, K] shapes");
  }
  MP_CHECK(T % 64 == 0 && gemm_ok(dt, N, K, T), "linear_wgrad_segments: unsupported shape");
  const int64_t lda = row_stride(dys[0], "dy"), ldb = row_stride(xs[0], "x");
  for (size_t i = 1; i < dys.size(); ++i)
    MP_CHECK(row_stride(dys[i], "dy") == lda && row_stride(xs[i], "x") == ldb,
             "linear_wgrad_segments: every micro-batch needs the same row strides");
  at::hip::HIPGuardMasqueradingAsCUDA guard(main_grad.device());
  const int total = (int)dys.size();
  auto args_for = [&](int first) {
    const int n = std::min(GemmArgs::kMaxSegs, total - first);
    GemmArgs g;
    g.C = main_grad.data_ptr();
    g.lda = lda; g.ldb = ldb; g.ldc = K; g.M = (int)N; g.N = (int)K; g.K = (int)(T * n);
    g.a_kc = false; g.b_kc = false; g.epi = (accumulate || first > 0) ? kEpiAccumF32 : kEpiStoreF32;
    g.seg_k = (int)T;
    for (int i = 0; i < n; ++i) {
      g.a_seg[i] = dys[first + i].data_ptr();
      g.b_seg[i] = xs[first + i].data_ptr();
    }
    g.A = g.a_seg[0]; g.B = g.b_seg[0];
    return g;
  };
  bool fold = false;
  if (bias_grad && dt == at::kBFloat16) {
    check_cuda(*bias_grad, "bias_grad");
    MP_CHECK(bias_grad->scalar_type() == at::kFloat && bias_grad->numel() == N && bias_grad->is_contiguous(),
             "linear_wgrad_segments: bias_grad must be a contiguous fp32 [N]");
    fold = true;
    for (int first = 0; first < total && fold; first += GemmArgs::kMaxSegs) fold = gemm_rowsum_ok(args_for(first));
  }
  for (int first = 0; first < total; first += GemmArgs::kMaxSegs) {
    GemmArgs g = args_for(first);
    if (fold) g.rowsum = bias_grad->data_ptr<float>();
    Tensor ws = split_k_workspace(g, dt, main_grad);
    gemm_run(dt, g, cur_stream(main_grad));
  }
  return fold;
}

// The same deferred weight gradient from the transposed inputs x_i^T [K, T]
// (written by the forward GEMMs, linear_fwd(xt=...)):
//   main_grad[N, K] += sum_i (x_i^T . dy_i)^T
// computed as C^T[K, N] with A = x^T read K-contiguous and B = dy read [T, N]
// -- the dgrad layout, one transposing LDS read per operand instead of two
// (profiles/wgrad_layout_probe.txt) -- and stored transposed into main_grad.
// bias_grad: colsum(dy) folded into the same GEMMs (GemmArgs::colsum) when
// the shape allows (returns whether it was).
bool py_linear_wgrad_xt_segments(std::vector<Tensor> dys, std::vector<Tensor> xts, Tensor main_grad,
                                 bool accumulate, std::optional<Tensor> bias_grad) {
  MP_CHECK(!dys.empty() && dys.size() == xts.size(), "linear_wgrad_xt_segments: need matching non-empty lists");
  check_cuda(main_grad, "main_grad");
  const int64_t T = dys[0].size(0), N = dys[0].size(1), K = xts[0].size(0);
  MP_CHECK(main_grad.scalar_type() == at::kFloat && main_grad.numel() == N * K && main_grad.is_contiguous(),
           "linear_wgrad_xt_segments: bad main_grad");
  for (size_t i = 0; i < dys.size(); ++i) {
    check_gemm_2d(dys[i], "dy");
    check_gemm_2d(xts[i], "xt");
    MP_CHECK(dys[i].scalar_type() == at::kBFloat16 && xts[i].scalar_type() == at::kBFloat16,
             "linear_wgrad_xt_segments: bf16 operands only");
    MP_CHECK(dys[i].size(0) == T && dys[i].size(1) == N && xts[i].size(0) == K && xts[i].size(1) == T,
             "linear_wgrad_xt_segments: every micro-batch needs dy [T, N] and xt [K, T]");
  }
  MP_CHECK(T % 64 == 0 && K % 8 == 0 && gemm_supported(K, N, T), "linear_wgrad_xt_segments: unsupported shape");
  const int64_t lda = row_stride(xts[0], "xt"), ldb = row_stride(dys[0], "dy");
  for (size_t i = 1; i < dys.size(); ++i)
    MP_CHECK(row_stride(dys[i], "dy") == ldb && row_stride(xts[i], "xt") == lda,
             "linear_wgrad_xt_segments: every micro-batch needs the same row strides");
  at::hip::HIPGuardMasqueradingAsCUDA guard(main_grad.device());
  const int total = (int)dys.size();
  auto args_for = [&](int first) {
    const int n = std::min(GemmArgs::kMaxSegs, total - first);
    GemmArgs g;
    g.C = main_grad.data_ptr();
    g.lda = lda; g.ldb = ldb; g.ldc = K; g.M = (int)K; g.N = (int)N; g.K = (int)(T * n);
    g.a_kc = true; g.b_kc = false; g.trans_c = true;
    g.epi = (accumulate || first > 0) ? kEpiAccumF32 : kEpiStoreF32;
    g.seg_k = (int)T;
    for (int i = 0; i < n; ++i) {
      g.a_seg[i] = xts[first + i].data_ptr();
      g.b_seg[i] = dys[first + i].data_ptr();
    }
    g.A = g.a_seg[0]; g.B = g.b_seg[0];
    return g;
  };
  bool fold = false;
  if (bias_grad) {
    check_cuda(*bias_grad, "bias_grad");
    MP_CHECK(bias_grad->scalar_type() == at::kFloat && bias_grad->numel() == N && bias_grad->is_contiguous(),
             "linear_wgrad_xt_segments: bias_grad must be a contiguous fp32 [N]");
    fold = true;
    for (int first = 0; first < total && fold; first += GemmArgs::kMaxSegs) fold = gemm_colsum_ok(args_for(first));
  }
  for (int first = 0; first < total; first += GemmArgs::kMaxSegs) {
    GemmArgs g = args_for(first);
    if (fold) g.colsum = bias_grad->data_ptr<float>();
    Tensor ws = split_k_workspace(g, at::kBFloat16, main_grad);
    Tensor cws;
    if (fold && g.k_splits > 1) {
      cws = at::empty({(int64_t)g.k_splits, N}, main_grad.options());
      g.colsum_ws = cws.data_ptr<float>();
    }
    gemm_bf16(g, cur_stream(main_grad));
  }
  return fold;
}

// Generic test entry: C[M,N] (fp32) = A . B with A given [M,K] (a_kc) or [K,M],
// B given [N,K] (b_kc) or [K,N].
Tensor py_gemm_f32(Tensor a, Tensor b, bool a_kc, bool b_kc) {
  check_gemm_2d(a, "a");
  check_gemm_2d(b, "b");
  check_same_dtype(a, b, "gemm");
  const auto dt = a.scalar_type();
  const int64_t M = a_kc ? a.size(0) : a.size(1);
  const int64_t K = a_kc ? a.size(1) : a.size(0);
  const int64_t N = b_kc ? b.size(0) : b.size(1);
  MP_CHECK((b_kc ? b.size(1) : b.size(0)) == K, "gemm: inner dims differ");
  MP_CHECK(gemm_ok(dt, M, N, K), "gemm: unsupported shape");
  at::hip::HIPGuardMasqueradingAsCUDA guard(a.device());
  auto c = at::empty({M, N}, a.options().dtype(at::kFloat));
  GemmArgs g;
  g.A = a.data_ptr(); g.B = b.data_ptr(); g.C = c.data_ptr();
  g.lda = row_stride(a, "a"); g.ldb = row_stride(b, "b"); g.ldc = N; g.M = (int)M; g.N = (int)N; g.K = (int)K;
  g.a_kc = a_kc; g.b_kc = b_kc; g.epi = kEpiStoreF32;
  gemm_run(dt, g, cur_stream(a));
  return c;
}

// ------------------------------------------------------------------ attention
// q, k, v: [B, S, H, D] views (unit stride on D, identical strides), bf16.
// q, k, v: bf16 (attention.hip) or fp32 (attention_f32.hip).
void check_bshd(const Tensor& t, const char* name) {
  MP_CHECK(t.is_cuda() && (t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kFloat), name,
           " must be a bf16 or fp32 GPU tensor");
  MP_CHECK(t.dim() == 4 && t.stride(3) == 1, name, " must be [B, S, H, D] with unit stride on D");
  const int64_t v = 16 / t.element_size();  // elements per 16 bytes
  MP_CHECK(t.stride(0) % v == 0 && t.stride(1) % v == 0 && t.stride(2) % v == 0 &&
               reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
           name, ": strides must keep 16-byte alignment");
}

bool attn_ok(at::ScalarType t, int S, int D) {
  return t == at::kFloat ? attention_f32_supported(S, D) : attention_supported(S, D);
}

void fill_qkv(AttnArgs& a, const Tensor& q, const Tensor& k, const Tensor& v) {
  check_bshd(q, "q");
  check_bshd(k, "k");
  check_bshd(v, "v");
  MP_CHECK(q.sizes() == k.sizes() && q.sizes() == v.sizes(), "attention: q, k, v shapes differ");
  MP_CHECK(q.strides() == k.strides() && q.strides() == v.strides(), "attention: q, k, v strides differ");
  MP_CHECK(q.scalar_type() == k.scalar_type() && q.scalar_type() == v.scalar_type(), "attention: q, k, v dtypes differ");
  a.q = q.data_ptr(); a.k = k.data_ptr(); a.v = v.data_ptr();
  a.B = (int)q.size(0); a.S = (int)q.size(1); a.H = (int)q.size(2); a.D = (int)q.size(3);
  a.sb_qkv = q.stride(0); a.ld_qkv = q.stride(1); a.sh_qkv = q.stride(2);
  MP_CHECK(attn_ok(q.scalar_type(), a.S, a.D), "attention: unsupported S=", a.S, " D=", a.D, " for ",
           q.scalar_type(), " (bf16: S % 64 == 0, D in {64,128,256}; fp32: S % 32 == 0, D in {64,128})");
}

// bf16 D = 64, S >= 256 run the long-sequence kernels (attention_long.hip);
// MIPIPE_ATTN_LONG=0 selects the previous kernels (A/B runs).
bool use_long(const Tensor& q, int S, int D) {
  static const int on = [] {
    const char* e = getenv("MIPIPE_ATTN_LONG");
    return e == nullptr ? 1 : atoi(e);
  }();
  return on && q.scalar_type() == at::kBFloat16 && attention_long_supported(S, D);
}

// Returns (o, lse, seed, offset, dropout keep bits): the bits tensor (int32
// [B*H, S/32, S]) is non-empty only for the long-sequence kernels with p > 0
// and must be handed back to attention_bwd.
// `words` (with the Philox draw it was made under): keep words an earlier forward of this same draw returned
// (a checkpoint's first forward, reused by its recompute) -- read instead of made, when the draw matches.
std::tuple<Tensor, Tensor, int64_t, int64_t, Tensor> py_attention_fwd(Tensor q, Tensor k, Tensor v, bool causal,
                                                                      double p, double scale, int64_t kv_len,
                                                                      std::optional<Tensor> words, int64_t words_seed,
                                                                      int64_t words_offset) {
  AttnArgs a;
  fill_qkv(a, q, k, v);
  MP_CHECK(p >= 0.0 && p < 1.0, "attention: bad dropout p");
  MP_CHECK(kv_len == 0 || (q.scalar_type() == at::kFloat && kv_len > 0 && kv_len <= a.S),
           "attention: kv_len (a key-length bound) is for fp32, 0 < kv_len <= S");
  a.kv_len = (int)kv_len;
  at::hip::HIPGuardMasqueradingAsCUDA guard(q.device());
  auto o = at::empty({a.B, a.S, a.H, a.D}, q.options());
  auto lse = at::empty({a.B, a.H, a.S}, q.options().dtype(at::kFloat));
  uint64_t seed = 0, offset = 0;
  if (p > 0.0) std::tie(seed, offset) = philox_draw(q.device(), 4);
  a.o = o.data_ptr(); a.sb_o = o.stride(0); a.ld_o = o.stride(1); a.sh_o = o.stride(2);
  a.lse = ptr<float>(lse);
  a.scale = (float)scale; a.p = (float)p; a.seed = seed; a.offset = offset; a.causal = causal;
  Tensor bits = at::empty({0}, q.options().dtype(at::kInt));
  if (q.scalar_type() == at::kFloat) {
    attention_f32_fwd(a, cur_stream(q));
  } else if (use_long(q, a.S, a.D)) {
    bool reuse = false;
    if (p > 0.0) {
      const std::vector<int64_t> shape = {(int64_t)a.B * a.H, a.S / 32, a.S};
      reuse = words && words->defined() && words->sizes() == at::IntArrayRef(shape) &&
              words->scalar_type() == at::kInt && words->is_contiguous() && words->device() == q.device() &&
              (uint64_t)words_seed == seed && (uint64_t)words_offset == offset;
      bits = reuse ? *words : at::empty(shape, q.options().dtype(at::kInt));
      a.dmask = reinterpret_cast<uint32_t*>(bits.data_ptr());
    }
    if (reuse) attention_long_fwd_words(a, cur_stream(q));
    else attention_long_fwd(a, cur_stream(q));
  } else {
    attention_fwd(a, cur_stream(q));
  }
  return {o, lse, (int64_t)seed, (int64_t)offset, bits};
}

void py_attention_bwd(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse, bool causal, double p,
                      double scale, int64_t seed, int64_t offset, Tensor dq, Tensor dk, Tensor dv,
                      std::optional<Tensor> bits, int64_t kv_len) {
  AttnArgs a;
  fill_qkv(a, q, k, v);
  MP_CHECK(kv_len == 0 || (q.scalar_type() == at::kFloat && kv_len > 0 && kv_len <= a.S),
           "attention_bwd: kv_len (a key-length bound) is for fp32, 0 < kv_len <= S");
  a.kv_len = (int)kv_len;
  check_bshd(o, "o");
  check_bshd(dout, "dout");
  MP_CHECK(o.strides() == dout.strides() && o.sizes() == dout.sizes(), "attention_bwd: o/dout layout differs");
  MP_CHECK(o.scalar_type() == q.scalar_type() && dout.scalar_type() == q.scalar_type() &&
               dq.scalar_type() == q.scalar_type(), "attention_bwd: dtypes differ");
  MP_CHECK(dq.strides() == q.strides() && dk.strides() == q.strides() && dv.strides() == q.strides(),
           "attention_bwd: gradient buffers must share q's layout");
  MP_CHECK(lse.scalar_type() == at::kFloat && lse.numel() == (int64_t)a.B * a.H * a.S, "attention_bwd: bad lse");
  at::hip::HIPGuardMasqueradingAsCUDA guard(q.device());
  auto delta = at::empty({a.B, a.H, a.S}, q.options().dtype(at::kFloat));
  a.o = o.data_ptr(); a.dout = dout.data_ptr();
  a.sb_o = o.stride(0); a.ld_o = o.stride(1); a.sh_o = o.stride(2);
  a.dq = dq.data_ptr(); a.dk = dk.data_ptr(); a.dv = dv.data_ptr();
  a.lse = ptr<float>(lse); a.delta = ptr<float>(delta);
  a.scale = (float)scale; a.p = (float)p; a.seed = (uint64_t)seed; a.offset = (uint64_t)offset; a.causal = causal;
  if (q.scalar_type() == at::kFloat) {
    attention_f32_bwd(a, cur_stream(q));
  } else if (use_long(q, a.S, a.D)) {
    if (p > 0.0) {
      MP_CHECK(bits && bits->is_cuda() && bits->scalar_type() == at::kInt &&
                   bits->numel() == (int64_t)a.B * a.H * (a.S / 32) * a.S,
               "attention_bwd: the long-sequence kernels need the forward's dropout bits");
      a.dmask = reinterpret_cast<uint32_t*>(bits->data_ptr());
    }
    attention_long_bwd(a, cur_stream(q));
  } else {
    attention_bwd(a, cur_stream(q));
  }
}

// ------------------------------------------------------------------ optimizer
Tensor py_sumsq(Tensor g) {
  check_cuda(g, "g");
  MP_CHECK(g.scalar_type() == at::kFloat, "sumsq: fp32 only");
  at::hip::HIPGuardMasqueradingAsCUDA guard(g.device());
  auto out = at::empty({1}, g.options());
  const int nparts = sumsq_parts(g.numel());
  auto part = at::empty({nparts}, g.options());
  sumsq(cptr<float>(g), g.numel(), ptr<float>(part), nparts, ptr<float>(out), cur_stream(g));
  return out;
}

void py_adam(Tensor master, std::optional<Tensor> model, Tensor grad, Tensor m, Tensor v, double lr, double b1,
             double b2, double eps, double wd, double bc1, double bc2, std::optional<Tensor> sumsq_t, double max_norm,
             bool adamw) {
  for (auto* t : {&master, &grad, &m, &v}) {
    check_cuda(*t, "adam buffer");
    MP_CHECK(t->scalar_type() == at::kFloat, "adam: master/grad/m/v must be fp32");
    MP_CHECK(t->numel() == master.numel(), "adam: size mismatch");
    MP_CHECK(t->is_contiguous() && reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0,
             "adam: buffers must be contiguous and 16-byte aligned (vectorised kernel)");
  }
  if (model) {
    MP_CHECK(model->numel() == master.numel() && model->is_contiguous(), "adam: model size mismatch");
    MP_CHECK(reinterpret_cast<uintptr_t>(model->data_ptr()) % 16 == 0, "adam: model copy must be 16-byte aligned");
  }
  if (sumsq_t) MP_CHECK(sumsq_t->scalar_type() == at::kFloat && sumsq_t->numel() == 1, "adam: bad sumsq");
  at::hip::HIPGuardMasqueradingAsCUDA guard(master.device());
  AdamHyper h;
  h.lr = (float)lr; h.beta1 = (float)b1; h.beta2 = (float)b2; h.eps = (float)eps; h.weight_decay = (float)wd;
  h.bias_correction1 = (float)bc1; h.bias_correction2 = (float)bc2; h.max_norm = (float)max_norm; h.adamw = adamw;
  auto s = cur_stream(master);
  const float* sq = sumsq_t ? cptr<float>(*sumsq_t) : nullptr;
  if (!model) {
    adam_step<float>(ptr<float>(master), (float*)nullptr, cptr<float>(grad), ptr<float>(m), ptr<float>(v),
                     master.numel(), h, sq, s);
  } else if (model->scalar_type() == at::kBFloat16) {
    adam_step<bf16_t>(ptr<float>(master), ptr<bf16_t>(*model), cptr<float>(grad), ptr<float>(m), ptr<float>(v),
                      master.numel(), h, sq, s);
  } else {
    MP_CHECK(model->scalar_type() == at::kFloat, "adam: model copy must be bf16 or fp32");
    adam_step<float>(ptr<float>(master), ptr<float>(*model), cptr<float>(grad), ptr<float>(m), ptr<float>(v),
                     master.numel(), h, sq, s);
  }
}

}  // namespace
}  // namespace mipipe

// ------------------------------------------------------------------ ipc links
// Python face of mipipe::ipc::Link (runtime/ipc.h).  Host-blocking calls drop
// the GIL so watchdog threads keep running while a rank waits for its peer.
namespace {

namespace ipc = mipipe::ipc;

void ipc_check_tensor(const Tensor& t, const ipc::Link& L) {
  MP_CHECK(t.is_contiguous(), "ipc link: tensors must be contiguous");
  MP_CHECK(L.host_mode() ? !t.is_cuda() : t.is_cuda(), "ipc link: host links move CPU tensors, device links GPU tensors");
}

}  // namespace

// Defined in the build-generated source_digest.cpp (mipipe/build.py): the
// digest of the sources this binary was compiled from, checked at import by
// mipipe/_native_loader.py.
extern "C" const char* mipipe_source_digest();

PYBIND11_MODULE(_C, m) {
  m.def("source_digest", []() { return std::string(mipipe_source_digest()); });
  m.def("adam_set_variant", &mipipe::adam_set_variant);
  py::class_<ipc::Link>(m, "IpcLink")
      .def_static("create", &ipc::Link::create, py::arg("name"), py::arg("device"), py::arg("nslots"),
                  py::arg("slot_bytes"))
      .def_static("attach", &ipc::Link::attach, py::arg("name"), py::arg("device"), py::arg("engine") = 0,
                  py::arg("timeout") = 60.0, py::call_guard<py::gil_scoped_release>())
      .def("send",
           [](ipc::Link& L, Tensor src, int64_t producer, double timeout) {
             ipc_check_tensor(src, L);
             const void* p = src.data_ptr();
             const size_t n = src.nbytes();
             py::gil_scoped_release nogil;
             return L.send(p, n, reinterpret_cast<hipStream_t>(producer), timeout);
           },
           py::arg("src"), py::arg("producer_stream"), py::arg("timeout") = 300.0)
      .def("post", &ipc::Link::post)
      .def("wait",
           [](ipc::Link& L, uint64_t seq, Tensor dst, int64_t consumer, double timeout) {
             ipc_check_tensor(dst, L);
             void* p = dst.data_ptr();
             const size_t n = dst.nbytes();
             py::gil_scoped_release nogil;
             L.wait(seq, p, n, reinterpret_cast<hipStream_t>(consumer), timeout);
           },
           py::arg("seq"), py::arg("dst"), py::arg("consumer_stream"), py::arg("timeout") = 300.0)
      // Zero-copy receive (device links): the consumer stream waits for message
      // `seq` on the GPU and the returned tensor IS its slot (no copy), valid
      // until release(seq).  The tensor does not own the memory: the Link (and
      // its Python owner) must outlive it.
      .def("slot_tensor",
           [](ipc::Link& L, uint64_t seq, std::vector<int64_t> shape, py::object dtype, int64_t device) {
             MP_CHECK(!L.host_mode() && !L.is_sender(), "ipc slot_tensor: receiving device links only");
             const auto st = torch::python::detail::py_object_to_dtype(dtype);
             int64_t n = 1;
             for (auto d : shape) n *= d;
             MP_CHECK(n * (int64_t)c10::elementSize(st) <= L.slot_bytes(), "ipc slot_tensor: tensor larger than a slot");
             return at::from_blob(L.slot_ptr(seq), shape,
                                  at::TensorOptions().dtype(st).device(at::kCUDA, (c10::DeviceIndex)device));
           },
           py::arg("seq"), py::arg("shape"), py::arg("dtype"), py::arg("device"))
      .def("acquire",
           [](ipc::Link& L, uint64_t seq, int64_t consumer) { L.acquire(seq, reinterpret_cast<hipStream_t>(consumer)); },
           py::arg("seq"), py::arg("consumer_stream"))
      .def("release",
           [](ipc::Link& L, uint64_t seq, int64_t consumer) { L.release(seq, reinterpret_cast<hipStream_t>(consumer)); },
           py::arg("seq"), py::arg("consumer_stream"))
      // several messages at once: one counter write for the in-order prefix
      .def("release_many",
           [](ipc::Link& L, std::vector<uint64_t> seqs, int64_t consumer) {
             L.release(seqs, reinterpret_cast<hipStream_t>(consumer));
           },
           py::arg("seqs"), py::arg("consumer_stream"))
      .def("done", &ipc::Link::done)
      .def("abort", &ipc::Link::abort)
      .def("drain", &ipc::Link::drain, py::arg("timeout_s"), py::call_guard<py::gil_scoped_release>())
      .def("message_bytes", &ipc::Link::message_bytes)
      .def("unlink", &ipc::Link::unlink)
      .def("describe", &ipc::Link::describe)
      .def_property_readonly("copy_stream", [](const ipc::Link& L) { return reinterpret_cast<int64_t>(L.copy_stream()); })
      .def_property_readonly("inline_copy", &ipc::Link::inline_copy)
      .def_property_readonly("dma_engine", &ipc::Link::dma_engine)
      .def_property_readonly("nslots", &ipc::Link::nslots)
      .def_property_readonly("slot_bytes", &ipc::Link::slot_bytes)
      .def_property_readonly("host_mode", &ipc::Link::host_mode)
      .def_property_readonly("is_sender", &ipc::Link::is_sender);
  using namespace mipipe;
  m.doc() = "mipipe native runtime + CDNA4 HIP kernels (gfx950)";
  // runtime
  m.def("stream_pool_acquire", &py_stream_acquire, py::arg("device"), py::arg("priority") = -1);
  m.def("stream_wait", &py_stream_wait);
  m.def("peer_copy", &py_peer_copy, py::arg("dst"), py::arg("src"), py::arg("src_stream"), py::arg("dst_stream"),
        py::arg("src_device"), py::arg("dst_device"), py::arg("engine") = 0);
  m.def("enable_peer_access", [](std::vector<int> d) { rt::enable_peer_access(d); });
  m.def("can_access_peer", [](int d, int q) { return rt::can_access_peer(d, q); });
  m.def("copy_nocu",
        [](Tensor dst, Tensor src, int64_t stream) {
          MP_CHECK(dst.is_cuda() && src.is_cuda() && dst.nbytes() == src.nbytes(), "copy_nocu: equal device tensors");
          return rt::copy_nocu(dst.data_ptr(), src.data_ptr(), src.nbytes(), reinterpret_cast<hipStream_t>(stream));
        },
        py::arg("dst"), py::arg("src"), py::arg("stream"));
  m.def("hip_runtime_version", []() {
    int v = 0;
    (void)hipRuntimeGetVersion(&v);
    return v;
  });
  m.def("range_push", [](const std::string& s) { rt::range_push(s); });
  m.def("range_pop", []() { rt::range_pop(); });
  m.def("mark", [](const std::string& s) { rt::mark(s); });
  m.def("gpu_sleep", &py_gpu_sleep);
  m.def("philox_draw", [](int64_t device, int64_t inc) {
    auto r = philox_draw(at::Device(at::kCUDA, (c10::DeviceIndex)device), (uint64_t)inc);
    return std::make_pair((int64_t)r.first, (int64_t)r.second);
  });
  // kernels
  m.def("layernorm_fwd", &py_layernorm_fwd);
  m.def("layernorm_bwd", &py_layernorm_bwd, py::arg("dy"), py::arg("z"), py::arg("mean"), py::arg("rstd"),
        py::arg("gamma"), py::arg("p"), py::arg("seed"), py::arg("offset"), py::arg("acc_gamma") = py::none(),
        py::arg("acc_beta") = py::none(), py::arg("addend") = py::none());
  m.def("bias_act_fwd", &py_bias_act_fwd);
  m.def("bias_act_bwd", &py_bias_act_bwd, py::arg("dy"), py::arg("saved"), py::arg("bias"), py::arg("act"),
        py::arg("p"), py::arg("seed"), py::arg("offset"), py::arg("need_dbias"), py::arg("dbias_acc") = py::none());
  m.def("column_sum", &py_column_sum, py::arg("x"), py::arg("out") = py::none(), py::arg("accumulate") = false);
  m.def("cross_entropy_fwd", &py_ce_fwd, py::arg("logits"), py::arg("target"), py::arg("ignore_index"),
        py::arg("t_offset") = 0);
  m.def("cross_entropy_bwd", &py_ce_bwd, py::arg("logits"), py::arg("target"), py::arg("lse"), py::arg("scale"),
        py::arg("ignore_index"), py::arg("row_scale") = py::none(), py::arg("out") = py::none(),
        py::arg("zero_pad") = false, py::arg("t_offset") = 0, py::arg("stat_out") = py::none());
  m.def("cross_entropy_mean_fwd", &py_ce_mean_fwd, py::arg("logits"), py::arg("target"), py::arg("ignore_index"));
  m.def("vsplit_head_fwd", &py_vsplit_head_fwd);
  m.def("vsplit_tail_fwd", &py_vsplit_tail_fwd);
  m.def("embedding_fwd", &py_embed_fwd);
  m.def("embedding_bwd", &py_embed_bwd, py::arg("tokens"), py::arg("dout"), py::arg("dweight"), py::arg("scale"),
        py::arg("p"), py::arg("seed"), py::arg("offset"), py::arg("dpe") = py::none());
  m.def("attention_supported", [](int64_t S, int64_t D) { return attention_supported((int)S, (int)D); });
  m.def("attention_f32_supported", [](int64_t S, int64_t D) { return attention_f32_supported((int)S, (int)D); });
  m.def("attention_fwd", &py_attention_fwd, py::arg("q"), py::arg("k"), py::arg("v"), py::arg("causal"), py::arg("p"),
        py::arg("scale"), py::arg("kv_len") = 0, py::arg("words") = py::none(), py::arg("words_seed") = 0,
        py::arg("words_offset") = 0);
  m.def("attention_bwd", &py_attention_bwd, py::arg("dout"), py::arg("q"), py::arg("k"), py::arg("v"), py::arg("o"),
        py::arg("lse"), py::arg("causal"), py::arg("p"), py::arg("scale"), py::arg("seed"), py::arg("offset"),
        py::arg("dq"), py::arg("dk"), py::arg("dv"), py::arg("bits") = py::none(), py::arg("kv_len") = 0);
  m.def("attention_long_supported", [](int64_t S, int64_t D) { return attention_long_supported((int)S, (int)D); });
  m.def("attention_long_set_fused_rng", &attention_long_set_fused_rng,
        "long-sequence attention: make the dropout keep words inside the forward kernel (true, default) or in a "
        "kernel of their own before it (false)");
  m.def("gemm_supported", &py_gemm_supported);
  m.def("gemm_f32_supported", &py_gemm_f32_supported);
  m.def("attention_set_fused_bwd", &attention_set_fused_bwd);
  m.def("gemm_set_schedule", &gemm_set_schedule,
        "256x256 GEMM main loop: 7 whole-tile ping-pong (default, the only one in the product build); a "
        "--gemm-ab build also has the A/B schedules 0-6 (kernels.h).  Returns false for a schedule not built in.");
  m.def("gemm_get_schedule", &gemm_get_schedule);
  m.def("gemm_ab_build", &gemm_ab_build, "true if the A/B GEMM schedules 0-6 are compiled in (-DMIPIPE_GEMM_AB)");
  m.def("gemm_set_rounds", &gemm_set_rounds,
        "multi-round GEMM grids whose last round is at most half full: 0 one launch, 1 (default) one launch per round "
        "of tiles when K >= 4096, 2 one launch per round at any K");
  m.def("gemm_set_splitk", &gemm_set_splitk, "split-K factor of under-filled long-K GEMMs: 0 off, 1 auto (default), n >= 2 forced");
  m.def("gemm_set_waves", &gemm_set_waves,
        "256x256 GEMM blocks: 4 = one wave per SIMD with a 128x128 tile each (gemm4w_kernel), 8 = the ping-pong kernel, "
        "0 = default");
  m.def("gemm_get_waves", &gemm_get_waves);
  m.def("gemm_set_width", &gemm_set_width, "256-row GEMM block width: 0 auto (grid-quantisation rule), 128, 256");
  m.def("linear_fwd", &py_linear_fwd, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("act"), py::arg("p"),
        py::arg("save_preact"), py::arg("res") = py::none(), py::arg("xt") = py::none(),
        py::arg("aux_grad") = false, py::arg("bits") = py::none());
  m.def("linear_bits_ok",
        [](int64_t M, int64_t N, int64_t K, int64_t act, double p) {
          GemmArgs g;
          g.M = (int)M; g.N = (int)N; g.K = (int)K; g.act = (int)act; g.p = (float)p;
          g.a_kc = true; g.b_kc = true; g.epi = kEpiStoreAct;
          return gemm_supported(M, N, K) && gemm_bits_ok(g);
        },
        py::arg("M"), py::arg("N"), py::arg("K"), py::arg("act"), py::arg("p"),
        "whether linear_fwd can also write the ReLU output's nonzero mask as bits (kActReluBits)");
  m.def("gemm_emit_ok", &gemm_emit_ok, py::arg("act"), py::arg("p"), py::arg("aux"),
        "whether linear_fwd can also write x^T for this activation / dropout / pre-activation output");
  m.def("linear_wgrad_xt_segments", &py_linear_wgrad_xt_segments, py::arg("dys"), py::arg("xts"),
        py::arg("main_grad"), py::arg("accumulate") = true, py::arg("bias_grad") = py::none());
  m.def("linear_dgrad", &py_linear_dgrad, py::arg("dy"), py::arg("w"), py::arg("res") = py::none(),
        py::arg("out") = py::none(), py::arg("act") = 0, py::arg("saved") = py::none(), py::arg("p") = 0.0,
        py::arg("seed") = 0, py::arg("offset") = 0);
  m.def("linear_wgrad", &py_linear_wgrad, py::arg("dy"), py::arg("x"), py::arg("main_grad"),
        py::arg("accumulate") = true);
  m.def("linear_wgrad_segments", &py_linear_wgrad_segments, py::arg("dys"), py::arg("xs"), py::arg("main_grad"),
        py::arg("accumulate") = true, py::arg("bias_grad") = py::none());
  m.def("column_sum_segments", &py_column_sum_segments);
  m.def("transpose_b16", &py_transpose_b16);
  m.def("gemm_f32", &py_gemm_f32);
  m.def("sumsq", &py_sumsq);
  m.def("adam_step", &py_adam);
}
