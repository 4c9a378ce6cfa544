"""fp32 on the HIP kernels -- the reference's own precision (main.py trains in fp32).

The fp32 GEMM (v_mfma_f32_32x32x2_f32, gemm_f32.hip) and fp32 flash attention
(attention_f32.hip) against float64 / fp32 PyTorch references; the fp32
TransformerEncoderLayer must run on them (no eager-math warning)."""
import math
import warnings

import pytest
import torch
import torch.nn.functional as F

from test_gpu_kernels import _philox4x32_10

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module")
def k():
    from mipipe._native_loader import kernels

    return kernels()


def _rel(a, b):
    return ((a.double() - b.double()).abs().max() / (b.double().abs().max() + 1e-30)).item()


@pytest.mark.parametrize("a_kc,b_kc", [(True, True), (True, False), (False, False), (False, True)])
@pytest.mark.parametrize("M,N,K", [(64, 64, 32), (128, 256, 96), (1024, 2048, 2048), (2048, 6144, 1024),
                                   (100, 36, 64), (1000, 1004, 160), (1024, 28784, 128)])
def test_gemm_f32_layouts(k, a_kc, b_kc, M, N, K):
    torch.manual_seed(1)
    a = torch.randn(M, K, device=DEV)
    b = torch.randn(K, N, device=DEV)
    a_store = a if a_kc else a.t().contiguous()
    b_store = b.t().contiguous() if b_kc else b
    c = k.gemm_f32(a_store, b_store, a_kc, b_kc)
    ref = a.double() @ b.double()
    # exact fp32 products, fp32 accumulation: ~1e-7 * sqrt(K) relative
    assert _rel(c, ref) < 2e-6 * math.sqrt(K / 64), _rel(c, ref)


def test_gemm_f32_supported(k):
    assert k.gemm_f32_supported(1024, 2048, 2048)
    assert k.gemm_f32_supported(100, 36, 64)
    assert not k.gemm_f32_supported(100, 35, 64)   # N % 4
    assert not k.gemm_f32_supported(128, 128, 48)  # K % 32


@pytest.mark.parametrize("act", [None, "relu", "gelu"])
@pytest.mark.parametrize("T,K,N", [(256, 512, 384), (520, 264, 136)])
def test_linear_f32_matches_torch(k, act, T, K, N):
    from mipipe.ops import linear

    torch.manual_seed(2)
    x = torch.randn(T, K, device=DEV, requires_grad=True)
    w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).requires_grad_()
    b = torch.randn(N, device=DEV, requires_grad=True)
    y = linear(x, w, b, act, 0.0, True)
    xr, wr, br = (t.detach().double().requires_grad_() for t in (x, w, b))
    ref = F.linear(xr, wr, br)
    ref = torch.relu(ref) if act == "relu" else (F.gelu(ref) if act == "gelu" else ref)
    assert _rel(y, ref) < 1e-5
    g = torch.randn_like(y)
    y.backward(g)
    ref.backward(g.double())
    assert _rel(x.grad, xr.grad) < 1e-5
    assert _rel(w.grad, wr.grad) < 1e-5
    assert _rel(b.grad, br.grad) < 1e-5


def test_linear_f32_main_grad_segments_and_dropout(k):
    """fp32 weight gradients into main_grad (direct and deferred / K-segmented) and
    the epilogue dropout mask reproduced by the elementwise backward."""
    from mipipe import ops

    torch.manual_seed(3)
    T, K, N, p = 256, 256, 384, 0.3
    w = (torch.randn(N, K, device=DEV) / 16).requires_grad_()
    w.main_grad = torch.zeros(N, K, device=DEV)
    xs = [torch.randn(T, K, device=DEV) for _ in range(3)]
    gs = [torch.randn(T, N, device=DEV) for _ in range(3)]
    keeps = []
    with ops.deferred_wgrad():
        for x, g in zip(xs, gs):
            y = ops.linear(x, w, None, None, p, True)
            keeps.append((y != 0).double())
            y.backward(g)
        assert w.main_grad.abs().max().item() == 0.0  # deferred: nothing ran yet
    expect = sum((g.double() * kp / (1 - p)).t() @ x.double() for x, g, kp in zip(xs, gs, keeps))
    assert abs(torch.stack(keeps).mean().item() - (1 - p)) < 0.02
    assert _rel(w.main_grad, expect) < 1e-5
    # the kept values are exactly x W^T / (1 - p)
    y = ops.linear(xs[0], w.detach(), None, None, p, True)
    pre = (xs[0].double() @ w.detach().double().t()) / (1 - p)
    kept = y != 0
    assert _rel(y[kept], pre[kept]) < 1e-5


def test_linear_residual_f32(k):
    from mipipe.ops import linear, linear_residual

    torch.manual_seed(6)
    T, K, N = 256, 512, 384
    x = torch.randn(T, K, device=DEV, requires_grad=True)
    w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).requires_grad_()
    b = torch.randn(N, device=DEV, requires_grad=True)
    r = torch.randn(T, N, device=DEV, requires_grad=True)
    y = linear_residual(x, w, b, r, 0.0, True)
    xr, wr, br, rr = (t.detach().double().requires_grad_() for t in (x, w, b, r))
    ref = rr + F.linear(xr, wr, br)
    assert _rel(y, ref) < 1e-5
    g = torch.randn_like(y)
    y.backward(g)
    ref.backward(g.double())
    for a_, b_ in ((x.grad, xr.grad), (w.grad, wr.grad), (b.grad, br.grad), (r.grad, rr.grad)):
        assert _rel(a_, b_) < 1e-5
    with torch.no_grad():
        torch.manual_seed(9)
        y1 = linear_residual(x, w, b, r, 0.2, True)
        torch.manual_seed(9)
        y2 = r + linear(x, w, b, None, 0.2, True)
    assert _rel(y1, y2) < 1e-6


def _keyquad_keep(B, H, S, p, seed, offset):
    """fp32 attention dropout mask: uniform of (q, k) = word (k & 3) of Philox
    counter (bh * S/4 + k/4) * S + q."""
    import numpy as np

    bh, q, key = np.meshgrid(np.arange(B * H), np.arange(S), np.arange(S), indexing="ij")
    sub = (bh.astype(np.uint64) * np.uint64(S // 4) + (key // 4).astype(np.uint64)) * np.uint64(S) + q.astype(np.uint64)
    seed &= 0xFFFFFFFFFFFFFFFF
    offset &= 0xFFFFFFFFFFFFFFFF
    m32 = np.uint64(0xFFFFFFFF)
    words = _philox4x32_10(sub & m32, sub >> np.uint64(32), np.uint64(offset) & m32, np.uint64(offset) >> np.uint64(32),
                           seed & 0xFFFFFFFF, seed >> 32)
    w = np.choose((key & 3), words)
    thr = min(int(p * 4294967296.0), 0xFFFFFFFF)
    return torch.from_numpy((w >= thr).reshape(B, H, S, S))


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("p", [0.0, 0.25])
@pytest.mark.parametrize("S,D", [(32, 64), (128, 64), (160, 64), (256, 64), (128, 128), (160, 128), (64, 96)])
def test_attention_f32(k, causal, p, S, D):
    """fp32 kernels: D = 64 (dK/dV in one kernel), D = 128 (dV and dK kernels),
    D = 96 (zero-padded to 128)."""
    from mipipe.ops import attention_packed

    if p > 0 and D not in (64, 128):
        pytest.skip("the mask replay below calls the kernel at the real head dim")
    torch.manual_seed(4)
    B, H = 2, 3
    scale = 1.0 / math.sqrt(D)
    qkv = torch.randn(B, S, 3, H, D, device=DEV, requires_grad=True)
    torch.manual_seed(11)
    o = attention_packed(qkv, causal, p, True)
    keep = None
    if p > 0:
        torch.manual_seed(11)  # the op's draw, replayed to read its (seed, offset)
        _, _, seed, offset, _ = k.attention_fwd(*(qkv.detach().select(2, i) for i in range(3)), causal, p, scale)
        keep = _keyquad_keep(B, H, S, p, seed, offset).to(DEV)
        assert abs(keep.double().mean().item() - (1 - p)) < 0.03
    qf = qkv.detach().double().requires_grad_()
    qh, kh, vh = (qf.select(2, i).transpose(1, 2) for i in range(3))
    s = (qh @ kh.transpose(-1, -2)) * scale
    if causal:
        s = s.masked_fill(torch.ones(S, S, dtype=torch.bool, device=DEV).triu(1), float("-inf"))
    pr = torch.softmax(s, -1)
    if keep is not None:
        pr = pr * keep.double() / (1 - p)
    ref = (pr @ vh).transpose(1, 2)
    assert _rel(o, ref) < 1e-5, _rel(o, ref)
    g = torch.randn_like(o)
    o.backward(g)
    ref.backward(g.double())
    assert _rel(qkv.grad, qf.grad) < 1e-4, _rel(qkv.grad, qf.grad)


def test_attention_f32_recompute_replays_mask(k):
    """Same (seed, offset) -> identical output and gradients (checkpoint recompute)."""
    torch.manual_seed(5)
    B, S, H, D = 2, 128, 4, 64
    q, kk, v = (torch.randn(B, S, H, D, device=DEV) for _ in range(3))
    torch.manual_seed(7)
    o1, lse1, s1, off1, _ = k.attention_fwd(q, kk, v, False, 0.2, 0.125)
    torch.manual_seed(7)
    o2, lse2, s2, off2, _ = k.attention_fwd(q, kk, v, False, 0.2, 0.125)
    assert (s1, off1) == (s2, off2) and torch.equal(o1, o2) and torch.equal(lse1, lse2)


@pytest.mark.parametrize("S", [128, 37, 40, 100])
def test_transformer_layer_fp32_on_kernels(k, S):
    """fp32 post-norm TransformerEncoderLayer (the reference's layer and precision) on the
    fp32 GEMM / attention / LN kernels vs nn.TransformerEncoderLayer: no eager fallback,
    also on the short tail windows of the reference's get_batch (S = 37 / 40 / 100: padded
    keys masked by the kernels' key bound; /root/reference/main.py:108-113)."""
    from torch import nn

    from mipipe.models import TransformerEncoderLayer

    torch.manual_seed(0)
    E, H, F_, B = 256, 4, 512, 8
    ref = nn.TransformerEncoderLayer(E, H, F_, dropout=0.0, batch_first=True).to(DEV)
    ours = TransformerEncoderLayer(E, H, F_, dropout=0.0, device=DEV).load_from_torch(ref)
    x = torch.randn(B, S, E, device=DEV, requires_grad=True)
    xr = x.detach().clone().requires_grad_()
    with warnings.catch_warnings():
        warnings.simplefilter("error")  # an eager-math fallback warns: make it fail
        y = ours(x)
    yr = ref(xr)
    assert _rel(y, yr) < 1e-4, _rel(y, yr)
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g)
    assert _rel(x.grad, xr.grad) < 1e-3, _rel(x.grad, xr.grad)
