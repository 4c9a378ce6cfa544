"""HIP kernels vs plain PyTorch fp32 references (one MI355X).

Every kernel here must come from mipipe/_C.so: the tests fail if the extension
is missing (no silent eager fallback)."""
import math

import pytest
import torch
import torch.nn.functional as F

from mipipe import ops
from mipipe.ops.linear import ActFold

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module")
def k():
    from mipipe._native_loader import kernels

    return kernels()


def _tol(dtype):
    return (2e-2, 2e-2) if dtype == torch.bfloat16 else (1e-4, 1e-4)


# ------------------------------------------------------------------ LayerNorm
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cols", [256, 1024, 4096, 1600])
@pytest.mark.parametrize("residual", [False, True])
@pytest.mark.parametrize("rows", [333, 1537])
def test_layernorm_fwd_bwd(k, dtype, cols, residual, rows):
    from mipipe.ops import add_dropout_layer_norm

    x = torch.randn(rows, cols, device=DEV, dtype=dtype, requires_grad=True)
    r = torch.randn(rows, cols, device=DEV, dtype=dtype, requires_grad=True) if residual else None
    w = (1 + 0.1 * torch.randn(cols, device=DEV)).to(dtype).requires_grad_()
    b = (0.1 * torch.randn(cols, device=DEV)).to(dtype).requires_grad_()
    y = add_dropout_layer_norm(x, r, w, b, 1e-5, 0.0, True)
    xf = x.detach().float().requires_grad_()
    rf = r.detach().float().requires_grad_() if residual else None
    wf = w.detach().float().requires_grad_()
    bf = b.detach().float().requires_grad_()
    ref = F.layer_norm(xf + (rf if residual else 0), (cols,), wf, bf, 1e-5)
    atol, rtol = _tol(dtype)
    assert torch.allclose(y.float(), ref, atol=atol, rtol=rtol)
    gy = torch.randn_like(ref)
    y.backward(gy.to(dtype))
    ref.backward(gy)
    assert torch.allclose(x.grad.float(), xf.grad, atol=atol * 5, rtol=rtol * 5)
    if residual:
        assert torch.allclose(r.grad.float(), rf.grad, atol=atol * 5, rtol=rtol * 5)
    assert torch.allclose(w.grad.float(), wf.grad, atol=atol * 20 * math.sqrt(rows / 100), rtol=rtol * 5)
    assert torch.allclose(b.grad.float(), bf.grad, atol=atol * 20 * math.sqrt(rows / 100), rtol=rtol * 5)


def test_layernorm_dropout_mask_consistent(k):
    from mipipe.ops import add_dropout_layer_norm

    rows, cols, p = 64, 512, 0.3
    x = torch.randn(rows, cols, device=DEV, requires_grad=True)
    r = torch.zeros(rows, cols, device=DEV)
    w = torch.ones(cols, device=DEV, requires_grad=True)
    b = torch.zeros(cols, device=DEV, requires_grad=True)
    torch.manual_seed(5)
    y = add_dropout_layer_norm(x, r, w, b, 1e-5, p, True)
    # kept fraction ~ 1-p, reproducible under the same seed
    torch.manual_seed(5)
    y2 = add_dropout_layer_norm(x, r, w, b, 1e-5, p, True)
    assert torch.equal(y, y2)
    y.backward(torch.randn_like(y))
    g = x.grad
    # gradient is exactly zero where the element was dropped
    dropped = (g == 0).float().mean().item()
    assert abs(dropped - p) < 0.03


# ------------------------------------------------------------------ bias + act + dropout
@pytest.mark.parametrize("act", [None, "relu", "gelu"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_bias_act(k, act, dtype):
    from mipipe.ops import bias_act_dropout
    from mipipe.ops.activation import bias_act_reference

    x = torch.randn(96, 520, device=DEV, dtype=dtype, requires_grad=True)
    b = torch.randn(520, device=DEV, dtype=dtype, requires_grad=True)
    y = bias_act_dropout(x, b, act, 0.0, True)
    xf = x.detach().float().requires_grad_()
    bf = b.detach().float().requires_grad_()
    ref = bias_act_reference(xf, bf, act, 0.0, True)
    atol, rtol = _tol(dtype)
    assert torch.allclose(y.float(), ref, atol=atol, rtol=rtol)
    g = torch.randn_like(ref)
    y.backward(g.to(dtype))
    ref.backward(g)
    assert torch.allclose(x.grad.float(), xf.grad, atol=atol * 2, rtol=rtol * 2)
    assert torch.allclose(b.grad.float(), bf.grad, atol=atol * 40, rtol=rtol * 5)


def test_bias_act_dropout_stats(k):
    from mipipe.ops import bias_act_dropout

    x = torch.ones(1024, 1024, device=DEV)
    y = bias_act_dropout(x, None, "relu", 0.25, True)
    kept = (y != 0).float().mean().item()
    assert abs(kept - 0.75) < 0.01
    assert torch.allclose(y[y != 0], torch.full_like(y[y != 0], 1 / 0.75))


@pytest.mark.parametrize("cols,rows", [(264, 1000), (28782, 1000), (4096, 4100), (1600, 37), (12288, 8192)])
def test_column_sum(k, cols, rows):
    x = torch.randn(rows, cols, device=DEV)
    assert torch.allclose(k.column_sum(x), x.sum(0), atol=2e-3, rtol=1e-4)
    out = torch.ones(cols, device=DEV)
    k.column_sum(x, out, True)
    assert torch.allclose(out, x.sum(0) + 1, atol=2e-3, rtol=1e-4)


# ------------------------------------------------------------------ cross entropy
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("V", [1000, 28782])
@pytest.mark.parametrize("padded", [False, True])
def test_cross_entropy(k, dtype, V, padded):
    from mipipe.ops import cross_entropy

    N = 200
    vp = (V + 255) // 256 * 256 if padded else V
    base = (3 * torch.randn(N, vp, device=DEV)).to(dtype)
    logits = base[:, :V].detach().requires_grad_() if not padded else None
    if padded:  # a [N, :V] view of a padded-vocabulary buffer (the Decoder's output)
        base.requires_grad_()
        logits = base[:, :V]
    t = torch.randint(0, V, (N,), device=DEV)
    t[3] = -100
    t[5] = V - 1  # a target in the scalar tail
    loss = cross_entropy(logits, t)
    lf = logits.detach().float().requires_grad_()
    ref = F.cross_entropy(lf, t, ignore_index=-100)
    assert abs(loss.item() - ref.item()) < 1e-3 * max(1, abs(ref.item()))
    loss.backward()
    ref.backward()
    atol = 1e-5 if dtype == torch.float32 else 2e-4
    g = base.grad[:, :V] if padded else logits.grad
    assert torch.allclose(g.float(), lf.grad, atol=atol, rtol=2e-2)
    if padded:
        assert base.grad[:, V:].abs().max().item() == 0.0


def test_cross_entropy_out_of_range_target_is_loud(k):
    """nn.CrossEntropyLoss raises on a target outside [0, V); the kernel mean
    poisons the loss (NaN) instead of silently leaving the row out of the mean."""
    from mipipe.ops import cross_entropy

    logits = torch.randn(64, 1000, device=DEV)
    t = torch.randint(0, 1000, (64,), device=DEV)
    t[0] = -100  # ignored: fine
    assert torch.isfinite(cross_entropy(logits, t)).item()
    t[7] = 1000
    assert torch.isnan(cross_entropy(logits, t)).item()


# ------------------------------------------------------------------ embedding
def test_embedding(k):
    from mipipe.models.lm import sinusoidal_positions
    from mipipe.ops import embed_scale_posenc_dropout

    V, E, B, S = 500, 256, 4, 32
    w = torch.randn(V, E, device=DEV, requires_grad=True)
    pe = sinusoidal_positions(64, E).to(DEV)
    tok = torch.randint(0, V, (B, S), device=DEV)
    tok[0, :4] = 7  # repeated ids exercise the atomic accumulation
    y = embed_scale_posenc_dropout(tok, w, pe, math.sqrt(E), 0.0, True)
    wf = w.detach().clone().requires_grad_()
    ref = F.embedding(tok, wf) * math.sqrt(E) + pe[:S]
    assert torch.allclose(y, ref, atol=1e-4)
    g = torch.randn_like(ref)
    y.backward(g)
    ref.backward(g)
    assert torch.allclose(w.grad, wf.grad, atol=1e-3)


# ------------------------------------------------------------------ optimizer
@pytest.mark.parametrize("variant", [0, 1, 2])
def test_flat_adam_matches_torch(k, variant):
    """Every Adam kernel (grid-stride, one-shot tiles, tiles with streaming
    stores -- the default; the flat group spans several tiles and ends in a
    scalar tail) against torch.optim.Adam."""
    from mipipe.optim import FlatAdam

    k.adam_set_variant(variant)
    torch.manual_seed(0)
    ps = [torch.randn(s, device=DEV, requires_grad=True) for s in [(17, 5), (33,), (4, 4, 4), (1031, 7)]]
    qs = [p.detach().clone().requires_grad_() for p in ps]
    opt = FlatAdam(ps, lr=1e-2, weight_decay=0.01, max_grad_norm=0.5)
    ref = torch.optim.Adam(qs, lr=1e-2, weight_decay=0.01)
    for _ in range(3):
        grads = [torch.randn_like(q) for q in qs]
        opt.zero_grad()
        for p, g in zip(ps, grads):
            p.grad = g.clone()
        opt.step()
        ref.zero_grad()
        for q, g in zip(qs, grads):
            q.grad = g.clone()
        torch.nn.utils.clip_grad_norm_(qs, 0.5)
        ref.step()
    k.adam_set_variant(2)
    for p, q in zip(ps, qs):
        assert torch.allclose(p, q, atol=1e-5)


def test_sumsq(k):
    g = torch.randn(1_000_003, device=DEV)
    assert torch.allclose(k.sumsq(g), g.double().pow(2).sum().float().reshape(1), rtol=1e-4)


# ------------------------------------------------------------------ runtime
def test_native_streams_and_wait(k):
    from mipipe.stream import new_stream, wait_stream

    d = torch.device(DEV, 0)
    s1, s2 = new_stream(d), new_stream(d)
    assert s1.cuda_stream != s2.cuda_stream
    x = torch.zeros(1 << 20, device=DEV)
    with torch.cuda.stream(s1):
        k.gpu_sleep(20000)
        x.fill_(1.0)
    wait_stream(s2, s1)
    with torch.cuda.stream(s2):
        y = x * 2
    s2.synchronize()
    assert torch.all(y == 2)


def test_streams_overlap(k):
    """Two 50 ms sleeps on independent native streams take ~50 ms, not 100."""
    import time

    from mipipe.stream import new_stream

    d = torch.device(DEV, 0)
    s1, s2 = new_stream(d), new_stream(d)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(s1):
        k.gpu_sleep(50000)
    with torch.cuda.stream(s2):
        k.gpu_sleep(50000)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    assert dt < 0.085, dt


def test_roctx_ranges(k):
    k.range_push("mipipe-test")
    k.mark("mark")
    k.range_pop()


def test_pipe_on_one_gpu_two_partitions(k):
    """Single-process Pipe with two partitions on the same GPU (balance=[1, 1]:
    copy streams, native D2D boundary copies, Wait events, a dedicated stream
    for the second stage, recompute) matches nn.Sequential."""
    import copy

    from torch import nn

    from mipipe import Pipe

    torch.manual_seed(0)
    a = nn.Linear(64, 64).to(DEV)
    b = nn.Linear(64, 64).to(DEV)
    seq = nn.Sequential(a, nn.Sequential(b))
    ref = copy.deepcopy(seq)
    x = torch.randn(32, 64, device=DEV)
    for mode in ("never", "always"):
        seq.zero_grad()
        ref.zero_grad()
        pipe = Pipe(seq, chunks=4, checkpoint=mode, balance=[1, 1], copy_same_device=True)
        assert len(pipe.partitions) == 2
        out = pipe(x).local_value()
        assert torch.allclose(out, ref(x), atol=1e-5)
        out.sum().backward()
        ref(x).sum().backward()
        for p, q in zip(seq.parameters(), ref.parameters()):
            assert torch.allclose(p.grad, q.grad, atol=1e-4)


@pytest.mark.multigpu
def test_peer_copy_two_gpus(k):
    from mipipe.copy import transfer
    from mipipe.stream import new_stream, use_stream

    s0 = new_stream(torch.device("cuda", 0))
    s1 = new_stream(torch.device("cuda", 1))
    x = torch.randn(1 << 20, device="cuda:0")
    with use_stream(s0), use_stream(s1):
        y = transfer(x, s0, s1)
    s1.synchronize()
    assert y.device == torch.device("cuda", 1)
    assert torch.equal(y.cpu(), x.cpu())


# ------------------------------------------------------------------ model / engine
@pytest.mark.parametrize("S", [37, 40, 100])
def test_fp32_tail_window_runs_on_kernels(k, S):
    """The reference's own fp32 model on its short tail window (get_batch yields
    S < 128 at the end of an epoch, /root/reference/main.py:108-113): fp32,
    head dim 64, NON-causal, S not a multiple of 32.  The sequence is padded to
    the next multiple of 32 and the fp32 kernels mask the padded keys with a
    key-length bound -- NO eager fallback -- and a TransformerEncoderLayer
    matches nn.TransformerEncoderLayer forward and backward (fp32 PyTorch)."""
    import warnings

    from torch import nn

    from mipipe.models import TransformerEncoderLayer
    from mipipe.ops import attention

    torch.manual_seed(0)
    E, H, F_, B = 256, 4, 512, 3  # head dim 64
    ref = nn.TransformerEncoderLayer(E, H, F_, dropout=0.0, batch_first=True).to(DEV)
    ours = TransformerEncoderLayer(E, H, F_, dropout=0.0, device=DEV).load_from_torch(ref)
    x = torch.randn(B, S, E, device=DEV, requires_grad=True)
    xr = x.detach().clone().requires_grad_()
    with warnings.catch_warnings():
        warnings.simplefilter("error")  # the eager-path note would raise here
        y = ours(x)
        g = torch.randn_like(y)
        y.backward(g)
    yr = ref(xr)
    yr.backward(g)
    assert torch.allclose(y, yr, atol=2e-4), (y - yr).abs().max()
    assert torch.allclose(x.grad, xr.grad, atol=2e-3), (x.grad - xr.grad).abs().max()
    # the op itself against fp32 math, q/k/v gradients included
    q, kk, v = (torch.randn(2, H, S, 64, device=DEV, requires_grad=True) for _ in range(3))
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        o = attention(q, kk, v, causal=False)
    qr, kr, vr = (t.detach().clone().requires_grad_() for t in (q, kk, v))
    orf = torch.softmax(qr @ kr.transpose(-1, -2) / 8.0, -1) @ vr
    assert torch.allclose(o, orf, atol=1e-4), (o - orf).abs().max()
    go = torch.randn_like(o)
    o.backward(go)
    orf.backward(go)
    for a_, b_ in ((q, qr), (kk, kr), (v, vr)):
        assert torch.allclose(a_.grad, b_.grad, atol=1e-4), (a_.grad - b_.grad).abs().max()


def test_attention_custom_scale_padding(k):
    """A tiny user scale must not let the bf16 spare-feature key mask leak weight
    onto padded keys: such shapes take a path that stays exact."""
    from mipipe.ops import attention

    torch.manual_seed(0)
    S, D = 40, 48
    q, kk, v = (torch.randn(2, 2, S, D, device=DEV, dtype=torch.bfloat16) for _ in range(3))
    for scale in (1e-3, 0.125):
        o = attention(q, kk, v, causal=False, scale=scale).float()
        orf = torch.softmax(q.float() @ kk.float().transpose(-1, -2) * scale, -1) @ v.float()
        assert torch.allclose(o, orf, atol=3e-2), (scale, (o - orf).abs().max())


def test_engine_one_gpu_step(k):
    from mipipe import ops
    from mipipe.models import CONFIGS, build_lm_blocks
    from mipipe.optim import FlatAdam
    from mipipe.parallel import PipelineEngine

    cfg = CONFIGS["tiny"]
    dev = torch.device(DEV, 0)
    stage = torch.nn.Sequential(*build_lm_blocks(cfg, device=dev, dtype=torch.bfloat16)).train()
    opt = FlatAdam(stage.parameters(), lr=1e-3, max_grad_norm=0.5)
    m, mb, S = 4, 2, cfg.seq_len
    eng = PipelineEngine(stage, chunks=m, checkpoint="except_last", act_shape=(mb, S, cfg.d_model),
                         act_dtype=torch.bfloat16,
                         loss_fn=lambda y, t: ops.cross_entropy(y.reshape(-1, cfg.vocab), t.reshape(-1)),
                         device=dev, measure=True)
    tok = torch.randint(0, cfg.vocab, (m, mb, S + 1), device=dev)
    losses = []
    for _ in range(5):
        opt.zero_grad()
        st = eng.step([tok[i, :, :S] for i in range(m)], [tok[i, :, 1:].contiguous() for i in range(m)])
        opt.step()
        losses.append(float(st.loss))
    assert all(l == l for l in losses)
    assert losses[-1] < losses[0]  # it learns the fixed batch
    assert st.busy_ms > 0


# ------------------------------------------------------------------ GEMM
@pytest.mark.parametrize("a_kc,b_kc", [(True, True), (True, False), (False, False), (False, True)])
@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (256, 384, 192), (512, 256, 1024), (2048, 4096, 256), (4096, 2048, 128),
                                   # edge tiles (GPT-2-XL widths 1600 / 4800, odd multiples of 8)
                                   (200, 136, 64), (1000, 1000, 128), (4096, 4800, 1600), (4800, 1600, 1024)])
def test_gemm_layouts(k, a_kc, b_kc, M, N, K):
    torch.manual_seed(1)
    a = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    b = torch.randn(K, N, device=DEV).to(torch.bfloat16)
    # asymmetric, non-trivial operands (A = I style checks hide transposes)
    a_store = a if a_kc else a.t().contiguous()
    b_store = b.t().contiguous() if b_kc else b
    c = k.gemm_f32(a_store, b_store, a_kc, b_kc)
    ref = a.float() @ b.float()
    err = (c - ref).abs().max().item()
    assert err < 1e-2 * math.sqrt(K / 64), err


@pytest.mark.parametrize("width", [256, 128])
@pytest.mark.parametrize("sched", [0, 1, 2, 3, 4, 5, 6, 7])
def test_gemm_main_loop_schedules(k, sched, width):
    """Every 256x256 main loop built in (the product build: the default whole-tile
    ping-pong; a --gemm-ab build also the per-tile barrier, ping-pong, the mixes,
    ping-pong with the B lead) on every layout, for 1, 2, 3 and many K-tiles, edge
    tiles, K-segments and the bf16 epilogue."""
    from mipipe.ops import linear

    if sched != 7 and not k.gemm_ab_build():
        assert not k.gemm_set_schedule(sched)  # refused, not silently ignored
        pytest.skip("A/B GEMM schedule not in the product build (python -m mipipe.build --gemm-ab)")
    old = k.gemm_get_schedule()
    assert k.gemm_set_schedule(sched)
    k.gemm_set_width(width)
    try:
        torch.manual_seed(7)
        for M, N, K in [(520, 264, 64), (1000, 1000, 128), (4096, 4800, 192), (2048, 4096, 1024), (256, 256, 320)]:
            a = torch.randn(M, K, device=DEV).to(torch.bfloat16)
            b = torch.randn(K, N, device=DEV).to(torch.bfloat16)
            ref = a.float() @ b.float()
            for a_kc, b_kc in [(True, True), (True, False), (False, False), (False, True)]:
                c = k.gemm_f32(a if a_kc else a.t().contiguous(), b.t().contiguous() if b_kc else b, a_kc, b_kc)
                err = (c - ref).abs().max().item()
                assert err < 1e-2 * math.sqrt(K / 64), (M, N, K, a_kc, b_kc, err)
        dys = [torch.randn(128, 264, device=DEV).to(torch.bfloat16) for _ in range(5)]
        xs = [torch.randn(128, 136, device=DEV).to(torch.bfloat16) for _ in range(5)]
        main = torch.zeros(264, 136, device=DEV)
        k.linear_wgrad_segments(dys, xs, main)
        expect = sum(d.float().t() @ x.float() for d, x in zip(dys, xs))
        assert ((main - expect).abs().max() / expect.abs().max()).item() < 1e-3
        x = torch.randn(1000, 512, device=DEV).to(torch.bfloat16)
        w = (torch.randn(1000, 512, device=DEV) / math.sqrt(512)).to(torch.bfloat16)
        bias = torch.randn(1000, device=DEV).to(torch.bfloat16)
        y = linear(x, w, bias, "gelu", 0.0, True)
        ref = F.gelu(x.float() @ w.float().t() + bias.float())
        assert torch.allclose(y.float(), ref, atol=3e-2, rtol=3e-2)
        # the residual addend (16-byte row chunks in the staged epilogue)
        r = torch.randn(1000, 1000, device=DEV).to(torch.bfloat16)
        y = k.linear_fwd(x, w, bias, 0, 0.0, False, r)[0]
        ref = x.float() @ w.float().t() + bias.float() + r.float()
        assert torch.allclose(y.float(), ref, atol=3e-2, rtol=3e-2)
    finally:
        k.gemm_set_schedule(old)
        k.gemm_set_width(0)


@pytest.mark.parametrize("sched", [0, 4, 5, 6, 7])
def test_wgrad_segments_fused_bias(k, sched):
    """The bias gradient folded into the K-segmented weight-gradient GEMM
    (GemmArgs::rowsum): equal to the column sums of every dY, accumulated; a
    shape that cannot take the fold (< 16 tile columns, or split-K) returns
    False and leaves the bias gradient alone."""
    if sched != 7 and not k.gemm_ab_build():
        pytest.skip("A/B GEMM schedule not in the product build (python -m mipipe.build --gemm-ab)")
    old = k.gemm_get_schedule()
    assert k.gemm_set_schedule(sched)
    try:
        torch.manual_seed(11)
        for N, Kin, T, nseg in [(520, 4096, 256, 3), (1000, 4104, 128, 18), (256, 512, 128, 2), (1024, 4096, 1024, 16)]:
            dys = [torch.randn(T, N, device=DEV).to(torch.bfloat16) for _ in range(nseg)]
            xs = [torch.randn(T, Kin, device=DEV).to(torch.bfloat16) for _ in range(nseg)]
            main = torch.zeros(N, Kin, device=DEV)
            bias = torch.full((N,), 0.5, device=DEV)
            fused = k.linear_wgrad_segments(dys, xs, main, True, bias)
            expect = sum(d.float().t() @ x.float() for d, x in zip(dys, xs))
            assert ((main - expect).abs().max() / expect.abs().max()).item() < 1e-3, (N, Kin, sched)
            if Kin < 4096:
                assert not fused
            if fused:
                ref = 0.5 + sum(d.float().sum(0) for d in dys)
                assert torch.allclose(bias, ref, atol=1e-2, rtol=1e-4), (N, Kin, sched, (bias - ref).abs().max())
            else:
                assert torch.all(bias == 0.5)
    finally:
        k.gemm_set_schedule(old)



@pytest.mark.parametrize("M,K,N", [(2048, 4096, 9216), (1000, 4096, 8192), (2048, 1600, 28928), (776, 1024, 16384)])
def test_linear_dgrad_split_k(k, M, K, N):
    """Under-filled grid with a long K (the T=2048 LM-head dgrad): K split over 2-4 blocks per
    tile, fp32 partials, one reduction (+ the fan-out residual) -- against fp32."""
    torch.manual_seed(8)
    dy = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) / math.sqrt(N)).to(torch.bfloat16)
    r = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    ref = dy.float() @ w.float()
    for res in (None, r):
        dx = k.linear_dgrad(dy, w, res)
        want = ref + (r.float() if res is not None else 0)
        err = ((dx.float() - want).abs().max() / want.abs().max()).item()
        assert err < 1e-2, (M, K, N, res is not None, err)


@pytest.mark.parametrize("N,K,T,nseg", [(1600, 1600, 4096, 4), (6400, 1600, 2048, 4), (520, 776, 8192, 1)])
def test_wgrad_split_k(k, N, K, T, nseg):
    """Weight gradients on under-filled grids (GPT-2-XL widths) split K over several blocks per
    tile: fp32 partials reduced into main_grad -- store (first write) and accumulate."""
    torch.manual_seed(9)
    dys = [torch.randn(T, N, device=DEV).to(torch.bfloat16) for _ in range(nseg)]
    xs = [torch.randn(T, K, device=DEV).to(torch.bfloat16) for _ in range(nseg)]
    expect = sum(d.float().t() @ x.float() for d, x in zip(dys, xs))
    for accumulate in (False, True):
        main = torch.randn(N, K, device=DEV)
        base = main.clone() if accumulate else torch.zeros_like(main)
        if nseg == 1:
            k.linear_wgrad(dys[0], xs[0], main, accumulate)
        else:
            k.linear_wgrad_segments(dys, xs, main, accumulate)
        err = ((main - base - expect).abs().max() / expect.abs().max()).item()
        assert err < 1e-3, (N, K, T, nseg, accumulate, err)


@pytest.mark.parametrize("M,N,K,bias,act", [
    (8192, 4096, 4096, True, 0),     # enc12 out-proj shape, one round
    (1000, 1000, 128, True, 1),      # edge rows (clamped), 256x128 blocks
    (2048, 9000, 512, True, 0),      # multi-round grid launched in chunks along N
    (4608, 1024, 256, False, 0),     # chunks along M (the emitted columns shift)
    (1024, 1024, 8192, False, 0),    # long K on a small grid: split-K blocks each emit their K-tiles
    (520, 264, 64, True, 1),         # one K-tile
    (2048, 512, 1024, True, 2),      # GELU without the pre-activation output (eval-style forward)
])
def test_linear_fwd_emits_x_transposed(k, M, N, K, bias, act):
    """The forward GEMM's A^T emission (GemmArgs::at): x^T bit-exact, and the
    forward output identical to the launch without it."""
    torch.manual_seed(21)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).to(torch.bfloat16)
    b = torch.randn(N, device=DEV).to(torch.bfloat16) if bias else None
    xt = torch.full((K, M), float("nan"), device=DEV).to(torch.bfloat16)
    p = 0.2 if act == 1 else 0.0  # ReLU + dropout: the enc12 FFN's extra-epilogue variant
    torch.manual_seed(5)
    y1, _, _, _ = k.linear_fwd(x, w, b, act, p, False, None, xt)
    torch.manual_seed(5)
    y0, _, _, _ = k.linear_fwd(x, w, b, act, p, False)
    assert torch.equal(xt, x.t())
    assert torch.equal(y1, y0)
    # the GELU epilogue with a pre-activation output cannot emit: refused loudly
    assert not k.gemm_emit_ok(2, 0.0, True) and not k.gemm_emit_ok(2, 0.1, False) and k.gemm_emit_ok(1, 0.2, False)
    with pytest.raises(RuntimeError, match="xt"):
        k.linear_fwd(x, w, b, 2, 0.0, True, None, xt)


@pytest.mark.parametrize("N,Kin,T,nseg,bias", [
    (12288, 4096, 256, 3, True),   # enc12 qkv widths: the bias fold, 16-column slices (>= 8 tile rows)
    (520, 4096, 128, 5, True),     # edge columns of C^T
    (1600, 1600, 1024, 4, True),   # GPT-2-XL: 7 tile rows -> 32-column slices
    (1600, 1600, 4096, 4, True),   # ... and with split-K
    (1600, 2048, 4096, 4, True),   # 8 tile rows, 56 tiles, K = 16384: the fold with split-K partials
    (6400, 1600, 512, 2, True),    # GPT-2-XL fc1
    (4800, 520, 256, 2, True),     # 3 tile rows (the last partial) -> 64-column slices
    (600, 256, 192, 3, True),      # 1 tile row -> 128-column slices, edge tile column
    (6400, 1600, 512, 2, False),
    (1000, 4104, 128, 18, True),   # > 16 segments: two launches, the second accumulates
])
def test_wgrad_xt_segments(k, N, Kin, T, nseg, bias):
    """The transposed weight gradient main_grad (+)= sum_i (x_i^T dy_i)^T and the
    B-side bias fold, against fp32, storing (first write) and accumulating."""
    torch.manual_seed(22)
    dys = [torch.randn(T, N, device=DEV).to(torch.bfloat16) for _ in range(nseg)]
    xs = [torch.randn(T, Kin, device=DEV).to(torch.bfloat16) for _ in range(nseg)]
    xts = [x.t().contiguous() for x in xs]
    expect = sum(d.float().t() @ x.float() for d, x in zip(dys, xs))
    for accumulate in (False, True):
        main = torch.randn(N, Kin, device=DEV)
        base = main.clone() if accumulate else torch.zeros_like(main)
        bg = torch.full((N,), 0.5, device=DEV) if bias else None
        fused = k.linear_wgrad_xt_segments(dys, xts, main, accumulate, bg)
        err = ((main - base - expect).abs().max() / expect.abs().max()).item()
        assert err < 1e-3, (N, Kin, T, nseg, accumulate, err)
        if bias:
            assert fused  # the slices widen until the tile rows cover the tile column
        if bias and fused:
            ref = 0.5 + sum(d.float().sum(0) for d in dys)
            assert torch.allclose(bg, ref, atol=1e-2, rtol=1e-4), (bg - ref).abs().max()
        elif bias:
            assert torch.all(bg == 0.5)


def test_linear_xt_path_matches_plain_wgrad(k):
    """A Linear trained through either x^T source -- emitted by the forward GEMM
    (MIPIPE_WGRAD_XT=emit) or transposed by the flush (auto; the width threshold
    lowered so this shape takes it) -- gets the same weight / bias gradients,
    deferred or not, as with the x^T path off (x kept, both operands read
    I-contiguous)."""
    import importlib

    L = importlib.import_module("mipipe.ops.linear")  # the module (mipipe.ops.linear is also a function)
    torch.manual_seed(23)
    T, K, N = 512, 4096, 1024
    x = torch.randn(T, K, device=DEV).to(torch.bfloat16)
    w = torch.nn.Parameter((torch.randn(N, K, device=DEV) / 64).to(torch.bfloat16))
    b = torch.nn.Parameter(torch.randn(N, device=DEV).to(torch.bfloat16))
    dy = torch.randn(T, N, device=DEV).to(torch.bfloat16)

    def grads(mode, deferred):
        old = L._EMIT_XT, L._XT_MODE, L._XT_MIN_N
        L._EMIT_XT, L._XT_MODE, L._XT_MIN_N = mode == "emit", mode, 0
        try:
            w.main_grad = torch.zeros(N, K, device=DEV)
            b.main_grad = torch.zeros(N, device=DEV)
            ctx = L.deferred_wgrad() if deferred else None
            if ctx:
                ctx.__enter__()
            for _ in range(2):  # two micro-batches
                L.linear(x, w, b, "relu").backward(dy)
            if ctx:
                ctx.__exit__(None, None, None)
            return w.main_grad.clone(), b.main_grad.clone()
        finally:
            L._EMIT_XT, L._XT_MODE, L._XT_MIN_N = old

    for deferred in (False, True):
        gw0, gb0 = grads("0", deferred)
        for mode in ("emit", "auto"):
            gw1, gb1 = grads(mode, deferred)
            assert ((gw1 - gw0).abs().max() / gw0.abs().max()).item() < 1e-5, (mode, deferred)
            assert torch.allclose(gb1, gb0, atol=1e-3, rtol=1e-5), (mode, deferred)


@pytest.mark.parametrize("R,C,ld", [(8192, 4096, 4096), (520, 264, 264), (64, 8, 8), (200, 1032, 1040), (8, 4104, 4104)])
def test_transpose_b16(k, R, C, ld):
    """transpose_b16 == torch's transpose, bit for bit, incl. partial 64-row/256-column tiles
    and a row stride wider than the row."""
    torch.manual_seed(R + C)
    base = torch.randn(R, ld, device=DEV).to(torch.bfloat16)
    x = base[:, :C]
    out = k.transpose_b16(x)
    assert out.shape == (C, R) and out.is_contiguous()
    assert torch.equal(out, x.t().contiguous())
    with pytest.raises(RuntimeError):
        k.transpose_b16(base[:, 1:C])  # misaligned


def test_gemm_round_launches_identical(k):
    """Multi-round grids launched one round of tiles at a time give the same bits as one
    launch -- forward with bias / ReLU / dropout (the mask keeps full-matrix coordinates),
    GELU with the pre-activation output, dgrad with the residual addend, segmented wgrad
    (split along M) -- and the unchunked result is right."""
    torch.manual_seed(12)
    T, K, N = 2048, 512, 9000  # 8 x 36 tiles: 2 launches along N, the second an edge chunk
    x = torch.randn(T, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).to(torch.bfloat16)
    b = torch.randn(N, device=DEV).to(torch.bfloat16)
    dy = torch.randn(4096, 1024, device=DEV).to(torch.bfloat16)  # dgrad 4096 x 4608: 16 x 18 tiles
    w2 = (torch.randn(1024, 4608, device=DEV) / 32).to(torch.bfloat16)
    r = torch.randn(4096, 4608, device=DEV).to(torch.bfloat16)
    dys = [torch.randn(256, 8200, device=DEV).to(torch.bfloat16) for _ in range(2)]  # wgrad 8200 x 2048: 33 x 8
    xs = [torch.randn(256, 2048, device=DEV).to(torch.bfloat16) for _ in range(2)]
    # 11 x 25 tiles: a 23-column chunk and a 2-column one that is an exact multiple of the
    # 128x128 kernel's tile (it stays on the 256-row kernel: GemmArgs::round_chunk)
    x3 = torch.randn(2816, 512, device=DEV).to(torch.bfloat16)
    w3 = (torch.randn(6400, 512, device=DEV) / math.sqrt(512)).to(torch.bfloat16)

    def run():
        torch.manual_seed(77)
        y1 = k.linear_fwd(x, w, b, 1, 0.3, False)[0]
        torch.manual_seed(78)
        y2, pre, _, _ = k.linear_fwd(x, w, b, 2, 0.0, True)
        dx = k.linear_dgrad(dy, w2, r)
        mg = torch.zeros(8200, 2048, device=DEV)
        k.linear_wgrad_segments(dys, xs, mg, False)
        y3 = k.linear_fwd(x3, w3, None, 0, 0.0, False)[0]
        return [y1, y2, pre, dx, mg, y3]

    try:
        k.gemm_set_rounds(0)
        ref = run()
        k.gemm_set_rounds(2)  # per-round launches at any K (the default 1 keeps K < 4096 in one launch)
        got = run()
    finally:
        k.gemm_set_rounds(1)
    for a, bb in zip(got, ref):
        assert torch.equal(a, bb)
    want = torch.relu(x.float() @ w.float().t() + b.float())
    pos = want > 0.05  # clearly positive under bf16 rounding: zero only where dropped
    kept = (ref[0] != 0) & pos
    assert abs(kept.float().sum().item() / pos.float().sum().item() - 0.7) < 0.02
    assert torch.allclose(ref[0].float()[kept], (want / 0.7)[kept], atol=5e-2, rtol=3e-2)
    assert torch.allclose(ref[3].float(), dy.float() @ w2.float() + r.float(), atol=0.5, rtol=3e-2)
    assert torch.allclose(ref[5].float(), x3.float() @ w3.float().t(), atol=5e-2, rtol=3e-2)


def test_linear_op_matches_reference(k):
    from mipipe.ops import linear

    torch.manual_seed(2)
    T, K, N = 256, 512, 384
    for act in (None, "relu", "gelu"):
        x = torch.randn(2, T // 2, K, device=DEV).to(torch.bfloat16).requires_grad_()
        w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).to(torch.bfloat16).requires_grad_()
        b = torch.randn(N, device=DEV).to(torch.bfloat16).requires_grad_()
        y = linear(x, w, b, act, 0.0, True)
        xf, wf, bf = (t.detach().float().requires_grad_() for t in (x, w, b))
        ref = xf @ wf.t() + bf
        ref = torch.relu(ref) if act == "relu" else (F.gelu(ref) if act == "gelu" else ref)
        assert torch.allclose(y.float(), ref, atol=3e-2, rtol=3e-2), act
        g = torch.randn_like(ref)
        y.backward(g.to(torch.bfloat16))
        ref.backward(g)
        assert torch.allclose(x.grad.float(), xf.grad, atol=6e-2, rtol=5e-2), act
        assert torch.allclose(w.grad.float(), wf.grad, atol=2e-1, rtol=5e-2), act
        assert torch.allclose(b.grad.float(), bf.grad, atol=2e-1, rtol=5e-2), act


@pytest.mark.parametrize("T,K,N", [(256, 512, 384), (520, 264, 136)])
def test_linear_residual_epilogue(k, T, K, N):
    """``res + dropout(x W^T + b)`` with the add in the GEMM epilogue, against fp32
    (p = 0) and against ``res + linear(...)`` with the same Philox draw (p > 0)."""
    from mipipe.ops import linear, linear_residual

    torch.manual_seed(6)
    x = torch.randn(T, K, device=DEV).to(torch.bfloat16).requires_grad_()
    w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).to(torch.bfloat16).requires_grad_()
    b = torch.randn(N, device=DEV).to(torch.bfloat16).requires_grad_()
    r = torch.randn(T, N, device=DEV).to(torch.bfloat16).requires_grad_()
    y = linear_residual(x, w, b, r, 0.0, True)
    xf, wf, bf, rf = (t.detach().float().requires_grad_() for t in (x, w, b, r))
    ref = rf + xf @ wf.t() + bf
    assert torch.allclose(y.float(), ref, atol=3e-2, rtol=3e-2)
    g = torch.randn_like(ref)
    y.backward(g.to(torch.bfloat16))
    ref.backward(g)
    assert torch.allclose(x.grad.float(), xf.grad, atol=6e-2, rtol=5e-2)
    assert torch.allclose(w.grad.float(), wf.grad, atol=2e-1, rtol=5e-2)
    assert torch.allclose(b.grad.float(), bf.grad, atol=2e-1, rtol=5e-2)
    assert torch.allclose(r.grad.float(), rf.grad, atol=1e-2, rtol=1e-2)
    with torch.no_grad():
        torch.manual_seed(9)
        y1 = linear_residual(x, w, b, r, 0.2, True)
        torch.manual_seed(9)
        y2 = r.float() + linear(x, w, b, None, 0.2, True).float()
    assert torch.allclose(y1.float(), y2, atol=6e-2, rtol=2e-2)


@pytest.mark.parametrize("T,K,N", [(2048, 1600, 4800), (1024, 6400, 1600), (520, 264, 136)])
def test_linear_edge_shapes_main_grad(k, T, K, N):
    """Non-multiple-of-256 widths (GPT-2-XL) go through the masked edge tiles in all three GEMMs."""
    from mipipe.ops import linear

    torch.manual_seed(4)
    x = torch.randn(T, K, device=DEV).to(torch.bfloat16).requires_grad_()
    w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).to(torch.bfloat16).requires_grad_()
    b = torch.randn(N, device=DEV).to(torch.bfloat16).requires_grad_()
    w.main_grad = torch.zeros(N, K, device=DEV)
    b.main_grad = torch.zeros(N, device=DEV)
    y = linear(x, w, b, "gelu", 0.0, True)
    xf, wf, bf = (t.detach().float().requires_grad_() for t in (x, w, b))
    ref = F.gelu(xf @ wf.t() + bf)
    g = torch.randn_like(ref)
    y.backward(g.to(torch.bfloat16))
    ref.backward(g)

    def rel(a, b):  # error relative to the tensor's scale (sums over up to 6400 bf16 products)
        return ((a.float() - b).abs().max() / b.abs().max()).item()

    assert rel(y, ref) < 2e-2
    assert rel(x.grad, xf.grad) < 2e-2
    assert rel(w.main_grad, wf.grad) < 2e-2
    assert rel(b.main_grad, bf.grad) < 2e-2
    # masked edge tiles must not write past N / M: check the last rows/cols explicitly
    assert rel(w.main_grad[-8:, -8:], wf.grad[-8:, -8:]) < 5e-2


@pytest.mark.parametrize("nseg,T,N,K", [(4, 256, 512, 384), (20, 128, 264, 136), (3, 1024, 1600, 4800)])
def test_wgrad_segments_matches_sum(k, nseg, T, N, K):
    """K-segmented weight-gradient GEMM (deferred wgrad) == sum of per-micro-batch dY^T X."""
    torch.manual_seed(5)
    dys = [torch.randn(T, N, device=DEV).to(torch.bfloat16) for _ in range(nseg)]
    xs = [torch.randn(T, K, device=DEV).to(torch.bfloat16) for _ in range(nseg)]
    main = torch.randn(N, K, device=DEV)
    expect = main.clone()
    for d, x in zip(dys, xs):
        expect += d.float().t() @ x.float()
    k.linear_wgrad_segments(dys, xs, main)
    err = ((main - expect).abs().max() / expect.abs().max()).item()
    assert err < 1e-3, err


def test_deferred_wgrad_op(k):
    from mipipe import ops

    torch.manual_seed(6)
    w = (torch.randn(384, 256, device=DEV) / 16).to(torch.bfloat16).requires_grad_()
    w.main_grad = torch.zeros(384, 256, device=DEV)
    xs = [torch.randn(128, 256, device=DEV).to(torch.bfloat16) for _ in range(3)]
    gs = [torch.randn(128, 384, device=DEV).to(torch.bfloat16) for _ in range(3)]
    with ops.deferred_wgrad():
        for x, g in zip(xs, gs):
            ops.linear(x, w, None, "relu", 0.0, True).backward(g)
        assert w.main_grad.abs().max().item() == 0.0  # nothing ran yet
    expect = torch.zeros(384, 256, device=DEV)
    for x, g in zip(xs, gs):
        pre = x.float() @ w.detach().float().t()
        expect += (g.float() * (pre > 0).float()).t() @ x.float()
    err = ((w.main_grad - expect).abs().max() / expect.abs().max()).item()
    assert err < 2e-2, err


@pytest.mark.parametrize("act,p,T", [(2, 0.0, 512), (2, 0.1, 512), (1, 0.2, 512), (2, 0.1, 8192), (1, 0.0, 384),
                                     (3, 0.0, 512), (3, 0.1, 8192), (3, 0.1, 384)])
def test_linear_dgrad_activation_backward_epilogue(k, act, p, T):
    """dgrad with the activation backward in the epilogue == (dy W) * mask * act'(saved):
    the mask regenerated from the forward GEMM's Philox layout (big and 128x128 kernels).
    act 3: a GELU forward that saved GELU'(pre) (aux_grad) and the one-multiply backward."""
    torch.manual_seed(30)
    E, F = 256, 1024
    x = torch.randn(T, E, device=DEV).to(torch.bfloat16)
    w1 = (torch.randn(F, E, device=DEV) * 0.05).to(torch.bfloat16)
    b1 = (torch.randn(F, device=DEV) * 0.1).to(torch.bfloat16)
    w2 = (torch.randn(E, F, device=DEV) * 0.05).to(torch.bfloat16)
    fwd_act = 2 if act == 3 else act
    y, saved_t, seed, offset = k.linear_fwd(x, w1, b1, fwd_act, p, fwd_act == 2, None, None, act == 3)
    saved = saved_t if fwd_act == 2 else y
    dy = torch.randn(T, E, device=DEV).to(torch.bfloat16)
    got = k.linear_dgrad(dy, w2, None, None, act, saved, p, seed, offset)
    dh = dy.float() @ w2.float()
    keep = (y != 0).float()  # GELU output is 0 only where dropped
    scale = 1.0 / (1.0 - p) if p > 0 else 1.0
    s = x.float() @ w1.float().t() + b1.float()  # the pre-activation, fp32
    grad = 0.5 * (1 + torch.erf(s / math.sqrt(2))) + s * torch.exp(-0.5 * s * s) / math.sqrt(2 * math.pi)
    if act == 3:
        # the saved tensor is GELU'(pre) itself, to bf16 rounding
        assert ((saved.float() - grad).abs().max()).item() < 2e-2
        # the elementwise backward with the same code: dy * saved * mask
        dpre, _ = k.bias_act_bwd(dh.to(torch.bfloat16), saved, None, 3, p, seed, offset, False)
        ref_e = dh * keep * scale * grad
        assert ((dpre.float() - ref_e).abs().max() / ref_e.abs().max()).item() < 2e-2
    if act in (2, 3):
        ref = dh * keep * scale * grad
    else:
        ref = dh * keep * scale
    err = ((got.float() - ref).abs().max() / ref.abs().max()).item()
    assert err < 2e-2 if act == 3 else 1e-2, err


@pytest.mark.parametrize("norm_first", [True, False])
def test_gelu_saved_grad_matches_saved_preactivation(k, norm_first):
    """A GELU FeedForwardBlock trained with GELU'(pre) saved (default; folded into fc_out's
    dgrad) gets the gradients of the pre-activation-saving path (unfolded elementwise GELU
    backward), same dropout masks."""
    import importlib

    from mipipe.models.transformer import FeedForwardBlock

    L = importlib.import_module("mipipe.ops.linear")
    torch.manual_seed(33)
    blk = FeedForwardBlock(256, 1024, 0.1, "gelu", norm_first=norm_first, device=DEV, dtype=torch.bfloat16)
    x0 = torch.randn(4, 128, 256, device=DEV).to(torch.bfloat16)
    grads = []
    for save_grad in (True, False):
        old = L._GELU_SAVE_GRAD
        L._GELU_SAVE_GRAD = save_grad
        try:
            for prm in blk.parameters():
                prm.grad = None
            x = x0.clone().requires_grad_()
            torch.cuda.manual_seed(6)
            f = ActFold() if save_grad else None
            h, xr = blk.fc_in.forward_fanout(x, True, f)
            out = blk.fc_out(xr, h, f)
            out.float().square().sum().backward()
            grads.append([x.grad.float().clone()] + [prm.grad.float().clone() for prm in blk.parameters()])
        finally:
            L._GELU_SAVE_GRAD = old
    for a, b in zip(*grads):
        assert ((a - b).abs().max() / (b.abs().max() + 1e-12)).item() < 2e-2


@pytest.mark.parametrize("activation,norm_first", [("relu", False), ("gelu", True), ("gelu", False)])
def test_feedforward_act_fold_matches_unfolded(k, activation, norm_first):
    """FeedForwardBlock with the activation backward folded into fc_out's dgrad
    == the same block without the fold (same dropout masks: reseeded)."""
    from mipipe.models.transformer import FeedForwardBlock

    torch.manual_seed(31)
    blk = FeedForwardBlock(256, 1024, 0.1, activation, norm_first=norm_first, device=DEV, dtype=torch.bfloat16)
    x0 = torch.randn(4, 128, 256, device=DEV).to(torch.bfloat16)
    grads = []
    for fold in (True, False):
        for prm in blk.parameters():
            prm.grad = None
        x = x0.clone().requires_grad_()
        torch.cuda.manual_seed(5)
        f = ActFold() if fold else None
        h, xr = blk.fc_in.forward_fanout(x, True, f)
        out = blk.fc_out(xr, h, f)
        out.float().square().sum().backward()
        if fold:
            assert f.act != 0 and f.saved is None and f.grad is None  # offered, taken over, folded, consumed
        grads.append([x.grad.float().clone()] + [prm.grad.float().clone() for prm in blk.parameters()])
    for a, b in zip(*grads):
        assert ((a - b).abs().max() / (b.abs().max() + 1e-12)).item() < 2e-2


def test_relu_bits_fold_bit_exact(k):
    """ReLU + dropout folded into fc_out's dgrad through the 1-bit nonzero mask the forward GEMM writes
    (kActReluBits) == the same fold re-reading the bf16 output, bit for bit; the bits are the output's
    nonzeros.  Shapes large enough for the 256-row kernel (the one that writes bits)."""
    import sys

    from mipipe.models.transformer import FeedForwardBlock

    L = sys.modules["mipipe.ops.linear"]  # the module (mipipe.ops re-exports a function of that name)
    torch.manual_seed(41)
    blk = FeedForwardBlock(1024, 2048, 0.2, "relu", device=DEV, dtype=torch.bfloat16)
    x0 = torch.randn(16, 256, 1024, device=DEV).to(torch.bfloat16)
    assert k.linear_bits_ok(16 * 256, 2048, 1024, 1, 0.2)
    grads, offered = [], []
    old = L._RELU_BITS
    try:
        for bits in (True, False):
            L._RELU_BITS = bits
            for prm in blk.parameters():
                prm.grad = None
            x = x0.clone().requires_grad_()
            torch.cuda.manual_seed(6)
            f = ActFold()
            h, xr = blk.fc_in.forward_fanout(x, True, f)
            offered.append((f.act, None if f.saved is None else f.saved.clone(), h.detach().clone()))
            out = blk.fc_out(xr, h, f)
            out.float().square().sum().backward()
            assert f.saved is None and f.grad is None  # folded and consumed
            grads.append([x.grad.clone()] + [prm.grad.clone() for prm in blk.parameters()])
    finally:
        L._RELU_BITS = old
    (act_b, bits_t, h_b), (act_y, _, _) = offered
    assert act_b == L.KACT_RELU_BITS and act_y == 1
    nz = (h_b.reshape(-1, 2048) != 0).to(torch.uint8).view(-1, 256, 8)
    packed = (nz << torch.arange(8, device=DEV, dtype=torch.uint8)).sum(-1, dtype=torch.int32).to(torch.uint8)
    assert torch.equal(bits_t, packed.view(-1, 256))
    for a, b in zip(*grads):
        assert torch.equal(a, b)


def test_act_fold_rejects_second_consumer(k):
    """The fold is only valid when h has one consumer: a second use is caught."""
    torch.manual_seed(32)
    x = torch.randn(256, 128, device=DEV).to(torch.bfloat16).requires_grad_()
    w1 = (torch.randn(512, 128, device=DEV) * 0.05).to(torch.bfloat16).requires_grad_()
    w2 = (torch.randn(128, 512, device=DEV) * 0.05).to(torch.bfloat16).requires_grad_()
    f = ActFold()
    h = ops.linear(x, w1, None, "gelu", 0.0, True, act_fold_out=f)
    y = ops.linear(h, w2, None, act_fold_in=f)
    with pytest.raises(RuntimeError, match="another consumer"):
        (y.float().sum() + h.float().sum()).backward()


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_learned_positions_fused_embedding(k, p):
    """GPT-2 learned positions through the fused embedding kernels: forward adds
    the table, backward accumulates its gradient by position (dropout mask
    shared with the token-table gradient)."""
    from mipipe.models.lm import Encoder

    torch.manual_seed(33)
    enc = Encoder(1000, 256, p, max_len=128, learned_positions=True, scale_embedding=False, device=DEV,
                  dtype=torch.bfloat16)
    tok = torch.randint(0, 1000, (4, 64), device=DEV)
    y = enc(tok)
    dy = torch.randn_like(y)
    y.backward(dy)
    keep = (y != 0).float() if p > 0 else torch.ones_like(y, dtype=torch.float32)
    scale = 1.0 / (1.0 - p) if p > 0 else 1.0
    g = dy.float() * keep * scale  # [B, S, E]
    ref_pos = torch.zeros(128, 256, device=DEV)
    ref_pos[:64] = g.sum(0)
    ref_tok = torch.zeros(1000, 256, device=DEV).index_add_(0, tok.reshape(-1), g.reshape(-1, 256))
    assert enc.pos_weight.grad is not None
    assert ((enc.pos_weight.grad.float() - ref_pos).abs().max() / ref_pos.abs().max()).item() < 1e-2
    assert ((enc.weight.grad.float() - ref_tok).abs().max() / ref_tok.abs().max()).item() < 2e-2
    # forward: table rows + position rows (where kept)
    ref_y = (enc.weight.float()[tok] + enc.pos_weight.float()[:64]) * scale * keep
    assert ((y.float() - ref_y).abs().max() / ref_y.abs().max()).item() < 1e-2


def test_linear_dropout_mask_and_main_grad(k):
    from mipipe.ops import linear

    torch.manual_seed(3)
    T, K, N, p = 256, 256, 256, 0.4
    x = torch.randn(T, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) / 16).to(torch.bfloat16).requires_grad_()
    w.main_grad = torch.zeros(N, K, device=DEV)
    y = linear(x, w, None, None, p, True)
    keep = (y != 0).float()
    assert abs(keep.mean().item() - (1 - p)) < 0.02
    g = torch.randn(T, N, device=DEV)
    y.backward(g.to(torch.bfloat16))
    assert w.grad is None  # accumulated in main_grad instead
    expect = ((g.to(torch.bfloat16).float() * keep / (1 - p)).t() @ x.float())
    assert torch.allclose(w.main_grad, expect, atol=2e-1, rtol=3e-2)
    # second micro-batch accumulates
    y2 = linear(x, w, None, None, p, True)
    y2.backward(g.to(torch.bfloat16))
    keep2 = (y2 != 0).float()
    expect2 = expect + ((g.to(torch.bfloat16).float() * keep2 / (1 - p)).t() @ x.float())
    assert torch.allclose(w.main_grad, expect2, atol=3e-1, rtol=3e-2)


# ------------------------------------------------------------------ attention
def _philox4x32_10(c0, c1, c2, c3, k0, k1):
    """numpy Philox4x32-10 (the kernels' RNG), vectorised over counters."""
    import numpy as np

    M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
    mask = np.uint64(0xFFFFFFFF)
    c0, c1, c2, c3 = (np.asarray(x, dtype=np.uint64) for x in (c0, c1, c2, c3))
    k0, k1 = np.uint64(k0), np.uint64(k1)
    for _ in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & mask
        hi1, lo1 = p1 >> np.uint64(32), p1 & mask
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & mask, lo1, (hi0 ^ c3 ^ k1) & mask, lo0
        k0 = (k0 + np.uint64(0x9E3779B9)) & mask
        k1 = (k1 + np.uint64(0xBB67AE85)) & mask
    return c0, c1, c2, c3


def _attn_keep_mask(B, H, S, p, seed, offset):
    import numpy as np

    bh, q, key = np.meshgrid(np.arange(B * H), np.arange(S), np.arange(S), indexing="ij")
    sub = (bh.astype(np.uint64) * np.uint64(S // 4) + (q // 4).astype(np.uint64)) * np.uint64(S) + key.astype(np.uint64)
    seed = seed & 0xFFFFFFFFFFFFFFFF
    offset = offset & 0xFFFFFFFFFFFFFFFF
    m32 = np.uint64(0xFFFFFFFF)
    words = _philox4x32_10(sub & m32, sub >> np.uint64(32), np.uint64(offset) & m32, np.uint64(offset) >> np.uint64(32),
                           seed & 0xFFFFFFFF, seed >> 32)
    w = np.choose((q & 3), words)
    thr = min(int(p * 4294967296.0), 0xFFFFFFFF)
    return torch.from_numpy((w >= thr).reshape(B, H, S, S))


def _long_keep_mask(B, H, S, p, seed, offset):
    """Dropout mask of the long-sequence kernels (attention_long.hip): the uniform of
    (q, key) of head bh is the SIGNED 16-bit half (q % 32) // 16 of word q % 4 of
    Philox counter ((bh * S/32 + q/32) * S + key) * 4 + (q % 16) // 4, kept iff it is
    >= (p * 2^32 >> 16) - 2^15."""
    import numpy as np

    bh, q, key = np.meshgrid(np.arange(B * H), np.arange(S), np.arange(S), indexing="ij")
    qq = q % 32
    sub = ((bh.astype(np.uint64) * np.uint64(S // 32) + (q // 32).astype(np.uint64)) * np.uint64(S)
           + key.astype(np.uint64)) * np.uint64(4) + ((qq % 16) // 4).astype(np.uint64)
    seed &= 0xFFFFFFFFFFFFFFFF
    offset &= 0xFFFFFFFFFFFFFFFF
    m32 = np.uint64(0xFFFFFFFF)
    words = _philox4x32_10(sub & m32, sub >> np.uint64(32), np.uint64(offset) & m32, np.uint64(offset) >> np.uint64(32),
                           seed & 0xFFFFFFFF, seed >> 32)
    w = np.choose(qq % 4, words)
    u16 = (w >> (np.uint64(16) * (qq // 16).astype(np.uint64))) & np.uint64(0xFFFF)
    s16 = u16.astype(np.int64) - (u16 >= np.uint64(0x8000)).astype(np.int64) * 65536
    thr = (min(int(p * 4294967296.0), 0xFFFFFFFF) >> 16) - 32768
    return torch.from_numpy((s16 >= thr).reshape(B, H, S, S))


def _bits_to_mask(bits, B, H, S):
    """Keep bits stored by the long-sequence forward: word [bh, q // 32, key], bit q % 32."""
    w = bits.view(B * H, S // 32, S).to(torch.int64) & 0xFFFFFFFF
    shifts = torch.arange(32, device=bits.device, dtype=torch.int64)
    m = (w.unsqueeze(2) >> shifts.view(1, 1, 32, 1)) & 1  # [bh, qblk, 32, key]
    return m.reshape(B, H, S, S).bool().cpu()


def _ref_attention_masked(q, k, v, causal, keep, p, scale):
    s = torch.matmul(q.float(), k.float().transpose(-1, -2)) * scale
    if causal:
        S = s.shape[-1]
        s = s.masked_fill(torch.ones(S, S, dtype=torch.bool, device=s.device).triu(1), float("-inf"))
    pr = torch.softmax(s, dim=-1)
    if keep is not None:
        pr = pr * keep.to(pr.device).float() / (1 - p)
    return torch.matmul(pr, v.float())


@pytest.mark.parametrize("D", [64, 128, 256])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("p", [0.0, 0.25])
@pytest.mark.parametrize("S,fused", [(128, 1), (128, 0), (256, 1), (512, 1), (320, 1)])
def test_attention_packed(k, D, causal, p, S, fused):
    """S = 128 runs the fused one-pass backward (fused=1) or the general
    delta + dK/dV + dQ kernels (fused=0); S = 256 always the general ones."""
    k.attention_set_fused_bwd(fused)
    try:
        _check_attention_packed(k, D, causal, p, S)
    finally:
        k.attention_set_fused_bwd(1)


def _check_attention_packed(k, D, causal, p, S):
    from mipipe.ops import attention_packed

    torch.manual_seed(4)
    B, H = 2, 2
    qkv = torch.randn(B, S, 3, H, D, device=DEV).to(torch.bfloat16).requires_grad_()
    scale = 1.0 / math.sqrt(D)
    long = k.attention_long_supported(S, D)
    if p > 0:
        q, kk, v = (qkv.detach().select(2, i) for i in range(3))
        o, lse, seed, offset, bits = k.attention_fwd(q, kk, v, causal, p, scale)
        if long:
            keep = _long_keep_mask(B, H, S, p, seed, offset)
            stored = _bits_to_mask(bits, B, H, S)
            if causal:  # blocks wholly above the diagonal are never written
                tri = torch.ones(S, S, dtype=torch.bool).tril()
                assert torch.equal(stored & tri, keep & tri)
            else:
                assert torch.equal(stored, keep)
        else:
            assert bits.numel() == 0
            keep = _attn_keep_mask(B, H, S, p, seed, offset)
        assert abs(keep.float().mean().item() - (1 - p)) < 0.02
    else:
        keep = None
    torch.manual_seed(11)
    o = attention_packed(qkv, causal, p, True)  # [B, S, H, D]
    if p > 0:
        # the op drew its own seed: rebuild the mask from the generator state it used
        torch.manual_seed(11)
        _, _, seed2, offset2, _ = k.attention_fwd(*(qkv.detach().select(2, i) for i in range(3)), causal, p, scale)
        keep = (_long_keep_mask if long else _attn_keep_mask)(B, H, S, p, seed2, offset2)
    qf = qkv.detach().float().requires_grad_()
    qh, kh, vh = (qf.select(2, i).transpose(1, 2) for i in range(3))
    ref = _ref_attention_masked(qh, kh, vh, causal, keep, p, scale).transpose(1, 2)
    err = (o.float() - ref).abs().max().item()
    assert err < 3e-2, err
    g = torch.randn_like(ref)
    o.backward(g.to(torch.bfloat16))
    ref.backward(g)
    gerr = (qkv.grad.float() - qf.grad).abs().max().item()
    gscale = qf.grad.abs().max().item()
    assert gerr < 3e-2 * max(1.0, gscale), (gerr, gscale)


@pytest.mark.parametrize("causal", [False, True])
def test_attention_keep_words_reused_bit_exact(k, causal):
    """A checkpoint's recompute reads the keep words its first forward made (ops/attention.py) instead of making
    them again: output and gradients bit-identical to the same checkpointed run with the reuse off, and to a run
    without checkpointing."""
    import sys

    from mipipe import checkpoint
    from mipipe.ops import attention_packed

    A = sys.modules["mipipe.ops.attention"]
    B, S, H, D, p = 2, 512, 3, 64, 0.15
    assert k.attention_long_supported(S, D)
    torch.manual_seed(5)
    base = torch.randn(B, S, 3, H, D, device=DEV).to(torch.bfloat16)
    g = torch.randn(B, S, H, D, device=DEV).to(torch.bfloat16)

    def run(ckpt: bool, reuse: bool):
        A._KEEP_REUSE = reuse
        A.clear_keep_words()
        x = base.clone().requires_grad_()
        torch.manual_seed(7)
        f = lambda t: attention_packed(t, causal, p, True)  # noqa: E731
        o = checkpoint(f, x) if ckpt else f(x)
        o.backward(g)
        torch.cuda.synchronize()
        return o.detach(), x.grad

    old = A._KEEP_REUSE
    try:
        before = dict(A.keep_stats)
        o1, g1 = run(True, True)
        assert A.keep_stats["stored"] == before["stored"] + 1 and A.keep_stats["reused"] == before["reused"] + 1
        assert not A._keep_words  # taken by the recompute
        o0, g0 = run(True, False)
        o2, g2 = run(False, True)
    finally:
        A._KEEP_REUSE = old
        A.clear_keep_words()
    assert torch.equal(o1, o0) and torch.equal(g1, g0)
    assert torch.equal(o1, o2) and torch.equal(g1, g2)


@pytest.mark.parametrize("causal", [False, True])
def test_attention_long_fused_rng_identical(k, causal):
    """Keep words made inside the long-sequence forward kernel (default) and by the
    stand-alone keep-bit kernel are the same words: output, LSE and stored bits match
    bitwise."""
    torch.manual_seed(2)
    B, H, S, D, p = 2, 3, 512, 64, 0.2
    qkv = torch.randn(B, S, 3, H, D, device=DEV).to(torch.bfloat16)
    q, kk, v = (qkv.select(2, i) for i in range(3))
    outs = []
    for fused in (True, False):
        k.attention_long_set_fused_rng(fused)
        try:
            torch.manual_seed(9)
            outs.append(k.attention_fwd(q, kk, v, causal, p, D ** -0.5))
        finally:
            k.attention_long_set_fused_rng(True)
    (o1, l1, s1, f1, b1), (o2, l2, s2, f2, b2) = outs
    assert (s1, f1) == (s2, f2)
    assert torch.equal(o1, o2) and torch.equal(l1, l2)
    m1, m2 = _bits_to_mask(b1, B, H, S), _bits_to_mask(b2, B, H, S)
    if causal:
        tri = torch.ones(S, S, dtype=torch.bool).tril()
        m1, m2 = m1 & tri, m2 & tri
    assert torch.equal(m1, m2)


@pytest.mark.parametrize("dtype,D", [(torch.bfloat16, 64), (torch.bfloat16, 128), (torch.float32, 64)])
@pytest.mark.parametrize("S", [37, 100, 200])
def test_attention_causal_any_length(k, dtype, D, S):
    """Causal sequences of unsupported lengths (the reference's get_batch tail window)
    run on the kernels zero-padded at the end -- exact for the real rows, no eager path."""
    import warnings

    from mipipe.ops import attention_packed, attention_reference

    torch.manual_seed(3)
    B, H = 2, 4
    qkv = (torch.randn(B, S, 3, H, D, device=DEV) * 0.5).to(dtype).requires_grad_()
    with warnings.catch_warnings():
        warnings.simplefilter("error")  # the eager fallback warns
        o = attention_packed(qkv, causal=True, dropout_p=0.0)
    assert o.shape == (B, S, H, D)
    qf = qkv.detach().float().requires_grad_()
    ref = attention_reference(*(qf.select(2, i).transpose(1, 2) for i in range(3)), True, 0.0).transpose(1, 2)
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    assert ((o.float() - ref).abs().max() / ref.abs().max()).item() < tol
    g = torch.randn_like(ref)
    o.backward(g.to(dtype))
    ref.backward(g)
    assert ((qkv.grad.float() - qf.grad).abs().max() / qf.grad.abs().max()).item() < 5 * tol


@pytest.mark.parametrize("dtype,D,S,causal", [(torch.bfloat16, 32, 128, False), (torch.bfloat16, 80, 256, True),
                                               (torch.bfloat16, 96, 128, False), (torch.bfloat16, 160, 100, True),
                                               (torch.float32, 32, 128, True), (torch.float32, 48, 64, False),
                                               (torch.bfloat16, 64, 100, False), (torch.bfloat16, 128, 200, False),
                                               (torch.bfloat16, 80, 37, False), (torch.float32, 32, 50, False)])
def test_attention_any_head_dim(k, dtype, D, S, causal):
    """Head dims the kernels do not tile run on them zero-padded to the next tiled one
    (scale of the real head dim, padded columns sliced off); non-causal sequences of
    other lengths run padded with the padded keys masked through a spare feature --
    no eager path."""
    import warnings

    from mipipe.ops import attention, attention_packed, attention_reference

    torch.manual_seed(6)
    B, H = 2, 3
    qkv = (torch.randn(B, S, 3, H, D, device=DEV) * 0.5).to(dtype).requires_grad_()
    with warnings.catch_warnings():
        warnings.simplefilter("error")  # the eager fallback warns
        o = attention_packed(qkv, causal=causal, dropout_p=0.0)
        o2 = attention(*(qkv.detach().select(2, i).transpose(1, 2) for i in range(3)), causal=causal)
    assert o.shape == (B, S, H, D) and o2.shape == (B, H, S, D)
    qf = qkv.detach().float().requires_grad_()
    ref = attention_reference(*(qf.select(2, i).transpose(1, 2) for i in range(3)), causal, 0.0).transpose(1, 2)
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    assert ((o.float() - ref).abs().max() / ref.abs().max()).item() < tol
    assert ((o2.transpose(1, 2).float() - ref).abs().max() / ref.abs().max()).item() < tol
    g = torch.randn_like(ref)
    o.backward(g.to(dtype))
    ref.backward(g)
    assert ((qkv.grad.float() - qf.grad).abs().max() / qf.grad.abs().max()).item() < 5 * tol


def test_attention_bhsd_api(k):
    from mipipe.ops import attention, attention_reference

    torch.manual_seed(5)
    q, kk, v = (torch.randn(2, 4, 192, 64, device=DEV).to(torch.bfloat16) for _ in range(3))
    o = attention(q, kk, v, causal=True)
    ref = attention_reference(q, kk, v, True, 0.0)
    assert (o.float() - ref.float()).abs().max().item() < 3e-2


def test_transformer_layer_bf16_kernels_vs_torch(k):
    """The bf16 hot path (MFMA GEMMs, flash attention, fused LN) vs nn.TransformerEncoderLayer in fp32."""
    from torch import nn

    from mipipe.models import TransformerEncoderLayer

    import copy

    torch.manual_seed(0)
    E, H, F_, B, S = 512, 4, 1024, 2, 128
    ref = nn.TransformerEncoderLayer(E, H, F_, dropout=0.0, batch_first=True).to(DEV)
    ref_bf16 = copy.deepcopy(ref).to(torch.bfloat16)  # PyTorch's own bf16 error sets the gradient bar
    ours = TransformerEncoderLayer(E, H, F_, dropout=0.0, device=DEV).load_from_torch(ref).to(torch.bfloat16)
    x = torch.randn(B, S, E, device=DEV)
    xb = x.to(torch.bfloat16).requires_grad_()
    xr = x.clone().requires_grad_()
    y = ours(xb)
    yr = ref(xr)
    err = (y.float() - yr).abs().max().item()
    assert err < 0.1, err
    # backward: input and every parameter gradient, relative to the fp32 gradient's scale
    g = torch.randn_like(yr)
    y.backward(g.to(torch.bfloat16))
    yr.backward(g)
    ref_bf16(x.to(torch.bfloat16)).backward(g.to(torch.bfloat16))

    def rel(a, b):
        return (a.float() - b.float()).abs().max().item() / (b.float().abs().max().item() + 1e-6)

    assert rel(xb.grad, xr.grad) < 3e-2, rel(xb.grad, xr.grad)
    attn, ff = ours[0], ours[1]
    names = [("self_attn.in_proj_weight", attn.core.in_proj_weight), ("self_attn.in_proj_bias", attn.core.in_proj_bias),
             ("self_attn.out_proj.weight", attn.out.out_proj_weight), ("self_attn.out_proj.bias", attn.out.out_proj_bias),
             ("norm1.weight", attn.out.norm_weight), ("norm1.bias", attn.out.norm_bias),
             ("linear1.weight", ff.fc_in.linear1_weight), ("linear1.bias", ff.fc_in.linear1_bias),
             ("linear2.weight", ff.fc_out.linear2_weight), ("linear2.bias", ff.fc_out.linear2_bias),
             ("norm2.weight", ff.fc_out.norm_weight), ("norm2.bias", ff.fc_out.norm_bias)]
    ref_p, bf_p = dict(ref.named_parameters()), dict(ref_bf16.named_parameters())

    def rel_fro(a, b):
        # norm-wise: a ReLU whose bf16 pre-activation lands on the other side of 0
        # moves single elements of the weight gradient by a whole token's share
        return (a.float() - b.float()).norm().item() / (b.float().norm().item() + 1e-6)

    for name, ours_p in names:
        got = ours_p.main_grad if getattr(ours_p, "main_grad", None) is not None else ours_p.grad
        assert got is not None
        err, torch_err = rel_fro(got, ref_p[name].grad), rel_fro(bf_p[name].grad, ref_p[name].grad)
        # within PyTorch's own bf16 error (linear1.weight: ~0.045 vs torch 0.050 -- ReLU flips)
        assert err < max(1.25 * torch_err, 2e-2), (name, err, torch_err)


def test_vocab_split_decoder_gpu(k):
    """Head/tail (MFMA logits, CE kernels with per-row scale) == decoder + fused CE."""
    from mipipe.models import Decoder, split_decoder
    from mipipe.ops import cross_entropy

    torch.manual_seed(8)
    dec = Decoder(1000, 256, device=DEV, dtype=torch.bfloat16)
    head, tail = split_decoder(dec)
    x = torch.randn(2, 64, 256, device=DEV).to(torch.bfloat16).requires_grad_()
    t = torch.randint(0, 1000, (2, 64), device=DEV)
    ref = cross_entropy(dec(x), t)
    ref.backward()
    x2 = x.detach().clone().requires_grad_()
    loss = tail(head(x2, t), t)
    loss.backward()
    assert abs(loss.item() - ref.item()) < 2e-3 * abs(ref.item())

    def rel(a, b):
        return ((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-12)).item()

    assert rel(x2.grad, x.grad) < 2e-2
    assert rel(head.weight.grad, dec.weight.grad[:512]) < 2e-2
    assert rel(tail.weight.grad[:488], dec.weight.grad[512:1000]) < 2e-2
    assert rel(tail.bias.grad[:488], dec.bias.grad[512:1000]) < 2e-2


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_vocab_split_ignore_index_and_dtypes(k, dtype):
    """Ignored targets (and targets in both halves) through the fused pack /
    merge / mean kernels, bf16 and fp32, against the fp32 PyTorch loss."""
    from mipipe.models import Decoder, split_decoder

    torch.manual_seed(18)
    dec = Decoder(1000, 256, device=DEV, dtype=dtype)
    head, tail = split_decoder(dec)
    x = torch.randn(2, 64, 256, device=DEV).to(dtype).requires_grad_()
    t = torch.randint(0, 1000, (2, 64), device=DEV)
    t[0, :7] = -100
    xr = x.detach().float().requires_grad_()
    wr = dec.weight.detach().float().requires_grad_()
    logits = (xr @ wr.t() + dec.bias.float())[..., :1000].reshape(-1, 1000)  # the decoder pads its rows
    ref = torch.nn.functional.cross_entropy(logits, t.reshape(-1), ignore_index=-100)
    ref.backward()
    loss = tail(head(x, t), t)
    loss.backward()
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    assert abs(loss.item() - ref.item()) < tol * abs(ref.item())

    def rel(a, b):
        return ((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-12)).item()

    assert rel(x.grad, xr.grad) < 3 * tol
    assert rel(head.weight.grad, wr.grad[:512]) < 3 * tol
    assert rel(tail.weight.grad[:488], wr.grad[512:1000]) < 3 * tol
    assert tail.weight.grad[488:].abs().max().item() == 0.0  # padded vocabulary rows
    # the fixed-order mean: bitwise reproducible
    again = tail(head(x.detach(), t), t)
    assert again.item() == loss.item()


def test_vocab_split_launches_no_aten_kernels(k):
    """Head + tail forward and backward run only mipipe kernels (plus copies of
    nothing): no elementwise / reduction / cat kernels from ATen."""
    from mipipe.models import Decoder, split_decoder

    torch.manual_seed(19)
    dec = Decoder(1000, 256, device=DEV, dtype=torch.bfloat16)
    head, tail = split_decoder(dec)
    x = torch.randn(2, 64, 256, device=DEV).to(torch.bfloat16).requires_grad_()
    t = torch.randint(0, 1000, (2, 64), device=DEV)
    seed = torch.ones((), device=DEV)  # the loss gradient, made outside the profiled region
    tail(head(x, t), t).backward(seed)  # warm (allocations, lazy init)
    for prm in (x, head.weight, head.bias, tail.weight, tail.bias):
        prm.grad = None  # no autograd accumulation adds in the profiled pass
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts) as prof:
        tail(head(x, t), t).backward(seed)
        torch.cuda.synchronize()
    names = [e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA]
    if not names:
        pytest.skip("the profiler recorded no device kernels on this build")
    aten = [n for n in names if "at::native" in n or "elementwise" in n.lower() or "reduce_kernel" in n]
    assert not aten, aten


def test_strided_gemm_operands(k):
    """linear_fwd / linear_dgrad / linear_wgrad on column slices of packed rows
    (row stride != width) and dgrad into a strided destination with a strided addend."""
    torch.manual_seed(20)
    M, E, N, S = 512, 256, 768, 8
    packed = torch.randn(M, E + S, device=DEV).to(torch.bfloat16)
    x = packed[:, :E]
    w = torch.randn(N, E, device=DEV).to(torch.bfloat16) * 0.05
    b = torch.randn(N, device=DEV).to(torch.bfloat16)
    y = k.linear_fwd(x, w, b, 0, 0.0, False)[0]
    ref = x.float() @ w.float().t() + b.float()
    assert ((y.float() - ref).abs().max() / ref.abs().max()).item() < 1e-2
    dy = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    dmsg = torch.randn(M, E + S, device=DEV).to(torch.bfloat16)
    out = torch.zeros(M, E + S, device=DEV, dtype=torch.bfloat16)
    k.linear_dgrad(dy, w, dmsg[:, :E], out[:, :E])
    ref = dy.float() @ w.float() + dmsg[:, :E].float()
    assert ((out[:, :E].float() - ref).abs().max() / ref.abs().max()).item() < 1e-2
    assert out[:, E:].abs().max().item() == 0.0  # the slots are untouched
    g = torch.zeros(N, E, device=DEV)
    k.linear_wgrad(dy, x, g, False)
    ref = dy.float().t() @ x.float()
    assert ((g - ref).abs().max() / ref.abs().max()).item() < 1e-2


def test_cross_entropy_target_offset(k):
    """t_offset: the logits are a vocabulary slice; targets outside it get loss 0."""
    torch.manual_seed(21)
    logits = torch.randn(64, 300, device=DEV)
    t = torch.randint(0, 900, (64,), device=DEV)
    loss, lse = k.cross_entropy_fwd(logits, t, -100, t_offset=300)
    inside = (t >= 300) & (t < 600)
    expect_lse = torch.logsumexp(logits, -1)
    expect = torch.where(inside, expect_lse - logits.gather(1, (t - 300).clamp(0, 299)[:, None])[:, 0],
                         torch.zeros_like(expect_lse))
    assert torch.allclose(lse, expect_lse, atol=1e-5)
    assert torch.allclose(loss, expect, atol=1e-5)


@pytest.mark.parametrize("cols", [264, 4096])
def test_column_sum_segments(k, cols):
    torch.manual_seed(9)
    xs = [torch.randn(r, cols, device=DEV).to(torch.bfloat16) for r in (128, 4096, 40)]
    out = torch.randn(cols, device=DEV)
    expect = out + sum(x.float().sum(0) for x in xs)
    k.column_sum_segments(xs, out, True)
    assert torch.allclose(out, expect, atol=5e-2, rtol=1e-3)


@pytest.mark.parametrize("cols,rows,nseg", [(4096, 4096, 4), (264, 300, 20), (12288, 512, 3)])
def test_column_sum_segments_one_launch(k, cols, rows, nseg):
    """Equally shaped segments: one stage-1 launch per 16 segments (grid.z = segment)."""
    torch.manual_seed(10)
    xs = [torch.randn(rows, cols, device=DEV).to(torch.bfloat16) for _ in range(nseg)]
    expect = sum(x.float().sum(0) for x in xs)
    out = torch.empty(cols, device=DEV)
    k.column_sum_segments(xs, out, False)
    assert torch.allclose(out, expect, atol=5e-2, rtol=1e-3)


def test_deferred_bias_grad(k):
    from mipipe import ops

    torch.manual_seed(10)
    w = (torch.randn(256, 128, device=DEV) / 12).to(torch.bfloat16).requires_grad_()
    b = torch.zeros(256, device=DEV).to(torch.bfloat16).requires_grad_()
    w.main_grad = torch.zeros(256, 128, device=DEV)
    b.main_grad = torch.zeros(256, device=DEV)
    gs = [torch.randn(64, 256, device=DEV).to(torch.bfloat16) for _ in range(3)]
    xs = [torch.randn(64, 128, device=DEV).to(torch.bfloat16) for _ in range(3)]
    with ops.deferred_wgrad():
        for x, g in zip(xs, gs):
            ops.linear(x, w, b, "relu", 0.0, True).backward(g)
        assert b.main_grad.abs().max().item() == 0.0
    expect = torch.zeros(256, device=DEV)
    for x, g in zip(xs, gs):
        pre = x.float() @ w.detach().float().t()
        expect += (g.float() * (pre > 0).float()).sum(0)
    assert ((b.main_grad - expect).abs().max() / expect.abs().max()).item() < 2e-2


def test_fanout_ops_match_plain(k):
    """linear_fanout / layer_norm_fanout: same values and gradients as the op
    plus an autograd add of the second consumer's gradient (fused in-kernel)."""
    from mipipe import ops

    torch.manual_seed(11)
    T, E, N = 256, 512, 768
    x0 = torch.randn(T, E, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, E, device=DEV) / 20).to(torch.bfloat16)
    b = (torch.randn(N, device=DEV) / 10).to(torch.bfloat16)
    gy = torch.randn(T, N, device=DEV).to(torch.bfloat16)
    gr = torch.randn(T, E, device=DEV).to(torch.bfloat16)
    for fused in (True, False):
        x = x0.clone().requires_grad_()
        if fused:
            y, xr = ops.linear_fanout(x, w, b, "relu", 0.0, True)
        else:
            y, xr = ops.linear(x, w, b, "relu", 0.0, True), x
        torch.autograd.backward([y, xr * 1.0], [gy, gr])
        if fused:
            g_fused = x.grad.float()
        else:
            g_plain = x.grad.float()
    assert torch.allclose(g_fused, g_plain, atol=3e-2, rtol=2e-2)
    # unused fan-out branch: plain gradient
    x = x0.clone().requires_grad_()
    y, _ = ops.linear_fanout(x, w, b, "relu", 0.0, True)
    y.backward(gy)
    assert torch.allclose(x.grad.float(), g_plain - gr.float(), atol=3e-2, rtol=2e-2)

    gamma = (1 + 0.1 * torch.randn(E, device=DEV)).to(torch.bfloat16)
    beta = (0.1 * torch.randn(E, device=DEV)).to(torch.bfloat16)
    gln = torch.randn(T, E, device=DEV).to(torch.bfloat16)
    grads = []
    for fused in (True, False):
        x = x0.clone().requires_grad_()
        if fused:
            yn, xr = ops.layer_norm_fanout(x, gamma, beta, 1e-5)
        else:
            yn, xr = ops.add_dropout_layer_norm(x, None, gamma, beta, 1e-5, 0.0, True), x
        torch.autograd.backward([yn, xr * 1.0], [gln, gr])
        grads.append(x.grad.float())
    assert torch.allclose(grads[0], grads[1], atol=3e-2, rtol=2e-2)


def test_decoder_padded_vocab_grad(k):
    """Decoder (padded vocabulary) + fused CE: the zero-padded CE gradient is
    handed to the decoder GEMM without a copy; gradients match fp32 torch."""
    from mipipe.models.lm import Decoder
    from mipipe.ops import cross_entropy

    torch.manual_seed(12)
    V, E, B, S = 1000, 256, 2, 64
    dec = Decoder(V, E, device=DEV, dtype=torch.bfloat16)
    assert dec.padded > V
    x = torch.randn(B, S, E, device=DEV).to(torch.bfloat16).requires_grad_()
    t = torch.randint(0, V, (B, S), device=DEV)
    y = dec(x)
    assert y.shape == (B, S, V)
    loss = cross_entropy(y.reshape(-1, V), t.reshape(-1))
    loss.backward()
    w = dec.weight.detach().float()[:V].requires_grad_()
    b = dec.bias.detach().float()[:V].requires_grad_()
    xf = x.detach().float().requires_grad_()
    ref = F.cross_entropy((xf @ w.t() + b).reshape(-1, V), t.reshape(-1))
    ref.backward()
    assert abs(loss.item() - ref.item()) < 2e-2
    assert torch.allclose(x.grad.float(), xf.grad, atol=2e-3, rtol=5e-2)
    assert torch.allclose(dec.weight.grad.float()[:V], w.grad, atol=2e-3, rtol=5e-2)
    assert dec.weight.grad.float()[V:].abs().max().item() == 0.0


def test_lazy_zero_grad_overwrites(k):
    """FlatAdam.zero_grad(lazy=True): GEMM-only weights are not zero-filled;
    their first weight-gradient GEMM of the step overwrites main_grad (deferred
    and immediate paths) -- gradients equal an eager zero_grad's, and a second
    step does not accumulate onto the first."""
    from mipipe import ops
    from mipipe.models import CONFIGS, build_lm_blocks
    from mipipe.optim import FlatAdam

    torch.manual_seed(13)
    cfg = CONFIGS["tiny"]
    model = torch.nn.Sequential(*build_lm_blocks(cfg, device=DEV, dtype=torch.bfloat16)).train()
    opt = FlatAdam(model.parameters(), lr=1e-3)
    tok = torch.randint(0, cfg.vocab, (2, 4, cfg.seq_len + 1), device=DEV)

    def run(lazy, defer):
        opt.zero_grad(lazy=lazy)
        ctx = ops.deferred_wgrad() if defer else None
        if ctx:
            ctx.__enter__()
        for i in range(2):
            torch.manual_seed(100 + i)
            y = model(tok[i, :, :-1])
            ops.cross_entropy(y.reshape(-1, cfg.vocab), tok[i, :, 1:].reshape(-1)).backward()
        if ctx:
            ctx.__exit__(None, None, None)
        opt.fold_grads()
        return torch.cat([g.main_grad.clone() for g in opt.groups])

    for defer in (True, False):
        eager = run(False, defer)
        lazy1 = run(True, defer)
        lazy2 = run(True, defer)
        assert torch.allclose(lazy1, lazy2, atol=1e-5, rtol=1e-4)  # embedding atomics: order-dependent
        assert torch.allclose(lazy1, eager, atol=1e-5, rtol=1e-4)
        assert any(getattr(p, "_mipipe_gemm_weight", False) for p in model.parameters())
