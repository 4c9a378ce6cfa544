"""Training-state save / resume (mipipe.utils.checkpoint_io): a run resumed from
a checkpoint is bit-identical to the uninterrupted run -- weights, Adam
moments, step count and the dropout RNG -- through the Pipe."""
import dataclasses

import pytest
import torch

import mipipe
from mipipe.models import CONFIGS, build_lm_blocks
from mipipe.ops import cross_entropy
from mipipe.optim import FlatAdam
from mipipe.utils.checkpoint_io import load_training_state, load_weights, rank_path, save_training_state


def _cfg():
    return dataclasses.replace(CONFIGS["tiny"], num_layers=2, d_model=32, nhead=4, dim_feedforward=64, vocab=100,
                               seq_len=8, dropout=0.2)


def _pipe(seed, device="cpu", dtype=torch.float32):
    torch.manual_seed(seed)
    blocks = build_lm_blocks(_cfg())
    seq = torch.nn.Sequential(torch.nn.Sequential(*blocks[:3]).to(device, dtype),
                              torch.nn.Sequential(*blocks[3:]).to(device, dtype))
    return mipipe.Pipe(seq, chunks=2, checkpoint="except_last", return_rref=False)


def _batches(n):
    g = torch.Generator().manual_seed(5)
    tok = torch.randint(0, 100, (n, 4, 9), generator=g)
    return [(tok[i, :, :8], tok[i, :, 1:]) for i in range(n)]


def _step(pipe, opt, x, t, flat):
    opt.zero_grad()
    dev = next(pipe.parameters()).device
    loss = cross_entropy(pipe(x.to(dev)).reshape(-1, 100), t.to(dev).reshape(-1))
    loss.backward()
    if not flat:
        torch.nn.utils.clip_grad_norm_(pipe.parameters(), 0.5)
    opt.step()
    return float(loss.detach())


def _resume_case(tmp_path, flat, device="cpu", dtype=torch.float32):
    data = _batches(4)

    def make(seed):
        pipe = _pipe(seed, device, dtype)
        opt = (FlatAdam(pipe.parameters(), lr=1e-2, max_grad_norm=0.5) if flat
               else torch.optim.Adam(pipe.parameters(), lr=1e-2))
        return pipe, opt

    pipe, opt = make(0)
    for x, t in data[:2]:
        _step(pipe, opt, x, t, flat)
    path = rank_path(str(tmp_path), 0)
    save_training_state(path, pipe.named_parameters(), opt, step=2, extra={"note": "after 2"})
    tail = [_step(pipe, opt, x, t, flat) for x, t in data[2:]]
    final = {n: p.detach().clone() for n, p in pipe.named_parameters()}

    pipe2, opt2 = make(1)  # different initial weights: everything must come from the file
    meta = load_training_state(path, pipe2.named_parameters(), opt2)
    assert meta["step"] == 2 and meta["extra"] == {"note": "after 2"}
    tail2 = [_step(pipe2, opt2, x, t, flat) for x, t in data[2:]]
    assert tail == tail2
    for n, p in pipe2.named_parameters():
        assert torch.equal(p, final[n]), n


@pytest.mark.parametrize("flat", [True, False])
def test_resume_is_bit_identical(tmp_path, flat):
    _resume_case(tmp_path, flat)


@pytest.mark.gpu
def test_resume_is_bit_identical_gpu(tmp_path):
    """On the MI355X: bf16 HIP kernels, dropout masks from the restored HIP
    generator (Philox seed/offset), FlatAdam's fused kernel."""
    _resume_case(tmp_path, True, "cuda:0", torch.bfloat16)


def test_load_weights_and_layout_check(tmp_path):
    pipe = _pipe(0)
    opt = FlatAdam(pipe.parameters(), lr=1e-2)
    path = str(tmp_path / "ck.safetensors")
    save_training_state(path, pipe.named_parameters(), opt)
    other = _pipe(1)
    load_weights(path, other.named_parameters())
    for (n, a), (_, b) in zip(pipe.named_parameters(), other.named_parameters()):
        assert torch.equal(a, b), n
    # an optimizer over a different parameter order is refused, not silently scrambled
    params = list(other.parameters())
    bad = FlatAdam(params[::-1], lr=1e-2)
    with pytest.raises(ValueError, match="layout"):
        load_training_state(path, other.named_parameters(), bad)
    with pytest.raises(ValueError, match="not a"):
        from safetensors.torch import save_file

        save_file({"x": torch.zeros(1)}, str(tmp_path / "foreign.safetensors"))
        load_weights(str(tmp_path / "foreign.safetensors"), other.named_parameters())


def test_rng_restores_onto_loaders_own_gpu(tmp_path, monkeypatch):
    """A file saved by a replica on cuda:0 restores the GPU generator of a
    replica whose parameters live on cuda:4: keys are positions
    among the rank's parameter devices, not device indices."""
    import mipipe.utils.checkpoint_io as cio

    lin = torch.nn.Linear(4, 4)
    states = {0: torch.arange(16, dtype=torch.uint8), 4: torch.zeros(16, dtype=torch.uint8)}
    restored = {}
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "get_rng_state", lambda d: states[d].clone())
    monkeypatch.setattr(torch.cuda, "set_rng_state", lambda st, d: restored.__setitem__(d, st.clone()))
    monkeypatch.setattr(cio, "_cuda_devices", lambda params: [0])
    path = rank_path(str(tmp_path), 0)
    save_training_state(path, lin.named_parameters(), None)
    monkeypatch.setattr(cio, "_cuda_devices", lambda params: [4])
    load_training_state(path, lin.named_parameters(), None)
    assert list(restored) == [4]
    assert torch.equal(restored[4], states[0])
    monkeypatch.setattr(cio, "_cuda_devices", lambda params: [4, 5])
    with pytest.raises(ValueError, match="RNG states for 1 GPU"):
        load_training_state(path, lin.named_parameters(), None)


def test_refused_load_leaves_state_untouched(tmp_path, monkeypatch):
    """every check that can refuse a file (RNG device count, optimizer
    layout, weight shapes) runs before anything is overwritten; parameters on no
    GPU skip the GPU generators with a warning instead of raising."""
    import mipipe.utils.checkpoint_io as cio

    lin = torch.nn.Linear(4, 4)
    states = {0: torch.arange(16, dtype=torch.uint8)}
    restored = {}
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "get_rng_state", lambda d: states[d].clone())
    monkeypatch.setattr(torch.cuda, "set_rng_state", lambda st, d: restored.__setitem__(d, st.clone()))
    monkeypatch.setattr(cio, "_cuda_devices", lambda params: [0])
    path = rank_path(str(tmp_path), 0)
    save_training_state(path, lin.named_parameters(), None)
    other = torch.nn.Linear(4, 4)
    before = [p.detach().clone() for p in other.parameters()]
    cpu_before = torch.get_rng_state()
    monkeypatch.setattr(cio, "_cuda_devices", lambda params: [0, 1])
    with pytest.raises(ValueError, match="RNG states for 1 GPU"):
        load_training_state(path, other.named_parameters(), None)
    assert all(torch.equal(a, b) for a, b in zip(before, other.parameters()))
    assert torch.equal(torch.get_rng_state(), cpu_before) and not restored
    monkeypatch.setattr(cio, "_cuda_devices", lambda params: [])
    with pytest.warns(UserWarning, match="no GPU"):
        load_training_state(path, other.named_parameters(), None)
    assert all(torch.equal(a, b) for a, b in zip(lin.parameters(), other.parameters()))
    assert not restored


def test_truncated_optimizer_state_leaves_the_model_untouched(tmp_path):
    """A file whose FlatAdam buffers are missing is refused BEFORE any parameter
    is overwritten (the parameters used to be copied first)."""
    from safetensors.torch import load_file, save_file

    pipe = _pipe(0)
    opt = FlatAdam(pipe.parameters(), lr=1e-2)
    path = str(tmp_path / "ck.safetensors")
    save_training_state(path, pipe.named_parameters(), opt)
    t = load_file(path)
    from safetensors import safe_open

    with safe_open(path, "pt") as f:
        meta = f.metadata()
    del t["flat.0.exp_avg"]
    cut = str(tmp_path / "cut.safetensors")
    save_file(t, cut, metadata=meta)
    other = _pipe(1)
    before = [p.detach().clone() for p in other.parameters()]
    opt2 = FlatAdam(other.parameters(), lr=1e-2)
    with pytest.raises(KeyError, match="flat.0.exp_avg"):
        load_training_state(cut, other.named_parameters(), opt2)
    for a, b in zip(before, other.parameters()):
        assert torch.equal(a, b)
