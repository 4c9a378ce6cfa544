"""Data pipeline, profiling helpers and the example driver."""
import os
import subprocess
import sys

import pytest
import torch

from mipipe.utils import data as D
from mipipe.utils import profiling as P

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_basic_english_tokenizer():
    assert D.basic_english("Hello, World! It's (very) good.") == [
        "hello", ",", "world", "!", "it", "'", "s", "(", "very", ")", "good", ".",
    ]
    assert D.basic_english("a;b:c  \"d\"") == ["a", "b", "c", "d"]


def test_vocab_frequency_order_and_unk():
    lines = ["b a a", "c a b"]
    vocab = D.build_vocab(map(D.basic_english, lines))
    assert vocab.itos[:4] == ["<unk>", "a", "b", "c"]
    assert vocab["zzz"] == 0
    assert vocab(["a", "c", "nope"]) == [1, 3, 0]
    assert vocab.lookup_tokens([2, 1]) == ["b", "a"]


def test_data_process_batchify_get_batch():
    vocab = D.build_vocab([["x", "y", "z"]])
    ids = D.data_process(["x y z", "", "z y x x"], vocab)
    assert ids.tolist() == [vocab[t] for t in "x y z z y x x".split()]

    stream = torch.arange(23)
    b = D.batchify(stream, 4)  # drops the 3 trailing tokens
    assert b.shape == (5, 4)
    assert b[:, 1].tolist() == [5, 6, 7, 8, 9]  # columns are contiguous runs
    data, target = D.get_batch(b, 0, 3)
    assert data.shape == (4, 3)  # batch-first
    assert torch.equal(data, b[0:3].t())
    assert torch.equal(target, b[1:4].reshape(-1))
    # last window is truncated to what remains
    data, target = D.get_batch(b, 3, 3)
    assert data.shape == (4, 1) and target.numel() == 4
    batches = list(D.iter_batches(b, 2))
    assert len(batches) == 2


def test_synthetic_corpus_deterministic():
    a = D.synthetic_corpus(1000, 50, seed=3)
    b = D.synthetic_corpus(1000, 50, seed=3)
    assert torch.equal(a, b)
    assert a.min() >= 0 and a.max() < 50
    # Zipf-like: token 0 is the most frequent
    assert torch.bincount(a, minlength=50).argmax().item() == 0


def test_bubble_fraction_and_timer_cpu():
    assert P.bubble_fraction([80.0, 60.0], 100.0) == pytest.approx(0.3)
    assert P.bubble_fraction([], 10.0) == 0.0
    t = P.StageTimer(torch.device("cpu"))
    with t.span():
        pass
    assert t.busy_ms() == 0.0
    assert P.memory_report([torch.device("cpu")]) == {}
    with P.range("cpu-range"):
        pass


def test_example_driver_runs_on_cpu(tmp_path):
    corpus = tmp_path / "train.txt"
    corpus.write_text("\n".join("the quick brown fox jumps over the lazy dog . " * 8 for _ in range(40)))
    out = subprocess.run(
        [sys.executable, os.path.join(ROOT, "examples", "train_lm.py"), "except_last", "--config", "tiny",
         "--batches", "3", "--batch-size", "4", "--bptt", "16", "--partitions", "3", "--train-file", str(corpus)],
        capture_output=True, text=True, timeout=300, env={**os.environ, "CUDA_VISIBLE_DEVICES": ""},
    )
    assert out.returncode == 0, out.stderr[-2000:]
    assert "Total parameters in model" in out.stdout
    assert out.stdout.count("| batch") == 3


def test_gpu_telemetry_degrades_without_a_gpu():
    """bench.py brackets its timed steps with GpuTelemetry; with no driver (or no
    amdsmi) it must report itself unavailable instead of raising."""
    from mipipe.utils.telemetry import GpuTelemetry

    t = GpuTelemetry(0, period=0.01).start()
    out = t.stop()
    assert isinstance(out, dict) and "available" in out
    if out["available"]:  # a GPU host: the fields the bench JSON documents
        assert "gfxclk_mhz" in out and "samples" in out
    else:
        assert out.get("error")
