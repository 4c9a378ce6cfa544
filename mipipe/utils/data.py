"""Language-model data pipeline.

Re-implements what the reference driver gets from torchtext
(``/root/reference/main.py:76-113``): a ``basic_english`` tokenizer, a vocabulary
with an ``<unk>`` default, ``data_process`` into one long id stream,
``batchify`` into ``[L / bsz, bsz]`` columns and ``get_batch`` windows of
``bptt`` tokens returned batch-first (the layout ``Pipe`` splits on dim 0).

There is no network access, so WikiText-2 cannot be downloaded; corpora come
from local text files, or :func:`synthetic_corpus` generates a deterministic
token stream of the same vocabulary size (28,782 for WikiText-2).
"""
from __future__ import annotations

import re
from collections import Counter
from typing import Dict, Iterable, Iterator, List, Optional, Sequence, Tuple

import torch
from torch import Tensor

__all__ = [
    "basic_english",
    "Vocab",
    "build_vocab",
    "data_process",
    "batchify",
    "get_batch",
    "iter_batches",
    "synthetic_corpus",
    "read_lines",
    "WIKITEXT2_VOCAB",
]

WIKITEXT2_VOCAB = 28782  # derived from the reference's parameter count

# torchtext's basic_english normalisation rules, re-derived.
_PATTERNS = [
    (re.compile(r"\'"), " '  "),
    (re.compile(r"\""), ""),
    (re.compile(r"\."), " . "),
    (re.compile(r"<br \/>"), " "),
    (re.compile(r","), " , "),
    (re.compile(r"\("), " ( "),
    (re.compile(r"\)"), " ) "),
    (re.compile(r"\!"), " ! "),
    (re.compile(r"\?"), " ? "),
    (re.compile(r"\;"), " "),
    (re.compile(r"\:"), " "),
    (re.compile(r"\s+"), " "),
]


def basic_english(line: str) -> List[str]:
    """Lower-cases, splits punctuation off and tokenises on whitespace."""
    line = line.lower()
    for pattern, repl in _PATTERNS:
        line = pattern.sub(repl, line)
    return line.split()


class Vocab:
    """Token <-> id map with a default index for unknown tokens."""

    def __init__(self, itos: Sequence[str], default: Optional[str] = "<unk>") -> None:
        self.itos: List[str] = list(itos)
        self.stoi: Dict[str, int] = {t: i for i, t in enumerate(self.itos)}
        self.default_index = self.stoi.get(default, None) if default is not None else None

    def set_default_index(self, index: int) -> None:
        self.default_index = index

    def __len__(self) -> int:
        return len(self.itos)

    def __getitem__(self, token: str) -> int:
        idx = self.stoi.get(token)
        if idx is None:
            if self.default_index is None:
                raise KeyError(token)
            return self.default_index
        return idx

    def __call__(self, tokens: Iterable[str]) -> List[int]:
        return [self[t] for t in tokens]

    def lookup_tokens(self, ids: Iterable[int]) -> List[str]:
        return [self.itos[i] for i in ids]


def build_vocab(token_iter: Iterable[List[str]], specials: Sequence[str] = ("<unk>",), min_freq: int = 1) -> Vocab:
    """Vocabulary ordered by descending frequency, ties by first appearance."""
    counts: Counter = Counter()
    for toks in token_iter:
        counts.update(toks)
    ordered = [t for t, c in sorted(counts.items(), key=lambda kv: -kv[1]) if c >= min_freq and t not in specials]
    return Vocab(list(specials) + ordered, default=specials[0] if specials else None)


def read_lines(path: str) -> Iterator[str]:
    with open(path, "r", encoding="utf-8") as f:
        for line in f:
            yield line


def data_process(lines: Iterable[str], vocab: Vocab, tokenizer=basic_english) -> Tensor:
    """All non-empty lines -> one flat int64 id tensor (``main.py:82-84``)."""
    pieces = [torch.tensor(vocab(tokenizer(line)), dtype=torch.long) for line in lines]
    pieces = [p for p in pieces if p.numel() > 0]
    return torch.cat(pieces) if pieces else torch.zeros(0, dtype=torch.long)


def batchify(data: Tensor, bsz: int, device: Optional[torch.device] = None) -> Tensor:
    """``[L] -> [L // bsz, bsz]``: bsz independent columns (``main.py:92-99``)."""
    nbatch = data.size(0) // bsz
    data = data.narrow(0, 0, nbatch * bsz)
    data = data.view(bsz, -1).t().contiguous()
    return data.to(device) if device is not None else data


def get_batch(source: Tensor, i: int, bptt: int) -> Tuple[Tensor, Tensor]:
    """Rows ``i .. i+bptt`` as a batch-first ``[bsz, seq]`` input and the flat
    next-token targets in the same (seq-major) order as the reference
    (``main.py:108-113``)."""
    seq_len = min(bptt, len(source) - 1 - i)
    data = source[i : i + seq_len]
    target = source[i + 1 : i + 1 + seq_len].reshape(-1)
    return data.t(), target


def iter_batches(source: Tensor, bptt: int, max_batches: Optional[int] = None) -> Iterator[Tuple[Tensor, Tensor]]:
    n = 0
    for i in range(0, source.size(0) - 1, bptt):
        if max_batches is not None and n >= max_batches:
            return
        yield get_batch(source, i, bptt)
        n += 1


def synthetic_corpus(num_tokens: int, vocab_size: int = WIKITEXT2_VOCAB, seed: int = 0) -> Tensor:
    """Deterministic Zipf-like token stream (stand-in for WikiText-2)."""
    g = torch.Generator().manual_seed(seed)
    ranks = torch.arange(1, vocab_size + 1, dtype=torch.float64)
    probs = 1.0 / ranks
    probs /= probs.sum()
    return torch.multinomial(probs, num_tokens, replacement=True, generator=g)
