"""Training-state save / resume.

The reference has no model or optimizer checkpointing ("checkpoint" there
always means activation checkpointing); a production pipeline needs it.  One
file per pipeline rank (each rank owns only its stages' parameters -- nothing
is gathered), in safetensors, whose loader executes nothing from the file:

* ``param.<name>``                    -- the model weights in their dtype (a plain
  inference checkpoint: :func:`load_weights` needs nothing else);
* ``flat.<g>.{master,exp_avg,exp_avg_sq}`` -- :class:`mipipe.optim.FlatAdam`'s
  fp32 flat buffers, saved as the contiguous device buffers they are (one
  tensor each, no per-parameter split), with the parameter layout in the
  metadata so a resume into a different partition fails loudly instead of
  scrambling moments;
* ``adam.<name>.{exp_avg,exp_avg_sq,step}`` -- ``torch.optim.Adam`` state;
* ``rng.cpu`` / ``rng.cuda.local.<k>`` -- generator states, so dropout masks
  after a resume are the ones the uninterrupted run would have drawn (the HIP
  dropout kernels take their Philox seed/offset from the torch generator).
  ``k`` is the position of the GPU among this rank's parameter devices (sorted),
  so a file saved by a replica on cuda:0 restores onto a replica on cuda:4.

A resumed run is bit-identical to the uninterrupted one
(``tests/test_checkpoint_io.py``).  Data-parallel replicas hold identical
state: save from replica 0 only and load the same file everywhere.
"""
from __future__ import annotations

import json
import os
import warnings
from typing import Dict, Iterable, Optional, Tuple

import torch
from torch import Tensor, nn

__all__ = ["save_training_state", "load_training_state", "load_weights", "rank_path"]

FORMAT = "mipipe-train-state/1"


def rank_path(directory: str, rank: int) -> str:
    """``<directory>/rank00003.safetensors``: one file per pipeline rank."""
    return os.path.join(directory, f"rank{rank:05d}.safetensors")


def _host(t: Tensor) -> Tensor:
    t = t.detach()
    return t.to("cpu") if t.device.type != "cpu" else t.clone()


def _cuda_devices(params: Iterable[nn.Parameter]) -> list:
    """Sorted indices of the GPUs holding ``params``."""
    return sorted({p.device.index if p.device.index is not None else torch.cuda.current_device()
                   for p in params if p.device.type == "cuda"})


def _named(params: Iterable[Tuple[str, nn.Parameter]]) -> Dict[str, nn.Parameter]:
    out: Dict[str, nn.Parameter] = {}
    for name, p in params:
        if name in out:
            raise ValueError(f"duplicate parameter name {name!r}")
        out[name] = p
    return out


def save_training_state(path: str, named_params: Iterable[Tuple[str, nn.Parameter]], optimizer=None, *,
                        step: int = 0, extra: Optional[dict] = None, rng: bool = True) -> None:
    """Writes this rank's weights, optimizer state and RNG state to ``path``.

    ``named_params``: e.g. ``stage.named_parameters()``; ``optimizer``: a
    :class:`~mipipe.optim.FlatAdam`, a ``torch.optim.Adam``/``AdamW`` or None."""
    from safetensors.torch import save_file

    from ..optim import FlatAdam

    params = _named(named_params)
    by_id = {id(p): n for n, p in params.items()}
    if isinstance(optimizer, FlatAdam):
        optimizer.wait_step()  # an overlapped step may still be writing the weights and the moments
    tensors: Dict[str, Tensor] = {f"param.{n}": _host(p) for n, p in params.items()}
    meta = {"format": FORMAT, "step": int(step), "extra": extra or {}}
    if isinstance(optimizer, FlatAdam):
        layout = []
        for gi, g in enumerate(optimizer.groups):
            layout.append([[by_id.get(id(p), "?"), list(p.shape)] for p in g.params])
            tensors[f"flat.{gi}.master"] = _host(g.master)
            tensors[f"flat.{gi}.exp_avg"] = _host(g.exp_avg)
            tensors[f"flat.{gi}.exp_avg_sq"] = _host(g.exp_avg_sq)
        meta["optimizer"] = {"kind": "FlatAdam", "step": optimizer.step_count, "lr": optimizer.lr,
                             "layout": layout}
    elif isinstance(optimizer, torch.optim.Optimizer):
        kinds = {}
        for p, st in optimizer.state.items():
            n = by_id.get(id(p))
            if n is None:
                raise ValueError("optimizer holds a parameter missing from named_params")
            for k, v in st.items():
                if torch.is_tensor(v):
                    tensors[f"adam.{n}.{k}"] = _host(v).reshape(v.shape)
                    kinds[k] = True
        meta["optimizer"] = {"kind": type(optimizer).__name__,
                             "lr": [g["lr"] for g in optimizer.param_groups]}
    elif optimizer is not None:
        raise TypeError(f"unsupported optimizer {type(optimizer).__name__}")
    if rng:
        tensors["rng.cpu"] = torch.get_rng_state()
        if torch.cuda.is_available():
            # keyed by position among this rank's parameter devices, not by
            # device index: a replica on another GPU (cuda:4+s for stage s)
            # restores the state onto ITS k-th device
            for k, d in enumerate(_cuda_devices(params.values())):
                tensors[f"rng.cuda.local.{k}"] = torch.cuda.get_rng_state(d)
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    tmp = path + ".tmp"
    save_file({k: v.contiguous() for k, v in tensors.items()}, tmp, metadata={"mipipe": json.dumps(meta)})
    os.replace(tmp, path)  # a crash mid-save never leaves a torn checkpoint behind


def _read(path: str):
    from safetensors import safe_open
    from safetensors.torch import load_file

    with safe_open(path, framework="pt") as f:
        meta = json.loads((f.metadata() or {}).get("mipipe", "{}"))
    if meta.get("format") != FORMAT:
        raise ValueError(f"{path}: not a {FORMAT} file")
    return load_file(path), meta


@torch.no_grad()
def load_weights(path: str, named_params: Iterable[Tuple[str, nn.Parameter]]) -> None:
    """Copies the saved weights into ``named_params`` (every name must be present)."""
    tensors, _ = _read(path)
    for n, p in _named(named_params).items():
        key = f"param.{n}"
        if key not in tensors:
            raise KeyError(f"{path}: no weights for {n!r}")
        if tuple(tensors[key].shape) != tuple(p.shape):
            raise ValueError(f"{path}: {n!r} is {tuple(tensors[key].shape)}, the model has {tuple(p.shape)}")
        p.copy_(tensors[key])


@torch.no_grad()
def load_training_state(path: str, named_params: Iterable[Tuple[str, nn.Parameter]], optimizer=None, *,
                        rng: bool = True) -> dict:
    """Restores what :func:`save_training_state` wrote; returns its metadata
    (``step``, ``extra``).  The optimizer must be built over the same
    parameters in the same order (FlatAdam layouts are checked)."""
    from ..optim import FlatAdam

    params = _named(named_params)
    tensors, meta = _read(path)
    # Every check that can refuse the file runs BEFORE anything is overwritten,
    # so a refused load leaves the model, optimizer and RNG untouched.
    cuda_rng = []  # (device, key) pairs to restore
    if rng and "rng.cpu" in tensors and torch.cuda.is_available():
        local = sorted((int(k.rsplit(".", 1)[1]), k) for k in tensors if k.startswith("rng.cuda.local."))
        if not local:  # files written before the device-independent keys: by saved index order
            local = sorted((int(k.rsplit(".", 1)[1]), k) for k in tensors if k.startswith("rng.cuda."))
        mine = _cuda_devices(params.values())
        if local and not mine:
            warnings.warn(f"{path}: the file holds GPU RNG states but this rank's parameters are on no GPU; "
                          f"the GPU generators are left as they are")
        elif len(local) != len(mine):
            raise ValueError(f"{path}: RNG states for {len(local)} GPU(s), this rank's parameters are on "
                             f"{len(mine)}")
        else:
            cuda_rng = [(d, key) for d, (_, key) in zip(mine, local)]
    opt_meta = meta.get("optimizer")
    if isinstance(optimizer, FlatAdam):
        if not opt_meta or opt_meta.get("kind") != "FlatAdam":
            raise ValueError(f"{path}: no FlatAdam state")
        by_id = {id(p): n for n, p in params.items()}
        layout = [[[by_id.get(id(p), "?"), list(p.shape)] for p in g.params] for g in optimizer.groups]
        if layout != opt_meta["layout"]:
            raise ValueError(f"{path}: the optimizer's parameter layout differs from the saved one "
                             f"(a different partition or model)")
        for gi, g in enumerate(optimizer.groups):  # the flat buffers: present and of the group's size
            for part in ("master", "exp_avg", "exp_avg_sq"):
                key = f"flat.{gi}.{part}"
                if key not in tensors:
                    raise KeyError(f"{path}: no {key} (a truncated or foreign file)")
                if tuple(tensors[key].shape) != tuple(g.master.shape):
                    raise ValueError(f"{path}: {key} is {tuple(tensors[key].shape)}, the optimizer's is "
                                     f"{tuple(g.master.shape)}")
    elif isinstance(optimizer, torch.optim.Optimizer):
        owned = {id(v) for v in params.values()}
        stray = sum(1 for grp in optimizer.param_groups for q in grp["params"] if id(q) not in owned)
        if stray:
            raise ValueError(f"{path}: {stray} optimizer parameter(s) are not among the model's parameters")
    for n, p in params.items():
        key = f"param.{n}"
        if key not in tensors:
            raise KeyError(f"{path}: no weights for {n!r}")
        if tuple(tensors[key].shape) != tuple(p.shape):
            raise ValueError(f"{path}: {n!r} is {tuple(tensors[key].shape)}, the model has {tuple(p.shape)}")
    if isinstance(optimizer, FlatAdam):
        optimizer.wait_step()
    for n, p in params.items():
        p.copy_(tensors[f"param.{n}"])
    if isinstance(optimizer, FlatAdam):
        for gi, g in enumerate(optimizer.groups):
            g.master.copy_(tensors[f"flat.{gi}.master"])
            g.exp_avg.copy_(tensors[f"flat.{gi}.exp_avg"])
            g.exp_avg_sq.copy_(tensors[f"flat.{gi}.exp_avg_sq"])
            if g.master is not g.model:
                g.model.copy_(g.master)
        optimizer.step_count = int(opt_meta["step"])
        optimizer.lr = float(opt_meta["lr"])
    elif isinstance(optimizer, torch.optim.Optimizer):
        for p in (q for grp in optimizer.param_groups for q in grp["params"]):
            n = next(k for k, v in params.items() if v is p)
            st = {}
            for key in [k for k in tensors if k.startswith(f"adam.{n}.")]:
                st[key[len(f"adam.{n}."):]] = tensors[key].to(p.device if key.split(".")[-1] != "step" else "cpu")
            if st:
                optimizer.state[p] = st
        for grp, lr in zip(optimizer.param_groups, (opt_meta or {}).get("lr", [])):
            grp["lr"] = lr
    if rng and "rng.cpu" in tensors:
        torch.set_rng_state(tensors["rng.cpu"])
        for d, key in cuda_rng:
            torch.cuda.set_rng_state(tensors[key], d)
    return {"step": meta.get("step", 0), "extra": meta.get("extra", {})}
