"""Stage planning: which blocks of a model each pipeline rank owns.

Costs are analytic training FLOPs per token of each block (plus a small
memory-traffic term for FLOP-free blocks such as the embedding), so ranks can
decide their slice *before* instantiating anything -- no rank ever builds the
whole 1.2B-parameter model.  The split minimises the slowest stage
(``mipipe.balance.blockpartition``), with stage boundaries allowed between the
attention and MLP halves of a layer.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Tuple

import torch
from torch import nn

from ..balance import balance_cost
from ..models.lm import LMConfig, build_lm_blocks
from ..models.transformer import merge_units, pipeline_units

__all__ = ["StagePlan", "plan_stages", "block_costs", "stage_input_shape", "build_stage"]


@dataclass
class StagePlan:
    balance: List[int]
    costs: List[float]

    def slice(self, rank: int) -> range:
        start = sum(self.balance[:rank])
        return range(start, start + self.balance[rank])

    def stage_cost(self, rank: int) -> float:
        return sum(self.costs[i] for i in self.slice(rank))

    def imbalance(self) -> float:
        """max stage cost / mean stage cost (1.0 = perfect)."""
        per = [self.stage_cost(r) for r in range(len(self.balance))]
        return max(per) / (sum(per) / len(per))


def block_costs(cfg: LMConfig) -> List[float]:
    """Training FLOPs per token of the pipeline units
    ``[Encoder, (attn core, attn out, mlp) x L, (final norm), Decoder]``
    (see ``mipipe.models.transformer.pipeline_units``)."""
    e, f, s, v = cfg.d_model, cfg.dim_feedforward, cfg.seq_len, cfg.vocab
    causal = 0.5 if cfg.causal else 1.0
    core = 3.0 * (2 * 3 * e * e + 4 * s * e * causal) + 3.0 * 10 * e
    out = 3.0 * (2 * e * e) + 3.0 * 10 * e  # + LN/dropout traffic
    mlp = 3.0 * (2 * 2 * e * f) + 3.0 * 20 * e
    enc = 3.0 * 40 * e  # gather + scatter-add traffic, expressed in FLOP-equivalents
    dec = 3.0 * (2 * e * v) + 3.0 * 4 * v  # GEMM + cross-entropy passes
    costs = [enc]
    for _ in range(cfg.num_layers):
        costs += [core, out, mlp]
    if cfg.norm_first:
        costs.append(3.0 * 10 * e)
    costs.append(dec)
    return costs


def plan_stages(cfg: LMConfig, stages: int) -> StagePlan:
    costs = block_costs(cfg)
    return StagePlan(balance_cost(costs, stages), costs)


def unit_is_packed_core(cfg: LMConfig, index: int) -> bool:
    """True if pipeline unit ``index`` is an attention core (packed output)."""
    return 1 <= index <= 3 * cfg.num_layers and (index - 1) % 3 == 0


def stage_input_shape(cfg: LMConfig, plan: StagePlan, rank: int, micro_batch: int) -> Tuple[int, ...]:
    """Shape of the activation stage ``rank`` receives (``[2, mb, S, E]`` after a
    packed attention core, else ``[mb, S, E]``)."""
    base = (micro_batch, cfg.seq_len, cfg.d_model)
    if rank == 0:
        return base
    prev = plan.slice(rank).start - 1
    return (2,) + base if unit_is_packed_core(cfg, prev) else base


def build_stage(cfg: LMConfig, plan: StagePlan, rank: int, *, device, dtype) -> nn.Sequential:
    """Instantiates ONLY this rank's units (on ``device``, in ``dtype``) and
    merges attention halves that ended up on the same stage."""
    with torch.device("meta"):
        proto = pipeline_units(build_lm_blocks(cfg))
    units = []
    for idx in plan.slice(rank):
        u = proto[idx].to_empty(device=device)
        u.reset_parameters()
        units.append(u)
    del proto
    stage = nn.Sequential(*merge_units(units))
    for p in stage.parameters():
        if p.dtype.is_floating_point:
            p.data = p.data.to(dtype)
    return stage
