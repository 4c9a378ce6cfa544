"""Stream-race checker (mipipe.debug): scheduled vs serialised runs.

On CPU the streams are no-ops, so both runs must agree exactly; a module whose
result changes between the runs stands in for a race and must be flagged.  The
engine form runs over gloo with two ranks; the GPU forms are in
tests/test_gpu_pipeline.py."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from torch import nn

from mipipe import Pipe
from mipipe.debug import RaceReport, check_engine, check_pipe

from test_engine import _data, _free_port, _loss_fn, _tiny


def _model(p=0.3):
    torch.manual_seed(0)
    return nn.Sequential(nn.Linear(16, 32), nn.Dropout(p), nn.ReLU(), nn.Linear(32, 32), nn.Dropout(p), nn.Linear(32, 8))


@pytest.mark.parametrize("checkpoint", ["never", "except_last", "always"])
def test_check_pipe_agrees_on_cpu(checkpoint):
    pipe = Pipe(_model(), chunks=4, checkpoint=checkpoint)  # CPU: one partition per child
    x = torch.randn(8, 16)
    rep = check_pipe(pipe, x)
    assert rep.ok and rep.worst()[1] == 0.0, rep.max_rel
    assert "output" in rep.max_rel and any(k.startswith("grad ") for k in rep.max_rel)
    # the serialised configuration is undone afterwards
    assert pipe.pipeline.sync_debug is (os.environ.get("MIPIPE_SYNC_DEBUG") == "1")


class _Flaky(nn.Module):
    """Adds the call count: the second (serialised) run differs, as a race would."""

    def __init__(self):
        super().__init__()
        self.calls = 0

    def forward(self, x):
        self.calls += 1
        return x + (self.calls > 4)


def test_check_pipe_flags_a_difference():
    torch.manual_seed(0)
    model = nn.Sequential(nn.Linear(4, 4), _Flaky(), nn.Linear(4, 4))
    pipe = Pipe(model, chunks=4)
    rep = check_pipe(pipe, torch.randn(8, 4))
    assert not rep.ok
    with pytest.raises(RuntimeError, match="stream race suspected"):
        rep.raise_if_failed()


def test_race_report():
    rep = RaceReport({"a": 0.0, "b": 2e-3}, tol=1e-3)
    assert not rep.ok and rep.worst() == ("b", 2e-3)
    assert RaceReport({"a": 1e-7}).ok


def _engine_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mipipe.models import TargetSequential, build_lm_blocks, lm_pipeline_units
        from mipipe.models.transformer import merge_units
        from mipipe.optim import FlatAdam
        from mipipe.parallel import PipelineEngine, plan_stages
        from mipipe.parallel.stage import stage_input_shape

        cfg = _tiny(dropout=0.2)
        m, mb = 4, 2
        torch.manual_seed(0)
        units = lm_pipeline_units(build_lm_blocks(cfg))
        plan = plan_stages(cfg, world, 1)
        stage = TargetSequential(*merge_units([units[i] for i in plan.slice(rank)])).train()
        FlatAdam(stage.parameters(), lr=1e-3)  # main_grad buffers, as in training
        eng = PipelineEngine(stage, chunks=m, checkpoint="except_last", act_shape=stage_input_shape(cfg, plan, rank, mb),
                             act_dtype=torch.float32, loss_fn=_loss_fn(cfg) if rank == world - 1 else None,
                             device=torch.device("cpu"))
        inputs, targets = _data(cfg, m, mb)
        torch.manual_seed(5)
        rep = check_engine(eng, inputs if rank == 0 else None, targets)
        q.put((rank, rep.ok, rep.worst(), sorted(rep.max_rel), eng.sync_debug))
    finally:
        dist.destroy_process_group()


def test_check_engine_two_ranks_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_engine_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok, worst, keys, sync_after in res:
        assert ok, (rank, worst)
        assert any(k.startswith("grad ") for k in keys)
        assert sync_after is False
    assert "loss" in res[1][3]  # the last stage compares the loss too
