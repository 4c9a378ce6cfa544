"""Measured-cost stage planning (mipipe.parallel.calibrate): unit kinds timed on
the CPU here -- alone, and in engine context (head / middle / tail stages run by
the PipelineEngine over loop-back channels; the same code times them on the GPU
in bench.py --plan measured) -- costs fed to the planner, and every rank of a
gloo group deriving the same numbers, hence the same plan, whether measured or
read from the cache."""
import dataclasses
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mipipe.models import CONFIGS
from mipipe.parallel.calibrate import (calibrated_costs, engine_unit_costs, measure_engine_costs, measure_unit_times,
                                       unit_costs, unit_kinds)
from mipipe.parallel.stage import block_costs, choose_virtual, plan_stages

CPU = torch.device("cpu")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_measure_unit_times_cpu():
    cfg = CONFIGS["tiny"]
    times = measure_unit_times(cfg, 2, chunks=2, device=CPU, dtype=torch.float32, reps=1)
    kinds = set(unit_kinds(cfg, False)) | set(unit_kinds(cfg, True))
    assert set(times) == kinds
    assert all(f > 0 and b >= 0 for f, b in times.values())
    for split in (False, True):
        costs = unit_costs(cfg, times, split, recompute=1.0)
        assert len(costs) == len(block_costs(cfg, split))
        # recompute prices the forward twice
        base = unit_costs(cfg, times, split, recompute=0.0)
        assert all(c >= b for c, b in zip(costs, base))
        plan = plan_stages(cfg, 2, 1, 4, split, costs=costs)
        assert sum(plan.balance) == len(costs) and plan.costs == costs
    with pytest.raises(ValueError):
        plan_stages(cfg, 2, 1, 4, False, costs=[1.0, 2.0])
    v, plan = choose_virtual(cfg, 2, 4, micro_batch=2, cost_fn=lambda s: unit_costs(cfg, times, s, 0.0))
    assert plan.ranks == 2 and plan.virtual == v


def _cfg3():
    return dataclasses.replace(CONFIGS["tiny"], num_layers=3)


def test_measure_engine_costs_cpu():
    cfg = _cfg3()
    costs = measure_engine_costs(cfg, 2, 4, "except_last", device=CPU, dtype=torch.float32, steps=1)
    kinds = set(unit_kinds(cfg, False)) | set(unit_kinds(cfg, True))
    assert kinds <= set(costs)
    # CPU timings of a tiny model are noisy: differences may clamp to 0, never go negative
    assert all(c >= 0 for c in costs.values()) and sum(costs.values()) > 0
    for split in (False, True):
        plan = plan_stages(cfg, 2, 1, 4, split, costs=engine_unit_costs(cfg, costs, split))
        assert sum(plan.balance) == len(block_costs(cfg, split))


def _worker(rank, port, cache, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MIPIPE_CALIB_DIR=cache)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        cfg = _cfg3()
        out = []
        for refresh in (True, False):  # measured (and cached by rank 0), then read back
            costs = calibrated_costs(cfg, 2, 4, "never", device=CPU, dtype=torch.float32, refresh=refresh,
                                     measure=lambda: measure_engine_costs(cfg, 2, 4, device=CPU,
                                                                          dtype=torch.float32, steps=1))
            v, plan = choose_virtual(cfg, 2, 4, micro_batch=2, cost_fn=lambda s: engine_unit_costs(cfg, costs, s))
            out.append((sorted(costs.items()), v, plan.balance, plan.split_decoder))
            dist.barrier()  # rank 0's cache file exists before the second round
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_calibrated_costs_agree_across_ranks(tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == res[1]  # same costs (all-reduced), same plan, in both rounds
    assert res[0][0] == res[0][1]  # the cached table is what was measured
    assert len(list(tmp_path.iterdir())) == 1


def _fail_worker(rank, port, cache, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MIPIPE_CALIB_DIR=cache)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        from mipipe.parallel.calibrate import CalibrationError

        cfg = _cfg3()

        def measure():
            if rank == 1:
                raise RuntimeError("boom")
            return measure_engine_costs(cfg, 2, 4, device=CPU, dtype=torch.float32, steps=1)

        try:
            calibrated_costs(cfg, 2, 4, "never", device=CPU, dtype=torch.float32, refresh=True, measure=measure)
            q.put((rank, "no error"))
        except CalibrationError as exc:
            dist.barrier()  # both ranks are still in step after the failure
            q.put((rank, str(exc)))
    finally:
        dist.destroy_process_group()


def test_calibration_failure_raises_on_every_rank(tmp_path):
    """One rank's failed measurement makes EVERY rank raise CalibrationError (no rank left in a collective)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fail_worker, args=(r, port, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all("failed on 1 of 2 ranks" in m for m in res.values()), res
    assert "boom" in res[1]
