"""Plan selection from emulated rank walls (mipipe.parallel.calibrate.select_plan_by_emulation,
stage.candidate_plans / simulate_from_walls): the unit-cost model ranks plans only to ~2-3 %, so
bench.py measures its few best candidates on every rank at once and keeps the fastest
(profiles/plan_table_r5.txt).  CPU: real emulation of a tiny model, and a 2-rank gloo group
that must agree on the pick -- or fall back together when one rank's emulation fails."""
import dataclasses
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mipipe.models import CONFIGS
from mipipe.parallel.calibrate import engine_unit_costs, emulate_rank_ms, select_plan_by_emulation, unit_kinds
from mipipe.parallel.stage import (StagePlan, block_costs, candidate_plans, plan_stages, simulate_from_walls,
                                   simulate_step)

CPU = torch.device("cpu")


def _cfg():
    return dataclasses.replace(CONFIGS["tiny"], num_layers=4)


def _unit_ms(cfg):
    base = {"enc": 0.2, "core": 2.0, "out": 0.8, "mlp_in": 0.8, "mlp_out": 0.8, "norm": 0.1, "dec": 3.0,
            "dec_head": 1.5, "dec_tail": 1.5}
    return {k: base[k] for k in set(unit_kinds(cfg, False)) | set(unit_kinds(cfg, True))}


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_simulate_from_walls_equal_walls_is_the_cost_simulation():
    """Walls proportional to the unit costs reproduce the unit-cost simulation."""
    cfg = _cfg()
    costs = engine_unit_costs(cfg, _unit_ms(cfg), False)
    plan = plan_stages(cfg, 2, 2, 8, False, costs=costs)
    m = 8
    walls = [plan.rank_cost(r) * m for r in range(2)]  # ms per step = per-micro-batch cost x chunks
    t, _ = simulate_from_walls(plan, walls, costs, m, 0, 0.0)
    t_ref, _ = simulate_step([plan.stage_cost(g) for g in range(4)], 2, 2, m, 2.0, deferred_w=1.0 / 3.0,
                             checkpoint_stop=0)
    assert abs(t - t_ref) < 1e-6 * t_ref


def test_candidate_plans_are_valid_and_ranked():
    cfg = _cfg()
    um = _unit_ms(cfg)
    cands = candidate_plans(cfg, 2, 8, 2.0, 2, lambda s: engine_unit_costs(cfg, um, s))
    assert 1 <= len(cands) <= 6
    for p in cands:
        assert sum(p.balance) == len(block_costs(cfg, p.split_decoder))
        assert p.ranks == 2 and all(k >= 1 for k in p.balance)
    assert len({(p.virtual, p.split_decoder, tuple(p.balance)) for p in cands}) == len(cands)


def test_emulate_rank_ms_cpu():
    cfg = _cfg()
    plan = plan_stages(cfg, 2, 1, 2, False)
    for r in range(2):
        assert emulate_rank_ms(cfg, plan, r, 2, 2, "never", device=CPU, dtype=torch.float32, steps=1) > 0


def _worker(rank, port, q, fail):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        cfg = _cfg()
        um = _unit_ms(cfg)
        costs = engine_unit_costs(cfg, um, False)
        cands = [StagePlan(b, costs, 1, False) for b in ([9, 9], [8, 10], [10, 8])]

        def emulate(plan, r):  # candidate [8, 10] is the fastest; rank 1 fails when asked to
            if fail and r == 1:
                raise RuntimeError("boom")
            return {(9, 9): 100.0, (8, 10): 80.0, (10, 8): 120.0}[tuple(plan.balance)] + r

        plan, rep = select_plan_by_emulation(cfg, cands, rank, 8, 2, "never", um, device=CPU, emulate=emulate)
        q.put((rank, list(plan.balance), rep["method"], len(rep["candidates"])))
    finally:
        dist.destroy_process_group()


def _run(fail):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, port, q, fail)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, rest) for r, *rest in (q.get(timeout=300) for _ in range(2)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_select_plan_by_emulation_agrees_across_ranks():
    res = _run(False)
    assert res[0] == res[1]
    assert res[0][0] == [8, 10] and res[0][1].startswith("emulated") and res[0][2] == 3


def test_select_plan_falls_back_together_when_a_rank_fails():
    res = _run(True)
    assert res[0][0] == res[1][0] == [9, 9]  # the model's first candidate on both ranks
    assert all(r[1].startswith("model (emulation failed") and r[2] == 0 for r in res.values())
    assert "boom" in res[1][1]


def _refine_worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        cfg = _cfg()
        um = _unit_ms(cfg)
        costs = engine_unit_costs(cfg, um, False)
        start = plan_stages(cfg, 2, 1, 8, False, costs=costs)
        calls = []

        def emulate(plan, r):  # the unit costs, plus work the cost model does not see on the last rank
            calls.append(tuple(plan.balance))
            return sum(costs[i] for s in plan.vstages(r) for i in plan.slice(s)) * 8 + (30.0 if r == 1 else 0.0)

        plan, rep = select_plan_by_emulation(cfg, [start], rank, 8, 2, "never", um, device=CPU, emulate=emulate)
        assert rep["chosen_balance"] == list(plan.balance)
        q.put((rank, list(start.balance), list(plan.balance), rep["refinement"][0]["moves"], len(calls)))
    finally:
        dist.destroy_process_group()


def test_refinement_moves_units_off_the_slowest_measured_rank():
    """The chosen plan is refined from its measured walls: single units move off the rank the walls show
    slowest (here: extra work on the last rank that the unit costs miss) while the simulated step improves;
    every rank takes the same moves, and a rank re-emulates only when its stages changed."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_refine_worker, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: rest for r, *rest in (q.get(timeout=300) for _ in range(2))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (s0, p0, h0, _), (s1, p1, h1, _) = res[0], res[1]
    assert p0 == p1 and h0 == h1 and s0 == s1
    assert sum(p0) == sum(s0) and all(k >= 1 for k in p0)
    accepted = [h for h in h0 if h.get("accepted")]
    assert accepted and p0[1] < s0[1]  # units left the slow last rank
    walls = [h["rank_walls_ms"] for h in accepted]
    assert max(walls[-1]) < max(walls[0]) or len(walls) == 1
    # each round re-emulated only the two ranks whose stages changed
    assert res[0][3] == 1 + len(h0) and res[1][3] == 1 + len(h0)


def test_move_candidates_looping_plan():
    """Moves for a v=2 plan: only the slowest rank's virtual stages give units, each to an adjacent virtual stage of
    ANOTHER rank, never emptying a stage, and only moves priced to lower the larger of the two walls."""
    from mipipe.parallel.calibrate import _move_candidates

    cfg = _cfg()
    costs = engine_unit_costs(cfg, _unit_ms(cfg), False)
    plan = plan_stages(cfg, 2, 2, 8, False, costs=costs)
    rank_cost = [plan.rank_cost(r) * 8 for r in range(2)]
    walls = [rank_cost[0], rank_cost[1] * 1.5]  # rank 1 measured far slower than its units price
    slow, moves = _move_candidates(plan, walls)
    assert slow == 1 and moves
    for s, nb in moves:
        assert s % 2 == 1 and nb % 2 == 0 and abs(s - nb) == 1 and plan.balance[s] > 1
    # balanced walls: nothing is predicted to help
    _, none = _move_candidates(plan, [100.0, 100.0])
    assert none == []
