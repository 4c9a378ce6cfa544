"""bench.py contract: one JSON line with the driver's fields, single and multi-rank.

Runs the CPU plumbing mode (``--device cpu``: gloo + fp32, tiny model) so the
torchrun launch, barriers, max-over-ranks timing and the rank-0 JSON line are
exercised here; the GPU/RCCL numbers come from the MI355X runs."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REQUIRED = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config"}


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


# (extra args, expected plan fields)
CASES = [
    (1, [], {}),
    (2, [], {}),
    (2, ["--chunks-per-rank", "1", "--checkpoint", "always"], {"virtual_chunks_per_rank": 1, "checkpoint": "always"}),
    (3, ["--skips", "unet", "--chunks-per-rank", "1"], {"virtual_chunks_per_rank": 1}),
    # the full-node plan shape forced on 4 ranks: looping stages, split LM head, except_last
    (4, ["--split-decoder", "on", "--chunks-per-rank", "2", "--checkpoint", "except_last"],
     {"virtual_chunks_per_rank": 2, "vocab_split_decoder": True, "checkpoint": "except_last"}),
    # 8 ranks in the plan shape the planner picks for enc12_d4096 at PP=8 (2 chunks per rank, split head,
    # except_last at 32 micro-batches; test_default_pp8_plan_matches_enc12) -- forced, since the tiny model
    # itself is launch-bound and plans one chunk per rank
    (8, ["--num-layers", "4", "--chunks-per-rank", "2", "--split-decoder", "on"],
     {"virtual_chunks_per_rank": 2, "vocab_split_decoder": True, "checkpoint": "except_last", "chunks": 32}),
    # the IPC-link transport (host-mode links on CPU): looping placement over shared-memory slot rings
    (4, ["--transport", "ipc", "--chunks-per-rank", "2", "--split-decoder", "on"],
     {"transport": "ipc", "virtual_chunks_per_rank": 2}),
]


def test_default_pp8_plan_matches_enc12():
    """The 8-rank contract case stands for the enc12_d4096 PP=8 plan."""
    import dataclasses

    from mipipe.models import CONFIGS
    from mipipe.parallel.stage import choose_virtual

    ck = 2.0 + 31 / 32
    v, plan = choose_virtual(CONFIGS["enc12_d4096"], 8, 32, bwd_ratio=ck, micro_batch=64)
    assert (v, plan.split_decoder) == (2, True)
    # a tiny model is launch-bound: the boundary/launch terms keep it on one chunk per rank
    tv, _ = choose_virtual(dataclasses.replace(CONFIGS["tiny"], num_layers=4), 8, 32, bwd_ratio=ck, micro_batch=2)
    assert tv == 1


@pytest.mark.parametrize("nproc,extra,expect", CASES)
def test_bench_json_contract(nproc, extra, expect):
    args = ["--gpus", str(nproc), "--steps", "2", "--warmup", "1", "--device", "cpu", "--config", "tiny",
            "--micro-batch", "2"] + extra
    if nproc == 1:
        cmd = [sys.executable, os.path.join(ROOT, "bench.py")] + args
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "bench.py")] + args
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd="/tmp",
                         env={**os.environ, "CUDA_VISIBLE_DEVICES": ""})
    assert out.returncode == 0, out.stderr[-3000:]
    lines = _json_lines(out.stdout)
    assert len(lines) == 1, out.stdout  # rank 0 only, exactly one line
    rec = lines[0]
    assert REQUIRED <= set(rec)
    assert rec["n_gpus"] == nproc and rec["steps"] == 2 and rec["warmup"] == 1
    assert rec["value"] > 0 and rec["higher_is_better"] is True and rec["scaling"] == "weak"
    # weak scaling means the same tokens per GPU per step as the N = 1 run of the same flags (chunks 4 x N)
    assert rec["config"]["tokens_per_gpu_per_step"] == 4 * rec["config"]["micro_batch"] * rec["config"]["seq_len"]
    # start-up breakdown, and (N > 1) the PP = 1 rate at this run's micro-batch / checkpoint
    su = rec["startup_s"]
    assert su["total_before_timed_steps"] >= su["warmup_steps"] >= 0 and su["process_init"] >= 0
    if nproc > 1:
        lfl = rec["like_for_like"]
        assert lfl["micro_batch"] == rec["config"]["micro_batch"] and lfl["checkpoint"] == rec["config"]["checkpoint"]
        assert "pp1_tokens_per_s" in lfl and lfl["source"]
        assert "transport" in su or "--skips" in extra  # with skips the engine builds its links itself
    else:
        assert rec["like_for_like"] is None
    cfg = rec["config"]
    assert {"model", "global_batch", "seq_len", "parallelism"} <= set(cfg)
    assert cfg["parallelism"] == f"pp{nproc}"
    assert cfg["global_batch"] == cfg["chunks"] * cfg["micro_batch"]
    tokens = cfg["global_batch"] * cfg["seq_len"]
    assert abs(rec["value"] - tokens / (rec["ms_per_step"] / 1e3)) / rec["value"] < 0.01
    assert rec["loss"] is not None and rec["loss"] > 0
    for k, v in expect.items():
        assert cfg[k] == v, (k, cfg[k], v)
    # metrics: per-GPU / per-stage lists (None on the CPU plumbing run), both bubble models
    assert rec["peak_hbm_gib_per_gpu"] is None and rec["stage_busy_ms"] is None
    assert rec["bubble_gpipe_v1_pct"] == pytest.approx(100.0 * (nproc - 1) / (cfg["chunks"] + nproc - 1), abs=0.01)
    v = cfg["virtual_chunks_per_rank"]
    assert rec["bubble_theory_pct"] == pytest.approx(100.0 * (nproc - 1) / (v * cfg["chunks"] + nproc - 1), abs=0.01)
    assert rec["vs_baseline"] is None  # not the reference's config
    # the communicators as the job saw them (a multi-GPU JSON checks itself against these)
    comm = rec["comm"]
    assert comm["world_size"] == nproc and [r["rank"] for r in comm["per_rank"]] == list(range(nproc))
    assert comm["rccl_version"] and comm["backend"] == (None if nproc == 1 else "gloo")
    if extra[:2] != ["--transport", "ipc"] and "ipc" not in extra:
        v = cfg["virtual_chunks_per_rank"]
        links = 2 * (nproc if v > 1 else nproc - 1)  # activation + gradient direction per pipeline link
        assert comm["pipeline_links"] == links and comm["pipeline_links_warmed"] == links
        for r in comm["per_rank"]:
            for c in r["channels"]:
                assert c["group_world"] == 2 and c["backend"] == "gloo" and c["warmed"]


def test_bench_pipe_impl_cpu():
    """--impl pipe: the single-process Pipe path emits the same contract."""
    args = ["--impl", "pipe", "--gpus", "2", "--steps", "2", "--warmup", "1", "--device", "cpu", "--config", "tiny",
            "--micro-batch", "2"]
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                         timeout=600, cwd="/tmp", env={**os.environ, "CUDA_VISIBLE_DEVICES": ""})
    assert out.returncode == 0, out.stderr[-3000:]
    (rec,) = _json_lines(out.stdout)
    assert REQUIRED <= set(rec) and rec["config"]["impl"].startswith("pipe")
    assert rec["n_gpus"] == 2 and rec["config"]["chunks"] == 8 and rec["value"] > 0


def test_vs_baseline_only_on_reference_config():
    import argparse
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    from mipipe.models import CONFIGS

    ns = argparse.Namespace(dtype="fp32", checkpoint="never")
    assert bench.matches_reference(CONFIGS["ref_main"], ns, 4, 8)
    assert not bench.matches_reference(CONFIGS["ref_main"], argparse.Namespace(dtype="bf16", checkpoint="never"), 4, 8)
    assert not bench.matches_reference(CONFIGS["enc12_d4096"], ns, 4, 8)
    assert not bench.matches_reference(CONFIGS["ref_main"], ns, 8, 4)


@pytest.mark.parametrize("transport", ["rccl", "ipc"])
def test_bench_data_parallel_contract(transport):
    """--dp 2 on 4 ranks: two 2-stage pipeline replicas; the JSON counts both
    replicas' tokens and names the layout."""
    args = ["--gpus", "4", "--dp", "2", "--steps", "2", "--warmup", "1", "--device", "cpu", "--config", "tiny",
            "--micro-batch", "2", "--transport", transport]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=4",
           "--master-addr", "127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "bench.py")] + args
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd="/tmp",
                         env={**os.environ, "CUDA_VISIBLE_DEVICES": ""})
    assert out.returncode == 0, out.stderr[-3000:]
    (rec,) = _json_lines(out.stdout)
    cfg = rec["config"]
    assert rec["n_gpus"] == 4 and cfg["parallelism"] == "pp2dp2"
    assert cfg["global_batch"] == 2 * cfg["chunks"] * cfg["micro_batch"] and cfg["chunks"] == 8
    tokens = cfg["global_batch"] * cfg["seq_len"]
    assert abs(rec["value"] - tokens / (rec["ms_per_step"] / 1e3)) / rec["value"] < 0.01
    assert rec["loss"] is not None and rec["loss"] > 0


def test_bench_emulated_plan_pick_cpu(tmp_path):
    """PP > 1 with measured costs: the bench runs its candidate plans on every rank and keeps the fastest
    (calibrate.select_plan_by_emulation) -- the path the GPU bench takes at N > 1, here over gloo."""
    args = ["--gpus", "2", "--steps", "1", "--warmup", "1", "--device", "cpu", "--config", "tiny", "--num-layers", "4",
            "--micro-batch", "2", "--plan", "measured", "--plan-select", "emulate", "--no-bubble"]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "bench.py")] + args
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=900, cwd="/tmp",
                         env={**os.environ, "CUDA_VISIBLE_DEVICES": "", "MIPIPE_CALIB_DIR": str(tmp_path)})
    assert out.returncode == 0, out.stderr[-3000:]
    rec = _json_lines(out.stdout)[0]
    cfg = rec["config"]
    sel = cfg["plan_selection"]
    assert sel is not None and cfg["plan_costs"].startswith("measured")
    if len(sel["candidates"]) > 1:
        assert sel["method"].startswith("emulated"), sel["method"]
        chosen = sel["candidates"][sel["chosen"]]
        assert all(len(c["rank_walls_ms"]) == 2 and min(c["rank_walls_ms"]) > 0 for c in sel["candidates"])
        # the pick: the fastest candidate, or the fastest after moving units off slow ranks (refine_plan_by_walls)
        refined = {r["candidate"]: r["step_ms"] for r in sel.get("refinement", []) if "candidate" in r}
        best = min([c["step_ms"] for c in sel["candidates"]] + list(refined.values()))
        assert refined.get(sel["chosen"], chosen["step_ms"]) == best
        assert cfg["balance"] == sel["chosen_balance"]
    else:
        chosen = sel["candidates"][0]
        assert chosen["balance"] == cfg["balance"]
    assert chosen["v"] == cfg["virtual_chunks_per_rank"]
    # measured costs: the like-for-like PP = 1 rate is priced from them, and the start-up is broken down
    assert rec["like_for_like"]["pp1_tokens_per_s"] > 0
    assert {"calibration", "plan_emulation", "transport", "warmup_steps"} <= set(rec["startup_s"])


@pytest.mark.parametrize("n", [1, 2, 4, 8])
def test_scaling_label_and_default_micro_batch(n):
    """The default enc12 run keeps 128 sequences per micro-batch and 4 x N chunks at every N: the same tokens per
    GPU per step, so 'weak' is the truthful label at N = 1, 2, 4, 8; an explicit --chunks
    fixes the job's work instead ('strong')."""
    import argparse
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    from mipipe.models import CONFIGS

    cfg = CONFIGS["enc12_d4096"]
    mb = bench._default_micro_batch(cfg, n)
    assert mb == 128
    ns = argparse.Namespace(chunks=None, micro_batch=None, dp=1)
    assert bench._scaling_label(cfg, ns, n, 4 * n, mb) == "weak"
    fixed = argparse.Namespace(chunks=8, micro_batch=None, dp=1)
    assert bench._scaling_label(cfg, fixed, n, 8, mb) == ("weak" if n == 1 else "strong")
