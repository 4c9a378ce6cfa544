"""torch.profiler view of one enc12_d4096 PP=1 training step (the bench step):
which ATen ops (not our kernels) launch GPU work, with input shapes.

    python tools/op_profile.py [micro_batch=64] [rows=25]
"""
import os
import sys

os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mipipe import ops  # noqa: E402
from mipipe.models import CONFIGS  # noqa: E402
from mipipe.optim import FlatAdam  # noqa: E402
from mipipe.parallel import PipelineEngine, plan_stages  # noqa: E402
from mipipe.parallel.stage import build_stage, stage_input_shape  # noqa: E402


def main():
    mb = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    rows = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    cfg = CONFIGS["enc12_d4096"]
    dev = torch.device("cuda", 0)
    m, S, V = 4, cfg.seq_len, cfg.vocab
    plan = plan_stages(cfg, 1, 1, m)
    torch.manual_seed(0)
    stage = build_stage(cfg, plan, 0, device=dev, dtype=torch.bfloat16).train()
    opt = FlatAdam(stage.parameters(), lr=1e-4, max_grad_norm=0.5)
    eng = PipelineEngine(stage, chunks=m, act_shape=stage_input_shape(cfg, plan, 0, mb), act_dtype=torch.bfloat16,
                         loss_fn=lambda y, t: ops.cross_entropy(y.reshape(-1, V), t.reshape(-1)), device=dev)
    tok = torch.randint(0, V, (m, mb, S + 1), device=dev)
    xs = [tok[i, :, :S] for i in range(m)]
    ts = [tok[i, :, 1:].contiguous() for i in range(m)]

    def step():
        opt.zero_grad()
        eng.step(xs, ts)
        opt.step(opt.grad_sumsq())

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, record_shapes=True) as prof:
        step()
        torch.cuda.synchronize()
    print(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=rows,
                                                             max_name_column_width=60, max_shapes_column_width=70))


if __name__ == "__main__":
    main()
