"""One rank of the watchdog end-to-end test (launched by tests/test_watchdog.py).

Two gloo ranks run one engine step of a tiny LM; rank 0 silently drops its
activation send of the LAST micro-batch.  Rank 1's engine then waits forever
for it and rank 0 waits for the matching gradient: each rank's watchdog must
name the transfer and end the process."""
import dataclasses
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from mipipe import ops  # noqa: E402
from mipipe.models import CONFIGS, TargetSequential, build_lm_blocks, lm_pipeline_units  # noqa: E402
from mipipe.models.transformer import merge_units  # noqa: E402
from mipipe.parallel import PipelineEngine, plan_stages  # noqa: E402
from mipipe.parallel.stage import stage_input_shape  # noqa: E402
from mipipe.parallel.watchdog import Watchdog  # noqa: E402


def main() -> int:
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    timeout = float(os.environ.get("WD_TIMEOUT", "3"))
    cfg = dataclasses.replace(CONFIGS["tiny"], dropout=0.0, num_layers=2, d_model=32, nhead=4,
                              dim_feedforward=64, vocab=50, seq_len=8)
    m, mb = 4, 2
    torch.manual_seed(0)
    units = lm_pipeline_units(build_lm_blocks(cfg))
    plan = plan_stages(cfg, world, 1)
    stage = TargetSequential(*merge_units([units[i] for i in plan.slice(rank)])).train()
    eng = PipelineEngine(stage, chunks=m, checkpoint="never", act_shape=stage_input_shape(cfg, plan, rank, mb),
                         act_dtype=torch.float32, device=torch.device("cpu"), watchdog=Watchdog(timeout),
                         loss_fn=(lambda y, t: ops.cross_entropy(y.reshape(-1, cfg.vocab), t.reshape(-1)))
                         if rank == world - 1 else None)
    if rank == 0 and os.environ.get("WD_DROP", "1") == "1":
        real = eng.chan.send_act
        count = [0]

        def dropping_send(t):
            count[0] += 1
            if count[0] == m:  # the last micro-batch's activation never leaves
                return _Done()
            return real(t)

        eng.chan.send_act = dropping_send
    g = torch.Generator().manual_seed(7)
    tok = torch.randint(0, cfg.vocab, (m, mb, cfg.seq_len + 1), generator=g)
    inputs = [tok[i, :, :-1] for i in range(m)]
    targets = [tok[i, :, 1:].contiguous() for i in range(m)]
    eng.step(inputs if rank == 0 else None, targets)
    print(f"rank {rank}: step finished", flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return 0


class _Done:
    def wait(self):
        return True

    def is_completed(self):
        return True


if __name__ == "__main__":
    sys.exit(main())
