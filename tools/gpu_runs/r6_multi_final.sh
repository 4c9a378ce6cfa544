#!/bin/bash
# Final-tree multi-rank rehearsal on one MI355X: the driver's N > 1 path at N = 2 (enc12 defaults, measured costs,
# emulated plan selection, IPC links + self-test), and GPT-2-XL at PP=2 (checkpoint='always': the keep-word reuse
# across the engine's recomputes).  Time-sliced ranks: functional, not throughput.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
bash tools/gpu_runs/r6_g5.sh 2:64:400 || exit 1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29711 bench.py --config gpt2_xl --gpus 2 --shared-gpu --micro-batch 4 --steps 3 --warmup 1 --no-bubble > gpurun_out/r6_multi_gpt.log 2>&1 || { tail -30 gpurun_out/r6_multi_gpt.log; exit 1; }
python - <<'PY'
import json
d = [json.loads(l) for l in open("gpurun_out/r6_multi_gpt.log") if l.startswith("{")][0]
c = d["config"]
print(f"gpt2_xl PP=2 shared: {d['value']} tok/s (time-sliced), transport {c['transport']}, loss {d.get('loss')}, "
      f"checkpoint {c.get('checkpoint')}, startup {d['startup_s'].get('total_before_timed_steps')}")
PY
