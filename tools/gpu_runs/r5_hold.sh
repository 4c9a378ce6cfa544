#!/bin/bash
# Round 5: driver-exact bench with telemetry, then the CU-hold probe (RCCL-shaped resident kernel, k CUs) beside
# the enc12 PP=1 step and the GPT-2-XL step; hipBLASLt's kernel choice for the enc12 forward shapes.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5_bench.log 2>&1 || { tail -20 gpurun_out/r5_bench.log; exit 1; }
grep '"metric"' gpurun_out/r5_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], json.dumps(d.get('telemetry')))"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/blaslt_id -o run -- python3 tools/blaslt_kernel_id.py > gpurun_out/blaslt_id.log 2>&1 || { tail -20 gpurun_out/blaslt_id.log; exit 1; }
grep TF/s gpurun_out/blaslt_id.log
find gpurun_out/blaslt_id -name "*kernel_stats.csv" | head -1 | xargs cut -c1-250 | head -8
timeout -k 10 900 python -u tools/cu_hold_probe.py --ks 0,1,2,4,8,16,0 --label "enc12 PP=1" > gpurun_out/r5_hold_enc.txt 2>&1 || { tail -20 gpurun_out/r5_hold_enc.txt; exit 1; }
tail -12 gpurun_out/r5_hold_enc.txt
timeout -k 10 900 python -u tools/cu_hold_probe.py --ks 0,1,4,16,0 --label "gpt2_xl PP=1" --bench "--config gpt2_xl --steps 10 --warmup 3 --no-bubble" > gpurun_out/r5_hold_gpt.txt 2>&1 || { tail -20 gpurun_out/r5_hold_gpt.txt; exit 1; }
tail -10 gpurun_out/r5_hold_gpt.txt
