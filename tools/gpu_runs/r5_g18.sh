#!/bin/bash
# Round 5: full GPU tier + smoke + driver-command bench, then the Adam variants A/B (streaming stores) and copy BW.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_gpu_tier.log 2>&1
rc=$?
tail -4 gpurun_out/r5_gpu_tier.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^ERROR" gpurun_out/r5_gpu_tier.log | head; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5_smoke.log 2>&1 || { tail -10 gpurun_out/r5_smoke.log; exit 1; }
tail -1 gpurun_out/r5_smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5_bench.log 2>&1 || { tail -20 gpurun_out/r5_bench.log; exit 1; }
grep '"metric"' gpurun_out/r5_bench.log | cut -c1-300
timeout -k 10 240 python -u tools/adam_ab.py > gpurun_out/adam_ab_r5.txt 2>&1 || { tail -20 gpurun_out/adam_ab_r5.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/adam_ab_r5.txt
