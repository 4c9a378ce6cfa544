#!/bin/bash
# Round 5: the full GPU tier on the current tree, smoke, then Pipe on the reference's structure with the new defaults.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_gpu_tier.log 2>&1
rc=$?
tail -15 gpurun_out/r5_gpu_tier.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_smoke.log 2>&1 || { tail -10 gpurun_out/r5_smoke.log; exit 1; }
tail -1 gpurun_out/r5_smoke.log
for ck in never except_last; do
  timeout -k 10 300 python -u bench.py --impl pipe --pipe-balance 8,8 --config ref_main --dtype fp32 --checkpoint $ck --steps 10 --warmup 3 > gpurun_out/pg5_$ck.log 2>&1 || { tail -20 gpurun_out/pg5_$ck.log; exit 1; }
  echo "pipe 8,8 $ck: $(grep -o '"value": [0-9.]*' gpurun_out/pg5_$ck.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/pg5_$ck.log) $(grep -o '"peak_hbm_gib_per_gpu": [^]]*]' gpurun_out/pg5_$ck.log)"
done
timeout -k 10 300 python -u bench.py --impl pipe --steps 10 --warmup 3 > gpurun_out/pg5_enc12.log 2>&1 || { tail -20 gpurun_out/pg5_enc12.log; exit 1; }
echo "pipe enc12 (one partition): $(grep -o '"value": [0-9.]*' gpurun_out/pg5_enc12.log)"
