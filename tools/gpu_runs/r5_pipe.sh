#!/bin/bash
# Round 5, VERDICT r4 item 6: why Pipe on the reference's own structure (ref_main fp32, balance 8,8 on one GPU) is
# slower than the engine on the same model.  Wall clock of three variants, then kernel time per step of two.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > gpurun_out/pg_$name.log 2>&1 || { tail -20 gpurun_out/pg_$name.log; exit 1; }
  echo "$name: $(grep -o '"value": [0-9.]*' gpurun_out/pg_$name.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/pg_$name.log)"
}
run pipe88 --impl pipe --pipe-balance 8,8 --config ref_main --dtype fp32 --checkpoint never --steps 10 --warmup 3
run pipe16 --impl pipe --pipe-balance 16 --config ref_main --dtype fp32 --checkpoint never --steps 10 --warmup 3
run engine --config ref_main --dtype fp32 --checkpoint never --chunks 4 --micro-batch 8 --steps 10 --warmup 3 --no-bubble
for v in pipe88 engine; do
  if [ $v = pipe88 ]; then a="--impl pipe --pipe-balance 8,8"; else a="--chunks 4 --micro-batch 8"; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/pgp_$v -o run -- python3 bench.py $a --config ref_main --dtype fp32 --checkpoint never --steps 3 --warmup 2 --no-bubble > gpurun_out/pgp_$v.log 2>&1 || { tail -5 gpurun_out/pgp_$v.log; exit 1; }
  python3 tools/prof_summary.py gpurun_out/pgp_$v/run_results.db 25 > gpurun_out/pgp_$v.txt 2>&1
  echo "== $v (5 steps traced)"; head -22 gpurun_out/pgp_$v.txt | cut -c1-170
  rm -rf gpurun_out/pgp_$v
done
