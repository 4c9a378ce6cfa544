#!/bin/bash
# Same-box A/B: ab_r3 (54c64be, the round-3 end state), ab_old (977d2cb, register-layout dropout/aux epilogue) vs HEAD (staged-layout epilogue);
# then the Pipe API vs the engine on one GPU under rocprofv3 (kernel time vs wall).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
val() { grep -o '"value": [0-9.]*' "$1" | head -1; }
for i in 1 2; do
  for arm in r3 old new; do
    b=bench.py; [ $arm = old ] && b=ab_old/bench.py; [ $arm = r3 ] && b=ab_r3/bench.py
    timeout -k 10 300 python -u $b --config gpt2_xl --steps 4 --warmup 2 --no-bubble > gpurun_out/ab7_gpt_${arm}_$i.log 2>&1 || { tail -20 gpurun_out/ab7_gpt_${arm}_$i.log; exit 1; }
    echo "gpt2_xl $arm run $i: $(val gpurun_out/ab7_gpt_${arm}_$i.log)"
  done
done
for i in 1 2; do
  for arm in r3 old new; do
    b=bench.py; [ $arm = old ] && b=ab_old/bench.py; [ $arm = r3 ] && b=ab_r3/bench.py
    timeout -k 10 200 python -u $b --steps 10 --warmup 3 --no-bubble > gpurun_out/ab7_enc_${arm}_$i.log 2>&1 || { tail -20 gpurun_out/ab7_enc_${arm}_$i.log; exit 1; }
    echo "enc12 $arm run $i: $(val gpurun_out/ab7_enc_${arm}_$i.log)"
  done
done
for impl in engine pipe; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof7_$impl -o run -- python3 bench.py --impl $impl --steps 4 --warmup 2 --no-bubble > gpurun_out/prof7_$impl.log 2>&1 || { tail -5 gpurun_out/prof7_$impl.log; exit 1; }
  echo "$impl under rocprof: $(val gpurun_out/prof7_$impl.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/prof7_$impl.log)"
  python3 tools/prof_summary.py gpurun_out/prof7_$impl/run_results.db 8 2>&1 | head -3
done
