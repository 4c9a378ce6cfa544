# rocprofv3 kernel traces of the two PP=1 benches (kernel-trace + stats only; no counters)
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gpt -o gpt -- python3 bench.py --config gpt2_xl --steps 2 --warmup 1 --no-bubble > gpurun_out/prof_gpt.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_enc -o enc -- python3 bench.py --steps 4 --warmup 2 --no-bubble > gpurun_out/prof_enc.log 2>&1
