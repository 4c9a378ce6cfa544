# round-3 end: GEMM vs hipBLASLt at the enc12 / GPT-2-XL shapes, then kernel traces of both PP=1 benches (no counters)
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/bench_gemm.py 8192 enc12 > gpurun_out/bg_enc_8192.log 2>&1
timeout -k 10 300 python -u tools/bench_gemm.py 4096 enc12 > gpurun_out/bg_enc_4096.log 2>&1
timeout -k 10 300 python -u tools/bench_gemm.py 18432 gpt2xl > gpurun_out/bg_gpt_18432.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/pf_gpt -o gpt -- python3 bench.py --config gpt2_xl --steps 2 --warmup 1 --no-bubble > gpurun_out/pf_gpt.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pf_enc -o enc -- python3 bench.py --steps 4 --warmup 2 --no-bubble > gpurun_out/pf_enc.log 2>&1
