# round 3 (re-entry): full GPU test tier, PP=1 benches of enc12 and GPT-2-XL, ATen audit
set -e
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_enc.log 2>&1
timeout -k 10 400 python -u bench.py --config gpt2_xl --steps 4 --warmup 2 --no-bubble > gpurun_out/bench_gpt.log 2>&1
timeout -k 10 200 python -u tools/aten_audit.py --config gpt2_xl > gpurun_out/aten_gpt.log 2>&1
timeout -k 10 200 python -u tools/aten_audit.py --config enc12_d4096 --checkpoint never --micro-batch 8 > gpurun_out/aten_enc.log 2>&1
