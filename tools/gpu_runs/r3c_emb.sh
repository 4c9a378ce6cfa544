# bf16 learned-position table read in place + no-grad forwards skip saved tensors: tests, audit, GPT-2-XL bench
set -e
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gputest3.log 2>&1
timeout -k 10 200 python -u tools/aten_audit.py --config gpt2_xl > gpurun_out/aten_gpt3.log 2>&1
timeout -k 10 200 python -u tools/aten_audit.py --config enc12_d4096 --checkpoint except_last --micro-batch 8 > gpurun_out/aten_enc3.log 2>&1
timeout -k 10 300 python -u bench.py --config gpt2_xl --steps 4 --warmup 2 --no-bubble > gpurun_out/bench_gpt3.log 2>&1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_enc3.log 2>&1
