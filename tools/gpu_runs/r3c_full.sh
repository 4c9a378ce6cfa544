# full GPU tier on the new default schedule (7) + bias fold + wave-per-row LN; benches; A/Bs; ATen audit
set -e
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gputest2.log 2>&1
for i in 1 2; do
  MIPIPE_FUSE_BIAS=0 timeout -k 10 200 python -u bench.py --steps 8 --warmup 3 --no-bubble > gpurun_out/fb0_$i.log 2>&1
  MIPIPE_FUSE_BIAS=1 timeout -k 10 200 python -u bench.py --steps 8 --warmup 3 --no-bubble > gpurun_out/fb1_$i.log 2>&1
done
for i in 1 2; do
  MIPIPE_LN_ROWS=0 timeout -k 10 300 python -u bench.py --config gpt2_xl --steps 3 --warmup 2 --no-bubble > gpurun_out/ln0_$i.log 2>&1
  MIPIPE_LN_ROWS=1 timeout -k 10 300 python -u bench.py --config gpt2_xl --steps 3 --warmup 2 --no-bubble > gpurun_out/ln1_$i.log 2>&1
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_enc2.log 2>&1
timeout -k 10 200 python -u tools/aten_audit.py --config gpt2_xl > gpurun_out/aten_gpt2.log 2>&1
