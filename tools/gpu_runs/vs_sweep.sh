set -e
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "vocab or strided or target_offset or cross_entropy or linear or fold or embed" > gpurun_out/vs_tests.log 2>&1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_pipeline.py > gpurun_out/vs_pipe.log 2>&1
timeout -k 10 120 python -u tools/adam_ab.py > gpurun_out/adam_ab.log 2>&1
for mb in 64 96 128; do timeout -k 10 240 python -u bench.py --steps 8 --warmup 3 --micro-batch $mb --no-bubble > gpurun_out/mbs$mb.log 2>&1; done
timeout -k 10 200 python -u tools/pp_rank_emulation.py --rank 7 --steps 4 > gpurun_out/emu7.log 2>&1
