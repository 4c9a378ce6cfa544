# GEMM schedule A/B (ping-pong vs B staged two tiles ahead) + a correctness pass of the GEMM tests under the new schedule
set -e
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
MIPIPE_GEMM_SCHED=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "linear or gemm or vocab or fold" > gpurun_out/sab_tests.log 2>&1
timeout -k 10 400 python -u tools/gemm_sched_ab.py 2 3 > gpurun_out/sched_ab.log 2>&1
