set -e
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "cross_entropy or decoder or vocab or lm" > gpurun_out/ae_tests.log 2>&1
timeout -k 10 200 python -u tools/aten_audit.py --config gpt2_xl > gpurun_out/aten_gpt.log 2>&1
timeout -k 10 200 python -u tools/aten_audit.py --config enc12_d4096 --checkpoint never --micro-batch 8 > gpurun_out/aten_enc.log 2>&1
timeout -k 10 900 python -u tools/pp_rank_emulation.py --config gpt2_xl --ranks all --steps 3 > gpurun_out/emu_gpt.log 2>&1
timeout -k 10 600 python -u tools/pp_rank_emulation.py --config enc12_d4096 --ranks all --steps 3 > gpurun_out/emu_enc.log 2>&1
