set -e
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u tools/pp_rank_emulation.py --config gpt2_xl --ranks all --steps 3 > gpurun_out/emu_gpt.log 2>&1
timeout -k 10 600 python -u tools/pp_rank_emulation.py --config enc12_d4096 --ranks all --steps 3 > gpurun_out/emu_enc.log 2>&1
