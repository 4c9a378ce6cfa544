# every rank of the PP=8 plans emulated on one GPU (loopback transport) with the round-3 kernels
set -e
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u tools/pp_rank_emulation.py --config gpt2_xl --ranks all --steps 3 > gpurun_out/emu_gpt.log 2>&1
timeout -k 10 500 python -u tools/pp_rank_emulation.py --config enc12_d4096 --micro-batch 64 --ranks all --steps 3 > gpurun_out/emu_enc_el.log 2>&1
timeout -k 10 500 python -u tools/pp_rank_emulation.py --config enc12_d4096 --micro-batch 64 --checkpoint never --ranks all --steps 3 > gpurun_out/emu_enc_nv.log 2>&1
