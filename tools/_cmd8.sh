cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "ref_fp32|400|python bench.py --config ref_main --dtype fp32 --steps 5 --warmup 2" \
 "ref_bf16|300|python bench.py --config ref_main --steps 10 --warmup 3" \
 "ref_bf16_el|300|python bench.py --config ref_main --steps 10 --warmup 3 --checkpoint except_last" \
 "prof_enc|300|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_enc -o run -- python bench.py --steps 3 --warmup 1 --no-bubble" \
 "prof_gpt2|400|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gpt2 -o run -- python bench.py --config gpt2_xl --steps 2 --warmup 1 --no-bubble"
