cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "gpt2_s6|300|python bench.py --config gpt2_xl --steps 6 --warmup 2" \
 "prof_gpt2|300|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gpt2 -o run -- python bench.py --config gpt2_xl --steps 2 --warmup 1 --no-bubble"
