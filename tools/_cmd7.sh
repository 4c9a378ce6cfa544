cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "gputests|600|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k lazy" \
 "p_lz1|300|rocprofv3 --kernel-trace --stats -d gpurun_out/plz1 -o run -- python bench.py --steps 3 --warmup 1 --no-bubble" \
 "p_lz0|300|MIPIPE_LAZY_ZERO=0 rocprofv3 --kernel-trace --stats -d gpurun_out/plz0 -o run -- python bench.py --steps 3 --warmup 1 --no-bubble"
