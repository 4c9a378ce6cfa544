cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "gputests|600|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "bench|300|python bench.py" \
 "prof|300|rocprofv3 --kernel-trace --stats -d gpurun_out/prof2 -o run -- python bench.py --steps 3 --warmup 1 --no-bubble"
