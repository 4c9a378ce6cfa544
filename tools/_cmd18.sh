cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "colsum_tests|300|python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k 'column_sum or deferred_bias' --timeout 120 --timeout-method thread" \
 "bench|300|python bench.py --steps 10 --warmup 3" \
 "prof|300|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_enc -o run -- python bench.py --steps 3 --warmup 1 --no-bubble"
