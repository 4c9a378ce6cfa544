cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "prof|300|rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 3 --warmup 1 --no-bubble" \
 "gemm|300|python tools/bench_gemm.py" \
 "bench_el|300|python bench.py --checkpoint except_last"
