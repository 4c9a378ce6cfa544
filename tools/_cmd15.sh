cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "gpu_tests|900|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "gpt2|300|python bench.py --config gpt2_xl --steps 6 --warmup 2" \
 "bench|300|python bench.py --steps 10 --warmup 3"
