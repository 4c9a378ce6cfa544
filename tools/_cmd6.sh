cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "gputests|600|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "b_lz1|300|python bench.py --no-bubble" \
 "b_lz0|300|MIPIPE_LAZY_ZERO=0 python bench.py --no-bubble" \
 "b_lz1b|300|python bench.py --no-bubble" \
 "b_lz0b|300|MIPIPE_LAZY_ZERO=0 python bench.py --no-bubble"
