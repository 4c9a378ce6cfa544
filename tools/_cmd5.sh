cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "b_fan1|300|python bench.py --no-bubble" \
 "b_fan0|300|MIPIPE_FANOUT=0 python bench.py --no-bubble" \
 "b_fan1b|300|python bench.py --no-bubble" \
 "b_fan0b|300|MIPIPE_FANOUT=0 python bench.py --no-bubble"
