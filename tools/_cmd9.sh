cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "attn_g0|120|python tools/bench_attn.py 8 1024 25 64 causal 0.0" \
 "attn_g1|120|python tools/bench_attn.py 8 1024 25 64 causal 0.1" \
 "attn_e0|120|python tools/bench_attn.py 32 128 16 256 nc 0.0" \
 "attn_e2|120|python tools/bench_attn.py 32 128 16 256 nc 0.2"
