cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh "wgrad_probe|200|python tools/wgrad_blaslt_probe.py"
