set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/wgrad_probe.py 3 4 > gpurun_out/wgrad_probe.log 2>&1
