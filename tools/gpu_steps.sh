#!/bin/bash
# Runs GPU steps on the gpurun box, each under its own time limit.
# Usage: bash tools/gpu_steps.sh "name1|timeout1|cmd1" "name2|timeout2|cmd2" ...
# A step that faults / aborts / times out (rc not in 0,1,2,5) ends the script:
# nothing else touches the GPU after it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"
  t="${rest%%|*}"; cmd="${rest#*|}"
  echo "== [$name] (limit ${t}s) $cmd"
  start=$(date +%s)
  timeout -k 10 "$t" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "[$name] rc=$rc in $(( $(date +%s) - start ))s"
  tail -n 15 "gpurun_out/$name.log"
  case $rc in
    0|1|2|5) ;;
    *) echo "[$name] fatal rc=$rc -- stopping"; exit "$rc" ;;
  esac
done
