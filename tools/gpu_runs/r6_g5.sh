#!/bin/bash
# Round 6 (VERDICT r5 Next #2): the driver's N > 1 start-up path -- measured unit costs (calibration) + emulated
# plan selection + IPC link set-up + self-test -- at the bench defaults (12 layers, chunks 4 x N), N ranks sharing
# ONE MI355X (--shared-gpu: gloo for the small collectives), micro-batch cut only as far as N ranks on one GPU need.
# Functional/start-up rehearsal: the ranks time-slice one GPU, so tokens/s is NOT a throughput number.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 MIPIPE_BENCH_PROGRESS=1 MIPIPE_CALIB_DIR="$GRAFT_REPO_ROOT/gpurun_out/calib6"
port=29631
for spec in "$@"; do
  IFS=: read n mb t <<< "$spec"
  port=$((port + 1))
  t0=$SECONDS; timeout -k 10 $t python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n --shared-gpu --plan measured --plan-select emulate --micro-batch $mb --steps 2 --warmup 1 --no-bubble > gpurun_out/r6_startup_pp$n.log 2>&1 || { tail -40 gpurun_out/r6_startup_pp$n.log; exit 1; }
  grep "^{" gpurun_out/r6_startup_pp$n.log > gpurun_out/r6_startup_pp$n.json
  python - "$n" <<'PY'
import json, sys
n = sys.argv[1]
d = json.loads(open(f"gpurun_out/r6_startup_pp{n}.json").read().splitlines()[0])
c = d["config"]
sel = c["plan_selection"] or {}
print(f"PP={n}: {d['value']} tok/s (time-sliced), v={c['virtual_chunks_per_rank']}, transport {c['transport']}, "
      f"plan_costs {c['plan_costs']!r}, selection {sel.get('method')!r}, {len(sel.get('candidates', []))} candidates")
print("  startup_s", d["startup_s"])
for rf in sel.get("refinement", []):
    print(f"  refined candidate {rf['candidate']}: {len([h for h in rf['moves'] if h.get('accepted')])} moves kept, "
          f"step {rf['step_ms']} ms")
print("  chosen", sel.get("chosen"), sel.get("chosen_balance"))
print("  like_for_like", d["like_for_like"])
PY
  echo "  wall of the whole run: $((SECONDS - t0)) s"
done
