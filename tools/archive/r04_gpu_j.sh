#!/bin/bash
# Round 4 GPU pass J: timing upper bound of a conflict-free V-slot placement (QLDPC_FAKE_PLACE=1:
# lane-linear slots, WRONG decodes, timing only) against the real annealed placement.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r04j}
mkdir -p "$O"
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local n=$1 t=$2
  shift 2
  echo "== $n" >&2
  timeout -k 10 "$t" "$@" > "$O/$n.out" 2> "$O/$n.err" || { echo "step $n failed ($?)"; tail -30 "$O/$n.out"; tail -5 "$O/$n.err"; exit 1; }
}
step real 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --fp32-line 0
QLDPC_FAKE_PLACE=1 step fake 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --fp32-line 0
echo "done: $O"
