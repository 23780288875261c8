#!/bin/bash
# Round 4 GPU pass G: the annealed V-slot placement extended to the fp64 tail family (config 5's
# space-time decoder, reads + stores) and the two-word fp64 family (stores only): parity + A/B.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r04g}
mkdir -p "$O"
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local n=$1 t=$2
  shift 2
  echo "== $n" >&2
  timeout -k 10 "$t" "$@" > "$O/$n.out" 2> "$O/$n.err" || { echo "step $n failed ($?)"; tail -30 "$O/$n.out"; tail -5 "$O/$n.err"; exit 1; }
}
step t_st 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_phenl.py tests/test_gpu_golden.py tests/test_gpu_parity.py
step phenl1 300 python -u bench.py --workload phenl --steps 3 --warmup 1 --no-cpu-baseline
QLDPC_M2S_ANNEAL=0 step phenl0 300 python -u bench.py --workload phenl --steps 3 --warmup 1 --no-cpu-baseline
step a4_1 300 python -u bench.py --code GenBicycleA4 --steps 5 --warmup 1 --no-cpu-baseline --fp32-line 0 --pmc-traffic 0
QLDPC_M2S_ANNEAL=0 step a4_0 300 python -u bench.py --code GenBicycleA4 --steps 5 --warmup 1 --no-cpu-baseline --fp32-line 0 --pmc-traffic 0
echo "done: $O"
