#!/bin/bash
# Round 4 GPU pass L: the distributed panel OSD search (QLDPC_OSD_PNL=2: every thread searches its
# own row's 32-column panel word, one barrier per pivot, the panel's pivot rows applied once per
# panel): parity on the BP+OSD / phenl / circuit tests, then A/B against the per-pivot elimination.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r04l}
mkdir -p "$O"
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local n=$1 t=$2
  shift 2
  echo "== $n" >&2
  timeout -k 10 "$t" "$@" > "$O/$n.out" 2> "$O/$n.err" || { echo "step $n failed ($?)"; tail -30 "$O/$n.out"; tail -5 "$O/$n.err"; exit 1; }
}
QLDPC_OSD_PNL=2 step t_pnl2 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bposd.py tests/test_gpu_phenl.py tests/test_gpu_circuit.py
for r in 1 2; do
  QLDPC_OSD_PNL=2 step pnl2_$r 300 python -u bench.py --workload bposd --p 0.04 --steps 2 --warmup 1 --no-cpu-baseline
  step pnl0_$r 300 python -u bench.py --workload bposd --p 0.04 --steps 2 --warmup 1 --no-cpu-baseline
done
QLDPC_OSD_PNL=2 step n225_pnl2 300 python -u bench.py --workload bposd --code hgp_34_n225 --p 0.06 --steps 2 --warmup 1 --no-cpu-baseline
step n225_pnl0 300 python -u bench.py --workload bposd --code hgp_34_n225 --p 0.06 --steps 2 --warmup 1 --no-cpu-baseline
echo "done: $O"
