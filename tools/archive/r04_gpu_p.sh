#!/bin/bash
# Round 4 GPU pass P: the lean per-pivot OSD loop (QLDPC_OSD_LEAN) A/B against the round-3 loop.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r04p}
mkdir -p "$O"
export TMPDIR=/tmp
L=$R/qldpc_fault_tolerance_amd
step() {  # name, timeout, command...
  local n=$1 t=$2
  shift 2
  echo "== $n" >&2
  timeout -k 10 "$t" "$@" > "$O/$n.out" 2> "$O/$n.err" || { echo "step $n failed ($?)"; tail -30 "$O/$n.out"; tail -5 "$O/$n.err"; exit 1; }
}
B="python -u bench.py --workload bposd --p 0.04 --steps 2 --warmup 1 --no-cpu-baseline"
X="env QLDPC_LIB=$L/libqldpc_hip_l0.so"
step t_osd 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bposd.py tests/test_gpu_phenl.py tests/test_gpu_circuit.py
step bposd_l1a 300 $B
step bposd_l0a 300 $X $B
step bposd_l1b 300 $B
step bposd_l0b 300 $X $B
step bposd_n225 300 python -u bench.py --workload bposd --code hgp_34_n225 --p 0.06 --steps 2 --warmup 1 --no-cpu-baseline
step bposd_n225_l0 300 $X python -u bench.py --workload bposd --code hgp_34_n225 --p 0.06 --steps 2 --warmup 1 --no-cpu-baseline
echo "done: $O"
