#!/bin/bash
# Round 4 GPU pass R: Four-Russians OSD groups (QLDPC_OSD_M4R, G = 4 default; G = 6 variant) A/B
# against the lean per-pivot loop (QLDPC_OSD_M4R=0), with the OSD / space-time / circuit GPU tests.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r04r}
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
N="python -u bench.py --workload bposd --code hgp_34_n225 --p 0.06 --steps 2 --warmup 1 --no-cpu-baseline"
X0="env QLDPC_LIB=$L/libqldpc_hip_m0.so"
X6="env QLDPC_LIB=$L/libqldpc_hip_g6.so"
step t_osd 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bposd.py tests/test_gpu_phenl.py tests/test_gpu_circuit.py
step bposd_g4a 300 $B
step bposd_m0a 300 $X0 $B
step bposd_g4b 300 $B
step bposd_m0b 300 $X0 $B
step n225_g4 300 $N
step n225_m0 300 $X0 $N
step t_osd_g6 600 $X6 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bposd.py
step bposd_g6 300 $X6 $B
echo "done: $O"
