#!/bin/bash
# Round 4 GPU pass N: the OSD's next-pivot search issued ahead of the row update (QLDPC_OSD_EARLY):
# OSD / space-time / circuit GPU tests on it, BP+OSD A/B against the QLDPC_OSD_EARLY=0 build, and
# the step stamps of the default and panel (QLDPC_OSD_PNL=2) eliminations.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r04n}
mkdir -p "$O"
export TMPDIR=/tmp
L=$R/qldpc_fault_tolerance_amd
step() {  # name, timeout, command...
  local n=$1 t=$2
  shift 2
  echo "== $n" >&2
  timeout -k 10 "$t" "$@" > "$O/$n.out" 2> "$O/$n.err" || { echo "step $n failed ($?)"; tail -30 "$O/$n.out"; tail -5 "$O/$n.err"; exit 1; }
}
step pytest_osd 900 python -u -m pytest tests/test_gpu_bposd.py tests/test_gpu_phenl.py tests/test_gpu_circuit.py -m gpu -x -q --timeout 300 --timeout-method thread
B="python -u bench.py --workload bposd --p 0.04 --steps 2 --warmup 1 --no-cpu-baseline"
step bposd_e1a 300 $B
step bposd_e0a 300 env QLDPC_LIB=$L/libqldpc_hip_e0.so $B
step bposd_e1b 300 $B
step bposd_e0b 300 env QLDPC_LIB=$L/libqldpc_hip_e0.so $B
step stamps 300 env QLDPC_LIB=$L/libqldpc_hip_stamps.so python -u tools/osd_stamps.py
step stamps_pnl2 300 env QLDPC_LIB=$L/libqldpc_hip_stamps.so QLDPC_OSD_PNL=2 python -u tools/osd_stamps.py
echo "done: $O"
