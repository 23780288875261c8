#!/bin/bash
# Round 5 GPU pass Q: OSD steps 4-5 from the register rows (osd_e / osd_0): BP+OSD / circuit parity
# tests, stamps, BP+OSD bench.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r05q}
mkdir -p "$O"
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local n=$1 t=$2
  shift 2
  echo "== $n" >&2
  timeout -k 10 "$t" "$@" > "$O/$n.out" 2> "$O/$n.err" || { echo "step $n failed ($?)"; tail -40 "$O/$n.out"; tail -5 "$O/$n.err"; exit 1; }
}
step pytest_osd 900 python -u -m pytest tests/test_gpu_bposd.py tests/test_gpu_circuit.py -x -q --timeout 300 --timeout-method thread
tail -2 "$O/pytest_osd.out"
QLDPC_LIB=$R/qldpc_fault_tolerance_amd/libqldpc_hip_stamps.so step stamps 300 python -u tools/osd_stamps.py hgp_34_n1600 0.04 65536
cat "$O/stamps.out"
step bposd 300 python -u bench.py --workload bposd --p 0.04 --steps 2 --warmup 1 --no-cpu-baseline
tail -1 "$O/bposd.out" | cut -c1-250
