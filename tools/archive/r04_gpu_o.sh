#!/bin/bash
# Round 4 GPU pass O: the OSD kernels without the hoisted write-out addresses (163 -> 118 VGPRs;
# two-syndrome osd_rr2_kernel 105 spilled VGPRs -> 1 dword): BP+OSD one vs two syndromes per workgroup.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r04o}
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
step t_nsy2 600 env QLDPC_LIB=$L/libqldpc_hip_x.so QLDPC_OSD_NSY=2 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bposd.py tests/test_gpu_phenl.py tests/test_gpu_circuit.py
step t_osd1 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bposd.py
step bposd1a 300 $B
step bposd2a 300 env QLDPC_LIB=$L/libqldpc_hip_x.so QLDPC_OSD_NSY=2 $B
step bposd1b 300 $B
step bposd2b 300 env QLDPC_LIB=$L/libqldpc_hip_x.so QLDPC_OSD_NSY=2 $B
echo "done: $O"
