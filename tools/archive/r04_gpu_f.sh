#!/bin/bash
# Round 4 GPU pass F: two OSD syndromes per workgroup (osd_rr2_kernel, QLDPC_OSD_NSY=2) against one.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r04f}
mkdir -p "$O"
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local n=$1 t=$2
  shift 2
  echo "== $n" >&2
  timeout -k 10 "$t" "$@" > "$O/$n.out" 2> "$O/$n.err" || { echo "step $n failed ($?)"; tail -30 "$O/$n.out"; tail -5 "$O/$n.err"; exit 1; }
}
QLDPC_OSD_NSY=2 step t_bposd2 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_bposd.py tests/test_gpu_phenl.py tests/test_gpu_circuit.py
QLDPC_OSD_NSY=2 step bposd2 300 python -u bench.py --workload bposd --p 0.04 --steps 2 --warmup 1 --no-cpu-baseline
step bposd1 300 python -u bench.py --workload bposd --p 0.04 --steps 2 --warmup 1 --no-cpu-baseline
echo "done: $O"
