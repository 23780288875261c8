#!/bin/bash
# Round 5 GPU pass B: the GPU OSD for non-uniform priors (osd.hip step 6') and the circuit loop
# without its host round trip: the BP+OSD and circuit GPU tests, the circuit bench line and its
# kernel trace.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r05b}
mkdir -p "$O"
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local n=$1 t=$2
  shift 2
  echo "== $n" >&2
  timeout -k 10 "$t" "$@" > "$O/$n.out" 2> "$O/$n.err" || { echo "step $n failed ($?)"; tail -40 "$O/$n.out"; tail -5 "$O/$n.err"; exit 1; }
}
step pytest_osd_circ 900 python -u -m pytest tests/test_gpu_bposd.py tests/test_gpu_circuit.py -x -v -s --timeout 300 --timeout-method thread
tail -5 "$O/pytest_osd_circ.out"
step circuit 300 python -u bench.py --workload circuit --steps 3 --warmup 1
cat "$O/circuit.out"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ctrace" -o t -- python3 "$R/bench.py" \
  --workload circuit --steps 3 --warmup 1 > "$O/circuit_under_trace.out" 2> "$O/ctrace.err") || { echo "trace failed"; exit 1; }
echo "done: $O"
