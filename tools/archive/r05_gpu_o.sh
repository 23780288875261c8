#!/bin/bash
# Round 5 GPU pass O: one-iteration min-sum decodes through the first-min step kernel: parity tests
# (direct, circuit loop), the circuit bench line and its kernel trace.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r05o}
mkdir -p "$O"
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local n=$1 t=$2
  shift 2
  echo "== $n" >&2
  timeout -k 10 "$t" "$@" > "$O/$n.out" 2> "$O/$n.err" || { echo "step $n failed ($?)"; tail -40 "$O/$n.out"; tail -5 "$O/$n.err"; exit 1; }
}
step pytest_bp1 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_circuit.py tests/test_gpu_phenl.py -x -q -k "one_iteration or circuit or firstmin or phen" --timeout 300 --timeout-method thread
tail -2 "$O/pytest_bp1.out"
step circuit 300 python -u bench.py --workload circuit --steps 3 --warmup 1
QLDPC_BP1=0 step circuit_engine 300 python -u bench.py --workload circuit --steps 3 --warmup 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o t -- python3 "$R/bench.py" \
  --workload circuit --steps 3 --warmup 1 > "$O/circuit_under_trace.out" 2> "$O/trace.err") || { echo "trace failed"; exit 1; }
head -8 "$O/trace/t_kernel_stats.csv" | cut -c1-150
for f in circuit circuit_engine; do tail -1 "$O/$f.out" | cut -c1-160; done
