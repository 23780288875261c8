#!/bin/bash
# Round 5: kernel trace of the circuit-level bench line on the final tree.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r05circ}
mkdir -p "$O"
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o t -- python3 "$R/bench.py" \
  --workload circuit --steps 3 --warmup 1 > "$O/circuit_under_trace.out" 2> "$O/trace.err") || { echo "trace failed"; tail -5 "$O/trace.err"; exit 1; }
head -12 "$O/trace/t_kernel_stats.csv" | cut -c1-160
tail -1 "$O/circuit_under_trace.out" | cut -c1-200
