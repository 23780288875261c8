#!/bin/bash
# Phenomenological space-time bring-up: its parity tests, then config-5 throughput.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/${1:-phenl}
mkdir -p "$O"
cd "$R" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_phenl.py -x -v --timeout 120 --timeout-method thread > "$O/pytest_phenl.log" 2>&1
rc=$?; tail -5 "$O/pytest_phenl.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/phenl_perf.py hgp_34_n1225_q3 0.01,0.02,0.03 32768 32 > "$O/phenl_perf.txt" 2>&1
rc=$?; cat "$O/phenl_perf.txt"; exit $rc
