#!/bin/bash
# Parity tests (default engine) + n1600 throughput of the register engines.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/${1:-quick}
mkdir -p "$O"
cd "$R" || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
VPLS=${VPLS:-7} timeout -k 10 240 python -u tools/quick_perf.py hgp_34_n1600 0.06 65536 > "$O/perf.txt" 2>&1 || { cat "$O/perf.txt"; exit 1; }
cat "$O/perf.txt"
