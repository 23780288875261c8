#!/bin/bash
# Engine-3 bring-up on the GPU box: parity tests, then throughput vs engine 2.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/${1:-e3}
mkdir -p "$O"
cd "$R" || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -5 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
VPLS=0,7,5,4 timeout -k 10 240 python -u tools/quick_perf.py hgp_34_n1600 0.06 65536 > "$O/perf_e3.txt" 2>&1 || { cat "$O/perf_e3.txt"; exit 1; }
cat "$O/perf_e3.txt"
QLDPC_ENGINE=2 timeout -k 10 120 python -u tools/quick_perf.py hgp_34_n1600 0.06 65536 > "$O/perf_e2.txt" 2>&1 || exit 1
cat "$O/perf_e2.txt"
PRECS=64 timeout -k 10 120 python -u tools/quick_perf.py hgp_34_n1600 0.06 32768 > "$O/perf_e3_f64.txt" 2>&1 || exit 1
cat "$O/perf_e3_f64.txt"
