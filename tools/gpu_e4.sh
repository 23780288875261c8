#!/bin/bash
# Engine-4 bring-up on the GPU box: parity tests under QLDPC_ENGINE=4, then throughput of engines 3/4.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/${1:-e4}
mkdir -p "$O"
cd "$R" || exit 1
QLDPC_ENGINE=4 timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/pytest_gpu_e4.log" 2>&1
rc=$?; tail -5 "$O/pytest_gpu_e4.log"; [ $rc -eq 0 ] || exit $rc
QLDPC_ENGINE=4 VPLS=0,7,4 timeout -k 10 240 python -u tools/quick_perf.py hgp_34_n1600 0.06 65536 > "$O/perf_e4.txt" 2>&1 || { cat "$O/perf_e4.txt"; exit 1; }
cat "$O/perf_e4.txt"
VPLS=7 timeout -k 10 240 python -u tools/quick_perf.py hgp_34_n1600 0.06 65536 > "$O/perf_e3.txt" 2>&1 || exit 1
cat "$O/perf_e3.txt"
QLDPC_ENGINE=4 PRECS=64 VPLS=7 timeout -k 10 120 python -u tools/quick_perf.py hgp_34_n1600 0.06 32768 > "$O/perf_e4_f64.txt" 2>&1 || exit 1
cat "$O/perf_e4_f64.txt"
