#!/bin/bash
# Occupancy scan: throughput vs resident workgroups per CU (grid = k * 256 CUs).
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/${1:-scan}
mkdir -p "$O"
cd "$R" || exit 1
GRIDS=256,512,768,1024 VPLS=7 timeout -k 10 300 python -u tools/quick_perf.py hgp_34_n1600 0.06 65536 > "$O/scan_e3.txt" 2>&1 || { cat "$O/scan_e3.txt"; exit 1; }
cat "$O/scan_e3.txt"
QLDPC_ENGINE=4 GRIDS=256,512,768,1024 VPLS=7 timeout -k 10 300 python -u tools/quick_perf.py hgp_34_n1600 0.06 65536 > "$O/scan_e4.txt" 2>&1 || exit 1
cat "$O/scan_e4.txt"
QLDPC_ENGINE=2 GRIDS=256,512,768,1024 timeout -k 10 300 python -u tools/quick_perf.py hgp_34_n1600 0.06 65536 > "$O/scan_e2.txt" 2>&1 || exit 1
cat "$O/scan_e2.txt"
