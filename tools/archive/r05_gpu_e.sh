#!/bin/bash
# Round 5 GPU pass E: OSD step stamps (QLDPC_STAMPS diagnostic build) of the blocked elimination and
# the lean per-pivot loop, n1600 p = 0.04 BP+OSD-E(10).
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r05e}
mkdir -p "$O"
export TMPDIR=/tmp
L=$R/qldpc_fault_tolerance_amd/libqldpc_hip_stamps.so
QLDPC_LIB=$L QLDPC_OSD_PNL=3 timeout -k 10 300 python -u tools/osd_stamps.py hgp_34_n1600 0.04 65536 > "$O/stamps_blk.txt" 2>&1 || { echo blk failed; tail "$O/stamps_blk.txt"; exit 1; }
QLDPC_LIB=$L timeout -k 10 300 python -u tools/osd_stamps.py hgp_34_n1600 0.04 65536 > "$O/stamps_lean.txt" 2>&1 || { echo lean failed; tail "$O/stamps_lean.txt"; exit 1; }
cat "$O/stamps_blk.txt" "$O/stamps_lean.txt"
