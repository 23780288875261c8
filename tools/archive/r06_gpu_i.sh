#!/bin/bash
# Round 6 pass I: phase stamps of config 5's space-time decode_batch (QLDPC_STAMPS diagnostic build
# libqldpc_hip_stst.so) at eval_p 0.06 and 0.005: where a decode's cycles go (setup / first check /
# iterations / epilogue).
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r06i}
mkdir -p "$O"
export TMPDIR=/tmp
for P in 0.06 0.005; do
  timeout -k 10 180 env QLDPC_LIB=$R/qldpc_fault_tolerance_amd/libqldpc_hip_stst.so python -u tools/stamps.py --st $P 65536 64 \
    > "$O/stamps_$P.txt" 2>&1 || { echo "stamps $P failed"; tail -5 "$O/stamps_$P.txt"; exit 1; }
  cat "$O/stamps_$P.txt"
done
