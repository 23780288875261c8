#!/bin/bash
# Round 4 GPU pass I: where the BP+OSD time goes after the pipelined row update: the OSD kernel's
# step stamps (diagnostic build) and the kernel trace of the BP+OSD bench.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r04i}
mkdir -p "$O"
export TMPDIR=/tmp
QLDPC_LIB=$R/qldpc_fault_tolerance_amd/libqldpc_hip_osdst.so timeout -k 10 300 python -u tools/osd_stamps.py > "$O/osd_stamps.txt" 2> "$O/osd_stamps.err" || { echo "stamps failed"; tail -5 "$O/osd_stamps.err"; exit 1; }
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o t -- python3 "$R/bench.py" \
  --workload bposd --p 0.04 --steps 2 --warmup 1 --no-cpu-baseline > "$O/bposd_under_trace.out" 2> "$O/trace.err") \
  || { echo "trace failed"; tail -5 "$O/trace.err"; exit 1; }
echo "done: $O"
