#!/bin/bash
# Round 4 GPU pass T: SQ counters of the GPU OSD kernel (lean per-pivot loop) over one BP+OSD
# bench step (n1600, p = 0.04); one counter group per rocprofv3 run.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r04t}
mkdir -p "$O"
cd /tmp || exit 1
export TMPDIR=/tmp
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
)
n=0
for pass in "${PASSES[@]}"; do
  n=$((n + 1))
  # shellcheck disable=SC2086
  timeout -s KILL 240 rocprofv3 --pmc $pass --output-format csv -d "$O/p$n" -o p -- \
    python3 "$R/bench.py" --workload bposd --p 0.04 --steps 1 --warmup 0 --no-cpu-baseline > "$O/p$n.log" 2>&1 || { echo "pass $n failed"; tail -5 "$O/p$n.log"; exit 1; }
done
echo "done: $O"
