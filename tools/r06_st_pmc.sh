#!/bin/bash
# Round 6: SQ counters of BASELINE config 5's fp64 space-time decoder (one decode_batch launch of
# 65,536 syndromes, tools/prof_st.py), three SQ passes, plus a kernel trace of the same command.
#   tools/r06_st_pmc.sh <outdir-under-gpurun_out> [p] [QLDPC_LIB]
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r06st}
P=${2:-0.06}
mkdir -p "$O"
cd /tmp || exit 1
export TMPDIR=/tmp
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
  "SQ_INSTS_LDS_LOAD_BANDWIDTH SQ_INSTS_LDS_STORE_BANDWIDTH SQ_INSTS_LDS_ATOMIC_BANDWIDTH SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU"
)
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o k -- \
  python3 "$R/tools/prof_st.py" "$P" 65536 64 > "$O/kt.log" 2>&1 || { echo "trace failed"; tail -5 "$O/kt.log"; exit 1; }
n=0
for pass in "${PASSES[@]}"; do
  n=$((n + 1))
  # shellcheck disable=SC2086
  timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d "$O/p$n" -o p -- \
    python3 "$R/tools/prof_st.py" "$P" 65536 64 > "$O/p$n.log" 2>&1 || { echo "pass $n failed"; tail -5 "$O/p$n.log"; exit 1; }
done
cd "$R" && python3 tools/pmc_summary.py "$O" rdec_kernel > "$O/pmc_summary.txt" && cat "$O/pmc_summary.txt"
