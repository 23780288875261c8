#!/bin/bash
# rocprofv3 PMC passes (one counter group per run, as gfx950 requires) over one
# fused MC launch.  Run ON the GPU box:  tools/pmc_passes.sh <outdir> [prof_one args...]
# (PROF_SCRIPT=prof_st.py: one space-time decode_batch launch instead)
#   outdir is relative to the repo root; results: <outdir>/p<N>/p_counter_collection.csv
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/$1
shift
mkdir -p "$OUT"
cd /tmp || exit 1
export TMPDIR=/tmp
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
  "SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_IFETCH SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL GRBM_COUNT"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
n=0
for pass in "${PASSES[@]}"; do
  n=$((n + 1))
  # shellcheck disable=SC2086
  timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d "$OUT/p$n" -o p -- \
    python3 "$R/tools/${PROF_SCRIPT:-prof_one.py}" "$@" > "$OUT/p$n.log" 2>&1 || { echo "pass $n failed"; exit 1; }
done
echo "pmc passes done: $OUT"
