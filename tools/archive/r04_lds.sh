#!/bin/bash
# Round 4: LDS mix microbenchmark + calibration of the LDS bandwidth counters, then the same
# counters over one headline launch (tools/prof_one.py).  Run ON the GPU box from the repo root.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r04lds}
mkdir -p "$O"
cd /tmp || exit 1
export TMPDIR=/tmp
CNT="SQ_INSTS_LDS_LOAD_BANDWIDTH SQ_INSTS_LDS_STORE_BANDWIDTH SQ_INSTS_LDS_ATOMIC_BANDWIDTH SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS"
timeout -k 10 120 "$R/tools/calib/lds_calib" 20000 > "$O/calib.jsonl" 2>&1 || { echo "calib failed"; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc $CNT --output-format csv -d "$O/calib_pmc" -o p -- "$R/tools/calib/lds_calib" 2000 \
  > "$O/calib_pmc.log" 2>&1 || { echo "calib pmc failed"; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc $CNT --output-format csv -d "$O/bench_pmc" -o p -- \
  python3 "$R/tools/prof_one.py" hgp_34_n1600 0.06 65536 0 64 Total 1373040338 10 > "$O/bench_pmc.log" 2>&1 \
  || { echo "bench pmc failed"; exit 1; }
echo "done: $O"
