#!/bin/bash
# Round 5 GPU pass A: LDS ceilings measured as the guide measures them (tools/calib/lds_peak.hip,
# continuous issue, immediate offsets) and the headline kernel's SQ issue / wait counters
# (three SQ passes of tools/pmc_passes.sh over one fp64 launch of the bench workload).
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r05a}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 120 "$R/tools/calib/lds_peak" > "$O/lds_peak.jsonl" 2> "$O/lds_peak.err" || { echo "lds_peak failed"; cat "$O/lds_peak.err"; exit 1; }
cat "$O/lds_peak.jsonl"
# headline kernel counters: 65,536 shots, fp64, both sectors, bench seed / p
cd /tmp || exit 1
n=0
for pass in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
  "SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_IFETCH SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL GRBM_COUNT"; do
  n=$((n + 1))
  # shellcheck disable=SC2086
  timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d "$O/pmc/p$n" -o p -- \
    python3 "$R/tools/prof_one.py" hgp_34_n1600 0.06 65536 0 64 Total 1372974802 10 > "$O/pmc_p$n.log" 2>&1 \
    || { echo "pmc pass $n failed"; tail -20 "$O/pmc_p$n.log"; exit 1; }
done
cd "$R" && python3 tools/pmc_summary2.py "$O/pmc" > "$O/pmc_summary.txt" && cat "$O/pmc_summary.txt"
echo "done: $O"
