#!/bin/bash
# SQ counters of the config-5 space-time decoder (fp32 byte-F family, then fp64 tail family)
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r03_stpmc
mkdir -p "$O"
cd "$R" || exit 1
for prec in 32 64; do
  PROF_SCRIPT=prof_st.py timeout -k 10 400 bash tools/pmc_passes.sh "gpurun_out/r03_stpmc/st$prec" 0.06 65536 $prec > "$O/st$prec.log" 2>&1 || { tail "$O/st$prec.log"; exit 1; }
  python3 tools/pmc_summary2.py "$O/st$prec" > "$O/st${prec}_summary.txt" 2>&1; echo "== fp$prec"; tail -9 "$O/st${prec}_summary.txt"
done
