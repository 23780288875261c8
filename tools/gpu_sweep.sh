#!/bin/bash
# Engine-3 geometry sweep (vars per thread) over the configs' codes, then PMC
# passes of the n1600 kernel.  Run ON the GPU box:  tools/gpu_sweep.sh <tag>
set -u
TAG=${1:-sweep}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R" || exit 1
for c in "hgp_34_n1600 0.06 65536 7,6,8,5" "hgp_34_n225 0.06 262144 1,2,3,4" "hgp_34_n625 0.06 131072 3,4,5,6,7" \
         "GenBicycleA4 0.06 131072 2,4,6,8" "GenBicycleA1 0.06 262144 1,2"; do
  set -- $c
  VPLS=$4 timeout -k 10 200 python -u tools/quick_perf.py "$1" "$2" "$3" >> "$O/perf.txt" 2>&1 || { tail "$O/perf.txt"; exit 1; }
done
cat "$O/perf.txt"
if [ "${PMC:-1}" = 1 ]; then
  timeout -k 10 600 bash tools/pmc_passes.sh "gpurun_out/$TAG/pmc" hgp_34_n1600 0.06 16384 7 || exit 1
  python tools/pmc_summary.py "$O/pmc" rmc_kernel > "$O/pmc_summary.txt"; cat "$O/pmc_summary.txt"
fi
