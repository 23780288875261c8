#!/bin/bash
# A/B throughput probe: tools/gpu_ab.sh <tag> "<ENV=.. ENV2=..>" "<ENV=..>" ...  (n1600, p=0.06, 262144 shots)
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/${1:-ab}
shift
mkdir -p "$O"
cd "$R" || exit 1
i=0
for cfg in "$@"; do
  echo "== $cfg" | tee -a "$O/ab.txt"
  env $cfg timeout -k 10 120 python -u tools/quick_perf.py hgp_34_n1600 0.06 262144 >> "$O/ab.txt" 2>&1 || { cat "$O/ab.txt"; exit 1; }
  i=$((i+1))
done
grep -v amdgpu.ids "$O/ab.txt"
