#!/bin/bash
# A/B of the headline bench: tools/gpu_ab_bench.sh <tag> "<ENV=..>" ...  (bench.py --steps 4 --warmup 1)
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/${1:-abb}
shift
mkdir -p "$O"
cd "$R" || exit 1
for cfg in "$@"; do
  v=$(env $cfg timeout -k 10 120 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline 2>>"$O/err.txt") || { tail "$O/err.txt"; exit 1; }
  echo "$cfg :: $(echo "$v" | python -c 'import json,sys; d=json.load(sys.stdin); print(round(d["value"]), round(d["decodes_per_s"]), d["roofline"]["frac"])')" | tee -a "$O/ab.txt"
done
