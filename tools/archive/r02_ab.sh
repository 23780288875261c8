#!/bin/bash
# A/B of env switches on the headline workload: tools/r02_ab.sh <tag> <precision> "<ENV=val ...>" ...
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
T=$1; P=$2; shift 2
O=$R/gpurun_out/$T
mkdir -p "$O"
cd "$R" || exit 1
i=0
for envs in "$@"; do
  i=$((i+1))
  env $envs timeout -k 10 200 python3 -u bench.py --precision $P --steps 4 --warmup 1 --shots 262144 --pmc-traffic 0 --fp32-line 0 --no-cpu-baseline > "$O/ab$i.json" 2> "$O/ab$i.err" || { tail -3 "$O/ab$i.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), round(d['roofline']['frac'],4), d['roofline']['kernel'])" "$O/ab$i.json" "$envs"
done
