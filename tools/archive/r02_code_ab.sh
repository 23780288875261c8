#!/bin/bash
# A/B of env switches on one code: tools/r02_code_ab.sh <tag> <code> <precision> "<ENV=val ...>" ...
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
T=$1; C=$2; P=$3; shift 3
O=$R/gpurun_out/$T
mkdir -p "$O"
cd "$R" || exit 1
i=0
for envs in "$@"; do
  i=$((i+1))
  env $envs timeout -k 10 200 python3 -u bench.py --code $C --precision $P --steps 3 --warmup 1 --pmc-traffic 0 --fp32-line 0 --no-cpu-baseline > "$O/ab$i.json" 2> "$O/ab$i.err" || { tail -3 "$O/ab$i.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), round(d['roofline']['frac'],4), d['roofline']['kernel'])" "$O/ab$i.json" "$envs"
done
