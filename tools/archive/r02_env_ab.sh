#!/bin/bash
# Interleaved A/B of environment settings on the headline workload (same library):
#   tools/r02_env_ab.sh <tag> <precision> <rounds> "VAR=a" "VAR=b" ...   ("-" = no setting)
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
T=$1; P=$2; N=$3; shift 3
O=$R/gpurun_out/$T
mkdir -p "$O"
cd "$R" || exit 1
for r in $(seq 1 $N); do
  i=0
  for e in "$@"; do
    i=$((i+1))
    E=""; [ "$e" != "-" ] && E=$e
    env $E timeout -k 10 200 python3 -u bench.py --precision $P --steps 4 --warmup 1 --pmc-traffic 0 --fp32-line 0 --no-cpu-baseline > "$O/r${r}_$i.json" 2> "$O/r${r}_$i.err" || { tail -3 "$O/r${r}_$i.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), round(d['roofline']['frac'],4), d['roofline']['kernel'])" "$O/r${r}_$i.json" "$e"
  done
done
