#!/bin/bash
# fp64 headline geometry sweep: tools/r02_tb.sh <tag> "<TB list>"
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$1
mkdir -p "$O"
cd "$R" || exit 1
for tb in $2; do
  QLDPC_TB=$tb timeout -k 10 200 python3 -u bench.py --steps 3 --warmup 1 --shots 131072 --pmc-traffic 0 --fp32-line 0 --no-cpu-baseline > "$O/tb$tb.json" 2> "$O/tb$tb.err" || { tail -3 "$O/tb$tb.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), round(d['roofline']['frac'],4), d['roofline']['kernel'])" "$O/tb$tb.json" $tb
done
