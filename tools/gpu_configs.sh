#!/bin/bash
# Headline-style lines for the other BASELINE configs (1 GPU): GBC A1-A4 (config 3), LP L30 (config 4).
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/${1:-configs}
mkdir -p "$O"
cd "$R" || exit 1
for c in GenBicycleA1 GenBicycleA2 GenBicycleA3 GenBicycleA4 LP_Matg8_L30_Dmin20; do
  timeout -k 10 200 python -u bench.py --code $c --steps 3 --warmup 1 --no-cpu-baseline --pmc-traffic 0 ${PREC:+--precision $PREC} > "$O/$c.json" 2>> "$O/err.txt" || { tail "$O/err.txt"; exit 1; }
  python -c "import json; d=json.load(open('$O/$c.json')); print('$c', round(d['value']), round(d['decodes_per_s']), round(d['mean_iters_per_decode'],1), d['roofline']['kernel'], round(d['roofline']['frac'],3))"
done
