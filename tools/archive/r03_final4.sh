#!/bin/bash
# End-of-round: configs 3/4 lines on the final tree (fp64 with the fp32 line), then smoke + GPU suite.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r03_final4
mkdir -p "$O"
cd "$R" || exit 1
for c in GenBicycleA1 GenBicycleA4 LP_Matg8_L30_Dmin20; do
  timeout -k 10 200 python3 -u bench.py --code $c --steps 3 --warmup 1 --no-cpu-baseline --pmc-traffic 0 > "$O/$c.json" 2>> "$O/err.txt" || { tail "$O/err.txt"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); f=d.get('fp32_fast_mode') or {}; print(sys.argv[2], round(d['value']), round(d['mean_iters_per_decode'],1), d['roofline']['kernel'], round(d['roofline']['frac'],3), 'fp32', round(f.get('value',0)), round(f.get('roofline_frac',0),3))" "$O/$c.json" $c
done
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
