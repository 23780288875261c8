#!/bin/bash
# Config 2 sweep on the rest of the family (n225, n625; 1e8 shots per p, fp64), then config 5
# (bench.py --workload phenl, fp64) at the notebook's phenomenological grid p = 0.01 / 0.02 / 0.03.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r03_c2b
mkdir -p "$O"
cd "$R" || exit 1
timeout -k 10 700 python -u tools/config2_sweep.py --codes hgp_34_n225 hgp_34_n625 --shots 1e8 --out "$O/n225_n625.jsonl" > "$O/n225_n625.log" 2>&1 || { tail "$O/n225_n625.log"; exit 1; }
grep -c eval_p "$O/n225_n625.jsonl"
for p in 0.01 0.02 0.03; do
  timeout -k 10 300 python -u bench.py --workload phenl --p $p --steps 5 --warmup 1 > "$O/phenl64_p$p.json" 2> "$O/phenl64_p$p.err" || { tail "$O/phenl64_p$p.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d['logical_error_rate'], d['nonconverged_frac'], round(d['roofline']['frac'],4))" "$O/phenl64_p$p.json" $p
done
