#!/bin/bash
# m2s label-search A/B: default (gathers weight 1, store groups weight 4), store groups off, labels off.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r03_label
mkdir -p "$O"
cd "$R" || exit 1
for r in 1 2; do for cfg in "QLDPC_LABEL=1" "QLDPC_LABEL_WS=0" "QLDPC_LABEL_WS=1" "QLDPC_LABEL_WG=4" "QLDPC_LABEL=0"; do
  env $cfg timeout -k 10 200 python3 -u bench.py --steps 4 --warmup 1 --pmc-traffic 0 --fp32-line 0 --no-cpu-baseline > "$O/ab.json" 2> "$O/ab.err" || { tail -5 "$O/ab.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), round(d['roofline']['frac'],4), round(d['roofline']['kernel_ms'],2))" "$O/ab.json" "$cfg" | tee -a "$O/ab.txt"
done; done
