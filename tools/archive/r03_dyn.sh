#!/bin/bash
# headline runtime knobs on the final kernel: chunk-queue granularity
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r03_dyn
mkdir -p "$O"
cd "$R" || exit 1
for cfg in "QLDPC_DYN_PER=64" "QLDPC_DYN_PER=16" "QLDPC_DYN_PER=256" "QLDPC_DYN=0" "QLDPC_DYN_PER=64"; do
  env $cfg timeout -k 10 200 python3 -u bench.py --steps 4 --warmup 1 --pmc-traffic 0 --fp32-line 0 --no-cpu-baseline > "$O/ab.json" 2> "$O/ab.err" || { tail -5 "$O/ab.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), round(d['roofline']['frac'],4), round(d['roofline']['kernel_ms'],2))" "$O/ab.json" "$cfg" | tee -a "$O/ab.txt"
done
