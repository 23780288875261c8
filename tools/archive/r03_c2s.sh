#!/bin/bash
# c2s family: parity tests of the one-slot families, then the headline A/B c2s vs m2s.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r03_c2s
mkdir -p "$O"
cd "$R" || exit 1
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_m2s.py > "$O/pytest_m2s.log" 2>&1 || { tail -30 "$O/pytest_m2s.log"; exit 1; }
tail -2 "$O/pytest_m2s.log"
for r in 1 2; do for cfg in "QLDPC_C2S=1" "QLDPC_C2S=0"; do
  env $cfg timeout -k 10 200 python3 -u bench.py --steps 4 --warmup 1 --pmc-traffic 0 --fp32-line 0 --no-cpu-baseline > "$O/ab.json" 2> "$O/ab.err" || { tail -5 "$O/ab.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), round(d['roofline']['frac'],4), round(d['roofline']['kernel_ms'],2), d['roofline']['kernel'], d['logical_error_rate'])" "$O/ab.json" "$cfg" | tee -a "$O/ab.txt"
done; done
