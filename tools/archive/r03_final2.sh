#!/bin/bash
# Closing evidence after the label change: GPU suite, default bench, rocprof trace, SQ passes, plus the
# config-5 lines at informative p (fp64 0.002 / 0.005, fp32 0.005, BP+OSD decoder2 at 0.005).
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
TAG=r03_final2 bash "$R/tools/r03_final.sh" || exit 1
O=$R/gpurun_out/r03_final2
cd "$R" || exit 1
for cfg in "64 0.002 bp" "64 0.005 bp" "32 0.005 bp" "64 0.005 bposd"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --workload phenl --precision $1 --p $2 --dec2 $3 --steps 5 --warmup 1 > "$O/phenl$1_p$2_$3.json" 2> "$O/phenl$1_p$2_$3.err" || { tail "$O/phenl$1_p$2_$3.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('phenl', sys.argv[2], round(d['value']), d['logical_error_rate'], round(d['nonconverged_frac'],3), round(r['frac'],4))" "$O/phenl$1_p$2_$3.json" "$cfg"
done
