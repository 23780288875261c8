#!/bin/bash
# Closing round-3 evidence on the final tree: GPU suite, default bench (+ PMC traffic, CPU baseline),
# rocprof trace, SQ passes, engine 6 LP L30, config-5 lines (fp32 / fp64 at 0.06, fp64 at 0.02,
# 0.005), the BP+OSD line at p = 0.04 with its kernel trace.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r03_final3
if [ "${PART:-1}" = 1 ]; then
  TAG=r03_final3 bash "$R/tools/r03_final.sh" || exit 1
  exit 0
fi
mkdir -p "$O"
cd "$R" || exit 1
for cfg in "32 0.06 bp" "64 0.06 bp" "64 0.02 bp" "64 0.005 bp" "32 0.005 bp"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --workload phenl --precision $1 --p $2 --dec2 $3 --steps 5 --warmup 1 --no-cpu-baseline > "$O/phenl$1_p$2_$3.json" 2> "$O/phenl$1_p$2_$3.err" || { tail "$O/phenl$1_p$2_$3.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('phenl', sys.argv[2], round(d['value']), d['logical_error_rate'], round(d['nonconverged_frac'],3), round(r['frac'],4))" "$O/phenl$1_p$2_$3.json" "$cfg"
done
timeout -k 10 300 python3 -u bench.py --workload bposd --p 0.04 --steps 3 --warmup 1 --no-cpu-baseline > "$O/bposd_p004.json" 2> "$O/bposd.err" || { tail -5 "$O/bposd.err"; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('bposd', round(d['value']), d.get('osd_frac_of_decodes'), d['logical_error_rate'], (d.get('roofline') or {}).get('frac'))" "$O/bposd_p004.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_bposd" -o b -- python3 "$R/bench.py" --workload bposd --p 0.04 --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2> "$O/trace_bposd.err" || { tail "$O/trace_bposd.err"; exit 1; }
f=$(find "$O/trace_bposd" -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cut -c1-160 "$f" | head -6
echo done
