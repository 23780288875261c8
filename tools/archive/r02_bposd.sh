#!/bin/bash
# BP+OSD shot loop (device-resident) measurements + kernel trace.  Run ON the GPU box: tools/r02_bposd.sh <tag>
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$1
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R" || exit 1
run() { local tag=$1; shift; timeout -k 10 300 python3 -u bench.py --workload bposd "$@" > "$O/$tag.json" 2> "$O/$tag.err" || { tail "$O/$tag.err"; exit 1; }; python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['dtype'], d['osd_frac_of_decodes'], d['logical_error_rate'])" "$O/$tag.json" $tag; }
run n1600_p004_f32 --code hgp_34_n1600 --p 0.04 --shots 65536 --steps 3 --warmup 1 --precision 32
run n1600_p004_f64 --code hgp_34_n1600 --p 0.04 --shots 65536 --steps 3 --warmup 1 --precision 64
run n225_p006_f64 --code hgp_34_n225 --p 0.06 --shots 262144 --steps 3 --warmup 1 --precision 64
cd /tmp || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_n1600" -o run -- python3 "$R/bench.py" --workload bposd --code hgp_34_n1600 --p 0.04 --shots 65536 --steps 1 --warmup 1 --precision 32 > /dev/null 2>&1 || exit 1
head -6 "$O/trace_n1600/run_kernel_stats.csv" | cut -c1-160
