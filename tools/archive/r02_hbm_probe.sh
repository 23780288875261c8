#!/bin/bash
# Engine-6 measurements: config 5 (phenl, fp64 now possible) and config 4 forced onto HBM
# messages vs the LDS engine, kernel traces.  Run ON the GPU box: tools/r02_hbm_probe.sh <tag>
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$1
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R" || exit 1
run() { local tag=$1; shift; timeout -k 10 300 python3 -u bench.py "$@" > "$O/$tag.json" 2> "$O/$tag.err" || { tail "$O/$tag.err"; exit 1; }; python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['dtype'], d.get('mean_iters_per_decode'), d['roofline'] and d['roofline'].get('frac'))" "$O/$tag.json" $tag; }
run phenl64 --workload phenl --p 0.005 --shots 65536 --steps 1 --warmup 1 --precision 64
run phenl32 --workload phenl --p 0.005 --shots 65536 --steps 3 --warmup 1 --precision 32
run lp30_lds64 --code LP_Matg8_L30_Dmin20 --p 0.05 --shots 65536 --steps 3 --warmup 1 --pmc-traffic 0 --fp32-line 0 --no-cpu-baseline
QLDPC_ENGINE=6 run lp30_hbm64 --code LP_Matg8_L30_Dmin20 --p 0.05 --shots 1048576 --steps 2 --warmup 1 --pmc-traffic 1 --fp32-line 0 --no-cpu-baseline
QLDPC_ENGINE=6 run lp30_hbm32 --code LP_Matg8_L30_Dmin20 --p 0.05 --shots 1048576 --steps 2 --warmup 1 --precision 32 --pmc-traffic 0 --fp32-line 0 --no-cpu-baseline
cd /tmp || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_phenl64" -o run -- python3 "$R/bench.py" --workload phenl --p 0.005 --shots 65536 --steps 1 --warmup 1 --precision 64 > /dev/null 2>&1 || exit 1
QLDPC_ENGINE=6 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_lp30_hbm64" -o run -- python3 "$R/bench.py" --code LP_Matg8_L30_Dmin20 --p 0.05 --shots 1048576 --steps 1 --warmup 1 --pmc-traffic 0 --fp32-line 0 --no-cpu-baseline > /dev/null 2>&1 || exit 1
head -5 "$O/trace_phenl64/run_kernel_stats.csv" | cut -c1-150
head -5 "$O/trace_lp30_hbm64/run_kernel_stats.csv" | cut -c1-150
