#!/bin/bash
# Default bench line (fp64 headline + fp32 side line + PMC traffic + CPU baseline) and a 2-rank
# rehearsal of bench.py --gpus 2 on one GPU (gloo).  Run ON the GPU box: tools/r02_bench.sh <tag>
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$1
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R" || exit 1
timeout -k 10 400 python3 -u bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail "$O/bench.err"; exit 1; }
cat "$O/bench.json"
QLDPC_SHARE_GPU=1 QLDPC_DIST_BACKEND=gloo timeout -k 10 300 python3 -u bench.py --gpus 2 --steps 3 --warmup 1 --shots 65536 > "$O/bench_g2.json" 2> "$O/bench_g2.err" || { tail "$O/bench_g2.err"; exit 1; }
cat "$O/bench_g2.json"
timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --shots 131072 --pmc-traffic 0 --fp32-line 0 --no-cpu-baseline > "$O/bench_g1s.json" 2> "$O/bench_g1s.err" || { tail "$O/bench_g1s.err"; exit 1; }
cat "$O/bench_g1s.json"
