#!/bin/bash
# Round-3 GPU check: GPU test suite, then the default bench line.  tools/r03_check.sh <tag>
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
T=$1
O=$R/gpurun_out/$T
mkdir -p "$O"
cd "$R" || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -3 "$O/pytest_gpu.log"
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > "$O/bench.json" 2> "$O/bench.err" || { tail "$O/bench.err"; exit 1; }
cat "$O/bench.json"
