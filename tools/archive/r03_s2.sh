#!/bin/bash
# Round-3 session-2 first GPU call: GPU suite, default bench line, a timing probe of the notebook pin.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r03_s2
mkdir -p "$O"
cd "$R" || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -3 "$O/pytest_gpu.log"
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > "$O/bench.json" 2> "$O/bench.err" || { tail "$O/bench.err"; exit 1; }
cat "$O/bench.json"
timeout -k 10 300 python -u tools/notebook_pin_run.py --cells 25 --mult 1 --draws 50 --out "$O/pin_probe.json" > "$O/pin_probe.log" 2>&1 || { tail "$O/pin_probe.log"; exit 1; }
tail -20 "$O/pin_probe.log"
