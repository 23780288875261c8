#!/bin/bash
# New GPU tests, then the notebook pin at 25x the notebook's sample counts (cells 25, 16, 20), 400 bootstrap draws.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r03_pin
mkdir -p "$O"
cd "$R" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_comm.py -x -v --timeout 120 --timeout-method thread > "$O/pytest_comm.log" 2>&1 || { tail -30 "$O/pytest_comm.log"; exit 1; }
tail -3 "$O/pytest_comm.log"
for c in 25 16 20; do
  timeout -k 10 540 python -u tools/notebook_pin_run.py --cells $c --mult ${MULT:-25} --draws 400 --out "$O/pin_c$c.json" > "$O/pin_c$c.log" 2>&1 || { tail "$O/pin_c$c.log"; exit 1; }
  grep -E "printed|\[" "$O/pin_c$c.log" | grep -v "^cell .* p=" || true
done
