#!/bin/bash
# Round 5: the full GPU suite and smoke on the current tree.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r05suite}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.out" 2> "$O/pytest_gpu.err" || { echo "suite failed"; tail -30 "$O/pytest_gpu.out"; exit 1; }
tail -3 "$O/pytest_gpu.out"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.out" 2>&1 || { echo "smoke failed"; tail -5 "$O/smoke.out"; exit 1; }
tail -1 "$O/smoke.out"
timeout -k 10 300 python -u bench.py --workload bposd --p 0.04 --steps 2 --warmup 1 --no-cpu-baseline > "$O/bposd.out" 2> "$O/bposd.err" || { echo "bposd failed"; tail -5 "$O/bposd.err"; exit 1; }
tail -1 "$O/bposd.out" | cut -c1-200
