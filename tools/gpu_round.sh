#!/bin/bash
# One GPU-box session: parity tests, the headline bench, its kernel trace and HBM
# traffic counters.  Run ON the GPU box from the repo root:  tools/gpu_round.sh <tag>
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
TAG=${1:-run}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R" || exit 1
step() { echo "== $*" ; }

step pytest
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc

step bench
timeout -k 10 300 python -u bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail "$O/bench.err"; exit 1; }
cat "$O/bench.json"

step kernel-trace
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- \
  python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$O/bench_trace.json" 2> "$O/bench_trace.err" || exit 1

step pmc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$O/pmc_$c" -o p -- \
    python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline > "$O/pmc_$c.json" 2> "$O/pmc_$c.err" || exit 1
done
step phenl
timeout -k 10 300 python3 "$R/bench.py" --workload phenl --p 0.005 --shots 65536 --steps 3 --warmup 1 > "$O/bench_phenl.json" 2> "$O/bench_phenl.err" || { tail "$O/bench_phenl.err"; exit 1; }
cat "$O/bench_phenl.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_phenl" -o run -- \
  python3 "$R/bench.py" --workload phenl --p 0.005 --shots 65536 --steps 1 --warmup 1 > "$O/bench_phenl_trace.json" 2> "$O/bench_phenl_trace.err" || exit 1

step sq-counters
timeout -k 10 400 bash "$R/tools/pmc_passes.sh" "gpurun_out/$TAG/sq" hgp_34_n1600 0.06 65536 > "$O/sq.log" 2>&1 || { tail "$O/sq.log"; exit 1; }
echo "done $TAG"
