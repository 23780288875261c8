#!/bin/bash
# Round-closing evidence on one GPU box:  tools/r02_final.sh <tag>
#  1. the default bench line under rocprofv3 --kernel-trace --stats (average kernel duration
#     must agree with the line's HIP-event kernel_ms);
#  2. config 5 (fp64 and fp32) under the kernel trace;
#  3. SQ / HBM counter passes over one launch of the fp64 and fp32 headline kernels.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
T=$1
O=$R/gpurun_out/$T
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- \
  python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --pmc-traffic 0 > "$O/bench_under_rocprof.json" 2> "$O/bench_trace.err" || exit 1
cat "$O/bench_under_rocprof.json"
for P in 64 32; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_phenl$P" -o run -- \
    python3 "$R/bench.py" --workload phenl --precision $P --shots 65536 --steps 2 --warmup 1 --no-cpu-baseline --pmc-traffic 0 --fp32-line 0 > "$O/phenl$P.json" 2> "$O/phenl$P.err" || exit 1
  cat "$O/phenl$P.json"
done
cd "$R" || exit 1
timeout -k 10 500 bash tools/pmc_passes.sh "gpurun_out/$T/pmc64" hgp_34_n1600 0.06 65536 0 64 Total > "$O/pmc64.log" 2>&1 || { tail "$O/pmc64.log"; exit 1; }
python3 tools/pmc_summary2.py "$O/pmc64" > "$O/pmc64_summary.txt"
timeout -k 10 500 bash tools/pmc_passes.sh "gpurun_out/$T/pmc32" hgp_34_n1600 0.06 65536 0 32 Total > "$O/pmc32.log" 2>&1 || { tail "$O/pmc32.log"; exit 1; }
python3 tools/pmc_summary2.py "$O/pmc32" > "$O/pmc32_summary.txt"
cat "$O/pmc64_summary.txt" "$O/pmc32_summary.txt"
echo "done $T"
