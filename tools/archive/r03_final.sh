#!/bin/bash
# Round-3 evidence on the current kernels: GPU suite, the default bench line (fp64 headline + PMC
# traffic + fp32 line + CPU baseline), its rocprofv3 kernel trace, SQ counter passes of the headline
# kernel, engine 6 forced on LP L30 fp64 (4M-shot batches) with PMC traffic.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/${TAG:-r03_final}
mkdir -p "$O"
cd "$R" || exit 1
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
  tail -2 "$O/pytest_gpu.log"
fi
timeout -k 10 400 python -u bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail "$O/bench.err"; exit 1; }
cat "$O/bench.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o t -- python3 "$R/bench.py" --steps 5 --warmup 1 --pmc-traffic 0 --fp32-line 1 --no-cpu-baseline > "$O/trace_bench.json" 2> "$O/trace.err" || { tail "$O/trace.err"; exit 1; }
f=$(find "$O/trace" -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cut -c1-150 "$f" | head -5
cd "$R"
timeout -k 10 500 bash tools/pmc_passes.sh "gpurun_out/${TAG:-r03_final}/pmc64" hgp_34_n1600 0.06 65536 0 64 Total > "$O/pmc64.log" 2>&1 || { tail "$O/pmc64.log"; exit 1; }
python3 tools/pmc_summary2.py "$O/pmc64" > "$O/pmc64_summary.txt" 2>&1; tail -25 "$O/pmc64_summary.txt"
QLDPC_ENGINE=6 timeout -k 10 400 python3 -u bench.py --code LP_Matg8_L30_Dmin20 --steps 2 --warmup 1 --shots 4194304 --fp32-line 0 --no-cpu-baseline > "$O/e6_lp30.json" 2> "$O/e6_lp30.err" || { tail -5 "$O/e6_lp30.err"; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('e6', round(d['value']), round(r['achieved']), round(r['frac'],4), r['traffic'], r['bytes_per_launch'], round(r['traffic']/r['bytes_per_launch'],3))" "$O/e6_lp30.json"
