#!/bin/bash
# GPU suite (panel OSD + uniform-prior m2s as defaults), BP+OSD A/B (panel vs per-pivot elimination),
# engine 6 forced on LP L30 fp64 with large staged batches (more decodes per lane: shorter tails).
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r03_pnl
mkdir -p "$O"
cd "$R" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_bposd.py tests/test_gpu_m2s.py -x -q --timeout 250 --timeout-method thread > "$O/pytest_bposd_m2s.log" 2>&1 || { tail -40 "$O/pytest_bposd_m2s.log"; exit 1; }
tail -2 "$O/pytest_bposd_m2s.log"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
for r in 1 2; do
  for pnl in 1 0; do
    QLDPC_OSD_PNL=$pnl timeout -k 10 300 python3 -u bench.py --workload bposd --p 0.04 --steps 3 --warmup 1 > "$O/bposd_pnl$pnl.json" 2> "$O/bposd_pnl$pnl.err" || { tail -5 "$O/bposd_pnl$pnl.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('bposd pnl', sys.argv[2], round(d['value']), d['osd_decodes'], d['logical_error_rate'])" "$O/bposd_pnl$pnl.json" $pnl | tee -a "$O/bposd_ab.txt"
  done
done
QLDPC_ENGINE=6 QLDPC_STAGED_BATCH=4194304 timeout -k 10 400 python3 -u bench.py --code LP_Matg8_L30_Dmin20 --steps 2 --warmup 1 --shots 4194304 --fp32-line 0 --no-cpu-baseline > "$O/e6_big.json" 2> "$O/e6_big.err" || { tail -5 "$O/e6_big.err"; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('e6 big', round(d['value']), round(d['roofline']['achieved']), round(r['frac'],4), r['traffic'], r['bytes_per_launch'], d['mean_iters_per_decode'])" "$O/e6_big.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/bposd_trace" -o t -- python3 "$R/bench.py" --workload bposd --p 0.04 --steps 2 --warmup 1 > "$O/bposd_trace.log" 2>&1 || { tail "$O/bposd_trace.log"; exit 1; }
f=$(find "$O/bposd_trace" -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cut -c1-160 "$f" | head -8
