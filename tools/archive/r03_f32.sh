#!/bin/bash
# fp32 engine-3 changes (4-VALU c2v, absolute SDWA addresses for the space-time families):
# full GPU suite, config-5 fp32 line, headline (fp64 + fp32 line).
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r03_f32
mkdir -p "$O"
cd "$R" || exit 1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
timeout -k 10 300 python3 -u bench.py --workload phenl --precision 32 --steps 3 --warmup 1 --no-cpu-baseline > "$O/phenl32.json" 2> "$O/phenl32.err" || { tail -5 "$O/phenl32.err"; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('phenl32', round(d['value']), round(r['frac'],4), round(r['kernel_ms'],2), r['kernel'])" "$O/phenl32.json"
timeout -k 10 300 python3 -u bench.py --steps 4 --warmup 1 --pmc-traffic 0 --no-cpu-baseline > "$O/bench.json" 2> "$O/bench.err" || { tail -5 "$O/bench.err"; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; f=d['fp32_fast_mode']; print('bench', round(d['value']), round(r['frac'],4), 'fp32', round(f['value']), round(f['roofline_frac'],4))" "$O/bench.json"
