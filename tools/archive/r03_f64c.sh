#!/bin/bash
# fp64 5-VALU c2v (two-word families): full GPU suite, config 5 fp64 / fp32, the two-word n1600 family
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r03_f64c
mkdir -p "$O"
cd "$R" || exit 1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
for prec in 64 32; do
timeout -k 10 300 python3 -u bench.py --workload phenl --precision $prec --steps 3 --warmup 1 --no-cpu-baseline > "$O/phenl$prec.json" 2> "$O/phenl$prec.err" || { tail -5 "$O/phenl$prec.err"; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('phenl', sys.argv[2], round(d['value']), round(r['frac'],4), round(r['kernel_ms'],2))" "$O/phenl$prec.json" $prec
done
QLDPC_M2S=0 timeout -k 10 300 python3 -u bench.py --steps 4 --warmup 1 --pmc-traffic 0 --fp32-line 0 --no-cpu-baseline > "$O/bench_2word.json" 2> "$O/bench_2word.err" || { tail -5 "$O/bench_2word.err"; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('two-word n1600', round(d['value']), round(r['frac'],4), r['kernel'])" "$O/bench_2word.json"
