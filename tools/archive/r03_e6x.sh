#!/bin/bash
# engine 6 with decisions as LDS ballot words: parity tests, then LP L30 fp64 forced (4M shots), A/B vs HBM decisions.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r03_e6x
mkdir -p "$O"
cd "$R" || exit 1
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_hbm.py > "$O/pytest_hbm.log" 2>&1 || { tail -30 "$O/pytest_hbm.log"; exit 1; }
tail -2 "$O/pytest_hbm.log"
for x in 1 0; do
QLDPC_HBM_XLDS=$x QLDPC_ENGINE=6 timeout -k 10 400 python3 -u bench.py --code LP_Matg8_L30_Dmin20 --steps 2 --warmup 1 --shots 4194304 --fp32-line 0 --no-cpu-baseline > "$O/e6_lp30_x$x.json" 2> "$O/e6_lp30_x$x.err" || { tail -5 "$O/e6_lp30_x$x.err"; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('e6 xlds', sys.argv[2], round(d['value']), round(r['achieved']), round(r['frac'],4), r['traffic'], r['bytes_per_launch'], round(r['traffic']/r['bytes_per_launch'],3), r['kernel'])" "$O/e6_lp30_x$x.json" $x
done
