#!/bin/bash
# m2s V-slot placement A/B (QLDPC_M2S_PLACE=1 default vs 0), m2s parity tests, engine 6 on LP L30 (4M batches).
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r03_place
mkdir -p "$O"
cd "$R" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_m2s.py tests/test_gpu_agreement.py tests/test_gpu_hbm.py tests/test_gpu_phenl.py -x -q --timeout 250 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -2 "$O/pytest.log"
for r in 1 2; do for pl in 1 0; do
  QLDPC_M2S_PLACE=$pl timeout -k 10 200 python3 -u bench.py --steps 4 --warmup 1 --pmc-traffic 0 --fp32-line 0 --no-cpu-baseline > "$O/ab.json" 2> "$O/ab.err" || { tail -5 "$O/ab.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('place', sys.argv[2], round(d['value']), round(d['roofline']['frac'],4), round(d['roofline']['kernel_ms'],2))" "$O/ab.json" $pl | tee -a "$O/ab.txt"
done; done
QLDPC_ENGINE=6 timeout -k 10 400 python3 -u bench.py --code LP_Matg8_L30_Dmin20 --steps 2 --warmup 1 --shots 4194304 --fp32-line 0 --no-cpu-baseline > "$O/e6_lp30.json" 2> "$O/e6_lp30.err" || { tail -5 "$O/e6_lp30.err"; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('e6', round(d['value']), round(r['achieved']), round(r['frac'],4), r['traffic'], r['bytes_per_launch'], round(r['traffic']/r['bytes_per_launch'],3))" "$O/e6_lp30.json"
timeout -k 10 300 python -u bench.py --workload phenl --precision 32 --steps 5 --warmup 1 > "$O/phenl32.json" 2> "$O/phenl32.err" || { tail "$O/phenl32.err"; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('phenl fp32', round(d['value']), round(r['frac'],4), r['kernel'], round(r['kernel_ms'],2))" "$O/phenl32.json"
