#!/bin/bash
# fp64 space-time D2K = 1 (engine id 101013): config-5 golden / phenl tests, fp64 config-5 line A/B
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r03_d2k64
mkdir -p "$O"
cd "$R" || exit 1
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_phenl.py tests/test_gpu_golden.py tests/test_gpu_hbm.py > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -2 "$O/pytest.log"
for r in 1 2; do for d in 1 0; do
QLDPC_D2K=$d timeout -k 10 300 python3 -u bench.py --workload phenl --precision 64 --steps 3 --warmup 1 --no-cpu-baseline > "$O/phenl64_d$d.json" 2> "$O/phenl64_d$d.err" || { tail -5 "$O/phenl64_d$d.err"; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('phenl64 d2k', sys.argv[2], round(d['value']), round(r['frac'],4), round(r['kernel_ms'],2), r['kernel'])" "$O/phenl64_d$d.json" $d | tee -a "$O/ab.txt"
done; done
