#!/bin/bash
# fp32 space-time byte-F family (config 5, 2 decodes per CU) + engine 6 with 32-bit decision-word
# loads: parity tests, then config 5 fp32 / fp64 lines and the engine-6 LP L30 line.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r03_stfb
mkdir -p "$O"
cd "$R" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_phenl.py tests/test_gpu_hbm.py -x -v --timeout 250 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -3 "$O/pytest.log"
for pr in 32 64; do for fb in 1 0; do
  [ $pr = 64 ] && [ $fb = 0 ] && continue
  QLDPC_E3_FB=$fb timeout -k 10 300 python -u bench.py --workload phenl --precision $pr --steps 5 --warmup 1 > "$O/phenl${pr}_fb$fb.json" 2> "$O/phenl${pr}_fb$fb.err" || { tail "$O/phenl${pr}_fb$fb.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], round(d['value']), round(r['frac'],4), r['kernel'], round(r['kernel_ms'],2))" "$O/phenl${pr}_fb$fb.json" "fp$pr fb=$fb"
done; done
QLDPC_ENGINE=6 timeout -k 10 400 python3 -u bench.py --code LP_Matg8_L30_Dmin20 --steps 2 --warmup 1 --shots 4194304 --fp32-line 0 --no-cpu-baseline > "$O/e6_lp30.json" 2> "$O/e6_lp30.err" || { tail -5 "$O/e6_lp30.err"; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('e6', round(d['value']), round(r['achieved']), round(r['frac'],4), r['traffic'], r['bytes_per_launch'], round(r['traffic']/r['bytes_per_launch'],3))" "$O/e6_lp30.json"
