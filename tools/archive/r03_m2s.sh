#!/bin/bash
# m2s family: its parity tests, the whole GPU suite, then an interleaved A/B of the headline
# (default = m2s PF 2; QLDPC_M2S=0 = the two-word family; libqldpc_hip_pf1.so = m2s PF 1).
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/${TAG:-r03_m2s}
mkdir -p "$O"
cd "$R" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_m2s.py -x -v --timeout 200 --timeout-method thread > "$O/pytest_m2s.log" 2>&1 || { tail -40 "$O/pytest_m2s.log"; exit 1; }
tail -3 "$O/pytest_m2s.log"
if [ "${FULL:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
  tail -3 "$O/pytest_gpu.log"
fi
for r in 1 2; do
  for cfg in "QLDPC_M2S=1" "QLDPC_M2S=0" "QLDPC_LIB=$R/qldpc_fault_tolerance_amd/libqldpc_hip_pf1.so"; do
    env $cfg timeout -k 10 200 python3 -u bench.py --steps 4 --warmup 1 --pmc-traffic 0 --fp32-line 0 --no-cpu-baseline > "$O/ab.json" 2> "$O/ab.err" || { tail -5 "$O/ab.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), round(d['roofline']['frac'],4), d['roofline']['kernel'], round(d['roofline']['kernel_ms'],2))" "$O/ab.json" "$cfg" | tee -a "$O/ab.txt"
  done
done
