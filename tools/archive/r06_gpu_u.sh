#!/bin/bash
# Round 6 pass U: paired rows in the space-time family's check phase (QLDPC_M2S_ROWPAIR = chunks of the
# second row loaded before the first is reduced; the product library is built with 2).  Parity tests on
# the product library, then config 5 at eval_p 0.06 / 0.005 with each library, interleaved.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r06u}
mkdir -p "$O"
timeout -k 10 700 python -u -m pytest -q -x --timeout 400 --timeout-method thread tests/test_gpu_st_m2s.py tests/test_gpu_phenl.py tests/test_gpu_golden.py \
  > "$O/pytest.out" 2>&1 || { echo "pytest failed"; tail -40 "$O/pytest.out"; exit 1; }
tail -2 "$O/pytest.out"
for i in 1 2; do
  for L in prod rp0 rp1 rp3; do
    if [ $L = prod ]; then E="QLDPC_X=0"; else E="QLDPC_LIB=$R/qldpc_fault_tolerance_amd/libqldpc_hip_$L.so"; fi
    for P in 0.06 0.005; do
      timeout -k 10 240 env $E python -u bench.py --workload phenl --p $P --steps 2 --warmup 1 --no-cpu-baseline --pmc-traffic 0 > "$O/${L}_${P}_$i.json" 2> "$O/${L}_${P}_$i.err" || { echo "$L $P failed"; tail -5 "$O/${L}_${P}_$i.err"; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/${L}_${P}_$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$L', '$P', round(r['kernel_ms'], 3), round(r['frac'], 4), round(d['value']))"
    done
  done
done
