#!/bin/bash
# Round 6 pass AA: the per-shot class cache of the fused data-error kernel (one Philox draw per shot and
# variable for both sectors).  The fused-MC parity tests, then the headline workload at eval_p 0.02 /
# 0.06 with the product library and the library before the cache (libqldpc_hip_cc0.so), interleaved.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r06aa}
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest -q -x --timeout 400 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_m2s.py tests/test_gpu_m2s8.py tests/test_gpu_golden.py tests/test_gpu_comm.py \
  > "$O/pytest.out" 2>&1 || { echo "pytest failed"; tail -40 "$O/pytest.out"; exit 1; }
tail -2 "$O/pytest.out"
for i in 1 2; do
  for L in new cc0; do
    if [ $L = new ]; then E="QLDPC_X=0"; else E="QLDPC_LIB=$R/qldpc_fault_tolerance_amd/libqldpc_hip_cc0.so"; fi
    for P in 0.02 0.06; do
      timeout -k 10 300 env $E python -u bench.py --p $P --shots 2097152 --steps 4 --warmup 1 --no-cpu-baseline --fp32-line 0 --pmc-traffic 0 > "$O/${L}_${P}_$i.json" 2> "$O/${L}_${P}_$i.err" || { echo "$L $P failed"; tail -5 "$O/${L}_${P}_$i.err"; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/${L}_${P}_$i.json').read().strip().splitlines()[-1]); print('$L', '$P', round(d['value']), round(d['ms_per_step'], 2), d['logical_error_rate'])"
    done
  done
done
