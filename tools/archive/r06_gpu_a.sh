#!/bin/bash
# Round 6 pass A: the one-word fp64 space-time family (engine id 111313) and the ADVICE r05 fixes.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r06a}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_phenl.py tests/test_gpu_golden.py tests/test_gpu_hbm.py tests/test_gpu_circuit.py \
  > "$O/pytest.out" 2>&1 || { echo "pytest failed"; tail -40 "$O/pytest.out"; exit 1; }
tail -3 "$O/pytest.out"
for P in 0.06 0.005; do
  timeout -k 10 300 python -u bench.py --workload phenl --p $P --steps 3 --warmup 1 --no-cpu-baseline \
    > "$O/phenl_p$P.json" 2> "$O/phenl_p$P.err" || { echo "phenl $P failed"; tail -5 "$O/phenl_p$P.err"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/phenl_p$P.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$P', round(d['value']), r['kernel_ms'], round(r['frac'],4), r['traffic_over_algorithmic'], r['lds_pmc'] and r['lds_pmc']['bank_conflict_share'], r['kernel'])"
done
QLDPC_M2ST=0 timeout -k 10 300 python -u bench.py --workload phenl --p 0.06 --steps 3 --warmup 1 --no-cpu-baseline --pmc-traffic 0 \
  > "$O/phenl_old_p0.06.json" 2> "$O/phenl_old.err" || { echo "phenl old failed"; tail -5 "$O/phenl_old.err"; exit 1; }
python3 -c "import json; d=json.loads(open('$O/phenl_old_p0.06.json').read().strip().splitlines()[-1]); r=d['roofline']; print('old 0.06', round(d['value']), r['kernel_ms'], round(r['frac'],4), r['kernel'])"
