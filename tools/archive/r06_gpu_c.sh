#!/bin/bash
# Round 6 pass C: config 5's lines (one-word fp64 space-time family with LDS PMC; the two-word family
# on the same box for A/B), then the tail of the GPU suite.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r06c}
mkdir -p "$O"
export TMPDIR=/tmp
for P in 0.06 0.005; do
  timeout -k 10 200 python -u bench.py --workload phenl --p $P --steps 3 --warmup 1 --no-cpu-baseline \
    > "$O/phenl_p$P.json" 2> "$O/phenl_p$P.err" || { echo "phenl $P failed"; tail -5 "$O/phenl_p$P.err"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/phenl_p$P.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$P', round(d['value']), r['kernel_ms'], round(r['frac'],4), r['traffic_over_algorithmic'], r['lds_pmc'] and r['lds_pmc']['bank_conflict_share'], r['kernel'])"
done
for P in 0.06 0.005; do
QLDPC_M2ST=0 timeout -k 10 200 python -u bench.py --workload phenl --p $P --steps 3 --warmup 1 --no-cpu-baseline --pmc-traffic 0 \
  > "$O/phenl_old_p$P.json" 2> "$O/phenl_old_p$P.err" || { echo "phenl old failed"; tail -5 "$O/phenl_old_p$P.err"; exit 1; }
python3 -c "import json; d=json.loads(open('$O/phenl_old_p$P.json').read().strip().splitlines()[-1]); r=d['roofline']; print('old $P', round(d['value']), r['kernel_ms'], round(r['frac'],4), r['kernel'])"
done
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_phenl.py tests/test_gpu_product_sum.py tests/test_gpu_simulators.py > "$O/pytest_tail.out" 2>&1 || { echo "pytest failed"; tail -30 "$O/pytest_tail.out"; exit 1; }
tail -2 "$O/pytest_tail.out"
