#!/bin/bash
# Round 6 pass D: product-sum soft output / BP+OSD tests; config-5 one-word family with check
# labelling (QLDPC_LABEL=1) A/B against the default on the same box.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r06d}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v -x --timeout 300 --timeout-method thread tests/test_gpu_product_sum.py tests/test_gpu_bposd.py \
  > "$O/pytest.out" 2>&1 || { echo "pytest failed"; tail -40 "$O/pytest.out"; exit 1; }
tail -2 "$O/pytest.out"; grep "ulp" "$O/pytest.out" | head
for L in 0 1; do
  QLDPC_LABEL=$L timeout -k 10 200 python -u bench.py --workload phenl --p 0.06 --steps 3 --warmup 1 --no-cpu-baseline --pmc-traffic 0 \
    > "$O/phenl_label$L.json" 2> "$O/phenl_label$L.err" || { echo "phenl failed"; tail -5 "$O/phenl_label$L.err"; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/phenl_label$L.json').read().strip().splitlines()[-1]); r=d['roofline']; print('label $L', round(d['value']), r['kernel_ms'], round(r['frac'],4))"
done
