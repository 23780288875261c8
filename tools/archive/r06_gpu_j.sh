#!/bin/bash
# Round 6 pass J: SIMD-balanced wave placement of config 5's space-time decoder (QLDPC_NW_BAL=1, the
# default) against wave order (QLDPC_NW_BAL=0), interleaved on one box, after the config-5 parity tests.
#   bash tools/r06_gpu_j.sh OUTDIR
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r06j}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_phenl.py tests/test_gpu_golden.py tests/test_gpu_hbm.py \
  > "$O/pytest.out" 2>&1 || { echo "pytest failed"; tail -40 "$O/pytest.out"; exit 1; }
tail -2 "$O/pytest.out"
line() {  # tag, env..., bench args
  local tag=$1; shift
  timeout -k 10 240 env "$@" > "$O/$tag.json" 2> "$O/$tag.err" || { echo "$tag failed"; tail -5 "$O/$tag.err"; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('$tag', round(d['value']), r.get('kernel_ms'), r.get('frac'))"
}
for i in 1 2; do
  for B in 1 0; do
    line st06_bal${B}_$i QLDPC_NW_BAL=$B python -u bench.py --workload phenl --p 0.06 --steps 3 --warmup 1 --no-cpu-baseline --pmc-traffic 0 || exit 1
    line st005_bal${B}_$i QLDPC_NW_BAL=$B python -u bench.py --workload phenl --p 0.005 --steps 3 --warmup 1 --no-cpu-baseline --pmc-traffic 0 || exit 1
  done
done
