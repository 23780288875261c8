#!/bin/bash
# Round 6 pass F: engine-3 parity tests on the tree with the check-phase row pointers / kept V-slot
# addresses / no static LDS, then A/B against the previous library (QLDPC_LIB=$2) on the same box:
# headline (hgp_34_n1600 fp64), LP L30 fp64 (config 4, m2s8 family) and config 5 (p = 0.06, 0.005).
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r06f}
BASE=${2:-}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_phenl.py tests/test_gpu_golden.py tests/test_gpu_m2s.py tests/test_gpu_m2s8.py tests/test_gpu_parity.py \
  > "$O/pytest.out" 2>&1 || { echo "pytest failed"; tail -40 "$O/pytest.out"; exit 1; }
tail -2 "$O/pytest.out"
line() {  # tag, env..., -- bench args
  local tag=$1; shift
  timeout -k 10 240 env "$@" > "$O/$tag.json" 2> "$O/$tag.err" || { echo "$tag failed"; tail -5 "$O/$tag.err"; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('$tag', round(d['value']), r.get('kernel_ms'), r.get('frac'), r.get('kernel','')[:60])"
}
for L in new base; do
  if [ $L = base ]; then [ -n "$BASE" ] || break; E="QLDPC_LIB=$BASE"; else E="QLDPC_X=0"; fi
  line head_$L $E python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --pmc-traffic 0 --fp32-line 0 || exit 1
  line lp30_$L $E python -u bench.py --code LP_Matg8_L30_Dmin20 --steps 5 --warmup 2 --no-cpu-baseline --pmc-traffic 0 --fp32-line 0 || exit 1
  line st06_$L $E python -u bench.py --workload phenl --p 0.06 --steps 3 --warmup 1 --no-cpu-baseline --pmc-traffic 0 || exit 1
  line st005_$L $E python -u bench.py --workload phenl --p 0.005 --steps 3 --warmup 1 --no-cpu-baseline --pmc-traffic 0 || exit 1
done
