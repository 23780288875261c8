#!/bin/bash
# Round 6 pass G: engine-3 parity tests on the current tree, then the headline, LP L30 and config 5
# lines with the in-tree library and with each A/B library given (QLDPC_LIB), on the same box.
#   bash tools/r06_gpu_g.sh OUTDIR [tag=lib.so ...]
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r06g}
shift
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_phenl.py tests/test_gpu_golden.py tests/test_gpu_m2s.py tests/test_gpu_m2s8.py tests/test_gpu_parity.py tests/test_gpu_bposd.py \
  > "$O/pytest.out" 2>&1 || { echo "pytest failed"; tail -40 "$O/pytest.out"; exit 1; }
tail -2 "$O/pytest.out"
line() {  # tag, env..., bench args
  local tag=$1; shift
  timeout -k 10 240 env "$@" > "$O/$tag.json" 2> "$O/$tag.err" || { echo "$tag failed"; tail -5 "$O/$tag.err"; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('$tag', round(d['value']), r.get('kernel_ms'), r.get('frac'), r.get('kernel','')[:60])"
}
for spec in new=in-tree "$@"; do
  L=${spec%%=*}; LIB=${spec#*=}
  if [ "$LIB" = in-tree ]; then E="QLDPC_X=0"; else E="QLDPC_LIB=$R/$LIB"; fi
  line head_$L $E python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --pmc-traffic 0 --fp32-line 0 || exit 1
  line lp30_$L $E python -u bench.py --code LP_Matg8_L30_Dmin20 --steps 5 --warmup 2 --no-cpu-baseline --pmc-traffic 0 --fp32-line 0 || exit 1
  line st06_$L $E python -u bench.py --workload phenl --p 0.06 --steps 3 --warmup 1 --no-cpu-baseline --pmc-traffic 0 || exit 1
  line st005_$L $E python -u bench.py --workload phenl --p 0.005 --steps 3 --warmup 1 --no-cpu-baseline --pmc-traffic 0 || exit 1
done
