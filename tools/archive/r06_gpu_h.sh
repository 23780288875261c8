#!/bin/bash
# Round 6 pass H: narrow waves in the fp64 space-time m2s family (config 5).  The config-5 parity
# tests on the current tree, then config 5 at eval_p 0.06 / 0.005 with QLDPC_NW=1 (default) and
# QLDPC_NW=0 (the pre-narrow slot plan) on the same box, then the SQ counters with narrow waves.
#   bash tools/r06_gpu_h.sh OUTDIR
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r06h}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_phenl.py tests/test_gpu_golden.py tests/test_gpu_hbm.py \
  > "$O/pytest.out" 2>&1 || { echo "pytest failed"; tail -40 "$O/pytest.out"; exit 1; }
tail -2 "$O/pytest.out"
line() {  # tag, env..., bench args
  local tag=$1; shift
  timeout -k 10 240 env "$@" > "$O/$tag.json" 2> "$O/$tag.err" || { echo "$tag failed"; tail -5 "$O/$tag.err"; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('$tag', round(d['value']), r.get('kernel_ms'), r.get('frac'), r.get('kernel','')[:70])"
}
for NW in 1 0 1; do
  line st06_nw$NW QLDPC_NW=$NW python -u bench.py --workload phenl --p 0.06 --steps 3 --warmup 1 --no-cpu-baseline --pmc-traffic 0 || exit 1
  line st005_nw$NW QLDPC_NW=$NW python -u bench.py --workload phenl --p 0.005 --steps 3 --warmup 1 --no-cpu-baseline --pmc-traffic 0 || exit 1
done
bash tools/r06_st_pmc.sh "${1:-r06h}/st" 0.06 > "$O/st_pmc.out" 2>&1 || { echo "st pmc failed"; tail -5 "$O/st_pmc.out"; exit 1; }
tail -25 "$O/st_pmc.out"
