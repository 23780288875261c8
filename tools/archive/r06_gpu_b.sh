#!/bin/bash
# Round 6 pass B: the full GPU suite and smoke on the current tree, then config 5's lines (one-word
# fp64 space-time family, with LDS PMC) and the two-word family on the same box for A/B.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r06b}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > "$O/pytest_gpu.out" 2> "$O/pytest_gpu.err" || { echo "suite failed"; tail -40 "$O/pytest_gpu.out"; exit 1; }
tail -2 "$O/pytest_gpu.out"
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.out" 2>&1 || { echo "smoke failed"; tail -5 "$O/smoke.out"; exit 1; }
tail -1 "$O/smoke.out"
for P in 0.06 0.005; do
  timeout -k 10 200 python -u bench.py --workload phenl --p $P --steps 3 --warmup 1 --no-cpu-baseline \
    > "$O/phenl_p$P.json" 2> "$O/phenl_p$P.err" || { echo "phenl $P failed"; tail -5 "$O/phenl_p$P.err"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/phenl_p$P.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$P', round(d['value']), r['kernel_ms'], round(r['frac'],4), r['traffic_over_algorithmic'], r['lds_pmc'] and r['lds_pmc']['bank_conflict_share'], r['kernel'])"
done
QLDPC_M2ST=0 timeout -k 10 200 python -u bench.py --workload phenl --p 0.06 --steps 3 --warmup 1 --no-cpu-baseline --pmc-traffic 0 \
  > "$O/phenl_old_p0.06.json" 2> "$O/phenl_old.err" || { echo "phenl old failed"; tail -5 "$O/phenl_old.err"; exit 1; }
python3 -c "import json; d=json.loads(open('$O/phenl_old_p0.06.json').read().strip().splitlines()[-1]); r=d['roofline']; print('old 0.06', round(d['value']), r['kernel_ms'], round(r['frac'],4), r['kernel'])"
