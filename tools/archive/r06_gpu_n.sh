#!/bin/bash
# Round 6 pass N: the widened fp64 tail-family routing.  The route survey, the space-time parity tests,
# then each re-routed graph timed on its new route against the pre-round-6 route (QLDPC_E3_TAIL64=0).
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r06n}
mkdir -p "$O"
timeout -k 10 200 python -u tools/route_survey.py 64 > "$O/route64.jsonl" 2> "$O/route64.err" || { echo "survey failed"; tail -5 "$O/route64.err"; exit 1; }
timeout -k 10 900 python -u -m pytest -q -x --timeout 400 --timeout-method thread tests/test_gpu_st_m2s.py tests/test_gpu_phenl.py tests/test_gpu_golden.py \
  > "$O/pytest.out" 2>&1 || { echo "pytest failed"; tail -40 "$O/pytest.out"; exit 1; }
tail -2 "$O/pytest.out"
for spec in "hgp_34_n625 3" "GenBicycleA4 2" "GenBicycleA4 3" "GenBicycleA3 4" "GenBicycleA3 5" "hgp_34_n1600 2"; do
  for T in 1 0; do
    for P in 0.01 0.05; do
      # shellcheck disable=SC2086
      timeout -k 10 200 env QLDPC_E3_TAIL64=$T python -u tools/st_route_ab.py $spec $P 32768 >> "$O/route.jsonl" 2>> "$O/route.err" \
        || { echo "failed: $spec $T $P"; tail -5 "$O/route.err"; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/route.jsonl').read().splitlines()[-1]); print(d['code'], d['t0'], d['p'], 'TAIL64=$T', d['engine'], d['kernel_id'], d['threads'], d['vpl'], round(d['ms'], 2))"
    done
  done
done
