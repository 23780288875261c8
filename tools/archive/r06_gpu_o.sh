#!/bin/bash
# Round 6 pass O: the small lifted-product codes on the rows-of-8 family at 128 threads.  Their parity
# tests (and the rest of the m2s8 / parity suites), the route survey, then hz decode timing on the new
# route against the old one (QLDPC_M2S8_SMALL=0: engine 2).
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r06o}
mkdir -p "$O"
timeout -k 10 200 python -u tools/route_survey.py 64 > "$O/route64.jsonl" 2> "$O/route64.err" || { echo "survey failed"; tail -5 "$O/route64.err"; exit 1; }
timeout -k 10 900 python -u -m pytest -q -x --timeout 400 --timeout-method thread tests/test_gpu_m2s8.py tests/test_gpu_parity.py tests/test_gpu_bposd.py \
  > "$O/pytest.out" 2>&1 || { echo "pytest failed"; tail -40 "$O/pytest.out"; exit 1; }
tail -2 "$O/pytest.out"
for spec in "LP_Matg8_L16_Dmin12 0" "LP_Matg8_L21_Dmin16 0" "LP_Matg8_L30_Dmin20 0"; do
  for T in 1 0; do
    for P in 0.02 0.06; do
      # shellcheck disable=SC2086
      timeout -k 10 200 env QLDPC_M2S8_SMALL=$T python -u tools/st_route_ab.py $spec $P 131072 >> "$O/route.jsonl" 2>> "$O/route.err" \
        || { echo "failed: $spec $T $P"; tail -5 "$O/route.err"; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/route.jsonl').read().splitlines()[-1]); print(d['code'], d['t0'], d['p'], 'SMALL=$T', d['engine'], d['kernel_id'], d['threads'], d['vpl'], round(d['ms'], 3), d['mean_iters'])"
    done
  done
done
