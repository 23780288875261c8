#!/bin/bash
# Round 6 pass R: the lifted-product [h | I] graphs on the degree-5 family with 5-chunk rows.  Parity
# tests, then decode timing against the old route (QLDPC_F64W=0 QLDPC_D5_256=0: engine 2).
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r06r}
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest -q -x --timeout 400 --timeout-method thread tests/test_gpu_m2s8.py tests/test_gpu_parity.py tests/test_gpu_phenl.py \
  > "$O/pytest.out" 2>&1 || { echo "pytest failed"; tail -40 "$O/pytest.out"; exit 1; }
tail -2 "$O/pytest.out"
for spec in "LP_Matg8_L30_Dmin20 1" "LP_Matg8_L16_Dmin12 1" "LP_Matg8_L21_Dmin16 1"; do
  for T in 1 0; do
    for P in 0.02 0.06; do
      # shellcheck disable=SC2086
      timeout -k 10 200 env QLDPC_F64W=$T QLDPC_D5_256=$T python -u tools/st_route_ab.py $spec $P 131072 >> "$O/route.jsonl" 2>> "$O/route.err" \
        || { echo "failed: $spec $T $P"; tail -5 "$O/route.err"; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/route.jsonl').read().splitlines()[-1]); print(d['code'], d['t0'], d['p'], 'NEW=$T', d['engine'], d['kernel_id'], d['threads'], d['vpl'], round(d['ms'], 3), d['mean_iters'])"
    done
  done
done
