#!/bin/bash
# Round 6 pass X: absolute row / tail / CS addresses in the two-word check phase (QLDPC_RC_RPTR=1, the
# product library) against the library without them (libqldpc_hip_rc0.so), interleaved: the fp32 line
# of the headline workload, config 5 in fp32, hgp_34_n1225 over two rounds (fp64 two-word tail family)
# and GenBicycleA4 hz (fp64 two-word 103 family) decode timing; parity tests first.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r06x}
mkdir -p "$O"
timeout -k 10 800 python -u -m pytest -q -x --timeout 400 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_phenl.py tests/test_gpu_golden.py tests/test_gpu_st_m2s.py \
  > "$O/pytest.out" 2>&1 || { echo "pytest failed"; tail -40 "$O/pytest.out"; exit 1; }
tail -2 "$O/pytest.out"
for i in 1 2; do
  for L in new rc0; do
    if [ $L = new ]; then E="QLDPC_X=0"; else E="QLDPC_LIB=$R/qldpc_fault_tolerance_amd/libqldpc_hip_rc0.so"; fi
    timeout -k 10 300 env $E python -u bench.py --precision 32 --fp32-line 0 --no-cpu-baseline --pmc-traffic 0 > "$O/f32_${L}_$i.json" 2> "$O/f32_${L}_$i.err" || { echo "f32 $L failed"; tail -5 "$O/f32_${L}_$i.err"; exit 1; }
    timeout -k 10 300 env $E python -u bench.py --workload phenl --precision 32 --p 0.06 --steps 2 --warmup 1 --no-cpu-baseline --pmc-traffic 0 > "$O/st32_${L}_$i.json" 2> "$O/st32_${L}_$i.err" || { echo "st32 $L failed"; tail -5 "$O/st32_${L}_$i.err"; exit 1; }
    for spec in "hgp_34_n1225_q3 2" "GenBicycleA4 0"; do
      # shellcheck disable=SC2086
      timeout -k 10 200 env $E python -u tools/st_route_ab.py $spec 0.05 65536 >> "$O/route_$L.jsonl" 2>> "$O/route.err" || { echo "route $L failed"; exit 1; }
    done
    python3 - "$O" "$L" "$i" <<'PY'
import json, sys
O, L, i = sys.argv[1:]
f = json.loads(open(f"{O}/f32_{L}_{i}.json").read().strip().splitlines()[-1])
st = json.loads(open(f"{O}/st32_{L}_{i}.json").read().strip().splitlines()[-1])
rs = [json.loads(x) for x in open(f"{O}/route_{L}.jsonl").read().splitlines()[-2:]]
print(L, i, "f32", round(f["value"]), round(f["ms_per_step"], 2), "st32", round(st["roofline"]["kernel_ms"], 2),
      " ".join(f"{r['code']}x{r['t0']} {r['kernel_id']} {r['ms']:.2f}" for r in rs))
PY
  done
done
