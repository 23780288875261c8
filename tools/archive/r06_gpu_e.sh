#!/bin/bash
# Round 6 pass E: product-sum soft output / BP+OSD and circuit tests; the circuit loop's kernel traces
# with the geometric-skip and keyed DEM samplers on the demo DEM (666 mechanisms) and on toric d13
# with every noise source (12,506 mechanisms); config-5 check-labelling A/B.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r06e}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_product_sum.py tests/test_gpu_circuit.py tests/test_gpu_bposd.py \
  > "$O/pytest.out" 2>&1 || { echo "pytest failed"; tail -40 "$O/pytest.out"; exit 1; }
tail -2 "$O/pytest.out"
cd /tmp
for cfg in "3 cx" "13 all"; do
  set -- $cfg
  for S in skip keyed; do
    tag=d$1_$S
    timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/tr_$tag" -o t -- \
      python3 "$R/bench.py" --workload circuit --dem-d $1 --circuit-noise $2 --sampler $S --steps 2 --warmup 1 --no-cpu-baseline \
      > "$O/circ_$tag.json" 2> "$O/circ_$tag.err" || { echo "circuit $tag failed"; tail -5 "$O/circ_$tag.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/circ_$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['value']), d['config']['dem_mechanisms'], d['logical_error_rate'])"
    python3 - "$O/tr_$tag" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)
rows = list(csv.DictReader(open(f[0])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:5]:
    print("   %-60s %6.2f%% %10.3f ms" % (r["Name"][:60], 100 * float(r["TotalDurationNs"]) / tot, float(r["TotalDurationNs"]) / 1e6))
PY
  done
done
cd "$R"
for L in 0 1; do
  QLDPC_LABEL=$L timeout -k 10 200 python -u bench.py --workload phenl --p 0.06 --steps 3 --warmup 1 --no-cpu-baseline --pmc-traffic 0 \
    > "$O/phenl_label$L.json" 2> "$O/phenl_label$L.err" || { echo "phenl failed"; tail -5 "$O/phenl_label$L.err"; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/phenl_label$L.json').read().strip().splitlines()[-1]); r=d['roofline']; print('label $L', round(d['value']), r['kernel_ms'], round(r['frac'],4))"
done
