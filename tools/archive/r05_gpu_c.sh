#!/bin/bash
# Round 5 GPU pass C: held-out notebook-pin counts, the default bench on the new roofline basis,
# config-5 lines at eval_p 0.005 / 0.06 with LDS PMC traffic, the circuit loop after the tally fix
# (tests + bench), the small-graph decoder probe.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r05c}
mkdir -p "$O"
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local n=$1 t=$2
  shift 2
  echo "== $n" >&2
  timeout -k 10 "$t" "$@" > "$O/$n.out" 2> "$O/$n.err" || { echo "step $n failed ($?)"; tail -40 "$O/$n.out"; tail -5 "$O/$n.err"; exit 1; }
}
step pin_heldout 600 python -u tools/notebook_pin_run.py --hyp adopted --seed $((0x55eed)) --mult 25 --counts-only --out "$O/pin_heldout_counts.json"
step circ_tests 600 python -u -m pytest tests/test_gpu_circuit.py -x -q --timeout 300 --timeout-method thread
step circuit 300 python -u bench.py --workload circuit --steps 3 --warmup 1
step probe_small 300 python -u tools/dev/probe_small_dec.py
step bench 600 python -u bench.py
step phenl_p006 300 python -u bench.py --workload phenl --p 0.06 --steps 3 --warmup 1 --no-cpu-baseline
step phenl_p0005 300 python -u bench.py --workload phenl --p 0.005 --steps 3 --warmup 1 --no-cpu-baseline
cat "$O/bench.out" "$O/circuit.out"
echo "done: $O"
