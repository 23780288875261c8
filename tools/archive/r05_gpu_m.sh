#!/bin/bash
# Round 5 GPU pass M: config-5 space-time fp64 kernel geometry A/B (threads per decode / variables
# per thread through QLDPC_TB): default 1024 x 6 vs 704 x 8 vs 832 x 7.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r05m}
mkdir -p "$O"
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local n=$1 t=$2
  shift 2
  echo "== $n" >&2
  timeout -k 10 "$t" "$@" > "$O/$n.out" 2> "$O/$n.err" || { echo "step $n failed ($?)"; tail -20 "$O/$n.out"; tail -5 "$O/$n.err"; exit 1; }
}
step ph_default 300 python -u bench.py --workload phenl --p 0.06 --steps 1 --warmup 1 --no-cpu-baseline
QLDPC_TB=704 step ph_tb704 300 python -u bench.py --workload phenl --p 0.06 --steps 1 --warmup 1 --no-cpu-baseline
QLDPC_TB=832 step ph_tb832 300 python -u bench.py --workload phenl --p 0.06 --steps 1 --warmup 1 --no-cpu-baseline
python3 - "$O" <<'PY'
import json, sys, os
for f in ("ph_default", "ph_tb704", "ph_tb832"):
    d = json.loads(open(os.path.join(sys.argv[1], f + ".out")).read().strip().split("\n")[-1])
    r = d["roofline"] or {}
    print(f, round(d["value"]), "LER", d["logical_error_rate"], "kernel", r.get("kernel"), "kernel_ms", r.get("kernel_ms"), "frac", r.get("frac"))
PY
