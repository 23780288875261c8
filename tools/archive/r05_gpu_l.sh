#!/bin/bash
# Round 5 GPU pass L: the lean OSD loop with two rows per thread, two workgroups per CU (QLDPC_OSD_RPT=2):
# parity tests, BP+OSD bench vs one row per thread.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r05l}
mkdir -p "$O"
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local n=$1 t=$2
  shift 2
  echo "== $n" >&2
  timeout -k 10 "$t" "$@" > "$O/$n.out" 2> "$O/$n.err" || { echo "step $n failed ($?)"; tail -40 "$O/$n.out"; tail -5 "$O/$n.err"; exit 1; }
}
step pytest_rpt2 600 python -u -m pytest tests/test_gpu_bposd.py -x -v -k "rpt2" --timeout 300 --timeout-method thread
tail -2 "$O/pytest_rpt2.out"
QLDPC_OSD_RPT=2 step bposd_rpt2 300 python -u bench.py --workload bposd --p 0.04 --steps 2 --warmup 1 --no-cpu-baseline
step bposd_default 300 python -u bench.py --workload bposd --p 0.04 --steps 2 --warmup 1 --no-cpu-baseline
python3 - "$O" <<'PY'
import json, sys, os
for f in ("bposd_default", "bposd_rpt2"):
    d = json.loads(open(os.path.join(sys.argv[1], f + ".out")).read().strip().split("\n")[-1])
    r = d["roofline"] or {}
    print(f, round(d["value"]), "LER", d["logical_error_rate"], "osd kernel ms/4096", r.get("kernel_ms"), "us/syn", r.get("us_per_syndrome_chip"))
PY
echo "done: $O"
