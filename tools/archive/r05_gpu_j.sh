#!/bin/bash
# Round 5 GPU pass J: sensitivity of the lean OSD loop to its row-update VALU work (diagnostic
# build with every row xor done three times) -- BP+OSD bench A/B on one box.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r05j}
mkdir -p "$O"
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local n=$1 t=$2
  shift 2
  echo "== $n" >&2
  timeout -k 10 "$t" "$@" > "$O/$n.out" 2> "$O/$n.err" || { echo "step $n failed ($?)"; tail -40 "$O/$n.out"; tail -5 "$O/$n.err"; exit 1; }
}
QLDPC_LIB=$R/qldpc_fault_tolerance_amd/libqldpc_hip_x3.so step bposd_x3 300 python -u bench.py --workload bposd --p 0.04 --steps 2 --warmup 1 --no-cpu-baseline
step bposd_default 300 python -u bench.py --workload bposd --p 0.04 --steps 2 --warmup 1 --no-cpu-baseline
QLDPC_LIB=$R/qldpc_fault_tolerance_amd/libqldpc_hip_x3.so step bposd_x3b 300 python -u bench.py --workload bposd --p 0.04 --steps 2 --warmup 1 --no-cpu-baseline
python3 - "$O" <<'PY'
import json, sys, os
for f in ("bposd_default", "bposd_x3", "bposd_x3b"):
    d = json.loads(open(os.path.join(sys.argv[1], f + ".out")).read().strip().split("\n")[-1])
    r = d["roofline"] or {}
    print(f, round(d["value"]), "LER", d["logical_error_rate"], "osd kernel ms/4096", r.get("kernel_ms"))
PY
