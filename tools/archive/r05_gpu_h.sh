#!/bin/bash
# Round 5 GPU pass H: the column-window OSD elimination (rows hold the first rank + nh + slack
# positions only; overruns redone at full width): BP+OSD parity tests, stamps, BP+OSD bench
# window (default) vs full width (QLDPC_OSD_WIN=0) vs one workgroup per CU (QLDPC_OSD_WPE=3).
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r05h}
mkdir -p "$O"
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local n=$1 t=$2
  shift 2
  echo "== $n" >&2
  timeout -k 10 "$t" "$@" > "$O/$n.out" 2> "$O/$n.err" || { echo "step $n failed ($?)"; tail -40 "$O/$n.out"; tail -5 "$O/$n.err"; exit 1; }
}
step pytest_bposd 900 python -u -m pytest tests/test_gpu_bposd.py -x -v --timeout 300 --timeout-method thread
tail -2 "$O/pytest_bposd.out"
L=$R/qldpc_fault_tolerance_amd/libqldpc_hip_stamps.so
QLDPC_LIB=$L step stamps_win 300 python -u tools/osd_stamps.py hgp_34_n1600 0.04 65536
cat "$O/stamps_win.out"
step bposd_win 300 python -u bench.py --workload bposd --p 0.04 --steps 2 --warmup 1 --no-cpu-baseline
QLDPC_OSD_WIN=0 step bposd_full 300 python -u bench.py --workload bposd --p 0.04 --steps 2 --warmup 1 --no-cpu-baseline
QLDPC_OSD_WPE=3 step bposd_wpe3 300 python -u bench.py --workload bposd --p 0.04 --steps 2 --warmup 1 --no-cpu-baseline
python3 - "$O" <<'PY'
import json, sys, os
for f in ("bposd_win", "bposd_full", "bposd_wpe3"):
    d = json.loads(open(os.path.join(sys.argv[1], f + ".out")).read().strip().split("\n")[-1])
    r = d["roofline"] or {}
    print(f, round(d["value"]), "LER", d["logical_error_rate"], "osd kernel ms/4096", r.get("kernel_ms"), "us/syn", r.get("us_per_syndrome_chip"))
PY
echo "done: $O"
