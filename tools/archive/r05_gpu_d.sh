#!/bin/bash
# Round 5 GPU pass D: the blocked OSD elimination (QLDPC_OSD_PNL=3) against the host stage / oracle,
# then BP+OSD shot-loop timing with and without it.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r05d}
mkdir -p "$O"
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local n=$1 t=$2
  shift 2
  echo "== $n" >&2
  timeout -k 10 "$t" "$@" > "$O/$n.out" 2> "$O/$n.err" || { echo "step $n failed ($?)"; tail -40 "$O/$n.out"; tail -5 "$O/$n.err"; exit 1; }
}
step pytest_blk 600 python -u -m pytest tests/test_gpu_bposd.py -x -v -k "blk" --timeout 300 --timeout-method thread
tail -3 "$O/pytest_blk.out"
step bposd_default 300 python -u bench.py --workload bposd --p 0.04 --steps 2 --warmup 1 --no-cpu-baseline
QLDPC_OSD_PNL=3 step bposd_blk 300 python -u bench.py --workload bposd --p 0.04 --steps 2 --warmup 1 --no-cpu-baseline
QLDPC_OSD_PNL=3 step bposd_blk_n225 300 python -u bench.py --workload bposd --code hgp_34_n225 --p 0.06 --steps 2 --warmup 1 --no-cpu-baseline
step bposd_default_n225 300 python -u bench.py --workload bposd --code hgp_34_n225 --p 0.06 --steps 2 --warmup 1 --no-cpu-baseline
python3 - "$O" <<'PY'
import json, sys, os
for f in ("bposd_default", "bposd_blk", "bposd_default_n225", "bposd_blk_n225"):
    d = json.loads(open(os.path.join(sys.argv[1], f + ".out")).read().strip().split("\n")[-1])
    r = d["roofline"] or {}
    print(f, round(d["value"]), "LER", d["logical_error_rate"], "osd kernel ms/4096", r.get("kernel_ms"), "us/syn", r.get("us_per_syndrome_chip"))
PY
echo "done: $O"
