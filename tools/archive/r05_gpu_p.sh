#!/bin/bash
# Round 5 GPU pass P: the wave-per-syndrome first-min kernel: parity tests and probes.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r05p}
mkdir -p "$O"
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local n=$1 t=$2
  shift 2
  echo "== $n" >&2
  timeout -k 10 "$t" "$@" > "$O/$n.out" 2> "$O/$n.err" || { echo "step $n failed ($?)"; tail -40 "$O/$n.out"; tail -5 "$O/$n.err"; exit 1; }
}
step pytest_fm 600 python -u -m pytest tests/test_gpu_phenl.py -x -q -k "firstmin or phen_single" --timeout 300 --timeout-method thread
tail -2 "$O/pytest_fm.out"
step probe 300 python -u tools/dev/probe_firstmin.py 65536
QLDPC_FM_WAVE=0 step probe_wg 300 python -u tools/dev/probe_firstmin.py 65536
step probe_phen 600 python -u tools/dev/probe_phen_firstmin.py hgp_34_n625 65536 5
cat "$O/probe.out" "$O/probe_wg.out" "$O/probe_phen.out"
