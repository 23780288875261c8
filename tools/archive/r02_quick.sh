#!/bin/bash
# Quick GPU iteration: [pytest -k filter] then a short fp64 bench.  Run ON the GPU box:
#   tools/r02_quick.sh <tag> "<pytest -k expr or ->" "<bench args>"
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$1
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R" || exit 1
if [ "$2" != "-" ]; then
  timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$2" > "$O/pytest.log" 2>&1
  rc=$?; tail -4 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python3 -u bench.py $3 > "$O/bench.json" 2> "$O/bench.err" || { tail "$O/bench.err"; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(d['value'], d['dtype'], r['frac'], r['kernel'], r['kernel_ms'])" "$O/bench.json"
