#!/bin/bash
# Round 6 pass P: the full GPU suite and smoke on the tree after the routing changes, plus the fp32
# route survey.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r06p}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > "$O/pytest_gpu.out" 2> "$O/pytest_gpu.err" \
  || { echo "pytest failed"; grep -E "FAILED|Error" "$O/pytest_gpu.out" | head -20; tail -5 "$O/pytest_gpu.out"; exit 1; }
tail -2 "$O/pytest_gpu.out"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.out" 2>&1 || { echo "smoke failed"; tail -5 "$O/smoke.out"; exit 1; }
cat "$O/smoke.out" | tail -1
timeout -k 10 200 python -u tools/route_survey.py 32 > "$O/route32.jsonl" 2> "$O/route32.err" || { echo "survey failed"; tail -5 "$O/route32.err"; exit 1; }
python3 -c "
import json
for l in open('$O/route32.jsonl'):
    d = json.loads(l)
    if d.get('engine') in (2, 6) or 'error' in d: print(d['code'], d['graph'], d['m'], d['n'], d['max_row'], d['max_col'], d.get('engine'), d.get('threads'), d.get('vars_per_thread'), d.get('error', ''))
"
