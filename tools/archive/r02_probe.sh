#!/bin/bash
# r02 baseline probe: fp64 headline geometry sweep + kernel trace.  Run ON the GPU box.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/${1:-r02_probe}
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R" || exit 1
for tb in 0 512 1024; do
  echo "== fp64 TB=$tb"
  QLDPC_TB=$tb timeout -k 10 240 python3 -u bench.py --precision 64 --steps 3 --warmup 1 --shots 131072 --no-cpu-baseline > "$O/b64_tb$tb.json" 2> "$O/b64_tb$tb.err" || { tail "$O/b64_tb$tb.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['roofline']['frac'], d['roofline']['kernel'], d['mean_iters_per_decode'])" "$O/b64_tb$tb.json"
done
cd /tmp || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace64" -o run -- \
  python3 "$R/bench.py" --precision 64 --steps 2 --warmup 1 --shots 131072 --no-cpu-baseline > "$O/trace64.json" 2> "$O/trace64.err" || exit 1
echo done
