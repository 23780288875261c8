#!/bin/bash
# c2s vs m2s: phase stamps (diagnostic build) and SQ counters of the c2s kernel.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r03_c2s2
mkdir -p "$O"
cd "$R" || exit 1
for cfg in "QLDPC_C2S=1" "QLDPC_C2S=0"; do
  env $cfg timeout -k 10 200 python3 -u bench.py --steps 4 --warmup 1 --pmc-traffic 0 --fp32-line 0 --no-cpu-baseline > "$O/ab.json" 2> "$O/ab.err" || { tail -5 "$O/ab.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), round(d['roofline']['frac'],4), round(d['roofline']['kernel_ms'],2), d['roofline']['kernel'])" "$O/ab.json" "$cfg" | tee -a "$O/ab.txt"
done
for c in 1 0; do
  QLDPC_C2S=$c QLDPC_LIB=$R/qldpc_fault_tolerance_amd/libqldpc_hip_stamps.so timeout -k 10 200 python3 -u tools/stamps.py hgp_34_n1600 0.06 65536 0 64 Total > "$O/stamps_c2s$c.txt" 2>&1 || { tail -5 "$O/stamps_c2s$c.txt"; exit 1; }
  echo "== c2s=$c"; tail -9 "$O/stamps_c2s$c.txt"
done
QLDPC_C2S=1 timeout -k 10 500 bash tools/pmc_passes.sh "gpurun_out/r03_c2s2/pmc64" hgp_34_n1600 0.06 65536 0 64 Total > "$O/pmc64.log" 2>&1 || { tail "$O/pmc64.log"; exit 1; }
python3 tools/pmc_summary2.py "$O/pmc64" > "$O/pmc64_summary.txt" 2>&1; tail -28 "$O/pmc64_summary.txt"
