#!/bin/bash
# Interleaved A/B of library variants on config 5 (space-time decoder kernel roofline):
#   tools/r02_phenl_ab.sh <tag> <precision> <p> <rounds> lib1.so lib2.so ...   ("-" = default lib)
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
T=$1; P=$2; EP=$3; N=$4; shift 4
O=$R/gpurun_out/$T
mkdir -p "$O"
cd "$R" || exit 1
for r in $(seq 1 $N); do
  i=0
  for lib in "$@"; do
    i=$((i+1))
    L=""; [ "$lib" != "-" ] && L=$R/qldpc_fault_tolerance_amd/$lib
    QLDPC_LIB=$L timeout -k 10 200 python3 -u bench.py --workload phenl --precision $P --p $EP --shots 65536 --steps 2 --warmup 1 --pmc-traffic 0 --fp32-line 0 --no-cpu-baseline > "$O/r${r}_$i.json" 2> "$O/r${r}_$i.err" || { tail -3 "$O/r${r}_$i.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), round(d['roofline']['frac'],4), round(d['roofline']['kernel_ms'],2))" "$O/r${r}_$i.json" "$lib"
  done
done
