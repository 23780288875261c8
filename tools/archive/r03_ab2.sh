#!/bin/bash
# (1) m2s A/B: default vs one uniform prior (QLDPC_M2S_UNIL) vs that + gathers two ahead;
# (2) FETCH_SIZE / WRITE_SIZE calibration for 4/8/16-B-per-lane and 512-B-segment accesses;
# (3) engine 6 forced on LP_Matg8_L30_Dmin20 fp64 at 8 and 16 resident waves per CU, with PMC traffic.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r03_ab2
mkdir -p "$O"
cd "$R" || exit 1
for r in 1 2; do
  for lib in "-" libqldpc_hip_unil.so libqldpc_hip_unil_pf2.so; do
    L=""; [ "$lib" != "-" ] && L=$R/qldpc_fault_tolerance_amd/$lib
    QLDPC_LIB=$L timeout -k 10 200 python3 -u bench.py --steps 4 --warmup 1 --pmc-traffic 0 --fp32-line 0 --no-cpu-baseline > "$O/ab.json" 2> "$O/ab.err" || { tail -5 "$O/ab.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), round(d['roofline']['frac'],4), round(d['roofline']['kernel_ms'],2))" "$O/ab.json" "$lib" | tee -a "$O/ab.txt"
  done
done
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d "$O/calib_$c" -o p -- "$R/tools/calib/fetch_calib" > "$O/calib_$c.log" 2>&1 || { echo "calib $c failed"; tail "$O/calib_$c.log"; exit 1; }
done
cd "$R"
python3 - "$O" <<'PY'
import csv, glob, sys, os
O = sys.argv[1]
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(os.path.join(O, f"calib_{c}", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") == c:
                print(c, row["Kernel_Name"][:40], "KB", row["Counter_Value"], "ratio_to_1GiB", float(row["Counter_Value"]) * 1024 / 2**30)
PY
for w in 8 16; do
  QLDPC_ENGINE=6 QLDPC_HBM_WAVES=$w timeout -k 10 300 python3 -u bench.py --code LP_Matg8_L30_Dmin20 --steps 2 --warmup 1 --shots 262144 --fp32-line 0 --no-cpu-baseline > "$O/e6_w$w.json" 2> "$O/e6_w$w.err" || { tail -5 "$O/e6_w$w.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('e6 waves', sys.argv[2], round(d['value']), r['bound'], round(r['achieved']), round(r['frac'],4), r['traffic'], r['bytes_per_launch'], r['hbm']['pmc'])" "$O/e6_w$w.json" $w | tee -a "$O/e6.txt"
done
