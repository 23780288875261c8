#!/bin/bash
# BASELINE config 2 as specified: 10 log-spaced p on [0.02, 0.12], 1e8 shots each, fp64, one MI355X.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r03_c2
mkdir -p "$O"
cd "$R" || exit 1
timeout -k 10 ${LIMIT:-1100} python -u tools/config2_sweep.py --codes ${CODES:-hgp_34_n1600} --shots ${SHOTS:-1e8} --out "$O/${TAG:-n1600}.jsonl" > "$O/${TAG:-n1600}.log" 2>&1 || { tail "$O/${TAG:-n1600}.log"; exit 1; }
tail -12 "$O/${TAG:-n1600}.log"
