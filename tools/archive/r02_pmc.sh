#!/bin/bash
# SQ/TCC counter passes over one fused MC launch: tools/r02_pmc.sh <tag> <prof_one args...>
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
T=$1; shift
timeout -k 10 500 bash "$R/tools/pmc_passes.sh" "gpurun_out/$T" "$@" > "$R/gpurun_out/$T.log" 2>&1 || { tail "$R/gpurun_out/$T.log"; exit 1; }
python3 "$R/tools/pmc_summary2.py" "$R/gpurun_out/$T"
