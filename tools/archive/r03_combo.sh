#!/bin/bash
# config 2 rest-of-family sweep + config 5 fp64 grid (r03_c2b.sh), then the m2s label A/B (r03_label.sh)
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
bash "$R/tools/r03_c2b.sh" && bash "$R/tools/r03_label.sh"
