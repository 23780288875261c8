#!/bin/bash
# Round 4 GPU pass A: LDS calibration (incl. the pipelined mix), circuit tests, full GPU suite.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r04a}
mkdir -p "$O"
timeout -k 10 120 "$R/tools/calib/lds_calib" 20000 > "$O/calib.jsonl" 2>&1 || { echo "calib failed"; exit 1; }
timeout -k 10 120 python -u tools/lds_model.py > "$O/lds_model.json" 2>&1 || { echo "lds model failed"; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_circuit.py -x -v --timeout 300 --timeout-method thread \
  > "$O/pytest_circuit.log" 2>&1 || { echo "circuit tests failed"; exit 1; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > "$O/pytest_gpu.log" 2>&1 || { echo "gpu suite failed"; exit 1; }
echo "done: $O"
