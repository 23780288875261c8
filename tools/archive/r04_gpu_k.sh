#!/bin/bash
# Round 4 GPU pass K: the m2s decision as a sign-bit test (QLDPC_XSIGN) A/B against the fp64 compare
# (variant library), twice interleaved, plus the m2s parity tests on it.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r04k}
mkdir -p "$O"
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local n=$1 t=$2
  shift 2
  echo "== $n" >&2
  timeout -k 10 "$t" "$@" > "$O/$n.out" 2> "$O/$n.err" || { echo "step $n failed ($?)"; tail -30 "$O/$n.out"; tail -5 "$O/$n.err"; exit 1; }
}
V=$R/qldpc_fault_tolerance_amd/libqldpc_hip_xs0.so
step t_m2s 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_m2s.py tests/test_gpu_m2s8.py tests/test_gpu_parity.py
for r in 1 2; do
  step new$r 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --fp32-line 0 --pmc-traffic 0
  QLDPC_LIB=$V step old$r 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --fp32-line 0 --pmc-traffic 0
done
step lp_new 300 python -u bench.py --code LP_Matg8_L30_Dmin20 --steps 5 --warmup 1 --no-cpu-baseline --fp32-line 0 --pmc-traffic 0
QLDPC_LIB=$V step lp_old 300 python -u bench.py --code LP_Matg8_L30_Dmin20 --steps 5 --warmup 1 --no-cpu-baseline --fp32-line 0 --pmc-traffic 0
echo "done: $O"
