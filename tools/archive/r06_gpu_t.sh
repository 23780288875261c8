#!/bin/bash
# Round 6 pass T (diagnostic): what the waves holding config 5's last variable slot cost.  Config 5's
# kernel at eval_p 0.06 (every decode runs to max_iter, so the iteration count does not depend on the
# results) with the product library and with a QLDPC_DIAG_NOLAST build in which no wave runs the last
# slot (results invalid), interleaved.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r06t}
mkdir -p "$O"
for i in 1 2; do
  for L in prod nolast; do
    if [ $L = prod ]; then E="QLDPC_X=0"; else E="QLDPC_LIB=$R/qldpc_fault_tolerance_amd/libqldpc_hip_nolast.so"; fi
    timeout -k 10 240 env $E python -u bench.py --workload phenl --p 0.06 --steps 2 --warmup 1 --no-cpu-baseline --pmc-traffic 0 > "$O/${L}_$i.json" 2> "$O/${L}_$i.err" || { echo "$L failed"; tail -5 "$O/${L}_$i.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${L}_$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$L', r['kernel_ms'], r['mean_iters'])"
  done
done
