#!/bin/bash
# m2s headline: SQ counters with check labelling on vs off (why labels measure slower), plus the
# label search's own gather-conflict estimate
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r03_labpmc
mkdir -p "$O"
cd "$R" || exit 1
for l in 1 0; do
  QLDPC_LABEL=$l timeout -k 10 400 bash tools/pmc_passes.sh "gpurun_out/r03_labpmc/lab$l" hgp_34_n1600 0.06 65536 0 64 Total > "$O/lab$l.log" 2>&1 || { tail "$O/lab$l.log"; exit 1; }
  python3 tools/pmc_summary2.py "$O/lab$l" > "$O/lab${l}_summary.txt" 2>&1; echo "== label $l"; grep -E "LDS_BANK|LDS_IDX|INSTS_LDS|WAVE_CYCLES  |WAIT_INST_LDS|INSTS_VALU" "$O/lab${l}_summary.txt"
done
QLDPC_LABEL=1 timeout -k 10 120 python3 -c "
from qldpc_fault_tolerance_amd import codes
from qldpc_fault_tolerance_amd.engine import DeviceBP
c = codes.get_code('hgp_34_n1600')
for H in (c.hz, c.hx):
    g = DeviceBP(H, 0.06, max_iter=160, precision=64).geometry(); print('label search gather conflicts', g.get('gather_conflicts'), g['kernel_id'])
" 2>&1 | tail -3
