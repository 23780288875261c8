#!/bin/bash
# Round 6 pass L: the fp64 space-time graphs whose images sit between 64 KiB and 160 KiB on the tail
# families (round-6 routing) against their old route (QLDPC_E3_TAIL=0: engine 2), interleaved.
set -u
R=$(pwd)
O=$R/gpurun_out/${1:-r06l}
mkdir -p "$O"
for spec in "hgp_34_n1600 2" "hgp_34_n1225_q3 2" "hgp_34_n625 4"; do
  for T in 1 0; do
    for P in 0.01 0.05; do
      # shellcheck disable=SC2086
      timeout -k 10 200 env QLDPC_E3_TAIL=$T python -u tools/st_route_ab.py $spec $P 32768 >> "$O/route.jsonl" 2>> "$O/route.err" \
        || { echo "failed: $spec $T $P"; tail -5 "$O/route.err"; exit 1; }
      tail -1 "$O/route.jsonl"
    done
  done
done
