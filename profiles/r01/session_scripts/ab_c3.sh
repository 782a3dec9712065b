#!/bin/bash
# Interleaved A/B of the sorted-map apply grid on C3 (indexed), 2 rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for v in 0 1 2; do
    PSX_ORD_GRID=$v timeout -k 10 120 python bench.py --workload c3 --steps 10 --warmup 2 --cpu-seconds 0 --indexed > gpurun_out/ab_c3_g${v}_r$r.log 2>&1 || exit $?
    echo "grid=$v r=$r $(grep -o '"value": [0-9.]*' gpurun_out/ab_c3_g${v}_r$r.log | head -1) $(grep -o '"ordered_apply": [0-9.]*' gpurun_out/ab_c3_g${v}_r$r.log)"
  done
done
