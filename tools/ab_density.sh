#!/bin/bash
# A/B of dense_apply variants on the 12.5%-density C2 variant (2 rounds, interleaved).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for v in 10 6 3 8; do
    PSX_APPLY_VARIANT=$v timeout -k 10 120 python bench.py --steps 20 --warmup 3 --cpu-seconds 0 --density 0.125 > gpurun_out/ab_d_v${v}_r$r.log 2>&1 || exit $?
    echo "v=$v r=$r $(grep -o '"dense_apply": [0-9.]*' gpurun_out/ab_d_v${v}_r$r.log | tail -1)"
  done
done
