#!/bin/bash
# A/B of dense_apply variants on the 12.5%-density C2 variant (2 rounds, interleaved):
# 10 = v3 (default), 11/12/13 = v4 compact (8 rows/16 slots, 4/8, 4/12).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for v in 10 11 12 13; do
    PSX_APPLY_VARIANT=$v timeout -k 10 120 python bench.py --steps 20 --warmup 3 --cpu-seconds 0 --density 0.125 > gpurun_out/ab_d_v${v}_r$r.log 2>&1 || exit $?
    echo "v=$v r=$r $(grep -o '"dense_apply": [0-9.]*' gpurun_out/ab_d_v${v}_r$r.log | tail -1)"
  done
done
for v in 10 13; do
  PSX_APPLY_VARIANT=$v timeout -k 10 120 python bench.py --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/ab_full_v${v}.log 2>&1 || exit $?
  echo "full density v=$v $(grep -o '"dense_apply": [0-9.]*' gpurun_out/ab_full_v${v}.log | tail -1)"
done
