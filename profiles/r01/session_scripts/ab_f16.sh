#!/bin/bash
# A/B of the binary16-record apply variants on C2 (interleaved, 2 rounds).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for v in 0 1 2 3; do
    PSX_H16_VARIANT=$v timeout -k 10 120 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 --f16-records > gpurun_out/ab_f16_v${v}_r$r.log 2>&1 || exit $?
    echo "v=$v r=$r $(grep -o '"dense_apply": [0-9.]*' gpurun_out/ab_f16_v${v}_r$r.log | tail -1)"
  done
done
