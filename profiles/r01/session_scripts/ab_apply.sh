#!/bin/bash
# Interleaved A/B of dense_apply kernels on C2: f32 records (apply variant 6 = v2 default,
# 10 = v3 saddr) and binary16 records (h16 variant 0 = v2 default, 2 = v3).  2 rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for v in 6 10; do
    PSX_APPLY_VARIANT=$v timeout -k 10 120 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/ab_f32_v${v}_r$r.log 2>&1 || exit $?
    echo "f32 v=$v r=$r $(grep -o '"dense_apply": [0-9.]*' gpurun_out/ab_f32_v${v}_r$r.log | tail -1)"
  done
  for v in 0 2; do
    PSX_H16_VARIANT=$v timeout -k 10 120 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 --f16-records > gpurun_out/ab_f16_v${v}_r$r.log 2>&1 || exit $?
    echo "f16 v=$v r=$r $(grep -o '"dense_apply": [0-9.]*' gpurun_out/ab_f16_v${v}_r$r.log | tail -1)"
  done
done
