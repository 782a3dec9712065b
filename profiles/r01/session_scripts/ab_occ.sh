#!/bin/bash
# A/B: dense_apply v3 at its natural occupancy vs held to 5 waves/SIMD (f32: apply 10 vs 14;
# binary16: h16 2 vs 3), C2, 2 rounds interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for v in 10 14; do
    PSX_APPLY_VARIANT=$v timeout -k 10 120 python bench.py --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/ab_occ_f32_${v}_r$r.log 2>&1 || exit $?
    echo "f32 v=$v r=$r $(grep -o '"dense_apply": [0-9.]*' gpurun_out/ab_occ_f32_${v}_r$r.log)"
  done
  for v in 2 3; do
    PSX_H16_VARIANT=$v timeout -k 10 120 python bench.py --steps 20 --warmup 3 --cpu-seconds 0 --f16-records > gpurun_out/ab_occ_f16_${v}_r$r.log 2>&1 || exit $?
    echo "f16 v=$v r=$r $(grep -o '"dense_apply": [0-9.]*' gpurun_out/ab_occ_f16_${v}_r$r.log)"
  done
done
