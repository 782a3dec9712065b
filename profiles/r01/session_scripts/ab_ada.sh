#!/bin/bash
# A/B of the AdaRevision apply kernels on C2 (ada variant 1 = default, 2 = 6 waves/SIMD).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for v in 2 3 4; do
    PSX_ADA_VARIANT=$v timeout -k 10 120 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 --adarevision > gpurun_out/ab_ada_${v}_r$r.log 2>&1 || exit $?
    echo "ada=$v r=$r $(grep -o '"ada_apply": [0-9.]*' gpurun_out/ab_ada_${v}_r$r.log)"
  done
done
