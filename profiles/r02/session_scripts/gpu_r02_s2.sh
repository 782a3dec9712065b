#!/bin/bash
# Round-2 GPU session 2: GPU suite (clocks/subscriptions/C5 added) and the interleaved
# A/B of the dense index load forms on C2.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s2
step() { echo "== $(date +%T) $*"; }
step pytest
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/s2/pytest.log 2>&1
rc=$?
grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/s2/pytest.log | tail -30
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit 1;; esac
step ab
timeout -k 10 400 python -u tools/ab_c2.py --configs 0:0,1:0,2:0,1:3 --rounds 7 --steps 5 > gpurun_out/s2/ab_index.json 2> gpurun_out/s2/ab_index.err || { tail -5 gpurun_out/s2/ab_index.err; exit 1; }
cat gpurun_out/s2/ab_index.json
step done
