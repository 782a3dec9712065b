#!/bin/bash
# Round-2 GPU session 4: the C1 App-API driver test first (verbose), then the GPU suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s4
echo "== $(date +%T) c1"
timeout -k 10 300 python -u -m pytest tests/test_matrixfact_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/s4/c1.log 2>&1
rc=$?
tail -30 gpurun_out/s4/c1.log
[ $rc -le 1 ] || exit 1
echo "== $(date +%T) pytest"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/s4/pytest.log 2>&1
rc=$?
grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/s4/pytest.log | tail -30
[ $rc -le 1 ] || exit 1
if [ $rc -eq 1 ]; then grep -B5 -A40 "^_____" gpurun_out/s4/pytest.log | head -150; fi
echo "== $(date +%T) done"
