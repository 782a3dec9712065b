#!/bin/bash
# Round-2 GPU session 3: the GPU suite after the client unpack / header codec additions.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s3
echo "== $(date +%T) pytest"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/s3/pytest.log 2>&1
rc=$?
grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/s3/pytest.log | tail -30
[ $rc -le 1 ] || exit 1
if [ $rc -eq 1 ]; then grep -B5 -A40 "^_____" gpurun_out/s3/pytest.log | head -150; fi
echo "== $(date +%T) done"
