set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s41
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_walk_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/s41/walk_tests.log 2>&1; rc=$?
tail -15 gpurun_out/s41/walk_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s41/tests.log 2>&1; rc=$?
tail -3 gpurun_out/s41/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload c3 --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/s41/c3.log 2>&1 || exit 1
tail -1 gpurun_out/s41/c3.log | cut -c1-900
timeout -k 10 300 python -u bench.py > gpurun_out/s41/bench.log 2>&1 || exit 1
tail -1 gpurun_out/s41/bench.log | cut -c1-3000
