set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/s23; mkdir -p $O; export TMPDIR=/tmp
echo "== rows tests"
timeout -k 10 600 python -u -m pytest tests/test_indexed_rows_gpu.py tests/test_dense_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
echo "== A/B"; timeout -k 10 300 python -u tools/ab_c2.py --configs 0,0:1 --rounds 7 --steps 5 > $O/ab.json 2>&1 || { tail -20 $O/ab.json; exit 1; }
cat $O/ab.json
TAG=s23 bash tools/gpu_run.sh pmc bench
