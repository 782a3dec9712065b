set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/s32; mkdir -p $O; export TMPDIR=/tmp
echo "== ordered-path tests"
timeout -k 10 600 python -u -m pytest tests/test_sparse_gpu.py tests/test_kats_gpu.py tests/test_indexed_gpu.py tests/test_ssp_gpu.py tests/test_contract_gpu.py tests/test_importance_gpu.py tests/test_push_body_gpu.py tests/test_matrixfact_gpu.py tests/test_configs_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
echo "== probe"; timeout -k 10 300 python -u tools/probe_inc_latency.py --out $O/c3_inc_latency.json > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
grep ns/Inc $O/probe.log | tr '\n' ' '; echo
cp $O/c3_inc_latency.json profiles/r02/c3_inc_latency.json
TAG=s32 bash tools/gpu_run.sh c3 c3idx stats3 c5
