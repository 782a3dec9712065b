set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/s13; mkdir -p $O; export TMPDIR=/tmp
echo "== ordered-path tests"
timeout -k 10 600 python -u -m pytest tests/test_sparse_gpu.py tests/test_indexed_gpu.py tests/test_kats_gpu.py tests/test_ssp_gpu.py tests/test_contract_gpu.py tests/test_importance_gpu.py tests/test_dense_gpu.py tests/test_pack_gpu.py tests/test_variants_gpu.py tests/test_c1_matrixfact.py tests/test_matrixfact_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
TAG=s13 bash tools/gpu_run.sh c3 c3idx stats3 || exit 1
