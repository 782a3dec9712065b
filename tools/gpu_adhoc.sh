set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/s9; mkdir -p $O; export TMPDIR=/tmp
echo "== dense variant tests"
timeout -k 10 300 python -u -m pytest tests/test_dense_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -k "variant" > $O/dense.log 2>&1 || { tail -30 $O/dense.log; exit 1; }
tail -1 $O/dense.log
echo "== probe"
timeout -k 10 300 tools/probe_ceiling 10 > $O/probe.log 2>&1 || { tail -30 $O/probe.log; exit 1; }
cat $O/probe.log
echo "== ab"
timeout -k 10 300 python -u tools/ab_c2.py --configs 0:0,0:4,0:5 --rounds 6 --steps 5 > $O/ab.log 2>&1 || { tail -30 $O/ab.log; exit 1; }
cat $O/ab.log
