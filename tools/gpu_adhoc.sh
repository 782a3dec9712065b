set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/s18; mkdir -p $O; export TMPDIR=/tmp
echo "== full GPU suite"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
echo "== bench rows (pipelined listed calls)"
timeout -k 10 300 python -u bench.py --record-rows --steps 40 --warmup 5 --cpu-seconds 0 > $O/bench_rows.log 2>&1 || { tail -20 $O/bench_rows.log; exit 1; }
tail -1 $O/bench_rows.log | cut -c1-180; grep -o '"avg_launch_ms": [0-9.]*' $O/bench_rows.log
echo "== bench walked"
timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --cpu-seconds 0 > $O/bench_walk.log 2>&1 || { tail -20 $O/bench_walk.log; exit 1; }
tail -1 $O/bench_walk.log | cut -c1-180; grep -o '"avg_launch_ms": [0-9.]*' $O/bench_walk.log
