set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-adhoc}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u bench.py --workload c3 --steps 20 --warmup 3 --cpu-seconds 0 > $O/c3.log 2>&1 || exit 1
tail -1 $O/c3.log | cut -c1-1200
timeout -k 10 300 python -u bench.py --workload c3 --indexed --steps 20 --warmup 3 --cpu-seconds 0 > $O/c3idx.log 2>&1 || exit 1
tail -1 $O/c3idx.log | cut -c1-700
timeout -k 10 300 python -u tools/probe_inc_latency.py --out $O/c3_inc_latency.json > $O/probe.log 2>&1 || exit 1
tail -5 $O/probe.log
