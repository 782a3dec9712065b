set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-adhoc}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats3 -o c3 -- python3 bench.py --workload c3 --steps 20 --warmup 3 --cpu-seconds 0 > $O/stats3.log 2>&1 || { tail -20 $O/stats3.log; exit 1; }
python3 tools/kernel_stats.py "$(find $O/stats3 -name '*.db' | head -1)" $O/c3_kernel_stats.csv && cut -c1-150 $O/c3_kernel_stats.csv
timeout -k 10 300 python -u tools/probe_inc_latency.py --out $O/c3_inc_latency.json > $O/probe.log 2>&1 || exit 1
tail -3 $O/probe.log
