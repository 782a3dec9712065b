#!/bin/bash
# Round-4 session 24: the bare bench as the driver runs it (timed), smoke, the C3 PMC pass and
# rocprof stats of C2 and C3 on this tree.
set -o pipefail
O=gpurun_out/r4s24
mkdir -p $O
export TMPDIR=/tmp
t0=$(date +%s)
timeout -k 10 900 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -30 $O/bench_default.err; exit 1; }
echo "bare bench took $(( $(date +%s) - t0 )) s"
tail -c 600 $O/bench_default.json
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
TAG=r4s24 bash tools/gpu_run.sh pmcc3 stats stats3
