#!/bin/bash
# Round-2 GPU session 5: C1 driver tests, then the headline bench under rocprofv3
# --kernel-trace --stats, three PMC passes on the current dense_apply kernel (request
# counts; FETCH_SIZE; WRITE_SIZE) summarised with its kernel signature, and the bench
# line carrying that traffic.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/s5
mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*"; }
step c1
timeout -k 10 300 python -u -m pytest tests/test_matrixfact_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/c1.log 2>&1 || { tail -40 $O/c1.log; exit 1; }
tail -2 $O/c1.log
step stats
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o c2 -- python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 \
  > $O/stats_bench.log 2>&1 || { tail -20 $O/stats_bench.log; exit 1; }
find $O/stats -name "*kernel_stats.csv" | head -3
P=1
for ctrs in "TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  step pmc pass $P: $ctrs
  timeout -s KILL 120 rocprofv3 --pmc $ctrs -d $O/pmc/p$P -o pmc -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 \
    > $O/pmc_p$P.log 2>&1 || { tail -5 $O/pmc_p$P.log; exit 1; }
  P=$((P+1))
done
python3 tools/pmc_summary.py $O/pmc $O/pmc_dense_apply.json || exit 1
step bench
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --pmc-json $O/pmc_dense_apply.json > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
step done
