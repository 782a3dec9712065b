#!/bin/bash
# Round-2 GPU session 1: the GPU suite, the headline bench, and the PMC request-size
# experiment on the C2 index and apply kernels (plain vs non-temporal loads).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s1
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*"; }
step pytest
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/s1/pytest.log 2>&1
rc=$?
grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/s1/pytest.log | tail -30
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit 1;; esac
step bench
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s1/bench.log 2>&1 || { tail -20 gpurun_out/s1/bench.log; exit 1; }
tail -1 gpurun_out/s1/bench.log | cut -c1-600
step counters
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/s1/avail.txt 2>&1 || true
grep -o "TCC_EA0_RDREQ[A-Z0-9_]*\|TCC_EA0_WRREQ[A-Z0-9_]*\|TCC_BUBBLE[A-Z0-9_]*" gpurun_out/s1/avail.txt | sort -u | head -40
for v in "0 0" "1 0" "0 3"; do
  set -- $v
  step pmc index=$1 apply=$2
  PSX_INDEX_VARIANT=$1 PSX_APPLY_VARIANT=$2 timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_WRREQ_sum -d gpurun_out/s1/pmc_i$1_a$2 -o pmc -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/s1/pmc_i$1_a$2.log 2>&1 || { tail -5 gpurun_out/s1/pmc_i$1_a$2.log; exit 1; }
done
for v in "1 0" "0 3" "0 0"; do
  set -- $v
  step timing index=$1 apply=$2
  PSX_INDEX_VARIANT=$1 PSX_APPLY_VARIANT=$2 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/s1/bench_i$1_a$2.log 2>&1 || exit 1
  tail -1 gpurun_out/s1/bench_i$1_a$2.log | grep -o '"kernel_ms_per_step": {[^}]*}'
done
step done
