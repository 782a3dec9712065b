#!/bin/bash
# GPU session: parity suite + smoke, every bench workload, rocprof stats of the main ones,
# PMC passes for ada_apply.  Stops at the first crash/fault/timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a "$OUT/session.log"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/session.log"
  tail -2 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 400 python bench.py --steps 20 --warmup 3 --cpu-seconds 12
run bench_ada 400 python bench.py --steps 10 --warmup 2 --cpu-seconds 12 --adarevision
run bench_f16 300 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 --f16-records
run bench_d125 300 python bench.py --steps 20 --warmup 3 --cpu-seconds 0 --density 0.125
run bench_imp 300 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 --importance
run bench_pcie 300 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 --pcie
run bench_c3 300 python bench.py --workload c3 --steps 10 --warmup 2 --cpu-seconds 8
run bench_c3_idx 300 python bench.py --workload c3 --steps 10 --warmup 2 --cpu-seconds 0 --indexed
run bench_c4 500 python bench.py --workload c4 --steps 5 --warmup 1
run bench_c5 400 python bench.py --workload c5 --steps 10 --warmup 2
cd /tmp
run rocprof 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 20 --warmup 3 --cpu-seconds 0
run rocprof_ada 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_ada" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --cpu-seconds 0 --adarevision
run rocprof_f16 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_f16" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --cpu-seconds 0 --f16-records
run rocprof_c3 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c3" -o run --output-format csv -- python3 "$ROOT/bench.py" --workload c3 --steps 10 --warmup 2 --cpu-seconds 0 --indexed
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  i=$((i+1))
  run pmc_ada$i 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/pmc_ada/p$i" -o run -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --cpu-seconds 0 --adarevision
done
cd "$ROOT" && python tools/pmc_summary.py "$OUT/pmc_ada" "$OUT/pmc_ada_apply.json" "ada_apply_v2_kernel<false, true, 6>"
echo done
