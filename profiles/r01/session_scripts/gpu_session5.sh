#!/bin/bash
# GPU session: parity suite, C2 bench (+ AdaRevision, float16 records), rocprof stats of
# each, PMC passes for dense_apply (v3 default) and ada_apply HBM traffic.
# Stops at the first crash/fault/timeout.
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
  tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
[ "${SKIP_TESTS:-0}" = 1 ] || run gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run bench 400 python bench.py --steps 20 --warmup 3 --cpu-seconds 12
run bench_ada 400 python bench.py --steps 10 --warmup 2 --cpu-seconds 12 --adarevision
run bench_f16 300 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 --f16-records
cd /tmp
run rocprof 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 20 --warmup 3 --cpu-seconds 0
run rocprof_ada 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_ada" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --cpu-seconds 0 --adarevision
run rocprof_f16 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_f16" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --cpu-seconds 0 --f16-records
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  i=$((i+1))
  run pmc$i 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/pmc/p$i" -o run -- python3 "$ROOT/tools/exp_dense.py" --apply 10 --index 2 --layouts 1 --rounds 1 --steps 2
  run pmc_ada$i 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/pmc_ada/p$i" -o run -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --cpu-seconds 0 --adarevision
done
cd "$ROOT" && python tools/pmc_summary.py "$OUT/pmc" "$OUT/pmc_dense_apply.json" && python tools/pmc_summary.py "$OUT/pmc_ada" "$OUT/pmc_ada_apply.json" "ada_apply_v2_kernel<false, true>"
echo done
