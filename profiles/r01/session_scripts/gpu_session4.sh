#!/bin/bash
# GPU session: parity suite, C2 bench (+ AdaRevision, float16 records), AdaRevision apply
# A/B, rocprof stats of the C2 and AdaRevision benches.  Stops at the first crash/fault/timeout.
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
run bench 400 python bench.py --steps 10 --warmup 2 --cpu-seconds 12
run bench_ada 400 python bench.py --steps 10 --warmup 2 --cpu-seconds 12 --adarevision
PSX_ADA_VARIANT=0 run bench_ada_v0 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --adarevision
run bench_f16 300 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 --f16-records
cd /tmp
run rocprof 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --cpu-seconds 0
run rocprof_ada 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_ada" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --cpu-seconds 0 --adarevision
echo done
