#!/bin/bash
# One GPU-box session: gpu tests -> bench -> rocprofv3 kernel trace.
# Stops at the first step that crashes/faults/times out (exit not in {0,1}).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=${STEPS:-10}
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/session.log"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/session.log"
  tail -5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
python -c "import __graft_entry__ as g; g.build()" > "$OUT/build.log" 2>&1 || { echo build failed; tail -20 "$OUT/build.log"; exit 1; }
[ "${SKIP_TESTS:-0}" = 1 ] || run gpu_tests 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
[ "${SKIP_BENCH:-0}" = 1 ] || run bench 400 python bench.py --steps "$STEPS" --warmup 2 --cpu-seconds "${CPU_SECONDS:-8}" ${BENCH_ARGS:-}
[ "${RUN_C4:-0}" = 1 ] && run bench_c4 500 python bench.py --workload c4 --steps 5 --warmup 1
[ "${SKIP_C3:-0}" = 1 ] || run bench_c3 400 python bench.py --workload c3 --steps "$STEPS" --warmup 2 --cpu-seconds "${CPU_SECONDS:-8}"
if [ "${SKIP_PROF:-0}" != 1 ]; then
  cd /tmp
  run rocprof 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps "$STEPS" --warmup 2 --cpu-seconds 0
fi
echo done
