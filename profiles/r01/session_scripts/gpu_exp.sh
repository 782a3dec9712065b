#!/bin/bash
# GPU session for kernel experiments: parity suite (all variants) then the A/B script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out
mkdir -p "$OUT"
python -c "import __graft_entry__ as g; g.build()" > "$OUT/build.log" 2>&1 || { tail -20 "$OUT/build.log"; exit 1; }
[ -x tools/probe_unaligned ] && { timeout -k 10 60 tools/probe_unaligned > "$OUT/probe.log" 2>&1; echo "probe rc=$? $(cat $OUT/probe.log)"; }
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; tail -3 "$OUT/gpu_tests.log"; echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python tools/exp_dense.py ${EXP_ARGS:-} > "$OUT/exp.log" 2>&1
rc=$?; cat "$OUT/exp.log" | tail -40; echo "exp rc=$rc"
exit $rc
