#!/bin/bash
# Round-4 session 15: the walk's shapes — parity (test_walk_gpu over every shape), then the
# interleaved A/B (tools/walk_sweep.py) and traces of the best-looking small shape.
set -o pipefail
O=gpurun_out/r4s15
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_walk_gpu.py tests/test_walk_count_gpu.py > $O/walk.log 2>&1 || { tail -40 $O/walk.log; exit 1; }
tail -1 $O/walk.log
timeout -k 10 300 python -u tools/walk_sweep.py > $O/sweep.json 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
cat $O/sweep.json | python -c "import json,sys;[print(d) for d in json.load(sys.stdin)]"
for S in 3 2; do
  PSX_WALK_SHAPE=$S PSX_WALK_CUS=4 timeout -k 10 200 python -u tools/walk_trace.py > $O/wt_s$S.json 2> $O/wt_s$S.err \
    || { tail -20 $O/wt_s$S.err; exit 1; }
done
echo traces done
