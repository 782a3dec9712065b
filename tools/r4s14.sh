#!/bin/bash
# Round-4 session 14: split/exchange tests (streams_v, self sub-stream from the send slot),
# walk traces at composed-map levels 4/2/0, a C3 levels sweep, C4 pipelined on one GPU.
set -o pipefail
O=gpurun_out/r4s14
mkdir -p $O
timeout -k 10 420 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_split_gpu.py > $O/split.log 2>&1 || { tail -30 $O/split.log; exit 1; }
tail -1 $O/split.log
for L in 4 2 0; do
  PSX_WALK_LEVELS=$L timeout -k 10 200 python -u tools/walk_trace.py > $O/wt$L.json 2> $O/wt$L.err \
    || { tail -20 $O/wt$L.err; exit 1; }
  echo "trace L=$L done"
done
for L in 2 3 1 2 3 1; do
  PSX_WALK_LEVELS=$L timeout -k 10 200 python -u bench.py --workload c3 --steps 20 --warmup 3 \
    --cpu-seconds 0 > $O/c3_L$L.json 2>> $O/c3.err || { tail -20 $O/c3.err; exit 1; }
  echo "L=$L $(python -c "import json,sys;d=json.loads(open('$O/c3_L$L.json').read().strip().splitlines()[-1]);print(d['value'],d.get('walked'),d['roofline']['achieved'])")"
done
timeout -k 10 300 python -u bench.py --workload c4 --steps 3 --warmup 1 --cpu-seconds 0 \
  > $O/c4.json 2> $O/c4.err || { tail -20 $O/c4.err; exit 1; }
tail -c 1500 $O/c4.json
