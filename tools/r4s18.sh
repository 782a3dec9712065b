#!/bin/bash
# Round-4 session 18: walk with the counts loaded straight from the message; stats events per
# sync interval; parity, traces, A/B and the rocprof timeline.
set -o pipefail
O=gpurun_out/r4s18
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_walk_gpu.py tests/test_walk_count_gpu.py tests/test_ctx_stats_gpu.py > $O/walk.log 2>&1 || { tail -40 $O/walk.log; exit 1; }
tail -1 $O/walk.log
for cfg in 0:0 4:1; do
  S=${cfg%%:*}; C=${cfg##*:}
  PSX_WALK_SHAPE=$S PSX_WALK_CUS=$C timeout -k 10 200 python -u tools/walk_trace.py > $O/wt_s${S}_c$C.json 2> $O/wt.err \
    || { tail -20 $O/wt.err; exit 1; }
done
timeout -k 10 300 python -u tools/walk_sweep.py --configs 0:0:4:0,0:0:4:3,4:1:4:0,4:1:4:3,4:2:4:0,2:2:4:0 > $O/sweep.json 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
python -c "import json;[print(d) for d in json.load(open('$O/sweep.json'))]"
for cfg in 4:1:4:0 4:1:4:3; do
  R=/tmp/r4s18prof_${cfg//:/_}
  timeout -k 10 200 rocprofv3 --kernel-trace -d $R -o c3 -- python3 tools/walk_sweep.py --configs $cfg --rounds 1 --steps 20 \
    > $O/prof_${cfg//:/_}.log 2>&1 || { tail -20 $O/prof_${cfg//:/_}.log; exit 1; }
  python3 tools/c3_timeline.py "$(find $R -name '*.db' | head -1)" > $O/timeline_${cfg//:/_}.json
  python3 -c "import json;d=json.load(open('$O/timeline_${cfg//:/_}.json'));print('$cfg', d['span_us_mean'], d['kernel_us_sum_mean'], [(k['kernel'][:24], k['us_mean']) for k in d['sequence']])"
done
