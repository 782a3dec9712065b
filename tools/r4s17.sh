#!/bin/bash
# Round-4 session 17: the walk's speculative sub-phases; C3 walked + pipelined at shape 0
# (half the CUs) and shape 4 (every CU), alternating.
set -o pipefail
O=gpurun_out/r4s17
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_walk_gpu.py tests/test_walk_count_gpu.py > $O/walk.log 2>&1 || { tail -40 $O/walk.log; exit 1; }
tail -1 $O/walk.log
for cfg in 0:0 4:1; do
  S=${cfg%%:*}; C=${cfg##*:}
  PSX_WALK_SHAPE=$S PSX_WALK_CUS=$C timeout -k 10 200 python -u tools/walk_trace.py > $O/wt_s${S}_c$C.json 2> $O/wt.err \
    || { tail -20 $O/wt.err; exit 1; }
done
for r in 1 2; do
for cfg in 0:0 4:1 4:2; do
  S=${cfg%%:*}; C=${cfg##*:}
  PSX_WALK_SHAPE=$S PSX_WALK_CUS=$C timeout -k 10 200 python -u bench.py --workload c3 --steps 20 --warmup 3 \
    --cpu-seconds 0 > $O/c3_s${S}_c${C}_$r.json 2>> $O/c3.err || { tail -20 $O/c3.err; exit 1; }
  echo "S=$S C=$C $(python -c "import json;d=json.loads(open('$O/c3_s${S}_c${C}_$r.json').read().strip().splitlines()[-1]);print(d['value'],d['pipelined']['value'],d['kernel_ms_per_step_breakdown_pass'])")"
done
done
timeout -k 10 420 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_split_gpu.py > $O/split.log 2>&1 || { tail -30 $O/split.log; exit 1; }
tail -1 $O/split.log
timeout -k 10 300 python -u bench.py --workload c4 --steps 3 --warmup 1 --cpu-seconds 0 \
  > $O/c4.json 2> $O/c4.err || { tail -20 $O/c4.err; exit 1; }
tail -c 1200 $O/c4.json
export TMPDIR=/tmp
for cfg in 4:1:4 0:0:4; do
  R=/tmp/r4s17prof_${cfg//:/_}
  timeout -k 10 200 rocprofv3 --kernel-trace -d $R -o c3 -- python3 tools/walk_sweep.py --configs $cfg --rounds 1 --steps 20 \
    > $O/prof_${cfg//:/_}.log 2>&1 || { tail -20 $O/prof_${cfg//:/_}.log; exit 1; }
  python3 tools/c3_timeline.py "$(find $R -name '*.db' | head -1)" > $O/timeline_${cfg//:/_}.json
  python3 -c "import json;d=json.load(open('$O/timeline_${cfg//:/_}.json'));print('$cfg', d['span_us_mean'], d['kernel_us_sum_mean'], [(k['kernel'][:24], k['us_mean'], k['gap_before_us_mean']) for k in d['sequence']])"
done
