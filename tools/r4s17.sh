#!/bin/bash
# Round-4 session 17: the walk's speculative sub-phases; C3 walked + pipelined at shape 0
# (half the CUs) and shape 4 (every CU), alternating.
set -o pipefail
O=gpurun_out/r4s17
mkdir -p $O
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
