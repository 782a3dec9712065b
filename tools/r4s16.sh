#!/bin/bash
# Round-4 session 16: walk traces with the composed exit's outcome per window.
set -o pipefail
O=gpurun_out/r4s16
mkdir -p $O
for cfg in 0:0 3:1 3:4 4:1; do
  S=${cfg%%:*}; C=${cfg##*:}
  PSX_WALK_SHAPE=$S PSX_WALK_CUS=$C timeout -k 10 200 python -u tools/walk_trace.py > $O/wt_s${S}_c$C.json 2> $O/wt.err \
    || { tail -20 $O/wt.err; exit 1; }
  echo "trace $cfg done"
done
timeout -k 10 300 python -u tools/walk_sweep.py --configs 0:0:4,0:1:4,4:1:4,4:2:4,3:1:4,3:2:4,2:1:4,1:1:4 > $O/sweep.json 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
python -c "import json;[print(d) for d in json.load(open('$O/sweep.json'))]"
