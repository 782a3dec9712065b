#!/bin/bash
# Round-4 session 21: ordered_offsets' one-tile path — the ordered/sparse GPU tests, the C3
# timeline, the C3 line; the C2 PMC passes for this round's profile.
set -o pipefail
O=gpurun_out/r4s21
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/ord.log 2>&1 || { tail -40 $O/ord.log; exit 1; }
tail -1 $O/ord.log
R=/tmp/r4s21prof
timeout -k 10 200 rocprofv3 --kernel-trace -d $R -o c3 -- python3 tools/walk_sweep.py --configs 4:1:4:0 --rounds 1 --steps 20 \
  > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 tools/c3_timeline.py "$(find $R -name '*.db' | head -1)" > $O/timeline.json
python3 -c "import json;d=json.load(open('$O/timeline.json'));print(d['span_us_mean'], d['kernel_us_sum_mean'], [(k['kernel'][:24], k['us_mean']) for k in d['sequence']])"
timeout -k 10 300 python -u bench.py --workload c3 --steps 20 --warmup 3 > $O/c3.json 2> $O/c3.err || { tail -20 $O/c3.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/c3.json').read().strip().splitlines()[-1]);print(d['value'], d['pipelined']['value'], d['roofline'])"
TAG=r4s21 bash tools/gpu_run.sh pmc
