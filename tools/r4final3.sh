#!/bin/bash
# Round-4 final check on the final tree: the C3 PMC pass and rocprof stats, the GPU suite,
# smoke, the bare bench as the driver runs it.
set -o pipefail
O=gpurun_out/r4final3
mkdir -p $O
TAG=r4final3 bash tools/gpu_run.sh pmcc3 stats stats3 || exit 1
cp $O/pmc_c3.json profiles/r04/pmc_c3.json   # this tree's C3 traffic for the bench below
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
t0=$(date +%s)
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
echo "bare bench $(( $(date +%s) - t0 )) s"
python3 -c "
import json
j=json.loads([l for l in open('$O/bench.json') if l.startswith('{')][-1])
print(j['value'], j['ms_per_step'], j['roofline']['frac'], j['roofline'].get('frac_of_read_sweep'), j['roofline'].get('traffic'), j['roofline'].get('traffic_note'))
for k,v in j['other_configs'].items(): print(k, v.get('value'), (v.get('pipelined') or {}).get('value'), v.get('error'), (v.get('roofline') or {}).get('sector_efficiency'))
"
