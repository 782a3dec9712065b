#!/bin/bash
# Round-4 session 30: the split scatter with four records in flight — split tests, then C4's
# pipeline with the split kept (tools/split_probe.py), this build vs ab_old, interleaved.
set -o pipefail
O=gpurun_out/r4s30
mkdir -p $O
timeout -k 10 420 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_split_gpu.py \
  > $O/split.log 2>&1 || { tail -30 $O/split.log; exit 1; }
tail -1 $O/split.log
for v in new old new old; do
  L=; [ $v = old ] && L=ab_old/libpsx.so
  PSX_LIB=$L timeout -k 10 300 python -u tools/split_probe.py > $O/probe_$v.log 2> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
  echo "$v $(tail -1 $O/probe_$v.log)"
done
