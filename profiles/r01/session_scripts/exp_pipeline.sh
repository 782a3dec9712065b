#!/bin/bash
# bench with the index/apply pipeline on and off, interleaved twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
for i in 1 2; do
  for p in 0 1; do
    PSX_PIPELINE=$p timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/pipe_${p}_${i}.log 2>&1 || exit $?
    echo "pipeline=$p run=$i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/pipe_${p}_${i}.log) $(grep -o '"kernel_ms_per_step": {[^}]*}' gpurun_out/pipe_${p}_${i}.log)"
  done
done
