# A/B of the spill launch's grid cap (PSX_VARIANT_SPILL_GRID 34), C3 walked+pipelined
mkdir -p gpurun_out/$1
i=0
for v in 768 256 64 768 256 64; do
  i=$((i+1))
  timeout -k 10 200 python -u bench.py --workload c3 --steps 40 --warmup 5 --cpu-seconds 0 --variant 34=$v > gpurun_out/$1/c3_${v}_$i.json 2> gpurun_out/$1/c3_${v}_$i.err || exit 1
done
