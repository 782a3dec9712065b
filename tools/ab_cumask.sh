mkdir -p gpurun_out/r6s12
i=0
for v in 0 2 4 -2 -4 0 2 4 -2 -4; do
  i=$((i+1))
  timeout -k 10 200 python -u bench.py --workload c3 --steps 40 --warmup 5 --cpu-seconds 0 --variant 32=$v > gpurun_out/r6s12/c3_${v}_$i.json 2> gpurun_out/r6s12/c3_${v}_$i.err || exit 1
done
