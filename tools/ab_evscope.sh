# A/B of the cross-stream events' release scope (PSX_VARIANT_EVENT_SCOPE 33), C3 walked+pipelined, indexed
mkdir -p gpurun_out/$1
i=0
for v in 0 1 2 0 1 2; do
  i=$((i+1))
  timeout -k 10 200 python -u bench.py --workload c3 --steps 40 --warmup 5 --cpu-seconds 0 --variant 33=$v > gpurun_out/$1/c3_${v}_$i.json 2> gpurun_out/$1/c3_${v}_$i.err || exit 1
  timeout -k 10 200 python -u bench.py --workload c3 --indexed --steps 40 --warmup 5 --cpu-seconds 0 --variant 33=$v > gpurun_out/$1/c3i_${v}_$i.json 2> gpurun_out/$1/c3i_${v}_$i.err || exit 1
done
