# walk count-atomic cost probes (debug build, PSX_ORD_PROBE bits 8/9: one extra atomic per record, results unchanged)
mkdir -p gpurun_out/r6s15
i=0
for v in 0 256 512 0 256 512; do
  i=$((i+1))
  PSX_LIB=parameter_server_amd/libpsx_debug.so PSX_ORD_PROBE=$v timeout -k 10 200 python -u bench.py --workload c3 --steps 40 --warmup 5 --cpu-seconds 0 > gpurun_out/r6s15/c3_${v}_$i.json 2> gpurun_out/r6s15/c3_${v}_$i.err || exit 1
done
