# interleaved A/B of two builds of libpsx (PSX_LIB), C3 bench only; $1 = output dir under gpurun_out
O=gpurun_out/$1; mkdir -p $O
i=0
for L in ab_old/libpsx_old.so parameter_server_amd/libpsx.so ab_old/libpsx_old.so parameter_server_amd/libpsx.so; do
  i=$((i+1)); n=$(basename $L .so)
  PSX_LIB=$L timeout -k 10 200 python -u bench.py --workload c3 --steps 40 --warmup 5 --cpu-seconds 0 > $O/c3_${n}_$i.json 2> $O/c3_${n}_$i.err || exit 1
  PSX_LIB=$L timeout -k 10 200 python -u bench.py --workload c3 --indexed --steps 40 --warmup 5 --cpu-seconds 0 > $O/c3i_${n}_$i.json 2> $O/c3i_${n}_$i.err || exit 1
done
