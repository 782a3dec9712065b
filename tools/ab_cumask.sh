# A/B of the prep stream's CU mask (PSX_VARIANT_SIDE_CU_MASK 32) x walk blocks per masked CU (28)
mkdir -p gpurun_out/r6s13
i=0
for r in 1 2; do
for kv in "0 0" "4 2" "4 3" "4 4" "3 1" "3 2" "8 4" "8 6"; do
  set -- $kv
  i=$((i+1))
  timeout -k 10 200 python -u bench.py --workload c3 --steps 40 --warmup 5 --cpu-seconds 0 --variant 32=$1 --variant 28=$2 > gpurun_out/r6s13/c3_${1}_${2}_$i.json 2> gpurun_out/r6s13/c3_${1}_${2}_$i.err || exit 1
done
done
