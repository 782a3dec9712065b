mkdir -p gpurun_out/r4s5
echo "== xchg"; timeout -k 10 120 python -u tools/probe_big.py xchg 60 > gpurun_out/r4s5/xchg.log 2>&1; tail -2 gpurun_out/r4s5/xchg.log
echo "== tests"; timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_split_gpu.py -k "large_sub_stream or shard_exchange" > gpurun_out/r4s5/t.log 2>&1; rc=$?; tail -3 gpurun_out/r4s5/t.log; [ $rc -ne 0 ] && exit 1
echo "== c4 2M"; PSX_BENCH_VERBOSE=1 PSX_BENCH_STACK_AFTER=100 timeout -k 10 200 python -u bench.py --workload c4 --c4-rows 2000000 --steps 2 --warmup 1 > gpurun_out/r4s5/c4small.log 2>&1; rc=$?; tail -2 gpurun_out/r4s5/c4small.log | cut -c1-1500; [ $rc -ne 0 ] && exit 1
echo "== c4 full"; PSX_BENCH_VERBOSE=1 PSX_BENCH_STACK_AFTER=170 timeout -k 10 300 python -u bench.py --workload c4 --steps 3 --warmup 1 > gpurun_out/r4s5/c4.log 2>&1; rc=$?; tail -1 gpurun_out/r4s5/c4.log | cut -c1-3000
exit $rc
