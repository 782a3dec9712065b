mkdir -p gpurun_out/r4s3
export PSX_BENCH_VERBOSE=1 PSX_BENCH_STACK_AFTER=60
for mb in 64 512 2048; do
  echo "== chunk $mb MiB"
  timeout -k 10 150 python -u -c "
import sys; sys.argv=['bench.py']; sys.path.insert(0,'.')
import bench, torch, json
torch.cuda.set_device(0)
m = bench.exchange_measure(600000, 1024, 1, 1, 1, 0, 0, max_bytes=min($mb*1048576, bench.C4_CHUNK_BYTES))
print(json.dumps(m)[:600])
" > gpurun_out/r4s3/c4_$mb.log 2>&1
  rc=$?; tail -4 gpurun_out/r4s3/c4_$mb.log; echo "rc=$rc"; [ $rc -ne 0 ] && break
done
exit 0
