set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/s35; mkdir -p $O; export TMPDIR=/tmp
echo "== tests"
timeout -k 10 900 python -u -m pytest tests/test_indexed_rows_gpu.py tests/test_dense_gpu.py tests/test_variants_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2; do
echo "== d125 run $k"; timeout -k 10 300 python -u bench.py --density 0.125 --steps 20 --warmup 3 --cpu-seconds 0 > $O/d125_$k.log 2>&1 || { tail -20 $O/d125_$k.log; exit 1; }
python3 -c "
import json
d=json.loads([x for x in open('$O/d125_$k.log') if x.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['walked'])"
done
