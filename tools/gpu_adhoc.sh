set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/s29; mkdir -p $O; export TMPDIR=/tmp
echo "== probe"; timeout -k 10 300 python -u tools/probe_inc_latency.py --out $O/c3_inc_latency.json > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
grep ns/Inc $O/probe.log | tr '\n' ' '; echo
cp $O/c3_inc_latency.json profiles/r02/c3_inc_latency.json
TAG=s29 bash tools/gpu_run.sh c3 c3idx stats3
