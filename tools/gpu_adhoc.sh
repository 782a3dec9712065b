set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/s33; mkdir -p $O; export TMPDIR=/tmp
for pr in 0 1 0 1; do
echo "== c3idx prio=$pr"; PSX_ORD_PRIO=$pr timeout -k 10 300 python -u bench.py --workload c3 --indexed --steps 20 --warmup 3 --cpu-seconds 0 > $O/c3idx_p$pr.log 2>&1 || { tail -20 $O/c3idx_p$pr.log; exit 1; }
grep -o '"value": [0-9.]*\|"ordered_apply_ms_per_step": [0-9.]*' $O/c3idx_p$pr.log | tr '\n' ' '; echo
done
