#!/bin/bash
# PMC passes (one counter group per pass, --kernel-trace only; no sys/runtime trace).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc
mkdir -p "$OUT"
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > "$OUT/build.log" 2>&1 || exit 1
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
CMD=${PMC_CMD:-"python3 $ROOT/tools/exp_dense.py --apply 4 --index 2 --rounds 1 --steps 2"}
GROUPS_STR=${PMC_GROUPS:-"FETCH_SIZE;WRITE_SIZE;TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum;TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum;TCC_HIT_sum TCC_MISS_sum"}
IFS=';' read -ra GRPS <<< "$GROUPS_STR"
i=0
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  cd /tmp
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/p$i" -o run -- $CMD > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; [ $rc -ne 1 ] && exit $rc; fi
done
echo done
