mkdir -p gpurun_out/r4s4
for m in apply xchg both; do
  echo "== $m"; timeout -k 10 120 python -u tools/probe_big.py $m 60 > gpurun_out/r4s4/$m.log 2>&1; rc=$?; grep -v "^$" gpurun_out/r4s4/$m.log | tail -6; echo "rc=$rc"
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && break
done
exit 0
