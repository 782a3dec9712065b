#!/bin/bash
# One GPU session on the gpurun box: the steps named on the command line, in order, each
# under its own time limit; the first failing step ends the session.
#   tests   pytest -m gpu (the whole suite, one process)
#   smoke   __graft_entry__.smoke()
#   bench   the default C2 bench line (with the PMC JSON of this tree when present)
#   stats   the default bench under rocprofv3 --kernel-trace --stats
#   pmc     three PMC passes on the C2 bench (request counts, FETCH_SIZE, WRITE_SIZE),
#           summarised with the kernel signature into $O/pmc_dense_apply.json
#   c3 | c3idx | c4 | c5 | ada | f16 | d125 | imp   the other workloads' bench lines
#   probe   tools/probe_ceiling (the C2 access pattern's hardware ceiling; build it first)
#   hbm     tools/probe_hbm: copy / read / random-chunk gather / C2-pattern rates (build it first)
# Output: gpurun_out/$TAG/ (TAG from the environment, default "run").
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-run}
mkdir -p "$O"
export TMPDIR=/tmp
PMC_JSON=$O/pmc_dense_apply.json
[ -f "$PMC_JSON" ] || PMC_JSON=profiles/r02/pmc_dense_apply.json
say() { echo "== $(date +%T) $*"; }
run() {  # run NAME SECONDS CMD...: output to $O/NAME.log; on failure print its tail and stop
  local name=$1 secs=$2; shift 2
  say "$name"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "!! $name rc=$rc"; tail -40 "$O/$name.log"; exit 1; fi
  tail -3 "$O/$name.log" | cut -c1-1500
}
for s in "$@"; do
  case $s in
    tests) run tests 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python -u bench.py --steps 20 --warmup 5 --pmc-json "$PMC_JSON" ;;
    walked) run walked 300 python -u bench.py --walked --steps 20 --warmup 5 --cpu-seconds 0 ;;
    stats) run stats 300 rocprofv3 --kernel-trace --stats -d "$O/stats" -o c2 -- python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 --skip-walked --no-extras
           python3 tools/kernel_stats.py "$(find "$O/stats" -name '*.db' | head -1)" "$O/c2_kernel_stats.csv" && head -4 "$O/c2_kernel_stats.csv" | cut -c1-160 ;;
    stats3) run stats3 300 rocprofv3 --kernel-trace --stats -d "$O/stats3" -o c3 -- python3 bench.py --workload c3 --steps 20 --warmup 3 --cpu-seconds 0
           python3 tools/kernel_stats.py "$(find "$O/stats3" -name '*.db' | head -1)" "$O/c3_kernel_stats.csv" && head -6 "$O/c3_kernel_stats.csv" | cut -c1-160 ;;
    pmc)
      P=1
      for ctrs in "TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "FETCH_SIZE" "WRITE_SIZE"; do
        say "pmc pass $P: $ctrs"
        timeout -s KILL 120 rocprofv3 --pmc $ctrs -d "$O/pmc/p$P" -o pmc -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --skip-walked --no-extras \
          > "$O/pmc_p$P.log" 2>&1 || { echo "!! pmc pass $P"; tail -5 "$O/pmc_p$P.log"; exit 1; }
        P=$((P+1))
      done
      python3 tools/pmc_summary.py "$O/pmc" "$O/pmc_dense_apply.json" || exit 1
      PMC_JSON=$O/pmc_dense_apply.json ;;
    c3) run c3 300 python -u bench.py --workload c3 --steps 20 --warmup 3 ;;
    c3idx) run c3idx 300 python -u bench.py --workload c3 --indexed --steps 20 --warmup 3 ;;
    c4) run c4 600 python -u bench.py --workload c4 --steps 3 --warmup 1 ;;
    c5) run c5 300 python -u bench.py --workload c5 --steps 10 --warmup 2 ;;
    ada) run ada 300 python -u bench.py --adarevision --steps 10 --warmup 2 --cpu-seconds 6 ;;
    f16) run f16 300 python -u bench.py --f16-records --steps 20 --warmup 3 --cpu-seconds 0 ;;
    d125) run d125 300 python -u bench.py --density 0.125 --steps 20 --warmup 3 --cpu-seconds 0 ;;
    imp) run imp 300 python -u bench.py --importance --steps 20 --warmup 3 --cpu-seconds 0 ;;
    probe) run probe 300 tools/probe_ceiling 10 ;;
    hbm) run hbm 400 tools/probe_hbm 10 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
say done
