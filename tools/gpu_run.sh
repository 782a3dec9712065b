#!/bin/bash
# Environment overrides of the kernel selectors (PSX_ORD_SPLIT, PSX_WALK_*, PSX_ORD_PROBE, ...)
# exist only in the debug build (make -C parameter_server_amd/csrc debug -> libpsx_debug.so):
# the modes that set one load that library through PSX_LIB.
# One GPU session on the gpurun box: the steps named on the command line, in order, each
# under its own time limit; the first failing step ends the session.
#   tests   pytest -m gpu (the whole suite, one process)
#   walktests the walk / sparse / record-row / split / KAT GPU test files only
#   newtests  the dense / record-row / split-apply GPU test files only
#   abdense tools/ab_c2.py over dense apply variants (ABCONF: its --configs)
#   smoke   __graft_entry__.smoke()
#   bench   the default C2 bench line (with the PMC JSON of this tree when present)
#   stats   the default bench under rocprofv3 --kernel-trace --stats
#   pmc     three PMC passes on the C2 bench (request counts, FETCH_SIZE, WRITE_SIZE),
#           summarised with the kernel signature into $O/pmc_dense_apply.json
#   c3split C3 with each split-apply form (PSX_ORD_SPLIT 1, 2, 3), twice, interleaved
#   c3walk  C3 with the walk on half / all CUs (PSX_WALK_CUS 0, 1), twice, interleaved
#   c3 | c3idx | c4 | c5 | ada | f16 | d125 | imp   the other workloads' bench lines
#   probe   tools/probe_ceiling (the C2 access pattern's hardware ceiling; build it first)
#   mixab   the mixing probe and the C2 apply A/B interleaved, three times (same box)
#   wtrace  tools/walk_trace.py: per-window timeline of the walk on the C3 batches
#   pmix    tools/probe_apply's mixing probe (records in random vs slot order; build it first)
#   c3lib   C3 with this tree's libpsx and ab_old/libpsx.so (PSX_LIB), interleaved twice
#   oldheavy the all-rows-heavy-and-spilling test on ab_old/libpsx.so (reported, never fatal)
#   splittests the split-apply / sparse / KAT GPU test files only
#   xtests  the split / exchange pipeline / walk-count / multi-rank GPU test files only
#   c3ab    C3 A/B over one variant: AB_VAR (an env override, default PSX_ORD_LITE) set to each
#           of AB_VALUES in turn (default "0 1 0 1")
#   salu    the C3 apply's instruction mix (SALU / VALU / branch / LDS / SMEM / VMEM per dispatch)
#           under PSX_ORD_PROBE 0 (full), 3 (setup only), 6 (image only)
#   c3libs  C3 with each build named in LIBS (space-separated PSX_LIB paths; new = this tree's), twice
#   c2ab    C2 (headline + walked) A/B over one variant: AB_VAR (default PSX_INDEX_SCALAR) over AB_VALUES
#   bare    the bare `python bench.py` line, as the driver runs it
#   t:FILE  pytest -v on one test file (FILE may carry a ::test selector)
#   pcopy   tools/probe_copy: copy / write / read / C2-mix under flat vs persistent grids (build it first)
#   hbm     tools/probe_hbm: copy / read / random-chunk gather / C2-pattern rates (build it first)
#   prand   tools/probe_rand: dependent-chain latency and random line-request rates vs wave count (build it first)
# Output: gpurun_out/$TAG/ (TAG from the environment, default "run").
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-run}
mkdir -p "$O"
export TMPDIR=/tmp
# raw profiler output (SQLite databases, hundreds of MB) stays on the box; $O gets summaries
R=/tmp/gr_${TAG:-run}
mkdir -p "$R"
PMC_JSON=$O/pmc_dense_apply.json
[ -f "$PMC_JSON" ] || PMC_JSON=profiles/r04/pmc_dense_apply.json
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
    stats) run stats 300 rocprofv3 --kernel-trace --stats -d "$R/stats" -o c2 -- python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 --skip-walked --no-extras
           python3 tools/kernel_stats.py "$(find "$R/stats" -name '*.db' | head -1)" "$O/c2_kernel_stats.csv" && head -4 "$O/c2_kernel_stats.csv" | cut -c1-160 ;;
    ptrace3) say "ptrace3"   # kernel trace of one pipelined C3 measurement (tools/c3_pipe_only.py)
      timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/ptrace3" -o pt -- python3 tools/c3_pipe_only.py --steps 30 --warmup 3 > "$O/ptrace3.log" 2>&1 || { echo "!! ptrace3"; tail -20 "$O/ptrace3.log"; exit 1; }
      f=$(find "$R/ptrace3" -name "*kernel_trace.csv" | head -1); cp "$f" "$O/c3_pipe_kernel_trace.csv" && tail -1 "$O/ptrace3.log" ;;
    stats3) run stats3 300 rocprofv3 --kernel-trace --stats -d "$R/stats3" -o c3 -- python3 bench.py --workload c3 --steps 20 --warmup 3 --cpu-seconds 0
           python3 tools/kernel_stats.py "$(find "$R/stats3" -name '*.db' | head -1)" "$O/c3_kernel_stats.csv" && head -6 "$O/c3_kernel_stats.csv" | cut -c1-160 ;;
    pmc)
      P=1
      for ctrs in "TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "FETCH_SIZE" "WRITE_SIZE"; do
        say "pmc pass $P: $ctrs"
        timeout -s KILL 120 rocprofv3 --pmc $ctrs -d "$R/pmc/p$P" -o pmc -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --skip-walked --no-extras \
          > "$O/pmc_p$P.log" 2>&1 || { echo "!! pmc pass $P"; tail -5 "$O/pmc_p$P.log"; exit 1; }
        P=$((P+1))
      done
      python3 tools/pmc_summary.py "$R/pmc" "$O/pmc_dense_apply.json" || exit 1
      PMC_JSON=$O/pmc_dense_apply.json ;;
    pmcc3)
      say "pmc c3: DRAM-side request bytes"
      timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum \
        -d "$R/pmcc3" -o pmc -- python3 bench.py --workload c3 --steps 10 --warmup 2 --cpu-seconds 0 > "$O/pmcc3.log" 2>&1 \
        || { echo "!! pmcc3"; tail -5 "$O/pmcc3.log"; exit 1; }
      python3 tools/pmc_c3.py "$R/pmcc3" "$O/pmc_c3.json" || exit 1 ;;
    spread)   # C2 spread vs translation: alternating layouts, each a fresh process under the UTCL1 counters
      i=0
      for lay in 0 1 0 1 0 1; do
        i=$((i+1)); say "spread pass $i layout $lay"
        timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_CLIENT_UTCL1_INFLIGHT_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_UTCL1_REQUEST_sum \
          -d "$R/spread/p$i" -o pmc -- python3 tools/spread_c2.py --layout $lay > "$O/spread_p$i.log" 2>&1 || { echo "!! spread $i"; tail -5 "$O/spread_p$i.log"; exit 1; }
        grep -h '^{' "$O/spread_p$i.log" | cut -c1-200
      done
      for i in 1 2 3 4 5 6; do
        python3 tools/pmc_db.py $(find "$R/spread/p$i" -name '*.db') > "$O/spread_pmc_p$i.json" || exit 1
      done
      for i in 1 2 3 4 5 6; do echo "=== p$i $(grep -h '^{' $O/spread_p$i.log | cut -c1-60)"; python3 -c "
import json; d=json.load(open('$O/spread_pmc_p$i.json'))
for db, ks in d.items():
    for k, v in ks.items():
        if 'dense_apply' in k:
            m=v.get('TCP_UTCL1_TRANSLATION_MISS_sum',0); f=v.get('TCP_CLIENT_UTCL1_INFLIGHT_sum',0)
            print(' miss', round(m), 'inflight/miss', round(f/m,1) if m else None, 'credits', round(v.get('TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum',0)), 'req', round(v.get('TCP_UTCL1_REQUEST_sum',0)))"; done ;;
    spread2)  # the same without the profiler: 12 rounds per process, layouts alternating
      i=0
      for lay in 0 1 0 1 0 1; do
        i=$((i+1)); run spread2_p$i 120 python3 tools/spread_c2.py --layout $lay --rounds 12 || exit 1
      done
      for i in 1 2 3 4 5 6; do grep -h '^{' $O/spread2_p$i.log | cut -c1-330; done ;;
    listpmc) timeout -s KILL 60 rocprofv3 -L > "$R/counters.txt" 2>&1; echo "listpmc rc=$?"; grep -o "SQ_[A-Z_0-9]*\|TCC_[A-Z_0-9]*\|TCP_[A-Z_0-9]*\|TA_[A-Z_0-9]*\|TD_[A-Z_0-9]*" "$R/counters.txt" | sort -u > "$O/counter_names.txt"; wc -l < "$O/counter_names.txt" ;;
    pmc3)
      P=1
      for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
                  "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
                  "TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH"; do
        say "pmc3 pass $P: $ctrs"
        timeout -s KILL 90 rocprofv3 --pmc $ctrs -d "$R/pmc3/p$P" -o pmc -- python3 bench.py --workload c3 --steps 3 --warmup 1 --cpu-seconds 0 \
          > "$O/pmc3_p$P.log" 2>&1 || { echo "!! pmc3 pass $P"; tail -5 "$O/pmc3_p$P.log"; exit 1; }
        P=$((P+1))
      done
      python3 tools/pmc_db.py $(find "$R/pmc3" -name '*.db' | sort) > "$O/pmc3.json" && echo "pmc3 summarised" ;;
    salu)   # instruction mix of the C3 apply per timing probe (PSX_ORD_PROBE 0 full, 3 setup only, 6 image only)
      for v in ${SALU_PROBES:-0 3 6}; do
        say "salu probe $v"
        PSX_LIB=parameter_server_amd/libpsx_debug.so PSX_ORD_PROBE=$v timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM \
          -d "$R/salu/v$v" -o pmc -- python3 bench.py --workload c3 --steps 3 --warmup 1 --cpu-seconds 0 \
          > "$O/salu_v$v.log" 2>&1 || { echo "!! salu probe $v"; tail -5 "$O/salu_v$v.log"; exit 1; }
        python3 tools/pmc_db.py $(find "$R/salu/v$v" -name '*.db' | sort) > "$O/salu_v$v.json" || exit 1
      done
      python3 - "$O" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(os.path.join(sys.argv[1], "salu_v*.json"))):
    d = json.load(open(f))
    for db, ks in d.items():
        for k, c in ks.items():
            if "ordered_apply_reg_kernel<int, 1, 4" in k:
                print(os.path.basename(f), {x: round(y) for x, y in c.items()})
PY
      ;;
    c3split) i=0; for v in 1 2 3 1 2 3; do i=$((i+1)); run c3split_${i}_v$v 300 env PSX_LIB=parameter_server_amd/libpsx_debug.so PSX_ORD_SPLIT=$v python -u bench.py --workload c3 --steps 20 --warmup 3 --cpu-seconds 0 || exit 1; done
             grep -h '^{' $O/c3split_*.log | cut -c1-400 ;;
    c3walk) i=0; for v in 0 1 0 1; do i=$((i+1)); run c3walk_${i}_cus$v 300 env PSX_LIB=parameter_server_amd/libpsx_debug.so PSX_WALK_CUS=$v python -u bench.py --workload c3 --steps 20 --warmup 3 --cpu-seconds 0 || exit 1; done
            for f in $O/c3walk_*.log; do echo "$f $(grep -h '^{' $f | cut -c1-120)"; done ;;
    wtrace1) run wtrace1 200 env PSX_LIB=parameter_server_amd/libpsx_debug.so PSX_WALK_CUS=1 python -u tools/walk_trace.py && head -c 1500 "$O/wtrace1.log" ;;
    c2layout) for i in 1 2; do run c2sep_$i 300 env PSX_BENCH_SEPARATE=1 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-extras && run c2buf_$i 300 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-extras || exit 1; done
              for f in $O/c2sep_* $O/c2buf_*; do echo "$f $(grep -h '^{' $f | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["roofline"]["avg_launch_ms"], d["walked"]["value"])')"; done ;;
    c2only) run c2only 300 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-extras ;;
    c3) run c3 300 python -u bench.py --workload c3 --steps 20 --warmup 3 ;;
    c3sweep) run c3sweep 300 python -u tools/walk_sweep.py --configs "${SWEEP:-4:1:4:0}" ;;
    c3idx) run c3idx 300 python -u bench.py --workload c3 --indexed --steps 20 --warmup 3 ;;
    c4) run c4 600 python -u bench.py --workload c4 --steps 3 --warmup 1 ;;
    c5) run c5 300 python -u bench.py --workload c5 --steps 10 --warmup 2 ;;
    ada) run ada 300 python -u bench.py --adarevision --steps 10 --warmup 2 --cpu-seconds 6 ;;
    f16) run f16 300 python -u bench.py --f16-records --steps 20 --warmup 3 --cpu-seconds 0 ;;
    d125) run d125 300 python -u bench.py --density 0.125 --steps 20 --warmup 3 --cpu-seconds 0 ;;
    imp) run imp 300 python -u bench.py --importance --steps 20 --warmup 3 --cpu-seconds 0 ;;
    probe) run probe 300 tools/probe_ceiling 10 ;;
    hbm) run hbm 400 tools/probe_hbm 10 ;;
    prand) run prand 300 tools/probe_rand 5 && cat "$O/prand.log" ;;
    abstore) run abstore 300 python -u tools/ab_c2.py --configs 0:1:0,0:1:1,0:1:3,0:0:0,0:0:1,0:0:3 --rounds 5 --steps 5 && cat "$O/abstore.log" | tail -60 ;;
    abdense) run abdense 400 python -u tools/ab_c2.py --configs ${ABCONF:-0:1:1,0:0:1} --rounds 5 --steps 5 && tail -60 "$O/abdense.log" ;;
    abzeros) run abzeros 400 python -u tools/ab_c2.py --zeros --configs ${ABCONF:-0:1:1,0:0:1} --rounds 5 --steps 5 && tail -30 "$O/abzeros.log" ;;
    pushtests) run pushtests 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_ssp_gpu.py tests/test_push_body_gpu.py tests/test_matrixfact_gpu.py tests/test_app_drivers_gpu.py tests/test_configs_gpu.py ;;
    mrtest) run mrtest 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_multi_rank_gpu.py tests/test_split_gpu.py ;;
    walktests) run walktests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_walk_gpu.py tests/test_sparse_gpu.py tests/test_indexed_rows_gpu.py tests/test_ord_split_gpu.py tests/test_kats_gpu.py ;;
    newtests) run newtests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dense_gpu.py tests/test_indexed_rows_gpu.py tests/test_ord_split_gpu.py ;;
    mixab) for i in 1 2 3; do run pmix_$i 300 tools/probe_apply 10 1 && run abdense_$i 400 python -u tools/ab_c2.py --configs 0:1:1,0:0:1 --rounds 3 --steps 5 || exit 1; done
           grep -h '"probe"' $O/pmix_*.log | head -3; grep -h -A2 '"apply0' $O/abdense_*.log | grep dense_apply ;;
    wtrace) run wtrace 200 python -u tools/walk_trace.py && head -c 3000 "$O/wtrace.log" ;;
    pphase) run pphase 120 tools/probe_phase 10 && cat "$O/pphase.log" ;;
    papply) run papply 300 tools/probe_apply 10 && cat "$O/papply.log" ;;
    pmix) run pmix 300 tools/probe_apply 10 1 && cat "$O/pmix.log" ;;
    c3lib) i=0; for v in new old new old; do i=$((i+1)); L=; [ $v = old ] && L=ab_old/libpsx.so
             run c3lib_${i}_$v 300 env PSX_LIB=$L python -u bench.py --workload c3 --steps 20 --warmup 3 --cpu-seconds 0 || exit 1; done
           for f in $O/c3lib_*.log; do echo "$f $(grep -h '^{' $f | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["kernel_ms_per_step_breakdown_pass"])')"; done ;;
    c3libs) i=0; for r in 1 2; do for L in ${LIBS:-new}; do i=$((i+1)); n=$(echo "$L" | tr '/' '_'); P=$L; [ "$L" = new ] && P=
              run c3libs_${i}_$n 300 env PSX_LIB=$P python -u bench.py --workload c3 --steps 20 --warmup 3 --cpu-seconds 0 || exit 1; done; done
            for f in $O/c3libs_*.log; do echo "$f $(grep -h '^{' $f | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["kernel_ms_per_step_breakdown_pass"])')"; done ;;
    c2lib) i=0; for v in new old new old; do i=$((i+1)); L=; [ $v = old ] && L=ab_old/libpsx.so
             run c2lib_${i}_$v 300 env PSX_LIB=$L python -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-extras --skip-walked || exit 1; done
           for f in $O/c2lib_*.log; do echo "$f $(grep -h '^{' $f | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["roofline"]["avg_launch_ms"], d["roofline"]["frac_of_read_sweep"])')"; done ;;
    drift) for i in 1 2 3; do run drift_$i 300 python -u tools/ab_c2.py --configs 0:1:1 --rounds ${DRIFT_ROUNDS:-60} --steps 20 --drift || exit 1; done
           for f in $O/drift_*.log; do echo "$f"; grep -h '"round"' $f | awk 'NR%6==1' | cut -c1-120; done ;;
    tlb) for i in 1 2 3 4; do
           say "tlb pass $i"
           timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum \
             -d "$R/tlb/p$i" -o pmc -- python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 --skip-walked --no-extras > "$O/tlb_p$i.log" 2>&1 || { echo "!! tlb pass $i"; tail -5 "$O/tlb_p$i.log"; exit 1; }
           grep -h '^{' "$O/tlb_p$i.log" | python3 -c 'import json,sys; d=json.load(sys.stdin); print("avg_launch_ms", d["roofline"]["avg_launch_ms"])'
         done
         python3 tools/pmc_db.py $(find "$R/tlb" -name '*.db' | sort) > "$O/tlb.json" && python3 -c "
import json; d=json.load(open('$O/tlb.json'))
for db, ks in d.items():
    for k, v in ks.items():
        if 'dense_apply' in k: print(db[-40:], {c: round(x) for c, x in v.items()})" ;;
    c3wc) i=0; for v in 1 0 1 0; do i=$((i+1)); run c3wc_${i}_v$v 300 env PSX_LIB=parameter_server_amd/libpsx_debug.so PSX_WALK_COUNT=$v python -u bench.py --workload c3 --steps 20 --warmup 3 --cpu-seconds 0 || exit 1; done
          for f in $O/c3wc_*.log; do echo "$f $(grep -h '^{' $f | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["kernel_ms_per_step_breakdown_pass"], d.get("pipelined",{}).get("value"))')"; done ;;
    wctests) run wctests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_walk_count_gpu.py tests/test_walk_gpu.py tests/test_sparse_gpu.py tests/test_ord_split_gpu.py tests/test_kats_gpu.py tests/test_indexed_rows_gpu.py ;;
    oldheavy) say oldheavy; timeout -k 10 300 env PSX_LIB=ab_old/libpsx.so python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ord_split_gpu.py -k every_row_heavy > "$O/oldheavy.log" 2>&1; echo "oldheavy rc=$? (the pre-fix library: a failure here is the collision)"; tail -5 "$O/oldheavy.log" ;;
    c3fold) i=0; for v in 1 0 1 0; do i=$((i+1)); run c3fold_${i}_v$v 300 env PSX_LIB=parameter_server_amd/libpsx_debug.so PSX_FOLD_FINISH=$v python -u bench.py --workload c3 --steps 20 --warmup 3 --cpu-seconds 0 || exit 1; done
            for f in $O/c3fold_*.log; do echo "$f $(grep -h '^{' $f | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["kernel_ms_per_step_breakdown_pass"], d.get("pipelined",{}).get("value"))')"; done ;;
    c3lev) i=0; for v in 4 0 4 0; do i=$((i+1)); run c3lev_${i}_v$v 300 env PSX_LIB=parameter_server_amd/libpsx_debug.so PSX_WALK_LEVELS=$v python -u bench.py --workload c3 --steps 20 --warmup 3 --cpu-seconds 0 || exit 1; done
            for f in $O/c3lev_*.log; do echo "$f $(grep -h '^{' $f | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["kernel_ms_per_step_breakdown_pass"], d.get("pipelined",{}).get("value"))')"; done ;;
    walkonly) run walkonly 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_walk_gpu.py ;;
    xtests) run xtests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_split_gpu.py tests/test_walk_count_gpu.py tests/test_multi_rank_gpu.py ;;
    splittests) run splittests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ord_split_gpu.py tests/test_sparse_gpu.py tests/test_kats_gpu.py ;;
    pcopy) run pcopy 300 tools/probe_copy 10 ${PCOPY:-all} && cat "$O/pcopy.log" ;;
    bare) run bare 900 python -u bench.py ;;
    c2ab) i=0; for v in ${AB_VALUES:-0 1 0 1}; do i=$((i+1)); run c2ab_${i}_v$v 300 env PSX_LIB=parameter_server_amd/libpsx_debug.so ${AB_VAR:-PSX_INDEX_SCALAR}=$v python -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-extras || exit 1; done
            for f in $O/c2ab_*.log; do echo "$f $(grep -h "^{" $f | python3 -c "import json,sys; d=json.load(sys.stdin); print(d[\"value\"], d[\"roofline\"][\"avg_launch_ms\"], d.get(\"walked\",{}).get(\"value\"), d.get(\"walked\",{}).get(\"ms_per_step\"))")"; done ;;
    c3ab) i=0; for v in ${AB_VALUES:-0 1 0 1}; do i=$((i+1)); run c3ab_${i}_v$v 300 env PSX_LIB=parameter_server_amd/libpsx_debug.so ${AB_VAR:-PSX_ORD_LITE}=$v python -u bench.py --workload c3 --steps 20 --warmup 3 --cpu-seconds 0 || exit 1; done
            for f in $O/c3ab_*.log; do echo "$f $(grep -h '^{' $f | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["kernel_ms_per_step_breakdown_pass"], d.get("pipelined",{}).get("value"))')"; done ;;
    t:*) f=${s#t:}; run t_$(basename "$f" .py) 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread "$f" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
say done
