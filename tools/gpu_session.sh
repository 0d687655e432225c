#!/usr/bin/env bash
# One gpurun session. Steps (FMGI_STEPS, space separated):
#   tests            pytest -m gpu
#   smoke            __graft_entry__.smoke()
#   tests_k          pytest -m gpu $TESTS_ARGS, with -k "$TESTS_K" when set
#   rad / radprof    tools/bench_rad.py $RAD_ARGS (plain / under rocprofv3 --kernel-trace --stats)
#   ref              reference-kernel pin (tests/golden/make_ref_fixtures.py)
#   tol              whole-launch reference sums, strict and relaxed (tests/golden/make_tolerance_fixtures.py)
#   ocml             the device library's sin/cos digest (tests/golden/make_ocml_fixture.py)
#   valu             VALU issue ceilings (tools/valu_peak)
#   valupmc          the same cases' SQ issue counters (one rocprofv3 --pmc pass per case, 1/2/4/8 waves)
#   dropin           drop-in boundary timing, cached and uncached (tools/bench_dropin.py)
#   dropinprof       the same under rocprofv3 --kernel-trace --stats
#   bench            python bench.py $BENCH_ARGS
#   env_<tag>        bench.py (no CPU legs) under the environment assignments in $ENV_<TAG>
#   ab               bench.py (no CPU legs) with each experiment build in $AB_LIBS (FMGI_LIB), then the default build
#   bench_<tag>      python bench.py with the args in $BENCH_<TAG> (e.g. BENCH_FX3="--accum fx3"), under the
#                    environment assignments in $ENVB_<TAG> if set
#   prof             rocprofv3 --kernel-trace --stats on a short bench ($PROF_ARGS)
#   prof_<tag>       the same with the bench args in $PROF_<TAG>
#   pmc              rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes on a short bench ($PROF_ARGS)
#   foldpmc          one rocprofv3 --pmc pass of LDS-pipe counters (the fold kernels' binding resource)
#   sq               two rocprofv3 --pmc passes of SQ instruction / wait counters ($PROF_ARGS)
#   grbm / tcp / sq3 one --pmc pass each: GRBM clock + SQ cycle split / TA-TD-TCP (vector memory path) / SQ memory issue
#   rehearse         bench.py's N-rank path with REHEARSE_N (default 2) gloo ranks sharing the box's one GPU
#   clock            bench with the in-kernel clock build (make -C <pkg> variant VNAME=clock VFLAGS=-DFMGI_CLOCK_STAMP)
#   counters         per config in $COUNTER_CONFIGS (default box200 example box2000), into $OUT/<config>/: the bench
#                    line (bench_<config>.log in $OUT), kernel trace, FETCH/WRITE, SQ, GRBM, TA/TD/TCP passes and the
#                    clock build; then tools/{timed_launches,sq_summary,pmc_summary}.py over them (the summaries are
#                    written to $OUT/sq_issue.json and $OUT/pmc_traffic.json; copy them to profiles/ after review)
#   adopt            copies this session's $OUT/sq_issue.json and pmc_traffic.json over profiles/ on the box, so that
#                    bench lines later in the session report them (commit the same files after review)
# Each GPU step has its own time limit; a crash/timeout (rc > 1) stops the session.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${FMGI_SESSION:-s1}
mkdir -p "$OUT"
step() {  # step <name> <timeout-seconds> <cmd...>
    local name=$1 t=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-2000
    if [ $rc -gt 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
python -c "import __graft_entry__ as g; g.build()" || exit 3
export TMPDIR=/tmp
for s in ${FMGI_STEPS:-tests ref bench prof}; do
  case $s in
    tests) step tests 1100 python -u -m pytest tests -m gpu -v -x -p no:cacheprovider --timeout 900 --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" ;;
    tests_k) if [ -n "${TESTS_K:-}" ]; then
               step tests_k 900 python -u -m pytest -m gpu -v -x -p no:cacheprovider --timeout 300 --timeout-method thread -k "$TESTS_K" ${TESTS_ARGS:-tests}
             else
               step tests_k 900 python -u -m pytest -m gpu -v -x -p no:cacheprovider --timeout 300 --timeout-method thread ${TESTS_ARGS:-tests}
             fi ;;
    rad)   step rad 900 python tools/bench_rad.py ${RAD_ARGS:-} ;;
    radprof) step radprof 900 rocprofv3 --kernel-trace --stats -d "$OUT/radprof" -o run --output-format csv -- python tools/bench_rad.py --reps 1 --no-cpu-baseline ${RAD_ARGS:-} ;;
    ref)   step ref 600 python tests/golden/make_ref_fixtures.py "$OUT" ;;
    tol)   step tol 1100 env GPU_MAX_HW_QUEUES=16 python -u tests/golden/make_tolerance_fixtures.py "$OUT" ;;
    ocml)  step ocml 300 python tests/golden/make_ocml_fixture.py "$OUT" ;;
    valu)  step valu 300 ./tools/valu_peak ;;
    valupmc) for c in fma8 fma64 pk_fma64 fma64_salu64; do
               step "valupmc_$c" 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -d "$OUT/valupmc_$c" -o run --output-format csv -- ./tools/valu_peak $c 1,2,4,8 --ms 20 || exit $?
             done ;;
    dropin) step dropin 600 python tools/bench_dropin.py && step dropin_nocache 600 python tools/bench_dropin.py --no-cache ;;
    dropinprof) step dropinprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/dropinprof" -o run --output-format csv -- python tools/bench_dropin.py --reps 2 ;;
    bench) step bench 600 python bench.py ${BENCH_ARGS:-} ;;
    ab)    for v in ${AB_LIBS:-base}; do step "ab_$v" 600 env FMGI_LIB=$v python bench.py --no-cpu-baseline ${AB_ARGS:-}; done &&
           step ab_default 600 python bench.py --no-cpu-baseline ${AB_ARGS:-} ;;
    env_*) v="ENV_$(echo "${s#env_}" | tr a-z A-Z)"; step "$s" 600 env ${!v} python bench.py --no-cpu-baseline ${AB_ARGS:-} ;;
    bench_*) v="BENCH_$(echo "${s#bench_}" | tr a-z A-Z)"; e="ENVB_$(echo "${s#bench_}" | tr a-z A-Z)"
             step "$s" 600 env ${!e:-} python bench.py ${!v:-} ;;
    prof_*) v="PROF_$(echo "${s#prof_}" | tr a-z A-Z)"
            step "$s" 600 rocprofv3 --kernel-trace --stats -d "$OUT/$s" -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline ${!v:-} ;;
    prof)  step prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline ${PROF_ARGS:-} ;;
    pmclist) step pmclist 120 rocprofv3 -L ;;
    sq)    step sq1 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU -d "$OUT/sq1" -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline ${PROF_ARGS:-} &&
           step sq2 600 rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_BRANCH -d "$OUT/sq2" -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline ${PROF_ARGS:-} ;;
    foldpmc) step fold_lds 600 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS -d "$OUT/fold_lds" -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline ${PROF_ARGS:-} ;;
    grbm)  step grbm 600 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d "$OUT/grbm" -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline ${PROF_ARGS:-} ;;
    tcp)   step tcp 600 rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum GRBM_GUI_ACTIVE -d "$OUT/tcp" -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline ${PROF_ARGS:-} ;;
    sq3)   step sq3 600 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_SCA -d "$OUT/sq3" -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline ${PROF_ARGS:-} ;;
    rehearse) step rehearse 600 env FMGI_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node ${REHEARSE_N:-2} --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus ${REHEARSE_N:-2} --steps 3 --warmup 1 --no-cpu-baseline ;;
    clock) step clock 600 env FMGI_LIB=clock python bench.py --steps 5 --warmup 3 --no-cpu-baseline ${PROF_ARGS:-} ;;
    counters) for cfg in ${COUNTER_CONFIGS:-box200 example box2000}; do
               C=(--config "$cfg"); D="$OUT/$cfg"; mkdir -p "$D"
               step "bench_$cfg" 600 python bench.py --no-cpu-baseline "${C[@]}" &&
               step "$cfg/prof" 600 rocprofv3 --kernel-trace --stats -d "$D/prof" -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline "${C[@]}" &&
               step "$cfg/pmc_fetch" 600 rocprofv3 --pmc FETCH_SIZE -d "$D/pmc_fetch" -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline "${C[@]}" &&
               step "$cfg/pmc_write" 600 rocprofv3 --pmc WRITE_SIZE -d "$D/pmc_write" -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline "${C[@]}" &&
               step "$cfg/sq1" 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU -d "$D/sq1" -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline "${C[@]}" &&
               step "$cfg/sq2" 600 rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_BRANCH -d "$D/sq2" -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline "${C[@]}" &&
               step "$cfg/sq3" 600 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_SCA -d "$D/sq3" -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline "${C[@]}" &&
               step "$cfg/grbm" 600 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d "$D/grbm" -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline "${C[@]}" &&
               step "$cfg/tcp" 600 rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum GRBM_GUI_ACTIVE -d "$D/tcp" -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline "${C[@]}" &&
               step "$cfg/clock" 600 env FMGI_LIB=clock python bench.py --steps 5 --warmup 3 --no-cpu-baseline "${C[@]}" || exit $?
               grep '^{' "$D/clock.log" > "$D/bench_clock.json"
               python tools/timed_launches.py "$D/prof/run_kernel_trace.csv" "$D/kernel_timed_launches.json" > /dev/null &&
               python tools/sq_summary.py "$D" "$cfg" --out "$OUT/sq_issue.json" > "$D/sq_summary.txt" &&
               python tools/pmc_summary.py "$D" "$cfg" --out "$OUT/pmc_traffic.json" > "$D/pmc_summary.txt" || exit 4
             done ;;
    adopt) cp "$OUT/sq_issue.json" "$OUT/pmc_traffic.json" profiles/ || exit 4 ;; # this session's summaries, for the bench lines after it
    pmc)   step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline ${PROF_ARGS:-} &&
           step pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline ${PROF_ARGS:-} ;;
  esac
done
echo "session done"
