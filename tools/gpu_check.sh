#!/bin/bash
# Runs ON THE GPU BOX (via gpurun): stages given as arguments, in order, each under its own
# time limit; stops at the first stage that faults / aborts / times out (pytest failures,
# rc=1, still let later stages run so a bench line is recorded).
#   stages: pytest smoke bench bench8 prof pmc sel walk wprof whbm wpmc cprof cpmc c5prof ...
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  echo "== $name: $*" >> gpurun_out/steps.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >> gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  return $rc
}
for st in "$@"; do
  case $st in
    pytest) run pytest_gpu 1200 python -m pytest tests -m gpu -x -q -p no:cacheprovider; rc=$?
            if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi ;;
    pyall)  run pytest_all 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf; rc=$?
            if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi ;;
    sel)    run pytest_sel 1100 python -u -m pytest ${PYSEL} -x -v --timeout 400 --timeout-method thread -p no:cacheprovider; rc=$?
            if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi ;;
    smoke)  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench)  run bench 900 python bench.py || exit $? ;;
    benchq) run benchq 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --net-steps 0 || exit $? ;;
    prof)   run prof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv \
                -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --net-steps 0 || exit $? ;;
    diag)   run diag 600 python tools/diag_c4.py || exit $? ;;
    pmc)    run pmc 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc -o pmc \
                --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
                -- python3 tools/one_search.py --reps 2 || exit $? ;;
    pmcx)   run pmcx 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmcx -o pmc \
                --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
                -- python3 tools/one_search.py --reps 2 --mode philox || exit $? ;;
    hbm)    run hbm_fetch 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/hbm -o fetch \
                --pmc FETCH_SIZE -- python3 tools/one_search.py --reps 2 || exit $?
            run hbm_write 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/hbm -o write \
                --pmc WRITE_SIZE -- python3 tools/one_search.py --reps 2 || exit $? ;;
    sprof)  run sprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/sprof -o run --output-format csv \
                -- python3 tools/prof_search.py --steps 60 || exit $? ;;
    spmc)   run spmc 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/spmc -o pmc \
                --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
                -- python3 tools/prof_search.py --steps 60 || exit $? ;;
    shbm)   run shbm_fetch 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/shbm -o fetch \
                --pmc FETCH_SIZE -- python3 tools/prof_search.py --steps 60 || exit $?
            run shbm_write 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/shbm -o write \
                --pmc WRITE_SIZE -- python3 tools/prof_search.py --steps 60 || exit $? ;;
    walk)   run walk 300 python3 tools/prof_walk.py --reps 5 || exit $? ;;
    wprof)  run wprof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/wprof -o run --output-format csv \
                -- python3 tools/prof_walk.py --reps 3 || exit $? ;;
    whbm)   run whbm_fetch 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/whbm -o fetch \
                --pmc FETCH_SIZE -- python3 tools/prof_walk.py --reps 3 || exit $?
            run whbm_write 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/whbm -o write \
                --pmc WRITE_SIZE -- python3 tools/prof_walk.py --reps 3 || exit $? ;;
    wpmc)   run wpmc 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/wpmc -o pmc \
                --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
                -- python3 tools/prof_walk.py --reps 3 || exit $? ;;
    cprof)  run cprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/cprof -o run --output-format csv \
                -- python3 tools/bench_chess.py --mode crude --steps 2 || exit $? ;;
    cpmc)   run cpmc 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/cpmc -o pmc \
                --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
                -- python3 tools/bench_chess.py --mode crude --steps 2 || exit $? ;;
    c5prof) ZC_PUCT_STREAMS=4 run c5prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/c5prof -o run --output-format csv \
                -- python3 tools/prof_c5.py --mode c5 --steps 3 || exit $? ;;
    ab)     run ab 900 env AB_ROOTS=mixed AB_ROUNDS=${AB_ROUNDS:-3} python tools/ab_search.py ${AB_LIBS} || exit $? ;;
    *) echo "unknown stage $st"; exit 2 ;;
  esac
done
