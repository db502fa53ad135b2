#!/bin/bash
# usage (on the GPU box via gpurun): tools/gpu_round.sh <tag> [tests|bench|prof]...
# Each GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
mkdir -p gpurun_out
for step in "$@"; do
  case $step in
    tests)
      timeout -k 10 1150 python -u -m pytest tests -m gpu -x -v --durations=40 --timeout 600 --timeout-method thread \
        > gpurun_out/tests_$TAG.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/tests_$TAG.log; exit 1; } ;;
    bench)
      timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
        || { echo "bench failed"; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
      head -c 2500 gpurun_out/bench_$TAG.json ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv \
        -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 \
        || { echo "prof failed"; tail -30 gpurun_out/prof_$TAG.log; exit 1; }
      find gpurun_out/prof_$TAG -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_$TAG.kernel_stats.csv \;
      head -25 gpurun_out/prof_$TAG.kernel_stats.csv ;;
    configs|configs:*)  # the other BASELINE shapes on one GPU, each with its CPU baseline (a bounded sample where the
      # full run is too long; bench.py CPU_SAMPLE_SCALE).  configs:<cfg>@<scale>,... picks them
      LIST="c1@1.0 c3@0.5 c3@1.0 c4@0.05 c4@0.4 c5@0.1 c5@0.3"
      [ "$step" != configs ] && LIST=$(echo "${step#configs:}" | tr ',' ' ')
      for cs in $LIST; do
        CFG=${cs%@*}; SC=${cs#*@}
        echo "config $CFG scale $SC" >&2
        timeout -k 10 500 python -u bench.py --config $CFG --scale $SC --steps 3 --warmup 1 --no-ingest \
          > gpurun_out/cfg_${TAG}_${CFG}_$SC.json 2> gpurun_out/cfg_${TAG}_${CFG}_$SC.err \
          || { echo "config $CFG $SC failed"; tail -20 gpurun_out/cfg_${TAG}_${CFG}_$SC.err; exit 1; }
        head -c 600 gpurun_out/cfg_${TAG}_${CFG}_$SC.json; echo
      done ;;
    cprof:*)  # cprof:<config>:<scale> -- kernel stats of one step of another BASELINE shape
      IFS=: read -r _ CFG SC <<< "$step"
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/cprof_${TAG}_$CFG -o run --output-format csv \
        -- python3 bench.py --config $CFG --scale $SC --steps 2 --warmup 1 --no-cpu-baseline --no-ingest \
        > gpurun_out/cprof_${TAG}_$CFG.log 2>&1 \
        || { echo "cprof $CFG failed"; tail -30 gpurun_out/cprof_${TAG}_$CFG.log; exit 1; }
      find gpurun_out/cprof_${TAG}_$CFG -name "*kernel_stats.csv" -exec cp {} gpurun_out/cprof_${TAG}_$CFG.kernel_stats.csv \;
      cut -c1-60,200- gpurun_out/cprof_${TAG}_$CFG.kernel_stats.csv | head -30 ;;
    qprof)
      timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/qprof_$TAG -o run --output-format csv \
        -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/qprof_$TAG.log 2>&1 \
        || { echo "qprof failed"; tail -30 gpurun_out/qprof_$TAG.log; exit 1; }
      python3 tools/trace_step.py gpurun_out/qprof_$TAG/run_kernel_trace.csv | awk '$2 > 40 || /total/' ;;
    pmc)
      tools/pmc.sh $TAG || exit 1 ;;
    pmc:*)  # pmc:<config>:<scale> -- the PMC passes on another BASELINE shape
      IFS=: read -r _ CFG SC <<< "$step"
      tools/pmc.sh ${TAG}_$CFG --config $CFG --scale $SC || exit 1 ;;
    lstats)
      timeout -k 10 300 python -u tools/light_stats.py c2 1.0 > gpurun_out/lstats_$TAG.log 2>&1 \
        || { echo "lstats failed"; tail -30 gpurun_out/lstats_$TAG.log; exit 1; }
      grep LIGHT_STATS gpurun_out/lstats_$TAG.log ;;
    quick)
      timeout -k 10 300 python -u tools/gpu_quick.py > gpurun_out/quick_$TAG.log 2>&1 \
        || { echo "quick failed"; tail -30 gpurun_out/quick_$TAG.log; exit 1; }
      tail -5 gpurun_out/quick_$TAG.log ;;
    distinct)
      timeout -k 10 300 python -u tools/distinct_bench.py > gpurun_out/distinct_$TAG.log 2>&1 \
        || { echo "distinct failed"; tail -30 gpurun_out/distinct_$TAG.log; exit 1; }
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/dprof_$TAG -o run --output-format csv \
        -- python3 tools/distinct_bench.py > gpurun_out/dprof_$TAG.log 2>&1 \
        || { echo "distinct prof failed"; tail -30 gpurun_out/dprof_$TAG.log; exit 1; }
      find gpurun_out/dprof_$TAG -name "*kernel_stats.csv" -exec cp {} gpurun_out/dprof_$TAG.kernel_stats.csv \;
      grep DISTINCT gpurun_out/distinct_$TAG.log; grep distinct gpurun_out/dprof_$TAG.kernel_stats.csv | cut -c1-40,150- ;;
    parse)
      timeout -k 10 400 python -u tools/parse_bench.py > gpurun_out/parse_$TAG.log 2>&1 \
        || { echo "parse failed"; tail -30 gpurun_out/parse_$TAG.log; exit 1; }
      grep -E "PARSE|text" gpurun_out/parse_$TAG.log ;;
    pprof)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/pprof_$TAG -o run --output-format csv \
        -- python3 tools/parse_bench.py > gpurun_out/pprof_$TAG.log 2>&1 \
        || { echo "parse prof failed"; tail -30 gpurun_out/pprof_$TAG.log; exit 1; }
      find gpurun_out/pprof_$TAG -name "*kernel_stats.csv" -exec cp {} gpurun_out/pprof_$TAG.kernel_stats.csv \;
      grep -E "k_nt|scan" gpurun_out/pprof_$TAG.kernel_stats.csv | cut -c1-40,150- ;;
    rehearse:*)  # rehearse:<config>:<scale>:<ranks> -- sharded bench with several ranks on the one GPU (gloo)
      IFS=: read -r _ CFG SC NR <<< "$step"
      tools/shard_rehearsal.sh ${TAG}_${CFG}_$NR $CFG $SC $NR || exit 1 ;;
    tfile:*)  # tfile:<test file>[,<test file>...][@-k expr] -- GPU test files (one pytest process), with a heartbeat
      SPEC=${step#tfile:}; FILES=$(echo "${SPEC%%@*}" | tr ',' ' '); KEXPR=""
      [[ "$SPEC" == *@* ]] && KEXPR="${SPEC#*@}"
      timeout -k 10 1000 python -u -m pytest $FILES -m gpu -x -v --timeout 600 --timeout-method thread ${KEXPR:+-k "$KEXPR"} \
        > gpurun_out/tfile_$TAG.log 2>&1 &
      PID=$!
      while kill -0 $PID 2>/dev/null; do sleep 30; echo "[hb $(date +%T)] $(grep -cE 'PASSED' gpurun_out/tfile_$TAG.log) passed"; done
      wait $PID || { echo "tfile failed"; tail -60 gpurun_out/tfile_$TAG.log; exit 1; }
      grep -cE "PASSED" gpurun_out/tfile_$TAG.log; tail -2 gpurun_out/tfile_$TAG.log ;;
    benchcfg:*)  # benchcfg:<config>:<scale>:<steps> -- one BASELINE shape on one GPU, with a heartbeat (long steps)
      IFS=: read -r _ CFG SC NS <<< "$step"
      timeout -k 10 1000 python -u bench.py --config $CFG --scale $SC --steps $NS --warmup 0 --no-cpu-baseline --no-ingest --no-resident --page-log \
        > gpurun_out/bcfg_${TAG}_$CFG.json 2> gpurun_out/bcfg_${TAG}_$CFG.err &
      PID=$!
      while kill -0 $PID 2>/dev/null; do sleep 30; echo "[hb $(date +%T)] $(tail -c 200 gpurun_out/bcfg_${TAG}_$CFG.err | tr '\n' ' ')"; done
      wait $PID || { echo "benchcfg $CFG failed"; tail -30 gpurun_out/bcfg_${TAG}_$CFG.err; exit 1; }
      cat gpurun_out/bcfg_${TAG}_$CFG.json ;;
    gtest:*)  # gtest:<pytest -k expression> -- a subset of the GPU tests
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${step#gtest:}" \
        > gpurun_out/gtest_$TAG.log 2>&1 || { echo "gtest failed"; tail -30 gpurun_out/gtest_$TAG.log; exit 1; }
      tail -3 gpurun_out/gtest_$TAG.log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "all steps ok"
