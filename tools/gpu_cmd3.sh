set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for cfg in "c1 1.0" "c3 0.5" "c3 1.0" "c4 0.05" "c4 0.4" "c5 0.1" "c5 0.3"; do
  set -- $cfg
  echo "config $1 scale $2"
  timeout -k 10 400 python -u bench.py --config $1 --scale $2 --steps 3 --warmup 1 --no-cpu-baseline --no-ingest \
    > gpurun_out/cfg_r03g_$1_$2.json 2> gpurun_out/cfg_r03g_$1_$2.err || { echo "config $1 $2 failed"; tail -20 gpurun_out/cfg_r03g_$1_$2.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['value'], d['config']['cinds'], d['kernel_ms'])" gpurun_out/cfg_r03g_$1_$2.json
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/cprof_r03g_c3 -o run --output-format csv \
  -- python3 bench.py --config c3 --scale 1.0 --steps 2 --warmup 1 --no-cpu-baseline --no-ingest > gpurun_out/cprof_r03g_c3.log 2>&1 || { echo "cprof failed"; tail -20 gpurun_out/cprof_r03g_c3.log; exit 1; }
find gpurun_out/cprof_r03g_c3 -name "*kernel_stats.csv" -exec cp {} gpurun_out/cprof_r03g_c3.kernel_stats.csv \;
echo done
