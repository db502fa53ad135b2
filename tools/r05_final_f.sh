set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/r05_suite.sh r05z || exit 1
( timeout -k 10 600 python -u bench.py > gpurun_out/final5_bench.json 2> gpurun_out/final5_bench.err; echo "rc=$?" >> gpurun_out/final5_bench.err ) &
PID=$!
while kill -0 $PID 2>/dev/null; do sleep 45; echo "[hb $(date +%T)] $(tail -c 150 gpurun_out/final5_bench.err | tr '\n' ' ')"; done
wait $PID
grep -q "rc=0" gpurun_out/final5_bench.err || { tail -30 gpurun_out/final5_bench.err; exit 1; }
head -c 1200 gpurun_out/final5_bench.json; echo
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final5_c2 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --c4-strong off > gpurun_out/prof_final5_c2.log 2>&1 || { tail -20 gpurun_out/prof_final5_c2.log; exit 1; }
find gpurun_out/prof_final5_c2 -name "*kernel_stats.csv" -exec cp {} gpurun_out/final5_c2_kernel_stats.csv \;
echo done
