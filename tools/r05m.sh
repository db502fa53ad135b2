set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05m_c4_0.4 -o run --output-format csv -- python3 bench.py --config c4 --scale 0.4 --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --no-resident --c4-strong off > gpurun_out/prof_r05m_c4_0.4.log 2>&1 || { tail -20 gpurun_out/prof_r05m_c4_0.4.log; exit 1; }
find gpurun_out/prof_r05m_c4_0.4 -name "*kernel_stats.csv" -exec cp {} gpurun_out/r05m_c4_0.4_kernel_stats.csv \;
tail -c 600 gpurun_out/prof_r05m_c4_0.4.log
echo done
