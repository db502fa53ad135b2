set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu.py tests/test_gpu_sharded.py -m gpu -x -q --timeout 300 --timeout-method thread -k "join_range" > gpurun_out/r05n_tests.log 2>&1 || { tail -30 gpurun_out/r05n_tests.log; exit 1; }
tail -2 gpurun_out/r05n_tests.log
timeout -k 10 300 python -u bench.py --config c4 --scale 1.0 --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --no-resident --c4-strong off > gpurun_out/c4_r05n.json 2> gpurun_out/c4_r05n.err || { tail -20 gpurun_out/c4_r05n.err; exit 1; }
python3 -c "
import json
b=json.loads(open('gpurun_out/c4_r05n.json').read().strip().splitlines()[-1])
print(b['ms_per_step'], {k:v['ms'] for k,v in b['families'].items()})"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05n_c4_0.4 -o run --output-format csv -- python3 bench.py --config c4 --scale 0.4 --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --no-resident --c4-strong off > gpurun_out/prof_r05n_c4_0.4.log 2>&1 || { tail -20 gpurun_out/prof_r05n_c4_0.4.log; exit 1; }
find gpurun_out/prof_r05n_c4_0.4 -name "*kernel_stats.csv" -exec cp {} gpurun_out/r05n_c4_0.4_kernel_stats.csv \;
echo done
