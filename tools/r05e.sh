set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "join_range or sharded_join or sharded_c4 or synthetic_configs" > gpurun_out/r05_tests_e.log 2>&1 || { tail -30 gpurun_out/r05_tests_e.log; exit 1; }
tail -2 gpurun_out/r05_tests_e.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4e -o run --output-format csv -- python3 bench.py --config c4 --scale 1.0 --steps 1 --warmup 1 --no-cpu-baseline --no-ingest --no-resident --c4-strong off > gpurun_out/prof_c4e.log 2>&1 || { tail -20 gpurun_out/prof_c4e.log; exit 1; }
find gpurun_out/prof_c4e -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_c4e.kernel_stats.csv \;
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-ingest --c4-strong off > gpurun_out/c2_r05e.json 2> gpurun_out/c2_r05e.err || exit 1
RDFIND_AB_LIBS=librdfind_hip.so,librdfind_hip_w4.so,librdfind_hip_w4b4.so,librdfind_hip_b4.so,librdfind_hip_it2.so timeout -k 10 400 python -u tools/light_ab.py c2:1.0 c3:0.5 > gpurun_out/light_ab_r05e.log 2>&1 || { tail -20 gpurun_out/light_ab_r05e.log; exit 1; }
echo done
