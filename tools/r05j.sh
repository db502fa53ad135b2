set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_gpu_program_paged.py -m gpu -x -q --timeout 300 --timeout-method thread -k "oom_fallback or join_range or synthetic_configs or random_parity or heavy_paths" > gpurun_out/r05j_tests.log 2>&1 || { tail -30 gpurun_out/r05j_tests.log; exit 1; }
tail -2 gpurun_out/r05j_tests.log
RDFIND_MEM_REPORT=1 timeout -k 10 300 python -u bench.py --config c4 --scale 1.0 --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --no-resident --c4-strong off > gpurun_out/c4mem_r05j.json 2> gpurun_out/c4mem_r05j.err || { tail -20 gpurun_out/c4mem_r05j.err; exit 1; }
grep MEM gpurun_out/c4mem_r05j.err | tail -1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05j_c2only -o run --output-format csv -- python3 bench.py --no-cpu-baseline --c4-strong off > gpurun_out/prof_r05j_c2only.log 2>&1 || { tail -20 gpurun_out/prof_r05j_c2only.log; exit 1; }
find gpurun_out/prof_r05j_c2only -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_r05j_c2only.kernel_stats.csv \;
RDFIND_AB_LIBS=librdfind_hip.so,librdfind_hip_sg32k.so,librdfind_hip_sr16.so,librdfind_hip_sr4g.so timeout -k 10 400 python -u tools/light_ab.py c4:0.4 > gpurun_out/k2_ab_r05j.log 2>&1 || { tail -20 gpurun_out/k2_ab_r05j.log; exit 1; }
echo done
