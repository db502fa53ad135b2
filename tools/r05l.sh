set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu.py tests/test_gpu_sharded.py -m gpu -x -q --timeout 300 --timeout-method thread -k "join_range" > gpurun_out/r05l_tests.log 2>&1 || { tail -30 gpurun_out/r05l_tests.log; exit 1; }
tail -2 gpurun_out/r05l_tests.log
RDFIND_MEM_REPORT=1 timeout -k 10 300 python -u bench.py --config c4 --scale 1.0 --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --no-resident --c4-strong off > gpurun_out/c4keep_r05l.json 2> gpurun_out/c4keep_r05l.err || { tail -20 gpurun_out/c4keep_r05l.err; exit 1; }
grep MEM gpurun_out/c4keep_r05l.err | tail -1
timeout -k 10 400 python -u -m pytest tests/test_gpu_full.py -m gpu -x -q --timeout 300 --timeout-method thread -k "c4_full_size_one_gpu" > gpurun_out/r05l_c4full.log 2>&1 || { tail -30 gpurun_out/r05l_c4full.log; exit 1; }
tail -2 gpurun_out/r05l_c4full.log
echo done
