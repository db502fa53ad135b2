set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu.py tests/test_gpu_sharded.py -m gpu -x -q --timeout 300 --timeout-method thread -k "join_range" > gpurun_out/r05s_tests.log 2>&1 || { tail -30 gpurun_out/r05s_tests.log; exit 1; }
tail -2 gpurun_out/r05s_tests.log
timeout -k 10 300 python -u bench.py --config c4 --scale 1.0 --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-resident --c4-strong off > gpurun_out/s_c4.json 2> gpurun_out/s_c4.err || { tail -20 gpurun_out/s_c4.err; exit 1; }
python3 -c "
import json
b=json.loads(open('gpurun_out/s_c4.json').read().strip().splitlines()[-1])
print('c4 1.0', b['ms_per_step'], b['config'].get('cinds'), {k:v['ms'] for k,v in b['families'].items()})"
RDFIND_AB_LIBS=librdfind_hip.so,librdfind_hip_rs24.so,librdfind_hip_rs32.so timeout -k 10 600 python -u tools/light_ab.py c2:1.0 c3:1.0 c4:0.4 > gpurun_out/rs_ab_r05s.log 2>&1 || { tail -20 gpurun_out/rs_ab_r05s.log; exit 1; }
cut -c1-600 gpurun_out/rs_ab_r05s.log
echo done
