set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for lend in 1 0; do
  RDFIND_DENSE_LEND=$lend RDFIND_DEBUG_LIGHT=1 timeout -k 10 300 python -u bench.py --config c4 --scale 1.0 --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-resident --c4-strong off > gpurun_out/w_c4_$lend.json 2> gpurun_out/w_c4_$lend.err || { tail -20 gpurun_out/w_c4_$lend.err; exit 1; }
  python3 -c "
import json
b=json.loads(open('gpurun_out/w_c4_$lend.json').read().strip().splitlines()[-1])
print('lend=$lend', b['ms_per_step'], b['config'].get('cinds'), {k:v['ms'] for k,v in b['families'].items()})"
  grep "dense:" gpurun_out/w_c4_$lend.err | tail -1 || true
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_sharded.py -m gpu -x -q --timeout 300 --timeout-method thread -k "c4_full_size_one_gpu or join_range" > gpurun_out/r05w_tests.log 2>&1 || { tail -30 gpurun_out/r05w_tests.log; exit 1; }
tail -2 gpurun_out/r05w_tests.log
echo done
