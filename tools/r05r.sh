set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_gpu_sharded.py -m gpu -x -q --timeout 300 --timeout-method thread -k "random_parity or synthetic_configs or join_range or k2_split" > gpurun_out/r05r_tests.log 2>&1 || { tail -30 gpurun_out/r05r_tests.log; exit 1; }
tail -2 gpurun_out/r05r_tests.log
for cfg in "c2 1.0" "c3 1.0" "c4 0.4" "c4 1.0"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --config $1 --scale $2 --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-resident --c4-strong off > gpurun_out/r_$1_$2.json 2> gpurun_out/r_$1_$2.err || { tail -20 gpurun_out/r_$1_$2.err; exit 1; }
  python3 -c "
import json
b=json.loads(open('gpurun_out/r_$1_$2.json').read().strip().splitlines()[-1])
print('$1 $2', b['ms_per_step'], b['config'].get('cinds'), {k:v['ms'] for k,v in b['families'].items()})"
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_full.py -m gpu -x -q --timeout 300 --timeout-method thread -k "c4_full_size_one_gpu" > gpurun_out/r05r_c4full.log 2>&1 || { tail -30 gpurun_out/r05r_c4full.log; exit 1; }
tail -2 gpurun_out/r05r_c4full.log
echo done
