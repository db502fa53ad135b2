set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_gpu_sharded.py -m gpu -x -q --timeout 300 --timeout-method thread -k "join_range or k2_split or synthetic_configs" > gpurun_out/r05o_tests.log 2>&1 || { tail -30 gpurun_out/r05o_tests.log; exit 1; }
tail -2 gpurun_out/r05o_tests.log
for cfg in "c4 0.4" "c3 1.0" "c4 1.0"; do
  set -- $cfg
  for rm in 134217728 999999999999; do
    RDFIND_B2_RADIX_MIN=$rm timeout -k 10 300 python -u bench.py --config $1 --scale $2 --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --no-resident --c4-strong off > gpurun_out/b_r05o_$1_$2_$rm.json 2> gpurun_out/b_r05o_$1_$2_$rm.err || { tail -20 gpurun_out/b_r05o_$1_$2_$rm.err; exit 1; }
    python3 -c "
import json,sys
b=json.loads(open('gpurun_out/b_r05o_$1_$2_$rm.json').read().strip().splitlines()[-1])
print('$1 $2 radix_min=$rm', b['ms_per_step'], 'cinds', b.get('cinds', b.get('config',{}).get('n_cinds')), {k:v['ms'] for k,v in b['families'].items() if k in ('binary','emit','sort','support','unary')})"
  done
done
echo done
