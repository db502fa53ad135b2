set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "random_parity or synthetic_configs or join_range or k2_split" > gpurun_out/r05q_tests.log 2>&1 || { tail -30 gpurun_out/r05q_tests.log; exit 1; }
tail -2 gpurun_out/r05q_tests.log
for cfg in "c2 1.0" "c3 1.0" "c4 1.0"; do
  set -- $cfg
  for s10 in 1 0; do
    RDFIND_SORT10=$s10 timeout -k 10 300 python -u bench.py --config $1 --scale $2 --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-resident --c4-strong off > gpurun_out/s10_$1_$s10.json 2> gpurun_out/s10_$1_$s10.err || { tail -20 gpurun_out/s10_$1_$s10.err; exit 1; }
    python3 -c "
import json
b=json.loads(open('gpurun_out/s10_$1_$s10.json').read().strip().splitlines()[-1])
print('$1 sort10=$s10', b['ms_per_step'], b['config'].get('cinds'), {k:v['ms'] for k,v in b['families'].items() if k in ('sort','groups','binary','emit','support')})"
  done
done
RDFIND_MEM_REPORT=1 RDFIND_HIP_LIB=$GRAFT_REPO_ROOT/rdfind_amd/librdfind_hip_jh13.so timeout -k 10 300 python -u bench.py --config c4 --scale 1.0 --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --no-resident --c4-strong off > gpurun_out/c4_q_jh13.json 2> gpurun_out/c4_q_jh13.err || { tail -20 gpurun_out/c4_q_jh13.err; exit 1; }
python3 -c "
import json
b=json.loads(open('gpurun_out/c4_q_jh13.json').read().strip().splitlines()[-1])
print('jh13', b['ms_per_step'], b['config'].get('cinds'), {k:v['ms'] for k,v in b['families'].items()})"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05q_c4_1.0 -o run --output-format csv -- python3 bench.py --config c4 --scale 1.0 --steps 1 --warmup 1 --no-cpu-baseline --no-ingest --no-resident --c4-strong off > gpurun_out/prof_r05q_c4_1.0.log 2>&1 || { tail -20 gpurun_out/prof_r05q_c4_1.0.log; exit 1; }
find gpurun_out/prof_r05q_c4_1.0 -name "*kernel_stats.csv" -exec cp {} gpurun_out/r05q_c4_1.0_kernel_stats.csv \;
RDFIND_MEM_REPORT=1 timeout -k 10 700 python -u tools/shard_check.py c4 0.5 2 --no-single > gpurun_out/shard_c4_0.5_2r_q.json 2> gpurun_out/shard_c4_0.5_2r_q.err || { tail -20 gpurun_out/shard_c4_0.5_2r_q.err; tail -c 1500 gpurun_out/shard_c4_0.5_2r_q.json; exit 1; }
tail -c 700 gpurun_out/shard_c4_0.5_2r_q.json; grep MEM gpurun_out/shard_c4_0.5_2r_q.err | cut -c1-300 | tail -4
echo done
