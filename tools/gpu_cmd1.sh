set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for L in 0 1; do
for cfg in "c4 0.05" "c3 0.5" "c5 0.1" "c1 1.0"; do
  set -- $cfg
  RDFIND_LIGHT2=$L timeout -k 10 300 python -u bench.py --config $1 --scale $2 --steps 3 --warmup 1 --no-cpu-baseline --no-ingest > gpurun_out/l2_$L_$1.json 2>/dev/null || { echo "fail $L $1"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('LIGHT2', sys.argv[2], sys.argv[3], 'resident', d['device_resident']['ms_per_step'], 'kernels', round(sum(d['kernel_ms'].values()),2), 'light', d['kernel_ms']['light'])" gpurun_out/l2_$L_$1.json $L $1
done; done
