set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
RDFIND_AB_LIBS=librdfind_hip_lk0.so,librdfind_hip.so,librdfind_hip_lk0.so,librdfind_hip.so timeout -k 10 900 python -u tools/light_ab.py c2:1.0 c3:1.0 c4:0.4 c1:1.0 > gpurun_out/lk_ab_r05zc.log 2>&1 || { tail -20 gpurun_out/lk_ab_r05zc.log; exit 1; }
python3 - <<'PY'
import json
for ln in open('gpurun_out/lk_ab_r05zc.log'):
    if ' {' not in ln: continue
    lib, js = ln.split(' ', 1)
    d = json.loads(js)
    print(lib, {k: (v['emit'], v['light'], v['total'], v['n'], v['sum'] % 100000) for k, v in d.items()})
PY
for lib in librdfind_hip_lk0.so librdfind_hip.so; do
  RDFIND_HIP_LIB=$GRAFT_REPO_ROOT/rdfind_amd/$lib timeout -k 10 300 python -u bench.py --config c4 --scale 1.0 --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --no-resident --c4-strong off > gpurun_out/lk_c4_$lib.json 2> gpurun_out/lk_c4_$lib.err || { tail -20 gpurun_out/lk_c4_$lib.err; exit 1; }
  python3 -c "
import json
b=json.loads(open('gpurun_out/lk_c4_$lib.json').read().strip().splitlines()[-1])
print('$lib c4 1.0', b['ms_per_step'], b['config'].get('cinds'), {k:v['ms'] for k,v in b['families'].items()})"
done
echo done
