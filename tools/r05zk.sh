set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
RDFIND_AB_LIBS=librdfind_hip.so,librdfind_hip_l0.so,librdfind_hip_l32.so,librdfind_hip.so,librdfind_hip_l0.so,librdfind_hip_l32.so timeout -k 10 800 python -u tools/light_ab.py c2:1.0 c3:1.0 c4:0.4 c1:1.0 > gpurun_out/light_xcd_ab.log 2>&1 || { tail -20 gpurun_out/light_xcd_ab.log; exit 1; }
python3 - <<'PY'
import json
for ln in open('gpurun_out/light_xcd_ab.log'):
    if ' {' not in ln: continue
    lib, js = ln.split(' ', 1)
    d = json.loads(js)
    print(lib, {k: (v['light'], v['total'], v['n'], v['sum'] % 100000) for k, v in d.items()})
PY
