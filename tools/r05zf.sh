set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
RDFIND_AB_LIBS=librdfind_hip.so,librdfind_hip_p2x.so,librdfind_hip.so,librdfind_hip_p2x.so timeout -k 10 900 python -u tools/light_ab.py c3:1.0 c4:0.4 c3:0.5 c4:0.05 > gpurun_out/p2x_ab_r05zf.log 2>&1 || { tail -20 gpurun_out/p2x_ab_r05zf.log; exit 1; }
python3 - <<'PY'
import json
for ln in open('gpurun_out/p2x_ab_r05zf.log'):
    if ' {' not in ln: continue
    lib, js = ln.split(' ', 1)
    d = json.loads(js)
    print(lib, {k: (v['light'], v['n'], v['sum'] % 100000) for k, v in d.items()})
PY
echo done
