set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
RDFIND_AB_LIBS=librdfind_hip.so,librdfind_hip.so@RDFIND_LIGHT_ORDER_CLASSES=1,librdfind_hip.so@RDFIND_LIGHT_ORDER_CLASSES=1@RDFIND_LIGHT_ORDER=1,librdfind_hip.so,librdfind_hip.so@RDFIND_LIGHT_ORDER_CLASSES=1 timeout -k 10 700 python -u tools/light_ab.py c2:1.0 c3:1.0 c4:0.4 c5:0.1 c1:1.0 > gpurun_out/cls_ab_r05za.log 2>&1 || { tail -20 gpurun_out/cls_ab_r05za.log; exit 1; }
python3 - <<'PY'
import json
for ln in open('gpurun_out/cls_ab_r05za.log'):
    if ' {' not in ln: continue
    lib, js = ln.split(' ', 1)
    d = json.loads(js)
    print(lib, {k: (v['light'], v['n'], v['sum'] % 100000) for k, v in d.items()})
PY
echo done
