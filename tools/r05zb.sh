set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
RDFIND_AB_LIBS=librdfind_hip_db4.so,librdfind_hip.so,librdfind_hip_few2.so,librdfind_hip_few2db4.so,librdfind_hip_db4.so,librdfind_hip.so,librdfind_hip_few2.so timeout -k 10 900 python -u tools/light_ab.py c2:1.0 c3:1.0 c4:0.4 c5:0.1 c1:1.0 > gpurun_out/db_ab_r05zb.log 2>&1 || { tail -20 gpurun_out/db_ab_r05zb.log; exit 1; }
python3 - <<'PY'
import json
for ln in open('gpurun_out/db_ab_r05zb.log'):
    if ' {' not in ln: continue
    lib, js = ln.split(' ', 1)
    d = json.loads(js)
    print(lib, {k: (v['light'], v['n'], v['sum'] % 100000) for k, v in d.items()})
PY
echo done
