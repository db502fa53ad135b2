set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
RDFIND_AB_LIBS=librdfind_hip.so,librdfind_hip_p0.so,librdfind_hip.so,librdfind_hip_p0.so timeout -k 10 700 python -u tools/light_ab.py c2:1.0 c3:1.0 c4:0.4 c1:1.0 > gpurun_out/part_xcd_ab.log 2>&1 || { tail -20 gpurun_out/part_xcd_ab.log; exit 1; }
python3 - <<'PY'
import json
for ln in open('gpurun_out/part_xcd_ab.log'):
    if ' {' not in ln: continue
    lib, js = ln.split(' ', 1)
    d = json.loads(js)
    print(lib, {k: (v['unary'], v['binary'], v['sort'], v['total'], v['n'], v['sum'] % 100000) for k, v in d.items()})
PY
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "random_parity or join_range or synthetic or sort or k2" > gpurun_out/part_xcd_tests.log 2>&1; rc=$?; tail -3 gpurun_out/part_xcd_tests.log; exit $rc
