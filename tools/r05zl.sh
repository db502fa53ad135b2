set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
RDFIND_AB_LIBS=librdfind_hip.so@RDFIND_EMIT_ONEPASS=1,librdfind_hip.so,librdfind_hip.so@RDFIND_EMIT_ONEPASS=1,librdfind_hip.so timeout -k 10 600 python -u tools/light_ab.py c2:1.0 c3:1.0 c4:0.05 c1:1.0 > gpurun_out/emit_onepass_ab.log 2>&1 || { tail -20 gpurun_out/emit_onepass_ab.log; exit 1; }
python3 - <<'PY'
import json
for ln in open('gpurun_out/emit_onepass_ab.log'):
    if ' {' not in ln: continue
    lib, js = ln.split(' ', 1)
    d = json.loads(js)
    print(lib, {k: (v['emit'], v['sort'], v['total'], v['n'], v['sum'] % 100000) for k, v in d.items()})
PY
RDFIND_EMIT_ONEPASS=1 timeout -k 10 500 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/emit_onepass_tests.log 2>&1; rc=$?; tail -3 gpurun_out/emit_onepass_tests.log; exit $rc
