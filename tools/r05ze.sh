set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
RDFIND_AB_LIBS=librdfind_hip_dd0.so,librdfind_hip.so,librdfind_hip_dd0.so,librdfind_hip.so timeout -k 10 900 python -u tools/light_ab.py c2:1.0 c3:1.0 c1:1.0 c5:0.1 > gpurun_out/dd_ab_r05ze.log 2>&1 || { tail -20 gpurun_out/dd_ab_r05ze.log; exit 1; }
python3 - <<'PY'
import json
for ln in open('gpurun_out/dd_ab_r05ze.log'):
    if ' {' not in ln: continue
    lib, js = ln.split(' ', 1)
    d = json.loads(js)
    print(lib, {k: (v['emit'], v['sort'], v['groups'], v['total'], v['n'], v['sum'] % 100000) for k, v in d.items()})
PY
timeout -k 10 500 python -u -m pytest tests/test_gpu.py tests/test_gpu_sharded.py -m gpu -x -q --timeout 300 --timeout-method thread -k "random_parity or join_range or synthetic" > gpurun_out/r05ze_tests.log 2>&1 || { tail -30 gpurun_out/r05ze_tests.log; exit 1; }
tail -2 gpurun_out/r05ze_tests.log
echo done
