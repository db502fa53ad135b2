set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
RDFIND_AB_LIBS=librdfind_hip_pu1.so,librdfind_hip.so,librdfind_hip_pu1.so,librdfind_hip.so timeout -k 10 900 python -u tools/light_ab.py c2:1.0 c3:1.0 c4:0.4 c5:0.1 c1:1.0 > gpurun_out/pu_ab_r05zd.log 2>&1 || { tail -20 gpurun_out/pu_ab_r05zd.log; exit 1; }
python3 - <<'PY'
import json
for ln in open('gpurun_out/pu_ab_r05zd.log'):
    if ' {' not in ln: continue
    lib, js = ln.split(' ', 1)
    d = json.loads(js)
    print(lib, {k: (v['pivot'], v['emit'], v['light'], v['total'], v['n'], v['sum'] % 100000) for k, v in d.items()})
PY
timeout -k 10 500 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "random_parity or heavy_paths or dense or light or paged or synthetic" > gpurun_out/r05zd_tests.log 2>&1 || { tail -30 gpurun_out/r05zd_tests.log; exit 1; }
tail -2 gpurun_out/r05zd_tests.log
echo done
