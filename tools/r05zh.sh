set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
RDFIND_AB_LIBS=librdfind_hip.so,librdfind_hip.so@RDFIND_B2_RADIX_MIN=1,librdfind_hip.so@RDFIND_B2_RADIX_MIN=1@RDFIND_PART_DIGIT=8,librdfind_hip.so,librdfind_hip.so@RDFIND_B2_RADIX_MIN=1,librdfind_hip.so@RDFIND_B2_RADIX_MIN=1@RDFIND_PART_DIGIT=8 timeout -k 10 600 python -u tools/light_ab.py c2:1.0 c1:1.0 c2:0.5 > gpurun_out/k2_c2_radix_ab.log 2>&1 || { tail -20 gpurun_out/k2_c2_radix_ab.log; exit 1; }
python3 - <<'PY'
import json
for ln in open('gpurun_out/k2_c2_radix_ab.log'):
    if ' {' not in ln: continue
    lib, js = ln.split(' ', 1)
    d = json.loads(js)
    print(lib, {k: (v['binary'], v['unary'], v['total'], v['n'], v['sum'] % 100000) for k, v in d.items()})
PY
