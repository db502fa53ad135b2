set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u tools/gpu_quick.py > gpurun_out/quick_dd.log 2>&1 || { tail -30 gpurun_out/quick_dd.log; exit 1; }
tail -4 gpurun_out/quick_dd.log | cut -c1-120
RDFIND_AB_LIBS="librdfind_hip_nodedup.so,librdfind_hip.so,librdfind_hip_nodedup.so,librdfind_hip.so" timeout -k 10 600 python -u tools/light_ab.py c2:1.0 c4:0.05 c3:0.5 > gpurun_out/ab_dd.log 2>&1 || { tail -20 gpurun_out/ab_dd.log; exit 1; }
python3 - <<'PY'
import json
for ln in open("gpurun_out/ab_dd.log"):
    lib, js = ln.split(" ", 1)
    d = json.loads(js)
    print(lib, {k: (v["emit"], v["sort"], v["support"], v["total"]) for k, v in d.items()})
PY
