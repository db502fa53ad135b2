set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u tools/gpu_quick.py > gpurun_out/quick_rl.log 2>&1 || { tail -30 gpurun_out/quick_rl.log; exit 1; }
tail -4 gpurun_out/quick_rl.log | cut -c1-120
RDFIND_AB_LIBS="librdfind_hip_norl.so,librdfind_hip.so,librdfind_hip_norl.so,librdfind_hip.so" timeout -k 10 600 python -u tools/light_ab.py c2:1.0 c4:0.05 c3:0.5 c5:0.1 > gpurun_out/ab_rl.log 2>&1 || { tail -20 gpurun_out/ab_rl.log; exit 1; }
python3 - <<'PY'
import json
for ln in open("gpurun_out/ab_rl.log"):
    lib, js = ln.split(" ", 1)
    d = json.loads(js)
    print(lib, {k: (v["light"], v["total"], v["n"], v["sum"] % 1000) for k, v in d.items()})
PY
