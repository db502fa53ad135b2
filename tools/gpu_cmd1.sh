set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
RDFIND_AB_LIBS="librdfind_hip.so@RDFIND_CROW_DIV=0,librdfind_hip.so,librdfind_hip_nopk.so,librdfind_hip.so@RDFIND_CROW_DIV=32" timeout -k 10 600 python -u tools/light_ab.py c2:1.0 c4:0.05 c5:0.1 > gpurun_out/ab_crow.log 2>&1 || { tail -20 gpurun_out/ab_crow.log; exit 1; }
cat gpurun_out/ab_crow.log
