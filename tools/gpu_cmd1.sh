set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
RDFIND_AB_LIBS="librdfind_hip_nodedup.so,librdfind_hip.so,librdfind_hip_nodedup.so,librdfind_hip.so" timeout -k 10 600 python -u tools/light_ab.py c2:1.0 c4:0.05 c3:0.5 > gpurun_out/ab_dd.log 2>&1 || { tail -20 gpurun_out/ab_dd.log; exit 1; }
cat gpurun_out/ab_dd.log
