set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u tools/gpu_quick.py > gpurun_out/quick_l2.log 2>&1 || { tail -30 gpurun_out/quick_l2.log; exit 1; }
tail -4 gpurun_out/quick_l2.log | cut -c1-300
RDFIND_AB_LIBS="librdfind_hip.so@RDFIND_LIGHT2=0,librdfind_hip.so,librdfind_hip_pre24.so,librdfind_hip_pre48.so" timeout -k 10 600 python -u tools/light_ab.py c2:1.0 c4:0.05 c5:0.1 c3:0.5 > gpurun_out/ab_l2.log 2>&1 || { tail -20 gpurun_out/ab_l2.log; exit 1; }
cat gpurun_out/ab_l2.log
