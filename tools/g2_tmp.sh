cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
tools/gpu_round.sh r02c tests bench prof &&
RDFIND_AB_LIBS="librdfind_hip.so,librdfind_hip_u15.so,librdfind_hip_u14.so" timeout -k 10 300 python -u tools/light_ab.py c2:1.0 c1:1.0 c3:0.5 > gpurun_out/g11_ab.log 2>&1
rc=$?; cat gpurun_out/g11_ab.log; exit $rc
