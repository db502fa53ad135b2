cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
RDFIND_AB_LIBS="librdfind_hip.so,librdfind_hip_cr1.so" timeout -k 10 300 python -u tools/light_ab.py c2:1.0 c3:0.5 > gpurun_out/g23_ab.log 2>&1 &&
tools/gpu_round.sh r02i tests bench prof pmc
rc=$?; cat gpurun_out/g23_ab.log; exit $rc
