# ad-hoc GPU step of the current session (dev): packed-path threshold A/B
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
RDFIND_AB_LIBS="librdfind_hip.so,librdfind_hip_nl8.so,librdfind_hip_nl32.so" timeout -k 10 500 python -u tools/light_ab.py c2:1.0 c3:0.5 c4:0.05 c5:0.1 > gpurun_out/g28_ab.log 2>&1
rc=$?; cat gpurun_out/g28_ab.log; exit $rc
