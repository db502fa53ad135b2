cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
timeout -k 10 500 python -u -m pytest tests/test_gpu.py tests/test_gpu_sharded.py -m gpu -x -v --timeout 300 --timeout-method thread -k "random or heavy or kat or edge or synthetic or projection or large_grids" > gpurun_out/g5_tests.log 2>&1 &&
RDFIND_AB_LIBS="librdfind_hip.so,librdfind_hip.so@RDFIND_PIV2=0,librdfind_hip_s4.so,librdfind_hip_s16.so,librdfind_hip.so@RDFIND_SIG=2,librdfind_hip.so@RDFIND_SIG=0" timeout -k 10 500 python -u tools/light_ab.py c3:0.5 c2:1.0 c5:0.1 > gpurun_out/g5_ab.log 2>&1
rc=$?; tail -3 gpurun_out/g5_tests.log; grep -E "FAIL|Error" gpurun_out/g5_tests.log | head; cat gpurun_out/g5_ab.log; exit $rc
