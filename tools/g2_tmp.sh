cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
timeout -k 10 500 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "random or heavy or kat or edge or synthetic or projection or large_grids" > gpurun_out/g10_tests.log 2>&1 &&
RDFIND_STAGE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "random or heavy or synthetic" > gpurun_out/g10_tests_stage.log 2>&1 &&
RDFIND_AB_LIBS="librdfind_hip.so,librdfind_hip.so@RDFIND_STAGE=0,librdfind_hip.so@RDFIND_STAGE=1,librdfind_hip_u16.so,librdfind_hip_u17.so" timeout -k 10 400 python -u tools/light_ab.py c3:0.5 c2:1.0 c5:0.1 c1:1.0 > gpurun_out/g10_ab.log 2>&1
rc=$?; tail -3 gpurun_out/g10_tests.log; tail -3 gpurun_out/g10_tests_stage.log; grep -E "FAIL|Error" gpurun_out/g10_tests*.log | head; cat gpurun_out/g10_ab.log; exit $rc
