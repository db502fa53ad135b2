cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_full.py -m gpu -x -v --timeout 400 --timeout-method thread -k "full_size_vs_oracle" > gpurun_out/g22_tests.log 2>&1 &&
RDFIND_AB_LIBS="librdfind_hip.so,librdfind_hip.so@RDFIND_B2_SPLIT=0" timeout -k 10 450 python -u tools/light_ab.py c3:1.0 c3:0.5 c2:1.0 > gpurun_out/g22_ab.log 2>&1
rc=$?; tail -3 gpurun_out/g22_tests.log; grep -E "FAIL|Error" gpurun_out/g22_tests.log | head; cat gpurun_out/g22_ab.log; exit $rc
