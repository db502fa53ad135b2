cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
timeout -k 10 500 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "random or heavy or kat or edge or synthetic or projection" > gpurun_out/g7_tests.log 2>&1 &&
RDFIND_AB_LIBS="librdfind_hip.so,librdfind_hip_p1.so,librdfind_hip_p8.so" timeout -k 10 400 python -u tools/light_ab.py c3:0.5 c2:1.0 c5:0.1 > gpurun_out/g7_ab.log 2>&1 &&
timeout -k 10 300 python -u tools/light_items.py c2 1.0 > gpurun_out/g7_items_c2.log 2>&1
rc=$?; tail -3 gpurun_out/g7_tests.log; grep -E "FAIL|Error" gpurun_out/g7_tests.log | head; cat gpurun_out/g7_ab.log; tail -30 gpurun_out/g7_items_c2.log; exit $rc
