cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_gpu_full.py -m gpu -x -v --timeout 400 --timeout-method thread -k "random or synthetic or heavy or full_size_vs_oracle or light_variants" > gpurun_out/g18_tests.log 2>&1 &&
RDFIND_AB_LIBS="librdfind_hip.so,librdfind_hip_nowide.so" timeout -k 10 500 python -u tools/light_ab.py c2:1.0 c3:0.5 c3:1.0 c5:0.1 > gpurun_out/g18_ab.log 2>&1
rc=$?; tail -3 gpurun_out/g18_tests.log; grep -E "FAIL|Error" gpurun_out/g18_tests.log | head; cat gpurun_out/g18_ab.log; exit $rc
