cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
timeout -k 10 700 python -u -m pytest tests/test_gpu.py tests/test_gpu_full.py tests/test_gpu_sharded.py -m gpu -x -v --timeout 400 --timeout-method thread -k "random or synthetic or heavy or full_size_vs_oracle or edge or kat" > gpurun_out/g19_tests.log 2>&1 &&
RDFIND_AB_LIBS="librdfind_hip.so,librdfind_hip_rs9.so,librdfind_hip_rs8.so" timeout -k 10 450 python -u tools/light_ab.py c2:1.0 c3:0.5 c3:1.0 > gpurun_out/g19_ab.log 2>&1
rc=$?; tail -3 gpurun_out/g19_tests.log; grep -E "FAIL|Error" gpurun_out/g19_tests.log | head; cat gpurun_out/g19_ab.log; exit $rc
