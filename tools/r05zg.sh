set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
RDFIND_AB_LIBS=librdfind_hip.so,librdfind_hip_scan0.so,librdfind_hip_ss32.so,librdfind_hip.so,librdfind_hip_scan0.so,librdfind_hip_ss32.so timeout -k 10 600 python -u tools/light_ab.py c2:1.0 c3:0.5 c4:0.05 c1:1.0 > gpurun_out/scan_ab_r05zg.log 2>&1 || { tail -20 gpurun_out/scan_ab_r05zg.log; exit 1; }
cat gpurun_out/scan_ab_r05zg.log
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "random_parity or join_range or synthetic or scan or sort" > gpurun_out/scan_tests_r05zg.log 2>&1; rc=$?; tail -3 gpurun_out/scan_tests_r05zg.log; exit $rc
