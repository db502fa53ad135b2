# ad-hoc GPU step of the current session (dev): c4 light switches A/B and per-item light profile
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
RDFIND_AB_LIBS="librdfind_hip.so,librdfind_hip.so@RDFIND_STAGE=1,librdfind_hip.so@RDFIND_SIG=1,librdfind_hip.so@RDFIND_SIG=0,librdfind_hip.so@RDFIND_PIV2=0" timeout -k 10 400 python -u tools/light_ab.py c4:0.05 > gpurun_out/g26_ab.log 2>&1 &&
timeout -k 10 300 python -u tools/light_items.py c4 0.05 > gpurun_out/g26_items_c4.log 2>&1
rc=$?; cat gpurun_out/g26_ab.log; tail -40 gpurun_out/g26_items_c4.log; exit $rc
