set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
RDFIND_AB_LIBS="librdfind_hip.so@RDFIND_CROW_DIV=0,librdfind_hip.so,librdfind_hip_nopk.so,librdfind_hip.so@RDFIND_CROW_DIV=32" timeout -k 10 600 python -u tools/light_ab.py c2:1.0 c4:0.05 c5:0.1 > gpurun_out/ab_crow.log 2>&1 || { tail -20 gpurun_out/ab_crow.log; exit 1; }
cat gpurun_out/ab_crow.log
for v in 0 256 32; do
  RDFIND_CROW_DIV=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pl_$v -o run --output-format csv -- python3 tools/light_ab.py --child c2:1.0 c4:0.05 > gpurun_out/pl_$v.log 2>&1 || { tail -20 gpurun_out/pl_$v.log; exit 1; }
  f=$(find gpurun_out/pl_$v -name "*kernel_stats.csv" | head -1); grep -E "k_light|k_crow|k_dense" $f | cut -c1-40,150-
done
