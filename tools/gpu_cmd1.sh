set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for L in 0 1; do
  RDFIND_LIGHT2=$L RDFIND_LIGHT2_LOG=1 timeout -k 10 600 python -u tools/light_ab.py --child c2:1.0 c4:0.05 c5:0.1 c3:0.5 c1:1.0 > gpurun_out/l2log_$L.log 2>&1 || { tail -20 gpurun_out/l2log_$L.log; exit 1; }
  grep -E "LIGHT2|^AB" gpurun_out/l2log_$L.log | sort | uniq -c | cut -c1-1500
done
