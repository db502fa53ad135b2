set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
RDFIND_AB_LIBS=librdfind_hip.so,librdfind_hip_it2.so,librdfind_hip_swu4.so,librdfind_hip_bat2.so,librdfind_hip_it2b2.so,librdfind_hip_it2w5.so,librdfind_hip.so timeout -k 10 600 python -u tools/light_ab.py c2:1.0 c3:0.5 c4:0.4 c5:0.1 > gpurun_out/light_ab_r05p.log 2>&1 || { tail -20 gpurun_out/light_ab_r05p.log; exit 1; }
cat gpurun_out/light_ab_r05p.log | cut -c1-400
for spec in "0.5 2" "0.5 4"; do
  set -- $spec
  RDFIND_MEM_REPORT=1 timeout -k 10 700 python -u tools/shard_check.py c4 $1 $2 --no-single > gpurun_out/shard_c4_$1_$2r.json 2> gpurun_out/shard_c4_$1_$2r.err || { tail -20 gpurun_out/shard_c4_$1_$2r.err; tail -c 1500 gpurun_out/shard_c4_$1_$2r.json; exit 1; }
  tail -c 1500 gpurun_out/shard_c4_$1_$2r.json; grep MEM gpurun_out/shard_c4_$1_$2r.err | tail -4
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05p_c4_1.0 -o run --output-format csv -- python3 bench.py --config c4 --scale 1.0 --steps 1 --warmup 1 --no-cpu-baseline --no-ingest --no-resident --c4-strong off > gpurun_out/prof_r05p_c4_1.0.log 2>&1 || { tail -20 gpurun_out/prof_r05p_c4_1.0.log; exit 1; }
find gpurun_out/prof_r05p_c4_1.0 -name "*kernel_stats.csv" -exec cp {} gpurun_out/r05p_c4_1.0_kernel_stats.csv \;
echo done
