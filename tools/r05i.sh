set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
RDFIND_MEM_REPORT=1 timeout -k 10 300 python -u bench.py --config c4 --scale 1.0 --steps 1 --warmup 0 --no-cpu-baseline --no-ingest --no-resident --c4-strong off > gpurun_out/c4mem_r05i.json 2> gpurun_out/c4mem_r05i.err || { tail -20 gpurun_out/c4mem_r05i.err; exit 1; }
grep MEM gpurun_out/c4mem_r05i.err | tail -1
RDFIND_MEM_REPORT=1 timeout -k 10 600 python -u tools/shard_check.py c4 0.6 2 > gpurun_out/shard_c4_0.6_2r.json 2> gpurun_out/shard_c4_0.6_2r.err || { tail -20 gpurun_out/shard_c4_0.6_2r.err; tail -c 1500 gpurun_out/shard_c4_0.6_2r.json; exit 1; }
tail -c 1200 gpurun_out/shard_c4_0.6_2r.json; grep MEM gpurun_out/shard_c4_0.6_2r.err | tail -3
RDFIND_AB_LIBS=librdfind_hip.so,librdfind_hip_sg32k.so,librdfind_hip_sr16.so,librdfind_hip_sr4g.so timeout -k 10 600 python -u tools/light_ab.py c4:0.4 c3:1.0 > gpurun_out/k2_ab_r05i.log 2>&1 || { tail -20 gpurun_out/k2_ab_r05i.log; exit 1; }
echo done
RDFIND_AB_LIBS=librdfind_hip.so,librdfind_hip_ps8.so,librdfind_hip_ps2.so,librdfind_hip_ser8.so,librdfind_hip_ser2.so timeout -k 10 600 python -u tools/light_ab.py c2:1.0 c3:0.5 c4:0.4 c5:0.1 > gpurun_out/light_ab2_r05i.log 2>&1 || { tail -20 gpurun_out/light_ab2_r05i.log; exit 1; }
echo done2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05i_c2only -o run --output-format csv -- python3 bench.py --no-cpu-baseline --c4-strong off > gpurun_out/prof_r05i_c2only.log 2>&1 || { tail -20 gpurun_out/prof_r05i_c2only.log; exit 1; }
find gpurun_out/prof_r05i_c2only -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_r05i_c2only.kernel_stats.csv \;
echo done3
