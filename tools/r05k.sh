set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
RDFIND_MEM_REPORT=1 timeout -k 10 700 python -u tools/shard_check.py c4 0.6 2 > gpurun_out/shard_c4_0.6_2r.json 2> gpurun_out/shard_c4_0.6_2r.err || { tail -20 gpurun_out/shard_c4_0.6_2r.err; tail -c 1500 gpurun_out/shard_c4_0.6_2r.json; exit 1; }
tail -c 1500 gpurun_out/shard_c4_0.6_2r.json; grep MEM gpurun_out/shard_c4_0.6_2r.err | tail -3
RDFIND_AB_LIBS=librdfind_hip.so,librdfind_hip_ps8.so,librdfind_hip_ps2.so,librdfind_hip_ser8.so,librdfind_hip_ser2.so timeout -k 10 500 python -u tools/light_ab.py c2:1.0 c3:0.5 c4:0.4 c5:0.1 > gpurun_out/light_ab2_r05k.log 2>&1 || { tail -20 gpurun_out/light_ab2_r05k.log; exit 1; }
echo done
