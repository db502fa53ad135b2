set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --config c4 --scale 1.0 --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --no-resident --c4-strong off > gpurun_out/c4full_r05f.json 2> gpurun_out/c4full_r05f.err || { tail -20 gpurun_out/c4full_r05f.err; exit 1; }
RDFIND_AB_LIBS=librdfind_hip.so,librdfind_hip_b4.so,librdfind_hip_b6.so,librdfind_hip_b4w4.so timeout -k 10 700 python -u tools/light_ab.py c2:1.0 c3:0.5 c4:0.4 c5:0.1 > gpurun_out/light_ab_r05f.log 2>&1 || { tail -20 gpurun_out/light_ab_r05f.log; exit 1; }
echo done
