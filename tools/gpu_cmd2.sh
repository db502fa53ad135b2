set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
PB=${1:-0}
timeout -k 10 900 python -u bench.py --config c5 --scale 1.0 --steps 1 --warmup 0 --no-cpu-baseline --no-ingest --no-resident --page-log --page-bytes $PB > gpurun_out/c5full_$PB.json 2> gpurun_out/c5full_$PB.err &
PID=$!
while kill -0 $PID 2>/dev/null; do sleep 20; echo "[hb] $(tail -c 300 gpurun_out/c5full_$PB.err | tr '\n' ' ')"; done
wait $PID || { echo "c5 full failed"; tail -30 gpurun_out/c5full_$PB.err; exit 1; }
cat gpurun_out/c5full_$PB.json | head -c 3000
