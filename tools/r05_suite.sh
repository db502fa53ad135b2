#!/bin/bash
# GPU box: the driver's GPU test command (one pytest process, durations kept) and the smoke, each under its own limit
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
TAG=${1:-suite}
mkdir -p gpurun_out
( timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --durations=40 --timeout 300 --timeout-method thread \
    > gpurun_out/tests_$TAG.log 2>&1; echo "pytest rc=$?" >> gpurun_out/tests_$TAG.log ) &
PID=$!
while kill -0 $PID 2>/dev/null; do sleep 45; echo "[hb $(date +%T)] $(tail -c 120 gpurun_out/tests_$TAG.log | tr '\n' ' ')"; done
wait $PID
tail -3 gpurun_out/tests_$TAG.log
grep -q "pytest rc=0" gpurun_out/tests_$TAG.log || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
cat gpurun_out/smoke_$TAG.log
