#!/bin/bash
# usage (GPU box): tools/pmc.sh <tag> [bench args]   -- one rocprofv3 --pmc pass per TCC counter group,
# each under its own time limit (MI355X_MICROARCH.md "HBM" / "rocprofv3 PMC slots": FETCH_SIZE and
# WRITE_SIZE cannot share a pass).  Summary -> gpurun_out/pmc_<tag>.json (tools/pmc_summary.py).
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $ctr --kernel-trace -d gpurun_out/pmc_${TAG}_$ctr -o run --output-format csv \
    -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-ingest --c4-strong off "$@" > gpurun_out/pmc_${TAG}_$ctr.log 2>&1 \
    || { echo "pmc pass $ctr failed"; tail -20 gpurun_out/pmc_${TAG}_$ctr.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/pmc_${TAG}_FETCH_SIZE gpurun_out/pmc_${TAG}_WRITE_SIZE > gpurun_out/pmc_$TAG.json
cat gpurun_out/pmc_$TAG.json
