#!/bin/bash
# usage: tools/prof.sh <tag> <bench args...>   (run on the GPU box)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
TAG=$1; shift
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py "$@" > gpurun_out/prof_$TAG.log 2>&1
rc=$?
find gpurun_out/prof_$TAG -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_$TAG.kernel_stats.csv \;
exit $rc
