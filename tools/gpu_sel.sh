#!/bin/bash
# GPU box: selected GPU tests (one pytest process, its own limit), then optionally the default bench.
# usage: tools/gpu_sel.sh <tag> <bench:0|1> <pytest -k expression or "">  [test paths...]
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
TAG=$1; BENCH=$2; K=$3; shift 3
mkdir -p gpurun_out
if [ -n "$K" ] || [ $# -gt 0 ]; then
  ( timeout -k 10 1000 python -u -m pytest ${@:-tests} -m gpu -x -v ${K:+-k "$K"} --durations=30 --timeout 600 \
      --timeout-method thread > gpurun_out/sel_$TAG.log 2>&1; echo "pytest rc=$?" >> gpurun_out/sel_$TAG.log ) &
  PID=$!
  while kill -0 $PID 2>/dev/null; do sleep 40; echo "[hb $(date +%T)] $(tail -c 150 gpurun_out/sel_$TAG.log | tr '\n' ' ')"; done
  wait $PID
  tail -15 gpurun_out/sel_$TAG.log
  grep -q "pytest rc=0" gpurun_out/sel_$TAG.log || exit 1
fi
if [ "$BENCH" = 1 ]; then
  timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
    || { echo "bench failed"; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
  head -c 1500 gpurun_out/bench_$TAG.json; echo; python3 -c "
import json; l=json.load(open('gpurun_out/bench_$TAG.json')); print('value',l['value'],'ms',l['ms_per_step']); print('c4',{k:l['c4_strong'].get(k) for k in ('ms_per_step','cinds','matches_golden','error')}); print(l['kernel_ms'])"
fi
