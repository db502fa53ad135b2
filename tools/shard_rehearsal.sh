#!/bin/bash
# usage (GPU box): tools/shard_rehearsal.sh <tag> <config> <scale> <ranks> [weak|strong] -- several ranks on the one
# GPU of the box, exchanging through gloo (host-staged), to rehearse the sharded-input protocol at size.  bench.py
# starts its own ranks (no external launcher); strong scaling by default, so the run compares with one GPU.
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
TAG=$1; CFG=$2; SC=$3; NR=$4; SCALING=${5:-strong}
timeout -k 10 600 python bench.py --gpus $NR --steps 2 --warmup 1 --config $CFG --scale $SC --scaling $SCALING \
  --backend gloo > gpurun_out/rehearse_${TAG}.json 2> gpurun_out/rehearse_${TAG}.err \
  || { echo "rehearsal failed"; tail -30 gpurun_out/rehearse_${TAG}.err; exit 1; }
head -c 3000 gpurun_out/rehearse_${TAG}.json
