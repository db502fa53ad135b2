#!/bin/bash
# usage (GPU box): tools/shard_rehearsal.sh <tag> <config> <scale> <ranks> -- several ranks on the one GPU of the
# box, exchanging through gloo (host-staged), to rehearse the sharded-input protocol at size.
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
TAG=$1; CFG=$2; SC=$3; NR=$4
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $NR --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus $NR --steps 2 --warmup 1 --config $CFG --scale $SC --backend gloo \
  > gpurun_out/rehearse_${TAG}.json 2> gpurun_out/rehearse_${TAG}.err || { echo "rehearsal failed"; tail -30 gpurun_out/rehearse_${TAG}.err; exit 1; }
cat gpurun_out/rehearse_${TAG}.json
