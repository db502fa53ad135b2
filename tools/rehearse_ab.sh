#!/bin/bash
# usage (GPU box): tools/rehearse_ab.sh <tag> <config> <scale> <ranks> [ENV=VAL ...] -- one strong-scaling rehearsal of
# the sharded protocol: <ranks> ranks on the box's one GPU exchanging through gloo (bench.py starts them), with the given
# library switches; the bench line (per-rank work and max_over_mean) -> gpurun_out/rehearse_<tag>.json
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
TAG=$1; CFG=$2; SC=$3; NR=$4; shift 4
mkdir -p gpurun_out
env "$@" timeout -k 10 500 python bench.py --gpus $NR --steps 1 --warmup 0 --config $CFG --scale $SC --scaling strong \
  --backend gloo --no-resident > gpurun_out/rehearse_${TAG}.json 2> gpurun_out/rehearse_${TAG}.err \
  || { echo "rehearsal $TAG failed"; tail -30 gpurun_out/rehearse_${TAG}.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['config']['cinds'], json.dumps(d['ranks']['max_over_mean']))" gpurun_out/rehearse_${TAG}.json
