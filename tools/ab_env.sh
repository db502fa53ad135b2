#!/bin/bash
# GPU box: A/B of library switches on one bench config.  usage: tools/ab_env.sh <tag> "<bench args>" "ENV=a ENV2=b" "ENV=c" ...
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
TAG=$1; ARGS=$2; shift 2
mkdir -p gpurun_out
i=0
for envs in "$@"; do
  env $envs timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-ingest --c4-strong off $ARGS \
      > gpurun_out/ab_${TAG}_$i.json 2> gpurun_out/ab_${TAG}_$i.err || { echo "run $i failed"; tail -5 gpurun_out/ab_${TAG}_$i.err; exit 1; }
  python3 -c "
import json,sys; l=json.load(open('gpurun_out/ab_${TAG}_$i.json')); k=l['kernel_ms']
print('$envs', '| ms', l['ms_per_step'], '| resident', l['device_resident']['ms_per_step'] if l['device_resident'] else None, '| cinds', l['config']['cinds'], '|', ' '.join(f'{a}={b:.3f}' for a,b in k.items() if b>0.05))"
  i=$((i+1))
done
