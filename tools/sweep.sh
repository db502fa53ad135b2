#!/bin/bash
# dev: bench each library variant on the given configs.  tools/sweep.sh "base seg512" "c2:1.0 c3:0.5"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in $1; do
  lib=rdfind_amd/librdfind_hip.so; [ "$v" != base ] && lib=rdfind_amd/librdfind_hip_$v.so
  for cs in $2; do
    IFS=: read -r cfg sc <<< "$cs"
    RDFIND_HIP_LIB=$PWD/$lib timeout -k 10 300 python3 -u bench.py --config $cfg --scale $sc --steps 3 --warmup 1 --no-cpu-baseline \
      > gpurun_out/sw_${v}_$cfg.json 2> gpurun_out/sw_${v}_$cfg.err || { echo "fail $v $cfg"; tail -5 gpurun_out/sw_${v}_$cfg.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/sw_${v}_$cfg.json').read()); print('$v', '$cfg', d['ms_per_step'], 'light', d['kernel_ms'].get('light'), 'cinds', d['config']['cinds'])"
  done
done
