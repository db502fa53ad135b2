set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for spec in "c2 1.0 RDFIND_B2_RADIX_MIN=1" "c2 1.0 RDFIND_B2_RADIX_MIN=134217728" "c4 0.4 RDFIND_PART_DIGIT=9" "c4 0.4 RDFIND_PART_DIGIT=8" "c4 1.0 RDFIND_PART_DIGIT=9" "c4 1.0 RDFIND_MEM_REPORT=1"; do
  set -- $spec
  tag=$1_$2_$(echo $3 | tr '=' '_')
  env $3 timeout -k 10 300 python -u bench.py --config $1 --scale $2 --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-resident --c4-strong off > gpurun_out/t_$tag.json 2> gpurun_out/t_$tag.err || { tail -20 gpurun_out/t_$tag.err; exit 1; }
  python3 -c "
import json
b=json.loads(open('gpurun_out/t_$tag.json').read().strip().splitlines()[-1])
print('$tag', b['ms_per_step'], b['config'].get('cinds'), {k:v['ms'] for k,v in b['families'].items() if k in ('binary','unary','emit','sort','support','groups')})"
  grep MEM gpurun_out/t_$tag.err | cut -c1-600 | tail -1 || true
done
echo done
