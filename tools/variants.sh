#!/bin/bash
# usage (GPU box): tools/variants.sh <tag> lib1.so lib2.so ...  -- bench each library variant (dev tool)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
mkdir -p gpurun_out
for lib in "$@"; do
  RDFIND_HIP_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 3 > gpurun_out/var_${TAG}_$(basename $lib .so).json 2>&1 \
    || { echo "variant $lib failed"; tail -20 gpurun_out/var_${TAG}_$(basename $lib .so).json; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['kernel_ms'])" gpurun_out/var_${TAG}_$(basename $lib .so).json $lib
done
