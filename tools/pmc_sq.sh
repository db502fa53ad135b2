#!/bin/bash
# usage (GPU box): tools/pmc_sq.sh <tag> <kernel-regex> [bench args] -- SQ issue/wait counters for the kernels
# matching the regex (one pass, 8 SQ counters max; MI355X_MICROARCH.md "rocprofv3 PMC slots").
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
TAG=$1; RE=$2; shift 2
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS \
  --kernel-include-regex "$RE" --kernel-trace -d gpurun_out/sq_$TAG -o run --output-format csv \
  -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/sq_$TAG.log 2>&1 \
  || { echo "sq pass failed"; tail -20 gpurun_out/sq_$TAG.log; exit 1; }
python3 - "$TAG" <<'PY'
import csv, glob, sys, collections
tag = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.defaultdict(set)
for f in glob.glob(f"gpurun_out/sq_{tag}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][-40:]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[k].add(r["Dispatch_Id"])
for k, v in acc.items():
    print(k, len(n[k]), {c: round(x / len(n[k])) for c, x in sorted(v.items())})
PY
