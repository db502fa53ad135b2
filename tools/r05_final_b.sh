set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_round.sh r05 configs || exit 1
for cs in c4@1.0 c5@1.0; do
  CFG=${cs%@*}; SC=${cs#*@}
  ( timeout -k 10 500 python -u bench.py --config $CFG --scale $SC --steps 2 --warmup 1 --no-ingest > gpurun_out/cfg_r05_${CFG}_$SC.json 2> gpurun_out/cfg_r05_${CFG}_$SC.err; echo "rc=$?" >> gpurun_out/cfg_r05_${CFG}_$SC.err ) &
  PID=$!
  while kill -0 $PID 2>/dev/null; do sleep 45; echo "[hb $(date +%T)] $(tail -c 150 gpurun_out/cfg_r05_${CFG}_$SC.err | tr '\n' ' ')"; done
  wait $PID
  grep -q "rc=0" gpurun_out/cfg_r05_${CFG}_$SC.err || { tail -30 gpurun_out/cfg_r05_${CFG}_$SC.err; exit 1; }
  head -c 600 gpurun_out/cfg_r05_${CFG}_$SC.json; echo
done
echo done
