#!/bin/bash
# usage (GPU box): tools/prof_hb.sh <tag> <bench args...> -- tools/prof.sh with a heartbeat line every 45 s (a long
# silent input generation under rocprofv3 otherwise looks hung to the runner)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
"$(dirname "$0")/prof.sh" "$@" &
PID=$!
while kill -0 $PID 2>/dev/null; do sleep 45; echo "[hb $(date +%T)] prof $1 running"; done
wait $PID
