set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
tools/gpu_round.sh r05h bench prof || exit 1
tools/pmc.sh r05h_c2 || exit 1
echo done
