cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
tools/gpu_round.sh r02g tests bench prof pmc
