# ad-hoc GPU step of the current session (dev): 2-rank rehearsal of c4 at 0.05 (gloo, one GPU)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
tools/gpu_round.sh r02k rehearse:c4:0.05:2
