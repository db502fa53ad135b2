cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r02.log 2>&1 &&
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/bench_final_quick.json 2> gpurun_out/bench_final_quick.err
rc=$?; cat gpurun_out/smoke_r02.log | tail -2; cut -c1-300 gpurun_out/bench_final_quick.json; exit $rc
