# ad-hoc GPU step of the current session (dev): smoke, a quick c2 bench, and c4 at 0.05 / c3 full bench lines
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r02.log 2>&1 &&
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-ingest --no-tdisc > gpurun_out/bench_final_quick.json 2> gpurun_out/bench_final_quick.err &&
timeout -k 10 400 python -u bench.py --config c4 --scale 0.05 --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-tdisc > gpurun_out/cfg_c4_0.05.json 2> gpurun_out/cfg_c4_0.05.err &&
timeout -k 10 400 python -u bench.py --config c3 --scale 1.0 --steps 3 --warmup 1 --no-cpu-baseline --no-ingest --no-tdisc > gpurun_out/cfg_c3_1.0.json 2> gpurun_out/cfg_c3_1.0.err
rc=$?; tail -2 gpurun_out/smoke_r02.log; cut -c1-200 gpurun_out/bench_final_quick.json gpurun_out/cfg_c4_0.05.json gpurun_out/cfg_c3_1.0.json; exit $rc
