set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/gputest_r5_final3.log 2>&1 || { tail -60 gpurun_out/gputest_r5_final3.log; exit 1; }
tail -3 gpurun_out/gputest_r5_final3.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r5_final3.log 2>&1; tail -2 gpurun_out/smoke_r5_final3.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r5_final3.json 2> gpurun_out/bench_r5_final3.err || { tail -30 gpurun_out/bench_r5_final3.err; exit 1; }
tail -c 300 gpurun_out/bench_r5_final3.json
