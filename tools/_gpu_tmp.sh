cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_view_templates_gpu.py tests/test_configs_gpu.py > gpurun_out/vt_t.log 2>&1 || { echo "tests failed $?"; tail -5 gpurun_out/vt_t.log; exit 1; }
tail -1 gpurun_out/vt_t.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r2i.json 2> gpurun_out/bench_r2i.err || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r2j.json 2> gpurun_out/bench_r2j.err || exit 1
