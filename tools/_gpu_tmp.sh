cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_view_templates_gpu.py tests/test_configs_gpu.py tests/test_sharded_multiproc_gpu.py tests/test_replay_gpu.py > gpurun_out/vt_nb4_test.log 2>&1 || { echo "tests failed $?"; tail -30 gpurun_out/vt_nb4_test.log; exit 1; }
tail -1 gpurun_out/vt_nb4_test.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r2f.json 2> gpurun_out/bench_r2f.err || exit 1
tail -c 300 gpurun_out/bench_r2f.json
